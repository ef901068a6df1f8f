#!/bin/bash
# Round 5 experiment: FED2 (grouped G = 2, 2 chain waves + 2 producers, 64 jobs per CU), built in
# place of FED4E in an A/B copy (efes_amd/lib/ab/libefeshash_fed2.so).  Parity first (every
# FED4E-parametrized GPU test through the variant), then launch times at 8 192 / 12 288 / 16 384
# x 4 MiB against the product's FED4, FED4E and GROUP4.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r05_fed2}
mkdir -p "$O"
V="$PWD/efes_amd/lib/ab/libefeshash_fed2.so"
timeout -k 10 400 env EFES_LIB_OVERRIDE="$V" python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k fed4e \
  -x -q --timeout 200 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
B="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off --latency-leg off \
 --receiver-leg off --drain-leg off --concurrency-leg off --mixed-leg off --ingest-leg off --span-leg off --steps 5 --warmup 1"
run() {  # name lib chunks mode
  local env_lib=""; [ "$2" = product ] || env_lib="EFES_LIB_OVERRIDE=$V"
  timeout -k 10 200 env $env_lib python3 bench.py $B --chunks $3 --mode $4 > "$O/$1.json" 2> "$O/$1.err" || { tail -5 "$O/$1.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], 'ms', d.get('clock',{}).get('mhz'))" "$O/$1.json" "$1" | tee -a "$O/ab.log"
}
for rep in 1 2; do
  run fed4_8192.$rep product 8192 fed4
  run fed2_8192.$rep fed2 8192 fed4e
  run fed4e_12288.$rep product 12288 fed4e
  run fed2_12288.$rep fed2 12288 fed4e
  run group4_16384.$rep product 16384 group4
  run fed2_16384.$rep fed2 16384 fed4e
done
