#!/bin/bash
# Round 5: DEEP chain-side A/B -- tools/gpu_r05_deep_ab.sh OUT VARIANT: the DEEP-parametrized
# GPU tests through the variant (efes_amd/lib/ab/libefeshash_VARIANT.so), then the headline
# (configs[2]) with the product and the variant, interleaved, twice.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r05_deep_ab}
VAR=${2:?variant}
mkdir -p "$O"
V="$PWD/efes_amd/lib/ab/libefeshash_$VAR.so"
timeout -k 10 400 env EFES_LIB_OVERRIDE="$V" python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k "deep" \
  -x -q --timeout 200 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
B="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off --latency-leg off \
 --receiver-leg off --drain-leg off --concurrency-leg off --mixed-leg off --ingest-leg off --span-leg off --steps 20 --warmup 3"
for rep in ${REPS:-1 2}; do
  for lib in product $VAR; do
    env_lib=""; [ $lib = product ] || env_lib="EFES_LIB_OVERRIDE=$V"
    timeout -k 10 200 env $env_lib python3 bench.py $B > "$O/$lib.$rep.json" 2> "$O/$lib.$rep.err" || { tail -5 "$O/$lib.$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b=d['binding_roofline']; print(sys.argv[2], sys.argv[3], d['value'], d['roofline']['kernel_ms'], 'ms', b['frac'], b['frac_at_clock'], b['clock_mhz'])" "$O/$lib.$rep.json" $rep $lib | tee -a "$O/ab.log"
  done
done
