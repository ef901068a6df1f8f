#!/bin/bash
# Round 5: span CRC A/B.  tools/gpu_r05_span_ab.sh OUT [variant ...]: the span parity tests with the
# product library, then the span leg of bench.py with the product library and each A/B build
# (efes_amd/lib/ab/libefeshash_NAME.so, tools/ab_variant.sh), interleaved, twice.  MB=1 runs the
# read-path microbenchmark first.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r05_span_ab}
shift || true
VARIANTS=("$@")
mkdir -p "$O"
if [ "${MB:-0}" = 1 ]; then
  timeout -k 10 150 tools/microbench/mb_glds 16 > "$O/mb_glds.log" 2>&1 || { cat "$O/mb_glds.log"; exit 1; }
  cat "$O/mb_glds.log"
fi
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_span.py -x -v --timeout 120 --timeout-method thread \
  > "$O/span_tests.log" 2>&1 || { tail -30 "$O/span_tests.log"; exit 1; }
tail -3 "$O/span_tests.log"
for lib in "${VARIANTS[@]}"; do  # every variant must be bit-exact before it is timed
  timeout -k 10 300 env EFES_LIB_OVERRIDE="$PWD/efes_amd/lib/ab/libefeshash_$lib.so" python3 -u -m pytest \
    tests/test_gpu_span.py -x -q --timeout 120 --timeout-method thread > "$O/span_tests_$lib.log" 2>&1 \
    || { tail -30 "$O/span_tests_$lib.log"; exit 1; }
  echo "$lib: $(tail -1 "$O/span_tests_$lib.log")"
done
B="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off --latency-leg off --receiver-leg off --drain-leg off --concurrency-leg off --mixed-leg off --ingest-leg off --steps 2 --warmup 1"
for rep in 1 2; do
  for lib in product "${VARIANTS[@]}"; do
    if [ "$lib" = product ]; then env_lib=""; else env_lib="EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/ab/libefeshash_$lib.so"; fi
    timeout -k 10 200 env $env_lib python3 bench.py $B > "$O/span_$lib.$rep.json" 2> "$O/span_$lib.$rep.err" || { tail -5 "$O/span_$lib.$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['span_crc']; print(sys.argv[2], sys.argv[3], d['value'], 'GiB/s', d['roofline']['achieved'], 'GB/s', d['roofline']['frac'], d['crc_matches_zlib'], d['clock'].get('mhz'))" "$O/span_$lib.$rep.json" $rep $lib | tee -a "$O/ab.log"
  done
done
