#!/bin/bash
# FED4 bring-up: its parity tests, then FED4 vs GROUP4 vs DEEP on 4 MiB chunks (one device, one call).
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/fed
timeout -k 10 240 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py -m gpu -x -v -k "fed4" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fed/tests.log 2>&1
rc=$?; tail -5 gpurun_out/fed/tests.log; [ $rc -eq 0 ] || exit $rc
for spec in "fed4 3072" "group4 3072" "fed4 12288" "group4 12288" "group4 16384" "fed4 6144"; do
  set -- $spec
  timeout -k 10 180 python bench.py --mode $1 --chunks $2 --steps 3 --warmup 1 --no-cpu-baseline --host-inclusive off \
    --ingest-leg off --mixed-leg off --concurrency-leg off --uploads-leg off > gpurun_out/fed/$1_$2.json 2> gpurun_out/fed/$1_$2.err || { echo "FAIL $spec"; tail -5 gpurun_out/fed/$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fed/$1_$2.json'));print('$1 $2', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
done
