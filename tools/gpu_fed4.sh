#!/bin/bash
# FED 4,3x (chain-side expansion): parity under the override, cycle accounting, timing.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/fed
EFES_FED_SHAPE=4,3x timeout -k 10 240 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py -m gpu -x -q -k "fed4" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fed/tests43x.log 2>&1
rc=$?; tail -2 gpurun_out/fed/tests43x.log; [ $rc -eq 0 ] || exit $rc
EFES_FED_SHAPE=4,3x EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/libefeshash_stats.so timeout -k 10 100 python tools/fed_stats.py 48 || exit 1
for n in 48 12288; do
  EFES_FED_SHAPE=4,3x timeout -k 10 120 python bench.py --mode fed4 --chunks $n --steps 3 --warmup 1 --no-cpu-baseline \
    --host-inclusive off --ingest-leg off --mixed-leg off --concurrency-leg off --uploads-leg off > gpurun_out/fed/s4,3x_$n.json 2> gpurun_out/fed/s4,3x_$n.err || { echo FAIL; tail -5 gpurun_out/fed/s4,3x_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fed/s4,3x_$n.json'));print('fed 4,3x x $n', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
done
