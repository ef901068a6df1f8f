#!/bin/bash
# FED shapes: cycle accounting (diagnostic build) and bench timings per shape (EFES_FED_SHAPE "G,C").
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/fed
for spec in "4,2 32" "4,3 48" "8,3 24"; do
  set -- $spec
  echo "== shape $1, $2 jobs (stats build)"
  EFES_FED_SHAPE=$1 EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/libefeshash_stats.so timeout -k 10 100 python tools/fed_stats.py $2 || exit 1
done
for spec in "4,2 32" "4,2 8192" "4,3 12288" "8,3 6144"; do
  set -- $spec
  EFES_FED_SHAPE=$1 timeout -k 10 120 python bench.py --mode fed4 --chunks $2 --steps 3 --warmup 1 --no-cpu-baseline \
    --host-inclusive off --ingest-leg off --mixed-leg off --concurrency-leg off --uploads-leg off > gpurun_out/fed/s$1_$2.json 2> gpurun_out/fed/s$1_$2.err || { echo "FAIL $spec"; tail -5 gpurun_out/fed/s$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fed/s$1_$2.json'));print('fed $1 x $2', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
done
