#!/bin/bash
# A/B of WIDE builds on one device for the configs[4] ingest workload: bash tools/gpu_wide_ab.sh <lib.so>...
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for lib in "$@"; do
    for batch in 196608 262144; do
      n=$(basename $lib .so)_$batch
      EFES_LIB_OVERRIDE=$PWD/$lib timeout -k 10 200 python bench.py --workload ingest --ingest-batch $batch --warmup 1 --no-cpu-baseline \
        > gpurun_out/wideab_$n.json 2> gpurun_out/wideab_$n.err || { echo "$n failed"; tail -5 gpurun_out/wideab_$n.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/wideab_$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['config'].get('kernel'))"
    done
  done
done
