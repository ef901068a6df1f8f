#!/bin/bash
# FED4 with 1, 2 and 3 chain waves per producer (16/32/48 jobs: one workgroup), 4 MiB jobs.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/fed
for spec in "fed4 16" "fed4 32" "fed4 48" "group4 16" "deep 16" ${EXTRA}; do
  set -- $spec
  timeout -k 10 120 python bench.py --mode $1 --chunks $2 --steps 3 --warmup 1 --no-cpu-baseline --host-inclusive off \
    --ingest-leg off --mixed-leg off --concurrency-leg off --uploads-leg off > gpurun_out/fed/$1_$2.json 2> gpurun_out/fed/$1_$2.err || { echo "FAIL $spec"; tail -5 gpurun_out/fed/$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fed/$1_$2.json'));print('$1 $2', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
done
