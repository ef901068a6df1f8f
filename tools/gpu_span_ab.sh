#!/bin/bash
# A/B of span CRC builds on one device: bash tools/gpu_span_ab.sh <lib.so>... (default: the in-tree library)
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
LEGS="--steps 1 --warmup 0 --no-cpu-baseline --host-inclusive off --ingest-leg off --uploads-leg off --receiver-leg off --concurrency-leg off --mixed-leg off"
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    EFES_LIB_OVERRIDE=$PWD/$lib timeout -k 10 200 python bench.py $LEGS > gpurun_out/spanab_$n.json 2> gpurun_out/spanab_$n.err || { echo "$n failed"; tail -5 gpurun_out/spanab_$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/spanab_$n.json'))['span_crc']; print('$n', d['roofline']['achieved'], d['roofline']['ms_per_call'], d['crc_matches_zlib'])"
  done
done
