#!/bin/bash
# Span CRC rate against the workgroup count (EFES_SPAN_GROUPS), one bench leg each.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
LEGS="--steps 1 --warmup 0 --no-cpu-baseline --host-inclusive off --ingest-leg off --uploads-leg off --receiver-leg off --concurrency-leg off --mixed-leg off"
for g in 256 512 128 384; do
  EFES_SPAN_GROUPS=$g timeout -k 10 200 python bench.py $LEGS > gpurun_out/span_g$g.json 2> gpurun_out/span_g$g.err || { echo "groups $g failed"; tail -5 gpurun_out/span_g$g.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/span_g$g.json'))['span_crc']; print($g, d['roofline'], d['crc_matches_zlib'])"
done
