#!/bin/bash
# Uploads harness: lockstep request groups (stagger 0) vs staggered half-groups (stagger 1),
# interleaved on one device.  Usage (GPU box, repo root): bash tools/gpu_uploads_stagger.sh
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/uploads_stagger
for rep in 1 2; do
  for spec in "16 128 8192" "32 128 16384" "32 256 16384"; do
    for st in 0 1; do
      set -- $spec
      out=gpurun_out/uploads_stagger/T$1_K$2_U$3_s${st}_r$rep.json
      timeout -k 10 300 ./tools/bench_uploads $1 $3 4194304 32768 $2 262144 $st > $out 2> gpurun_out/up.err || { echo "FAIL $spec $st"; tail -5 gpurun_out/up.err; exit 1; }
      python3 -c "import json;d=json.load(open('$out'));print('T=$1 K=$2 U=$3 stagger=$st', d['value'], 'GiB/s', d['seconds'], 's', d['all_sums_equal'], d['errors'])"
    done
  done
done
