#!/bin/bash
# A/B of the per-upload staging cap (EFES_QUEUE_AHEAD) and of the staging size per request thread
# (EFES_BENCH_CHUNKS_PER_UPLOAD) on the receiver, interleaved, 3 repeats:
#   bash tools/gpu_queue_ahead_ab.sh
cd "${GRAFT_REPO_ROOT:?}" || exit 1
OUT=gpurun_out/queue_ahead; mkdir -p $OUT
D=/dev/shm/efes_ab_$$; mkdir -p "$D" || exit 1
trap 'rm -rf "$D"' EXIT
M=$((4 << 20))
for rep in 1 2 3; do
  for AC in "0 4" "3 4" "0 6" "3 6" "3 8"; do
    set -- $AC; A=$1; C=$2
    for cfg in "64 $M" "256 $M" "256 $((1 << 20))" "1024 $M" "1024 $((1 << 20))"; do
      set -- $cfg
      tag=a${A}_c${C}_t$1_p$2_r$rep
      EFES_QUEUE_AHEAD=$A EFES_BENCH_CHUNKS_PER_UPLOAD=$C timeout -k 10 120 ./tools/bench_receiver receiver "$D" $1 $((4096 / $1)) $M $2 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "FAIL $tag"; exit 1; }
      echo "$tag $(python3 -c "import json,sys;print(json.load(open(sys.argv[1]))['value'])" $OUT/$tag.json)"
    done
  done
done
echo ALL_DONE
