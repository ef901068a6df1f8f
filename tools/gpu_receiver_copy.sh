#!/bin/bash
# Receiver vs its host ceiling (the same io.Copy without hashing) on one MI355X:
#   bash tools/gpu_receiver_copy.sh [dir]
cd "${GRAFT_REPO_ROOT:?}" || exit 1
OUT=gpurun_out/receiver_copy; mkdir -p $OUT
D=${1:-/dev/shm}
D=$D/efes_bench_$$; mkdir -p "$D" || exit 1
trap 'rm -rf "$D"' EXIT
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 120 ./tools/bench_receiver "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "FAIL $tag"; tail -5 $OUT/$tag.err; exit 1; }
  echo "$tag $(cat $OUT/$tag.json)"
}
M=$((4 << 20))
for T in 64 256 1024; do
  run copy_t$T       copy     "$D" $T $((4096 / T)) $M
  run recv_t${T}_p4m receiver "$D" $T $((4096 / T)) $M $M
  run recv_t${T}_p1m receiver "$D" $T $((4096 / T)) $M $((1 << 20))
done
echo ALL_DONE
