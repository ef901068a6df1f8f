#!/bin/bash
# Receiver (saveFile through ServeHTTP, files + fsync + GPU hashing) and Sha1File read-back rates
# on one MI355X, native threads:  bash tools/gpu_receiver.sh [dir]
cd "${GRAFT_REPO_ROOT:?}" || exit 1
OUT=gpurun_out/receiver; mkdir -p $OUT
D=${1:-/dev/shm}
df -h "$D" /tmp > $OUT/df.txt 2>&1
D=$D/efes_bench_$$; mkdir -p "$D" || exit 1
trap 'rm -rf "$D"' EXIT
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 120 ./tools/bench_receiver "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "FAIL $tag"; tail -5 $OUT/$tag.err; exit 1; }
  echo "$tag $(cat $OUT/$tag.json)"
}
M=$((4 << 20))
run recv_t64_p1m   receiver "$D" 64  4 $M $((1 << 20))
run recv_t256_p1m  receiver "$D" 256 4 $M $((1 << 20))
run recv_t256_p4m  receiver "$D" 256 4 $M $M
run recv_t512_p4m  receiver "$D" 512 4 $M $M
run recv_t1024_p4m receiver "$D" 1024 2 $M $M
run sf_t1_16m      sha1file "$D" 1   2 $((16 << 20))
run sf_t64_16m     sha1file "$D" 64  2 $((16 << 20))
run sf_t256_16m    sha1file "$D" 256 2 $((16 << 20))
run sf_t1024_4m    sha1file "$D" 1024 2 $M
run files_t256     files "$D" 256 2 $M
run files_t1024    files "$D" 1024 2 $M
echo ALL_DONE
