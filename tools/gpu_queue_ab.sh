#!/bin/bash
# A/B of two library builds on the concurrent-upload paths (same device, interleaved):
#   bash tools/gpu_queue_ab.sh libA.so libB.so      (files under efes_amd/lib/)
# Each build is put first on LD_LIBRARY_PATH (the tools' RUNPATH comes after it).
cd "${GRAFT_REPO_ROOT:?}" || exit 1
OUT=gpurun_out/queue_ab; mkdir -p $OUT
D=/dev/shm/efes_qab_$$; mkdir -p $D || exit 1
trap 'rm -rf "$D" "$OUT"/lib_*' EXIT
for v in "$@"; do mkdir -p $OUT/lib_$v && cp efes_amd/lib/$v $OUT/lib_$v/libefeshash.so; done
M=$((4 << 20))
for rep in 1 2; do
  for v in "$@"; do
    L=$PWD/$OUT/lib_$v
    for t in "sha1file $D 256 2 $((16 << 20))" "receiver $D 1024 2 $M $M" "receiver $D 256 4 $M $M"; do
      r=$(LD_LIBRARY_PATH=$L timeout -k 10 120 ./tools/bench_receiver $t 2>>$OUT/err.log) || { echo "FAIL $v $t"; tail -3 $OUT/err.log; exit 1; }
      echo "$v | $t | $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "GiB/s", d["seconds"], "s", d["all_sums_equal"])')"
    done
    r=$(LD_LIBRARY_PATH=$L timeout -k 10 120 ./tools/bench_uploads 32 8192 $M 32768 256 2>>$OUT/err.log) || { echo "FAIL $v uploads"; exit 1; }
    echo "$v | uploads 32x256 | $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "GiB/s", d["all_sums_equal"])')"
  done
done
echo ALL_DONE
