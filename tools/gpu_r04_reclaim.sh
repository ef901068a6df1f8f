#!/bin/bash
# Round 4: the digest queue with more upload slots than staging chunks (dispatcher reclaim of idle
# holders' partly filled chunks) against round 3's one-slot-per-chunk queue, over-subscribed; then
# the bench configuration; then the digest-surface tests in both regimes.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_reclaim}
mkdir -p "$O"
run() {  # tag env... cmd...
  local tag=$1; shift
  timeout -k 10 200 env "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { echo "FAIL $tag"; tail -3 "$O/$tag.err"; return 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], 'GiB/s settles', d['settles'], 'pairs', d['pairs'], 'hashed/byte', d['hashed_bytes_per_byte'], 'launches', d['launches'], 'jobs', d['jobs'], 'patch p50/p99 ms', d['patch_group_ms']['p50'], d['patch_group_ms']['p99'], 'ok', d['all_equal'])" "$O/$tag.json" "$tag" | tee -a "$O/reclaim.log"
}
for rep in 1 2; do
  run k256_t32_u16384_slots4095 EFES_DIGEST_SLOTS=4095 tools/bench_go_surface 32 16384 4194304 32768 256 1 256 1024 || exit 1
  run k256_t32_u16384_reclaim tools/bench_go_surface 32 16384 4194304 32768 256 1 256 1024 || exit 1
  run k1_t64_chunks16_slots15 EFES_DIGEST_SLOTS=15 EFES_DIGEST_STAGING_MIB=4 tools/bench_go_surface 64 384 4194304 32768 1 1 || exit 1
  run k1_t64_chunks16_reclaim EFES_DIGEST_STAGING_MIB=4 tools/bench_go_surface 64 384 4194304 32768 1 1 || exit 1
  run bench_config tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 || exit 1
  run k64_t32_default tools/bench_go_surface 32 4096 4194304 32768 64 1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairs.py tests/test_gpu_boundary.py tests/test_gpu_consumer.py \
  tests/test_gpu_go_surface.py -v --durations=5 --timeout 200 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; tail -15 "$O/tests.log"; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r04_tsan.sh r04_tsan_reclaim
