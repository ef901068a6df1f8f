#!/bin/bash
# Round 4: eviction patience (EFES_DIGEST_EVICT_MS, default 50; 0 = round 3's evict-at-once) with the
# digest queue over-subscribed -- one pair per request thread (64 threads on 15 slots) and 256 pairs
# per thread (8 192 on 4 095 slots) -- and the new default queue (1 GiB, 256 KiB chunks) below its
# slots; then the digest-surface tests (their time included).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_evict}
mkdir -p "$O"
run() {  # tag env... -- args
  local tag=$1; shift
  env "$@" > /dev/null 2>&1  # (env validity)
  timeout -k 10 200 env "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { echo "FAIL $tag"; tail -3 "$O/$tag.err"; return 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], 'GiB/s settles', d['settles'], 'pairs', d['pairs'], 'patch p50/p99 ms', d['patch_group_ms']['p50'], d['patch_group_ms']['p99'], 'ok', d['all_equal'])" "$O/$tag.json" "$tag" | tee -a "$O/evict.log"
}
for ms in 0 50; do
  run k1_t64_slots15_ms$ms EFES_DIGEST_EVICT_MS=$ms EFES_DIGEST_STAGING_MIB=4 tools/bench_go_surface 64 384 4194304 32768 1 1 || exit 1
  run k256_t32_slots4095_ms$ms EFES_DIGEST_EVICT_MS=$ms tools/bench_go_surface 32 16384 4194304 32768 256 1 256 1024 || exit 1
done
run k64_t32_default tools/bench_go_surface 32 4096 4194304 32768 64 1 256 1024 || exit 1
run k16_t32_default tools/bench_go_surface 32 1024 4194304 32768 16 1 256 1024 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairs.py tests/test_gpu_boundary.py tests/test_gpu_consumer.py \
  tests/test_gpu_go_surface.py -v --durations=0 --timeout 200 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; tail -25 "$O/tests.log"; exit $rc
