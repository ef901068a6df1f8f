#!/bin/bash
# Round 4: ThreadSanitizer over the fused digest pairs (build first: bash tools/tsan_build.sh): the C
# consumer (resumable PATCHes + diverging pair scripts from 16 threads) on a 15-slot and a default
# digest queue, and the Go-surface harness with pairs evicted between their members' calls.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_tsan}
mkdir -p "$O"
export TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0 history_size=4 log_path=$O/tsan suppressions=$PWD/tools/tsan.supp"
timeout -k 10 180 ./tests/c/efes_consumer_test 16 6 > "$O/consumer_plain.log" 2>&1
rc=$?; echo "rc=$rc consumer (uninstrumented)"; tail -4 "$O/consumer_plain.log"; [ $rc -ne 0 ] && exit $rc
EFES_DIGEST_STAGING_MIB=1 EFES_DIGEST_SLOTS=15 timeout -k 10 400 ./tests/c/efes_consumer_test_tsan 16 4 > "$O/consumer_small.log" 2>&1
rc=$?; echo "rc=$rc consumer tsan (15 slots, eviction)"; tail -4 "$O/consumer_small.log"; [ $rc -ne 0 ] && [ $rc -ne 66 ] && exit $rc
EFES_DIGEST_STAGING_MIB=1 timeout -k 10 400 ./tests/c/efes_consumer_test_tsan 16 4 > "$O/consumer_reclaim.log" 2>&1
rc=$?; echo "rc=$rc consumer tsan (16 chunks, 65 536 slots: reclaim)"; tail -4 "$O/consumer_reclaim.log"; [ $rc -ne 0 ] && [ $rc -ne 66 ] && exit $rc
timeout -k 10 400 ./tests/c/efes_consumer_test_tsan 16 3 > "$O/consumer_default.log" 2>&1
rc=$?; echo "rc=$rc consumer tsan (default queue)"; tail -4 "$O/consumer_default.log"; [ $rc -ne 0 ] && [ $rc -ne 66 ] && exit $rc
EFES_DIGEST_STAGING_MIB=2 EFES_DIGEST_SLOTS=31 timeout -k 10 400 ./tools/bench_go_surface_tsan 16 128 1048576 32768 4 3 64 2 > "$O/go_surface_evict.json" 2> "$O/go_surface_evict.err"
rc=$?; echo "rc=$rc go_surface tsan (31 slots: eviction)"; cat "$O/go_surface_evict.json"; [ $rc -ne 0 ] && [ $rc -ne 66 ] && exit $rc
EFES_DIGEST_STAGING_MIB=2 timeout -k 10 400 ./tools/bench_go_surface_tsan 16 128 1048576 32768 4 3 64 2 > "$O/go_surface.json" 2> "$O/go_surface.err"
rc=$?; echo "rc=$rc go_surface tsan (32 chunks, 65 536 slots: reclaim, 64 pairs open)"; cat "$O/go_surface.json"; [ $rc -ne 0 ] && [ $rc -ne 66 ] && exit $rc
python3 - "$O" <<'PY'
import glob, re, sys
n = ours = 0
for f in glob.glob(sys.argv[1] + "/tsan.*"):
    for r in open(f).read().split("WARNING: ThreadSanitizer")[1:]:
        n += 1
        accesses = re.split(r"\n  (?:Previous )?(?:atomic )?(?:[Ww]rite|[Rr]ead)", r)[1:]
        tops = []
        for a in accesses:
            frames = [l for l in a.splitlines() if re.match(r"\s+#\d", l) and "tsan_" not in l]
            tops.append(frames[0] if frames else "")
        if any("efes_amd/csrc" in t or "efes_hash.h" in t or "bench_go_surface.cpp" in t or "efes_consumer_test" in t
               for t in tops):
            ours += 1
            print("\n".join(r.splitlines()[:30]))
print(f"ThreadSanitizer: {n} reports after suppressions, {ours} with an access in efes code")
PY
