# Run the uploads harness under ThreadSanitizer (build first: bash tools/tsan_build.sh):
# concurrent writers, the dispatcher thread and the per-upload sync points on the real GPU.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
export TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0 history_size=4 log_path=gpurun_out/tsan suppressions=$PWD/tools/tsan.supp"
for spec in "8 512 1048576 32768 32 262144" "16 256 262144 4096 16 65536"; do
  timeout -k 10 300 ./tools/bench_uploads_tsan $spec > gpurun_out/tsan_run.json 2> gpurun_out/tsan_run.err
  rc=$?; echo "rc=$rc $spec"; cat gpurun_out/tsan_run.json; tail -3 gpurun_out/tsan_run.err
  [ $rc -ne 0 ] && [ $rc -ne 66 ] && exit $rc
done
# the Go-surface digests (efes_stream.cpp) with a 15-slot digest queue: 16 request threads x 2
# digests each keep the slots short, so Writes evict idle digests of other threads all the time
EFES_DIGEST_STAGING_MIB=1 timeout -k 10 300 ./tests/c/efes_consumer_test_tsan 16 4 > gpurun_out/tsan_consumer.log 2>&1
rc=$?; echo "rc=$rc consumer (EFES_DIGEST_STAGING_MIB=1)"; tail -2 gpurun_out/tsan_consumer.log
[ $rc -ne 0 ] && [ $rc -ne 66 ] && exit $rc
# a report counts when the first non-interceptor frame of either access is in efes code
python3 - <<'PY'
import glob, re
n = ours = 0
for f in glob.glob("gpurun_out/tsan.*"):
    for r in open(f).read().split("WARNING: ThreadSanitizer")[1:]:
        n += 1
        accesses = re.split(r"\n  (?:Previous )?(?:atomic )?(?:[Ww]rite|[Rr]ead)", r)[1:]
        tops = []
        for a in accesses:
            frames = [l for l in a.splitlines() if re.match(r"\s+#\d", l) and "tsan_" not in l]
            tops.append(frames[0] if frames else "")
        if any("efes_amd/csrc" in t or "efes_hash.h" in t or "bench_uploads.cpp" in t or "efes_consumer_test" in t
               for t in tops):
            ours += 1
            print("\n".join(r.splitlines()[:20]))
print(f"ThreadSanitizer: {n} reports after suppressions, {ours} with an access in efes code")
PY
