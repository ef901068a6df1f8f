# Full-size BASELINE configs beyond the default: concurrent uploads, mixed (configs[3]).
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload uploads > gpurun_out/cfg_uploads.json 2> gpurun_out/cfg_uploads.err; rc=$?
echo "uploads rc=$rc"; cat gpurun_out/cfg_uploads.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/cfg_uploads.err; exit $rc; }
timeout -k 10 600 python bench.py --workload mixed --mixed-chunks 65536 --warmup 0 --progress > gpurun_out/cfg_mixed.json 2> gpurun_out/cfg_mixed.err; rc=$?
echo "mixed rc=$rc"; cat gpurun_out/cfg_mixed.json; tail -3 gpurun_out/cfg_mixed.err; exit $rc
