cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
timeout -k 10 1100 python bench.py --workload ingest --ingest-batch 131072 --warmup 0 --progress > gpurun_out/cfg_ingest.json 2> gpurun_out/cfg_ingest.err; rc=$?
echo "ingest rc=$rc"; cat gpurun_out/cfg_ingest.json; grep -v amdgpu gpurun_out/cfg_ingest.err | tail -5; exit $rc
