set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -40 gpurun_out/gpu_tests.log
exit $rc
