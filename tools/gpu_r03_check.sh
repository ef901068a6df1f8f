# Round-3 check on one GPU box: the whole -m gpu suite, the default bench line, and the N=2 path
# rehearsed with 2 gloo ranks on device 0 (ingest leg at every N).
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
TAG=${1:-r03}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo bench ok
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --all-ranks-on-device0 --ingest-scale 0.3 \
  > gpurun_out/dist2_$TAG.json 2> gpurun_out/dist2_$TAG.err || { tail -20 gpurun_out/dist2_$TAG.err; exit 1; }
echo dist2 ok
