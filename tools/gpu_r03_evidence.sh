# Round-3 evidence on one GPU box: -m gpu suite, default bench line, rocprof kernel stats of the
# headline + configs[1] + configs[4] legs, FETCH_SIZE of the SHA-1-only headline, N=2 rehearsal.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py \
  --steps 10 --warmup 2 --no-cpu-baseline --host-inclusive off --mixed-leg off --concurrency-leg off --uploads-leg off \
  --receiver-leg off --span-leg off --drain-leg off > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err \
  || { tail -5 gpurun_out/prof_$TAG.err; exit 1; }
echo prof ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_sha1_$TAG -o run -- python3 bench.py \
  --sha1-only --steps 5 --warmup 1 --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off --concurrency-leg off \
  --uploads-leg off --receiver-leg off --span-leg off --drain-leg off --sha1-leg off > gpurun_out/pmc_sha1_$TAG.log 2>&1 \
  || { tail -5 gpurun_out/pmc_sha1_$TAG.log; exit 1; }
echo pmc ok
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --all-ranks-on-device0 --ingest-scale 0.3 \
  > gpurun_out/dist2_$TAG.json 2> gpurun_out/dist2_$TAG.err || { tail -20 gpurun_out/dist2_$TAG.err; exit 1; }
echo dist2 ok
