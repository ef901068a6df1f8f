#!/bin/bash
# Round-end rehearsal of what the driver runs: the default bench line (N=1) and bench.py's N>1 code
# path with 2 ranks on device 0 (gloo barrier/max), each under its own time limit.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/final_bench.err; exit 1; }
cat gpurun_out/final_bench.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --all-ranks-on-device0 > gpurun_out/final_dist2.json 2> gpurun_out/final_dist2.err \
  || { echo "dist2 failed"; tail -5 gpurun_out/final_dist2.err; exit 1; }
cat gpurun_out/final_dist2.json
