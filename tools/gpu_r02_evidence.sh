#!/bin/bash
# Round-2 evidence on one device: FETCH_SIZE of the metric's kernel, PMC passes of FED4 at 8192 jobs,
# and the N>1 code path of bench.py (2 ranks on device 0, gloo barrier/max).
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_round.sh r02 pmc || exit 1
bash tools/gpu_pmc.sh fed4 --mode fed4 --chunks 8192 --steps 3 > gpurun_out/pmc_fed4_summary.txt 2>&1 || { tail -5 gpurun_out/pmc_fed4_summary.txt; exit 1; }
cat gpurun_out/pmc_fed4_summary.txt
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --all-ranks-on-device0 > gpurun_out/dist2_r02.json 2> gpurun_out/dist2_r02.err \
  || { echo "dist2 failed"; tail -5 gpurun_out/dist2_r02.err; exit 1; }
cat gpurun_out/dist2_r02.json
