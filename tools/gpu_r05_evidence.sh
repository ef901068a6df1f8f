#!/bin/bash
# Round-5 evidence on one GPU box (the final tree): smoke, the -m gpu suite, the default bench line,
# rocprofv3 kernel stats of the headline + configs[1] + configs[4] legs, FETCH_SIZE of the fused
# headline, of the SHA-1-only configs[1] and of one configs[4]-geometry WIDE launch (196 608 x 1 MiB),
# and the N=2 rehearsal (gloo, both ranks on device 0).  Stops at the first failing step.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:?}"
export TMPDIR=/tmp
TAG=${1:-r05}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
tail -2 "$O/gpu_tests.log"
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err"
echo bench ok
LEGS_OFF="--no-cpu-baseline --host-inclusive off --mixed-leg off --concurrency-leg off --uploads-leg off --go-surface-leg off \
 --latency-leg off --receiver-leg off --span-leg off --drain-leg off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py \
  --steps 10 --warmup 2 $LEGS_OFF > "$O/prof.json" 2> "$O/prof.err"
echo prof ok
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fused" -o run -- python3 bench.py \
  --steps 5 --warmup 1 $LEGS_OFF --ingest-leg off --sha1-leg off > "$O/pmc_fused.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_sha1" -o run -- python3 bench.py \
  --sha1-only --steps 5 --warmup 1 $LEGS_OFF --ingest-leg off --sha1-leg off > "$O/pmc_sha1.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_wide" -o run -- python3 bench.py \
  --chunks 196608 --chunk-bytes 1048576 --mode wide --steps 3 --warmup 1 $LEGS_OFF --ingest-leg off --sha1-leg off \
  > "$O/pmc_wide.log" 2>&1
echo pmc ok
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --all-ranks-on-device0 --ingest-scale 0.3 \
  > "$O/dist2.json" 2> "$O/dist2.err"
echo dist2 ok
