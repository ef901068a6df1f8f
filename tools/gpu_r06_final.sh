#!/bin/bash
# Round 6 evidence on the final tree: smoke, the -m gpu suite, the default bench line, rocprofv3 kernel
# stats of the headline + configs[1] + configs[4] + span legs (the same bench command with the other
# legs off), the N=2 rehearsal (gloo, both ranks on device 0).  Stops at the first failing step.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r06f}
mkdir -p "$O"
timeout -k 10 300 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || { tail -5 "$O/smoke.log"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --durations=15 --timeout 120 --timeout-method thread \
  > "$O/gpu_tests.log" 2>&1
rc=$?; tail -3 "$O/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; tail -20 "$O/bench.err"; exit 1; }
echo bench ok
LEGS_OFF="--no-cpu-baseline --host-inclusive off --mixed-leg off --concurrency-leg off --uploads-leg off --go-surface-leg off \
 --latency-leg off --receiver-leg off --drain-leg off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py \
  --steps 10 --warmup 2 $LEGS_OFF > "$O/prof.json" 2> "$O/prof.err" || { echo "prof failed"; tail -5 "$O/prof.err"; exit 1; }
echo prof ok
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --all-ranks-on-device0 --ingest-scale 0.3 \
  > "$O/dist2.json" 2> "$O/dist2.err" || { echo "dist2 failed"; tail -20 "$O/dist2.err"; exit 1; }
echo dist2 ok
