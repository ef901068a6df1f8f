#!/bin/bash
# Round 6, second GPU pass (the multi-device harnesses, per-rank bench records, stale-error and
# enumeration tests, the reclaim change): the -m gpu suite, the default bench line, the N=2 rehearsal
# (gloo, both ranks on device 0: the per-rank records and the rehearsal flag), then ThreadSanitizer
# over the digest layer (build first: bash tools/tsan_build.sh).  Stops at the first failing step.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_check2}
mkdir -p "$O"
timeout -k 10 300 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || { tail -5 "$O/smoke.log"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --durations=15 --timeout 120 --timeout-method thread \
  > "$O/gpu_tests.log" 2>&1
rc=$?; tail -3 "$O/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; tail -20 "$O/bench.err"; exit 1; }
echo bench ok
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --all-ranks-on-device0 --ingest-scale 0.3 \
  > "$O/dist2.json" 2> "$O/dist2.err" || { echo "dist2 failed"; tail -20 "$O/dist2.err"; exit 1; }
echo dist2 ok
bash tools/gpu_r04_tsan.sh "$(basename "$O")/tsan"
