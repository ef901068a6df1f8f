#!/bin/bash
# Round 4: where the fused pair's leader Write waits for the follower's (EFES_PAIR_STAGE): in a
# per-thread scratch buffer with the follower staging by streaming stores (scratch, the default since
# this A/B), staged with ordinary stores (cached), or staged with streaming stores (stream).  The pair / Go-surface /
# boundary tests run under the scratch mode first; then the bench configuration, interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_pair_stage_ab}
mkdir -p "$O"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  EFES_PAIR_STAGE=scratch timeout -k 10 600 python -u -m pytest tests/test_gpu_pairs.py tests/test_gpu_go_surface.py tests/test_gpu_consumer.py \
    tests/test_gpu_boundary.py -x -q --timeout 200 --timeout-method thread > "$O/tests_scratch.log" 2>&1 || { tail -30 "$O/tests_scratch.log"; exit 1; }
  tail -1 "$O/tests_scratch.log"
fi
for rep in 1 2 3; do
  timeout -k 10 120 tools/bench_uploads 32 8192 4194304 32768 256 > "$O/uploads.$rep.json" || exit 1
  for m in cached stream scratch; do
    timeout -k 10 120 env EFES_PAIR_STAGE=$m tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 > "$O/$m.$rep.json" || exit 1
  done
  python3 - "$O" $rep <<'PY' | tee -a "$O/ab.log"
import json, sys
O, r = sys.argv[1], sys.argv[2]
u = json.load(open(f"{O}/uploads.{r}.json"))["value"]
v = {m: json.load(open(f"{O}/{m}.{r}.json")) for m in ("cached", "stream", "scratch")}
print(f"rep {r}: uploads {u}  " + "  ".join(f"{m} {d['value']}" for m, d in v.items())
      + f"  ok {all(d['all_equal'] for d in v.values())}")
PY
done
