#!/bin/bash
# Round 4: the fused pair's leader staging with ordinary stores (default since this A/B, so the
# follower's memcmp hits the cache) vs streaming stores (EFES_PAIR_STAGE=stream), interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_pair_stage_ab}
mkdir -p "$O"
for rep in 1 2 3; do
  timeout -k 10 120 tools/bench_uploads 32 8192 4194304 32768 256 > "$O/uploads.$rep.json" || exit 1
  timeout -k 10 120 env EFES_PAIR_STAGE=stream tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 > "$O/nt.$rep.json" || exit 1
  timeout -k 10 120 tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 > "$O/cached.$rep.json" || exit 1
  python3 - "$O" $rep <<'PY' | tee -a "$O/ab.log"
import json, sys
O, r = sys.argv[1], sys.argv[2]
u = json.load(open(f"{O}/uploads.{r}.json"))["value"]
a = json.load(open(f"{O}/nt.{r}.json"))
b = json.load(open(f"{O}/cached.{r}.json"))
print(f"rep {r}: uploads {u}  go_surface streaming stores {a['value']}  ordinary stores {b['value']}  ok {a['all_equal'] and b['all_equal']}")
PY
done
