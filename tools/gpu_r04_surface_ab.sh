#!/bin/bash
# Round 4: the bench's go_surface configuration (32 x 256 uploads, 8 192 x 4 MiB, 1 GiB... 8 GiB staging)
# with the reclaiming digest queue (65 536 slots) against one slot per chunk (EFES_DIGEST_SLOTS=32831),
# interleaved on one box, beside tools/bench_uploads.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_surface_ab}
mkdir -p "$O"
for rep in 1 2 3; do
  timeout -k 10 120 tools/bench_uploads 32 8192 4194304 32768 256 > "$O/uploads.$rep.json" || exit 1
  timeout -k 10 120 env EFES_DIGEST_SLOTS=32831 tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 > "$O/slots32831.$rep.json" || exit 1
  timeout -k 10 120 tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 > "$O/reclaim.$rep.json" || exit 1
  python3 - "$O" $rep <<'PY' | tee -a "$O/ab.log"
import json, sys
O, r = sys.argv[1], sys.argv[2]
u = json.load(open(f"{O}/uploads.{r}.json"))["value"]
a = json.load(open(f"{O}/slots32831.{r}.json"))
b = json.load(open(f"{O}/reclaim.{r}.json"))
print(f"rep {r}: uploads {u}  go_surface one-slot-per-chunk {a['value']} (launches {a['launches']})  reclaiming {b['value']} (launches {b['launches']})")
PY
done
