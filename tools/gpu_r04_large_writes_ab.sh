#!/bin/bash
# Round 4: the Go surface across Write sizes with the library before any-size pair fusion
# (ab_old/libefeshash.so) against the current one, interleaved on one box, beside efes_upload.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_large_writes_ab}
mkdir -p "$O"
for rep in 1 2; do
  for w in 1460 32768 262144 1048576; do
    timeout -k 10 120 tools/bench_uploads 32 8192 4194304 $w 256 > "$O/uploads_w$w.$rep.json" || exit 1
    timeout -k 10 120 env LD_LIBRARY_PATH=$PWD/ab_old tools/bench_go_surface 32 8192 4194304 $w 256 1 256 8208 > "$O/old_w$w.$rep.json" || exit 1
    timeout -k 10 120 tools/bench_go_surface 32 8192 4194304 $w 256 1 256 8208 > "$O/new_w$w.$rep.json" || exit 1
    python3 - "$O" $w $rep <<'PY' | tee -a "$O/ab.log"
import json, sys
O, w, r = sys.argv[1:4]
u = json.load(open(f"{O}/uploads_w{w}.{r}.json"))["value"]
a = json.load(open(f"{O}/old_w{w}.{r}.json")); b = json.load(open(f"{O}/new_w{w}.{r}.json"))
print(f"rep {r} write {w}: uploads {u}  go_surface before {a['value']} ({a['value']/u:.3f} x, hashed/byte {a['hashed_bytes_per_byte']})  now {b['value']} ({b['value']/u:.3f} x, hashed/byte {b['hashed_bytes_per_byte']}, pairs {b['pairs']}, settles {b['settles']})  ok {a['all_equal'] and b['all_equal']}")
PY
  done
done
