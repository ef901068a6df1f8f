#!/bin/bash
# Round 4: small Writes (a socket read returns what has arrived, often far less than io.Copy's
# 32 KiB buffer): efes_upload vs the Go surface at 1460 B .. 32 KiB Writes, 8 192 uploads x 1 MiB.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_small_writes}
mkdir -p "$O"
for w in 1460 4096 8192 16384 32768; do
  timeout -k 10 120 tools/bench_uploads 32 8192 1048576 $w 256 > "$O/uploads_w$w.json" || exit 1
  timeout -k 10 120 tools/bench_go_surface 32 8192 1048576 $w 256 1 256 8208 > "$O/go_w$w.json" || exit 1
  python3 - "$O" $w <<'PY' | tee -a "$O/sweep.log"
import json, sys
O, w = sys.argv[1:3]
u = json.load(open(f"{O}/uploads_w{w}.json")); g = json.load(open(f"{O}/go_w{w}.json"))
print(f"write {w}: uploads {u['value']} GiB/s | go_surface {g['value']} ({g['value']/u['value']:.3f} x) pairs {g['pairs']} settles {g['settles']} hashed/byte {g['hashed_bytes_per_byte']} ok {g['all_equal'] and u['all_sums_equal']}")
PY
done
