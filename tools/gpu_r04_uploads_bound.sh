#!/bin/bash
# Round 4: is the server path (efes_upload / the Go surface) bound by the host writers or by the
# kernels' PCIe reads?  Writer threads and Write size swept at 8 192 uploads x 4 MiB in flight.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_uploads_bound}
mkdir -p "$O"
for cfg in "16 32768" "32 32768" "64 32768" "32 262144" "64 262144" "32 1048576"; do
  set -- $cfg
  timeout -k 10 120 tools/bench_uploads $1 8192 4194304 $2 $((8192 / $1)) > "$O/uploads_t$1_w$2.json" || exit 1
  timeout -k 10 120 tools/bench_go_surface $1 8192 4194304 $2 $((8192 / $1)) 1 256 8208 > "$O/go_t$1_w$2.json" || exit 1
  python3 - "$O" $1 $2 <<'PY' | tee -a "$O/sweep.log"
import json, sys
O, t, w = sys.argv[1:4]
u = json.load(open(f"{O}/uploads_t{t}_w{w}.json")); g = json.load(open(f"{O}/go_t{t}_w{w}.json"))
print(f"threads {t} write {w}: uploads {u['value']} GiB/s launches {u.get('launches')} | go_surface {g['value']} launches {g['launches']} jobs/launch {g['jobs']/g['launches']:.0f} ok {g['all_equal']}")
PY
done
