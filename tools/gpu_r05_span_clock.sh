#!/bin/bash
# Round 5: the span leg's clock three ways -- the bench's meter (per-CU s_memtime probe, amdsmi)
# outside the profiler, then GRBM_GUI_ACTIVE / 8 / kernel ns per span_kernel dispatch under
# rocprofv3 --pmc with the meter running in the same process.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_span_clock}
mkdir -p "$O"
B="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off --latency-leg off \
 --receiver-leg off --drain-leg off --concurrency-leg off --mixed-leg off --ingest-leg off --steps 2 --warmup 1"
show() {
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["span_crc"]
c = d["clock"]
print(f"span {d['value']} GiB/s  probe {c.get('probe_mhz')} MHz ({c.get('probe_cus')} CUs, {c.get('probe_seconds')} s)  "
      f"smi mean {c.get('smi_mhz_mean')} (n={c.get('smi_samples')})")
PY
}
timeout -k 10 200 python3 bench.py $B > "$O/bench.json" 2> "$O/bench.err" || { tail -5 "$O/bench.err"; exit 1; }
show "$O/bench.json"
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d "$O/pmc" -o run -- \
  python3 bench.py $B > "$O/pmc_bench.json" 2> "$O/pmc.err" || { echo "pmc failed"; tail -5 "$O/pmc.err"; exit 1; }
show "$O/pmc_bench.json"
python3 - "$O" <<'PY'
import csv, collections, sys
rows = collections.defaultdict(dict)
for r in csv.DictReader(open(f"{sys.argv[1]}/pmc/run_counter_collection.csv")):
    if not r["Kernel_Name"].startswith("efes::span_kernel"):
        continue
    key = r.get("Dispatch_Id") or r.get("Correlation_Id")
    rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
    rows[key]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, m in sorted(rows.items(), key=lambda x: int(x[0])):
    print(f"dispatch {k}: {m['_ns']/1e6:.3f} ms  GRBM clock {m['GRBM_GUI_ACTIVE']/8/m['_ns']*1000:.1f} MHz  "
          f"SQ_BUSY_CYCLES/8/ns {m.get('SQ_BUSY_CYCLES', 0)/8/m['_ns']*1000:.1f}")
PY
