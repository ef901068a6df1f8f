#!/bin/bash
# Round 5: the clock meter (per-CU matched probe + amdsmi) against GRBM_GUI_ACTIVE on the same box,
# and WIDE's VALU per 64-B block on the final tree (SQ_INSTS_VALU over a configs[4] run).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_clock2}
mkdir -p "$O"
B="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off --latency-leg off --receiver-leg off --drain-leg off --concurrency-leg off --mixed-leg off"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $B > "$O/bench.$rep.json" 2> "$O/bench.$rep.err" || { tail -5 "$O/bench.$rep.err"; exit 1; }
  python3 - "$O/bench.$rep.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for name, leg in (("headline", d), ("ingest", d["ingest_config"]), ("span", d["span_crc"])):
    c = leg["clock"]; b = leg.get("binding_roofline") or {}
    print(f"{name:8s} value {leg['value']}  smi {c.get('smi_mhz_mean')}  probe {c.get('probe_mhz')} ({c.get('probe_cus')} CUs)  frac@clock {b.get('frac_at_clock')}")
PY
done
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv \
  -d "$O/pmc" -o run -- python3 bench.py $B --span-leg off > "$O/pmc.log" 2>&1 || { echo "pmc failed"; tail -5 "$O/pmc.log"; exit 1; }
python3 - "$O" <<'PY'
import csv, collections, statistics, sys
O = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f"{O}/pmc/run_counter_collection.csv")):
    k = r["Kernel_Name"].split("(")[0]
    if k not in ("efes::deep_kernel", "efes::wide_kernel"):
        continue
    ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    agg[k]["_ns"].append(ns)
for k, m in agg.items():
    med = {c: statistics.median(v) for c, v in m.items()}
    ghz = med["GRBM_GUI_ACTIVE"] / 8 / med["_ns"]
    print(f"{k}: kernel {med['_ns']/1e6:.2f} ms, GRBM clock {ghz*1000:.1f} MHz, SQ_INSTS_VALU {med['SQ_INSTS_VALU']:.4g}, "
          f"VALU busy {med['SQ_ACTIVE_INST_VALU']*4/1024/(med['GRBM_GUI_ACTIVE']/8):.3f}")
    if k == "efes::wide_kernel":
        # the ingest leg: launches of 196 608 and 131 072 x 1 MiB jobs, 64 lanes per wave
        blocks = [v for v in m["SQ_INSTS_VALU"]]
        print("  per launch SQ_INSTS_VALU:", [f"{v:.4g}" for v in blocks])
        print(f"  VALU per 64-B block per wave (196 608-job launches): {statistics.median([v for v in blocks if v > 3.0e10]) / (3072 * 16384):.1f}")
    else:
        print(f"  VALU per 64-B block per message: {med['SQ_INSTS_VALU'] / (1024 * 65536):.1f}")
PY
