#!/bin/bash
# Round 5: what bounds the span kernel at its clock -- SQ counters over the span leg (LDS
# instructions, bank-conflict cycles, LDS / VALU activity, wave cycles), two passes of <= 8 SQ counters.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_span_pmc}
mkdir -p "$O"
B="python3 bench.py --no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off \
 --latency-leg off --receiver-leg off --drain-leg off --concurrency-leg off --mixed-leg off --ingest-leg off --steps 2 --warmup 1"
i=0
for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d "$O/pmc_$i" -o run -- $B > "$O/pmc_$i.log" 2>&1 \
    || { echo "pass $i failed"; tail -5 "$O/pmc_$i.log"; exit 1; }
done
python3 - "$O" <<'PY'
import csv, collections, glob, statistics, sys
O = sys.argv[1]
agg = collections.defaultdict(list)
ns = []
for f in glob.glob(f"{O}/pmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if not r["Kernel_Name"].startswith("efes::span_kernel"):
            continue
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if d < 1_000_000:  # the 16 GiB launches only (not the 1 GiB check)
            continue
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        ns.append(d)
med = {k: statistics.median(v) for k, v in agg.items()}
for k, v in sorted(med.items()):
    print(f"{k:24s} {v:.6g}")
print("kernel ns (median):", statistics.median(ns))
PY
