#!/bin/bash
# Round 4: WIDE's LDS bank conflicts priced with the same kernel on bank-deciding data
# (tools/wide_lds_probe.py): time, then per mode the clock and LDS counters of the launches.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:?}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_lds_probe}
mkdir -p "$O"
for rep in 1 2; do
  timeout -k 10 300 python3 tools/wide_lds_probe.py random conflict_free same_bank random conflict_free | tee -a "$O/time.log"
done
for mode in random conflict_free same_bank; do
  timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    --output-format csv -d "$O/pmc_$mode" -o run -- python3 tools/wide_lds_probe.py $mode > "$O/pmc_$mode.log" 2>&1
  python3 - "$O" "$mode" <<'PY' | tee -a "$O/clock.log"
import csv, glob, sys, collections, statistics
O, mode = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(f"{O}/pmc_{mode}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wide_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                agg["_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
m = {k: statistics.median(v) for k, v in agg.items()}
print(f"{mode:14s} kernel {m['_ns']/1e6:.2f} ms  clock {m['GRBM_GUI_ACTIVE']/8/m['_ns']:.3f} GHz  "
      f"VALU busy {m['SQ_ACTIVE_INST_VALU']*4/1024/(m['GRBM_GUI_ACTIVE']/8):.3f}  VALU/block {m['SQ_INSTS_VALU']/(3072*16384):.1f}  "
      f"LDS conflicts/instr {m['SQ_LDS_BANK_CONFLICT']/m['SQ_INSTS_LDS']:.2f}  LDS array cycles/instr {m['SQ_LDS_IDX_ACTIVE']/m['SQ_INSTS_LDS']:.2f}")
PY
done
