# Round 5: calibrate the clock probe.  s_memtime vs s_memrealtime in a sleeping one-wave probe
# (idle chip, and beside an all-CU VALU kernel), amdsmi's gfxclk polled meanwhile, and
# GRBM_GUI_ACTIVE of the same busy kernel from a rocprofv3 counter pass.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/r05_clock; export TMPDIR=/tmp
O=gpurun_out/r05_clock
timeout -k 10 120 python3 tools/clock_smi.py $O/smi.jsonl -- tools/microbench/mb_clock ${1:-1000000} 3 > $O/probe.log 2>&1 || { echo "probe failed"; cat $O/probe.log; exit 1; }
cat $O/probe.log
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/pmc -o run -- tools/microbench/mb_clock ${1:-1000000} 1 > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r05_clock/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        v = float(r["Counter_Value"])
        extra = f"  -> {v / 8 / ns:.3f} GHz" if r["Counter_Name"] == "GRBM_GUI_ACTIVE" else ""
        print(r["Kernel_Name"][:20], r["Counter_Name"], v, ns, extra)
PY
