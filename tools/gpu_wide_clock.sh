# WIDE on distinct data (196 608 x 1 MiB) with and without pacing: the clock (GRBM_GUI_ACTIVE),
# VALU activity, and the per-wave timeline (diagnostic build).
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
for pace in 0 1; do
  EFES_WIDE_PACE=$pace timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES \
    --output-format csv -d gpurun_out/pmc_clock_p$pace -o run -- python3 bench.py --no-cpu-baseline --host-inclusive off \
    --ingest-leg off --mixed-leg off --concurrency-leg off --uploads-leg off --receiver-leg off --span-leg off --sha1-leg off \
    --drain-leg off --chunks 196608 --chunk-bytes 1048576 --mode wide --steps 3 --warmup 1 > gpurun_out/pmc_clock_p$pace.log 2>&1 \
    || { echo "pmc $pace failed"; tail -3 gpurun_out/pmc_clock_p$pace.log; exit 1; }
  python3 - $pace <<'PY'
import csv, sys, collections, statistics
p = sys.argv[1]
rows = [r for r in csv.DictReader(open(f"gpurun_out/pmc_clock_p{p}/run_counter_collection.csv")) if "wide_kernel" in r["Kernel_Name"]]
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    agg["_ns"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
m = {k: statistics.median(v) for k, v in agg.items()}
ghz = m["GRBM_GUI_ACTIVE"] / 8 / m["_ns"]
busy = m["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (m["GRBM_GUI_ACTIVE"] / 8)
print(f"pace={p} kernel {m['_ns']/1e6:.2f} ms  clock {ghz:.3f} GHz  VALU busy {busy:.3f}  VALU/block {m['SQ_INSTS_VALU']/(3072*16384):.1f}")
PY
done | tee gpurun_out/wide_clock.log
for pace in 0 1; do
  EFES_WIDE_PACE=$pace EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/libefeshash_widestats.so timeout -k 10 200 python tools/wide_stats.py 196608 1048576 200 > gpurun_out/ws_pace$pace.json 2> gpurun_out/ws_pace$pace.err || exit 1
  cat gpurun_out/ws_pace$pace.json
done
