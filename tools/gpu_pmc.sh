# PMC passes (each its own run, kernel-trace only): bash tools/gpu_pmc.sh <tag> <bench args...>
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_${TAG}_$i -o run -- python3 bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off --concurrency-leg off --uploads-leg off --warmup 1 "$@" > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
  python3 - "$TAG" "$i" <<'PY'
import csv, glob, sys, collections
tag, i = sys.argv[1], sys.argv[2]
rows = [r for f in glob.glob(f"gpurun_out/pmc_{tag}_{i}/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
agg = collections.defaultdict(list)
for r in rows:
    if "efes::" in r["Kernel_Name"] and "fill" not in r["Kernel_Name"]:
        agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:22s} {c:24s} n={len(v)} median={sorted(v)[len(v)//2]:.6g}")
PY
done
