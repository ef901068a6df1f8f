# Round-3 PMC passes of one bench.py workload, each counter set in its own kernel-trace-only run:
#   bash tools/gpu_pmc3.sh <tag> <bench args...>
# Summaries (median per kernel) -> gpurun_out/pmc_<tag>_summary.txt; raw CSVs under gpurun_out/pmc_<tag>_<i>/.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD" \
           "FETCH_SIZE" \
           "SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_SMEM SQ_THREAD_CYCLES_VALU SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_${TAG}_$i -o run -- \
    python3 bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off --concurrency-leg off \
    --uploads-leg off --receiver-leg off --span-leg off "$@" > gpurun_out/pmc_${TAG}_$i.log 2>&1 \
    || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
  python3 - "$TAG" "$i" >> gpurun_out/pmc_${TAG}_summary.txt <<'PY'
import csv, glob, sys, collections
tag, i = sys.argv[1], sys.argv[2]
rows = [r for f in glob.glob(f"gpurun_out/pmc_{tag}_{i}/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
agg = collections.defaultdict(list)
for r in rows:
    if "efes::" in r["Kernel_Name"] and "fill" not in r["Kernel_Name"]:
        agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:26s} {c:24s} n={len(v)} median={sorted(v)[len(v)//2]:.6g}")
PY
done
cat gpurun_out/pmc_${TAG}_summary.txt
