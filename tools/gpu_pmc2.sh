# Extra PMC passes (instruction cache, LDS/scalar activity): bash tools/gpu_pmc2.sh <tag> <bench args...>
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
i=10
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_IFETCH SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_${TAG}_$i -o run -- python3 bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off --warmup 1 "$@" > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
  python3 - "$TAG" "$i" <<'PY'
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
