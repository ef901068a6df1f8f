# Kernel trace of planned mixed (configs[3]) runs: per-part kernel start/end and LDS per workgroup.
#   bash tools/gpu_mixed_trace.sh <force> ...
cd "${GRAFT_REPO_ROOT:?}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/mixtrace
for f in "$@"; do
  tag=$(echo "$f" | tr ':,' '_-')
  EFES_PLAN_FORCE=$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mixtrace/$tag -o run -- \
      python3 bench.py --workload mixed --steps 1 --warmup 0 --no-cpu-baseline --pool-gib 64 > gpurun_out/mixtrace/$tag.json 2> gpurun_out/mixtrace/$tag.err \
      || { echo "FAIL $f"; tail -5 gpurun_out/mixtrace/$tag.err; exit 1; }
  python - "$tag" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
path = glob.glob(f"gpurun_out/mixtrace/{tag}/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(path)) if "efes::" in r["Kernel_Name"] and "fill" not in r["Kernel_Name"]]
t0 = min(int(r["Start_Timestamp"]) for r in rows)
for r in rows:
    print(tag, r["Kernel_Name"].split("(")[0], "grid", r.get("Grid_Size_X"), "lds", r["LDS_Block_Size"],
          "start %.3f end %.3f s" % ((int(r["Start_Timestamp"]) - t0) / 1e9, (int(r["End_Timestamp"]) - t0) / 1e9))
PY
done
