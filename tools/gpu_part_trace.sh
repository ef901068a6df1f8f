# Kernel trace of planned configs[3] in a fresh process: per-part start/end with CU-masked part
# streams (default) and with ordinary ones (EFES_PART_STREAMS=plain).
cd "${GRAFT_REPO_ROOT:?}" || exit 1; export TMPDIR=/tmp; O=gpurun_out/parttrace; mkdir -p $O
for v in masked plain; do
  if [ $v = plain ]; then export EFES_PART_STREAMS=plain; else unset EFES_PART_STREAMS; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- \
    python3 bench.py --workload mixed --steps 1 --warmup 1 --no-cpu-baseline > $O/$v.json 2> $O/$v.err \
    || { echo "FAIL $v"; tail -5 $O/$v.err; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
path = glob.glob(f"gpurun_out/parttrace/{v}/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(path)) if "efes::" in r["Kernel_Name"] and "fill" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-3:]  # the timed step's three parts
t0 = min(int(r["Start_Timestamp"]) for r in last)
for r in last:
    print(v, r["Kernel_Name"].split("(")[0], "queue", r.get("Queue_Id"), "stream", r.get("Stream_Id"),
          "start %.3f end %.3f s" % ((int(r["Start_Timestamp"]) - t0) / 1e9, (int(r["End_Timestamp"]) - t0) / 1e9))
PY
done
