#!/bin/bash
# Span CRC evidence: rocprofv3 kernel stats and a FETCH_SIZE pass of the bench's span_crc leg alone.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
LEGS="--steps 1 --warmup 0 --no-cpu-baseline --host-inclusive off --ingest-leg off --uploads-leg off --receiver-leg off --concurrency-leg off --mixed-leg off --span-leg on"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/spanv3_prof -o run -- python3 bench.py $LEGS \
  > gpurun_out/spanv3_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/spanv3_prof.log; exit 1; }
grep -h span gpurun_out/spanv3_prof/run_kernel_stats.csv
grep -o '"span_crc": {[^}]*}[^}]*}' gpurun_out/spanv3_prof.log | head -1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/spanv3_pmc -o run -- python3 bench.py $LEGS \
  > gpurun_out/spanv3_pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/spanv3_pmc.log; exit 1; }
python3 - <<'PY'
import csv, statistics
rows = [r for r in csv.DictReader(open("gpurun_out/spanv3_pmc/run_counter_collection.csv")) if "span_kernel" in r["Kernel_Name"]]
v = sorted(float(r["Counter_Value"]) for r in rows)
print("span_kernel FETCH_SIZE KiB per dispatch:", v, "x1024x2 median bytes:", statistics.median(v) * 2048)
PY
