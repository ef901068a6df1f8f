#!/bin/bash
# Round 5: the span CRC's kernel statistics and HBM counters on the bench's span leg (one 16 GiB
# object): rocprofv3 --kernel-trace --stats, then one counter set per run -- FETCH_SIZE (the
# traffic bench.py reports, tools/pmc_traffic.py), the EA read requests (64-B vs 32-B) and the L2
# hit/miss split (so the x2 FETCH_SIZE correction can be checked for LDS-DMA reads).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:?}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r05_span_prof}
mkdir -p "$out"
BENCH="python3 bench.py --no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off \
 --latency-leg off --receiver-leg off --drain-leg off --concurrency-leg off --mixed-leg off --ingest-leg off --steps 2 --warmup 1"
summ() {  # $1 = run dir: median of every counter per kernel
  python3 - "$1" <<'PY'
import csv, glob, sys, collections
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    if "span" in k:
        print(f"{sys.argv[1].split('/')[-1]:10s} {k:28s} {c:22s} n={len(v)} median={sorted(v)[len(v)//2]:.10g}")
PY
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- $BENCH \
  > "$out/prof.json" 2> "$out/prof.err"
echo prof ok
i=0
for set in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d "$out/pmc_$i" -o run -- $BENCH > "$out/pmc_$i.log" 2>&1
  summ "$out/pmc_$i" >> "$out/summary.txt"
done
cat "$out/summary.txt"
