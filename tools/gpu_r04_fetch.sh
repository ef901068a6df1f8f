#!/bin/bash
# Round 4, VERDICT r03 item 2: calibrate FETCH_SIZE for WIDE's access pattern on a known byte count
# (tools/microbench/mb_wide_fetch: coalesced / WIDE's 64-B blocks / whole 128-B lines, with and
# without WIDE-like work between loads), then the same counters for wide_kernel itself on the
# configs[4] launch geometry (196 608 distinct 1 MiB messages).  One counter set per rocprofv3 run.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:?}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_fetch}
mkdir -p "$out"
MB=tools/microbench/mb_wide_fetch
BENCH="python3 bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off --concurrency-leg off \
 --uploads-leg off --go-surface-leg off --latency-leg off --receiver-leg off --drain-leg off --span-leg off --sha1-leg off \
 --chunks 196608 --chunk-bytes 1048576 --mode wide --steps 3 --warmup 1"
timeout -k 10 150 $MB 196608 1048576 0 2 > "$out/timing_pad0.json"
timeout -k 10 240 $MB 196608 1048576 120 2 > "$out/timing_pad120.json"
summ() {  # $1 = run dir: median of every counter per kernel
  python3 - "$1" <<'PY'
import csv, glob, sys, collections
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{sys.argv[1].split('/')[-1]:18s} {k:40s} {c:22s} n={len(v)} median={sorted(v)[len(v)//2]:.10g}")
PY
}
i=0
for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  for pad in 0 120; do
    timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d "$out/mb_pad${pad}_$i" -o run -- \
      $MB 196608 1048576 $pad 2 > "$out/mb_pad${pad}_$i.log" 2>&1
    summ "$out/mb_pad${pad}_$i" >> "$out/summary.txt"
  done
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d "$out/wide_$i" -o run -- $BENCH > "$out/wide_$i.log" 2>&1
  summ "$out/wide_$i" >> "$out/summary.txt"
done
cat "$out"/timing_*.json "$out/summary.txt"
