#!/bin/bash
# Round 4, VERDICT r03 item 4: configs[3] (65 536 mixed ChunkSize chunks, 752 GiB) placed in a 64 GiB
# pool (bench default until round 3: ~12 aliases per byte) against a 200 GiB pool (3.8), interleaved
# in one call on one device; the planner's launch is the same.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:?}"
O=gpurun_out/${1:-r04_mixed_pool}
mkdir -p "$O"
for rep in 1 2 3; do
  for pool in 64 200; do
    timeout -k 10 300 python3 bench.py --workload mixed --pool-gib $pool --steps 1 --warmup 1 --no-cpu-baseline \
      > "$O/pool$pool.$rep.json" 2> "$O/pool$pool.$rep.err"
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('pool', sys.argv[2], 'GiB/s', d['value'], 'ms', d['ms_per_step'], d['config'].get('kernel'))" "$O/pool$pool.$rep.json" $pool | tee -a "$O/ab.log"
  done
done
