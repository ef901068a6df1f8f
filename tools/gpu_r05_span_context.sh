#!/bin/bash
# Round 5: the span leg alone, inside the full default bench, and alone again right after it --
# to separate the kernel from the state the earlier legs leave the chip in.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r05_span_context}
mkdir -p "$O"
ONLY="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off --latency-leg off \
 --receiver-leg off --drain-leg off --concurrency-leg off --mixed-leg off --ingest-leg off --steps 2 --warmup 1"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['span_crc']; print(sys.argv[2], d['value'], 'GiB/s', d['roofline']['achieved'], 'GB/s', d['roofline']['frac'], d['clock'].get('mhz'), 'MHz')" "$1" "$2" | tee -a "$O/summary.txt"; }
timeout -k 10 200 python3 bench.py $ONLY > "$O/alone1.json" 2> "$O/alone1.err" || { tail -5 "$O/alone1.err"; exit 1; }
show "$O/alone1.json" "alone, first"
timeout -k 10 700 python3 bench.py > "$O/full.json" 2> "$O/full.err" || { tail -5 "$O/full.err"; exit 1; }
show "$O/full.json" "inside the full bench"
timeout -k 10 200 python3 bench.py $ONLY > "$O/alone2.json" 2> "$O/alone2.err" || { tail -5 "$O/alone2.err"; exit 1; }
show "$O/alone2.json" "alone, right after"
timeout -k 10 200 python3 bench.py $ONLY --mixed-leg on > "$O/after_mixed.json" 2> "$O/after_mixed.err" || { tail -5 "$O/after_mixed.err"; exit 1; }
show "$O/after_mixed.json" "after the mixed leg only"
