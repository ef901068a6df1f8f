#!/bin/bash
# Round 6: the driver's round-end GPU steps on the final tree -- smoke, then `pytest tests -x -q -m gpu`
# as the driver runs it (plus per-test durations), then the default bench line.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_suite}
mkdir -p "$O"
timeout -k 10 300 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || { tail -5 "$O/smoke.log"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --durations=5 --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -3 "$O/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; tail -20 "$O/bench.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['roofline']['frac'], d['ranks_check']['ok'], sum(d['leg_seconds'].values()))"
