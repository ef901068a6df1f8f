#!/bin/bash
# Round 4: configs[4] (bench.py --workload ingest) with the library before this session's host-side
# changes (ab_old/libefeshash.so, via EFES_LIB_OVERRIDE) against the current one, interleaved on one box.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_ingest_ab}
mkdir -p "$O"
for rep in ${REPS:-1 2}; do
  if [ "${NEW_FIRST:-0}" = 1 ]; then
    timeout -k 10 300 python3 bench.py --workload ingest --no-cpu-baseline > "$O/new.$rep.json" 2> "$O/new.$rep.err" || exit 1
  fi
  timeout -k 10 300 env EFES_LIB_OVERRIDE=$PWD/ab_old/libefeshash.so python3 bench.py --workload ingest --no-cpu-baseline > "$O/old.$rep.json" 2> "$O/old.$rep.err" || exit 1
  if [ "${NEW_FIRST:-0}" != 1 ]; then
    timeout -k 10 300 python3 bench.py --workload ingest --no-cpu-baseline > "$O/new.$rep.json" 2> "$O/new.$rep.err" || exit 1
  fi
  python3 - "$O" $rep <<'PY' | tee -a "$O/ab.log"
import json, sys
O, r = sys.argv[1:3]
a = json.loads(open(f"{O}/old.{r}.json").read().strip().splitlines()[-1]); b = json.loads(open(f"{O}/new.{r}.json").read().strip().splitlines()[-1])
print(f"rep {r}: ingest previous library {a['value']} GiB/s (kernel {a['roofline']['kernel_ms']} ms)  current {b['value']} GiB/s (kernel {b['roofline']['kernel_ms']} ms)")
PY
done
