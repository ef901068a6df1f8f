#!/bin/bash
# Round 5: the default bench line on the final tree (clock = the per-CU matched probe), then the
# configs[4] leg twice more on the same box (the spread of frac at the measured clock).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r05b}
mkdir -p "$O"
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -5 "$O/bench.err"; exit 1; }
echo bench ok
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --workload ingest --no-cpu-baseline > "$O/ingest.$rep.json" 2> "$O/ingest.$rep.err" || { tail -5 "$O/ingest.$rep.err"; exit 1; }
done
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
d = json.loads(open(f"{O}/bench.json").read().strip().splitlines()[-1])
print("headline", d["value"], d["clock"].get("mhz"), d["binding_roofline"]["frac"], d["binding_roofline"]["frac_at_clock"])
i = d["ingest_config"]; print("ingest leg", i["value"], i["clock"].get("mhz"), i["binding_roofline"]["frac"], i["binding_roofline"]["frac_at_clock"])
for r in (1, 2):
    e = json.loads(open(f"{O}/ingest.{r}.json").read().strip().splitlines()[-1])
    print("ingest run", r, e["value"], e["clock"].get("mhz"), e["binding_roofline"]["frac"], e["binding_roofline"]["frac_at_clock"])
PY
