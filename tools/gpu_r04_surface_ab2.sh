#!/bin/bash
# Round 4: go_surface at the bench configuration with the library of the evidence commit 13b0e52
# (ab_old/libefeshash.so, via LD_LIBRARY_PATH: the harness's RUNPATH comes after it) against the
# current one, interleaved on one box, beside tools/bench_uploads.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_surface_ab2}
mkdir -p "$O"
for rep in 1 2 3; do
  timeout -k 10 120 tools/bench_uploads 32 8192 4194304 32768 256 > "$O/uploads.$rep.json" || exit 1
  timeout -k 10 120 env LD_LIBRARY_PATH=$PWD/ab_old tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 > "$O/old.$rep.json" || exit 1
  timeout -k 10 120 tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 > "$O/new.$rep.json" || exit 1
  python3 - "$O" $rep <<'PY' | tee -a "$O/ab.log"
import json, sys
O, r = sys.argv[1], sys.argv[2]
u = json.load(open(f"{O}/uploads.{r}.json"))["value"]
a = json.load(open(f"{O}/old.{r}.json"))
b = json.load(open(f"{O}/new.{r}.json"))
print(f"rep {r}: uploads {u}  go_surface 13b0e52 {a['value']} (launches {a['launches']})  current {b['value']} (launches {b['launches']})")
PY
done
