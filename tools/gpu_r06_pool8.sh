#!/bin/bash
# Round 6: the one-process, eight-queue shape of an 8-GPU storage server rehearsed on one GPU -- the
# Go-surface harness (go_surface_path's configuration: 32 request threads x 256 uploads in flight,
# 8 192 x 4 MiB) and the uploads harness over eight contexts of GPU 0 against one, and the new GPU
# tests of the pooled harnesses.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r06_pool8}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_go_surface.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/tests.log" 2>&1; rc=$?; tail -2 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for devs in 0 0,0,0,0,0,0,0,0; do
  timeout -k 10 200 ./tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 - same $devs > "$O/surface_$devs.json" 2> "$O/surface_$devs.err" \
    || { echo "surface $devs failed"; tail -3 "$O/surface_$devs.err"; exit 1; }
  timeout -k 10 200 ./tools/bench_uploads 32 8192 4194304 32768 256 262144 0 $devs > "$O/uploads_$devs.json" 2> "$O/uploads_$devs.err" \
    || { echo "uploads $devs failed"; tail -3 "$O/uploads_$devs.err"; exit 1; }
  python3 - "$O" "$devs" <<'PY' | tee -a "$O/pool8.log"
import json, sys
O, devs = sys.argv[1:]
for name in ("surface", "uploads"):
    d = json.loads(open(f"{O}/{name}_{devs}.json").read().strip().splitlines()[-1])
    ok = d.get("all_equal", d.get("all_sums_equal")) and d["errors"] == 0
    print(f"{name:8s} devices {devs:16s} {d['value']:7.2f} GiB/s  ok {ok}  per device jobs {[x['jobs'] for x in d['devices']]}")
PY
done
