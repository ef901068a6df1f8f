#!/bin/bash
# Round 6, first GPU pass: smoke, the -m gpu suite with per-test durations (the bench test's child
# now logs its legs and arms faulthandler), then kernel traces of the PATCH-latency harness at 1 and
# 16 uploads in flight (the 4 MiB PATCH's launches, their durations and gaps).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_check}
mkdir -p "$O"
timeout -k 10 300 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || { tail -5 "$O/smoke.log"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --durations=25 --timeout 120 --timeout-method thread \
  > "$O/gpu_tests.log" 2>&1
rc=$?; tail -3 "$O/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
for k in 1 16; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/patch_$k" -o run -- \
    ./tools/bench_go_surface $k $((k * 8)) 4194304 32768 1 1 256 1024 > "$O/patch_$k.json" 2> "$O/patch_$k.err" \
    || { echo "trace $k failed"; tail -5 "$O/patch_$k.err"; exit 1; }
  echo "patch $k: $(cat "$O/patch_$k.json")"
done
