#!/bin/bash
# Round 5 diagnostic: the span rate on buffers of different allocation histories
# (tools/span_alloc_probe.py), with the product and with A/B builds given as arguments.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r05_span_alloc}
shift || true
mkdir -p "$O"
for lib in product "$@" product "$@"; do
  env_lib=""; [ "$lib" = product ] || env_lib="EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/ab/libefeshash_$lib.so"
  echo "== $lib" | tee -a "$O/summary.txt"
  timeout -k 10 300 env $env_lib python3 tools/span_alloc_probe.py 2>&1 | grep -v amdgpu.ids | tee -a "$O/summary.txt" || exit 1
done
