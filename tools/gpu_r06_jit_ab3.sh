#!/bin/bash
# Round 6: the JIT dispatcher with clipped per-byte samples against the previous dispatcher (A/B as in
# tools/gpu_r06_jit_ab.sh), then ThreadSanitizer over the final digest layer and dispatcher (build first:
# bash tools/tsan_build.sh).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=${1:-r06_jit_ab3}
bash tools/gpu_r06_jit_ab.sh "$O" || exit 1
bash tools/gpu_r04_tsan.sh "$O/tsan"
