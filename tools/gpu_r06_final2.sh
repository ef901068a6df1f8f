#!/bin/bash
# Round 6 evidence on the final tree (after the adaptive JIT margin): tools/gpu_r06_final.sh, then
# ThreadSanitizer over the final dispatcher and digest layer (build first: bash tools/tsan_build.sh).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=${1:-r06h}
bash tools/gpu_r06_final.sh "$O" || exit 1
bash tools/gpu_r04_tsan.sh "$O/tsan"
