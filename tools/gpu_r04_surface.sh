#!/bin/bash
# Round 4: the unchanged Go surface (tools/bench_go_surface) fused vs unfused, beside the fused
# efes_upload path (tools/bench_uploads) at the same concurrency; boundary + consumer tests first.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:?}"
out=gpurun_out/${1:-r04a}
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_pairs.py tests/test_gpu_boundary.py tests/test_gpu_consumer.py > "$out/tests.log" 2>&1
for i in 1 2; do
  timeout -k 10 120 tools/bench_uploads 32 8192 4194304 32768 256 > "$out/uploads_$i.json"
  timeout -k 10 120 tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 > "$out/go_fused_$i.json"
  EFES_DIGEST_FUSE=0 timeout -k 10 120 tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 > "$out/go_unfused_$i.json"
done
timeout -k 10 120 tools/bench_go_surface 32 8192 4194304 32768 256 4 256 8208 > "$out/go_fused_4patches.json"
cat "$out"/*.json
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_parity.py::test_full_size_ingest_segmented_as_benched" > "$out/test_cfg4_segmented.log" 2>&1
