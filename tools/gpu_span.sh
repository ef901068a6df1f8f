#!/bin/bash
# Span CRC (efes_crc32_span): parity tests, the bench leg alone, and its rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
LEGS="--no-cpu-baseline --host-inclusive off --ingest-leg off --uploads-leg off --receiver-leg off --concurrency-leg off --mixed-leg off"
timeout -k 10 300 python -u -m pytest tests/test_gpu_span.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/span_tests.log 2>&1 || { echo "span tests failed"; tail -30 gpurun_out/span_tests.log; exit 1; }
tail -8 gpurun_out/span_tests.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 $LEGS > gpurun_out/span_bench.json 2> gpurun_out/span_bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/span_bench.err; exit 1; }
cat gpurun_out/span_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/span_prof -o run -- \
  python3 bench.py --steps 3 --warmup 1 $LEGS > gpurun_out/span_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/span_prof.log; exit 1; }
find gpurun_out/span_prof -name "*kernel_stats.csv" -exec cat {} \;
