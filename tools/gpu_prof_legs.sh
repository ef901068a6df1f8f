#!/bin/bash
# rocprofv3 kernel-trace summaries of the configs[4] (ingest, WIDE) and configs[3] (mixed, planned)
# workloads, for the bench line's ingest_config / mixed_config kernel times.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
for w in ingest mixed; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$w -o run -- \
    python3 bench.py --workload $w --warmup 1 --no-cpu-baseline --host-inclusive off > gpurun_out/prof_$w.json 2> gpurun_out/prof_$w.err \
    || { echo "FAIL $w"; tail -5 gpurun_out/prof_$w.err; exit 1; }
  echo "== $w"; tail -c 600 gpurun_out/prof_$w.json; echo
  find gpurun_out/prof_$w -name "*kernel_stats.csv" -exec cat {} \;
done
