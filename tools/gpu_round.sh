#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel trace -> PMC FETCH_SIZE pass.
# Stops at the first step that faults, aborts or times out (never retries a GPU step).
# Usage (from the repo root on the GPU box): bash tools/gpu_round.sh <tag> [steps...]
cd "${GRAFT_REPO_ROOT:?}" || exit 1
TAG=${1:-r01}; shift
STEPS=${*:-"smoke tests bench prof pmc"}
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
fatal() {  # rc of a GPU step: continue only on a plain failure (1) without a device error in its log
  local rc=$1 log=$2
  if [ "$rc" -ne 0 ] && { [ "$rc" -ne 1 ] || grep -qE "illegal memory|hipError|HIP error|Memory access fault|core dumped" "$log"; }; then
    echo "FATAL rc=$rc in $log"; tail -30 "$log"; exit "$rc"
  fi
}
for s in $STEPS; do
  case $s in
    smoke) timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke_$TAG.log 2>&1; rc=$?
           echo "smoke rc=$rc"; tail -3 $OUT/smoke_$TAG.log; fatal $rc $OUT/smoke_$TAG.log ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_$TAG.log 2>&1; rc=$?
           echo "tests rc=$rc"; tail -15 $OUT/gpu_tests_$TAG.log; fatal $rc $OUT/gpu_tests_$TAG.log ;;
    bench) timeout -k 10 400 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?
           echo "bench rc=$rc"; cat $OUT/bench_$TAG.json; tail -5 $OUT/bench_$TAG.err; fatal $rc $OUT/bench_$TAG.err ;;
    bench_*) a=${s#bench_}; timeout -k 10 400 python bench.py --no-cpu-baseline --mode ${a} > $OUT/bench_${TAG}_$a.json 2> $OUT/bench_${TAG}_$a.err; rc=$?
           echo "$s rc=$rc"; cat $OUT/bench_${TAG}_$a.json; fatal $rc $OUT/bench_${TAG}_$a.err ;;
    prof)  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
               python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off --concurrency-leg off --uploads-leg off --receiver-leg off --span-leg off > $OUT/prof_$TAG.log 2>&1; rc=$?
           echo "prof rc=$rc"; tail -3 $OUT/prof_$TAG.log; fatal $rc $OUT/prof_$TAG.log
           find $OUT/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \; ;;
    pmc)   timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$TAG -o run -- \
               python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off --concurrency-leg off --uploads-leg off --receiver-leg off --span-leg off > $OUT/pmc_$TAG.log 2>&1; rc=$?
           echo "pmc rc=$rc"; tail -3 $OUT/pmc_$TAG.log; fatal $rc $OUT/pmc_$TAG.log
           find $OUT/pmc_$TAG -name "*.csv" | head ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo ALL_DONE
