#!/bin/bash
# FED kernels on one device (DESIGN.md §4 "FED kernel"):
#   bash tools/gpu_fed.sh tests                  # parity of the FED shapes (pytest -k fed4)
#   bash tools/gpu_fed.sh stats G,C[x] JOBS ...  # cycle accounting, diagnostic build (tools/fed_stats.py)
#   bash tools/gpu_fed.sh time MODE JOBS ...     # bench.py --mode MODE --chunks JOBS (EFES_FED_SHAPE may be set)
#   bash tools/gpu_fed.sh mixed NAME=FORCE ...   # configs[3] under EFES_PLAN_FORCE (NAME= for the planner)
# Outputs under gpurun_out/fed/.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/fed
what=$1; shift
legs="--no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off --concurrency-leg off --uploads-leg off"
case $what in
  tests)
    timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py -m gpu -x -q -k "fed4" \
      --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fed/tests.log 2>&1
    rc=$?; tail -2 gpurun_out/fed/tests.log; exit $rc ;;
  stats)
    while [ $# -ge 2 ]; do
      echo "== shape $1, $2 jobs (stats build)"
      EFES_FED_SHAPE=$1 EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/libefeshash_stats.so timeout -k 10 100 python tools/fed_stats.py $2 || exit 1
      shift 2
    done ;;
  time)
    while [ $# -ge 2 ]; do
      out=gpurun_out/fed/${1}_${EFES_FED_SHAPE:-default}_$2
      timeout -k 10 180 python bench.py --mode $1 --chunks $2 --steps 3 --warmup 1 $legs > $out.json 2> $out.err \
        || { echo "FAIL $1 $2"; tail -5 $out.err; exit 1; }
      python3 -c "import json;d=json.load(open('$out.json'));print('$1 $2', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
      shift 2
    done ;;
  mixed)
    for spec in "$@"; do
      name=${spec%%=*}; force=${spec#*=}
      EFES_PLAN_FORCE="$force" timeout -k 10 200 python bench.py --workload mixed --steps 2 --warmup 1 --no-cpu-baseline \
        > gpurun_out/fed/mixed_$name.json 2> gpurun_out/fed/mixed_$name.err || { echo "FAIL $name"; tail -5 gpurun_out/fed/mixed_$name.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/fed/mixed_$name.json'));print('$name', d['value'], 'GiB/s', d['ms_per_step'], 'ms', [(p['jobs'],p['kernel'],p['exclusive_cus']) for p in d['config']['plan']['parts']])"
    done ;;
  *) echo "usage: $0 tests | stats G,C[x] JOBS ... | time MODE JOBS ... | mixed NAME=FORCE ..."; exit 2 ;;
esac
