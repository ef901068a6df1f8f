#!/bin/bash
# FED4E parity, then configs[3] under the planner and forced alternatives.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/fed
timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_consumer.py -m gpu -x -q -k "fed4 or plan or auto or consumer" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fed/tests_fed4e.log 2>&1
rc=$?; tail -2 gpurun_out/fed/tests_fed4e.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, EFES_PLAN_FORCE ("" = planner)
  EFES_PLAN_FORCE="$2" timeout -k 10 200 python bench.py --workload mixed --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/fed/mixed2_$1.json 2> gpurun_out/fed/mixed2_$1.err || { echo "FAIL $1"; tail -5 gpurun_out/fed/mixed2_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fed/mixed2_$1.json'));print('$1', d['value'], 'GiB/s', d['ms_per_step'], 'ms', [(p['jobs'],p['kernel'],p['exclusive_cus']) for p in d['config']['plan']['parts']])"
}
run plan ""
run g4_old "4:12046x"
run fe_g4 "2:6019x,4:6027x"
run fe_only "2:6019x"
run fe_g8 "2:6019x,8:6027x"
