#!/bin/bash
# configs[3] with every plan part on the context's own streams: planner, 4-part, exclusive rest; trace.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/fed
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q -k "plan" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fed/tests_plan5.log 2>&1
rc=$?; tail -2 gpurun_out/fed/tests_plan5.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, EFES_PLAN_FORCE ("" = planner)
  EFES_PLAN_FORCE="$2" timeout -k 10 200 python bench.py --workload mixed --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/fed/mixed5_$1.json 2> gpurun_out/fed/mixed5_$1.err || { echo "FAIL $1"; tail -5 gpurun_out/fed/mixed5_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fed/mixed5_$1.json'));print('$1', d['value'], 'GiB/s', d['ms_per_step'], 'ms', [(p['jobs'],p['kernel'],p['exclusive_cus']) for p in d['config']['plan']['parts']])"
}
run plan ""
run fe_g4_w16x "2:6019x,4:6027x,0:6056x"
run fe_g4_w16_8x "2:6019x,4:6027x,0:12092x"
run fe_g4_wx "2:6019x,4:6027x,0:53490x"
run g4_old "4:12046x"
bash tools/gpu_mixed_trace.sh 2:6019x,4:6027x,0:6056x 2:6019x,4:6027x
