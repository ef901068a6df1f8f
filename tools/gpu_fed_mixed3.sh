#!/bin/bash
# configs[3]: planner vs a fourth part (the 16 MiB class as WIDE with one wave per SIMD).
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/fed
run() {  # name, EFES_PLAN_FORCE ("" = planner)
  EFES_PLAN_FORCE="$2" timeout -k 10 200 python bench.py --workload mixed --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/fed/mixed3_$1.json 2> gpurun_out/fed/mixed3_$1.err || { echo "FAIL $1"; tail -5 gpurun_out/fed/mixed3_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fed/mixed3_$1.json'));print('$1', d['value'], 'GiB/s', d['ms_per_step'], 'ms', [(p['jobs'],p['kernel'],p['exclusive_cus']) for p in d['config']['plan']['parts']])"
}
run plan ""
run fe_g4_w16x "2:6019x,4:6027x,0:5975x"
run fe_g4_g4_16 "2:6019x,4:6027x,4:5975"
run fe_g4_w16x8x "2:6019x,4:6027x,0:11950x"
