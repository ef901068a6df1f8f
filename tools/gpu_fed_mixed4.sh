#!/bin/bash
# configs[3]: the rest as WIDE with one wave per SIMD (exclusive) vs shared, 3 parts.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/fed
run() {  # name, EFES_PLAN_FORCE ("" = planner)
  EFES_PLAN_FORCE="$2" timeout -k 10 200 python bench.py --workload mixed --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/fed/mixed4_$1.json 2> gpurun_out/fed/mixed4_$1.err || { echo "FAIL $1"; tail -5 gpurun_out/fed/mixed4_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fed/mixed4_$1.json'));print('$1', d['value'], 'GiB/s', d['ms_per_step'], 'ms', [(p['jobs'],p['kernel'],p['exclusive_cus']) for p in d['config']['plan']['parts']])"
}
run plan ""
run fe_g4_wx "2:6019x,4:6027x,0:53490x"
run g4_wx "4:12046x,0:53490x"
