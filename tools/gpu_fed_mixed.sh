#!/bin/bash
# configs[3] (mixed ChunkSize 64K..64M x 65536) under the planner and forced placements, one device.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/fed
run() {  # name, EFES_PLAN_FORCE ("" = planner)
  EFES_PLAN_FORCE="$2" timeout -k 10 200 python bench.py --workload mixed --steps 1 --warmup 1 --no-cpu-baseline \
    > gpurun_out/fed/mixed_$1.json 2> gpurun_out/fed/mixed_$1.err || { echo "FAIL $1"; tail -5 gpurun_out/fed/mixed_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fed/mixed_$1.json'));print('$1', d['value'], 'GiB/s', d['ms_per_step'], 'ms', d['config'].get('plan'))"
}
run plan ""
run fed_wx "1:6019x,0:6027x"
run fed_only "1:6019x"
run g4_old "4:12046x"
run fed_g4 "1:6019x,4:6027"
