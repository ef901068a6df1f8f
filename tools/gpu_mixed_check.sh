# Why `bench.py --workload mixed` (main path) measured slower than the bench line's mixed leg:
# the plan's part streams sharing hardware queues.  CU-masked part streams (default) vs plain ones
# (EFES_PART_STREAMS=plain), with 4 (default) and 8 hardware queues.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/mixed_check; O=gpurun_out/mixed_check
B="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --receiver-leg off --drain-leg off --concurrency-leg off --span-leg off --ingest-leg off"
run() { local tag=$1; shift; timeout -k 10 300 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));m=d.get('mixed_config');print(sys.argv[2],'main',d['value'],d['ms_per_step'],'leg',m and (m['value'],m['roofline']['kernel_ms']))" $O/$tag.json $tag; }
for rep in 1 2; do
run main_plain env EFES_PART_STREAMS=plain python bench.py $B --workload mixed --steps 2 --warmup 1
run main_masked python bench.py $B --workload mixed --steps 2 --warmup 1
run main_plain_q8 env EFES_PART_STREAMS=plain GPU_MAX_HW_QUEUES=8 python bench.py $B --workload mixed --steps 2 --warmup 1
run leg_masked python bench.py $B --mixed-leg on --steps 3 --warmup 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "plan" --timeout 120 --timeout-method thread > $O/plan_tests.log 2>&1; rc=$?; tail -2 $O/plan_tests.log; exit $rc
