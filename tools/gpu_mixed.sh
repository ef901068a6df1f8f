# BASELINE configs[3] (mixed ChunkSize 64K..64M x 65536) under several placements, one device:
#   bash tools/gpu_mixed.sh [force ...]    force = "<lanes per job>:<deep jobs>" (EFES_PLAN_FORCE)
cd "${GRAFT_REPO_ROOT:?}" || exit 1
mkdir -p gpurun_out/mixed
run() {  # tag, extra env/args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload mixed --steps 1 --warmup 1 --no-cpu-baseline --pool-gib 64 \
      $MIXED_ARGS > gpurun_out/mixed/$tag.json 2> gpurun_out/mixed/$tag.err || { echo "FAIL $tag"; tail -5 gpurun_out/mixed/$tag.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], 'GiB/s', d['ms_per_step'], 'ms', d['config'].get('plan'))" gpurun_out/mixed/$tag.json $tag
}
run wide EFES_PLAN_FORCE=0:0
run plan EFES_NOTHING=1
for f in "$@"; do run "f${f/:/_}" EFES_PLAN_FORCE=$f; done
