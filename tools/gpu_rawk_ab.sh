# K on the chain's v_add3 (raw schedule) vs W+K expanded, for the shapes whose chain wave expands its
# own schedule (GROUPn, FED4E): the GPU tests on the new build, then interleaved runs of both builds.
#   bash tools/gpu_rawk_ab.sh   (efes_amd/lib/libefeshash_base.so = the previous build)
cd "${GRAFT_REPO_ROOT:?}" || exit 1; O=gpurun_out/rawk_ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --receiver-leg off --drain-leg off --concurrency-leg off --span-leg off --ingest-leg off --mixed-leg off"
for rep in 1 2; do
  for lib in libefeshash_base.so libefeshash.so; do
    for args in "--chunks 16384 --mode group4 --steps 3 --warmup 1" "--chunks 12288 --mode fed4e --steps 3 --warmup 1" "--chunks 8192 --mode fed4 --steps 3 --warmup 1" "--workload mixed --steps 2 --warmup 1"; do
      EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/$lib timeout -k 10 300 python bench.py $B $args > $O/r.json 2> $O/r.err || { echo "FAIL $lib $args"; tail -5 $O/r.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3][:28], d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms', d['config'].get('kernel'))" $O/r.json $lib "$args"
    done
  done
done
