# WIDE pacing with one LDS read + v_readlane vs the VALU loop over siblings (round 3): the WIDE
# GPU tests on the new build, then interleaved configs[4] ingest runs of both builds.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; O=gpurun_out/wide_pace2_ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "wide or fuzz or ingest or full_size" > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --receiver-leg off --drain-leg off --concurrency-leg off --span-leg off --mixed-leg off"
for rep in 1 2 3; do
  for lib in libefeshash_base.so libefeshash.so; do
    EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/$lib timeout -k 10 300 python bench.py $B --steps 3 --warmup 1 > $O/r.json 2> $O/r.err || { echo "FAIL $lib"; tail -5 $O/r.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));i=d['ingest_config'];print(sys.argv[2],'ingest',i['value'],i['roofline']['kernel_ms'],'spot',i['digests_spot_check'])" $O/r.json $lib
  done
done
