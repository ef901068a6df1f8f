# WIDE CRC from position tables vs slicing-by-8 (round 3): the GPU tests on the new build, then
# interleaved bench runs of both builds (headline, configs[4] ingest, configs[3] mixed).
#   bash tools/gpu_wide_crc_ab.sh   (expects efes_amd/lib/libefeshash_base.so = the slicing-by-8 build)
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/wide_crc_ab
O=gpurun_out/wide_crc_ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for lib in libefeshash_base.so libefeshash.so; do
    EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline \
      --host-inclusive off --sha1-leg off --uploads-leg off --receiver-leg off --drain-leg off --concurrency-leg off \
      --span-leg off > $O/$lib.$rep.json 2> $O/$lib.$rep.err || { echo "FAIL $lib"; tail -5 $O/$lib.$rep.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));i=d['ingest_config'];m=d['mixed_config'];print(sys.argv[2], 'head', d['value'], 'ingest', i['value'], i['roofline']['kernel_ms'], 'mixed', m['value'], m['roofline']['kernel_ms'], 'spot', i['digests_spot_check'])" $O/$lib.$rep.json $lib
  done
done
