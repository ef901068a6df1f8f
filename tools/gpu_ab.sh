# A/B builds of the library on the SAME device, interleaved 3x:
#   LIBS="libefeshash_va.so libefeshash_vb.so" bash tools/gpu_ab.sh [bench args]
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in $LIBS; do
    EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off "$@" > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "FAIL $lib"; tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));print(sys.argv[1], d['value'], 'GiB/s', d['roofline']['kernel_ms'],'ms/launch')" $lib
  done
done
