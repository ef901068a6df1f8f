# A/B of WIDE library builds (e.g. prefetch depth), interleaved on one device, on aliased and on
# distinct (non-aliased) data:  LIBS="libefeshash_w3.so libefeshash_w4.so" bash tools/gpu_wide_depth_ab.sh [reps]
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
REPS=${1:-2}
for rep in $(seq "$REPS"); do
  for lib in $LIBS; do
    for args in ${ARGS_LIST:-"--workload ingest --ingest-scale 0.6 --mode wide --steps 3 --warmup 1" \
                "--chunks 196608 --chunk-bytes 1048576 --mode wide --steps 3 --warmup 1" \
                "--chunks 196608 --chunk-bytes 1048576 --mode wide --steps 3 --warmup 1 --sha1-only"}; do
      EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --host-inclusive off \
        --ingest-leg off --mixed-leg off --concurrency-leg off --uploads-leg off --receiver-leg off --span-leg off \
        --sha1-leg off --drain-leg off $args > gpurun_out/abd.json 2> gpurun_out/abd.err \
        || { echo "FAIL $lib $args"; tail -5 gpurun_out/abd.err; exit 1; }
      python -c "import json,sys;d=json.load(open('gpurun_out/abd.json'));print(sys.argv[1].ljust(22), sys.argv[2][:72].ljust(72), d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms/launch', d['roofline']['achieved'], 'GB/s')" $lib "$args" | tee -a gpurun_out/wide_depth_ab.log
    done
  done
done
