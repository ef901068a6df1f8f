# A/B of library builds on WIDE-heavy workloads (same device, interleaved):
#   LIBS="a.so b.so" bash tools/gpu_ab_wide.sh
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
for rep in 1 2; do
  for lib in $LIBS; do
    for args in "--chunks 8192 --mode wide --steps 3 --warmup 1" "--workload ingest --ingest-scale 0.4 --ingest-batch 131072 --mode wide --warmup 1" "--chunks 65536 --chunk-bytes 65536 --mode wide --steps 5 --warmup 1"; do
      EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off $args > gpurun_out/abw.json 2> gpurun_out/abw.err || { echo "FAIL $lib $args"; tail -5 gpurun_out/abw.err; exit 1; }
      python -c "import json,sys;d=json.load(open('gpurun_out/abw.json'));print(sys.argv[1], sys.argv[2][:40], d['value'], 'GiB/s', d['roofline']['kernel_ms'],'ms/launch')" $lib "$args"
    done
  done
done
