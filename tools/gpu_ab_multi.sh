# A/B of library builds over several bench workloads (same device, interleaved):
#   LIBS="a.so b.so" REPS=2 bash tools/gpu_ab_multi.sh "<bench args 1>" "<bench args 2>" ...
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for args in "$@"; do
    for lib in $LIBS; do
      EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off $args > gpurun_out/abm.json 2> gpurun_out/abm.err || { echo "FAIL $lib $args"; tail -5 gpurun_out/abm.err; exit 1; }
      python -c "import json,sys;d=json.load(open('gpurun_out/abm.json'));print(sys.argv[1], '|', sys.argv[2], '|', d['value'], 'GiB/s', d['roofline']['kernel_ms'],'ms')" $lib "$args"
    done
  done
done
