# WIDE pacing (sibling-progress priorities, one workgroup per CU) vs EFES_WIDE_PACE=0, interleaved,
# after the WIDE parity tests.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -k "wide or plan or full_size" > gpurun_out/t_pace.log 2>&1
rc=$?; tail -2 gpurun_out/t_pace.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for pace in 0 1; do
    for args in "--chunks 196608 --chunk-bytes 1048576 --mode wide --steps 3 --warmup 1" \
                "--chunks 196608 --chunk-bytes 1048576 --mode wide --steps 3 --warmup 1 --sha1-only" \
                "--chunks 131072 --chunk-bytes 1048576 --mode wide --steps 3 --warmup 1" \
                "--workload ingest --mode wide --warmup 1"; do
      EFES_WIDE_PACE=$pace timeout -k 10 300 python bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off \
        --mixed-leg off --concurrency-leg off --uploads-leg off --receiver-leg off --span-leg off --sha1-leg off \
        --drain-leg off $args > gpurun_out/abp.json 2> gpurun_out/abp.err || { echo "FAIL $pace $args"; tail -5 gpurun_out/abp.err; exit 1; }
      python -c "import json,sys;d=json.load(open('gpurun_out/abp.json'));print('pace='+sys.argv[1], sys.argv[2][:72].ljust(72), d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms/launch')" $pace "$args" | tee -a gpurun_out/wide_pace_ab.log
    done
  done
done
