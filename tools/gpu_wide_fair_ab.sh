# A/B of WIDE's priority rotation (EFES_WIDE_FAIR=0: the hardware's oldest-first issue order),
# interleaved on one device:  bash tools/gpu_wide_fair_ab.sh [reps]
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
REPS=${1:-2}
for rep in $(seq "$REPS"); do
  for fair in 0 1; do
    for args in "--workload ingest --ingest-scale 0.6 --mode wide --steps 3 --warmup 1" \
                "--workload ingest --ingest-scale 0.6 --mode wide --steps 3 --warmup 1 --sha1-only" \
                "--workload ingest --ingest-scale 0.4 --ingest-batch 131072 --mode wide --warmup 1" \
                "--chunks 65536 --chunk-bytes 65536 --mode wide --steps 5 --warmup 1"; do
      EFES_WIDE_FAIR=$fair timeout -k 10 300 python bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off \
        --mixed-leg off --concurrency-leg off --uploads-leg off --receiver-leg off --span-leg off $args \
        > gpurun_out/abf.json 2> gpurun_out/abf.err || { echo "FAIL fair=$fair $args"; tail -5 gpurun_out/abf.err; exit 1; }
      python -c "import json,sys;d=json.load(open('gpurun_out/abf.json'));print('fair='+sys.argv[1], sys.argv[2][:72].ljust(72), d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms/launch', d['roofline']['achieved'], 'GB/s')" $fair "$args" | tee -a gpurun_out/wide_fair_ab.log
    done
  done
done
