# configs[4] ingest launches over a 64 GiB vs a 200 GiB aliased pool (how many chunks share a slot),
# interleaved, plus a FETCH_SIZE pass of WIDE over distinct data (196608 x 1 MiB, no aliasing).
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do
  for pool in 64 200; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off \
      --concurrency-leg off --uploads-leg off --receiver-leg off --span-leg off --sha1-leg off --drain-leg off \
      --workload ingest --mode wide --warmup 1 --pool-gib $pool > gpurun_out/ip.json 2> gpurun_out/ip.err \
      || { echo "FAIL pool $pool"; tail -5 gpurun_out/ip.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/ip.json'));print('pool', sys.argv[1], d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms/launch')" $pool | tee -a gpurun_out/ingest_pool.log
  done
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_wide_distinct -o run -- \
  python3 bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off --concurrency-leg off \
  --uploads-leg off --receiver-leg off --span-leg off --sha1-leg off --drain-leg off \
  --chunks 196608 --chunk-bytes 1048576 --mode wide --steps 3 --warmup 1 > gpurun_out/pmc_wide_distinct.log 2>&1 \
  || { echo "pmc failed"; tail -5 gpurun_out/pmc_wide_distinct.log; exit 1; }
echo pmc ok
