cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for args in "--sha1-only" "--chunks 65536 --chunk-bytes 65536 --mode wide" "--chunks 262144 --chunk-bytes 16384 --mode wide" "--chunks 16384 --chunk-bytes 262144 --mode wide" "--chunks 16384 --chunk-bytes 262144 --mode deep"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 $args > gpurun_out/b.json 2> gpurun_out/b.err || { echo "FAIL $args"; tail -5 gpurun_out/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$args', d['value'], 'GiB/s', d['roofline']['kernel_ms'],'ms', d['config']['kernel'])"
done
