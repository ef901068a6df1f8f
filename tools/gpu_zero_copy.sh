# Zero-copy (kernel reads pinned host memory over PCIe) vs segmented H2D, for batch shapes of the
# uploads dispatcher:  bash tools/gpu_zero_copy.sh "<chunks> <chunk_bytes>" ...
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/zc
for spec in "$@"; do
  set -- $spec
  timeout -k 10 300 python bench.py --chunks $1 --chunk-bytes $2 --host-inclusive on --no-cpu-baseline --ingest-leg off --mixed-leg off --steps 3 --warmup 1 > gpurun_out/zc/c$1_b$2.json 2> gpurun_out/zc/err || { echo "FAIL $spec"; tail -5 gpurun_out/zc/err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/zc/c$1_b$2.json'));h=d['host_inclusive'];print('$1 x $2', 'device', d['value'], 'segmented', h['value'], 'zero-copy', h['zero_copy_value'], d['config'].get('kernel'))"
done
