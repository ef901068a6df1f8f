# Concurrent-uploads path (tools/bench_uploads) over writer threads, uploads in flight and chunk size:
#   bash tools/gpu_uploads_scan.sh "<T K chunk>" ...
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/uploads
for spec in "$@"; do
  set -- $spec
  timeout -k 10 300 ./tools/bench_uploads $1 8192 4194304 32768 $2 $3 > gpurun_out/uploads/T$1_K$2_c$3.json 2> gpurun_out/up.err || { echo "FAIL $spec"; tail -5 gpurun_out/up.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/uploads/T$1_K$2_c$3.json'));print('T=$1 K=$2 chunk=$3', d['value'], 'GiB/s', d['seconds'], 's', d['all_sums_equal'], d['errors'])"
done
