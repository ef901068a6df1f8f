cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
for spec in "16 64 262144" "16 128 262144" "32 64 262144" "16 64 131072"; do
  set -- $spec
  timeout -k 10 300 ./tools/bench_uploads $1 4096 4194304 32768 $2 $3 > gpurun_out/up.json 2> gpurun_out/up.err || { echo "FAIL $spec"; tail -5 gpurun_out/up.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/up.json'));print('T=$1 K=$2 chunk=$3', d['value'], 'GiB/s', d['seconds'], 's', d['all_sums_equal'], d['errors'])"
done
