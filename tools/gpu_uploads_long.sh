cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out/uploads
for spec in "16 128 8192" "16 128 16384" "32 128 16384"; do
  set -- $spec
  timeout -k 10 300 ./tools/bench_uploads $1 $3 4194304 32768 $2 262144 > gpurun_out/uploads/long_T$1_K$2_U$3.json 2> gpurun_out/up.err || { echo "FAIL $spec"; tail -5 gpurun_out/up.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/uploads/long_T$1_K$2_U$3.json'));print('T=$1 K=$2 U=$3', d['value'], 'GiB/s', d['seconds'], 's', d['all_sums_equal'], d['errors'])"
done
