# A/B of the upload dispatcher's kernel shape: default lib vs efes_amd/lib/ab_deep (DEEP forced).
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
for rep in 1 2; do
  for v in default ab_deep; do
    for spec in "16 64 262144" "16 128 262144" "32 128 262144"; do
      set -- $spec
      if [ $v = ab_deep ]; then LP=$PWD/efes_amd/lib/ab_deep; else LP=; fi
      LD_LIBRARY_PATH=$LP timeout -k 10 300 ./tools/bench_uploads $1 8192 4194304 32768 $2 $3 > gpurun_out/up.json 2> gpurun_out/up.err || { echo "FAIL $v $spec"; tail -5 gpurun_out/up.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/up.json'));print('$v T=$1 K=$2 chunk=$3', d['value'], 'GiB/s', d['seconds'], 's', d['all_sums_equal'], d['errors'])"
    done
  done
done
