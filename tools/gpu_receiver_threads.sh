# Receiver vs copy ceiling by request threads (4 MiB PATCHes, tmpfs), twice each.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out; TAG=${TAG:-sweep}
D=$(mktemp -d /dev/shm/efes_rth.XXXXXX) || exit 1
trap 'rm -rf "$D"' EXIT
for rep in 1 2; do
  for t in ${THREADS:-128 256 512 768}; do
    u=$(( (3072 + t - 1) / t ))
    for mode in receiver copy; do
      if [ $mode = receiver ]; then args="receiver $D $t $u 4194304 4194304"; else args="copy $D $t $u 4194304"; fi
      timeout -k 10 120 ./tools/bench_receiver $args > gpurun_out/rth.json 2> gpurun_out/rth.err || { echo "FAIL $mode $t"; tail -3 gpurun_out/rth.err; exit 1; }
      python3 -c "import json,sys;d=json.loads(open('gpurun_out/rth.json').read().strip().splitlines()[-1]);print(sys.argv[1].ljust(8), 'threads', sys.argv[2].rjust(4), d['value'], 'GiB/s  cpu_s/GiB', d.get('cpu_s_per_gib'), ' sys', d.get('sys_share'))" $mode $t | tee -a gpurun_out/receiver_threads_$TAG.log
    done
  done
done
