# Receiver host-cost experiments (bench_receiver receiver, 768 threads x 4 MiB PATCHes, tmpfs),
# interleaved with the copy ceiling: prints GiB/s, CPU-seconds per GiB and the system share.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
D=$(mktemp -d /dev/shm/efes_rab.XXXXXX) || exit 1
trap 'rm -rf "$D"' EXIT
for rep in 1 2; do
  for v in ${VARIANTS:-default spin phases copy}; do
    case $v in
      default) env= ; mode=receiver ;;
      spin) env="EFES_QUEUE_SYNC=spin" ; mode=receiver ;;
      phases) env="EFES_RECEIVER_PHASES=1" ; mode=receiver ;;
      copybuf) env="EFES_RECEIVER_PHASES=1 EFES_RECEIVER_COPYBUF=1" ; mode=receiver ;;
      ahead0) env="EFES_QUEUE_AHEAD=0" ; mode=receiver ;;
      ahead8) env="EFES_QUEUE_AHEAD=8" ; mode=receiver ;;
      copy) env= ; mode=copy ;;
    esac
    if [ $mode = receiver ]; then args="receiver $D 768 4 4194304 4194304"; else args="copy $D 768 4 4194304"; fi
    env $env timeout -k 10 120 ./tools/bench_receiver $args > gpurun_out/rab.json 2> gpurun_out/rab.err || { echo "FAIL $v"; tail -3 gpurun_out/rab.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/rab.json').read().strip().splitlines()[-1]);print(sys.argv[1].ljust(8), d['value'], 'GiB/s  cpu_s/GiB', d.get('cpu_s_per_gib'), ' sys', d.get('sys_share'), d.get('phase_cpu_s_per_gib', ''), d.get('request_threads_cpu_s_per_gib', ''), d.get('unlink_cpu_s_per_gib', ''))" $v | tee -a gpurun_out/receiver_ab.log
  done
done
