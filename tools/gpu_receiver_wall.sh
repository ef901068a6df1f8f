# Where a receiver request's WALL time goes (EFES_RECEIVER_PHASE_CLOCK=wall), and how many uploads
# each launch of the batching queue carries, by request threads and per-upload pacing
# (bench_receiver receiver, 4 MiB one-PATCH uploads, tmpfs).  Diagnostic, not the bench.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
D=$(mktemp -d /dev/shm/efes_rwall.XXXXXX) || exit 1
trap 'rm -rf "$D"' EXIT
for cfg in ${CONFIGS:-"768 3" "768 0" "256 3" "512 3"}; do
  set -- $cfg
  T=$1; A=$2
  EFES_QUEUE_AHEAD=$A EFES_RECEIVER_PHASES=1 EFES_RECEIVER_PHASE_CLOCK=wall timeout -k 10 120 \
    ./tools/bench_receiver receiver "$D" "$T" $((3072 / T)) 4194304 4194304 > gpurun_out/rwall.json 2> gpurun_out/rwall.err \
    || { echo "FAIL $cfg"; tail -3 gpurun_out/rwall.err; exit 1; }
  python3 - "$T" "$A" <<'PY' | tee -a gpurun_out/receiver_wall.log
import json, sys
d = json.loads(open('gpurun_out/rwall.json').read().strip().splitlines()[-1])
T = int(sys.argv[1]); n = d['uploads']; gib = n * d['upload_bytes'] / 2**30
ms = {k: v * gib / n * 1e3 for k, v in d['phase_cpu_s_per_gib'].items()}  # wall ms per request
print(f"threads {T} ahead {sys.argv[2]}: {d['value']} GiB/s cpu_s/GiB {d['cpu_s_per_gib']} "
      f"jobs/launch {d['jobs_per_launch']} launches {d['queue_launches']} | wall ms per request: "
      + " ".join(f"{k} {v:.1f}" for k, v in ms.items()) + f" | total {sum(ms.values()):.1f}")
PY
done
