# Drainer read-back by files in flight: GiB/s, host CPU-seconds per GiB and jobs per launch of the
# digest queue (bench_receiver drain, 4 MiB files on tmpfs, 4 or 16 files per worker).  Diagnostic.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
D=$(mktemp -d /dev/shm/efes_dst.XXXXXX) || exit 1
trap 'rm -rf "$D"' EXIT
python3 - "$D" <<'PY'
import os, sys
z = 0x9E3779B97F4A7C15; m = (1 << 64) - 1; out = bytearray(4 << 20)
for i in range(len(out)):
    z ^= (z << 13) & m; z ^= z >> 7; z ^= (z << 17) & m; out[i] = z & 0xFF
for i in range(256):
    open(os.path.join(sys.argv[1], f"{i}.fid"), "wb").write(out)
PY
for per in ${PER:-4 16}; do
  for k in ${WORKERS:-64 256 512}; do
    timeout -k 10 120 ./tools/bench_receiver drain $D $k $((per * k)) 4194304 256 > gpurun_out/dst.json 2> gpurun_out/dst.err || { echo "FAIL $per $k"; tail -3 gpurun_out/dst.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/dst.json').read().strip().splitlines()[-1]);print('files/worker', sys.argv[1], 'workers', sys.argv[2], d['value'], 'GiB/s  cpu_s/GiB', d['cpu_s_per_gib'], 'sys', d['sys_share'], 'jobs/launch', d['jobs_per_launch'], 'launches', d['queue_launches'], 'ok', d['all_sums_equal'])" $per $k | tee -a gpurun_out/drain_stats.log
  done
done
