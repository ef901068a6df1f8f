# Drainer read-back at 256 / 512 files in flight (16 files per worker): per-upload pacing of the
# digest queue (EFES_QUEUE_AHEAD 3 = default, 0 = off, 8) and digest chunk size.  Diagnostic.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
D=$(mktemp -d /dev/shm/efes_dpa.XXXXXX) || exit 1
trap 'rm -rf "$D"' EXIT
python3 - "$D" <<'PY'
import os, sys
z = 0x9E3779B97F4A7C15; m = (1 << 64) - 1; out = bytearray(4 << 20)
for i in range(len(out)):
    z ^= (z << 13) & m; z ^= z >> 7; z ^= (z << 17) & m; out[i] = z & 0xFF
for i in range(256):
    open(os.path.join(sys.argv[1], f"{i}.fid"), "wb").write(out)
PY
for rep in 1 2; do
  for cfg in "3 64" "0 64" "8 64" "3 128" "0 128"; do
    set -- $cfg
    for k in 256 512; do
      EFES_QUEUE_AHEAD=$1 EFES_DIGEST_CHUNK_KIB=$2 timeout -k 10 120 ./tools/bench_receiver drain $D $k $((16 * k)) 4194304 256 > gpurun_out/dpa.json 2> gpurun_out/dpa.err || { echo "FAIL $cfg $k"; tail -3 gpurun_out/dpa.err; exit 1; }
      python3 -c "import json,sys;d=json.loads(open('gpurun_out/dpa.json').read().strip().splitlines()[-1]);print('ahead', sys.argv[1], 'chunk_kib', sys.argv[2], 'workers', sys.argv[3], d['value'], 'GiB/s  cpu_s/GiB', d['cpu_s_per_gib'], 'sys', d['sys_share'], 'jobs/launch', d['jobs_per_launch'], 'ok', d['all_sums_equal'])" $1 $2 $k | tee -a gpurun_out/drain_pace.log
    done
  done
done
