# Drainer read-back (bench_receiver drain, 4 MiB files on tmpfs) by workers and digest chunk size.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
D=$(mktemp -d /dev/shm/efes_dab.XXXXXX) || exit 1
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
  for kib in 64 256 1024; do
    for k in 64 256 512; do
      EFES_DIGEST_CHUNK_KIB=$kib timeout -k 10 120 ./tools/bench_receiver drain $D $k $((4 * k)) 4194304 256 > gpurun_out/dab.json 2> gpurun_out/dab.err || { echo "FAIL $kib $k"; tail -3 gpurun_out/dab.err; exit 1; }
      python3 -c "import json,sys;d=json.loads(open('gpurun_out/dab.json').read().strip().splitlines()[-1]);print('chunk', sys.argv[1], 'KiB workers', sys.argv[2], d['value'], 'GiB/s', d['all_sums_equal'])" $kib $k | tee -a gpurun_out/drain_ab.log
    done
  done
done
timeout -k 10 120 ./oracle/drain_cpu $D 16 4096 4194304 256 | tee -a gpurun_out/drain_ab.log
