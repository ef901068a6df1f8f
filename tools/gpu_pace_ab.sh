# A/B of the queue's pacing rule: ab_old/libefeshash.so (scarce = free chunks <= max_uploads) vs the
# in-tree library (scarce = free chunks <= uploads open now), interleaved on one device: drainer at
# 256 / 512 files in flight (16 files per worker), receiver at 768 threads, uploads 32 x 256.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
D=$(mktemp -d /dev/shm/efes_pab.XXXXXX) || exit 1
trap 'rm -rf "$D"' EXIT
python3 - "$D" <<'PY'
import os, sys
z = 0x9E3779B97F4A7C15; m = (1 << 64) - 1; out = bytearray(4 << 20)
for i in range(len(out)):
    z ^= (z << 13) & m; z ^= z >> 7; z ^= (z << 17) & m; out[i] = z & 0xFF
os.makedirs(os.path.join(sys.argv[1], "drain"))
for i in range(256):
    open(os.path.join(sys.argv[1], "drain", f"{i}.fid"), "wb").write(out)
PY
show() { python3 -c "import json,sys;d=json.loads(open('gpurun_out/pab.json').read().strip().splitlines()[-1]);print(sys.argv[1].ljust(4), sys.argv[2].ljust(14), d['value'], 'GiB/s cpu_s/GiB', d.get('cpu_s_per_gib'), 'jobs/launch', d.get('jobs_per_launch'), 'ok', d.get('all_sums_equal', d.get('digests_match')), 'errors', d.get('errors'))" "$1" "$2" | tee -a gpurun_out/pace_ab.log; }
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=$PWD/ab_old; else L=; fi
    for k in 256 512; do
      LD_LIBRARY_PATH=$L timeout -k 10 120 ./tools/bench_receiver drain $D/drain $k $((16 * k)) 4194304 256 > gpurun_out/pab.json 2> gpurun_out/pab.err || { echo "FAIL drain $v $k"; tail -3 gpurun_out/pab.err; exit 1; }
      show $v "drain$k"
    done
    LD_LIBRARY_PATH=$L timeout -k 10 120 ./tools/bench_receiver receiver $D 768 4 4194304 4194304 > gpurun_out/pab.json 2> gpurun_out/pab.err || { echo "FAIL receiver $v"; tail -3 gpurun_out/pab.err; exit 1; }
    show $v receiver768
    LD_LIBRARY_PATH=$L timeout -k 10 120 ./tools/bench_uploads 32 8192 4194304 32768 256 > gpurun_out/pab.json 2> gpurun_out/pab.err || { echo "FAIL uploads $v"; tail -3 gpurun_out/pab.err; exit 1; }
    show $v uploads32x256
  done
done
