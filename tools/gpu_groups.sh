# Grouped-DEEP calibration: one wave per SIMD for each lanes-per-job (n jobs x 4 MiB, 64/n jobs per wave).
cd "${GRAFT_REPO_ROOT:?}" || exit 1
mkdir -p gpurun_out/groups
one() {  # tag chunks mode
  timeout -k 10 300 python bench.py --chunks $2 --mode $3 --steps 3 --warmup 1 --no-cpu-baseline --host-inclusive off \
      --ingest-leg off --mixed-leg off > gpurun_out/groups/$1.json 2> gpurun_out/groups/$1.err || { echo "FAIL $1"; tail -5 gpurun_out/groups/$1.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms/launch')" gpurun_out/groups/$1.json $1
}
one deep1024 1024 deep
one g32_2048 2048 group32
one g16_4096 4096 group16
one g8_8192 8192 group8
one g4_16384 16384 group4
one wide8192 8192 wide
one deep8192 8192 deep
one g8_16384 16384 group8
