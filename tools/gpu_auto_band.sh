#!/bin/bash
# AUTO's GROUP4/WIDE boundary: 4 MiB chunks at 16K..28K per launch in both shapes, one device.
#   bash tools/gpu_auto_band.sh
cd "${GRAFT_REPO_ROOT:?}" || exit 1
OUT=gpurun_out/auto_band; mkdir -p $OUT
for n in 16384 18432 20480 24576 28672; do
  for m in group4 wide plan; do
    [ $m = plan ] && mm=auto || mm=$m
    timeout -k 10 200 python bench.py --chunks $n --mode $mm --steps 3 --warmup 1 --no-cpu-baseline --host-inclusive off \
        --ingest-leg off --uploads-leg off --receiver-leg off --concurrency-leg off --mixed-leg off \
        > $OUT/${n}_$m.json 2> $OUT/${n}_$m.err || { echo "FAIL $n $m"; tail -5 $OUT/${n}_$m.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], d['value'], 'GiB/s', d['ms_per_step'], 'ms', d['config']['kernel'])" $OUT/${n}_$m.json $n $m
  done
done
echo ALL_DONE
