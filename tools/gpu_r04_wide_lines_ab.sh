#!/bin/bash
# Round 4: WIDE loading a whole 128-B line (two blocks) at a time (default build) against one block
# at a time (libefeshash_blocks.so = -DEFES_WIDE_BLOCKLOADS, the round-3 kernel): the kernel-shape
# GPU tests on the new build, then interleaved bench runs (headline, configs[4] ingest, configs[3]
# mixed), then per build the clock / VALU counters and FETCH_SIZE of a configs[4]-sized launch.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:?}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_wide_lines}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -v --timeout 200 \
  --timeout-method thread > "$O/gpu_tests.log" 2>&1
tail -2 "$O/gpu_tests.log"
LEGS="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off --latency-leg off \
 --receiver-leg off --drain-leg off --concurrency-leg off --span-leg off"
for rep in 1 2 3; do
  for lib in libefeshash_blocks.so libefeshash.so; do
    EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 $LEGS \
      > "$O/$lib.$rep.json" 2> "$O/$lib.$rep.err"
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));i=d['ingest_config'];m=d['mixed_config'];print(sys.argv[2], 'head', d['value'], 'ingest', i['value'], i['roofline']['kernel_ms'], 'mixed', m['value'], m['roofline']['kernel_ms'], 'spot', i['digests_spot_check'])" "$O/$lib.$rep.json" $lib | tee -a "$O/ab.log"
  done
done
ONE="python3 bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off --concurrency-leg off \
 --uploads-leg off --go-surface-leg off --latency-leg off --receiver-leg off --drain-leg off --span-leg off --sha1-leg off \
 --chunks 196608 --chunk-bytes 1048576 --mode wide --steps 3 --warmup 1"
for lib in libefeshash_blocks.so libefeshash.so; do
  for set in "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "FETCH_SIZE"; do
    tag=$lib.$(echo $set | cut -c1-5)
    EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/$lib timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv \
      -d "$O/pmc_$tag" -o run -- $ONE > "$O/pmc_$tag.log" 2>&1
  done
  python3 - "$O" "$lib" <<'PY' | tee -a "$O/clock.log"
import csv, glob, sys, collections, statistics
O, lib = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(f"{O}/pmc_{lib}.*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wide_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                agg["_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
m = {k: statistics.median(v) for k, v in agg.items()}
alg = 196608 * (1 << 20)
print(f"{lib:24s} kernel {m['_ns']/1e6:.2f} ms  clock {m['GRBM_GUI_ACTIVE']/8/m['_ns']:.3f} GHz  "
      f"VALU busy {m['SQ_ACTIVE_INST_VALU']*4/1024/(m['GRBM_GUI_ACTIVE']/8):.3f}  VALU/block {m['SQ_INSTS_VALU']/(3072*16384):.1f}  "
      f"LDS conflicts/instr {m['SQ_LDS_BANK_CONFLICT']/m['SQ_INSTS_LDS']:.2f}  "
      f"FETCH_SIZE x2 / algorithmic {m['FETCH_SIZE']*1024*2/alg:.4f}")
PY
done
