#!/bin/bash
# Round 5: the default bench line (every leg, with the clock meter) and the WIDE pacing A/B on
# configs[4] (the product library against two patched-copy builds from tools/ab_variant.sh,
# interleaved, each line with its clock and binding-roofline fraction at that clock).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_bench_ab}
mkdir -p "$O"
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -5 "$O/bench.err"; exit 1; }
echo bench ok
for rep in 1 2; do
  for lib in product pace32 nopace; do
    if [ $lib = product ]; then env_lib=""; else env_lib="EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/ab/libefeshash_$lib.so"; fi
    timeout -k 10 300 env $env_lib python3 bench.py --workload ingest --no-cpu-baseline > "$O/ab_$lib.$rep.json" 2> "$O/ab_$lib.$rep.err" \
      || { echo "ab $lib failed"; tail -5 "$O/ab_$lib.$rep.err"; exit 1; }
    python3 - "$O/ab_$lib.$rep.json" $lib $rep <<'PY' | tee -a "$O/ab.log"
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b = d["binding_roofline"]; c = d["clock"]
print(f"rep {sys.argv[3]} {sys.argv[2]:8s} {d['value']:9.1f} GiB/s  kernel {d['roofline']['kernel_ms']:7.3f} ms  clock smi {c.get('smi_mhz_mean')} probe {c.get('probe_mhz')} MHz  frac@2.4 {b['frac']}  frac@clock {b.get('frac_at_clock')}")
PY
  done
done
