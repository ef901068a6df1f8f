#!/bin/bash
# Round 5: the span leg run after the mixed leg in one process (its buffer allocated after the
# 200 GiB pool was freed), product against A/B builds, interleaved, twice.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r05_span_after_mixed}
shift || true
mkdir -p "$O"
B="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off --latency-leg off \
 --receiver-leg off --drain-leg off --concurrency-leg off --ingest-leg off --mixed-leg on --steps 2 --warmup 1"
for rep in 1 2; do
  for lib in product "$@"; do
    env_lib=""; [ "$lib" = product ] || env_lib="EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/ab/libefeshash_$lib.so"
    timeout -k 10 300 env $env_lib python3 bench.py $B > "$O/$lib.$rep.json" 2> "$O/$lib.$rep.err" || { tail -5 "$O/$lib.$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['span_crc']; m=d['mixed_config']; print(sys.argv[2], sys.argv[3], 'span', s['value'], 'GiB/s', s['roofline']['achieved'], 'GB/s', s['clock'].get('mhz'), 'MHz', s['crc_matches_zlib'], '| mixed', m['value'])" "$O/$lib.$rep.json" $rep $lib | tee -a "$O/ab.log"
  done
done
