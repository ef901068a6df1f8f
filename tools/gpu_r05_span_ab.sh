#!/bin/bash
# Round 5: the read-path microbenchmark (plain / nontemporal register loads, LDS-DMA default / nt),
# then the span CRC leg with the product library and with nontemporal line loads (patched copy),
# interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r05_span_ab}
mkdir -p "$O"
timeout -k 10 150 tools/microbench/mb_glds 16 > "$O/mb_glds.log" 2>&1 || { cat "$O/mb_glds.log"; exit 1; }
cat "$O/mb_glds.log"
B="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off --latency-leg off --receiver-leg off --drain-leg off --concurrency-leg off --mixed-leg off --ingest-leg off --steps 2 --warmup 1"
for rep in 1 2; do
  for lib in product span_nt; do
    if [ $lib = product ]; then env_lib=""; else env_lib="EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/ab/libefeshash_$lib.so"; fi
    timeout -k 10 200 env $env_lib python3 bench.py $B > "$O/span_$lib.$rep.json" 2> "$O/span_$lib.$rep.err" || { tail -5 "$O/span_$lib.$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['span_crc']; print(sys.argv[2], sys.argv[3], d['value'], 'GiB/s', d['roofline']['achieved'], 'GB/s', d['roofline']['frac'], d['crc_matches_zlib'], d['clock'].get('mhz'))" "$O/span_$lib.$rep.json" $rep $lib | tee -a "$O/ab.log"
  done
done
