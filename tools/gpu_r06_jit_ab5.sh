#!/bin/bash
# Round 6: the JIT dispatcher's tail at high load -- builds in $LIBS (product = the tree's library, others
# efes_amd/lib/ab/libefeshash_<name>.so), interleaved, two reps: one 4 MiB PATCH's latency at 1, 16, 64,
# 128, 192 and 256 uploads in flight (the patch_latency leg's rounds: 20 / 8 / 6 / 4 / 4 / 4 PATCHes per
# thread) and the Go surface at 8 192 in flight.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r06_jit_ab5}
LIBS=${LIBS:-product prejit}
mkdir -p "$O"
for lib in $LIBS; do
  [ $lib = product ] && continue
  mkdir -p /tmp/ab_$lib && cp efes_amd/lib/ab/libefeshash_$lib.so /tmp/ab_$lib/libefeshash.so
done
for rep in 1 2; do
  for lib in $LIBS; do
    if [ $lib = product ]; then LP=""; else LP=/tmp/ab_$lib; fi
    line="rep $rep $(printf %-8s $lib)"
    for k in 1 16 64 128 192 256; do
      rounds=$([ $k = 1 ] && echo 20 || ([ $k -le 16 ] && echo 8 || ([ $k -le 64 ] && echo 6 || echo 4)))
      LD_LIBRARY_PATH=$LP timeout -k 10 120 ./tools/bench_go_surface $k $((k * rounds)) 4194304 32768 1 1 256 1024 \
        > "$O/lat_${lib}_${k}.$rep.json" 2> "$O/lat_${lib}_${k}.$rep.err" || { echo "lat $lib $k failed"; exit 1; }
      line="$line $(python3 -c "
import json; d=json.loads(open('$O/lat_${lib}_${k}.$rep.json').read().strip().splitlines()[-1]); p=d['patch_group_ms']
assert d['all_equal'] and d['errors'] == 0
print('%d:%.2f/%.2f/%.2fms %.2fG' % ($k, p['p50'], p['p90'], p['p99'], d['value']))")"
    done
    LD_LIBRARY_PATH=$LP timeout -k 10 200 ./tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 \
      > "$O/surface_$lib.$rep.json" 2> "$O/surface_$lib.$rep.err" || { echo "surface $lib failed"; exit 1; }
    line="$line | surface $(python3 -c "import json; print(json.loads(open('$O/surface_$lib.$rep.json').read().strip().splitlines()[-1])['value'])")"
    echo "$line" | tee -a "$O/ab.log"
  done
done
