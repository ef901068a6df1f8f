#!/bin/bash
# Round 6 (LIBS="product jitv3 prejit" to compare more builds): where the JIT dispatcher's PATCH p99 at 192-256 uploads in flight comes from -- the product
# library against the previous dispatcher (efes_amd/lib/ab/libefeshash_prejit.so), interleaved, three
# reps of 8 rounds at 192 and 256 in flight, then a kernel trace of each at 256 (GPU gaps between DEEP
# launches: a late dispatcher wake-up idles the GPU under JIT).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r06_jit_p99}
LIBS=${LIBS:-product prejit}
mkdir -p "$O"
for lib in $LIBS; do
  [ $lib = product ] && continue
  mkdir -p /tmp/ab_$lib && cp efes_amd/lib/ab/libefeshash_$lib.so /tmp/ab_$lib/libefeshash.so
done
for rep in 1 2 3; do
  for lib in $LIBS; do
    if [ $lib = product ]; then LP=""; else LP=/tmp/ab_$lib; fi
    for k in 192 256; do
      LD_LIBRARY_PATH=$LP timeout -k 10 120 ./tools/bench_go_surface $k $((k * 8)) 4194304 32768 1 1 256 1024 \
        > "$O/lat_${lib}_${k}.$rep.json" 2> "$O/lat_${lib}_${k}.$rep.err" || { echo "lat $lib $k failed"; exit 1; }
      python3 -c "
import json,sys; d=json.loads(open('$O/lat_${lib}_${k}.$rep.json').read().strip().splitlines()[-1]); p=d['patch_group_ms']
print('rep $rep $lib $k: p50 %.2f p90 %.2f p99 %.2f ms  %.2f GiB/s  launches %d' % (p['p50'], p['p90'], p['p99'], d['value'], d['launches']))" | tee -a "$O/p99.log"
    done
  done
done
for lib in $LIBS; do
  if [ $lib = product ]; then LP=""; else LP=/tmp/ab_$lib; fi
  LD_LIBRARY_PATH=$LP timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_$lib" -o run -- \
    ./tools/bench_go_surface 256 1024 4194304 32768 1 1 256 1024 > "$O/trace_$lib.json" 2> "$O/trace_$lib.err" \
    || { echo "trace $lib failed"; tail -3 "$O/trace_$lib.err"; exit 1; }
  echo "$lib: $(python3 tools/patch_trace.py $O/trace_$lib/run_kernel_trace.csv $O/trace_$lib.json | tr '\n' ' ')" | tee -a "$O/p99.log"
done
