#!/bin/bash
# Round 6 (LIBS="product jitv3 prejit" for more builds): just-in-time batch assembly in the upload dispatcher (efes_queue.cpp) against the previous
# dispatcher (tools/ab_variant.sh prejit "git:<rev>" efes_queue.cpp), interleaved on one box: one 4 MiB
# PATCH's latency at 1 / 16 / 64 / 256 uploads in flight (the patch_latency leg's harness), the
# unchanged Go surface at 8 192 in flight (go_surface_path) and efes_upload (uploads_path).  The
# harnesses link libefeshash through RUNPATH, so LD_LIBRARY_PATH selects the variant.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r06_jit_ab}
LIBS=${LIBS:-product prejit}
mkdir -p "$O"
for lib in $LIBS; do
  [ $lib = product ] && continue
  mkdir -p /tmp/ab_$lib && cp efes_amd/lib/ab/libefeshash_$lib.so /tmp/ab_$lib/libefeshash.so
done
for rep in 1 2; do
  for lib in $LIBS; do
    if [ $lib = product ]; then LP=""; else LP=/tmp/ab_$lib; fi
    for k in 1 16 64 256; do
      rounds=$([ $k = 1 ] && echo 20 || ([ $k -le 16 ] && echo 8 || ([ $k -le 64 ] && echo 6 || echo 4)))
      LD_LIBRARY_PATH=$LP timeout -k 10 120 ./tools/bench_go_surface $k $((k * rounds)) 4194304 32768 1 1 256 1024 \
        > "$O/lat_${lib}_${k}.$rep.json" 2> "$O/lat_${lib}_${k}.$rep.err" || { echo "lat $lib $k failed"; tail -5 "$O/lat_${lib}_${k}.$rep.err"; exit 1; }
    done
    LD_LIBRARY_PATH=$LP timeout -k 10 200 ./tools/bench_go_surface 32 8192 4194304 32768 256 1 256 8208 \
      > "$O/surface_$lib.$rep.json" 2> "$O/surface_$lib.$rep.err" || { echo "surface $lib failed"; tail -5 "$O/surface_$lib.$rep.err"; exit 1; }
    LD_LIBRARY_PATH=$LP timeout -k 10 200 ./tools/bench_uploads 32 8192 4194304 32768 256 \
      > "$O/uploads_$lib.$rep.json" 2> "$O/uploads_$lib.$rep.err" || { echo "uploads $lib failed"; tail -5 "$O/uploads_$lib.$rep.err"; exit 1; }
    python3 - "$O" $lib $rep <<'PY' | tee -a "$O/ab.log"
import json, sys
O, lib, rep = sys.argv[1:]
def j(f): return json.loads(open(f"{O}/{f}").read().strip().splitlines()[-1])
lat = []
for k in (1, 16, 64, 256):
    d = j(f"lat_{lib}_{k}.{rep}.json"); p = d["patch_group_ms"]
    assert d["all_equal"] and d["errors"] == 0
    lat.append(f"{k}:{p['p50']:.2f}/{p['p99']:.2f}ms {d['value']:.2f}GiB/s")
s, u = j(f"surface_{lib}.{rep}.json"), j(f"uploads_{lib}.{rep}.json")
assert s["all_equal"] and u["all_sums_equal"]
print(f"rep {rep} {lib:8s} PATCH p50/p99: {'  '.join(lat)} | go_surface {s['value']:.2f} GiB/s ({s['launches']} launches) | uploads {u['value']:.2f} GiB/s")
PY
  done
done
