"""Developer tool: the per-wave timeline of one WIDE launch (diagnostic build -DEFES_WIDE_STATS).

Build:  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DEFES_WIDE_STATS -I include \\
            -o efes_amd/lib/libefeshash_widestats.so efes_amd/csrc/efes_*.hip efes_amd/csrc/efes_*.cpp
Run:    EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/libefeshash_widestats.so python tools/wide_stats.py [chunks] [chunk_bytes]
Prints when the waves start and end (s_memtime, relative to the launch), and for the waves that
share a SIMD the order in which they finish -- whether a launch's tail is waves running alone.
"""
import collections
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from efes_amd._lib import MODE_WIDE, lib  # noqa: E402
from efes_amd.batch import DeviceBatch  # noqa: E402
from efes_amd.hashing import default_context  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 196608
size = int(sys.argv[2]) if len(sys.argv) > 2 else 4 << 20
pool = int(sys.argv[3]) << 30 if len(sys.argv) > 3 else 16 << 30  # GiB; n * size <= pool: no aliasing
ctx = default_context(0)
buf = torch.empty(pool, dtype=torch.uint8, device="cuda:0")
ctx.fill_synthetic(buf.data_ptr(), pool, 1, torch.cuda.current_stream().cuda_stream)
slots = pool // size
b = DeviceBatch(buf.data_ptr(), (np.arange(n) % slots) * size, np.full(n, size), fresh=True, ctx=ctx)
b.run(MODE_WIDE)  # warm-up
b.reset()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
b.submit(MODE_WIDE)  # two launches back to back (as bench.py's steps): the stats are the second's
b.submit(MODE_WIDE)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 2
W = 8192
out = (ctypes.c_ulonglong * (W * 6))()
L = lib()
L.efes_debug_wide_stats.argtypes = [ctypes.c_void_p]
assert L.efes_debug_wide_stats(out) == 0
v = np.frombuffer(out, dtype=np.uint64).reshape(W, 6)[: (n + 63) // 64].astype(np.int64)
t0, t1, t2, hw, xcc, rt = v.T
r0 = rt & 0xFFFFFFFF  # s_memrealtime (100 MHz, one clock for the whole chip) at entry, and the lifetime
rlife = rt >> 32
r0 = (r0 - r0.min()) & 0xFFFFFFFF
np.save(os.path.join(ROOT, "gpurun_out", f"wide_stats_raw_f{os.environ.get('EFES_WIDE_FAIR', 'd')}.npy"), v)
# s_memtime counts per XCD with its own offset: times are taken relative to each XCD's first start
xs = (xcc & 0xF).astype(int)
base = np.zeros(len(v), np.int64)
span = np.zeros(len(v), np.int64)
for x in np.unique(xs):
    m = xs == x
    base[m] = t0[m].min()
    span[m] = t2[m].max() - t0[m].min()
rel = lambda t: (t - base) / span  # noqa: E731
simd_key = collections.defaultdict(list)
for i in range(v.shape[0]):
    h = int(hw[i])
    key = (int(xs[i]), (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 15, (h >> 4) & 3)
    simd_key[key].append((float(rel(t2)[i]), h & 15, float(rel(t0)[i])))
per = collections.Counter(len(x) for x in simd_key.values())
rank_end = collections.defaultdict(list)
for waves in simd_key.values():
    for r, (end, slot, start) in enumerate(sorted(waves)):
        rank_end[(len(waves), r)].append(end)
ticks_per_ms = float(np.median(span)) / ms
res = {
    "chunks": n, "chunk_bytes": size, "kernel_ms_events": round(ms, 3), "waves": int(v.shape[0]),
    "xcds": int(len(np.unique(xs))), "memtime_ticks_per_ms": round(ticks_per_ms, 1),
    "fair_env": os.environ.get("EFES_WIDE_FAIR", "default"),
    "start_rel_pct": [round(float(x), 4) for x in np.percentile(rel(t0), [0, 50, 90, 99, 100])],
    "bulk_end_rel_pct": [round(float(x), 4) for x in np.percentile(rel(t1), [0, 10, 50, 90, 100])],
    "end_rel_pct": [round(float(x), 4) for x in np.percentile(rel(t2), [0, 10, 50, 90, 100])],
    "mean_lifetime_rel": round(float(np.mean(rel(t2) - rel(t0))), 4),
    "realtime_start_ms_pct": [round(float(x) / 1e5, 3) for x in np.percentile(r0, [0, 10, 50, 90, 100])],
    "realtime_end_ms_pct": [round(float(x) / 1e5, 3) for x in np.percentile(r0 + rlife, [0, 10, 50, 90, 100])],
    "realtime_life_ms_by_slot": {int(sl): [round(float(x) / 1e5, 2) for x in np.percentile(rlife[(hw & 15) == sl],
                                                                                       [0, 50, 100])]
                                 for sl in np.unique(hw & 15)},
    "waves_per_simd_histogram": {str(k): c for k, c in sorted(per.items())},
    "mean_end_by_rank_on_simd": {f"{k[0]}w_rank{k[1]}": round(float(np.mean(e)), 4) for k, e in sorted(rank_end.items())},
}
print(json.dumps(res))
