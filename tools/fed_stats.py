"""Developer tool: cycle accounting of the FED kernel (diagnostic build with -DEFES_FED_STATS).

Build:  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DEFES_FED_STATS -I include \\
            -o efes_amd/lib/libefeshash_stats.so efes_amd/csrc/efes_*.hip efes_amd/csrc/efes_*.cpp
Run:    EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/libefeshash_stats.so python tools/fed_stats.py [jobs]
Prints, for workgroup 0: per chain wave the cycles spent waiting for the producer and in the
whole consume loop per super-step, the producer's cycles per item, and each wave's SIMD.
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from efes_amd._lib import MODE_FED4, lib  # noqa: E402
from efes_amd.batch import DeviceBatch  # noqa: E402
from efes_amd.hashing import default_context  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 48
size = 4 << 20
ctx = default_context(0)
buf = torch.empty(n * size, dtype=torch.uint8, device="cuda:0")
ctx.fill_synthetic(buf.data_ptr(), buf.numel(), 1, torch.cuda.current_stream().cuda_stream)
b = DeviceBatch(buf.data_ptr(), np.arange(n) * size, np.full(n, size), fresh=True, ctx=ctx)
b.run(MODE_FED4)
out = (ctypes.c_ulonglong * 16)()
L = lib()
L.efes_debug_fed_stats.argtypes = [ctypes.c_void_p]
assert L.efes_debug_fed_stats(out) == 0
v = list(out)
for w in range(3):
    wait, tot, ss, hw = v[4 * w:4 * w + 4]
    if ss:
        print(f"chain {w}: simd {(hw >> 4) & 3} cu {(hw >> 8) & 15}  super-steps {ss}  cycles/super-step {tot / ss:.0f}"
              f"  waiting for the producer {wait / ss:.0f}")
tp, np_, tall, hw = v[12:16]
print(f"producer: simd {(hw >> 4) & 3} cu {(hw >> 8) & 15}  items {np_}  cycles/item {tp / max(np_, 1):.0f}"
      f"  busy {tp / max(tall, 1):.2f}")
