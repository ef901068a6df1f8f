"""Developer tool: run the golden synthetic vectors through the range-checked debug build.

Build:  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DEFES_CHECKED -I include \
            -o efes_amd/lib/libefeshash_checked.so efes_amd/csrc/efes_*.hip efes_amd/csrc/efes_*.cpp
Run:    EFES_LIB_OVERRIDE=$PWD/efes_amd/lib/libefeshash_checked.so python tools/debug_checked.py
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from efes_amd import MODE_DEEP, MODE_WIDE  # noqa: E402
from efes_amd.batch import DeviceBatch  # noqa: E402
from efes_amd.hashing import default_context  # noqa: E402
from oracle import oracle  # noqa: E402

oracle.build()
vecs = json.load(open(os.path.join(ROOT, "tests", "golden", "synthetic.json")))
ctx = default_context(0)
stride = (max(v["length"] for v in vecs) + 4096 + 4095) // 4096 * 4096
host = np.zeros(stride * len(vecs), dtype=np.uint8)
for i, v in enumerate(vecs):
    host[i * stride:i * stride + v["length"]] = oracle.fill_synthetic(v["length"], v["seed"])
buf = torch.from_numpy(host).to("cuda:0")
torch.cuda.synchronize()
mode = MODE_WIDE if "wide" in sys.argv else MODE_DEEP
bad = 0
for i, v in enumerate(vecs):
    b = DeviceBatch(buf.data_ptr(), [i * stride], [v["length"]], ctx=ctx)
    b.run(mode)
    ok = b.sha1_hex()[0] == v["sha1"] and "%08x" % b.crc_sum()[0] == v["crc32"]
    bad += not ok
    print("single", v["length"], "ok" if ok else "MISMATCH", flush=True)
b = DeviceBatch(buf.data_ptr(), [i * stride for i in range(len(vecs))], [v["length"] for v in vecs], ctx=ctx)
b.run(mode)
for v, sha, crc in zip(vecs, b.sha1_hex(), b.crc_sum()):
    if sha != v["sha1"] or "%08x" % crc != v["crc32"]:
        bad += 1
        print("batch MISMATCH", v["length"], flush=True)
print("DONE bad=%d" % bad)
