"""How much do WIDE's LDS bank conflicts cost?  (DESIGN_NOTES.md §4 "WIDE at full load".)

WIDE's CRC-32 looks up pos[o][byte] for the 64 byte positions o of every block; for one position all
lanes of a 32-lane group read the same 1 KiB table, so the bank is byte mod 32 and random bytes give
random bank conflicts (4.27 extra LDS cycles per ds_read_b32 in profiles/r03_wide_crc_pmc).  Instead of
building a conflict-free table layout first, this probe runs the SAME kernel on data that decides the
banks: a configs[4]-sized launch (196 608 messages of 1 MiB, one per lane) whose lane j has bytes
  random         : splitmix64 (the benchmarks' data)
  conflict_free  : (j mod 32) + 32 * r, r random in 0..7 -- the 32 lanes of a group hit 32 banks
  same_bank      : 5 + 32 * r -- every lane of a group on one bank (up to 8-way)
(60 of the 64 lookups per block index data bytes; the first four index crc ^ data).  Timed with HIP
events; run under rocprofv3 --pmc for the clock (GRBM_GUI_ACTIVE) and SQ_LDS_BANK_CONFLICT.
Prints one JSON line per mode.  Digests of two lanes per mode are checked against hashlib/zlib.

    python tools/wide_lds_probe.py [modes...]
"""
import hashlib
import json
import os
import sys
import zlib

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from efes_amd import MODE_WIDE  # noqa: E402
from efes_amd.batch import DeviceBatch  # noqa: E402
from efes_amd.hashing import default_context  # noqa: E402


def main(modes):
    m, seg = 196608, 1 << 20
    ctx = default_context(0)
    data = torch.empty(m * seg, dtype=torch.uint8, device="cuda:0")
    offs, lens = np.arange(m, dtype=np.uint64) * np.uint64(seg), np.full(m, seg, np.uint64)
    for mode in modes:
        if mode == "random":
            ctx.fill_synthetic(data.data_ptr(), data.numel(), 0x1DA7A, torch.cuda.current_stream().cuda_stream)
        else:
            rows = 8192  # 8 GiB at a time
            g = torch.Generator(device="cuda:0").manual_seed(7)
            for r0 in range(0, m, rows):
                r = torch.randint(0, 8, (rows, seg), dtype=torch.uint8, device="cuda:0", generator=g) * 32
                if mode == "conflict_free":
                    r += (torch.arange(r0, r0 + rows, device="cuda:0", dtype=torch.int64) % 32).to(torch.uint8)[:, None]
                else:
                    r += 5
                data.view(m, seg)[r0:r0 + rows].copy_(r)
                del r
        torch.cuda.synchronize()
        b = DeviceBatch(data.data_ptr(), offs, lens, fresh=True, ctx=ctx)
        b.run(MODE_WIDE)  # warm-up
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        e0.record()
        for _ in range(reps):
            b.submit(MODE_WIDE)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        ok = bool((b.status_host() == 0).all())
        shas, crcs = b.sha1_hex(), b.crc_sum()
        for j in (0, m - 1):
            d = data[j * seg:(j + 1) * seg].cpu().numpy().tobytes()
            ok = ok and shas[j] == hashlib.sha1(d).hexdigest() and int(crcs[j]) == zlib.crc32(d)
        print(json.dumps({"mode": mode, "messages": m, "bytes": m * seg, "ms_per_launch": round(ms, 3),
                          "GB/s": round(m * seg / (ms * 1e-3) / 1e9, 1), "digests_ok": ok}), flush=True)
        del b


if __name__ == "__main__":
    main(sys.argv[1:] or ["random", "conflict_free", "same_bank"])
