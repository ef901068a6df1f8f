"""Round 5 diagnostic: does the span CRC's rate depend on where its 16 GiB buffer was allocated?
Times efes_crc32_span on a buffer allocated first (A), then after a 200 GiB allocation is made and
freed (B), then on A again -- nothing else runs in between."""
import sys
import time

import torch

sys.path.insert(0, ".")
from efes_amd import hashing  # noqa: E402


def rate(ctx, buf, st, stream, reps=5):
    n = buf.numel()
    ctx.crc32_span(buf.data_ptr(), n, st.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        ctx.crc32_span(buf.data_ptr(), n, st.data_ptr(), stream.cuda_stream)
    e1.record(stream)
    stream.synchronize()
    return n / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9


def main():
    ctx = hashing.default_context(0)
    stream = torch.cuda.Stream()
    n = 16 << 30
    st = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    a = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    ctx.fill_synthetic(a.data_ptr(), n, 0x5BA4, stream.cuda_stream)
    print(f"A (allocated first): {rate(ctx, a, st, stream):.1f} GB/s", flush=True)
    big = torch.empty(200 << 30, dtype=torch.uint8, device="cuda:0")
    big[:: 1 << 20].fill_(1)  # touch it
    torch.cuda.synchronize()
    del big
    torch.cuda.empty_cache()
    b = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    ctx.fill_synthetic(b.data_ptr(), n, 0x5BA4, stream.cuda_stream)
    print(f"B (after a 200 GiB alloc/free): {rate(ctx, b, st, stream):.1f} GB/s", flush=True)
    print(f"A again: {rate(ctx, a, st, stream):.1f} GB/s", flush=True)
    del b
    torch.cuda.empty_cache()
    c = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    ctx.fill_synthetic(c.data_ptr(), n, 0x5BA4, stream.cuda_stream)
    print(f"C (another fresh 16 GiB): {rate(ctx, c, st, stream):.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
