// mb_wide_fetch.hip -- calibrates rocprofv3's FETCH_SIZE for the WIDE kernel's access pattern
// (DESIGN_NOTES.md §4 "WIDE at full load").  MI355X_MICROARCH.md calibrates FETCH_SIZE
// only for wide coalesced streams (it reports exactly half of their bytes); WIDE instead reads, per
// lane, its own message in 64-B blocks as four 16-B global_load_dwordx4 (one lane per message, so one
// wave-instruction touches 64 distinct cache lines), two blocks ahead of the block being hashed.
// This program reads a KNOWN byte count -- every byte of `lanes` messages of `msg` bytes, once -- in
// the same geometry as a configs[4] launch (196 608 lanes of 1 MiB, one 768-lane workgroup per CU =
// three waves per SIMD), in three shapes:
//   coal    : each wave-instruction reads 1 KiB contiguous (the guide's calibrated case)
//   wide64  : WIDE's order -- per lane block b hashed while b+1, b+2 are in flight (three 64-B buffers)
//   wide128 : per lane two blocks (a whole 128-B line) loaded back to back, the next line in flight
// with `pad` dependent VALU ops per 64-B block standing in for the SHA-1 + CRC work (≈ 700 in WIDE),
// so the time between the two halves of a 128-B line is WIDE's.  Run it under
//   rocprofv3 --pmc FETCH_SIZE -- tools/microbench/mb_wide_fetch
// and divide FETCH_SIZE (KiB) x 1024 by the bytes printed: that is the counter's factor for the shape.
// Usage: mb_wide_fetch [lanes] [msg_bytes] [pad] [reps]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct Blk {
  v4u q[4];
};

__device__ __forceinline__ Blk load64(const v4u* p) {
  Blk b;
#pragma unroll
  for (int k = 0; k < 4; ++k) b.q[k] = p[k];
  return b;
}

// The block's "hash": fold it into acc, then `pad` dependent VALU pairs (WIDE's work per block).
__device__ __forceinline__ void work(v4u& acc, const Blk& b, uint32_t pad) {
#pragma unroll
  for (int k = 0; k < 4; ++k) acc ^= b.q[k];
  for (uint32_t i = 0; i < pad; ++i) {
    acc.x = __builtin_amdgcn_alignbit(acc.x, acc.y, 5) + acc.z;
    acc.y ^= acc.x;
  }
}

// Lane j reads message j: nblk 64-B blocks at base + j * msg.
__global__ __launch_bounds__(768, 1) void wide64(const uint8_t* __restrict__ base, uint64_t msg, uint64_t nblk,
                                                 uint32_t pad, uint32_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const v4u* q = reinterpret_cast<const v4u*>(base + j * msg);
  v4u acc = {0, 0, 0, 0};
  Blk A = load64(q), B = load64(q + 4), C;
  uint64_t b = 0;
  for (; b + 3 <= nblk; b += 3) {  // as wide_bulk: block b hashed while b+1, b+2 are in flight
    C = b + 2 < nblk ? load64(q + 4 * (b + 2)) : A;
    work(acc, A, pad);
    A = b + 3 < nblk ? load64(q + 4 * (b + 3)) : A;
    work(acc, B, pad);
    B = b + 4 < nblk ? load64(q + 4 * (b + 4)) : B;
    work(acc, C, pad);
  }
  for (; b < nblk; ++b) {
    work(acc, A, pad);
    A = B;
  }
  out[j] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// Lane j reads message j a whole 128-B line (two blocks) at a time, the next line in flight.
__global__ __launch_bounds__(768, 1) void wide128(const uint8_t* __restrict__ base, uint64_t msg, uint64_t nblk,
                                                  uint32_t pad, uint32_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const v4u* q = reinterpret_cast<const v4u*>(base + j * msg);
  v4u acc = {0, 0, 0, 0};
  Blk A0 = load64(q), A1 = load64(q + 4), B0, B1;
  for (uint64_t b = 0; b + 2 <= nblk; b += 2) {
    const bool more = b + 2 < nblk;
    B0 = more ? load64(q + 4 * (b + 2)) : A0;
    B1 = more ? load64(q + 4 * (b + 3)) : A1;
    work(acc, A0, pad);
    work(acc, A1, pad);
    A0 = B0;
    A1 = B1;
  }
  out[j] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// The same bytes read coalesced: wave-instruction k of the grid reads 1 KiB contiguous.
__global__ __launch_bounds__(768, 1) void coal(const uint8_t* __restrict__ base, uint64_t total, uint32_t pad,
                                               uint32_t* __restrict__ out) {
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x, j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const v4u* p = reinterpret_cast<const v4u*>(base);
  v4u acc = {0, 0, 0, 0};
  const uint64_t rows = total / (16 * lanes);
  for (uint64_t r = 0; r < rows; r += 4) {
    Blk b;
#pragma unroll
    for (int k = 0; k < 4; ++k) b.q[k] = r + k < rows ? p[(r + k) * lanes + j] : v4u{0, 0, 0, 0};
    work(acc, b, pad);
  }
  out[j] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

__global__ void fill_random(uint64_t* d, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    d[i] = z ^ (z >> 31);
  }
}

int main(int argc, char** argv) {
  const uint64_t lanes = argc > 1 ? strtoull(argv[1], 0, 10) : 196608;
  const uint64_t msg = argc > 2 ? strtoull(argv[2], 0, 10) : (1u << 20);
  const uint32_t pad = argc > 3 ? (uint32_t)atoi(argv[3]) : 0;
  const int reps = argc > 4 ? atoi(argv[4]) : 3;
  if (lanes % 768 || msg % 128 || lanes == 0 || msg == 0) {
    fprintf(stderr, "lanes must be a multiple of 768, msg a multiple of 128\n");
    return 2;
  }
  const uint64_t total = lanes * msg, nblk = msg / 64;
  uint8_t* d = nullptr;
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&d, total));
  CHECK(hipMalloc(reinterpret_cast<void**>(&out), lanes * 4));
  hipLaunchKernelGGL(fill_random, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(d), total / 8);
  CHECK(hipDeviceSynchronize());
  const dim3 grid((uint32_t)(lanes / 768)), block(768);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int shape = 0; shape < 3; ++shape) {
    const char* name = shape == 0 ? "coal" : shape == 1 ? "wide64" : "wide128";
    float ms_sum = 0;
    for (int r = 0; r < reps; ++r) {
      CHECK(hipEventRecord(a, 0));
      if (shape == 0) hipLaunchKernelGGL(coal, grid, block, 0, 0, d, total, pad, out);
      else if (shape == 1) hipLaunchKernelGGL(wide64, grid, block, 0, 0, d, msg, nblk, pad, out);
      else hipLaunchKernelGGL(wide128, grid, block, 0, 0, d, msg, nblk, pad, out);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(b, 0));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      ms_sum += ms;
    }
    const double ms = ms_sum / reps;
    printf("{\"shape\": \"%s\", \"lanes\": %llu, \"msg_bytes\": %llu, \"pad\": %u, \"bytes_per_dispatch\": %llu, "
           "\"ms\": %.3f, \"TB/s\": %.3f}\n", name, (unsigned long long)lanes, (unsigned long long)msg, pad,
           (unsigned long long)total, ms, total / (ms * 1e-3) / 1e12);
    fflush(stdout);
  }
  CHECK(hipFree(d));
  CHECK(hipFree(out));
  return 0;
}
