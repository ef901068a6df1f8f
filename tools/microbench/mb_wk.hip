// Microbenchmark: cost of feeding W[i]+K[i] to a lone-wave SHA-1 chain on gfx950.
//   regs : WK held in VGPRs (no loads in the loop) -- the pure 405-VALU floor
//   lds  : 20 ds_read_b128 per block right before use (the DEEP kernel today)
//   pipe : next block's 20 ds_read_b128 issued while the current block runs (2x unrolled)
// Not part of the product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include "../../efes_amd/csrc/sha1_device.hpp"
using namespace efes;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1;}}while(0)

template <int Q> struct RegQuad {
  __device__ __forceinline__ static void run(uint32_t (&s)[5], const uint4 (&w)[20]) {
    round_wk<4 * Q + 0>(s, w[Q].x); round_wk<4 * Q + 1>(s, w[Q].y);
    round_wk<4 * Q + 2>(s, w[Q].z); round_wk<4 * Q + 3>(s, w[Q].w);
    RegQuad<Q + 1>::run(s, w);
  }
};
template <> struct RegQuad<20> { __device__ __forceinline__ static void run(uint32_t (&)[5], const uint4 (&)[20]) {} };
__device__ __forceinline__ void compress_regs(uint32_t (&h)[5], const uint4 (&w)[20]) {
  uint32_t s[5] = {h[0], h[1], h[2], h[3], h[4]};
  RegQuad<0>::run(s, w);
  h[0] += s[0]; h[1] += s[1]; h[2] += s[2]; h[3] += s[3]; h[4] += s[4];
}

template <int Q> struct SQuad {
  __device__ __forceinline__ static void run(uint32_t (&s)[5], const uint32_t (&w)[80]) {
    round_wk<4 * Q + 0>(s, w[4 * Q]); round_wk<4 * Q + 1>(s, w[4 * Q + 1]);
    round_wk<4 * Q + 2>(s, w[4 * Q + 2]); round_wk<4 * Q + 3>(s, w[4 * Q + 3]);
    SQuad<Q + 1>::run(s, w);
  }
};
template <> struct SQuad<20> { __device__ __forceinline__ static void run(uint32_t (&)[5], const uint32_t (&)[80]) {} };

// WK from a read-only global ring through scalar loads (uniform address -> s_load_dwordx16).
template <int RING>
__global__ __launch_bounds__(64) void ks(const uint32_t* __restrict__ g, uint32_t* out, uint64_t* cyc, int nblocks) {
  uint32_t h[5] = {0x67452301u + blockIdx.x, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int b = 0; b < nblocks; ++b) {
    struct alignas(64) V16 { uint4 q[4]; };
    const V16* w16 = reinterpret_cast<const V16*>(g + (b & (RING - 1)) * 80);
    uint32_t w[80];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const V16 v = w16[i];
#pragma unroll
      for (int k = 0; k < 4; ++k) { w[16*i+4*k] = v.q[k].x; w[16*i+4*k+1] = v.q[k].y; w[16*i+4*k+2] = v.q[k].z; w[16*i+4*k+3] = v.q[k].w; }
    }
    uint32_t s[5] = {h[0], h[1], h[2], h[3], h[4]};
    SQuad<0>::run(s, w);
    h[0] += s[0]; h[1] += s[1]; h[2] += s[2]; h[3] += s[3]; h[4] += s[4];
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// ---- scalar-fed chain: WK streamed into SGPRs by s_load (glc: straight from L2), one quarter
// (20 words) ahead, double-buffered.  SMEM returns out of order, so each wait is lgkmcnt(0);
// the wait names the buffer it guards ("+s") so no use of it can be scheduled above it.
typedef uint32_t v16u __attribute__((ext_vector_type(16)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
struct QBuf { v16u a; v4u b; };
__device__ __forceinline__ void sload_q(QBuf& q, const uint32_t* p) {
  asm volatile("s_load_dwordx16 %0, %2, 0x0 glc\n\ts_load_dwordx4 %1, %2, 0x40 glc" : "=s"(q.a), "=s"(q.b) : "s"(p) : "memory");
}
__device__ __forceinline__ void swait_q(QBuf& q) { asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(q.a), "+s"(q.b) :: "memory"); }
template <int Q, int I> struct SQ20 {
  __device__ __forceinline__ static void run(uint32_t (&s)[5], const QBuf& w) {
    round_wk<20 * Q + I>(s, I < 16 ? w.a[I & 15] : w.b[(I - 16) & 3]);
    SQ20<Q, I + 1>::run(s, w);
  }
};
template <int Q> struct SQ20<Q, 20> { __device__ __forceinline__ static void run(uint32_t (&)[5], const QBuf&) {} };

__global__ __launch_bounds__(64) void kq(const uint32_t* __restrict__ g, uint32_t* out, uint64_t* cyc, int nblocks) {
  uint32_t h[5] = {0x67452301u + blockIdx.x, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  const uint32_t* base = g;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  QBuf A, B;
  sload_q(A, base);
  for (int b = 0; b < nblocks; ++b) {
    const uint32_t* w = base + (b & 63) * 80;
    const uint32_t* wn = base + ((b + 1) & 63) * 80;
    uint32_t s[5] = {h[0], h[1], h[2], h[3], h[4]};
    swait_q(A); sload_q(B, w + 20); SQ20<0, 0>::run(s, A);
    swait_q(B); sload_q(A, w + 40); SQ20<1, 0>::run(s, B);
    swait_q(A); sload_q(B, w + 60); SQ20<2, 0>::run(s, A);
    swait_q(B); sload_q(A, wn);     SQ20<3, 0>::run(s, B);
    h[0] += s[0]; h[1] += s[1]; h[2] += s[2]; h[3] += s[3]; h[4] += s[4];
  }
  swait_q(A);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// WK from global memory with vector loads (uniform address: one cache line per instruction),
// next block prefetched into a second register set while the current block runs.
template <int ALL>
__global__ __launch_bounds__(64) void kg(const uint32_t* __restrict__ g, uint32_t* out, uint64_t* cyc, int nblocks) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const __attribute__((address_space(1))) v4u* ring = (const __attribute__((address_space(1))) v4u*)g;
  uint32_t h[5] = {0x67452301u + blockIdx.x, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  const bool fetch = ALL || (threadIdx.x & 63) == 0;
  uint32_t vz = 0;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vz));  // a VGPR zero: keeps the loads on the vector path
  ring += vz;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint4 A[20], B[20];
  if (fetch) {
#pragma unroll
    for (int q = 0; q < 20; ++q) { v4u v = ring[q]; A[q] = make_uint4(v.x, v.y, v.z, v.w); }
  }
  for (int b = 0; b < nblocks; b += 2) {
    if (fetch) {
#pragma unroll
      for (int q = 0; q < 20; ++q) { v4u v = ring[((b + 1) & 63) * 20 + q]; B[q] = make_uint4(v.x, v.y, v.z, v.w); }
    }
    compress_regs(h, A);
    if (fetch) {
#pragma unroll
      for (int q = 0; q < 20; ++q) { v4u v = ring[((b + 2) & 63) * 20 + q]; A[q] = make_uint4(v.x, v.y, v.z, v.w); }
    }
    compress_regs(h, B);
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
__global__ __launch_bounds__(64) void k(uint32_t* out, uint64_t* cyc, int nblocks) {
  __shared__ __attribute__((aligned(16))) uint4 ring[64][20];
  for (int i = threadIdx.x; i < 64 * 20; i += 64) ring[i / 20][i % 20] = make_uint4(i * 0x9E3779B9u, i, i ^ 7, i * 3);
  __syncthreads();
  uint32_t h[5] = {0x67452301u + blockIdx.x, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  if constexpr (MODE == 0) {
    uint4 w[20];
    for (int q = 0; q < 20; ++q) w[q] = ring[q][q];
    for (int b = 0; b < nblocks; ++b) compress_regs(h, w);
  } else if constexpr (MODE == 1) {
    for (int b = 0; b < nblocks; ++b) compress_wk(h, ring[b & 63]);
  } else if constexpr (MODE == 3 || MODE == 4) {
    // Only a few lanes fetch WK (the chain's result is read from lane 0 only).
    const bool fetch = MODE == 3 ? (threadIdx.x & 63) < 16 : (threadIdx.x & 63) == 0;
    for (int b = 0; b < nblocks; ++b) {
      uint4 w[20];
      if (fetch) {
#pragma unroll
        for (int q = 0; q < 20; ++q) w[q] = ring[b & 63][q];
      }
      compress_regs(h, w);
    }
  } else if constexpr (MODE == 5) {
    const bool fetch = (threadIdx.x & 63) == 0;
    uint4 A[20], B[20];
    if (fetch) {
#pragma unroll
      for (int q = 0; q < 20; ++q) A[q] = ring[0][q];
    }
    for (int b = 0; b < nblocks; b += 2) {
      if (fetch) {
#pragma unroll
        for (int q = 0; q < 20; ++q) B[q] = ring[(b + 1) & 63][q];
      }
      compress_regs(h, A);
      if (fetch) {
#pragma unroll
        for (int q = 0; q < 20; ++q) A[q] = ring[(b + 2) & 63][q];
      }
      compress_regs(h, B);
    }
  } else {
    uint4 A[20], B[20];
#pragma unroll
    for (int q = 0; q < 20; ++q) A[q] = ring[0][q];
    for (int b = 0; b < nblocks; b += 2) {
#pragma unroll
      for (int q = 0; q < 20; ++q) B[q] = ring[(b + 1) & 63][q];
      compress_regs(h, A);
#pragma unroll
      for (int q = 0; q < 20; ++q) A[q] = ring[(b + 2) & 63][q];
      compress_regs(h, B);
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  uint32_t* out; uint64_t* cyc;
  CK(hipMalloc(&out, 1 << 24)); CK(hipMalloc(&cyc, 1 << 20));
  std::vector<uint64_t> hc(2048);
  const int nb = 20000;
  auto run = [&](const char* name, auto kern, int grid) {
    hipLaunchKernelGGL(kern, grid, 64, 0, 0, out, cyc, 16); CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0)); hipLaunchKernelGGL(kern, grid, 64, 0, 0, out, cyc, nb); CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(hc.data(), cyc, 8 * grid, hipMemcpyDeviceToHost));
    double mx = 0; for (int i = 0; i < grid; ++i) mx = hc[i] > mx ? hc[i] : mx;
    printf("%-10s grid=%5d cyc/block=%7.1f  wall/block=%6.1f ns  per-msg %.1f MB/s  aggregate %.1f GB/s\n", name, grid,
           mx / nb, ms * 1e6 / nb, nb * 64.0 / (ms * 1e3), grid * nb * 64.0 / (ms * 1e6));
    return 0;
  };
  uint32_t* gring; CK(hipMalloc(&gring, 64 * 80 * 4)); CK(hipMemset(gring, 0x5a, 64 * 80 * 4));
  auto runs = [&](const char* name, auto kern, int grid) {
    hipLaunchKernelGGL(kern, grid, 64, 0, 0, gring, out, cyc, 16); CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0)); hipLaunchKernelGGL(kern, grid, 64, 0, 0, gring, out, cyc, nb); CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(hc.data(), cyc, 8 * grid, hipMemcpyDeviceToHost));
    double mx = 0; for (int i = 0; i < grid; ++i) mx = hc[i] > mx ? hc[i] : mx;
    printf("%-10s grid=%5d cyc/block=%7.1f  wall/block=%6.1f ns  per-msg %.1f MB/s  aggregate %.1f GB/s\n", name, grid,
           mx / nb, ms * 1e6 / nb, nb * 64.0 / (ms * 1e3), grid * nb * 64.0 / (ms * 1e6));
    return 0;
  };
  for (int g : {1, 1024}) { run("regs", k<0>, g); run("lds", k<1>, g); run("pipe", k<2>, g); run("lds16", k<3>, g); run("lds1", k<4>, g); run("pipe1", k<5>, g);
                            runs("smem4", ks<4>, g); runs("smem64", ks<64>, g); runs("squarter", kq, g); runs("gpipe", kg<1>, g); runs("gpipe1", kg<0>, g); }
  return 0;
}
