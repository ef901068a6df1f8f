// Microbenchmark: can a lone wave run the SHA-1 chain on the SCALAR unit faster than on the VALU,
// and does SALU work co-issue with the same wave's VALU work?  Not part of the product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1;}}while(0)

__device__ __forceinline__ uint32_t U(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
// Scalar rotate (SALU has none): lshl + lshr + or, pinned so the compiler cannot move it to v_alignbit.
template <int N> __device__ __forceinline__ uint32_t srotl(uint32_t x) {
  uint32_t r, t;
  asm("s_lshl_b32 %0, %2, %3\n\ts_lshr_b32 %1, %2, %4\n\ts_or_b32 %0, %0, %1"
      : "=&s"(r), "=&s"(t) : "s"(x), "i"(N), "i"(32 - N) : "scc");
  return r;
}

template <int R> __device__ __forceinline__ uint32_t sF(uint32_t b, uint32_t c, uint32_t d) {
  if constexpr (R < 20) return d ^ (b & (c ^ d));
  else if constexpr (R < 40 || R >= 60) return b ^ c ^ d;
  else return (b & c) | (d & (b | c));
}
template <int R> struct SR {
  __device__ __forceinline__ static void run(uint32_t (&s)[5], const uint32_t* __restrict__ wk) {
    constexpr int r = R % 5;
    constexpr int A = (5 - r) % 5, B = (6 - r) % 5, C = (7 - r) % 5, D = (8 - r) % 5, E = (9 - r) % 5;
    s[E] = srotl<5>(s[A]) + sF<R>(s[B], s[C], s[D]) + s[E] + wk[R];
    s[B] = srotl<30>(s[B]);
    SR<R + 1>::run(s, wk);
  }
};
template <> struct SR<80> { __device__ __forceinline__ static void run(uint32_t (&)[5], const uint32_t* __restrict__) {} };

// Scalar chain: state in SGPRs, WK from a read-only global ring via s_load.  Optionally the
// lanes run an independent VALU stream (nv VALU ops per round) to test co-issue.
template <int NV>
__global__ void k_schain(const uint32_t* __restrict__ ring, uint32_t* out, uint64_t* cyc, int nblocks) {
  uint32_t h[5] = {U(0x67452301u + blockIdx.x), U(0xEFCDAB89u), U(0x98BADCFEu), U(0x10325476u), U(0xC3D2E1F0u)};
  uint32_t v0 = threadIdx.x, v1 = v0 ^ 0x55, v2 = v0 ^ 0x99, v3 = v0 * 7;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int blk = 0; blk < nblocks; ++blk) {
    const uint32_t* wk = ring + (blk & 63) * 80;
    uint32_t s[5] = {h[0], h[1], h[2], h[3], h[4]};
    SR<0>::run(s, wk);
    for (int k = 0; k < 5; ++k) h[k] += s[k];
#pragma unroll
    for (int j = 0; j < NV * 20; ++j) {  // NV*80 VALU ops per block = NV per round
      asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v0) : "v"(v1), "v"(v2));
      asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(v1));
      asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(v2) : "v"(v3), "v"(v0));
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(v3) : "v"(v1));
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4] ^ v0 ^ v1 ^ v2 ^ v3;
  if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

// VALU-only stream of NV*80 ops per block (reference for the co-issue test).
template <int NV>
__global__ void k_vonly(const uint32_t* __restrict__ ring, uint32_t* out, uint64_t* cyc, int nblocks) {
  uint32_t v0 = threadIdx.x, v1 = v0 ^ 0x55, v2 = v0 ^ 0x99, v3 = v0 * 7;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int blk = 0; blk < nblocks; ++blk) {
#pragma unroll
    for (int j = 0; j < NV * 20; ++j) {
      asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v0) : "v"(v1), "v"(v2));
      asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(v1));
      asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(v2) : "v"(v3), "v"(v0));
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(v3) : "v"(v1));
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ ring[0];
  if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

int main() {
  uint32_t *ring, *out; uint64_t* cyc;
  CK(hipMalloc(&ring, 64 * 80 * 4)); CK(hipMalloc(&out, 1 << 24)); CK(hipMalloc(&cyc, 1 << 20));
  std::vector<uint32_t> hr(64 * 80); for (size_t i = 0; i < hr.size(); ++i) hr[i] = (uint32_t)(i * 0x9E3779B9u);
  CK(hipMemcpy(ring, hr.data(), hr.size() * 4, hipMemcpyHostToDevice));
  std::vector<uint64_t> hc(4096);
  const int nb = 4000;
  auto run = [&](const char* name, auto k, int grid) {
    hipLaunchKernelGGL(k, grid, 64, 0, 0, ring, out, cyc, 4); CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0); hipLaunchKernelGGL(k, grid, 64, 0, 0, ring, out, cyc, nb); hipEventRecord(e1);
    CK(hipEventSynchronize(e1)); float ms; hipEventElapsedTime(&ms, e0, e1);
    CK(hipMemcpy(hc.data(), cyc, 8 * grid, hipMemcpyDeviceToHost));
    double mx = 0; for (int i = 0; i < grid; ++i) mx = hc[i] > mx ? hc[i] : mx;
    printf("%-34s grid=%4d cyc/block=%8.1f  cyc/round=%6.2f  wall %.3f ms -> %.1f MB/s per wave\n", name, grid, mx / nb,
           mx / nb / 80, ms, nb * 64.0 / (ms * 1e3));
    return 0;
  };
  run("SALU chain only", k_schain<0>, 1);
  run("SALU chain + 1 VALU/round", k_schain<1>, 1);
  run("SALU chain + 2 VALU/round", k_schain<2>, 1);
  run("SALU chain + 4 VALU/round", k_schain<4>, 1);
  run("VALU only 1/round", k_vonly<1>, 1);
  run("VALU only 2/round", k_vonly<2>, 1);
  run("VALU only 4/round", k_vonly<4>, 1);
  run("SALU chain only x1024 waves", k_schain<0>, 1024);
  run("SALU chain + 4 VALU x1024", k_schain<4>, 1024);
  return 0;
}
