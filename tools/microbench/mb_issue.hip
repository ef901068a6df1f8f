// Microbenchmark 2: lone-wave issue rates by instruction class, SALU/VALU co-issue,
// and SHA-1 chain with 2 interleaved messages per wave. Not part of the product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1;}}while(0)

#define KHEAD(name) __global__ void name(uint32_t* out, uint64_t* cyc, int iters, uint32_t seed) { \
  uint32_t x0 = seed + threadIdx.x, x1 = x0^1, x2 = x0^2, x3 = x0^3, x4=x0^4, x5=x0^5, x6=x0^6, x7=x0^7; \
  uint32_t s0 = seed, s1 = seed^1, s2 = seed^2, s3 = seed^3, s4 = seed^4, s5=seed^5, s6=seed^6, s7=seed^7; \
  uint64_t t0 = __builtin_amdgcn_s_memtime(); \
  for (int i = 0; i < iters; ++i) {
#define KTAIL } uint64_t t1 = __builtin_amdgcn_s_memtime(); \
  out[blockIdx.x*blockDim.x+threadIdx.x] = x0^x1^x2^x3^x4^x5^x6^x7^s0^s1^s2^s3^s4^s5^s6^s7; \
  if (threadIdx.x % 64 == 0) cyc[(blockIdx.x*blockDim.x+threadIdx.x)/64] = t1 - t0; }

#define V3(x) asm volatile("v_add3_u32 %0, %0, %0, %0" : "+v"(x));
#define V2(x) asm volatile("v_add_u32_e32 %0, %0, %0" : "+v"(x));
#define VA(x) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x));
#define SA(x) asm volatile("s_add_u32 %0, %0, %0" : "+s"(x) :: "scc");
// 32 instructions per iteration in every kernel
KHEAD(k_v3_dep)   for(int j=0;j<32;++j){ V3(x0) } KTAIL
KHEAD(k_v2_dep)   for(int j=0;j<32;++j){ V2(x0) } KTAIL
KHEAD(k_va_dep)   for(int j=0;j<32;++j){ VA(x0) } KTAIL
KHEAD(k_s_dep)    for(int j=0;j<32;++j){ SA(s0) } KTAIL
KHEAD(k_v3_ind8)  for(int j=0;j<4;++j){ V3(x0) V3(x1) V3(x2) V3(x3) V3(x4) V3(x5) V3(x6) V3(x7) } KTAIL
KHEAD(k_v2_ind8)  for(int j=0;j<4;++j){ V2(x0) V2(x1) V2(x2) V2(x3) V2(x4) V2(x5) V2(x6) V2(x7) } KTAIL
KHEAD(k_s_ind8)   for(int j=0;j<4;++j){ SA(s0) SA(s1) SA(s2) SA(s3) SA(s4) SA(s5) SA(s6) SA(s7) } KTAIL
KHEAD(k_mix_v3s)  for(int j=0;j<4;++j){ V3(x0) SA(s0) V3(x1) SA(s1) V3(x2) SA(s2) V3(x3) SA(s3) } KTAIL
KHEAD(k_mix_v3s2) for(int j=0;j<4;++j){ V3(x0) SA(s0) SA(s4) V3(x1) SA(s1) SA(s5) V3(x2) SA(s2) SA(s6) V3(x3) SA(s3) SA(s7) } KTAIL  // 48/iter
KHEAD(k_v3_dep_h) if ((threadIdx.x & 63) < 32) { for(int j=0;j<32;++j){ V3(x0) } } KTAIL
KHEAD(k_v3_ind_h) if ((threadIdx.x & 63) < 32) { for(int j=0;j<4;++j){ V3(x0) V3(x1) V3(x2) V3(x3) V3(x4) V3(x5) V3(x6) V3(x7) } } KTAIL

// SHA-1 chain with WK from LDS, M independent messages interleaved per lane
__device__ __forceinline__ uint32_t rotl(uint32_t x, int n){ return __builtin_rotateleft32(x, n); }
template <int R, int M>
__device__ __forceinline__ void rnd(uint32_t (&s)[5][M], const uint32_t (&W)[M]) {
  constexpr int LUT = R < 20 ? 0xCA : (R < 40 ? 0x96 : (R < 60 ? 0xE8 : 0x96));
  constexpr int r = R % 5;
  constexpr int A = (5 - r) % 5, B = (6 - r) % 5, C = (7 - r) % 5, D = (8 - r) % 5, E = (9 - r) % 5;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    uint32_t z = s[E][m] + W[m];
    s[E][m] = (rotl(s[A][m], 5) + __builtin_amdgcn_bitop3_b32(s[B][m], s[C][m], s[D][m], LUT)) + z;
    s[B][m] = rotl(s[B][m], 30);
  }
}
template <int Q, int M> struct Quad {
  __device__ __forceinline__ static void run(uint32_t (&s)[5][M], const uint4* const (&wk4)[M]) {
    uint32_t W0[M], W1[M], W2[M], W3[M];
#pragma unroll
    for (int m = 0; m < M; ++m) { uint4 v = wk4[m][Q]; W0[m]=v.x; W1[m]=v.y; W2[m]=v.z; W3[m]=v.w; }
    rnd<4*Q, M>(s, W0); rnd<4*Q+1, M>(s, W1); rnd<4*Q+2, M>(s, W2); rnd<4*Q+3, M>(s, W3);
    Quad<Q + 1, M>::run(s, wk4);
  }
};
template <int M> struct Quad<20, M> { __device__ __forceinline__ static void run(uint32_t (&)[5][M], const uint4* const (&)[M]) {} };

template <int M>
__global__ void k_chain(uint32_t* out, uint64_t* cyc, int nblocks) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  int wv = threadIdx.x / 64, ln = threadIdx.x % 64;
  uint32_t* ring = lds + wv * 64 * 80;
  for (int i = ln; i < 64*80; i += 64) ring[i] = i * 0x9E3779B9u + wv;
  __syncthreads();
  uint32_t h[5][M];
#pragma unroll
  for (int m = 0; m < M; ++m) { h[0][m]=0x67452301u+m; h[1][m]=0xEFCDAB89u; h[2][m]=0x98BADCFEu; h[3][m]=0x10325476u; h[4][m]=0xC3D2E1F0u; }
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int blk = 0; blk < nblocks; ++blk) {
    uint32_t s[5][M];
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int m = 0; m < M; ++m) s[k][m] = h[k][m];
    const uint4* wk4[M];
#pragma unroll
    for (int m = 0; m < M; ++m) wk4[m] = (const uint4*)(ring + ((blk + 17*m) & 63) * 80);
    Quad<0, M>::run(s, wk4);
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int m = 0; m < M; ++m) h[k][m] += s[k][m];
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t r = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) r ^= h[0][m]^h[1][m]^h[2][m]^h[3][m]^h[4][m];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (ln == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

int main() {
  uint32_t* out; uint64_t* cyc; CK(hipMalloc(&out, 1<<24)); CK(hipMalloc(&cyc, 1<<20));
  std::vector<uint64_t> hc(4096);
  auto run = [&](const char* name, void (*k)(uint32_t*, uint64_t*, int, uint32_t), double per_iter) {
    hipLaunchKernelGGL(k, 1, 64, 0, 0, out, cyc, 10, 1u); hipDeviceSynchronize();
    hipLaunchKernelGGL(k, 1, 64, 0, 0, out, cyc, 20000, 1u); hipDeviceSynchronize();
    hipMemcpy(hc.data(), cyc, 8, hipMemcpyDeviceToHost);
    printf("%-28s cyc/instr = %6.2f\n", name, hc[0] / (20000.0 * per_iter));
  };
  run("v_add3 dep", k_v3_dep, 32); run("v_add_e32 dep", k_v2_dep, 32); run("v_alignbit dep", k_va_dep, 32);
  run("s_add dep", k_s_dep, 32); run("v_add3 8-indep", k_v3_ind8, 32); run("v_add_e32 8-indep", k_v2_ind8, 32);
  run("s_add 8-indep", k_s_ind8, 32); run("mix v3+s 1:1 (per instr)", k_mix_v3s, 32); run("mix v3+s 1:2 (per instr)", k_mix_v3s2, 48);
  run("v_add3 dep, 32 lanes", k_v3_dep_h, 32); run("v_add3 8-ind, 32 lanes", k_v3_ind_h, 32);
  int nb = 20000;
  auto chain = [&](const char* name, auto kern, int M, int blocks, int threads) {
    size_t lds = (threads/64) * 64 * 80 * 4;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0); hipLaunchKernelGGL(kern, blocks, threads, lds, 0, out, cyc, nb); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    int nw = blocks*threads/64; hipMemcpy(hc.data(), cyc, nw*8, hipMemcpyDeviceToHost);
    double mx=0; for(int i=0;i<nw;++i) mx = hc[i]>mx?hc[i]:mx;
    printf("%-28s waves=%4d cyc/block/msg=%7.1f  per-msg %.1f MB/s  aggregate %.1f GB/s (msgs=%d)\n", name, nw, mx/nb/M, nb*64.0/(ms*1e3), (double)nw*M*nb*64/(ms*1e6), nw*M);
  };
  chain("chain M=1", k_chain<1>, 1, 1, 64); chain("chain M=2", k_chain<2>, 2, 1, 64); chain("chain M=3", k_chain<3>, 3, 1, 64);
  chain("chain M=1 x1024 waves", k_chain<1>, 1, 256, 256); chain("chain M=2 x512 waves", k_chain<2>, 2, 128, 256);
  chain("chain M=2 x1024 waves", k_chain<2>, 2, 256, 256);
  return 0;
}
