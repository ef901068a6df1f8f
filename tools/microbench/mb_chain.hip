// Microbenchmark: per-wave issue rate and SHA-1 chain cost on gfx950.
// Used once to pick the kernel shape (DESIGN_NOTES.md "Measured constants"). Not part of the product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <string.h>

#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1;}}while(0)

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n){ return __builtin_rotateleft32(x, n); }
__device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t c){ return a + b + c; }

// ---- 1. raw VALU issue: dependent chain and 4 independent chains
__global__ void mb_dep(uint32_t* out, uint64_t* cyc, int iters, uint32_t seed){
  uint32_t x = seed + threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 32; ++j) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x) : "v"(x));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}
__global__ void mb_indep(uint32_t* out, uint64_t* cyc, int iters, uint32_t seed){
  uint32_t x = seed + threadIdx.x, y = x ^ 1, z = x ^ 2, w = x ^ 3;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x) : "v"(x));
      asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(y) : "v"(y));
      asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(z) : "v"(z));
      asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(w) : "v"(w));
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x ^ y ^ z ^ w;
  if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

// ---- 2. SHA-1 compression, schedule inline, lane = message
#define F_CH 0xCA
#define F_PAR 0x96
#define F_MAJ 0xE8
#define RND(a,b,c,d,e,LUT,K,W) { uint32_t z_ = add3(e, (W), (K)); e = add3(rotl(a,5), __builtin_amdgcn_bitop3_b32(b,c,d,LUT), z_); b = rotl(b,30); }
#define SCHED(i) (w[(i)&15] = rotl(__builtin_amdgcn_bitop3_b32(w[((i)-3)&15], w[((i)-8)&15], w[((i)-14)&15], F_PAR) ^ w[(i)&15], 1))

__device__ __forceinline__ void compress_inline(uint32_t h[5], uint32_t w[16]) {
  uint32_t a=h[0],b=h[1],c=h[2],d=h[3],e=h[4];
#define R5(i,LUT,K,WX) RND(a,b,c,d,e,LUT,K,WX(i)) RND(e,a,b,c,d,LUT,K,WX(i+1)) RND(d,e,a,b,c,LUT,K,WX(i+2)) RND(c,d,e,a,b,LUT,K,WX(i+3)) RND(b,c,d,e,a,LUT,K,WX(i+4))
#define WD(i) w[i]
  R5(0,F_CH,0x5A827999u,WD) R5(5,F_CH,0x5A827999u,WD) R5(10,F_CH,0x5A827999u,WD)
  RND(a,b,c,d,e,F_CH,0x5A827999u,w[15]) RND(e,a,b,c,d,F_CH,0x5A827999u,SCHED(16)) RND(d,e,a,b,c,F_CH,0x5A827999u,SCHED(17)) RND(c,d,e,a,b,F_CH,0x5A827999u,SCHED(18)) RND(b,c,d,e,a,F_CH,0x5A827999u,SCHED(19))
  R5(20,F_PAR,0x6ED9EBA1u,SCHED) R5(25,F_PAR,0x6ED9EBA1u,SCHED) R5(30,F_PAR,0x6ED9EBA1u,SCHED) R5(35,F_PAR,0x6ED9EBA1u,SCHED)
  R5(40,F_MAJ,0x8F1BBCDCu,SCHED) R5(45,F_MAJ,0x8F1BBCDCu,SCHED) R5(50,F_MAJ,0x8F1BBCDCu,SCHED) R5(55,F_MAJ,0x8F1BBCDCu,SCHED)
  R5(60,F_PAR,0xCA62C1D6u,SCHED) R5(65,F_PAR,0xCA62C1D6u,SCHED) R5(70,F_PAR,0xCA62C1D6u,SCHED) R5(75,F_PAR,0xCA62C1D6u,SCHED)
  h[0]+=a; h[1]+=b; h[2]+=c; h[3]+=d; h[4]+=e;
}

__global__ void mb_sha_inline(const uint4* __restrict__ data, uint32_t* out, uint64_t* cyc, int nblocks, size_t lane_stride16) {
  int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const uint4* p = data + (size_t)gl * lane_stride16;
  uint32_t h[5] = {0x67452301u,0xEFCDAB89u,0x98BADCFEu,0x10325476u,0xC3D2E1F0u};
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int blk = 0; blk < nblocks; ++blk) {
    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) { uint4 v = p[blk*4+q]; w[4*q]=__builtin_bswap32(v.x); w[4*q+1]=__builtin_bswap32(v.y); w[4*q+2]=__builtin_bswap32(v.z); w[4*q+3]=__builtin_bswap32(v.w); }
    compress_inline(h, w);
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[gl] = h[0]^h[1]^h[2]^h[3]^h[4];
  if (threadIdx.x % 64 == 0) cyc[gl / 64] = t1 - t0;
}

// ---- 3. chain only: WK from LDS (wave-uniform address), 64-block ring per wave
__global__ void mb_chain_lds(uint32_t* out, uint64_t* cyc, int nblocks) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  int wv = threadIdx.x / 64, ln = threadIdx.x % 64;
  uint32_t* ring = lds + wv * 64 * 80;
  for (int i = ln; i < 64*80; i += 64) ring[i] = i * 0x9E3779B9u + wv;
  __syncthreads();
  uint32_t h[5] = {0x67452301u,0xEFCDAB89u,0x98BADCFEu,0x10325476u,0xC3D2E1F0u};
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int blk = 0; blk < nblocks; ++blk) {
    const uint4* wk4 = (const uint4*)(ring + (blk & 63) * 80);
    uint32_t wk[80];
#pragma unroll
    for (int q = 0; q < 20; ++q) { uint4 v = wk4[q]; wk[4*q]=v.x; wk[4*q+1]=v.y; wk[4*q+2]=v.z; wk[4*q+3]=v.w; }
    uint32_t a=h[0],b=h[1],c=h[2],d=h[3],e=h[4];
#define RL(a,b,c,d,e,LUT,K,WK) { uint32_t z_ = e + (WK); e = add3(rotl(a,5), __builtin_amdgcn_bitop3_b32(b,c,d,LUT), z_); b = rotl(b,30); }
#define RL5(i,LUT) RL(a,b,c,d,e,LUT,0,wk[i]) RL(e,a,b,c,d,LUT,0,wk[i+1]) RL(d,e,a,b,c,LUT,0,wk[i+2]) RL(c,d,e,a,b,LUT,0,wk[i+3]) RL(b,c,d,e,a,LUT,0,wk[i+4])
    RL5(0,F_CH) RL5(5,F_CH) RL5(10,F_CH) RL5(15,F_CH)
    RL5(20,F_PAR) RL5(25,F_PAR) RL5(30,F_PAR) RL5(35,F_PAR)
    RL5(40,F_MAJ) RL5(45,F_MAJ) RL5(50,F_MAJ) RL5(55,F_MAJ)
    RL5(60,F_PAR) RL5(65,F_PAR) RL5(70,F_PAR) RL5(75,F_PAR)
    h[0]+=a; h[1]+=b; h[2]+=c; h[3]+=d; h[4]+=e;
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = h[0]^h[1]^h[2]^h[3]^h[4];
  if (ln == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

static double now_ms(hipEvent_t a, hipEvent_t b){ float ms; hipEventElapsedTime(&ms, a, b); return ms; }

int main() {
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs %d clock %d kHz\n", prop.name, prop.multiProcessorCount, prop.clockRate);
  uint32_t* out; uint64_t* cyc; CK(hipMalloc(&out, 1<<24)); CK(hipMalloc(&cyc, 1<<20));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  std::vector<uint64_t> hc(16384);
  auto report = [&](const char* name, int nwaves, double ms, double work_per_wave, const char* unit) {
    CK(hipMemcpy(hc.data(), cyc, nwaves * 8, hipMemcpyDeviceToHost));
    double mx = 0, sum = 0; for (int i = 0; i < nwaves; ++i) { mx = hc[i] > mx ? hc[i] : mx; sum += hc[i]; }
    printf("%-34s waves=%5d wall=%8.3f ms  cyc/%s(mean)=%8.2f  cyc/%s(max)=%8.2f  eff_clk=%.2f GHz\n", name, nwaves, ms,
           unit, sum / nwaves / work_per_wave, unit, mx / work_per_wave, mx / (ms * 1e6));
    return 0;
  };
  int iters = 20000;
  struct G { int blocks, threads; } cfgs[] = {{1,64},{256,256},{256,512},{256,1024}};
  for (auto g : cfgs) {
    int nw = g.blocks * g.threads / 64;
    hipLaunchKernelGGL(mb_dep, g.blocks, g.threads, 0, 0, out, cyc, 100, 1u); CK(hipDeviceSynchronize());
    hipEventRecord(e0); hipLaunchKernelGGL(mb_dep, g.blocks, g.threads, 0, 0, out, cyc, iters, 1u); hipEventRecord(e1); CK(hipEventSynchronize(e1));
    report("valu dep add3", nw, now_ms(e0,e1), iters*32.0, "instr");
    hipEventRecord(e0); hipLaunchKernelGGL(mb_indep, g.blocks, g.threads, 0, 0, out, cyc, iters, 1u); hipEventRecord(e1); CK(hipEventSynchronize(e1));
    report("valu 4-indep add3", nw, now_ms(e0,e1), iters*32.0, "instr");
  }
  // SHA inline, lane = message; each lane owns 256 KiB (4096 blocks)
  int nblk = 4096; size_t lane_bytes = (size_t)nblk * 64;
  struct G2 { int blocks, threads; } scfg[] = {{1,64},{16,64},{256,256},{256,512},{512,512}};
  size_t maxlanes = 512*512; uint4* data; CK(hipMalloc(&data, maxlanes * lane_bytes / 16 * 16 / 16 > 0 ? (size_t)1 << 34 : 0));
  CK(hipMemset(data, 0x5a, (size_t)1 << 34));
  for (auto g : scfg) {
    int lanes = g.blocks * g.threads; int nw = lanes / 64;
    size_t stride16 = lane_bytes / 16;
    int nb = nblk;
    if ((size_t)lanes * lane_bytes > ((size_t)1 << 34)) { stride16 = ((size_t)1<<34) / lanes / 16 / 4 * 4; nb = (int)(stride16 / 4); }
    hipEventRecord(e0); hipLaunchKernelGGL(mb_sha_inline, g.blocks, g.threads, 0, 0, data, out, cyc, nb, stride16); hipEventRecord(e1); CK(hipEventSynchronize(e1));
    double ms = now_ms(e0,e1);
    report("sha inline (lane=msg)", nw, ms, nb, "block");
    printf("    -> per-message %.1f MB/s, aggregate %.1f GB/s\n", nb*64.0/(ms*1e3), (double)lanes*nb*64.0/(ms*1e6));
  }
  // chain with WK in LDS
  struct G3 { int blocks, threads; } ccfg[] = {{1,64},{256,256},{256,512}};
  for (auto g : ccfg) {
    int nw = g.blocks * g.threads / 64; int nb = 20000;
    size_t lds = (g.threads/64) * 64 * 80 * 4;
    hipEventRecord(e0); hipLaunchKernelGGL(mb_chain_lds, g.blocks, g.threads, lds, 0, out, cyc, nb); hipEventRecord(e1); CK(hipEventSynchronize(e1));
    double ms = now_ms(e0,e1);
    report("chain WK-from-LDS (wave=msg)", nw, ms, nb, "block");
    printf("    -> per-message %.1f MB/s, aggregate(1 msg/wave) %.1f GB/s\n", nb*64.0/(ms*1e3), (double)nw*nb*64.0/(ms*1e6));
  }
  return 0;
}
