// Microbenchmark: issue cost of the cross-lane moves the DEEP chain could hand its chaining value
// on with (one wave per SIMD, 8 independent moves per step).  The chain uses 5 DPP wave_shr:1
// moves per 64-B block; DESIGN_NOTES.md's accounting puts them at ~7.6 cycles each.  Not part of the
// product.
//   hipcc --offload-arch=gfx950 -O3 -o mb_dpp mb_dpp.hip && ./mb_dpp
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1;}}while(0)

#define KHEAD(name) __global__ void name(uint32_t* out, uint64_t* cyc, int iters, uint32_t seed) { \
  uint32_t x0 = seed + threadIdx.x, x1 = x0^1, x2 = x0^2, x3 = x0^3, x4=x0^4, x5=x0^5, x6=x0^6, x7=x0^7; \
  uint64_t t0 = __builtin_amdgcn_s_memtime(); \
  for (int i = 0; i < iters; ++i) { for (int j = 0; j < 4; ++j) {
#define KTAIL }} uint64_t t1 = __builtin_amdgcn_s_memtime(); \
  out[blockIdx.x*blockDim.x+threadIdx.x] = x0^x1^x2^x3^x4^x5^x6^x7; \
  if (threadIdx.x % 64 == 0) cyc[(blockIdx.x*blockDim.x+threadIdx.x)/64] = t1 - t0; }

#define OP8(M) M(x0) M(x1) M(x2) M(x3) M(x4) M(x5) M(x6) M(x7)
#define MOV(x)  asm volatile("v_mov_b32_e32 %0, %0" : "+v"(x));
#define WSHR(x) asm volatile("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0" : "+v"(x));
#define RSHR(x) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0" : "+v"(x));
#define QPRM(x) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf" : "+v"(x));
#define ADDD(x) asm volatile("v_add_u32_dpp %0, %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0" : "+v"(x));
#define RDLN(x) { uint32_t s_; asm volatile("v_readlane_b32 %0, %1, 7" : "=s"(s_) : "v"(x)); asm volatile("v_mov_b32_e32 %0, %1" : "=v"(x) : "s"(s_)); }
#define ALGN(x) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x));
KHEAD(k_mov)  OP8(MOV)  KTAIL
KHEAD(k_wshr) OP8(WSHR) KTAIL
KHEAD(k_rshr) OP8(RSHR) KTAIL
KHEAD(k_qprm) OP8(QPRM) KTAIL
KHEAD(k_addd) OP8(ADDD) KTAIL
KHEAD(k_rdln) OP8(RDLN) KTAIL
KHEAD(k_algn) OP8(ALGN) KTAIL
// the chain's pattern: four rotates, then one wave_shr move (1 DPP per 5 VALU)
KHEAD(k_mix) ALGN(x0) ALGN(x1) ALGN(x2) ALGN(x3) WSHR(x4) ALGN(x5) ALGN(x6) ALGN(x7) KTAIL

typedef void (*kfn)(uint32_t*, uint64_t*, int, uint32_t);

int main() {
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  struct K { const char* name; kfn f; int per; } ks[] = {
    {"v_mov_b32_e32", k_mov, 32}, {"v_mov_b32_dpp wave_shr:1", k_wshr, 32}, {"v_mov_b32_dpp row_shr:1", k_rshr, 32},
    {"v_mov_b32_dpp quad_perm", k_qprm, 32}, {"v_add_u32_dpp wave_shr:1", k_addd, 32},
    {"v_readlane + v_mov from SGPR", k_rdln, 64}, {"v_alignbit_b32", k_algn, 32}, {"7 alignbit + 1 wave_shr", k_mix, 32}};
  const int iters = 20000;
  uint32_t* out; uint64_t* cyc;
  CK(hipMalloc(&out, sizeof(uint32_t) * cus * 64 * 4 * 2));
  CK(hipMalloc(&cyc, sizeof(uint64_t) * cus * 4 * 2));
  printf("%d CUs; lone wave per SIMD; cycles per instruction (s_memtime, slowest wave)\n", cus);
  for (const K& k : ks) {
    for (int w : {1, 2}) {
      const int threads = 64 * 4 * w;
      hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), 0, 0, out, cyc, 10, 1u);
      CK(hipDeviceSynchronize());
      hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), 0, 0, out, cyc, iters, 1u);
      CK(hipDeviceSynchronize());
      std::vector<uint64_t> c(cus * 4 * w);
      CK(hipMemcpy(c.data(), cyc, c.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
      uint64_t mx = 0; for (auto v : c) mx = v > mx ? v : mx;
      printf("%-30s waves/SIMD=%d  per-wave cyc/instr %.2f  SIMD cyc/instr %.2f\n", k.name, w,
             double(mx) / (iters * (double)k.per), double(mx) / (w * iters * (double)k.per));
    }
  }
  return 0;
}
