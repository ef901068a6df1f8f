// Microbenchmark: SIMD-level VALU throughput by instruction class with W waves per SIMD.
// Settles whether the integer ops of the SHA-1/CRC kernels (VOP2 v_add/v_xor, VOP3 v_add3/
// v_bitop3/v_alignbit, SDWA v_lshlrev) get the 2-cycle SIMD-32 rate the MI355X guide quotes
// for v_fma_f32 once two or more waves share a SIMD. Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -o mb_rate mb_rate.hip && ./mb_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1;}}while(0)

#define KHEAD(name) __global__ void name(uint32_t* out, uint64_t* cyc, int iters, uint32_t seed) { \
  uint32_t x0 = seed + threadIdx.x, x1 = x0^1, x2 = x0^2, x3 = x0^3, x4=x0^4, x5=x0^5, x6=x0^6, x7=x0^7; \
  const uint32_t k = seed | 1u; \
  uint64_t t0 = __builtin_amdgcn_s_memtime(); \
  for (int i = 0; i < iters; ++i) { for (int j = 0; j < 4; ++j) {
#define KTAIL }} uint64_t t1 = __builtin_amdgcn_s_memtime(); \
  out[blockIdx.x*blockDim.x+threadIdx.x] = x0^x1^x2^x3^x4^x5^x6^x7; \
  if (threadIdx.x % 64 == 0) cyc[(blockIdx.x*blockDim.x+threadIdx.x)/64] = t1 - t0; }

#define OP8(M) M(x0) M(x1) M(x2) M(x3) M(x4) M(x5) M(x6) M(x7)
#define ADD2(x) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(x) : "v"(k));
#define XOR2(x) asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(x) : "v"(k));
#define ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
#define BOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(x) : "v"(k));
#define ALGN(x) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x));
#define SDWA(x) asm volatile("v_lshlrev_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(x) : "v"(k));
#define FMA(x)  asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
#define ADD64(x) asm volatile("v_add_co_u32_e32 %0, vcc, %1, %0" : "+v"(x) : "v"(k) : "vcc");
// 32 instructions per inner j-loop pass x 4 passes = 32 per (i) iteration... (8 per OP8, 4 j passes)
KHEAD(k_add2) OP8(ADD2) KTAIL
KHEAD(k_xor2) OP8(XOR2) KTAIL
KHEAD(k_add3) OP8(ADD3) KTAIL
KHEAD(k_bop3) OP8(BOP3) KTAIL
KHEAD(k_algn) OP8(ALGN) KTAIL
KHEAD(k_sdwa) OP8(SDWA) KTAIL
KHEAD(k_fma)  OP8(FMA)  KTAIL
KHEAD(k_mix)  ADD2(x0) BOP3(x1) ADD3(x2) ALGN(x3) XOR2(x4) BOP3(x5) ADD3(x6) ALGN(x7) KTAIL

typedef void (*kfn)(uint32_t*, uint64_t*, int, uint32_t);

int main() {
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  struct K { const char* name; kfn f; } ks[] = {
    {"v_add_u32_e32 (VOP2)", k_add2}, {"v_xor_b32_e32 (VOP2)", k_xor2}, {"v_add3_u32 (VOP3)", k_add3},
    {"v_bitop3_b32 (VOP3)", k_bop3}, {"v_alignbit_b32 (VOP3)", k_algn}, {"v_lshlrev_b32_sdwa", k_sdwa},
    {"v_fma_f32 (control)", k_fma}, {"SHA-1 round mix", k_mix}};
  const int iters = 20000;
  uint32_t* out; uint64_t* cyc;
  CK(hipMalloc(&out, sizeof(uint32_t) * cus * 64 * 4 * 8));
  CK(hipMalloc(&cyc, sizeof(uint64_t) * cus * 4 * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  printf("%d CUs; instructions per wave = %d; SIMD-level cycles per wave64 instruction at the measured clock\n", cus, iters * 32);
  for (const K& k : ks) {
    for (int w : {1, 2, 4}) {
      const int threads = 64 * 4 * w;  // w waves on each of the 4 SIMDs of one CU
      hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), 0, 0, out, cyc, 10, 1u);  // warm
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), 0, 0, out, cyc, iters, 1u);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<uint64_t> c(cus * 4 * w);
      CK(hipMemcpy(c.data(), cyc, c.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
      uint64_t mx = 0; for (auto v : c) mx = v > mx ? v : mx;
      const double instr_per_simd = double(w) * iters * 32;
      // wall-clock cycles at 2.4 GHz and at the s_memtime count (shader clock) of the slowest wave
      printf("%-24s waves/SIMD=%d  %.3f ms  cyc/instr/SIMD: %.2f @2.4GHz  %.2f @memtime  (lone-wave view: %.2f)\n",
             k.name, w, ms, ms * 1e-3 * 2.4e9 / instr_per_simd, double(mx) / instr_per_simd,
             double(mx) / (iters * 32.0));
    }
  }
  return 0;
}
