// Microbenchmark / probe: what ds_read_b32 returns for an address that is NOT a multiple of 4
// (is the address aligned down, or is it an unaligned 4-byte read?).  Decides whether a CRC
// table index can be formed by one shift/bit-field op (low two address bits left as garbage).
// Not part of the product.   hipcc --offload-arch=gfx950 -O3 -o mb_lds_align mb_lds_align.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__global__ void probe(uint32_t* out) {
  __shared__ uint32_t t[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) t[i] = 0x01010101u * (uint32_t)i;
  __syncthreads();
  const uint32_t addr = (uint32_t)(uintptr_t)t + 4u * (threadIdx.x / 4) + (threadIdx.x & 3);
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr));
  out[threadIdx.x] = v;
}
int main() {
  uint32_t* d; hipMalloc(&d, 64 * 4);
  hipLaunchKernelGGL(probe, 1, 64, 0, 0, d);
  uint32_t h[64]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  int aligned_down = 1, unaligned = 1;
  for (int i = 0; i < 64; ++i) {
    const uint32_t e = 0x01010101u * (uint32_t)(i / 4);
    const uint32_t lo = 0x01010101u * (uint32_t)(i / 4), hi = 0x01010101u * (uint32_t)(i / 4 + 1);
    const int r = i & 3;
    const uint32_t u = r ? (lo >> (8 * r)) | (hi << (32 - 8 * r)) : lo;
    if (h[i] != e) aligned_down = 0;
    if (h[i] != u) unaligned = 0;
    if (i < 8) printf("lane %2d addr +%d: 0x%08x\n", i, r, h[i]);
  }
  printf("ds_read_b32 misaligned: %s\n", aligned_down ? "ALIGNED DOWN (low bits ignored)" : unaligned ? "UNALIGNED READ" : "OTHER");
  return 0;
}
