// Which SIMD does each wave of a workgroup land on?  (s_getreg HW_ID: SIMD_ID = bits [5:4])
// Prints, per workgroup shape, the SIMD of waves 0..n-1 for the first few workgroups.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void where(uint32_t* out) {
  uint32_t hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = hw;
  // keep the waves resident for a while so later workgroups see occupied SIMDs
  uint64_t t0 = __builtin_readcyclecounter();
  while (__builtin_readcyclecounter() - t0 < 200000) {}
}

int main() {
  for (int waves : {4, 8}) {
    const int blocks = 512;
    uint32_t* d;
    hipMalloc(&d, blocks * waves * 4);
    hipLaunchKernelGGL(where, dim3(blocks), dim3(64 * waves), 120 * 1024, 0, d);  // 120 KiB LDS: one WG per CU
    hipDeviceSynchronize();
    uint32_t h[512 * 8];
    hipMemcpy(h, d, blocks * waves * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int b = 0; b < blocks; ++b) {
      int cnt[4] = {0, 0, 0, 0};
      for (int w = 0; w < waves; ++w) cnt[(h[b * waves + w] >> 4) & 3]++;
      for (int s = 0; s < 4; ++s) bad += cnt[s] != waves / 4;
      if (b < 6) {
        printf("waves=%d wg=%d simd:", waves, b);
        for (int w = 0; w < waves; ++w) printf(" %u", (h[b * waves + w] >> 4) & 3);
        printf("  (cu %u se %u)\n", (h[b * waves] >> 8) & 15, (h[b * waves] >> 13) & 7);
      }
    }
    int same = 0;  // waves w and w+4 on the same SIMD
    if (waves == 8)
      for (int b = 0; b < blocks; ++b)
        for (int w = 0; w < 4; ++w) same += ((h[b * 8 + w] >> 4) & 3) == ((h[b * 8 + w + 4] >> 4) & 3);
    printf("waves=%d: %d workgroups with an uneven SIMD split; pairs (w, w+4) on one SIMD: %d of %d\n", waves, bad,
           same, waves == 8 ? blocks * 4 : 0);
    hipFree(d);
  }
  return 0;
}
