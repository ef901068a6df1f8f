// mb_glds.hip -- is an LDS-DMA ring (global_load_lds_dwordx4, default or nontemporal policy) a
// faster way to stream a buffer once than plain global_load_dwordx4 into registers?  (Round 5: the
// headroom of the span CRC, DESIGN.md §4 / DESIGN_NOTES.md §4 "Span CRC".)  Every byte of a 16 GiB
// buffer is read once and XOR-folded.  Each wave streams its own 4 KiB chunks (one chunk = four
// coalesced 1-KiB wave-instructions) through a ring of R slots in LDS, R chunks in flight; lanes then
// read their 64-B line of the chunk back with four ds_read_b128 (as the span CRC's lanes would).
// Usage: mb_glds [gib]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int kWaves = 4;  // per workgroup

// s_waitcnt with vmcnt <= n (gfx9 encoding: vmcnt[3:0] + vmcnt[5:4] at [15:14], expcnt and lgkmcnt max)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int R, int AUX>
__global__ __launch_bounds__(64 * kWaves) void glds_kernel(const uint8_t* __restrict__ src, uint64_t chunks_total,
                                                           uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) v4u ring[kWaves][R][256];  // 4 KiB per slot
  const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t per_wg = chunks_total / gridDim.x;  // callers pass a multiple
  const uint64_t first = (uint64_t)blockIdx.x * per_wg;
  const uint64_t n = per_wg / kWaves;  // chunks of this wave: first + kWaves*i + wave
  auto issue = [&](uint64_t i, int slot) {
    const uint8_t* c = src + (first + (uint64_t)kWaves * i + wave) * 4096;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(c + 1024 * q + 16 * lane),
                                       (__attribute__((address_space(3))) void*)(&ring[wave][slot][64 * q]), 16, 0, AUX);
  };
  for (int s = 0; s < R; ++s)
    if ((uint64_t)s < n) issue(s, s);
  v4u acc = {0, 0, 0, 0};
  for (uint64_t i = 0; i < n; ++i) {
    const int slot = (int)(i % R);
    if (i + R <= n) wait_vm<4 * (R - 1)>();  // the oldest chunk has landed
    else wait_vm<0>();
    // the line's four 16-B pieces, read in inline asm: hipcc's waitcnt pass would otherwise put a
    // vmcnt(0) before any LDS read while an LDS-DMA is in flight (draining the ring)
    const uint32_t addr = (uint32_t)(uintptr_t)(&ring[wave][slot][4 * lane]);
    v4u r0, r1, r2, r3;
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\t"
                 "ds_read_b128 %3, %4 offset:48\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3) : "v"(addr) : "memory");
    acc ^= r0 ^ r1 ^ r2 ^ r3;
    if (i + R < n) issue(i + R, slot);
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// the plain register path in the same per-wave chunk order: lane j reads its 64-B line with four dwordx4
template <int B, bool NT = false>
__global__ __launch_bounds__(64 * kWaves) void reg_kernel(const uint8_t* __restrict__ src, uint64_t chunks_total,
                                                          uint32_t* __restrict__ out) {
  const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t per_wg = chunks_total / gridDim.x, first = (uint64_t)blockIdx.x * per_wg, n = per_wg / kWaves;
  v4u acc = {0, 0, 0, 0};
  for (uint64_t i = 0; i < n; i += B) {
    v4u v[B][4];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const v4u* c = reinterpret_cast<const v4u*>(src + (first + (uint64_t)kWaves * (i + b) + wave) * 4096 + 64 * lane);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[b][k] = NT ? __builtin_nontemporal_load(c + k) : c[k];
    }
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc ^= v[b][k];
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// 16 waves per workgroup (the span kernel's 1024 lanes per CU), each lane one 64-B line per row
template <int B, bool NT>
__global__ __launch_bounds__(1024) void reg_kernel16(const uint8_t* __restrict__ src, uint64_t chunks_total,
                                                     uint32_t* __restrict__ out) {
  const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t per_wg = chunks_total / gridDim.x, first = (uint64_t)blockIdx.x * per_wg, n = per_wg / 16;
  v4u acc = {0, 0, 0, 0};
  for (uint64_t i = 0; i < n; i += B) {
    v4u v[B][4];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const v4u* c = reinterpret_cast<const v4u*>(src + (first + 16 * (i + b) + wave) * 4096 + 64 * lane);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[b][k] = NT ? __builtin_nontemporal_load(c + k) : c[k];
    }
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc ^= v[b][k];
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// The span CRC's LDS budget: 64 KiB of tables (simulated: `tables`, kept live) leave ~90 KiB for a
// ring.  W waves per workgroup (one workgroup per CU), each with R slots of CH bytes (CH / 1024
// wave-instructions per chunk); COPY: the lane's piece is copied out to registers right after it
// lands and the slot refilled at once (the load overlaps the compute on the registers).
template <int W, int R, int CH, bool COPY, bool ST = false, int AUX = 2>
__global__ __launch_bounds__(64 * W) void ring_kernel(const uint8_t* __restrict__ src, uint64_t chunks_total,
                                                      uint32_t* __restrict__ out) {
  constexpr int Q = CH / 1024;  // wave-instructions per chunk
  constexpr int P = CH / 64 / 16;  // 16-B pieces per lane per chunk
  __shared__ __attribute__((aligned(16))) v4u ring[W][R][CH / 16];
  __shared__ uint32_t tables[16384];  // 64 KiB: the span's tables
  const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  tables[threadIdx.x] = threadIdx.x;
  const uint64_t per_wg = chunks_total / gridDim.x, first = (uint64_t)blockIdx.x * per_wg, n = per_wg / W;
  auto issue = [&](uint64_t i, int slot) {
    const uint8_t* c = src + (first + (uint64_t)W * i + wave) * CH;
#pragma unroll
    for (int q = 0; q < Q; ++q)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(ST ? c + 64 * lane + 16 * q : c + 1024 * q + 16 * lane),
          (__attribute__((address_space(3))) void*)(&ring[wave][slot][64 * q]), 16, 0, AUX);
  };
  for (int s = 0; s < R; ++s)
    if ((uint64_t)s < n) issue(s, s);
  v4u acc = {0, 0, 0, 0};
  for (uint64_t i = 0; i < n; ++i) {
    const int slot = (int)(i % R);
    if (i + R <= n) wait_vm<Q * (R - 1)>();
    else wait_vm<0>();
    const uint32_t addr = (uint32_t)(uintptr_t)(&ring[wave][slot][P * lane]);
    v4u r[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[k]) : "v"(addr), "i"(16 * k) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (COPY && i + R < n) issue(i + R, slot);
#pragma unroll
    for (int k = 0; k < P; ++k) acc ^= r[k];
    if (!COPY && i + R < n) issue(i + R, slot);
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w ^ tables[(threadIdx.x * 7) & 16383];
}

template <int W, int R, int CH, bool COPY, bool ST = false, int AUX = 2>
static double run_ring(const uint8_t* d, uint64_t bytes, uint32_t* out) {
  const int wgs = 256;
  const uint64_t chunks = bytes / CH / (uint64_t)(wgs * W) * (uint64_t)(wgs * W);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((ring_kernel<W, R, CH, COPY, ST, AUX>), dim3(wgs), dim3(64 * W), 0, 0, d, chunks, out);
  CHECK(hipEventRecord(a, 0));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((ring_kernel<W, R, CH, COPY, ST, AUX>), dim3(wgs), dim3(64 * W), 0, 0, d, chunks, out);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipGetLastError());
  return (double)chunks * CH * 5 / (ms * 1e-3) / 1e12;
}

__global__ void fill_random(uint64_t* d, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    d[i] = z ^ (z >> 31);
  }
}

template <class K>
static double run(K kernel, const uint8_t* d, uint64_t bytes, int wgs, uint32_t* out) {
  const uint64_t chunks = bytes / 4096 / (uint64_t)(wgs * kWaves) * (uint64_t)(wgs * kWaves);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(kernel, dim3(wgs), dim3(64 * kWaves), 0, 0, d, chunks, out);  // warm-up
  CHECK(hipEventRecord(a, 0));
  const int reps = 5;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(kernel, dim3(wgs), dim3(64 * kWaves), 0, 0, d, chunks, out);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipGetLastError());
  return (double)chunks * 4096 * reps / (ms * 1e-3) / 1e12;
}

template <class K>
static double run16(K kernel, const uint8_t* d, uint64_t bytes, int wgs, uint32_t* out) {
  const uint64_t chunks = bytes / 4096 / (uint64_t)(wgs * 16) * (uint64_t)(wgs * 16);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(kernel, dim3(wgs), dim3(1024), 0, 0, d, chunks, out);
  CHECK(hipEventRecord(a, 0));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kernel, dim3(wgs), dim3(1024), 0, 0, d, chunks, out);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipGetLastError());
  return (double)chunks * 4096 * 5 / (ms * 1e-3) / 1e12;
}

int main(int argc, char** argv) {
  const uint64_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 16) << 30;
  uint8_t* d = nullptr;
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(reinterpret_cast<void**>(&out), 1u << 24));
  hipLaunchKernelGGL(fill_random, dim3(8192), dim3(256), 0, 0, (uint64_t*)d, bytes / 8);
  CHECK(hipDeviceSynchronize());
  for (int wgs : {512, 1024, 2048}) {
    printf("wgs %4d (x %d waves): reg B=2 %.2f  reg B=4 %.2f  reg nt B=2 %.2f  B=4 %.2f  glds R=4 %.2f  R=8 %.2f  "
           "R=4 nt %.2f  R=8 nt %.2f TB/s\n", wgs, kWaves, run(reg_kernel<2>, d, bytes, wgs, out),
           run(reg_kernel<4>, d, bytes, wgs, out), run(reg_kernel<2, true>, d, bytes, wgs, out),
           run(reg_kernel<4, true>, d, bytes, wgs, out), run(glds_kernel<4, 0>, d, bytes, wgs, out),
           run(glds_kernel<8, 0>, d, bytes, wgs, out), run(glds_kernel<4, 2>, d, bytes, wgs, out),
           run(glds_kernel<8, 2>, d, bytes, wgs, out));
    fflush(stdout);
  }
  printf("ring nt, 64 KiB of tables beside it, one workgroup per CU:\n");
  printf("  16 waves x 1 x 4 KiB: %.2f  copy-out %.2f TB/s\n", run_ring<16, 1, 4096, false>(d, bytes, out),
         run_ring<16, 1, 4096, true>(d, bytes, out));
  printf("  16 waves x 1 x 4 KiB, strided fetch (lane: 16 B of its own line): nt %.2f  plain %.2f TB/s\n",
         run_ring<16, 1, 4096, true, true, 2>(d, bytes, out), run_ring<16, 1, 4096, true, true, 0>(d, bytes, out));
  printf("  16 waves x 1 x 4 KiB, coalesced, plain: %.2f TB/s\n", run_ring<16, 1, 4096, true, false, 0>(d, bytes, out));
  printf("  16 waves x 2 x 2 KiB: %.2f  copy-out %.2f TB/s\n", run_ring<16, 2, 2048, false>(d, bytes, out),
         run_ring<16, 2, 2048, true>(d, bytes, out));
  printf("  8 waves x 2 x 4 KiB: %.2f  copy-out %.2f TB/s\n", run_ring<8, 2, 4096, false>(d, bytes, out),
         run_ring<8, 2, 4096, true>(d, bytes, out));
  printf("  8 waves x 4 x 2 KiB: %.2f  copy-out %.2f TB/s\n", run_ring<8, 4, 2048, false>(d, bytes, out),
         run_ring<8, 4, 2048, true>(d, bytes, out));
  printf("  4 waves x 4 x 4 KiB: %.2f  copy-out %.2f TB/s\n", run_ring<4, 4, 4096, false>(d, bytes, out),
         run_ring<4, 4, 4096, true>(d, bytes, out));
  fflush(stdout);
  // the span kernel's own shape: 1024 threads per workgroup, one workgroup per CU
  printf("span shape (256 x 16 waves): reg B=2 %.2f  reg nt B=2 %.2f TB/s\n",
         run16(reg_kernel16<2, false>, d, bytes, 256, out), run16(reg_kernel16<2, true>, d, bytes, 256, out));
  CHECK(hipFree(d));
  CHECK(hipFree(out));
  return 0;
}
