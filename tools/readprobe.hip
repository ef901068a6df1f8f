// readprobe.hip -- the HBM read ceiling of ONE buffer, measured on the GPU itself (bench.py's
// span leg: `read_ceiling`; measurement infrastructure, not part of libefeshash).
//
// The span CRC's rate depends on the buffer it reads (its allocation: DESIGN.md §4 "Span CRC"), so
// its roofline fraction is also reported against a pure read of the SAME buffer, in the access
// shape the span kernel uses: one workgroup of 16 waves per CU, each wave streaming 4 KiB at a
// time into its own LDS slot by LDS-DMA with the nontemporal policy (rows dealt round-robin over the
// workgroups), reading the slot back and XOR-folding it (one word per lane stored at the end, so
// nothing is elided).  No hashing, no tables: what the memory system delivers to this shape.
// tools/microbench/mb_glds.hip is the same read in more shapes, on a fresh buffer.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kWaves = 16, kSlot = 4096;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64 * kWaves) void read_kernel(const uint8_t* __restrict__ src, uint64_t rows,
                                                           uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) v4u ring[kWaves][kSlot / 16];
  const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  constexpr uint64_t kRow = (uint64_t)kWaves * kSlot;  // 64 KiB: one row of one workgroup
  v4u acc = {0, 0, 0, 0};
  for (uint64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const uint8_t* c = src + r * kRow + (uint64_t)wave * kSlot;
#pragma unroll
    for (int q = 0; q < kSlot / 1024; ++q)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(c + 1024 * q + 16 * lane),
                                       (__attribute__((address_space(3))) void*)(&ring[wave][64 * q]), 16, 0, 2);
    __builtin_amdgcn_s_waitcnt(0);  // (the compiler also waits before the LDS reads below)
#pragma unroll
    for (int k = 0; k < kSlot / 1024; ++k) acc ^= ring[wave][64 * k + lane];
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

uint32_t* g_out[64] = {};

}  // namespace

extern "C" {

// Reads the first bytes - bytes % 64 KiB of buf (device memory of `device`) once, on `stream`, with
// `groups` workgroups (one per CU).  Asynchronous; time it with events on the same stream.
int readprobe_launch(int device, const void* buf, uint64_t bytes, int groups, void* stream) {
  if (device < 0 || device >= 64 || groups <= 0 || !buf) return -1;
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return -2;
  int rc = 0;
  if (!g_out[device] &&
      hipMalloc(reinterpret_cast<void**>(&g_out[device]), (size_t)1024 * 64 * kWaves * sizeof(uint32_t)) != hipSuccess)
    rc = -3;
  if (!rc) {
    const int g = groups < 1024 ? groups : 1024;
    hipLaunchKernelGGL(read_kernel, dim3(g), dim3(64 * kWaves), 0, static_cast<hipStream_t>(stream),
                       static_cast<const uint8_t*>(buf), bytes / ((uint64_t)kWaves * kSlot), g_out[device]);
    rc = hipGetLastError() == hipSuccess ? 0 : -4;
  }
  (void)hipSetDevice(prev);
  return rc;
}

}  // extern "C"
