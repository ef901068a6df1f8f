// mb_clock.hip -- is s_memtime a core-clock counter on gfx950, and does a sleeping one-wave
// probe on a queue of its own read the engine clock of a busy chip?
//
// Phase "idle":   the probe alone for ~200 ms.
// Phase "loaded": the probe, then an all-CU VALU-bound kernel on another stream; the probe is
//                 stopped (host-coherent flag) once the busy kernel has ended.
// Prints memtime ticks, realtime ticks (100 MHz) and their ratio x 100 MHz per phase, plus the busy
// kernel's event time.  Compare with GRBM_GUI_ACTIVE / 8 / ns of the busy kernel (rocprofv3 pass).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <chrono>
#include <thread>
#include <atomic>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void probe(unsigned long long* out, const int* stop, unsigned long long max_rt) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long r = r0, n = 0;
  for (;;) {
    __builtin_amdgcn_s_sleep(127);
    r = __builtin_amdgcn_s_memrealtime();
    ++n;
    if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 || r - r0 > max_rt) break;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[0] = t1 - t0;
  out[1] = r - r0;
  out[2] = n;
}

__global__ void busy(uint32_t* out, int iters) {
  uint32_t a = threadIdx.x, b = blockIdx.x, c = 0x12345u, d = 7u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll 16
    for (int k = 0; k < 16; ++k) {
      a = __builtin_amdgcn_alignbit(a, b, 5) + c;
      b = __builtin_amdgcn_bitop3_b32(a, b, d, 0x96);
      c += b;
      d ^= a;
    }
  }
  if ((a ^ b ^ c ^ d) == 0x5a5a5a5au) out[0] = a;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 40000;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  int* stop = nullptr;
  CK(hipHostMalloc(&stop, 64, hipHostMallocCoherent));
  unsigned long long* d_out = nullptr;
  uint32_t* d_sink = nullptr;
  CK(hipMalloc(&d_out, 64));
  CK(hipMalloc(&d_sink, 64));
  hipDeviceProp_t prop{};
  CK(hipGetDeviceProperties(&prop, 0));
  uint32_t mask[8];
  for (int w = 0; w < 8; ++w) {
    const int left = prop.multiProcessorCount - 32 * w;
    mask[w] = left >= 32 ? 0xffffffffu : left > 0 ? (1u << left) - 1u : 0u;
  }
  hipStream_t ps, bs;
  CK(hipExtStreamCreateWithCUMask(&ps, 8, mask));
  CK(hipStreamCreateWithFlags(&bs, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  busy<<<1, 64, 0, bs>>>(d_sink, 10);  // load the code objects
  probe<<<1, 64, 0, ps>>>(d_out, stop, 1000ull);
  CK(hipDeviceSynchronize());
  const int grid = 4 * prop.multiProcessorCount * 2;  // two waves of 256 per SIMD... 8 waves per CU
  for (int rep = 0; rep < reps; ++rep) {
    for (int loaded = 0; loaded < 2; ++loaded) {
      *stop = 0;
      std::atomic_thread_fence(std::memory_order_seq_cst);
      probe<<<1, 64, 0, ps>>>(d_out, stop, 2000000000ull);  // <= 20 s whatever happens
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
      float ms = 0;
      if (loaded) {
        CK(hipEventRecord(e0, bs));
        busy<<<grid, 256, 0, bs>>>(d_sink, iters);
        CK(hipEventRecord(e1, bs));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
      } else {
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
      }
      __atomic_store_n(stop, 1, __ATOMIC_SEQ_CST);
      CK(hipStreamSynchronize(ps));
      unsigned long long h[3];
      CK(hipMemcpy(h, d_out, sizeof h, hipMemcpyDeviceToHost));
      printf("{\"phase\": \"%s\", \"rep\": %d, \"memtime\": %llu, \"realtime\": %llu, \"polls\": %llu, "
             "\"memtime_mhz\": %.1f, \"busy_ms\": %.3f}\n",
             loaded ? "loaded" : "idle", rep, h[0], h[1], h[2], 100.0 * (double)h[0] / (double)h[1], ms);
      fflush(stdout);
    }
  }
  return 0;
}
