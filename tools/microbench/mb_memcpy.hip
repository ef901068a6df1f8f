// Host memcpy rate into staging memory of different kinds, T threads writing 32 KiB pieces
// round-robin over their own 256 KiB chunks (the efes_upload_write pattern), optionally while
// the GPU reads the same kind of memory over PCIe (zero-copy kernel) -- is the uploads path's
// ~37 GiB/s the writers' memcpy?
//   mb_memcpy <threads> [gpu_read 0/1]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

__global__ void sum_kernel(const uint4* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

static double run(uint8_t* dst, size_t bytes, int T, const uint8_t* src, size_t piece, int reps) {
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  const size_t per = bytes / T;
  for (int t = 0; t < T; ++t)
    th.emplace_back([=] {
      uint8_t* base = dst + per * t;
      for (int r = 0; r < reps; ++r)
        for (size_t o = 0; o + piece <= per; o += piece) memcpy(base + o, src + (o % (4u << 20)), piece);
    });
  for (auto& x : th) x.join();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return (double)per * T * reps / s / (1u << 30);
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 16;
  const int gpu = argc > 2 ? atoi(argv[2]) : 0;
  const size_t bytes = (size_t)2 << 30, piece = 32 << 10;
  std::vector<uint8_t> src(4u << 20, 7);
  struct Kind { const char* name; unsigned flags; int pageable; } kinds[] = {
      {"pageable", 0, 1},
      {"pinned_mapped", hipHostMallocMapped, 0},
      {"pinned_mapped_noncoherent", hipHostMallocMapped | hipHostMallocNonCoherent, 0},
      {"pinned_mapped_wc", hipHostMallocMapped | hipHostMallocWriteCombined, 0},
  };
  uint32_t* d_out;
  hipMalloc(&d_out, 4);
  for (auto& k : kinds) {
    uint8_t* p = nullptr;
    if (k.pageable) {
      p = (uint8_t*)aligned_alloc(4096, bytes);
    } else if (hipHostMalloc((void**)&p, bytes, k.flags) != hipSuccess) {
      printf("%s: alloc failed\n", k.name);
      continue;
    }
    memset(p, 1, bytes);
    run(p, bytes, T, src.data(), piece, 1);  // warm
    std::atomic<bool> stop{false};
    std::thread g;
    double gpu_gbs = 0;
    if (gpu && !k.pageable) {
      g = std::thread([&] {
        uint8_t* dp;
        hipHostGetDevicePointer((void**)&dp, p, 0);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        int n = 0;
        hipEventRecord(a, 0);
        while (!stop) {
          hipLaunchKernelGGL(sum_kernel, dim3(4096), dim3(256), 0, 0, (const uint4*)dp, bytes / 16, d_out);
          hipDeviceSynchronize();
          ++n;
        }
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        gpu_gbs = (double)bytes * n / (ms / 1e3) / (1u << 30);
      });
    }
    const double gbs = run(p, bytes, T, src.data(), piece, 4);
    stop = true;
    if (g.joinable()) g.join();
    printf("%-28s T=%d memcpy %.1f GiB/s%s", k.name, T, gbs, gpu && !k.pageable ? "" : "\n");
    if (gpu && !k.pageable) printf("  concurrent GPU zero-copy read %.1f GiB/s\n", gpu_gbs);
    if (k.pageable) free(p);
    else hipHostFree(p);
  }
  return 0;
}
