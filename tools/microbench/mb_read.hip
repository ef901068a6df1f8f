// mb_read.hip -- the practical HBM read ceiling for the span CRC's access shapes (DESIGN_NOTES.md §4 "Span CRC").
// Every byte of a 16 GiB buffer is read once with global_load_dwordx4 and XOR-folded (one store per
// lane at the end), in the shapes the span kernel can use:
//   coal : each wave-instruction reads 1 KiB contiguous (lane j: 16 B at 16 j)
//   lane64 / lane128 : lane j reads 64 / 128 contiguous bytes (4 / 8 dwordx4 at stride 64 / 128 B
//          across lanes), rows of a workgroup interleaved as in span_kernel
// Usage: mb_read [gib] [threads_per_wg] [wgs]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                            \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// W = bytes per lane per row (16: coalesced 1 KiB per wave-instruction; 64, 128: per-lane lines).
template <int W>
__global__ void read_kernel(const v4u* __restrict__ src, uint64_t rows_total, uint32_t* __restrict__ out) {
  const uint32_t L = blockDim.x, j = threadIdx.x;
  const uint64_t q = rows_total / gridDim.x, r = rows_total % gridDim.x, w = blockIdx.x;
  const uint64_t rows = q + (w < r ? 1 : 0), start = w < r ? w * (q + 1) : r * (q + 1) + (w - r) * q;
  constexpr int V = W / 16;  // dwordx4 per lane per row
  v4u acc = {0, 0, 0, 0};
  const v4u* base = src + start * (uint64_t)L * V;
  for (uint64_t i = 0; i < rows; ++i) {
    const v4u* row = base + i * (uint64_t)L * V;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const v4u v = W == 16 ? row[j] : row[(uint64_t)j * V + k];
      acc ^= v;
    }
  }
  out[(uint64_t)w * L + j] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// splitmix64 bytes, as the benchmarks' synthetic data (random bits on the HBM bus)
__global__ void fill_random(uint64_t* d, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    d[i] = z ^ (z >> 31);
  }
}

template <int W>
static double run(const v4u* d, uint64_t bytes, int threads, int wgs, uint32_t* out) {
  const uint64_t rows = bytes / ((uint64_t)threads * W);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(read_kernel<W>, dim3(wgs), dim3(threads), 0, 0, d, rows, out);  // warm-up
  CHECK(hipEventRecord(a, 0));
  const int reps = 5;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(read_kernel<W>, dim3(wgs), dim3(threads), 0, 0, d, rows, out);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return (double)rows * threads * W * reps / (ms * 1e-3) / 1e12;
}

int main(int argc, char** argv) {
  const uint64_t gib = argc > 1 ? strtoull(argv[1], 0, 10) : 16;
  const uint64_t bytes = gib << 30;
  void* d = nullptr;
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(reinterpret_cast<void**>(&out), 1u << 24));
  CHECK(hipMemset(d, 0x5a, bytes));
  const int shapes[][2] = {{1024, 256}, {512, 512}, {256, 1024}, {256, 2048}, {1024, 512}};
  for (int pass = 0; pass < 2; ++pass)
  for (auto& s : shapes) {
    if (pass == 1 && &s == &shapes[0]) {
      hipLaunchKernelGGL(fill_random, dim3(8192), dim3(256), 0, 0, (uint64_t*)d, bytes / 8);
      CHECK(hipDeviceSynchronize());
      printf("random data:\n");
    }
    const int t = argc > 2 ? atoi(argv[2]) : s[0], g = argc > 3 ? atoi(argv[3]) : s[1];
    printf("  threads %4d wgs %4d: coal %.2f TB/s  lane64 %.2f TB/s  lane128 %.2f TB/s\n", t, g,
           run<16>((const v4u*)d, bytes, t, g, out), run<64>((const v4u*)d, bytes, t, g, out),
           run<128>((const v4u*)d, bytes, t, g, out));
    if (argc > 2) break;
  }
  CHECK(hipFree(d));
  CHECK(hipFree(out));
  return 0;
}
