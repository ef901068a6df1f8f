// H2D bandwidth from pinned host memory: one contiguous hipMemcpyAsync vs strided
// hipMemcpy2DAsync (the segmented ingest's copy of 1 MiB of each of 1024 chunks), on 1, 2, 4
// streams.  Prints GB/s per variant.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
  const size_t nchunk = 1024, chunk = 4 << 20, seg = 1 << 20;
  void* host;
  CK(hipHostMalloc(&host, nchunk * chunk, hipHostMallocDefault));
  void* dev;
  CK(hipMalloc(&dev, nchunk * seg * 2));
  memset(host, 1, nchunk * chunk);
  std::vector<hipStream_t> st(4);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep)
    for (int kind = 0; kind < 2; ++kind)
      for (int ns : {1, 2, 4}) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        const int iters = 4;
        for (int it = 0; it < iters; ++it)
          for (int k = 0; k < ns; ++k) {
            const size_t c0 = nchunk * k / ns, c1 = nchunk * (k + 1) / ns;
            if (kind == 0)  // contiguous: the same byte count
              CK(hipMemcpyAsync((char*)dev + c0 * seg, (char*)host + c0 * seg, (c1 - c0) * seg, hipMemcpyHostToDevice, st[k]));
            else            // strided: 1 MiB of each chunk
              CK(hipMemcpy2DAsync((char*)dev + c0 * seg, seg, (char*)host + c0 * chunk + it * seg, chunk, seg, c1 - c0,
                                  hipMemcpyHostToDevice, st[k]));
          }
        for (int k = 0; k < ns; ++k) CK(hipStreamSynchronize(st[k]));
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%s streams=%d: %.1f GB/s\n", kind ? "2D strided " : "contiguous", ns, iters * nchunk * seg / (ms * 1e-3) / 1e9);
      }
  return 0;
}
