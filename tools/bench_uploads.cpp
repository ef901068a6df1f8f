// Native driver for the concurrent-uploads path (efes_queue / efes_upload), the way the Go
// server would use it: T threads stand in for the request goroutines; each keeps K uploads open
// at once and feeds them round-robin with Write calls of W bytes (io.Copy's 32 KiB buffers,
// filereceiver.go:209) from ordinary pageable memory, then Sums each (filereceiver.go:99-100).
// T x K concurrent uploads is what fills the GPU: each upload's SHA-1 is a serial chain.
// Devices: one efes_queue per visible GPU that opens (as go/upload_gpu.go's uploadQueue() over
// hash_gpu.go's pool()), each upload opened on the queue with the most free upload slots; or the
// ordinals of `devices` ("0,0": two queues on two contexts of GPU 0).  Per-device counters in the line.
// Prints one JSON line.  Not part of the product library.
//   tools/bench_uploads <threads> <uploads> <upload_bytes> <write_bytes> [open_per_thread] [chunk_bytes] [stagger]
//                       [devices|all]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "efes_hash.h"
#include "cpu_quota.hpp"
#include "efes_devices.hpp"

int main(int argc, char** argv) {
  const int pinned_cpus = pin_to_cpu_quota();  // see cpu_quota.hpp
  if (argc < 5) {
    fprintf(stderr, "usage: %s threads uploads upload_bytes write_bytes [open_per_thread] [chunk_bytes] [stagger]\n", argv[0]);
    return 2;
  }
  const int T = atoi(argv[1]);
  const long U = atol(argv[2]);
  const size_t S = strtoull(argv[3], nullptr, 10), W = strtoull(argv[4], nullptr, 10);
  const int K = argc > 5 ? atoi(argv[5]) : 64;
  const uint64_t chunk = argc > 6 ? strtoull(argv[6], nullptr, 10) : (256u << 10);
  const int stagger = argc > 7 ? atoi(argv[7]) : 0;
  const char* dev_list = argc > 8 ? argv[8] : "all";
  EfesDevices devs = efes_open_devices(dev_list);
  const int ndev = (int)devs.ctxs.size();
  if (ndev == 0) {
    fprintf(stderr, "no device opened (%d visible)\n", devs.visible);
    return 1;
  }
  // Every queue can hold every upload (placement may be uneven); the staging is split over the GPUs.
  const uint32_t max_uploads = (uint32_t)(T * K);
  const uint32_t max_chunks = std::max<uint32_t>(4 * max_uploads / (uint32_t)ndev, max_uploads) + 64;
  std::vector<efes_queue*> qs(ndev, nullptr);
  int rc = 0;
  for (int i = 0; i < ndev; ++i) {
    rc = efes_queue_create(devs.ctxs[i], chunk, max_chunks, max_uploads, &qs[i]);
    if (rc) {
      fprintf(stderr, "efes_queue_create on device %d: %s\n", devs.ords[i], efes_strerror(rc));
      return 1;
    }
  }
  efes_queue* q = qs[0];
  // upload_gpu.go uploadQueue(): the queue with the most free upload slots
  auto pick = [&]() {
    efes_queue* best = qs[0];
    uint32_t most = 0;
    for (efes_queue* x : qs) {
      efes_queue_stats st;
      if (efes_queue_get_stats(x, &st) == EFES_OK && st.free_uploads > most) {
        best = x;
        most = st.free_uploads;
      }
    }
    return best;
  };
  auto stats = [&] {
    std::vector<efes_queue_stats> v(ndev);
    for (int i = 0; i < ndev; ++i) efes_queue_get_stats(qs[i], &v[i]);
    return v;
  };
  std::vector<uint8_t> src(S);
  uint64_t z = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < S; ++i) {
    z ^= z << 13; z ^= z >> 7; z ^= z << 17;
    src[i] = (uint8_t)z;
  }
  // The expected digest pair, from one upload before the clock starts (every upload hashes the
  // same bytes, so every Sum must equal it).
  uint8_t first[24] = {};
  {
    efes_upload* up = nullptr;
    rc = efes_upload_open(q, EFES_HASH_SHA1 | EFES_HASH_CRC32, nullptr, nullptr, &up);
    for (size_t a = 0; rc == 0 && a < S; a += W) rc = efes_upload_write(up, src.data() + a, a + W <= S ? W : S - a);
    if (rc == 0) rc = efes_upload_sum(up, first);
    if (up) efes_upload_close(up);
    if (rc) {
      fprintf(stderr, "reference upload: %s\n", efes_strerror(rc));
      return 1;
    }
  }
  std::atomic<int> bad{0}, errs{0};
  const std::vector<efes_queue_stats> d0 = stats();
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      std::vector<long> mine;
      for (long u = t; u < U; u += T) mine.push_back(u);
      // stagger 0: lockstep groups of K (open, write all, Sum all).  stagger 1: half-groups of
      // K/2, each half's Sums taken after the NEXT half has been written, so a thread's Sum waits
      // overlap its own writes (request goroutines at different phases, as on a real server).
      const size_t grp = stagger ? std::max<size_t>(1, (size_t)K / 2) : (size_t)K;
      std::vector<efes_upload*> pending, ups;
      // Error exit: close every upload this thread still holds (efes_queue_destroy requires it).
      auto fail = [&] {
        ++errs;
        for (auto* up : ups)
          if (up) efes_upload_close(up);
        for (auto* up : pending) efes_upload_close(up);
        ups.clear();
        pending.clear();
      };
      auto sum_close = [&](std::vector<efes_upload*>& ups) {
        for (auto* up : ups) {
          uint8_t sum[24];
          if (efes_upload_sum(up, sum)) ++errs;
          else if (memcmp(first, sum, 24)) ++bad;
          efes_upload_close(up);
        }
        ups.clear();
      };
      for (size_t g = 0; g < mine.size(); g += grp) {
        const size_t n = std::min(mine.size() - g, grp);
        ups.assign(n, nullptr);
        for (auto& up : ups)
          if (efes_upload_open(pick(), EFES_HASH_SHA1 | EFES_HASH_CRC32, nullptr, nullptr, &up)) return fail();
        for (size_t a = 0; a < S; a += W)
          for (auto* up : ups)
            if (efes_upload_write(up, src.data() + a, a + W <= S ? W : S - a)) return fail();
        sum_close(pending);
        pending = std::move(ups);
        if (!stagger) sum_close(pending);
      }
      sum_close(pending);
    });
  for (auto& x : th) x.join();
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const std::vector<efes_queue_stats> d1 = stats();
  for (efes_queue* x : qs) efes_queue_destroy(x);
  const std::string per_dev = efes_devices_json(devs, d0, d1);
  efes_close_devices(devs);
  char hex[49];
  for (int i = 0; i < 24; ++i) snprintf(hex + 2 * i, 3, "%02x", first[i]);
  printf("{\"workload\": \"uploads\", \"pinned_cpus\": %d, \"threads\": %d, \"uploads\": %ld, \"upload_bytes\": %zu, \"write_bytes\": %zu, "
         "\"open_per_thread\": %d, \"stagger\": %d, \"chunk_bytes\": %llu, \"max_chunks\": %u, \"seconds\": %.4f, \"value\": %.3f, \"unit\": \"GiB/s\", "
         "\"devices_visible\": %d, \"devices_opened\": %d, \"devices_skipped\": %d, \"devices\": %s, "
         "\"sum_sha1_crc32\": \"%s\", \"all_sums_equal\": %s, \"errors\": %d}\n",
         pinned_cpus, T, U, S, W, K, stagger, (unsigned long long)chunk, max_chunks, secs, (double)U * S / secs / (1u << 30),
         devs.visible, ndev, devs.skipped, per_dev.c_str(), hex, bad ? "false" : "true", errs.load());
  return errs || bad ? 1 : 0;
}
