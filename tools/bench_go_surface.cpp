// Native driver for the UNCHANGED Go surface (efes_hash.h layer 2), making exactly the calls the
// cgo binding of INTEGRATION.md §2 (hash_gpu.go) makes under filereceiver.go's saveFile:
//   per PATCH   efes_sha1_new_pool + efes_crc32_new_pool           (newFileInfo, fileinfo.go:20-27)
//               efes_sha1_unmarshal_text + efes_crc32_unmarshal_text of the saved .info state
//                                                                   (ReadFileInfo, filereceiver.go:182)
//               per io.Copy buffer of W bytes: efes_crc32_write then efes_sha1_write of the SAME (p, n)
//                                                                   (MultiWriter(f, CRC32, Sha1), :208-209)
//               last PATCH: efes_sha1_sum then efes_crc32_sum       (digest headers, :99-100)
//               else:       efes_sha1_marshal_text then efes_crc32_marshal_text (SaveFileInfo, :226)
//               efes_sha1_free + efes_crc32_free                    (the finalizers)
// T threads stand in for request goroutines; each keeps K uploads in flight (lockstep groups, as
// tools/bench_uploads does for the fused efes_upload path) over its OWN copy of the object bytes
// (each request has its own io.Copy buffer).  All uploads hash the same bytes with the same PATCH
// boundaries, so every Sum and every saved text must equal the first upload's, which bench.py and
// tests/test_gpu_go_surface.py check against hashlib/zlib and the oracle.  Prints one JSON line.
// `writes` = same (default: MultiWriter, both digests get the same buffer, the library fuses the
// pair) or copy (the SHA-1 digest gets an equal copy at another address: the pair never binds, the
// two digests are two uploads -- round 3's behaviour, each byte staged and hashed twice).
// Not part of the product library.
// Devices: like hash_gpu.go's pool(), one context per visible GPU (efes_device_count, a GPU whose
// context fails is skipped) and one efes_pool over them -- a storage server is one process on every
// GPU of its node (server.go:130) -- or the ordinals of `devices` ("0,0": two contexts of GPU 0).  The
// staging per GPU is staging_mib / GPUs (at least 256 MiB); the line reports per-device launches,
// jobs and bytes.
//   tools/bench_go_surface <threads> <uploads> <upload_bytes> <write_bytes> [open_per_thread]
//                          [patches] [chunk_kib] [staging_mib] [texts_out|-] [writes] [devices|all]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "efes_hash.h"
#include "cpu_quota.hpp"
#include "efes_devices.hpp"

namespace {

using clk = std::chrono::steady_clock;

struct Expect {
  std::vector<std::string> sha_text, crc_text;  // after PATCH p (p < patches - 1)
  uint8_t sha[20] = {}, crc[4] = {};
};

// One group of uploads through one PATCH: new digests, resume, MultiWriter Writes, sync point.
// Returns the number of mismatches against `ex` (or records into it when `record`).
int patch_group(efes_pool* pool, const uint8_t* buf, const uint8_t* sha_buf, size_t from, size_t to, size_t W, int p,
                int patches,
                std::vector<std::string>& sha_state, std::vector<std::string>& crc_state, Expect& ex, bool record,
                std::atomic<int>& errs) {
  const size_t K = sha_state.size();
  std::vector<efes_sha1*> sha(K, nullptr);
  std::vector<efes_crc32*> crc(K, nullptr);
  int bad = 0;
  for (size_t i = 0; i < K; ++i) {
    if (efes_sha1_new_pool(pool, &sha[i]) || efes_crc32_new_pool(pool, &crc[i])) ++errs;
    if (p > 0 && (efes_sha1_unmarshal_text(sha[i], sha_state[i].data(), sha_state[i].size()) ||
                  efes_crc32_unmarshal_text(crc[i], crc_state[i].data(), crc_state[i].size())))
      ++errs;
  }
  for (size_t a = from; a < to; a += W) {
    const size_t m = std::min(W, to - a);
    for (size_t i = 0; i < K; ++i)
      if (efes_crc32_write(crc[i], buf + a, m) || efes_sha1_write(sha[i], sha_buf + a, m)) ++errs;
  }
  const bool last = p == patches - 1;
  for (size_t i = 0; i < K; ++i) {
    if (last) {
      uint8_t s[20], c[4];
      if (efes_sha1_sum(sha[i], s) || efes_crc32_sum(crc[i], c)) {
        ++errs;
      } else if (record && i == 0) {
        memcpy(ex.sha, s, 20);
        memcpy(ex.crc, c, 4);
      } else if (memcmp(s, ex.sha, 20) || memcmp(c, ex.crc, 4)) {
        ++bad;
      }
    } else {
      char st[200], ct[8];
      if (efes_sha1_marshal_text(sha[i], st) || efes_crc32_marshal_text(crc[i], ct)) {
        ++errs;
        continue;
      }
      sha_state[i].assign(st, 200);
      crc_state[i].assign(ct, 8);
      if (record && i == 0) {
        ex.sha_text[p] = sha_state[i];
        ex.crc_text[p] = crc_state[i];
      } else if (sha_state[i] != ex.sha_text[p] || crc_state[i] != ex.crc_text[p]) {
        ++bad;
      }
    }
  }
  for (size_t i = 0; i < K; ++i) {
    efes_sha1_free(sha[i]);
    efes_crc32_free(crc[i]);
  }
  return bad;
}

double pct(std::vector<double> v, double q) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1) + 0.5))];
}

}  // namespace

int main(int argc, char** argv) {
  const int pinned_cpus = pin_to_cpu_quota();  // see cpu_quota.hpp
  if (argc < 5) {
    fprintf(stderr, "usage: %s threads uploads upload_bytes write_bytes [open_per_thread] [patches] [chunk_kib] "
                    "[staging_mib] [texts_out|-] [same|copy]\n", argv[0]);
    return 2;
  }
  const int T = atoi(argv[1]);
  const long U = atol(argv[2]);
  const size_t S = strtoull(argv[3], nullptr, 10), W = strtoull(argv[4], nullptr, 10);
  const int K = argc > 5 ? atoi(argv[5]) : 64;
  const int P = argc > 6 ? std::max(1, atoi(argv[6])) : 1;
  const char* chunk_kib = argc > 7 ? argv[7] : "256";
  const char* staging_mib = argc > 8 ? argv[8] : "8192";
  const char* texts_out = argc > 9 && strcmp(argv[9], "-") ? argv[9] : nullptr;
  const bool copy_writes = argc > 10 && !strcmp(argv[10], "copy");
  const char* dev_list = argc > 11 ? argv[11] : "all";
  if (T < 1 || U < 1 || S < 1 || W < 1 || K < 1) return 2;
  EfesDevices devs = efes_open_devices(dev_list);  // hash_gpu.go pool(): every GPU that opens
  const int ndev = (int)devs.ctxs.size();
  if (ndev == 0) {
    fprintf(stderr, "no device opened (%d visible)\n", devs.visible);
    return 1;
  }
  // The digest queues are created at each GPU's first digest Write: size them like bench_uploads'
  // queue, the staging split over the GPUs.
  char per_gpu_mib[32];
  snprintf(per_gpu_mib, sizeof per_gpu_mib, "%ld", std::max(256L, atol(staging_mib) / ndev));
  setenv("EFES_DIGEST_CHUNK_KIB", chunk_kib, 0);
  setenv("EFES_DIGEST_STAGING_MIB", per_gpu_mib, 0);
  int rc = 0;
  efes_pool* pool = nullptr;
  rc = efes_pool_create(devs.ctxs.data(), (uint32_t)ndev, &pool);  // hash_gpu.go: one context per GPU, one pool
  if (rc) {
    fprintf(stderr, "efes_pool_create: %s\n", efes_strerror(rc));
    return 1;
  }
  std::vector<uint8_t> src(S);
  uint64_t z = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < S; ++i) {
    z ^= z << 13; z ^= z >> 7; z ^= z << 17;
    src[i] = (uint8_t)z;
  }
  std::vector<size_t> cut(P + 1);  // PATCH boundaries (write.go: one PATCH per ChunkSize piece)
  for (int p = 0; p <= P; ++p) cut[p] = S * (size_t)p / (size_t)P;
  std::atomic<int> errs{0}, bad{0};
  // The expected texts and digests: one upload through the same calls before the clock starts.
  Expect ex;
  ex.sha_text.resize(P);
  ex.crc_text.resize(P);
  {
    std::vector<std::string> ss(1), cs(1);
    for (int p = 0; p < P; ++p)
      patch_group(pool, src.data(), src.data(), cut[p], cut[p + 1], W, p, P, ss, cs, ex, true, errs);
    if (errs) {
      fprintf(stderr, "reference upload failed\n");
      return 1;
    }
  }
  auto pool_stats = [&] {
    std::vector<efes_queue_stats> v(ndev);
    for (int i = 0; i < ndev; ++i) efes_pool_stats(pool, (uint32_t)i, &v[i]);
    return v;
  };
  auto total = [](const std::vector<efes_queue_stats>& v) {
    efes_queue_stats t{};
    for (const auto& x : v) {
      t.launches += x.launches;
      t.jobs += x.jobs;
      t.bytes += x.bytes;
    }
    return t;
  };
  const std::vector<efes_queue_stats> d0 = pool_stats();
  const efes_queue_stats q0 = total(d0);
  efes_pair_stats f0{};
  efes_pair_stats_get(&f0);
  std::mutex lat_mu;
  std::vector<double> group_ms;  // wall time of one PATCH of a group of K uploads
  auto t0 = clk::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      std::vector<uint8_t> buf(src);  // this request's own bytes (its own io.Copy buffers)
      std::vector<uint8_t> buf2(copy_writes ? src : std::vector<uint8_t>());
      const uint8_t* sha_buf = copy_writes ? buf2.data() : buf.data();
      std::vector<long> mine;
      for (long u = t; u < U; u += T) mine.push_back(u);
      std::vector<double> ms;
      for (size_t g = 0; g < mine.size(); g += (size_t)K) {
        const size_t n = std::min(mine.size() - g, (size_t)K);
        std::vector<std::string> ss(n), cs(n);
        for (int p = 0; p < P; ++p) {
          const auto a = clk::now();
          bad += patch_group(pool, buf.data(), sha_buf, cut[p], cut[p + 1], W, p, P, ss, cs, ex, false, errs);
          ms.push_back(std::chrono::duration<double, std::milli>(clk::now() - a).count());
        }
      }
      std::lock_guard<std::mutex> lk(lat_mu);
      group_ms.insert(group_ms.end(), ms.begin(), ms.end());
    });
  for (auto& x : th) x.join();
  const double secs = std::chrono::duration<double>(clk::now() - t0).count();
  const std::vector<efes_queue_stats> d1 = pool_stats();
  const efes_queue_stats q1 = total(d1);
  efes_pair_stats f1{};
  efes_pair_stats_get(&f1);
  if (texts_out) {  // for the oracle check in tests/test_gpu_go_surface.py
    if (FILE* f = fopen(texts_out, "w")) {
      for (int p = 0; p + 1 < P; ++p) fprintf(f, "%s %s\n", ex.sha_text[p].c_str(), ex.crc_text[p].c_str());
      fclose(f);
    }
  }
  efes_pool_destroy(pool);
  const std::string per_dev = efes_devices_json(devs, d0, d1);
  efes_close_devices(devs);
  char hex[49];
  for (int i = 0; i < 20; ++i) snprintf(hex + 2 * i, 3, "%02x", ex.sha[i]);
  for (int i = 0; i < 4; ++i) snprintf(hex + 40 + 2 * i, 3, "%02x", ex.crc[i]);
  const double bytes = (double)U * (double)S;
  printf("{\"workload\": \"go_surface\", \"pinned_cpus\": %d, \"threads\": %d, \"uploads\": %ld, \"upload_bytes\": %zu, "
         "\"write_bytes\": %zu, \"open_per_thread\": %d, \"patches\": %d, \"chunk_kib\": %s, \"staging_mib\": %s, "
         "\"writes\": \"%s\", \"seconds\": %.4f, \"value\": %.3f, \"unit\": \"GiB/s\", "
         "\"launches\": %llu, \"jobs\": %llu, \"hashed_bytes_per_byte\": %.4f, "
         "\"pairs\": %llu, \"fused_bytes_per_byte\": %.4f, \"settles\": %llu, "
         "\"patch_group_ms\": {\"p50\": %.3f, \"p90\": %.3f, \"p99\": %.3f, \"n\": %zu}, "
         "\"devices_visible\": %d, \"devices_opened\": %d, \"devices_skipped\": %d, \"staging_mib_per_gpu\": %s, "
         "\"devices\": %s, "
         "\"sum_sha1_crc32\": \"%s\", \"all_equal\": %s, \"errors\": %d}\n",
         pinned_cpus, T, U, S, W, K, P, chunk_kib, staging_mib,
         copy_writes ? "copy" : "same", secs,
         bytes / secs / (1u << 30), (unsigned long long)(q1.launches - q0.launches),
         (unsigned long long)(q1.jobs - q0.jobs), (double)(q1.bytes - q0.bytes) / bytes,
         (unsigned long long)(f1.pairs - f0.pairs), (double)(f1.fused_bytes - f0.fused_bytes) / bytes,
         (unsigned long long)(f1.settles - f0.settles), pct(group_ms, 0.5), pct(group_ms, 0.9), pct(group_ms, 0.99),
         group_ms.size(), devs.visible, ndev, devs.skipped, getenv("EFES_DIGEST_STAGING_MIB"), per_dev.c_str(), hex,
         bad ? "false" : "true", errs.load());
  return errs || bad ? 1 : 0;
}
