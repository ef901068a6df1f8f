// Native driver for the upload receiver above the C ABI (efes_amd/host/efes_receiver.hpp): the
// storage server's PATCH path end to end -- file write, fsync, the fused SHA-1 + CRC-32 on the
// GPU, the .info state between PATCHes and the digest headers of the last one -- with T threads
// standing in for the request goroutines of server.go:130 (one PATCH at a time each, as net/http
// runs a handler), and the read-back path (Sha1File over files, write.go:69 / drain.go:125).
// Prints one JSON line per mode.  Not part of the product library.
//
//   tools/bench_receiver receiver <dir> <threads> <uploads_per_thread> <upload_bytes> <patch_bytes> [gpus]
//                                 (gpus > 1: one process over several GPUs, a queue per GPU, each
//                                  PATCH on the least-loaded one -- a storage server is one process)
//   tools/bench_receiver sha1file <dir> <threads> <files_per_thread> <file_bytes>
//   tools/bench_receiver drain    <dir> <workers> <fids> <file_bytes> [nfiles]  (the drainer's read-back,
//                                 drain.go:87-125: <fids> moves of the existing files <dir>/<i % nfiles>.fid
//                                 (nfiles defaults to fids), each moved by
//                                 write.go's sendFile -- read through Sha1File, hashed on the GPU,
//                                 one PATCH per ChunkSize -- to a sink server; <workers> files in
//                                 flight at once, their hashing batched by the digest queue)
//   tools/bench_receiver files    <dir> <threads> <files_per_thread> <file_bytes>   (no hashing:
//                                 the file-system side of the receiver alone)
//   tools/bench_receiver copy     <dir> <threads> <uploads_per_thread> <upload_bytes>  (no hashing:
//                                 saveFile without the digests -- createFile with its .info, open,
//                                 io.Copy(f, body) in 32 KiB socket reads, fsync, close, the .info
//                                 removed: the receiver's host ceiling for the same PATCH)
//
// Every upload carries the same bytes, so every finished upload must report the digests of a
// reference upload made before the clock starts; each file is removed when its upload is done
// (the store keeps it; the benchmark bounds the space it needs to threads x upload_bytes).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <sys/resource.h>
#include <sys/statfs.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "../efes_amd/host/efes_receiver.hpp"
#include "cpu_quota.hpp"

using namespace efes;

namespace {

// An io.Reader over caller memory, at most `max_read` bytes per Read (a socket's reads).
struct SpanReader : Reader {
  const uint8_t* p;
  size_t n, pos = 0, max_read;
  SpanReader(const uint8_t* d, size_t len, size_t mr) : p(d), n(len), max_read(mr) {}
  size_t Read(uint8_t* dst, size_t cap, Error* err) override {
    *err = Error{};
    if (pos >= n) {
      *err = make_error(ERR_EOF, "EOF");
      return 0;
    }
    const size_t k = std::min(std::min(cap, max_read), n - pos);
    memcpy(dst, p + pos, k);
    pos += k;
    return k;
  }
};

// CPU seconds (user + system) of the whole process so far; *sys gets the system part.
double cpu_seconds(double* sys = nullptr) {
  struct rusage ru;
  getrusage(RUSAGE_SELF, &ru);
  if (sys) *sys = ru.ru_stime.tv_sec + 1e-6 * ru.ru_stime.tv_usec;
  return ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
}

uint64_t thread_cpu_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

std::vector<uint8_t> content(size_t n) {
  std::vector<uint8_t> v(n);
  uint64_t z = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < n; ++i) {
    z ^= z << 13; z ^= z >> 7; z ^= z << 17;
    v[i] = (uint8_t)z;
  }
  return v;
}

const char* fs_name(const std::string& dir) {
  struct statfs s;
  if (statfs(dir.c_str(), &s) != 0) return "unknown";
  return s.f_type == 0x01021994 ? "tmpfs" : "disk";
}

// One upload through ServeHTTP, PATCH by PATCH; returns the final response.
Response upload(FileReceiver& fr, const std::string& path, const std::vector<uint8_t>& src, size_t patch) {
  Response w;
  size_t off = 0;
  do {
    const size_t n = std::min(patch, src.size() - off);
    SpanReader body(src.data() + off, n, 32 << 10);
    Request r;
    r.Method = "PATCH";
    r.Path = path;
    r.Headers["efes-file-offset"] = std::to_string(off);
    r.Headers["efes-file-length"] = std::to_string(src.size());
    r.Body = &body;
    w = fr.ServeHTTP(r);
    if (w.Code != 200) return w;
    off += n;
  } while (off < src.size());
  return w;
}

// The destination server of a drain, without its storage: takes each PATCH body (the socket
// reads of the real transport), acknowledges the offset, and on the last PATCH answers the SHA-1
// the content must have (known from a reference read) -- so only the source side's hashing is timed.
struct SinkTransport : Transport {
  std::string sha1_hex;
  Response RoundTrip(const Request& r, Error* err) override {
    *err = Error{};
    Response w;
    if (r.Method == "HEAD") {  // no broken PATCHes here: the sink always has what was sent
      w.Headers["efes-file-offset"] = "0";
      return w;
    }
    int64_t off = 0, len = -1;
    (void)ParseInt(r.Headers.count("efes-file-offset") ? r.Headers.at("efes-file-offset") : "0", &off);
    if (r.Headers.count("efes-file-length")) (void)ParseInt(r.Headers.at("efes-file-length"), &len);
    uint8_t buf[32 << 10];
    int64_t n = 0;
    for (Error e; r.Body;) {
      n += (int64_t)r.Body->Read(buf, sizeof buf, &e);
      if (e) break;
    }
    if (off + n == len) {
      w.Headers["efes-file-sha1"] = sha1_hex;
      w.Headers["efes-file-crc32"] = "00000000";  // sendFile passes it through unchecked (write.go:112)
    }
    w.Headers["efes-file-offset"] = std::to_string(off + n);
    return w;
  }
};

}  // namespace

int main(int argc, char** argv) {
  const int pinned_cpus = pin_to_cpu_quota();  // see cpu_quota.hpp
  if (argc < 7 && !(argc >= 6 && (std::string(argv[1]) == "sha1file" || std::string(argv[1]) == "files" ||
                                  std::string(argv[1]) == "copy" || std::string(argv[1]) == "drain"))) {
    fprintf(stderr,
            "usage: %s receiver <dir> <threads> <uploads_per_thread> <upload_bytes> <patch_bytes>\n"
            "       %s sha1file <dir> <threads> <files_per_thread> <file_bytes>\n",
            argv[0], argv[0]);
    return 2;
  }
  const std::string mode = argv[1], dir = argv[2];
  const int T = atoi(argv[3]);
  const long U = atol(argv[4]);
  const size_t S = strtoull(argv[5], nullptr, 10);
  efes_ctx* ctx = nullptr;
  int rc = efes_ctx_create(0, &ctx);
  if (rc) {
    fprintf(stderr, "efes_ctx_create: %s\n", efes_strerror(rc));
    return 1;
  }
  const std::vector<uint8_t> src = content(S);
  std::atomic<int> bad{0}, errs{0};
  double secs = 0;
  std::string first;

  if (mode == "receiver") {
    const size_t P = strtoull(argv[6], nullptr, 10);
    const int G = argc > 7 ? atoi(argv[7]) : 1;
    std::vector<efes_ctx*> ctxs{ctx};
    for (int g = 1; g < G; ++g) {
      efes_ctx* c = nullptr;
      if ((rc = efes_ctx_create(g, &c))) {
        fprintf(stderr, "efes_ctx_create(%d): %s\n", g, efes_strerror(rc));
        return 1;
      }
      ctxs.push_back(c);
    }
    Hasher* h = nullptr;
    // staging: `per` chunks of 256 KiB per request thread (+64); EFES_BENCH_CHUNKS_PER_UPLOAD overrides
    const char* pe = getenv("EFES_BENCH_CHUNKS_PER_UPLOAD");
    const uint32_t per = pe && *pe ? (uint32_t)atoi(pe) : 8u;
    Error e = Hasher::Create(ctxs, 256 << 10, per * (uint32_t)T + 64, (uint32_t)T, &h);
    if (e) {
      fprintf(stderr, "Hasher::Create: %s\n", e.msg.c_str());
      return 1;
    }
    FileReceiver fr(dir, h);
    {  // the expected headers, from one upload before the clock
      Response w = upload(fr, "/bench/reference.fid", src, P);
      first = w.Headers["efes-file-sha1"] + w.Headers["efes-file-crc32"];
      if (w.Code != 200 || first.size() != 48) {
        fprintf(stderr, "reference upload: %d %s\n", w.Code, w.Body.c_str());
        return 1;
      }
      (void)deleteFile(JoinPath(dir, "/bench/reference.fid"));
    }
    const char* ph = getenv("EFES_RECEIVER_PHASES");
    const bool phases = ph && *ph == '1';
    const char* pclk = getenv("EFES_RECEIVER_PHASE_CLOCK");  // this tool's switch, not the library's
    EnableSavePhases(phases, pclk && !strcmp(pclk, "wall"));
    std::atomic<uint64_t> req_cpu_ns{0}, unlink_cpu_ns{0};
    double s0 = 0, s1 = 0;
    const double c0 = cpu_seconds(&s0);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        for (long u = 0; u < U; ++u) {
          const std::string path = "/bench/" + std::to_string(t) + "/" + std::to_string(u) + ".fid";
          Response w = upload(fr, path, src, P);
          if (w.Code != 200) {
            ++errs;
            fprintf(stderr, "%s: %d %s\n", path.c_str(), w.Code, w.Body.c_str());
            return;
          }
          if (w.Headers["efes-file-sha1"] + w.Headers["efes-file-crc32"] != first) ++bad;
          const uint64_t u0 = thread_cpu_ns();
          (void)deleteFile(JoinPath(dir, path));
          unlink_cpu_ns += thread_cpu_ns() - u0;
        }
        struct timespec ts;
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
        req_cpu_ns += (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
      });
    for (auto& x : th) x.join();
    secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double cpu_s = cpu_seconds(&s1) - c0;
    std::string phase_json;
    if (phases) {  // request-thread CPU seconds per GiB in each saveFile phase (the rest: outside saveFile)
      uint64_t ns[kPhases];
      SavePhaseTotals(ns);
      const double gib = (double)T * U * S / (1u << 30);
      phase_json = ", \"phase_cpu_s_per_gib\": {";
      for (int p = 0; p < kPhases; ++p) {
        char b[96];
        snprintf(b, sizeof b, "%s\"%s\": %.4f", p ? ", " : "", SavePhaseName(p), ns[p] * 1e-9 / gib);
        phase_json += b;
      }
      char b[96];
      snprintf(b, sizeof b, "}, \"request_threads_cpu_s_per_gib\": %.4f, \"unlink_cpu_s_per_gib\": %.4f",
               req_cpu_ns.load() * 1e-9 / gib, unlink_cpu_ns.load() * 1e-9 / gib);
      phase_json += b;
      const char* pc = getenv("EFES_RECEIVER_PHASE_CLOCK");
      snprintf(b, sizeof b, ", \"phase_clock\": \"%s\"", pc && !strcmp(pc, "wall") ? "wall" : "thread_cpu");
      phase_json += b;
      EnableSavePhases(false);
    }
    {  // launches of the batching queue(s): jobs per launch = uploads hashed side by side
      efes_queue_stats qs{};
      uint64_t launches = 0, jobs = 0;
      for (size_t g = 0; g < ctxs.size(); ++g)
        if (efes_queue_get_stats(h->queue(g), &qs) == EFES_OK) launches += qs.launches, jobs += qs.jobs;
      char b[128];
      snprintf(b, sizeof b, ", \"queue_launches\": %llu, \"jobs_per_launch\": %.1f", (unsigned long long)launches,
               launches ? (double)jobs / launches : 0.0);
      phase_json += b;
    }
    delete h;
    for (size_t g = 1; g < ctxs.size(); ++g) efes_ctx_destroy(ctxs[g]);
    printf("{\"workload\": \"receiver\", \"pinned_cpus\": %d, \"gpus\": %d, \"staging_chunks\": %u, \"threads\": %d, \"uploads\": %ld, \"upload_bytes\": %zu, \"patch_bytes\": %zu, "
           "\"read_bytes\": 32768, \"dir_fs\": \"%s\", \"seconds\": %.4f, \"value\": %.3f, \"unit\": \"GiB/s\", "
           "\"sum_sha1_crc32\": \"%s\", \"all_sums_equal\": %s, \"errors\": %d, \"cpu_s_per_gib\": %.4f, \"sys_share\": %.3f%s}\n",
           pinned_cpus, G, per * (uint32_t)T + 64, T, T * U, S, P, fs_name(dir), secs, (double)T * U * S / secs / (1u << 30), first.c_str(),
           bad ? "false" : "true", errs.load(), cpu_s / ((double)T * U * S / (1u << 30)), (s1 - s0) / cpu_s,
           phase_json.c_str());
  } else if (mode == "files") {
    // The file-system side of the receiver alone (no hashing): per upload, create + 32 KiB
    // writes + fsync + close + unlink, T threads -- the ceiling the receiver can reach here.
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        const std::string d = dir + "/files/" + std::to_string(t);
        if (system(("mkdir -p '" + d + "'").c_str()) != 0) {
          ++errs;
          return;
        }
        for (long u = 0; u < U; ++u) {
          const std::string path = d + "/" + std::to_string(u) + ".fid";
          FILE* f = fopen(path.c_str(), "wb");
          if (!f) {
            ++errs;
            return;
          }
          for (size_t a = 0; a < S; a += 32 << 10)
            if (fwrite(src.data() + a, 1, std::min<size_t>(32 << 10, S - a), f) == 0) ++errs;
          fflush(f);
          if (fsync(fileno(f)) != 0 || fclose(f) != 0) ++errs;
          unlink(path.c_str());
        }
      });
    for (auto& x : th) x.join();
    secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"workload\": \"files\", \"pinned_cpus\": %d, \"threads\": %d, \"files\": %ld, \"file_bytes\": %zu, \"dir_fs\": \"%s\", "
           "\"seconds\": %.4f, \"value\": %.3f, \"unit\": \"GiB/s\", \"errors\": %d}\n",
           pinned_cpus, T, T * U, S, fs_name(dir), secs, (double)T * U * S / secs / (1u << 30), errs.load());
  } else if (mode == "copy") {
    // saveFile without the digests (filereceiver.go:171-224 with MultiWriter(f) only), the file
    // work of the receiver's single-PATCH upload exactly: createFile (os.Create + Close + the
    // newFileInfo .info, :148-165 -- a PATCH at offset 0 makes it, :173-178), OpenFile(O_WRONLY),
    // io.Copy from the body (32 KiB reads into a buffer, one write each), fsync, close, and
    // DeleteFileInfo once offset == length (:220-223).
    std::atomic<uint64_t> copy_ph[5] = {};
    double s0 = 0, s1 = 0;
    const double c0 = cpu_seconds(&s0);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        const std::string d = dir + "/copy/" + std::to_string(t);
        if (system(("mkdir -p '" + d + "'").c_str()) != 0) {
          ++errs;
          return;
        }
        std::vector<uint8_t> buf(32 << 10);
        uint64_t ph[5] = {0, 0, 0, 0, 0}, t = thread_cpu_ns();
        auto mark = [&](int p) {
          const uint64_t now = thread_cpu_ns();
          ph[p] += now - t;
          t = now;
        };
        for (long u = 0; u < U; ++u) {
          const std::string path = d + "/" + std::to_string(u) + ".fid";
          if (createFile(path)) {
            ++errs;
            return;
          }
          mark(0);
          const int fd = ::open(path.c_str(), O_WRONLY | O_CLOEXEC);
          if (fd < 0) {
            ++errs;
            return;
          }
          SpanReader body(src.data(), S, 32 << 10);
          Error e;
          for (;;) {
            const size_t n = body.Read(buf.data(), buf.size(), &e);
            if (n && ::write(fd, buf.data(), n) != (ssize_t)n) ++errs;
            if (e) break;
          }
          mark(1);
          if (::fsync(fd) != 0 || ::close(fd) != 0) ++errs;
          mark(2);
          if (DeleteFileInfo(path)) ++errs;
          mark(3);
          unlink(path.c_str());
          mark(4);
        }
        for (int p = 0; p < 5; ++p) copy_ph[p] += ph[p];
      });
    for (auto& x : th) x.join();
    secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double cpu_s = cpu_seconds(&s1) - c0;
    printf("{\"workload\": \"copy\", \"pinned_cpus\": %d, \"threads\": %d, \"uploads\": %ld, \"upload_bytes\": %zu, "
           "\"read_bytes\": 32768, \"dir_fs\": \"%s\", \"seconds\": %.4f, \"value\": %.3f, \"unit\": \"GiB/s\", \"errors\": %d, "
           "\"cpu_s_per_gib\": %.4f, \"sys_share\": %.3f, \"phase_cpu_s_per_gib\": {\"create\": %.4f, "
           "\"read_write\": %.4f, \"sync_close\": %.4f, \"info\": %.4f, \"unlink\": %.4f}}\n",
           pinned_cpus, T, T * U, S, fs_name(dir), secs, (double)T * U * S / secs / (1u << 30), errs.load(),
           cpu_s / ((double)T * U * S / (1u << 30)), (s1 - s0) / cpu_s,
           copy_ph[0] * 1e-9 / ((double)T * U * S / (1u << 30)), copy_ph[1] * 1e-9 / ((double)T * U * S / (1u << 30)),
           copy_ph[2] * 1e-9 / ((double)T * U * S / (1u << 30)), copy_ph[3] * 1e-9 / ((double)T * U * S / (1u << 30)),
           copy_ph[4] * 1e-9 / ((double)T * U * S / (1u << 30)));
  } else if (mode == "sha1file") {
    // One source file read by every thread U times through Sha1File (32 KiB reads).
    const std::string path = dir + "/bench_sha1file.dat";
    FILE* f = fopen(path.c_str(), "wb");
    if (!f || fwrite(src.data(), 1, S, f) != S || fclose(f) != 0) {
      fprintf(stderr, "cannot write %s\n", path.c_str());
      return 1;
    }
    auto read_one = [&](std::string* hex) -> bool {
      FileReader* fr = nullptr;
      if (FileReader::Open(path, &fr)) return false;
      Sha1File* sf = nullptr;
      bool ok = !Sha1File::New(fr, ctx, &sf);
      std::vector<uint8_t> buf(32 << 10);
      Error e;
      while (ok) {
        sf->Read(buf.data(), buf.size(), &e);
        if (e.code == ERR_EOF) break;
        if (e) ok = false;
      }
      uint8_t d[20];
      if (ok) ok = !sf->Sum(d);
      if (ok) *hex = HexEncode(d, 20);
      delete sf;
      delete fr;
      return ok;
    };
    if (!read_one(&first)) {
      fprintf(stderr, "reference read failed\n");
      return 1;
    }
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&] {
        for (long u = 0; u < U; ++u) {
          std::string hx;
          if (!read_one(&hx)) ++errs;
          else if (hx != first) ++bad;
        }
      });
    for (auto& x : th) x.join();
    secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    unlink(path.c_str());
    printf("{\"workload\": \"sha1file\", \"pinned_cpus\": %d, \"threads\": %d, \"files\": %ld, \"file_bytes\": %zu, \"read_bytes\": 32768, "
           "\"dir_fs\": \"%s\", \"seconds\": %.4f, \"value\": %.3f, \"unit\": \"GiB/s\", \"sum_sha1\": \"%s\", "
           "\"all_sums_equal\": %s, \"errors\": %d}\n",
           pinned_cpus, T, T * U, S, fs_name(dir), secs, (double)T * U * S / secs / (1u << 30), first.c_str(), bad ? "false" : "true",
           errs.load());
  } else if (mode == "drain") {
    // Files 0..U-1 (written by the caller) moved by T workers, each taking the next fid.
    const long F = U, NF = argc > 6 ? std::max(1L, atol(argv[6])) : U;
    auto fid_path = [&](long i) { return dir + "/" + std::to_string(i % NF) + ".fid"; };
    SinkTransport sink;
    {  // the content's SHA-1 from one reference read (bench.py checks it against hashlib)
      FileReader* fr = nullptr;
      Sha1File* sf = nullptr;
      if (FileReader::Open(fid_path(0), &fr) || Sha1File::New(fr, ctx, &sf)) {
        fprintf(stderr, "cannot open %s\n", fid_path(0).c_str());
        return 1;
      }
      std::vector<uint8_t> buf(32 << 10);
      Error e;
      while (!e) sf->Read(buf.data(), buf.size(), &e);
      uint8_t d[20];
      if (e.code != ERR_EOF || sf->Sum(d)) {
        fprintf(stderr, "reference read failed\n");
        return 1;
      }
      sink.sha1_hex = first = HexEncode(d, 20);
      delete sf;
      delete fr;
    }
    ClientConfig cfg;
    cfg.Drainer = true;  // efes-drain: true (write.go:163-165)
    std::atomic<long> next{0};
    efes_pool* stats_pool = nullptr;  // only to read the digest queue's launch counters
    efes_queue_stats q0{}, q1{};
    if (efes_pool_create(&ctx, 1, &stats_pool) == EFES_OK) (void)efes_pool_stats(stats_pool, 0, &q0);
    double s0 = 0, s1 = 0;
    const double c0 = cpu_seconds(&s0);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&] {
        for (long i; (i = next++) < F;) {  // drain.go:87-101, one fid after the other per worker
          FileReader* fr = nullptr;
          if (FileReader::Open(fid_path(i), &fr)) {
            ++errs;
            continue;
          }
          Checksums cs;
          Error e = sendFile(sink, ctx, "/drain/" + std::to_string(i) + ".fid", *fr, (int64_t)S, cfg, &cs);
          if (e) {
            ++errs;
            fprintf(stderr, "fid %ld: %s\n", i, e.msg.c_str());
          } else if (cs.Sha1 != first) {
            ++bad;
          }
          delete fr;
        }
      });
    for (auto& x : th) x.join();
    secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double cpu_s = cpu_seconds(&s1) - c0, gib = (double)F * S / (1u << 30);
    if (stats_pool) (void)efes_pool_stats(stats_pool, 0, &q1);
    efes_pool_destroy(stats_pool);
    const uint64_t nl = q1.launches - q0.launches;
    printf("{\"workload\": \"drain\", \"pinned_cpus\": %d, \"workers\": %d, \"files\": %ld, \"file_bytes\": %zu, "
           "\"read_bytes\": 32768, \"dir_fs\": \"%s\", \"seconds\": %.4f, \"value\": %.3f, \"unit\": \"GiB/s\", "
           "\"sum_sha1\": \"%s\", \"all_sums_equal\": %s, \"errors\": %d, \"cpu_s_per_gib\": %.4f, \"sys_share\": %.3f, "
           "\"queue_launches\": %llu, \"jobs_per_launch\": %.1f}\n",
           pinned_cpus, T, F, S, fs_name(dir), secs, gib / secs, first.c_str(), bad ? "false" : "true", errs.load(),
           cpu_s / gib, cpu_s > 0 ? (s1 - s0) / cpu_s : 0.0, (unsigned long long)nl,
           nl ? (double)(q1.jobs - q0.jobs) / nl : 0.0);
  } else {
    fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  }
  efes_ctx_destroy(ctx);
  return errs || bad ? 1 : 0;
}
