/*
 * receiver_cpu.c -- the CPU baseline of bench.py's receiver leg (test infrastructure, like the rest
 * of oracle/: run only by bench.py as the reference-side rate, never part of the product).
 *
 * The reference's saveFile (filereceiver.go:171-227) for a one-PATCH upload, with its digests on
 * the CPU port (the oracle's restatement of sha1.go's generic block and crc32.go's slicing-by-8):
 * createFile (os.Create + Close + the newFileInfo .info, :148-165), OpenFile, io.Copy from the body
 * in 32 KiB reads through MultiWriter(f, CRC32, Sha1) (:208-209), f.Sync, Close, Sum of both
 * digests (:99-100) and DeleteFileInfo (:220-223); then the file is removed (the benchmark bounds
 * its space; bench_receiver does the same).  T threads, each one request at a time.
 *
 *   receiver_cpu <dir> <threads> <uploads_per_thread> <upload_bytes>   -> one JSON line
 * The body is the xorshift64 stream of tools/bench_receiver.cpp; every Sum must equal the first.
 */
#include <fcntl.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "efes_oracle.h"

static const char* g_dir;
static long g_uploads;
static size_t g_bytes;
static uint8_t* g_src;
static uint8_t g_first[24];
static atomic_long g_bad, g_err;

/* fileinfo.go:47-58 json.NewEncoder(f).Encode(newFileInfo()): the fresh digests' texts */
static int save_info(const char* path) {
  oracle_sha1 s;
  oracle_crc32 c;
  oracle_sha1_reset(&s);
  oracle_crc32_reset(&c);
  char st[201], ct[9], buf[512];
  oracle_sha1_marshal_text(&s, st);
  oracle_crc32_marshal_text(&c, ct);
  st[200] = ct[8] = 0;
  const int n = snprintf(buf, sizeof buf, "{\"offset\":0,\"digest\":{\"sha1\":\"%s\",\"crc32\":\"%s\"}}\n", st, ct);
  char ip[4200];
  snprintf(ip, sizeof ip, "%s.info", path);
  const int fd = open(ip, O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
  if (fd < 0) return -1;
  const int ok = write(fd, buf, (size_t)n) == n;
  return close(fd) == 0 && ok ? 0 : -1;
}

static int upload(const char* path, uint8_t out[24]) {
  int fd = open(path, O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0666); /* createFile */
  if (fd < 0 || close(fd) != 0 || save_info(path)) return -1;
  fd = open(path, O_WRONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  oracle_sha1 s;
  oracle_crc32 c;
  oracle_sha1_reset(&s);
  oracle_crc32_reset(&c);
  static __thread uint8_t buf[32 << 10];
  for (size_t off = 0; off < g_bytes;) { /* io.Copy: socket read, then MultiWriter(f, CRC32, Sha1) */
    const size_t n = g_bytes - off < sizeof buf ? g_bytes - off : sizeof buf;
    memcpy(buf, g_src + off, n);
    if (write(fd, buf, n) != (ssize_t)n) {
      close(fd);
      return -1;
    }
    oracle_crc32_write(&c, buf, n);
    oracle_sha1_write(&s, buf, n);
    off += n;
  }
  if (fsync(fd) != 0 || close(fd) != 0) return -1;
  if (oracle_sha1_sum(&s, out)) return -1;
  const uint32_t v = oracle_crc32_sum32(&c);
  out[20] = (uint8_t)(v >> 24); out[21] = (uint8_t)(v >> 16); out[22] = (uint8_t)(v >> 8); out[23] = (uint8_t)v;
  char ip[4200];
  snprintf(ip, sizeof ip, "%s.info", path); /* DeleteFileInfo */
  return unlink(ip);
}

static void* worker(void* arg) {
  const long t = (long)(intptr_t)arg;
  char d[4096];
  snprintf(d, sizeof d, "%s/cpu/%ld", g_dir, t);
  char cmd[4200];
  snprintf(cmd, sizeof cmd, "mkdir -p '%s'", d);
  if (system(cmd) != 0) {
    atomic_fetch_add(&g_err, 1);
    return NULL;
  }
  for (long u = 0; u < g_uploads; ++u) {
    char p[4200];
    snprintf(p, sizeof p, "%s/%ld.fid", d, u);
    uint8_t out[24];
    if (upload(p, out)) atomic_fetch_add(&g_err, 1);
    else if (memcmp(out, g_first, 24)) atomic_fetch_add(&g_bad, 1);
    unlink(p);
  }
  return NULL;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s <dir> <threads> <uploads_per_thread> <upload_bytes>\n", argv[0]);
    return 2;
  }
  g_dir = argv[1];
  const int T = atoi(argv[2]);
  g_uploads = atol(argv[3]);
  g_bytes = (size_t)atol(argv[4]);
  g_src = malloc(g_bytes ? g_bytes : 1);
  uint64_t z = 0x9E3779B97F4A7C15ull; /* tools/bench_receiver.cpp content() */
  for (size_t i = 0; i < g_bytes; ++i) {
    z ^= z << 13; z ^= z >> 7; z ^= z << 17;
    g_src[i] = (uint8_t)z;
  }
  char ref[4200];
  snprintf(ref, sizeof ref, "%s/cpu_reference.fid", g_dir);
  if (upload(ref, g_first)) {
    fprintf(stderr, "reference upload failed\n");
    return 1;
  }
  unlink(ref);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  pthread_t* th = calloc((size_t)T, sizeof *th);
  for (long t = 0; t < T; ++t) pthread_create(&th[t], NULL, worker, (void*)(intptr_t)t);
  for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th);
  const double secs = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  char hex[49];
  for (int k = 0; k < 24; ++k) sprintf(hex + 2 * k, "%02x", g_first[k]);
  printf("{\"workload\": \"receiver_cpu\", \"threads\": %d, \"uploads\": %ld, \"upload_bytes\": %zu, \"seconds\": %.4f, "
         "\"value\": %.3f, \"unit\": \"GiB/s\", \"sum_sha1_crc32\": \"%s\", \"all_sums_equal\": %s, \"errors\": %ld}\n",
         T, (long)T * g_uploads, g_bytes, secs, (double)T * (double)g_uploads * (double)g_bytes / secs / (double)(1u << 30),
         hex, atomic_load(&g_bad) ? "false" : "true", atomic_load(&g_err));
  free(g_src);
  return atomic_load(&g_bad) || atomic_load(&g_err) ? 1 : 0;
}
