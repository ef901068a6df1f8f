/*
 * drain_cpu.c -- the CPU baseline of bench.py's drain leg (test infrastructure, like the rest of
 * oracle/: run only by bench.py as the reference-side rate, never part of the product).
 *
 * The drainer's read-back as the reference runs it on the CPU: drain.go:87-125 moves fid after fid
 * through write.go:68-117 sendFile, whose Sha1File (sha1file.go:23-37) hashes every 32 KiB read
 * with sha1digest.Write -- here the oracle's restatement of sha1.go's generic block.  T threads
 * (one file in flight each) over the same files the GPU leg drains; the network side is left out
 * on both legs.
 *
 *   drain_cpu <dir> <threads> <fids> <file_bytes> <nfiles>   -> one JSON line
 * Files are <dir>/<fid % nfiles>.fid; every digest must equal the first.
 */
#include <fcntl.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "efes_oracle.h"

static const char* g_dir;
static long g_fids, g_nfiles;
static atomic_long g_next, g_bad, g_err;
static uint8_t g_first[20];

static int hash_file(long fid, uint8_t out[20]) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%ld.fid", g_dir, fid % g_nfiles);
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  static __thread uint8_t buf[32 << 10];
  oracle_sha1 d;
  oracle_sha1_reset(&d);
  for (;;) {
    const ssize_t n = read(fd, buf, sizeof buf);  /* io.Copy's 32 KiB reads through Sha1File */
    if (n < 0) {
      close(fd);
      return -1;
    }
    if (n == 0) break;
    oracle_sha1_write(&d, buf, (size_t)n);
  }
  close(fd);
  return oracle_sha1_sum(&d, out);
}

static void* worker(void* arg) {
  (void)arg;
  for (long i; (i = atomic_fetch_add(&g_next, 1)) < g_fids;) {
    uint8_t d[20];
    if (hash_file(i, d)) atomic_fetch_add(&g_err, 1);
    else if (memcmp(d, g_first, 20)) atomic_fetch_add(&g_bad, 1);
  }
  return NULL;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s <dir> <threads> <fids> <file_bytes> <nfiles>\n", argv[0]);
    return 2;
  }
  g_dir = argv[1];
  const int T = atoi(argv[2]);
  g_fids = atol(argv[3]);
  const long S = atol(argv[4]);
  g_nfiles = atol(argv[5]) > 0 ? atol(argv[5]) : 1;
  if (hash_file(0, g_first)) {
    fprintf(stderr, "cannot hash %s/0.fid\n", g_dir);
    return 1;
  }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  pthread_t* th = calloc((size_t)T, sizeof *th);
  for (int t = 0; t < T; ++t) pthread_create(&th[t], NULL, worker, NULL);
  for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th);
  const double secs = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  char hex[41];
  for (int k = 0; k < 20; ++k) sprintf(hex + 2 * k, "%02x", g_first[k]);
  printf("{\"workload\": \"drain_cpu\", \"threads\": %d, \"fids\": %ld, \"file_bytes\": %ld, \"seconds\": %.4f, "
         "\"value\": %.3f, \"unit\": \"GiB/s\", \"sum_sha1\": \"%s\", \"all_sums_equal\": %s, \"errors\": %ld}\n",
         T, g_fids, S, secs, (double)g_fids * (double)S / secs / (double)(1u << 30), hex,
         atomic_load(&g_bad) ? "false" : "true", atomic_load(&g_err));
  return atomic_load(&g_bad) || atomic_load(&g_err) ? 1 : 0;
}
