/*
 * patch_cpu.c -- the CPU baseline of bench.py's PATCH-latency leg (test infrastructure, like the rest
 * of oracle/: run only by bench.py as the reference-side figure, never part of the product).
 *
 * One PATCH's hashing as the reference runs it on the CPU: saveFile's io.Copy(MultiWriter(f, CRC32,
 * Sha1), body) (filereceiver.go:208-209) in 32 KiB buffers -- crc32digest.Write (crc32.go:76-86,
 * slicing-by-8) then sha1digest.Write (sha1.go:58-79, the generic block) of each -- then both Sums
 * (filereceiver.go:99-100), here the oracle's restatements.  T request threads (the uploads in
 * flight; net/http runs one goroutine per request) run PATCHes of S bytes back to back from memory
 * for about `seconds`, on as many CPUs as the cgroup's quota grants (GOMAXPROCS = the quota, as
 * INTEGRATION.md advises for the server), exactly like tools/bench_go_surface on the GPU path.
 *
 *   patch_cpu <threads> <patch_bytes> <seconds>   -> one JSON line (latency percentiles, GiB/s)
 */
#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "efes_oracle.h"

static size_t g_size;
static double g_seconds;
static uint8_t* g_src;
static uint8_t g_first[24];
static atomic_long g_bad, g_patches;
static double* g_lat;  /* per thread: up to kMaxPer latencies (ms) */
static long* g_nlat;
enum { kMaxPer = 4096 };

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void patch(uint8_t out[24]) {
  oracle_sha1 s;
  oracle_crc32 c;
  memset(&s, 0, sizeof s);
  oracle_sha1_reset(&s);  /* NewSha1 (sha1.go:48-52) */
  oracle_crc32_reset(&c); /* NewCRC32IEEE (crc32.go:68) */
  for (size_t a = 0; a < g_size; a += 32768) {
    const size_t m = g_size - a < 32768 ? g_size - a : 32768;
    oracle_crc32_write(&c, g_src + a, m);
    oracle_sha1_write(&s, g_src + a, m);
  }
  oracle_sha1_sum(&s, out);
  const uint32_t v = oracle_crc32_sum32(&c);
  out[20] = (uint8_t)(v >> 24); out[21] = (uint8_t)(v >> 16); out[22] = (uint8_t)(v >> 8); out[23] = (uint8_t)v;
}

static void* worker(void* arg) {
  const long t = (long)(intptr_t)arg;
  const double end = now() + g_seconds;
  long k = 0;
  do {
    const double a = now();
    uint8_t d[24];
    patch(d);
    if (memcmp(d, g_first, 24)) atomic_fetch_add(&g_bad, 1);
    if (k < kMaxPer) g_lat[t * kMaxPer + k] = 1e3 * (now() - a);
    ++k;
  } while (now() < end);
  g_nlat[t] = k < kMaxPer ? k : kMaxPer;
  atomic_fetch_add(&g_patches, k);
  return NULL;
}

static int cmp(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

/* Pins the process to as many CPUs as the cgroup quota grants (tools/cpu_quota.hpp, in C). */
static int pin_to_quota(void) {
  FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r");
  if (!f) return 0;
  char q[32] = {0};
  long period = 0;
  const int got = fscanf(f, "%31s %ld", q, &period);
  fclose(f);
  if (got != 2 || q[0] == 'm' || period <= 0) return 0;
  int want = (int)ceil(atof(q) / (double)period);
  if (want < 1) want = 1;
  cpu_set_t cur, pin;
  if (sched_getaffinity(0, sizeof cur, &cur) != 0 || CPU_COUNT(&cur) <= want) return 0;
  CPU_ZERO(&pin);
  int n = 0;
  for (int c = 0; c < CPU_SETSIZE && n < want; ++c)
    if (CPU_ISSET(c, &cur)) {
      CPU_SET(c, &pin);
      ++n;
    }
  return sched_setaffinity(0, sizeof pin, &pin) == 0 ? n : 0;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <threads> <patch_bytes> <seconds>\n", argv[0]);
    return 2;
  }
  const int pinned = pin_to_quota();
  const int T = atoi(argv[1]);
  g_size = strtoull(argv[2], NULL, 10);
  g_seconds = atof(argv[3]);
  if (T < 1 || g_size < 1) return 2;
  g_src = malloc(g_size);
  uint64_t z = 0x9E3779B97F4A7C15ull; /* the bytes tools/bench_go_surface hashes */
  for (size_t i = 0; i < g_size; ++i) {
    z ^= z << 13; z ^= z >> 7; z ^= z << 17;
    g_src[i] = (uint8_t)z;
  }
  oracle_crc32_init_tables();
  patch(g_first);
  g_lat = calloc((size_t)T * kMaxPer, sizeof *g_lat);
  g_nlat = calloc((size_t)T, sizeof *g_nlat);
  const double t0 = now();
  pthread_t* th = calloc((size_t)T, sizeof *th);
  for (long t = 0; t < T; ++t) pthread_create(&th[t], NULL, worker, (void*)(intptr_t)t);
  for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
  const double secs = now() - t0;
  long n = 0;
  for (int t = 0; t < T; ++t) {
    memmove(g_lat + n, g_lat + (size_t)t * kMaxPer, (size_t)g_nlat[t] * sizeof *g_lat);
    n += g_nlat[t];
  }
  qsort(g_lat, (size_t)n, sizeof *g_lat, cmp);
#define PCT(q) (n ? g_lat[(long)((q) * (double)(n - 1) + 0.5)] : 0.0)
  char hex[49];
  for (int k = 0; k < 24; ++k) sprintf(hex + 2 * k, "%02x", g_first[k]);
  printf("{\"workload\": \"patch_cpu\", \"pinned_cpus\": %d, \"threads\": %d, \"patch_bytes\": %zu, \"seconds\": %.3f, "
         "\"patches\": %ld, \"value\": %.3f, \"unit\": \"GiB/s\", \"patch_ms\": {\"p50\": %.3f, \"p90\": %.3f, "
         "\"p99\": %.3f, \"n\": %ld}, \"sum_sha1_crc32\": \"%s\", \"all_equal\": %s}\n",
         pinned, T, g_size, secs, atomic_load(&g_patches),
         (double)atomic_load(&g_patches) * (double)g_size / secs / (double)(1u << 30), PCT(0.5), PCT(0.9), PCT(0.99), n,
         hex, atomic_load(&g_bad) ? "false" : "true");
  return atomic_load(&g_bad) ? 1 : 0;
}
