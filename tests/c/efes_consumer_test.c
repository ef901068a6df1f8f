/*
 * efes_consumer_test.c -- the C ABI (include/efes_hash.h) driven the way the Go binding of
 * INTEGRATION.md would drive it, checked against the CPU oracle.  Test infrastructure: built by
 * __graft_entry__.build() (gcc, links libefeshash.so and oracle/liboracle.so), run by
 * tests/test_gpu_consumer.py on the GPU box.
 *
 *   patch   -- filereceiver.go:171-227 saveFile, per request goroutine: each PATCH reads the
 *              resumable state (.info JSON: ReadFileInfo -> UnmarshalText, fileinfo.go:29-45,
 *              sha1_efes.go:40-64, crc32_efes.go:26-40), streams the body through
 *              MultiWriter(f, CRC32, Sha1) in io.Copy's 32 KiB buffers (filereceiver.go:208-209),
 *              then either finalises (Sum -> efes-file-sha1 / efes-file-crc32 headers,
 *              filereceiver.go:99-100) or saves the state (MarshalText, filereceiver.go:226).
 *              T threads, each with its own uploads, PATCH sizes drawn like write.go:126's
 *              ChunkSize pieces plus ragged tails; every saved text and every final digest is
 *              compared with the oracle doing the same Writes.
 *   batch   -- efes_hash_submit[_mode] over device buffers from efes_device_alloc (the cgo
 *              path without an allocator of its own), every kernel shape.
 *   errors  -- errInvalidDigest and the Go panic states surface as error codes.
 * Prints one line "efes_consumer_test ok ..." and exits 0, or names the first mismatch.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/efes_hash.h"
#include "../../oracle/efes_oracle.h"

static efes_ctx* g_ctx;
static int g_fail;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

#define FAIL(...)                          \
  do {                                     \
    pthread_mutex_lock(&g_mu);             \
    if (!g_fail) {                         \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");               \
    }                                      \
    g_fail = 1;                            \
    pthread_mutex_unlock(&g_mu);           \
  } while (0)

static uint64_t rnd(uint64_t* s) { /* xorshift64* */
  *s ^= *s >> 12; *s ^= *s << 25; *s ^= *s >> 27;
  return *s * 0x2545F4914F6CDD1Dull;
}

/* ---- patch: concurrent resumable uploads ---------------------------------------------------- */
typedef struct {
  int id, uploads;
  long patches, bytes;
} patch_arg;

static void* patch_worker(void* p) {
  patch_arg* a = (patch_arg*)p;
  uint64_t s = 0x9E3779B97F4A7C15ull ^ (uint64_t)(a->id + 1) * 0xD1B54A32D192ED03ull;
  for (int u = 0; u < a->uploads && !g_fail; ++u) {
    const size_t len = (rnd(&s) % 4 == 0) ? rnd(&s) % 100 : rnd(&s) % (3u << 20);
    uint8_t* obj = malloc(len ? len : 1);
    oracle_fill_synthetic(obj, len, rnd(&s));
    char sha_text[201] = {0}, crc_text[9] = {0};  /* the .info state between PATCHes */
    oracle_sha1 o_sha;
    oracle_crc32 o_crc;
    memset(&o_sha, 0, sizeof o_sha);  /* NewSha1: a zero-value sha1digest, then Reset (sha1.go:48-52) */
    oracle_sha1_reset(&o_sha);
    oracle_crc32_reset(&o_crc);
    size_t off = 0;
    do {
      size_t n = (rnd(&s) % 3 == 0) ? rnd(&s) % 70000 : (size_t)(1 + rnd(&s) % (1u << 20));
      if (n > len - off) n = len - off;
      const int last = off + n == len;
      efes_sha1* sha = NULL;
      efes_crc32* crc = NULL;
      if (efes_sha1_new(g_ctx, &sha) || efes_crc32_new(g_ctx, &crc)) { FAIL("new"); break; }
      if (off > 0) {  /* ReadFileInfo (filereceiver.go:182) */
        if (efes_sha1_unmarshal_text(sha, sha_text, 200) || efes_crc32_unmarshal_text(crc, crc_text, 8)) {
          FAIL("unmarshal upload %d.%d", a->id, u);
          break;
        }
      }
      for (size_t q = 0; q < n; q += 32768) {  /* io.Copy(MultiWriter(f, CRC32, Sha1), body) */
        const size_t m = n - q < 32768 ? n - q : 32768;
        if (efes_crc32_write(crc, obj + off + q, m) || efes_sha1_write(sha, obj + off + q, m)) {
          FAIL("write upload %d.%d", a->id, u);
          break;
        }
        oracle_crc32_write(&o_crc, obj + off + q, m);
        oracle_sha1_write(&o_sha, obj + off + q, m);
      }
      off += n;
      a->patches++;
      if (last) {  /* filereceiver.go:99-100 */
        uint8_t d[20], e[20], c[4];
        if (efes_sha1_sum(sha, d) || efes_crc32_sum(crc, c)) FAIL("sum upload %d.%d", a->id, u);
        oracle_sha1_sum(&o_sha, e);
        const uint32_t oc = oracle_crc32_sum32(&o_crc);
        const uint8_t ec[4] = {(uint8_t)(oc >> 24), (uint8_t)(oc >> 16), (uint8_t)(oc >> 8), (uint8_t)oc};
        if (memcmp(d, e, 20)) FAIL("sha1 digest upload %d.%d len %zu", a->id, u, len);
        if (memcmp(c, ec, 4)) FAIL("crc32 digest upload %d.%d len %zu", a->id, u, len);
      } else {  /* SaveFileInfo (filereceiver.go:226) */
        char want_sha[200], want_crc[8];
        if (efes_sha1_marshal_text(sha, sha_text) || efes_crc32_marshal_text(crc, crc_text)) FAIL("marshal");
        oracle_sha1_marshal_text(&o_sha, want_sha);
        oracle_crc32_marshal_text(&o_crc, want_crc);
        if (memcmp(sha_text, want_sha, 200)) {
          char again[200];
          efes_sha1_marshal_text(sha, again);
          FAIL("sha1 MarshalText upload %d.%d at %zu (PATCH %zu bytes)\n got  %.200s\n want %.200s\n again %s",
               a->id, u, off, n, sha_text, want_sha, memcmp(again, sha_text, 200) ? "differs" : "same");
        }
        if (memcmp(crc_text, want_crc, 8)) FAIL("crc32 MarshalText upload %d.%d at %zu", a->id, u, off);
      }
      efes_sha1_free(sha);
      efes_crc32_free(crc);
    } while (off < len && !g_fail);
    a->bytes += (long)len;
    free(obj);
  }
  return NULL;
}

static int test_patch(int threads, int uploads) {
  pthread_t th[64];
  patch_arg args[64];
  long patches = 0, bytes = 0;
  for (int t = 0; t < threads; ++t) {
    args[t] = (patch_arg){t, uploads, 0, 0};
    pthread_create(&th[t], NULL, patch_worker, &args[t]);
  }
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    patches += args[t].patches;
    bytes += args[t].bytes;
  }
  printf("patch: %d threads x %d uploads, %ld PATCHes, %ld bytes\n", threads, uploads, patches, bytes);
  return !g_fail;
}

/* ---- batch: device-resident jobs, every kernel shape -------------------------------------- */
static int test_batch(void) {
  enum { N = 300 };
  uint64_t s = 12345;
  size_t off[N], len[N], total = 0;
  for (int i = 0; i < N; ++i) {
    total += rnd(&s) % 7;
    off[i] = total;
    len[i] = (i % 5 == 0) ? rnd(&s) % 130 : rnd(&s) % 200000;
    total += len[i];
  }
  uint8_t* host = malloc(total + 64);
  oracle_fill_synthetic(host, total + 64, 77);
  void *d_data = NULL, *d_jobs = NULL, *d_st = NULL, *d_crc = NULL, *d_sum = NULL, *d_status = NULL;
  int rc = efes_device_alloc(g_ctx, total + 64, &d_data);
  rc = rc ? rc : efes_device_alloc(g_ctx, sizeof(efes_job) * N, &d_jobs);
  rc = rc ? rc : efes_device_alloc(g_ctx, sizeof(efes_sha1_state) * N, &d_st);
  rc = rc ? rc : efes_device_alloc(g_ctx, 4 * N, &d_crc);
  rc = rc ? rc : efes_device_alloc(g_ctx, 24 * N, &d_sum);
  rc = rc ? rc : efes_device_alloc(g_ctx, 4 * N, &d_status);
  rc = rc ? rc : efes_copy_to_device(g_ctx, d_data, host, total + 64, NULL);
  if (rc) { FAIL("batch alloc/copy: %s", efes_strerror(rc)); return 0; }
  efes_job jobs[N];
  for (int i = 0; i < N; ++i) {
    jobs[i].data = (uint8_t*)d_data + off[i];
    jobs[i].length = len[i];
    jobs[i].sha1 = (efes_sha1_state*)d_st + i;
    jobs[i].crc32 = (efes_crc32_state*)d_crc + i;
    jobs[i].sum = (uint8_t*)d_sum + 24 * i;
    jobs[i].status = (int32_t*)d_status + i;
    jobs[i].flags = EFES_JOB_INIT | EFES_JOB_FINALIZE;
    jobs[i]._reserved = 0;
  }
  static const int modes[] = {EFES_MODE_AUTO, EFES_MODE_DEEP, EFES_MODE_WIDE, EFES_MODE_GROUP4, EFES_MODE_GROUP8,
                              EFES_MODE_GROUP16, EFES_MODE_GROUP32};
  uint8_t sums[24 * N];
  int32_t status[N];
  for (size_t m = 0; m < sizeof modes / sizeof modes[0] && !g_fail; ++m) {
    memset(sums, 0, sizeof sums);
    rc = efes_copy_to_device(g_ctx, d_sum, sums, sizeof sums, NULL);
    rc = rc ? rc : efes_copy_to_device(g_ctx, d_jobs, jobs, sizeof jobs, NULL);
    rc = rc ? rc : efes_hash_submit_mode(g_ctx, d_jobs, N, NULL, modes[m]);
    rc = rc ? rc : efes_sync(g_ctx, NULL);
    rc = rc ? rc : efes_copy_to_host(g_ctx, sums, d_sum, sizeof sums, NULL);
    rc = rc ? rc : efes_copy_to_host(g_ctx, status, d_status, sizeof status, NULL);
    if (rc) { FAIL("batch mode %d: %s", modes[m], efes_strerror(rc)); break; }
    for (int i = 0; i < N; ++i) {
      uint8_t e[20];
      uint32_t c;
      oracle_hash_message(host + off[i], len[i], 32768, e, &c);
      const uint8_t ec[4] = {(uint8_t)(c >> 24), (uint8_t)(c >> 16), (uint8_t)(c >> 8), (uint8_t)c};
      if (status[i] || memcmp(sums + 24 * i, e, 20) || memcmp(sums + 24 * i + 20, ec, 4)) {
        FAIL("batch mode %d job %d len %zu", modes[m], i, len[i]);
        break;
      }
    }
  }
  efes_device_free(g_ctx, d_data); efes_device_free(g_ctx, d_jobs); efes_device_free(g_ctx, d_st);
  efes_device_free(g_ctx, d_crc); efes_device_free(g_ctx, d_sum); efes_device_free(g_ctx, d_status);
  free(host);
  printf("batch: %d jobs x 7 shapes\n", N);
  return !g_fail;
}

/* ---- errors ------------------------------------------------------------------------------- */
static int test_errors(void) {
  efes_sha1* d = NULL;
  efes_crc32* c = NULL;
  if (efes_sha1_new(g_ctx, &d) || efes_crc32_new(g_ctx, &c)) { FAIL("new"); return 0; }
  char text[200];
  memset(text, 'z', sizeof text);
  if (efes_sha1_unmarshal_text(d, text, 200) != EFES_ERR_INVALID_DIGEST) FAIL("bad hex accepted");
  if (efes_sha1_unmarshal_text(d, text, 199) != EFES_ERR_INVALID_DIGEST) FAIL("bad length accepted");
  if (efes_crc32_unmarshal_text(c, "0000000", 7) != EFES_ERR_INVALID_DIGEST) FAIL("bad crc text accepted");
  efes_sha1_state st;
  efes_sha1_state_init(&st);
  memset(st.x, 0, sizeof st.x);
  st.nx = 65;  /* copy(d.x[d.nx:], p) panics (sha1.go:62) */
  efes_sha1_set_state(d, &st);
  if (efes_sha1_write(d, "x", 1) != EFES_ERR_STATE) FAIL("nx > 64 Write not EFES_ERR_STATE");
  st.nx = 3; st.len = 0;  /* checkSum's panic("d.nx != 0") (sha1.go:107-109) */
  efes_sha1_set_state(d, &st);
  uint8_t out[20];
  if (efes_sha1_sum(d, out) != EFES_ERR_STATE) FAIL("inconsistent state Sum not EFES_ERR_STATE");
  if (efes_sha1_marshal_text(d, text) != EFES_OK) FAIL("MarshalText after a failed Sum");
  efes_sha1_free(d);
  efes_crc32_free(c);
  printf("errors: ok\n");
  return !g_fail;
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 16;
  const int uploads = argc > 2 ? atoi(argv[2]) : 6;
  if (threads < 1 || threads > 64) return 2;
  int rc = efes_ctx_create(0, &g_ctx);
  if (rc) {
    fprintf(stderr, "efes_ctx_create: %s\n", efes_strerror(rc));
    return 1;
  }
  oracle_crc32_init_tables();
  int ok = test_errors() && test_batch() && test_patch(threads, uploads);
  efes_ctx_destroy(g_ctx);
  if (!ok) return 1;
  printf("efes_consumer_test ok\n");
  return 0;
}
