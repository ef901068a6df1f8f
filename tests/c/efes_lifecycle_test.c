/*
 * efes_lifecycle_test.c -- the object lifecycle of INTEGRATION.md §2's Go binding (hash_gpu.go),
 * replayed through the C ABI and built with AddressSanitizer on the host code (tools/asan_build.sh:
 * the library's host side and this program; device code untouched).  Test infrastructure, run by
 * tests/test_gpu_lifecycle.py on the GPU box.
 *
 * A Go digest is a struct owning one C handle; Go frees it only through its finalizer, which the
 * garbage collector runs on its own goroutine some time after the object became unreachable.  Here a
 * `go_sha1` / `go_crc32` is a heap struct holding the handle, and a "collector" thread runs the
 * finalizers (efes_*_free, then free of the struct) of dropped objects after a random delay,
 * concurrently with the request threads -- as Go's finalizer goroutine does.
 *
 *   fixed  -- the binding as INTEGRATION.md writes it now.  Per request thread and upload, PATCH by
 *             PATCH as filereceiver.go:171-227 runs them:
 *               PATCH 0  newFileInfo (fileinfo.go:20-27): NewSha1 / NewCRC32IEEE (open, in place);
 *               PATCH k  ReadExistingFileInfo (fileinfo.go:43): encoding/json allocates a ZERO
 *                        digest (handle nil) for each nil field and calls UnmarshalText on it, whose
 *                        handle() opens the handle in that object;
 *               32 KiB MultiWriter Writes (filereceiver.go:208-209); Sum on the last PATCH
 *               (:99-100), else MarshalText (:226); the FileInfo is then garbage: both digests go
 *               to the collector, which frees them while the next PATCH's digests are in use.
 *             Also `var d sha1digest` (sha1_efes_test.go): a zero value used directly.  Every text
 *             and digest is compared with the oracle; AddressSanitizer must stay silent.
 *   old    -- round 4's binding: UnmarshalText's nil branch did `*d = *newSha1Handle(true)`, copying
 *             the handle out of a temporary whose finalizer then freed it.  The next call on d uses
 *             freed memory; under AddressSanitizer this mode must die with heap-use-after-free
 *             (the negative control: the test can see the bug it guards against).
 */
#define _DEFAULT_SOURCE /* usleep */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../../include/efes_hash.h"
#include "../../oracle/efes_oracle.h"

static efes_pool* g_pool;
static int g_fail;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

#define FAIL(...)                            \
  do {                                       \
    pthread_mutex_lock(&g_mu);               \
    if (!g_fail) {                           \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");                 \
    }                                        \
    g_fail = 1;                              \
    pthread_mutex_unlock(&g_mu);             \
  } while (0)

static uint64_t rnd(uint64_t* s) { /* xorshift64* */
  *s ^= *s >> 12; *s ^= *s << 25; *s ^= *s >> 27;
  return *s * 0x2545F4914F6CDD1Dull;
}

/* ---- the Go objects ------------------------------------------------------------------------ */
typedef struct { efes_sha1* c; } go_sha1;   /* type sha1digest struct{ c *C.efes_sha1 } */
typedef struct { efes_crc32* c; } go_crc32; /* type crc32digest struct{ c *C.efes_crc32 } */

static void sha_open(go_sha1* d, int zero) { /* (*sha1digest).open */
  if ((zero ? efes_sha1_new_zero_pool(g_pool, &d->c) : efes_sha1_new_pool(g_pool, &d->c)) != EFES_OK) FAIL("sha open");
}
static efes_sha1* sha_handle(go_sha1* d) { /* (*sha1digest).handle */
  if (!d->c) sha_open(d, 1);
  return d->c;
}
static void crc_open(go_crc32* d) {
  if (efes_crc32_new_pool(g_pool, &d->c) != EFES_OK) FAIL("crc open");
}
static efes_crc32* crc_handle(go_crc32* d) {
  if (!d->c) crc_open(d);
  return d->c;
}

/* ---- the collector: finalizers of unreachable objects, on a thread of their own ----------- */
typedef struct garbage {
  struct garbage* next;
  go_sha1* s;
  go_crc32* c;
} garbage;
static garbage* g_heap;
static int g_done;
static pthread_mutex_t g_gc_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_gc_cv = PTHREAD_COND_INITIALIZER;
static long g_finalized;

static void drop(go_sha1* s, go_crc32* c) { /* the object became unreachable */
  garbage* g = malloc(sizeof *g);
  g->s = s;
  g->c = c;
  pthread_mutex_lock(&g_gc_mu);
  g->next = g_heap;
  g_heap = g;
  pthread_cond_signal(&g_gc_cv);
  pthread_mutex_unlock(&g_gc_mu);
}

static void finalize(garbage* g) { /* runtime.SetFinalizer(d, (*sha1digest).free) etc. */
  if (g->s) {
    efes_sha1_free(g->s->c);
    free(g->s);
  }
  if (g->c) {
    efes_crc32_free(g->c->c);
    free(g->c);
  }
  free(g);
}

static void* collector(void* arg) {
  uint64_t s = 0xC011EC7ull;
  (void)arg;
  pthread_mutex_lock(&g_gc_mu);
  for (;;) {
    while (!g_heap && !g_done) pthread_cond_wait(&g_gc_cv, &g_gc_mu);
    if (!g_heap && g_done) break;
    garbage* g = g_heap;
    g_heap = g->next;
    pthread_mutex_unlock(&g_gc_mu);
    usleep((useconds_t)(rnd(&s) % 300)); /* some time after it became unreachable */
    finalize(g);
    pthread_mutex_lock(&g_gc_mu);
    ++g_finalized;
  }
  pthread_mutex_unlock(&g_gc_mu);
  return NULL;
}

/* ---- fixed: request threads --------------------------------------------------------------- */
typedef struct {
  int id, uploads, patches;
  long done;
} req_arg;

static void* request_thread(void* p) {
  req_arg* a = (req_arg*)p;
  uint64_t s = 0x51F7ull + (uint64_t)a->id * 0x9E3779B97F4A7C15ull;
  for (int u = 0; u < a->uploads && !g_fail; ++u) {
    const size_t len = 1 + rnd(&s) % (2u << 20);
    uint8_t* obj = malloc(len);
    oracle_fill_synthetic(obj, len, rnd(&s));
    oracle_sha1 os;
    oracle_crc32 oc;
    memset(&os, 0, sizeof os);
    oracle_sha1_reset(&os);
    oracle_crc32_reset(&oc);
    char sha_text[200], crc_text[8];
    for (int k = 0; k < a->patches && !g_fail; ++k) {
      const size_t from = len * (size_t)k / (size_t)a->patches, to = len * (size_t)(k + 1) / (size_t)a->patches;
      go_sha1* sd = calloc(1, sizeof *sd);
      go_crc32* cd = calloc(1, sizeof *cd);
      if (k == 0) { /* newFileInfo */
        sha_open(sd, 0);
        crc_open(cd);
      } else { /* json: zero objects, UnmarshalText on each (handle() opens it in place) */
        if (efes_sha1_unmarshal_text(sha_handle(sd), sha_text, 200) != EFES_OK ||
            efes_crc32_unmarshal_text(crc_handle(cd), crc_text, 8) != EFES_OK)
          FAIL("unmarshal %d.%d.%d", a->id, u, k);
      }
      for (size_t q = from; q < to; q += 32768) { /* io.Copy(MultiWriter(f, CRC32, Sha1), body) */
        const size_t m = to - q < 32768 ? to - q : 32768;
        if (efes_crc32_write(crc_handle(cd), obj + q, m) != EFES_OK || efes_sha1_write(sha_handle(sd), obj + q, m) != EFES_OK)
          FAIL("write %d.%d.%d", a->id, u, k);
        oracle_crc32_write(&oc, obj + q, m);
        oracle_sha1_write(&os, obj + q, m);
      }
      if (k == a->patches - 1) { /* filereceiver.go:99-100 */
        uint8_t d[20], e[20], c[4];
        if (efes_sha1_sum(sha_handle(sd), d) != EFES_OK || efes_crc32_sum(crc_handle(cd), c) != EFES_OK) FAIL("sum");
        oracle_sha1_sum(&os, e);
        const uint32_t x = oracle_crc32_sum32(&oc);
        const uint8_t ec[4] = {(uint8_t)(x >> 24), (uint8_t)(x >> 16), (uint8_t)(x >> 8), (uint8_t)x};
        if (memcmp(d, e, 20) || memcmp(c, ec, 4)) FAIL("digest %d.%d len %zu", a->id, u, len);
      } else { /* SaveFileInfo */
        char ws[200], wc[8];
        if (efes_sha1_marshal_text(sha_handle(sd), sha_text) != EFES_OK ||
            efes_crc32_marshal_text(crc_handle(cd), crc_text) != EFES_OK)
          FAIL("marshal");
        oracle_sha1_marshal_text(&os, ws);
        oracle_crc32_marshal_text(&oc, wc);
        if (memcmp(sha_text, ws, 200) || memcmp(crc_text, wc, 8)) FAIL("text %d.%d.%d", a->id, u, k);
      }
      drop(sd, cd); /* the PATCH's FileInfo is garbage now */
      a->done++;
    }
    free(obj);
  }
  return NULL;
}

static int zero_value(void) { /* sha1_efes_test.go: var d sha1digest; d.Write; Sum; MarshalText; var d2 */
  static const char msg[] = "hello world";
  go_sha1 d = {NULL}, d2 = {NULL};
  uint8_t h1[20], h2[20], e[20];
  char text[200];
  int ok = efes_sha1_write(sha_handle(&d), msg, 11) == EFES_OK && efes_sha1_sum(sha_handle(&d), h1) == EFES_OK &&
           efes_sha1_marshal_text(sha_handle(&d), text) == EFES_OK &&
           efes_sha1_unmarshal_text(sha_handle(&d2), text, 200) == EFES_OK && efes_sha1_sum(sha_handle(&d2), h2) == EFES_OK;
  oracle_sha1 o;
  memset(&o, 0, sizeof o); /* the zero value: h all zero, not NewSha1's IV */
  oracle_sha1_write(&o, (const uint8_t*)msg, 11);
  oracle_sha1_sum(&o, e);
  efes_sha1_free(d.c);
  efes_sha1_free(d2.c);
  if (!ok || memcmp(h1, h2, 20) || memcmp(h1, e, 20)) {
    FAIL("zero value");
    return 0;
  }
  return 1;
}

/* ---- old: round 4's nil branch, the use-after-free ---------------------------------------- */
static int old_binding(void) {
  go_sha1* tmp = calloc(1, sizeof *tmp); /* newSha1Handle(true): a temporary with the finalizer */
  sha_open(tmp, 1);
  go_sha1* d = calloc(1, sizeof *d); /* json's new(sha1digest) */
  *d = *tmp;                         /* *d = *newSha1Handle(true): the handle copied out */
  drop(tmp, NULL);                   /* the temporary is garbage at once ... */
  for (;;) {                         /* ... and its finalizer frees the handle d still uses */
    pthread_mutex_lock(&g_gc_mu);
    const long n = g_finalized;
    pthread_mutex_unlock(&g_gc_mu);
    if (n) break;
    usleep(100);
  }
  char text[200];
  oracle_sha1 o;
  memset(&o, 0, sizeof o);
  oracle_sha1_reset(&o);
  oracle_sha1_marshal_text(&o, text);
  const int rc = efes_sha1_unmarshal_text(d->c, text, 200); /* heap-use-after-free under ASan */
  fprintf(stderr, "old binding: UnmarshalText on the freed handle returned %d (no sanitizer report?)\n", rc);
  return 0;
}

int main(int argc, char** argv) {
  const int old = argc > 1 && !strcmp(argv[1], "old");
  const int threads = argc > 2 ? atoi(argv[2]) : 8;
  const int uploads = argc > 3 ? atoi(argv[3]) : 3;
  if (threads < 1 || threads > 64) return 2;
  efes_ctx* ctx = NULL;
  int rc = efes_ctx_create(0, &ctx);
  if (rc == EFES_OK) rc = efes_pool_create(&ctx, 1, &g_pool);
  if (rc) {
    fprintf(stderr, "setup: %s\n", efes_strerror(rc));
    return 1;
  }
  oracle_crc32_init_tables();
  pthread_t gc;
  pthread_create(&gc, NULL, collector, NULL);
  int ok;
  long patches = 0;
  if (old) {
    ok = old_binding();
  } else {
    pthread_t th[64];
    req_arg args[64];
    for (int t = 0; t < threads; ++t) {
      args[t] = (req_arg){t, uploads, 4, 0};
      pthread_create(&th[t], NULL, request_thread, &args[t]);
    }
    for (int t = 0; t < threads; ++t) {
      pthread_join(th[t], NULL);
      patches += args[t].done;
    }
    ok = !g_fail && zero_value();
  }
  pthread_mutex_lock(&g_gc_mu);
  g_done = 1;
  pthread_cond_signal(&g_gc_cv);
  pthread_mutex_unlock(&g_gc_mu);
  pthread_join(gc, NULL);
  efes_pool_destroy(g_pool);
  efes_ctx_destroy(ctx);
  if (!ok || g_fail) return 1;
  printf("efes_lifecycle_test ok: %d threads, %ld PATCHes, %ld objects finalized on the collector thread\n", threads,
         patches, g_finalized);
  return 0;
}
