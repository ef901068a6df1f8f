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
 *   pairs   -- fused MultiWriter digest pairs (ABI 6) driven through every call pattern that splits
 *              them, from T threads, each sync point against the oracle.
 *   errors  -- errInvalidDigest and the Go panic states surface as error codes.
 *   enumerate <ordinals> -- go/hash_gpu.go pool()'s device loop over a given ordinal list (a failing
 *              ordinal in the middle stands in for a GPU whose context does not open): failures are
 *              reported and skipped, never the end of the loop; the contexts that opened form one
 *              efes_pool and the patch uploads run on pooled digests (efes_*_new_pool); every context
 *              of the pool, the one after the failure included, must hash.
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
static efes_pool* g_pool; /* enumerate: pooled digests (hash_gpu.go) instead of g_ctx's */
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
      const int rn = g_pool ? efes_sha1_new_pool(g_pool, &sha) || efes_crc32_new_pool(g_pool, &crc)
                            : efes_sha1_new(g_ctx, &sha) || efes_crc32_new(g_ctx, &crc);
      if (rn) { FAIL("new"); break; }
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

/* ---- pairs: MultiWriter digest pairs that diverge (efes_stream.cpp fused pairs, ABI 6) ------ */
/* Random scripts of Go-surface calls on one object's two digests, mostly the MultiWriter pattern
 * (CRC then SHA-1, same buffer) mixed with everything that splits a fused pair: one-digest Writes,
 * the buffer changed between the two Writes, other lengths, SHA-1 first, empty Writes, Writes larger
 * than a staging chunk, Reset / UnmarshalText of either, sync points in either order, a member freed
 * and replaced mid-stream.  Every sync point is compared with the oracle doing the same calls. */
typedef struct {
  efes_sha1* s;
  efes_crc32* c;
  oracle_sha1 os;
  oracle_crc32 oc;
} pair_obj;

static void pair_new(pair_obj* o, int fresh_oracle) {
  if (efes_sha1_new(g_ctx, &o->s) || efes_crc32_new(g_ctx, &o->c)) FAIL("pair new");
  if (fresh_oracle) {
    memset(&o->os, 0, sizeof o->os);
    oracle_sha1_reset(&o->os);
    oracle_crc32_reset(&o->oc);
  }
}

static void pair_check(pair_obj* o, int sha_first, const char* what, int id, int k) {
  char st[200], ct[8], ws[200], wc[8];
  int r1, r2;
  if (sha_first) {
    r1 = efes_sha1_marshal_text(o->s, st);
    r2 = efes_crc32_marshal_text(o->c, ct);
  } else {
    r2 = efes_crc32_marshal_text(o->c, ct);
    r1 = efes_sha1_marshal_text(o->s, st);
  }
  oracle_sha1_marshal_text(&o->os, ws);
  oracle_crc32_marshal_text(&o->oc, wc);
  if (r1 || r2 || memcmp(st, ws, 200) || memcmp(ct, wc, 8)) FAIL("pair %s thread %d step %d", what, id, k);
}

static void* pair_worker(void* p) {
  patch_arg* a = (patch_arg*)p;
  uint64_t s = 0xA0761D6478BD642Full ^ (uint64_t)(a->id + 1) * 0xE7037ED1A0B428DBull;
  enum { SIZE = 400000 };
  uint8_t* buf = malloc(SIZE);
  for (int u = 0; u < a->uploads && !g_fail; ++u) {
    oracle_fill_synthetic(buf, SIZE, rnd(&s));
    pair_obj o;
    pair_new(&o, 1);
    for (int k = 0; k < 20 && !g_fail; ++k) {
      static const size_t ns[] = {1, 55, 64, 4096, 32768, 32768, 40000, 65536};
      const size_t n = ns[rnd(&s) % 8], off = rnd(&s) % (SIZE - 170000);
      const uint8_t* q = buf + off;
      switch (rnd(&s) % 16) {
        case 0: case 1: case 2: case 3: case 4: /* MultiWriter(f, CRC32, Sha1) */
          efes_crc32_write(o.c, q, n); oracle_crc32_write(&o.oc, q, n);
          efes_sha1_write(o.s, q, n); oracle_sha1_write(&o.os, q, n);
          break;
        case 5: efes_crc32_write(o.c, q, n); oracle_crc32_write(&o.oc, q, n); break;
        case 6: efes_sha1_write(o.s, q, n); oracle_sha1_write(&o.os, q, n); break;
        case 7: { /* the buffer changes between the two Writes (same pointer, other bytes) */
          efes_crc32_write(o.c, q, n); oracle_crc32_write(&o.oc, q, n);
          buf[off + rnd(&s) % n] ^= 0x5a;
          efes_sha1_write(o.s, q, n); oracle_sha1_write(&o.os, q, n);
          break;
        }
        case 8: { /* another length */
          const size_t m = n > 2 ? n - 1 - rnd(&s) % 2 : 0;
          efes_crc32_write(o.c, q, n); oracle_crc32_write(&o.oc, q, n);
          efes_sha1_write(o.s, q, m); oracle_sha1_write(&o.os, q, m);
          break;
        }
        case 9: /* SHA-1 first, then an empty SHA-1 Write */
          efes_sha1_write(o.s, q, n); oracle_sha1_write(&o.os, q, n);
          efes_crc32_write(o.c, q, n); oracle_crc32_write(&o.oc, q, n);
          efes_sha1_write(o.s, q, 0); oracle_sha1_write(&o.os, q, 0);
          break;
        case 10: /* a Write larger than a staging chunk */
          efes_crc32_write(o.c, q, 100000 + n); oracle_crc32_write(&o.oc, q, 100000 + n);
          efes_sha1_write(o.s, q, 100000 + n); oracle_sha1_write(&o.os, q, 100000 + n);
          break;
        case 11: /* Reset of one member with the CRC's Write unconfirmed */
          efes_crc32_write(o.c, q, n); oracle_crc32_write(&o.oc, q, n);
          if (rnd(&s) & 1) { efes_crc32_reset(o.c); oracle_crc32_reset(&o.oc); }
          else { efes_sha1_reset(o.s); oracle_sha1_reset(&o.os); }
          efes_sha1_write(o.s, q, n); oracle_sha1_write(&o.os, q, n);
          break;
        case 12: { /* UnmarshalText of one member (a resumed PATCH) */
          char t[200];
          if (rnd(&s) & 1) {
            oracle_sha1 x; memset(&x, 0, sizeof x); oracle_sha1_reset(&x); oracle_sha1_write(&x, q, 1 + n % 150);
            oracle_sha1_marshal_text(&x, t);
            if (efes_sha1_unmarshal_text(o.s, t, 200) || oracle_sha1_unmarshal_text(&o.os, t, 200)) FAIL("pair unmarshal");
          } else {
            oracle_crc32 x; oracle_crc32_reset(&x); oracle_crc32_write(&x, q, 77);
            oracle_crc32_marshal_text(&x, t);
            if (efes_crc32_unmarshal_text(o.c, t, 8) || oracle_crc32_unmarshal_text(&o.oc, t, 8)) FAIL("pair unmarshal");
          }
          break;
        }
        case 13: pair_check(&o, (int)(rnd(&s) & 1), "text", a->id, k); break;
        case 14: { /* a member freed mid-stream (its finalizer) and replaced by one resumed from its text */
          efes_crc32_write(o.c, q, n); oracle_crc32_write(&o.oc, q, n);
          char t[200];
          if (rnd(&s) & 1) {
            if (efes_crc32_marshal_text(o.c, t)) FAIL("pair crc text");
            efes_crc32_free(o.c);
            if (efes_crc32_new(g_ctx, &o.c) || efes_crc32_unmarshal_text(o.c, t, 8)) FAIL("pair crc renew");
          } else {
            if (efes_sha1_marshal_text(o.s, t)) FAIL("pair sha text");
            efes_sha1_free(o.s);
            if (efes_sha1_new(g_ctx, &o.s) || efes_sha1_unmarshal_text(o.s, t, 200)) FAIL("pair sha renew");
          }
          efes_sha1_write(o.s, q, n); oracle_sha1_write(&o.os, q, n);
          break;
        }
        default: { /* Sums in either order */
          uint8_t d[20], e[20], c[4];
          const int sf = (int)(rnd(&s) & 1);
          int r = sf ? efes_sha1_sum(o.s, d) | efes_crc32_sum(o.c, c) : efes_crc32_sum(o.c, c) | efes_sha1_sum(o.s, d);
          const int orc = oracle_sha1_sum(&o.os, e);
          const uint32_t oc = oracle_crc32_sum32(&o.oc);
          const uint8_t ec[4] = {(uint8_t)(oc >> 24), (uint8_t)(oc >> 16), (uint8_t)(oc >> 8), (uint8_t)oc};
          if (orc == 0 && (r || memcmp(d, e, 20) || memcmp(c, ec, 4))) FAIL("pair sum thread %d step %d", a->id, k);
          break;
        }
      }
    }
    pair_check(&o, 1, "end", a->id, -1);
    efes_sha1_free(o.s);
    efes_crc32_free(o.c);
    a->patches++;
  }
  free(buf);
  return NULL;
}

static int test_pairs(int threads, int scripts) {
  pthread_t th[64];
  patch_arg args[64];
  efes_pair_stats p0, p1;
  efes_pair_stats_get(&p0);
  for (int t = 0; t < threads; ++t) {
    args[t] = (patch_arg){t, scripts, 0, 0};
    pthread_create(&th[t], NULL, pair_worker, &args[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  efes_pair_stats_get(&p1);
  printf("pairs: %d threads x %d scripts, %llu pairs bound, %llu settled\n", threads, scripts,
         (unsigned long long)(p1.pairs - p0.pairs), (unsigned long long)(p1.settles - p0.settles));
  if (p1.pairs == p0.pairs || p1.settles == p0.settles) FAIL("pairs: no pair bound or settled");
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

/* ---- enumerate: go/hash_gpu.go pool() -------------------------------------------------------- */
static int test_enumerate(const char* list, int threads, int uploads) {
  enum { MAXC = 16 };
  efes_ctx* ctxs[MAXC];
  int devs[MAXC], opened = 0, listed = 0, skipped = 0;
  const int visible = efes_device_count();
  for (const char* p = list; *p && opened < MAXC;) {
    char* end;
    const int dev = (int)strtol(p, &end, 10);
    if (end == p) break;
    p = *end == ',' ? end + 1 : end;
    ++listed;
    efes_ctx* c = NULL;
    const int rc = efes_ctx_create(dev, &c);
    if (rc != EFES_OK) { /* hash_gpu.go: log, count, and go on with the next GPU */
      printf("enumerate: device %d skipped: %s\n", dev, efes_strerror(rc));
      if (c) FAIL("efes_ctx_create failed but returned a context");
      ++skipped;
      continue;
    }
    ctxs[opened] = c;
    devs[opened++] = dev;
  }
  if (!opened || !skipped) {
    FAIL("enumerate: %d opened, %d skipped of %d listed (want both)", opened, skipped, listed);
    return 0;
  }
  int rc = efes_pool_create(ctxs, (uint32_t)opened, &g_pool);
  if (rc) { FAIL("efes_pool_create: %s", efes_strerror(rc)); return 0; }
  const int ok = test_patch(threads, uploads);
  printf("enumerate: visible %d, listed %d, opened %d, skipped %d; jobs per context:", visible, listed, opened,
         skipped);
  for (int i = 0; i < opened; ++i) {
    efes_queue_stats st;
    if (efes_pool_stats(g_pool, (uint32_t)i, &st)) FAIL("efes_pool_stats %d", i);
    printf(" %d:%llu", devs[i], (unsigned long long)st.jobs);
    if (ok && st.jobs == 0) FAIL("context %d (device %d) of the pool hashed nothing", i, devs[i]);
  }
  printf("\n");
  efes_pool_destroy(g_pool);
  g_pool = NULL;
  for (int i = 0; i < opened; ++i) efes_ctx_destroy(ctxs[i]);
  return !g_fail;
}

int main(int argc, char** argv) {
  if (argc > 2 && !strcmp(argv[1], "enumerate")) {
    oracle_crc32_init_tables();
    const int ok = test_enumerate(argv[2], argc > 3 ? atoi(argv[3]) : 16, argc > 4 ? atoi(argv[4]) : 4);
    if (!ok) return 1;
    printf("efes_consumer_test ok (enumerate)\n");
    return 0;
  }
  const int threads = argc > 1 ? atoi(argv[1]) : 16;
  const int uploads = argc > 2 ? atoi(argv[2]) : 6;
  if (threads < 1 || threads > 64) return 2;
  int rc = efes_ctx_create(0, &g_ctx);
  if (rc) {
    fprintf(stderr, "efes_ctx_create: %s\n", efes_strerror(rc));
    return 1;
  }
  oracle_crc32_init_tables();
  int ok = test_errors() && test_batch() && test_patch(threads, uploads) && test_pairs(threads, uploads);
  efes_ctx_destroy(g_ctx);
  if (!ok) return 1;
  printf("efes_consumer_test ok\n");
  return 0;
}
