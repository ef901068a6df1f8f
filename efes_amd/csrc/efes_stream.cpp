// efes_stream.cpp -- the Go-surface streaming digests (layer 2 of efes_hash.h) on top of the
// upload dispatcher (efes_queue.cpp).
//
// sha1digest (sha1.go:29-120, sha1_efes.go:25-64) and crc32digest (crc32.go:48-93,
// crc32_efes.go:18-40) keep their method sets; each object is an efes_upload of the context's
// shared queue that keeps only its own hash (EFES_HASH_SHA1 or EFES_HASH_CRC32).  So the Go
// code of filereceiver.go -- io.MultiWriter(f, CRC32, Sha1) in every request goroutine --
// drops in unchanged and still gets batched launches across all concurrent requests: a Write
// stages into pinned memory and returns; Sum / MarshalText are the sync points.
//
// An object opens its upload on first use and reopens it when its state is replaced
// (UnmarshalText, Reset), so idle digests hold no queue resources.  Go's Reset leaves x as it
// is (sha1.go:36-44): the reopened state keeps the replayed tail bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <new>

#include "efes_internal.hpp"

namespace {

// Shared queue sizing: EFES_DIGEST_STAGING_MIB of pinned staging in 64 KiB chunks (default
// 256 MiB = 4096 chunks, so up to 4095 digests hold a chunk at once).
efes_queue* create_digest_queue(efes_ctx* ctx, int* rc) {
  uint64_t mib = 256;
  if (const char* e = getenv("EFES_DIGEST_STAGING_MIB")) mib = strtoull(e, nullptr, 10);
  if (mib < 1) mib = 1;
  const uint64_t chunk = 64 << 10;
  const uint32_t chunks = (uint32_t)((mib << 20) / chunk) < 16 ? 16u : (uint32_t)((mib << 20) / chunk);
  efes_queue* q = nullptr;
  *rc = efes_queue_create(ctx, chunk, chunks, chunks - 1, &q);
  return *rc == EFES_OK ? q : nullptr;
}

}  // namespace

efes_queue* efes::stream_queue(efes_ctx* ctx, int* rc) {
  std::lock_guard<std::mutex> lk(ctx->mu);
  *rc = EFES_OK;
  if (!ctx->digests) ctx->digests = create_digest_queue(ctx, rc);
  return ctx->digests;
}

struct efes_sha1 {
  efes_ctx* ctx = nullptr;
  efes_upload* u = nullptr;  // opened on first use
  efes_sha1_state base{};    // the state the upload (re)opens with
  int latched = EFES_OK;     // Go would have panicked: every later call reports it
};

struct efes_crc32 {
  efes_ctx* ctx = nullptr;
  efes_upload* u = nullptr;
  efes_crc32_state base{};
  int latched = EFES_OK;
};

namespace {

template <class D>
int ensure_open(D* d, uint32_t hashes, const efes_sha1_state* sha1, const efes_crc32_state* crc) {
  if (d->latched) return d->latched;
  if (d->u) return EFES_OK;
  int rc = EFES_OK;
  efes_queue* q = efes::stream_queue(d->ctx, &rc);
  if (!q) return rc;
  return efes_upload_open(q, hashes, sha1, crc, &d->u);
}

template <class D>
void close_upload(D* d) {
  if (d->u) efes_upload_close(d->u);
  d->u = nullptr;
}

int sha1_open(efes_sha1* d) { return ensure_open(d, EFES_HASH_SHA1, &d->base, nullptr); }
int crc32_open(efes_crc32* d) { return ensure_open(d, EFES_HASH_CRC32, nullptr, &d->base); }

// The full Go state now: h from the device after every staged byte, x/nx/len replayed.
int sha1_state_now(efes_sha1* d, efes_sha1_state* out) {
  if (d->latched) return d->latched;
  if (!d->u) {
    *out = d->base;
    return EFES_OK;
  }
  const int rc = efes_upload_state(d->u, out, nullptr);
  if (rc && rc != EFES_ERR_STATE) d->latched = rc;
  return rc;
}

int sha1_alloc(efes_ctx* ctx, efes_sha1** out, bool reset) {
  if (!ctx || !out) return EFES_ERR_ARG;
  efes_sha1* d = new (std::nothrow) efes_sha1;
  if (!d) return EFES_ERR_NOMEM;
  d->ctx = ctx;
  memset(&d->base, 0, sizeof d->base);
  if (reset) efes_sha1_state_init(&d->base);  // NewSha1 (sha1.go:48-52); else `var d sha1digest`
  *out = d;
  return EFES_OK;
}

}  // namespace

extern "C" {

// ---- streaming SHA-1 (sha1digest) --------------------------------------------------------------
int efes_sha1_new(efes_ctx* ctx, efes_sha1** out) { return sha1_alloc(ctx, out, true); }
int efes_sha1_new_zero(efes_ctx* ctx, efes_sha1** out) { return sha1_alloc(ctx, out, false); }

void efes_sha1_free(efes_sha1* d) {
  if (!d) return;
  close_upload(d);
  delete d;
}

void efes_sha1_reset(efes_sha1* d) {  // sha1.go:36-44: h = IV, nx = len = 0, x untouched
  if (!d) return;
  const efes_sha1_state cur = d->u ? efes::upload_shadow(d->u) : d->base;
  close_upload(d);
  efes_sha1_state_init(&d->base);
  memcpy(d->base.x, cur.x, sizeof d->base.x);
  d->latched = EFES_OK;
}

int efes_sha1_size(void) { return 20; }
int efes_sha1_block_size(void) { return 64; }

int efes_sha1_write(efes_sha1* d, const void* p, size_t n) {  // sha1.go:58-79
  if (!d || (!p && n)) return EFES_ERR_ARG;
  int rc = sha1_open(d);
  if (rc) return rc;
  rc = efes_upload_write(d->u, p, n);
  if (rc) d->latched = rc;
  return rc;
}

int efes_sha1_sum(efes_sha1* d, uint8_t out[20]) {  // sha1.go:82-87 (non-destructive)
  if (!d || !out) return EFES_ERR_ARG;
  int rc = sha1_open(d);
  if (rc) return rc;
  uint8_t s[24];
  rc = efes_upload_sum(d->u, s);
  if (rc == EFES_OK) memcpy(out, s, 20);
  else if (rc != EFES_ERR_STATE) d->latched = rc;
  return rc;
}

int efes_sha1_marshal_text(efes_sha1* d, char out[200]) {  // sha1_efes.go:25-38
  if (!d || !out) return EFES_ERR_ARG;
  efes_sha1_state st;
  const int rc = sha1_state_now(d, &st);
  if (rc) return rc;
  efes_sha1_state_marshal_text(&st, out);
  return EFES_OK;
}

int efes_sha1_unmarshal_text(efes_sha1* d, const char* text, size_t n) {  // sha1_efes.go:40-64
  if (!d) return EFES_ERR_ARG;
  efes_sha1_state s;
  const int rc = efes_sha1_state_unmarshal_text(&s, text, n);
  if (rc) return rc;  // Go leaves the digest untouched on this path
  return efes_sha1_set_state(d, &s);
}

int efes_sha1_get_state(efes_sha1* d, efes_sha1_state* out) {
  if (!d || !out) return EFES_ERR_ARG;
  return sha1_state_now(d, out);
}

int efes_sha1_set_state(efes_sha1* d, const efes_sha1_state* in) {
  if (!d || !in) return EFES_ERR_ARG;
  close_upload(d);
  d->base = *in;
  d->latched = EFES_OK;
  return EFES_OK;
}

// ---- streaming CRC-32 (crc32digest) ------------------------------------------------------------
int efes_crc32_new(efes_ctx* ctx, efes_crc32** out) {  // crc32.go:68 NewCRC32IEEE
  if (!ctx || !out) return EFES_ERR_ARG;
  efes_crc32* d = new (std::nothrow) efes_crc32;
  if (!d) return EFES_ERR_NOMEM;
  d->ctx = ctx;
  d->base.crc = 0;
  *out = d;
  return EFES_OK;
}

void efes_crc32_free(efes_crc32* d) {
  if (!d) return;
  close_upload(d);
  delete d;
}

void efes_crc32_reset(efes_crc32* d) {  // crc32.go:74
  if (!d) return;
  close_upload(d);
  d->base.crc = 0;
  d->latched = EFES_OK;
}

int efes_crc32_size(void) { return 4; }
int efes_crc32_block_size(void) { return 1; }

int efes_crc32_write(efes_crc32* d, const void* p, size_t n) {  // crc32.go:76-86
  if (!d || (!p && n)) return EFES_ERR_ARG;
  int rc = crc32_open(d);
  if (rc) return rc;
  rc = efes_upload_write(d->u, p, n);
  if (rc) d->latched = rc;
  return rc;
}

int efes_crc32_sum32(efes_crc32* d, uint32_t* out) {  // crc32.go:88
  if (!d || !out) return EFES_ERR_ARG;
  if (d->latched) return d->latched;
  if (!d->u) {
    *out = d->base.crc;
    return EFES_OK;
  }
  efes_crc32_state c;
  const int rc = efes_upload_state(d->u, nullptr, &c);
  if (rc) return d->latched = rc;
  *out = c.crc;
  return EFES_OK;
}

int efes_crc32_sum(efes_crc32* d, uint8_t out[4]) {  // crc32.go:90-93
  uint32_t v;
  const int rc = efes_crc32_sum32(d, &v);
  if (rc) return rc;
  out[0] = (uint8_t)(v >> 24); out[1] = (uint8_t)(v >> 16); out[2] = (uint8_t)(v >> 8); out[3] = (uint8_t)v;
  return EFES_OK;
}

int efes_crc32_marshal_text(efes_crc32* d, char out[8]) {  // crc32_efes.go:18-24
  if (!d || !out) return EFES_ERR_ARG;
  efes_crc32_state s;
  const int rc = efes_crc32_sum32(d, &s.crc);
  if (rc) return rc;
  efes_crc32_state_marshal_text(&s, out);
  return EFES_OK;
}

int efes_crc32_unmarshal_text(efes_crc32* d, const char* text, size_t n) {  // crc32_efes.go:26-40
  if (!d) return EFES_ERR_ARG;
  efes_crc32_state s;
  const int rc = efes_crc32_state_unmarshal_text(&s, text, n);
  if (rc) return rc;
  close_upload(d);
  d->base = s;
  d->latched = EFES_OK;
  return EFES_OK;
}

}  // extern "C"
