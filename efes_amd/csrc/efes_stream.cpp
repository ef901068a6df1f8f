// efes_stream.cpp -- the Go-surface streaming digests (layer 2 of efes_hash.h) on top of the
// upload dispatcher (efes_queue.cpp).
//
// sha1digest (sha1.go:29-120, sha1_efes.go:25-64) and crc32digest (crc32.go:48-93,
// crc32_efes.go:18-40) keep their method sets; each object is an efes_upload of a context's
// shared digest queue that keeps only its own hash (EFES_HASH_SHA1 or EFES_HASH_CRC32).  So the Go
// code of filereceiver.go -- io.MultiWriter(f, CRC32, Sha1) in every request goroutine --
// drops in unchanged and still gets batched launches across all concurrent requests: a Write
// stages into pinned memory and returns; Sum / MarshalText are the sync points.
//
// Go's Write never fails, and the Go code frees digests only through the garbage collector, so an
// upload slot is held only while it is needed (efes_hash.h, layer 2):
//   * between a sync point and the next Write a digest is PARKED: its state lives on the host
//     (`sbase` / `cbase`) and it holds no upload;
//   * a Write (or a Sum of a parked digest) opens an upload from the parked state; when the
//     queue has no free slot it EVICTS the oldest digest that is not inside a call (hashes what
//     that one staged, parks it) and takes the slot, or waits for a holder to leave its call;
//   * device faults are latched by Write, which still returns EFES_OK; the sync points report them.
// Every call holds the digest's mutex (one goroutine per digest, so it is uncontended), which is
// what lets another thread evict the digest safely between calls.
//
// Placement: a digest made on a context uses that context's queue; one made on a pool
// (efes_pool_create) opens each upload on the pool's context with the most free slots.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <new>
#include <vector>

#include "efes_internal.hpp"

struct efes_pool {
  std::vector<efes_ctx*> ctxs;
  std::atomic<uint32_t> next{0};  // round-robin start for ties
};

namespace efes {

struct Digest {
  std::mutex mu;               // held for every call on the object, and by an evictor
  efes_ctx* home = nullptr;    // fixed placement, or
  efes_pool* pool = nullptr;   // a context chosen at every (re)open
  uint32_t hashes = 0;         // EFES_HASH_SHA1 or EFES_HASH_CRC32
  efes_ctx* on = nullptr;      // the context whose digest queue holds `u`
  efes_upload* u = nullptr;    // null while parked
  std::list<Digest*>::iterator pos;  // in on->dreg.open while u != nullptr
  efes_sha1_state sbase{};     // the parked state (sha1digest)
  efes_crc32_state cbase{};    // the parked state (crc32digest)
  int latched = EFES_OK;       // an error the next sync point reports (Go would have panicked, or a fault)
  bool sha() const { return hashes == EFES_HASH_SHA1; }
};

}  // namespace efes

struct efes_sha1 : efes::Digest {};
struct efes_crc32 : efes::Digest {};

using efes::Digest;

namespace {

// Shared queue sizing: EFES_DIGEST_STAGING_MIB of pinned staging (default 256 MiB) in chunks of
// EFES_DIGEST_CHUNK_KIB (default 64 KiB: 4096 chunks, so up to 4095 digests hold an upload at once).
efes_queue* create_digest_queue(efes_ctx* ctx, int* rc) {
  uint64_t mib = 256, kib = 64;
  if (const char* e = getenv("EFES_DIGEST_STAGING_MIB")) mib = strtoull(e, nullptr, 10);
  if (const char* e = getenv("EFES_DIGEST_CHUNK_KIB")) kib = strtoull(e, nullptr, 10);
  if (mib < 1) mib = 1;
  if (kib < 4 || kib > 4096) kib = 64;
  const uint64_t chunk = kib << 10;
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

namespace {

void unlist(Digest* d) {  // d->mu held, d->u open
  efes::DigestRegistry& r = d->on->dreg;
  {
    std::lock_guard<std::mutex> lk(r.mu);
    r.open.erase(d->pos);
  }
  r.released.notify_all();
}

// Gives the upload back, dropping bytes staged since the last sync point (the state is being
// replaced: UnmarshalText, Reset, free).  d->mu held.
void drop(Digest* d) {
  if (!d->u) return;
  efes_upload* u = d->u;
  unlist(d);
  d->u = nullptr;
  d->on = nullptr;
  efes_upload_close(u);
}

// Parks the digest: the state after every staged byte (h / crc from the device, Go's x/nx/len
// replayed on the host) moves to sbase / cbase and the upload is given back.  A failure is
// latched for the next sync point.  d->mu held.
void park(Digest* d) {
  if (!d->u) return;
  efes_sha1_state s = efes::upload_shadow(d->u);  // x/nx/len (Reset keeps x even after a failure)
  efes_crc32_state c{};
  const int rc = efes_upload_state(d->u, d->sha() ? &s : nullptr, d->sha() ? nullptr : &c);
  if (d->sha()) d->sbase = s;
  else if (rc == EFES_OK) d->cbase = c;
  if (rc != EFES_OK && d->latched == EFES_OK) d->latched = rc;
  drop(d);
}

// Evicts the oldest digest of ctx's queue that is not inside a call (and is not `self`).
bool evict_one(efes_ctx* ctx, Digest* self) {
  Digest* victim = nullptr;
  {
    std::lock_guard<std::mutex> lk(ctx->dreg.mu);
    for (Digest* d : ctx->dreg.open)
      if (d != self && d->mu.try_lock()) {
        victim = d;
        break;
      }
  }
  if (!victim) return false;
  park(victim);
  victim->mu.unlock();
  return true;
}

efes_ctx* place(Digest* d) {
  if (!d->pool) return d->home;
  const auto& cs = d->pool->ctxs;
  const uint32_t n = (uint32_t)cs.size(), start = d->pool->next.fetch_add(1, std::memory_order_relaxed);
  efes_ctx* best = nullptr;
  int64_t most = -1;
  for (uint32_t k = 0; k < n; ++k) {
    efes_ctx* c = cs[(start + k) % n];
    int rc = EFES_OK;
    efes_queue* q = efes::stream_queue(c, &rc);
    if (!q) continue;
    const int64_t f = efes::queue_free_slots(q);
    if (f > most) {
      most = f;
      best = c;
    }
  }
  return best ? best : cs[start % n];
}

// An upload holding the parked state; evicts or waits while the chosen queue is full.  d->mu held.
int acquire(Digest* d) {
  if (d->latched) return d->latched;
  if (d->u) return EFES_OK;
  for (;;) {
    efes_ctx* c = place(d);
    int rc = EFES_OK;
    efes_queue* q = efes::stream_queue(c, &rc);
    if (!q) return rc;
    bool no_slot = false;
    rc = efes::upload_open_slot(q, d->hashes, d->sha() ? &d->sbase : nullptr, d->sha() ? nullptr : &d->cbase,
                                &d->u, &no_slot);
    if (rc == EFES_OK) {
      d->on = c;
      std::lock_guard<std::mutex> lk(c->dreg.mu);
      d->pos = c->dreg.open.insert(c->dreg.open.end(), d);
      return EFES_OK;
    }
    if (!no_slot) return rc;
    if (evict_one(c, d)) continue;
    // Every holder is inside a call (writing, or waiting for its own jobs): each of those calls
    // ends, and its digest becomes evictable.  The timed wait also covers a release that
    // happened between the scan and the wait.
    std::unique_lock<std::mutex> lk(c->dreg.mu);
    c->dreg.released.wait_for(lk, std::chrono::milliseconds(1));
  }
}

// Write(p): Go's never fails except where it panics (nx > 64 -> EFES_ERR_STATE).  Other errors
// are latched for the next sync point.
int digest_write(Digest* d, const void* p, size_t n) {
  if (!d || (!p && n)) return EFES_ERR_ARG;
  std::lock_guard<std::mutex> lk(d->mu);
  if (d->latched) return d->latched == EFES_ERR_STATE ? EFES_ERR_STATE : EFES_OK;
  int rc = acquire(d);
  if (rc == EFES_OK) rc = efes_upload_write(d->u, p, n);
  if (rc == EFES_OK) return EFES_OK;
  d->latched = rc;
  return rc == EFES_ERR_STATE ? EFES_ERR_STATE : EFES_OK;
}

template <class D>
D* make(efes_ctx* ctx, efes_pool* pool, uint32_t hashes) {
  D* d = new (std::nothrow) D;
  if (!d) return nullptr;
  d->home = ctx;
  d->pool = pool;
  d->hashes = hashes;
  return d;
}

int sha1_alloc(efes_ctx* ctx, efes_pool* pool, efes_sha1** out, bool reset) {
  if ((!ctx && !pool) || !out) return EFES_ERR_ARG;
  efes_sha1* d = make<efes_sha1>(ctx, pool, EFES_HASH_SHA1);
  if (!d) return EFES_ERR_NOMEM;
  memset(&d->sbase, 0, sizeof d->sbase);
  if (reset) efes_sha1_state_init(&d->sbase);  // NewSha1 (sha1.go:48-52); else `var d sha1digest`
  *out = d;
  return EFES_OK;
}

int crc32_alloc(efes_ctx* ctx, efes_pool* pool, efes_crc32** out) {
  if ((!ctx && !pool) || !out) return EFES_ERR_ARG;
  efes_crc32* d = make<efes_crc32>(ctx, pool, EFES_HASH_CRC32);
  if (!d) return EFES_ERR_NOMEM;
  d->cbase.crc = 0;  // NewCRC32IEEE (crc32.go:68)
  *out = d;
  return EFES_OK;
}

void digest_free(Digest* d) {
  if (!d) return;
  {
    std::lock_guard<std::mutex> lk(d->mu);
    drop(d);
  }
  delete d;
}

// The full Go state now (h from the device after every staged byte, x/nx/len replayed); parks.
int sha1_state_now(efes_sha1* d, efes_sha1_state* out) {  // d->mu held
  park(d);
  if (d->latched) return d->latched;
  *out = d->sbase;
  return EFES_OK;
}

}  // namespace

extern "C" {

// ---- pools -----------------------------------------------------------------------------------
int efes_pool_create(efes_ctx* const* ctxs, uint32_t n, efes_pool** out) {
  if (!ctxs || n == 0 || !out) return EFES_ERR_ARG;
  *out = nullptr;
  for (uint32_t i = 0; i < n; ++i)
    if (!ctxs[i]) return EFES_ERR_ARG;
  efes_pool* p = new (std::nothrow) efes_pool;
  if (!p) return EFES_ERR_NOMEM;
  try {
    p->ctxs.assign(ctxs, ctxs + n);
  } catch (...) {
    delete p;
    return EFES_ERR_NOMEM;
  }
  *out = p;
  return EFES_OK;
}

void efes_pool_destroy(efes_pool* p) { delete p; }

int efes_pool_stats(efes_pool* p, uint32_t i, efes_queue_stats* out) {
  if (!p || !out || i >= p->ctxs.size()) return EFES_ERR_ARG;
  efes_ctx* c = p->ctxs[i];
  efes_queue* q;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    q = c->digests;
  }
  if (!q) {
    memset(out, 0, sizeof *out);
    return EFES_OK;
  }
  return efes_queue_get_stats(q, out);
}

// ---- streaming SHA-1 (sha1digest) --------------------------------------------------------------
int efes_sha1_new(efes_ctx* ctx, efes_sha1** out) { return sha1_alloc(ctx, nullptr, out, true); }
int efes_sha1_new_zero(efes_ctx* ctx, efes_sha1** out) { return sha1_alloc(ctx, nullptr, out, false); }
int efes_sha1_new_pool(efes_pool* p, efes_sha1** out) { return p ? sha1_alloc(nullptr, p, out, true) : EFES_ERR_ARG; }
int efes_sha1_new_zero_pool(efes_pool* p, efes_sha1** out) {
  return p ? sha1_alloc(nullptr, p, out, false) : EFES_ERR_ARG;
}

void efes_sha1_free(efes_sha1* d) { digest_free(d); }

void efes_sha1_reset(efes_sha1* d) {  // sha1.go:36-44: h = IV, nx = len = 0, x untouched
  if (!d) return;
  std::lock_guard<std::mutex> lk(d->mu);
  const efes_sha1_state cur = d->u ? efes::upload_shadow(d->u) : d->sbase;
  drop(d);
  efes_sha1_state_init(&d->sbase);
  memcpy(d->sbase.x, cur.x, sizeof d->sbase.x);
  d->latched = EFES_OK;
}

int efes_sha1_size(void) { return 20; }
int efes_sha1_block_size(void) { return 64; }

int efes_sha1_write(efes_sha1* d, const void* p, size_t n) { return digest_write(d, p, n); }  // sha1.go:58-79

int efes_sha1_sum(efes_sha1* d, uint8_t out[20]) {  // sha1.go:82-87 (non-destructive)
  if (!d || !out) return EFES_ERR_ARG;
  std::lock_guard<std::mutex> lk(d->mu);
  int rc = acquire(d);
  if (rc) return rc;
  uint8_t s[24];
  rc = efes_upload_sum(d->u, s);
  if (rc == EFES_OK) memcpy(out, s, 20);
  else if (rc != EFES_ERR_STATE) d->latched = rc;  // checkSum's panic leaves the digest usable
  park(d);
  return rc == EFES_OK && d->latched ? d->latched : rc;
}

int efes_sha1_marshal_text(efes_sha1* d, char out[200]) {  // sha1_efes.go:25-38
  if (!d || !out) return EFES_ERR_ARG;
  std::lock_guard<std::mutex> lk(d->mu);
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
  std::lock_guard<std::mutex> lk(d->mu);
  return sha1_state_now(d, out);
}

int efes_sha1_set_state(efes_sha1* d, const efes_sha1_state* in) {
  if (!d || !in) return EFES_ERR_ARG;
  std::lock_guard<std::mutex> lk(d->mu);
  drop(d);
  d->sbase = *in;
  d->latched = EFES_OK;
  return EFES_OK;
}

// ---- streaming CRC-32 (crc32digest) ------------------------------------------------------------
int efes_crc32_new(efes_ctx* ctx, efes_crc32** out) { return crc32_alloc(ctx, nullptr, out); }  // crc32.go:68
int efes_crc32_new_pool(efes_pool* p, efes_crc32** out) { return p ? crc32_alloc(nullptr, p, out) : EFES_ERR_ARG; }

void efes_crc32_free(efes_crc32* d) { digest_free(d); }

void efes_crc32_reset(efes_crc32* d) {  // crc32.go:74
  if (!d) return;
  std::lock_guard<std::mutex> lk(d->mu);
  drop(d);
  d->cbase.crc = 0;
  d->latched = EFES_OK;
}

int efes_crc32_size(void) { return 4; }
int efes_crc32_block_size(void) { return 1; }

int efes_crc32_write(efes_crc32* d, const void* p, size_t n) { return digest_write(d, p, n); }  // crc32.go:76-86

int efes_crc32_sum32(efes_crc32* d, uint32_t* out) {  // crc32.go:88
  if (!d || !out) return EFES_ERR_ARG;
  std::lock_guard<std::mutex> lk(d->mu);
  park(d);
  if (d->latched) return d->latched;
  *out = d->cbase.crc;
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
  std::lock_guard<std::mutex> lk(d->mu);
  drop(d);
  d->cbase = s;
  d->latched = EFES_OK;
  return EFES_OK;
}

}  // extern "C"
