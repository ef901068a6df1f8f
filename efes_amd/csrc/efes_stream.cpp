// efes_stream.cpp -- the Go-surface streaming digests (layer 2 of efes_hash.h) on top of the
// upload dispatcher (efes_queue.cpp).
//
// sha1digest (sha1.go:29-120, sha1_efes.go:25-64) and crc32digest (crc32.go:48-93,
// crc32_efes.go:18-40) keep their method sets; each object is an efes_upload of a context's
// shared digest queue.  So the Go code of filereceiver.go -- io.MultiWriter(f, CRC32, Sha1) in
// every request goroutine -- drops in unchanged and still gets batched launches across all
// concurrent requests: a Write stages into pinned memory and returns; Sum / MarshalText are the
// sync points.
//
// Go's Write never fails, and the Go code frees digests only through the garbage collector, so an
// upload slot is held only while it is needed (efes_hash.h, layer 2):
//   * between a sync point and the next Write a digest is PARKED: its state lives on the host
//     (`sbase` / `cbase`) and it holds no upload;
//   * a Write (or a Sum of a parked digest) opens an upload from the parked state; when the
//     queue has no free slot it waits for a holder's sync point, EVICTING (hashing what it
//     staged, parking it) the oldest holder that is not inside a call and has been idle for
//     EFES_DIGEST_EVICT_MS -- or, once the Write has waited that long, any holder not in a call;
//   * device faults are latched by Write, which still returns EFES_OK; the sync points report them.
// Every call holds the digest's mutex (one goroutine per digest, so it is uncontended), which is
// what lets another thread evict the digest safely between calls.
//
// FUSED PAIRS (round 4).  MultiWriter(f, CRC32, Sha1) (filereceiver.go:208-209, fileinfo.go:20-27)
// hands every body buffer p to the CRC digest and then, unchanged, to the SHA-1 digest.  Two
// separate uploads would stage p twice and launch two jobs that each read it over PCIe.  Instead:
//   * a CRC digest's first Write after a sync point waits in a scratch buffer and registers (p, n)
//     as a candidate;
//   * a parked SHA-1 digest whose Write has the same (p, n) BINDS to it: the pair opens ONE upload
//     keeping both hashes (SHA-1 from the SHA-1 digest's parked state, CRC from the CRC digest's)
//     and the waiting Write becomes the pair's open leader Write;
//   * from then on the leader's (CRC) Write waits in a cache-hot scratch buffer; the follower's
//     (SHA-1) Write of the same (p, n) is staged with streaming stores and compared with it in the
//     same pass, which confirms it -- one staging copy and one fused job per body byte;
//   * anything else -- a Write to one digest only, different bytes, a Sum / MarshalText of the
//     leader first, Reset / UnmarshalText / free of one, an eviction -- SETTLES the pair: every
//     confirmed byte is hashed into both states, the leader's unconfirmed bytes into its state
//     only, and both digests continue alone (a follower's sync point or a member whose state is
//     being replaced just LEAVES, the partner keeping the upload).
// So a wrong guess costs time, never correctness: every digest hashes exactly the bytes of its
// own Writes, in order.
//
// Placement: a digest made on a context uses that context's queue; one made on a pool
// (efes_pool_create) opens each upload on the pool's context with the most free slots, skipping
// contexts whose queue has latched a device fault.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <chrono>
#include <new>
#include <unordered_map>
#include <utility>
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
  efes_upload* u = nullptr;    // null while parked (and while fused: the pair holds the upload)
  std::list<OpenRef>::iterator pos;  // in on->dreg.open while u != nullptr
  efes_sha1_state sbase{};     // the parked state (sha1digest)
  efes_crc32_state cbase{};    // the parked state (crc32digest)
  int latched = EFES_OK;       // an error the next sync point reports (Go would have panicked, or a fault)
  Fused* fz = nullptr;         // the fused pair this digest is a member of (u/on unused meanwhile)
  const void* cand_p = nullptr;  // a CRC digest whose upload holds exactly its first Write (cand_p, cand_n)
  size_t cand_n = 0;
  std::atomic<int64_t> last_ns{0};  // end of its last call (eviction prefers long-idle holders)
  // a CRC digest's first Write after a sync point waits here, as the candidate, until a SHA-1
  // digest binds to it or the digest's next call stages it
  uint8_t* defer = nullptr;
  size_t defer_cap = 0, defer_n = 0;
  bool sha() const { return hashes == EFES_HASH_SHA1; }
  virtual ~Digest() { free(defer); }
};

// One upload shared by a CRC digest (the leader: MultiWriter writes it first) and a SHA-1 digest
// (the follower).  Guarded by `mu`, taken after the member's own mutex.
struct Fused {
  std::mutex mu;
  efes_upload* u = nullptr;        // null once settled
  efes_ctx* on = nullptr;
  std::list<OpenRef>::iterator pos;  // in on->dreg.open while u != nullptr
  bool lead_in = true, follow_in = true;  // members still sharing the upload
  int refs = 2;                    // members whose fz still points here
  // the leader's last Write, waiting in `scratch`, not yet matched by the follower
  bool open = false;
  const void* op = nullptr;
  size_t on_bytes = 0;
  // after settle(): both states after every byte, for the members to pick up at their next call
  bool settled = false;
  efes_sha1_state sha_out{};
  efes_crc32_state crc_out{};
  int rc_sha = EFES_OK, rc_crc = EFES_OK;
  std::atomic<int64_t> last_ns{0};  // end of a member's last call on the pair
  uint8_t* scratch = nullptr;
  size_t scratch_cap = 0;
  size_t conf = 0;  // bytes of the open scratch Write the follower has confirmed (staged in pieces)
  ~Fused() { free(scratch); }
};

}  // namespace efes

struct efes_sha1 : efes::Digest {};
struct efes_crc32 : efes::Digest {};

using efes::Digest;
using efes::Fused;
using efes::OpenRef;

namespace {

// Process-wide counters (efes_pair_stats_get), sharded by thread: every fused Write counts, and one
// shared cache line bounced between 32 request threads cost more than the pair check at small Writes.
struct alignas(64) PairCounters {
  std::atomic<uint64_t> pairs{0}, fused_writes{0}, fused_bytes{0}, settles{0};
};
constexpr uint32_t kCounterShards = 64;
PairCounters g_counters[kCounterShards];

PairCounters& counters() {
  static std::atomic<uint32_t> next{0};
  thread_local PairCounters* mine = &g_counters[next.fetch_add(1, std::memory_order_relaxed) % kCounterShards];
  return *mine;
}

// Idle times for eviction (a 50 ms patience) need no better than the coarse clock's few ms, and it
// costs a fraction of a precise read on every call.
int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC_COARSE, &ts);
  return (int64_t)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}

// Eviction patience (EFES_DIGEST_EVICT_MS, default 50): a Write that finds every slot taken first
// waits for a holder's sync point and evicts only holders idle for this long (a stalled client, an
// abandoned digest); once it has waited this long itself it evicts the oldest idle holder, active or
// not (progress).  Evicting active holders at once (0) made every Write of an over-subscribed queue
// settle another upload and wait for the GPU (profiles/r04_evict/evict.log).  Read once when the
// library is loaded (by one thread, before any call): a function-local static initialised on first
// use is first read by request threads racing each other.
const int64_t g_evict_patience_ns = [] {
  const char* e = getenv("EFES_DIGEST_EVICT_MS");
  return (e && *e ? strtoll(e, nullptr, 10) : 50ll) * 1000000ll;
}();

int64_t evict_patience_ns() { return g_evict_patience_ns; }

// Where the leader's Write waits for the follower's: a cache-hot per-thread scratch buffer, so the
// follower's Write stages with streaming stores while comparing against it in the same pass (no
// read-for-ownership of the staging lines, no second pass over the bytes).  Round 4 measured the
// alternatives -- the leader staged in the upload with ordinary stores (the compare hits the cache,
// every staging line is read for ownership first) or with streaming stores (the compare reads DRAM):
// scratch 46.8-47.7, cached 45.9-46.4, stream 46.3-47.5 GiB/s against efes_upload 48.9-49.3
// (profiles/r04_pair_stage_ab2/ab.log), and removed them in round 5.

// Scratch buffers: a few per thread, reused last-in first-out so the one a
// leader Write copies into is still in this core's cache when the follower's Write (normally on
// the same thread, right after) compares against it.  A buffer may be returned on another thread.
// The per-thread slots are trivially destructible, so a digest call made while the thread is being
// torn down (after the reaper below has freed the slots) still finds valid storage: it frees the
// buffer instead of caching it.
struct ScratchBuf {
  uint8_t* p;
  size_t cap;
};
constexpr uint32_t kScratchPerThread = 4;
constexpr size_t kScratchKeepMax = 1u << 20;  // larger buffers (Writes of more than 1 MiB) are not kept
thread_local ScratchBuf t_scratch[kScratchPerThread];
thread_local uint32_t t_nscratch = 0;
thread_local bool t_scratch_reaped = false;
struct ScratchReaper {
  ~ScratchReaper() {
    for (uint32_t i = 0; i < t_nscratch; ++i) free(t_scratch[i].p);
    t_nscratch = 0;
    t_scratch_reaped = true;
  }
};
thread_local ScratchReaper t_scratch_reaper;

uint8_t* scratch_get(size_t n, size_t* cap) {
  for (uint32_t i = t_nscratch; i-- > 0;)
    if (t_scratch[i].cap >= n) {
      const ScratchBuf b = t_scratch[i];
      for (uint32_t k = i + 1; k < t_nscratch; ++k) t_scratch[k - 1] = t_scratch[k];
      --t_nscratch;
      *cap = b.cap;
      return b.p;
    }
  const size_t c = (n + 65535) & ~(size_t)65535;
  uint8_t* p = static_cast<uint8_t*>(aligned_alloc(64, c));
  *cap = p ? c : 0;
  return p;
}

void scratch_put(uint8_t* p, size_t cap) {
  if (t_scratch_reaped || cap > kScratchKeepMax) {
    free(p);
    return;
  }
  (void)&t_scratch_reaper;  // registers the reaper for this thread
  if (t_nscratch == kScratchPerThread) {
    free(t_scratch[0].p);
    for (uint32_t k = 1; k < kScratchPerThread; ++k) t_scratch[k - 1] = t_scratch[k];
    --t_nscratch;
  }
  t_scratch[t_nscratch++] = ScratchBuf{p, cap};
}


bool reclaim_chunks(void* arg, uint32_t want);

// Default pinned staging per context, and the floor a failed allocation is retried down to.
constexpr uint64_t kDigestStagingMib = 1024, kDigestStagingMinMib = 256;

// Shared queue sizing: EFES_DIGEST_STAGING_MIB of pinned staging (default 1024 MiB) in chunks of
// EFES_DIGEST_CHUNK_KIB (default 256 KiB: 4096 chunks; 256 KiB chunks ran 34.8 against 31.8 GiB/s
// for 64 KiB with 2 048 uploads in flight, profiles/r04_digest_queue/sweep.log), and
// EFES_DIGEST_SLOTS upload slots (default 65 536: 256 B of pinned state each).  A digest or fused
// pair holds a slot from its first Write to its sync point; with more slots than chunks, the
// dispatcher hands idle holders' partly filled chunks over when writers wait for one
// (reclaim_chunks), so requests in flight are bounded by the slots, not by the staging -- with one
// slot per chunk, 8 192 uploads in flight on 4 095 slots ran at 0.9 GiB/s, every Write evicting
// (settling) another upload.  EFES_DIGEST_SLOTS below the chunks gives round 3's queue (slots =
// min(EFES_DIGEST_SLOTS, chunks - 1), no reclaim).
efes_queue* create_digest_queue(efes_ctx* ctx, int* rc) {
  uint64_t mib = kDigestStagingMib, kib = 256, slots = 65536;
  if (const char* e = getenv("EFES_DIGEST_STAGING_MIB")) mib = strtoull(e, nullptr, 10);
  if (const char* e = getenv("EFES_DIGEST_CHUNK_KIB")) kib = strtoull(e, nullptr, 10);
  if (const char* e = getenv("EFES_DIGEST_SLOTS")) slots = strtoull(e, nullptr, 10);
  if (mib < 1) mib = 1;
  if (kib < 4 || kib > 4096) kib = 256;
  if (slots < 1) slots = 1;
  if (slots > (1u << 22)) slots = 1u << 22;
  const uint64_t chunk = kib << 10;
  efes_queue* q = nullptr;
  for (;;) {
    const uint32_t chunks = (uint32_t)((mib << 20) / chunk) < 16 ? 16u : (uint32_t)((mib << 20) / chunk);
    if (slots >= chunks)
      *rc = efes::queue_create_reclaiming(ctx, chunk, chunks, (uint32_t)slots, reclaim_chunks, ctx, &q);
    else
      *rc = efes_queue_create(ctx, chunk, chunks, (uint32_t)slots, &q);
    // The pinned staging did not fit (host memory locked by others, a small cgroup): halve it down
    // to kDigestStagingMinMib before the error is latched into every digest of the context.
    if (*rc == EFES_OK || (*rc != EFES_ERR_HIP && *rc != EFES_ERR_NOMEM) || mib <= kDigestStagingMinMib) break;
    mib = std::max<uint64_t>(kDigestStagingMinMib, mib / 2);
  }
  if (*rc == EFES_OK && ctx->fault_after) efes::queue_set_fault_after(q, ctx->fault_after);
  return *rc == EFES_OK ? q : nullptr;
}

// ---- leader candidates: CRC digests whose fresh upload holds exactly one Write (p, n) -----------
struct CandShard {
  std::mutex mu;
  std::unordered_map<const void*, Digest*> m;
};
CandShard g_cand[64];

CandShard& shard_of(const void* p) {
  const uint64_t h = (uint64_t)reinterpret_cast<uintptr_t>(p) * 0x9E3779B97F4A7C15ull;
  return g_cand[h >> 58];
}

void uncandidate(Digest* d) {  // d->mu held
  if (!d->cand_p) return;
  CandShard& s = shard_of(d->cand_p);
  {
    std::lock_guard<std::mutex> lk(s.mu);
    auto it = s.m.find(d->cand_p);
    if (it != s.m.end() && it->second == d) s.m.erase(it);
  }
  d->cand_p = nullptr;
}

void candidate(Digest* d, const void* p, size_t n) {  // d->mu held
  CandShard& s = shard_of(p);
  std::lock_guard<std::mutex> lk(s.mu);
  s.m[p] = d;
  d->cand_p = p;
  d->cand_n = n;
}

}  // namespace

efes_queue* efes::stream_queue(efes_ctx* ctx, int* rc) {
  std::lock_guard<std::mutex> lk(ctx->mu);
  *rc = EFES_OK;
  if (!ctx->digests) ctx->digests = create_digest_queue(ctx, rc);
  return ctx->digests;
}

namespace {

void unlist(efes_ctx* on, std::list<OpenRef>::iterator pos) {
  efes::DigestRegistry& r = on->dreg;
  {
    std::lock_guard<std::mutex> lk(r.mu);
    r.open.erase(pos);
  }
  r.released.notify_all();
}

// Gives the upload back, dropping bytes staged since the last sync point (the state is being
// replaced: UnmarshalText, Reset, free).  d->mu held, d not fused.
void drop(Digest* d) {
  if (!d->u) return;
  efes_upload* u = d->u;
  unlist(d->on, d->pos);
  d->u = nullptr;
  d->on = nullptr;
  efes_upload_close(u);
}

// Parks the digest: the state after every staged byte (h / crc from the device, Go's x/nx/len
// replayed on the host) moves to sbase / cbase and the upload is given back.  A failure is
// latched for the next sync point.  d->mu held, d not fused.
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

// ---- fused pairs --------------------------------------------------------------------------------
// The leader's open Write (what of it the follower has not confirmed), in its scratch buffer.
const uint8_t* pending(const Fused* z) { return z->scratch + z->conf; }
size_t pending_n(const Fused* z) { return z->on_bytes - z->conf; }

// Gives the leader's open Write up (z->mu held).
void drop_pending(Fused* z) {
  scratch_put(z->scratch, z->scratch_cap);
  z->scratch = nullptr;
  z->open = false;
  z->conf = 0;
}

// Settles the pair (z->mu held): every matched byte is hashed into both states, the leader's
// unmatched Write (if any) into the CRC state alone; both states are left for the members to pick
// up and the upload is given back.
void settle(Fused* z) {
  efes_upload* u = z->u;
  if (!u) return;
  std::vector<uint8_t> tail;
  if (z->open) {  // the leader's bytes the follower never matched: hashed for the leader only
    const uint8_t* t = pending(z);
    tail.assign(t, t + pending_n(z));
    drop_pending(z);
  }
  efes_sha1_state s = efes::upload_shadow(u);
  efes_crc32_state c{};
  const int rc = efes_upload_state(u, &s, &c);  // waits for every matched byte (both hashes)
  z->sha_out = s;
  z->rc_sha = rc;
  z->crc_out = c;
  z->rc_crc = rc;
  if (!tail.empty() && rc == EFES_OK && z->lead_in) {
    efes::upload_keep(u, EFES_HASH_CRC32);
    int rc2 = efes_upload_write(u, tail.data(), tail.size());
    if (rc2 == EFES_OK) rc2 = efes_upload_state(u, nullptr, &c);
    z->crc_out = c;
    z->rc_crc = rc2;
  }
  unlist(z->on, z->pos);
  efes_upload_close(u);
  z->u = nullptr;
  z->on = nullptr;
  z->settled = true;
  counters().settles.fetch_add(1, std::memory_order_relaxed);
}

// d stops being a member of z (z->mu held through zk, released here); the last member frees z.
void detach(Digest* d, Fused* z, std::unique_lock<std::mutex>& zk) {
  d->fz = nullptr;
  const bool last = --z->refs == 0;
  zk.unlock();
  if (last) delete z;
}

// d takes its state from a settled pair (park's conventions for failures).
void pickup(Digest* d, const Fused* z) {
  if (d->sha()) {
    d->sbase = z->sha_out;
    if (z->rc_sha != EFES_OK && d->latched == EFES_OK) d->latched = z->rc_sha;
  } else if (z->rc_crc == EFES_OK) {
    d->cbase = z->crc_out;
  } else if (d->latched == EFES_OK) {
    d->latched = z->rc_crc;
  }
}

// The partner left: d holds the upload alone from now on (its hashes are d's already).
void adopt(Digest* d, Fused* z) {
  d->u = z->u;
  d->on = z->on;
  d->pos = z->pos;
  {
    std::lock_guard<std::mutex> lk(d->on->dreg.mu);
    *d->pos = OpenRef{d, nullptr};
  }
  z->u = nullptr;
  z->on = nullptr;
}

// d gives its share of the pair up and the partner keeps the upload (taking it over at its next
// call).  sync: d's state after every matched byte is read first (d's sync point; the caller has
// checked that no leader Write is unmatched); else d's state is being replaced and the leader's
// unmatched bytes, if d is the leader, are dropped.  Returns the state read's error.
int leave(Digest* d, Fused* z, bool sync, std::unique_lock<std::mutex>& zk) {
  efes_upload* u = z->u;
  int rc = EFES_OK;
  if (d->sha()) {
    if (sync) {
      efes_sha1_state s = efes::upload_shadow(u);
      rc = efes_upload_state(u, &s, nullptr);
      d->sbase = s;
      if (rc != EFES_OK && d->latched == EFES_OK) d->latched = rc;
    }
    efes::upload_keep(u, EFES_HASH_CRC32);
    if (z->open) {  // the leader's open Write is its own: into the (now CRC-only) upload
      (void)efes_upload_write(u, pending(z), pending_n(z));  // a fault is latched in u
      drop_pending(z);
    }
    z->follow_in = false;
  } else {
    if (z->open) drop_pending(z);
    if (sync) {
      efes_crc32_state c{};
      rc = efes_upload_state(u, nullptr, &c);
      if (rc == EFES_OK) d->cbase = c;
      else if (d->latched == EFES_OK) d->latched = rc;
    }
    efes::upload_keep(u, EFES_HASH_SHA1);
    z->lead_in = false;
  }
  detach(d, z, zk);
  return rc;
}

int acquire(Digest* d);

// A CRC digest's deferred first Write (no SHA-1 digest bound to it before the digest's next call)
// goes into an upload of its own -- or is dropped when the digest's state is being replaced.
// d->mu held.
void undefer(Digest* d, bool keep) {
  uint8_t* b = d->defer;
  if (!b) return;
  d->defer = nullptr;
  if (keep) {
    int rc = acquire(d);
    if (rc == EFES_OK) rc = efes_upload_write(d->u, b, d->defer_n);
    if (rc != EFES_OK && d->latched == EFES_OK) d->latched = rc;
  }
  scratch_put(b, d->defer_cap);
}

// One call on a digest: d->mu, and for a member of a live pair the pair's mutex too (`z` set).  A
// member of a settled pair picks up its state, one whose partner left takes the upload over; both
// are alone again (`z` null).  A CRC digest's candidacy ends with its next call, and its deferred
// first Write is staged (keep) or dropped (the call replaces the state: free, Reset, UnmarshalText).
struct Call {
  Digest* d;
  Fused* z = nullptr;
  std::unique_lock<std::mutex> lk, zk;
  ~Call() {  // still holding d->mu (and z->mu when z is set)
    const int64_t t = now_ns();
    d->last_ns.store(t, std::memory_order_relaxed);
    if (z) z->last_ns.store(t, std::memory_order_relaxed);
  }
  explicit Call(Digest* dd, bool keep = true) : d(dd), lk(dd->mu) {
    uncandidate(d);
    undefer(d, keep);
    Fused* f = d->fz;
    if (!f) return;
    zk = std::unique_lock<std::mutex>(f->mu);
    if (f->settled) {
      pickup(d, f);
      detach(d, f, zk);
    } else if (!(d->sha() ? f->lead_in : f->follow_in)) {
      adopt(d, f);
      detach(d, f, zk);
    } else {
      z = f;
    }
  }
  // the pair cannot go on for this call: settle it and continue alone
  void split() {
    settle(z);
    pickup(d, z);
    Fused* f = z;
    z = nullptr;
    detach(d, f, zk);
  }
  int leave(bool sync) {
    Fused* f = z;
    z = nullptr;
    return ::leave(d, f, sync, zk);
  }
};

// The digest queue's reclaim hook (run by its dispatcher thread, which holds no digest, pair or
// queue lock): every chunk sits partly filled in an upload while `want` writers wait for one, so up
// to `want` holders that are not inside a call hand their partly filled chunks over (hashed like a
// full one, then freed).  Holders idle for kReclaimIdleNs or longer go first -- an abandoned or
// stalled upload's chunk before that of one whose writer is between two Writes (which would fill it
// soon anyway) -- then the other holders, oldest first.  They are try-locked under dreg.mu and handed
// over after it is released (a locked holder cannot be freed, parked or settled meanwhile, as in
// evict_one), so the context's acquire / adopt / evict calls never wait behind the hand-overs
// (ADVICE r05).  (A fused pair's unconfirmed leader Write waits in its scratch buffer, never in the
// chunk.)  Lock order: dreg.mu, then holders by try_lock only; the queue's mutex inside the hand-over
// is taken with dreg.mu released -- nothing takes dreg.mu while holding a queue's mutex.  Returns
// whether anything was handed over.
constexpr int64_t kReclaimIdleNs = 1000000;  // 1 ms: longer than any gap between a writer's Writes

bool reclaim_chunks(void* arg, uint32_t want) {
  efes_ctx* ctx = static_cast<efes_ctx*>(arg);
  std::vector<std::pair<std::mutex*, efes_upload*>> held;
  held.reserve(std::min<uint32_t>(want, 4096));
  {
    std::lock_guard<std::mutex> lk(ctx->dreg.mu);
    const int64_t horizon = now_ns() - kReclaimIdleNs;
    for (int pass = 0; pass < 2 && held.size() < want; ++pass) {
      for (const OpenRef& r : ctx->dreg.open) {
        if (held.size() >= want) break;
        const bool idle = (r.d ? r.d->last_ns : r.f->last_ns).load(std::memory_order_relaxed) <= horizon;
        if (idle != (pass == 0)) continue;  // pass 0: the idle holders; pass 1: the others
        std::mutex& m = r.d ? r.d->mu : r.f->mu;
        if (!m.try_lock()) continue;
        efes_upload* u = r.d ? r.d->u : r.f->u;
        if (u && efes::upload_partial(u)) {  // only holders that have a partly filled chunk to hand over
          held.emplace_back(&m, u);
        } else {
          m.unlock();
        }
      }
    }
  }
  uint32_t got = 0;
  for (auto& [m, u] : held) {
    if (efes::upload_handover(u)) ++got;
    m->unlock();
  }
  return got > 0;
}

// Evicts the oldest digest (or fused pair) of ctx's queue that is not inside a call, has been idle
// for at least min_idle_ns, and is not `self`.
bool evict_one(efes_ctx* ctx, Digest* self, int64_t min_idle_ns) {
  Digest* victim = nullptr;
  Fused* pair = nullptr;
  const int64_t horizon = now_ns() - min_idle_ns;
  {
    std::lock_guard<std::mutex> lk(ctx->dreg.mu);
    for (const OpenRef& r : ctx->dreg.open) {
      if ((r.d ? r.d->last_ns : r.f->last_ns).load(std::memory_order_relaxed) > horizon) continue;
      if (r.d) {
        if (r.d != self && r.d->mu.try_lock()) {
          victim = r.d;
          break;
        }
      } else if (r.f->mu.try_lock()) {  // no member is inside an operation on the pair
        pair = r.f;
        break;
      }
    }
  }
  if (victim) {
    park(victim);
    victim->mu.unlock();
    return true;
  }
  if (pair) {
    settle(pair);  // the members pick their states up at their next calls
    pair->mu.unlock();
    return true;
  }
  return false;
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
    const int64_t f = efes::queue_free_slots(q);  // -1: the queue latched a device fault
    if (f > most) {
      most = f;
      best = c;
    }
  }
  return best ? best : cs[start % n];  // every queue faulted: the sync point reports it
}

bool placed_on(const Digest* d, const efes_ctx* c) {
  if (!d->pool) return c == d->home;
  for (const efes_ctx* x : d->pool->ctxs)
    if (x == c) return true;
  return false;
}

// An upload holding the parked state; evicts or waits while the chosen queue is full.  d->mu held.
int acquire(Digest* d) {
  if (d->latched) return d->latched;
  if (d->u) return EFES_OK;
  const int64_t t0 = now_ns();
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
      d->pos = c->dreg.open.insert(c->dreg.open.end(), OpenRef{d, nullptr});
      return EFES_OK;
    }
    if (!no_slot) return rc;
    const int64_t patience = evict_patience_ns();
    if (evict_one(c, d, now_ns() - t0 >= patience ? 0 : patience)) continue;
    // No holder may be evicted yet: every one is inside a call (writing, or waiting for its own
    // jobs) or was active within the patience -- each call ends and each holder either reaches its
    // sync point (releasing the slot) or becomes evictable.  The timed wait also covers a release
    // that happened between the scan and the wait.
    std::unique_lock<std::mutex> lk(c->dreg.mu);
    c->dreg.released.wait_for(lk, std::chrono::milliseconds(1));
  }
}

void count_fused(size_t n) {
  PairCounters& k = counters();
  k.fused_writes.fetch_add(1, std::memory_order_relaxed);
  k.fused_bytes.fetch_add(n, std::memory_order_relaxed);
}

enum class Bind { kNo, kPending };

// A parked SHA-1 digest's Write (p, n) joins the CRC digest whose last Write was the same (p, n)
// (MultiWriter(f, CRC32, Sha1) just made it) and is deferred in its scratch buffer.  c.d is the
// SHA-1 digest (its mutex held), parked and not fused.  The pair opens ONE upload keeping both
// hashes (SHA-1 from the SHA-1 digest's parked state, CRC from the CRC digest's) and the deferred
// bytes become the pair's open leader Write, which the SHA-1 Write then confirms as a follower
// (kPending: c.z and c.zk are set).
Bind try_bind(Call& c, const uint8_t* p, size_t n) {
  Digest* f = c.d;
  Digest* l;
  {
    CandShard& s = shard_of(p);
    std::lock_guard<std::mutex> lk(s.mu);
    auto it = s.m.find(p);
    if (it == s.m.end()) return Bind::kNo;
    l = it->second;
    // try_lock: l's owner may be inside a call (or freeing l, which first takes l->mu and then
    // this shard's lock): then no bind.  Holding the shard lock keeps l alive until we hold l->mu.
    if (l == f || l->cand_n != n || !l->mu.try_lock()) return Bind::kNo;
    s.m.erase(it);
    l->cand_p = nullptr;
  }
  std::unique_lock<std::mutex> llk(l->mu, std::adopt_lock);
  if (l->fz || l->latched || l->sha() || !l->defer || l->u || l->defer_n != n) return Bind::kNo;
  efes_ctx* on = place(l);
  if (!placed_on(f, on)) return Bind::kNo;
  int rc = EFES_OK;
  efes_queue* q = efes::stream_queue(on, &rc);
  if (!q) return Bind::kNo;
  bool no_slot = false;
  efes_upload* u = nullptr;
  if (efes::upload_open_slot(q, EFES_HASH_SHA1 | EFES_HASH_CRC32, &f->sbase, &l->cbase, &u, &no_slot) != EFES_OK)
    return Bind::kNo;  // no free slot: both go on alone (l stages its Write at its next call)
  Fused* z = new (std::nothrow) Fused;
  if (!z) {
    efes_upload_close(u);
    return Bind::kNo;
  }
  // the pair is locked before an evictor or the reclaim hook can find it in the registry
  c.zk = std::unique_lock<std::mutex>(z->mu);
  c.z = z;
  z->u = u;
  z->on = on;
  z->open = true;  // l's deferred Write is the pair's open leader Write
  z->op = p;
  z->on_bytes = n;
  z->scratch = l->defer;
  z->scratch_cap = l->defer_cap;
  l->defer = nullptr;
  z->last_ns.store(now_ns(), std::memory_order_relaxed);
  {
    std::lock_guard<std::mutex> lk(on->dreg.mu);
    z->pos = on->dreg.open.insert(on->dreg.open.end(), OpenRef{nullptr, z});
  }
  l->fz = z;
  f->fz = z;
  counters().pairs.fetch_add(1, std::memory_order_relaxed);
  return Bind::kPending;
}

// The leader's (CRC) Write in a live pair: it waits for the follower's.  False: the pair splits.
bool lead(Call& c, const uint8_t* p, size_t n) {
  Fused* z = c.z;
  if (n == 0) return true;    // crc32.go:76-86 of nothing
  if (z->open) return false;  // the follower never confirmed the previous one
  size_t cap = 0;
  uint8_t* b = scratch_get(n, &cap);
  if (!b) return false;  // no memory for a scratch buffer
  memcpy(b, p, n);
  z->scratch = b;
  z->scratch_cap = cap;
  z->conf = 0;
  z->open = true;
  z->op = p;
  z->on_bytes = n;
  return true;
}

// The follower's (SHA-1) Write in a live pair: the leader's open Write must be the same (p, n) and
// the same bytes.  True: done.  False: the pair splits and the follower writes p[0, n) alone -- after
// a scratch Write confirmed in part, p / n are advanced past the confirmed bytes and *whole is the
// Go state after the single Write (the caller's pieces would leave other stale bytes in x[nx:]).
bool follow(Call& c, const uint8_t*& p, size_t& n, efes_sha1_state* whole, bool* split_mid) {
  Fused* z = c.z;
  efes_upload* u = z->u;
  if (n == 0) return efes::upload_shadow(u).nx != 64;  // an empty Write changes nothing (else: alone)
  if (!z->open || p != z->op || n != z->on_bytes) return false;
  const efes_sha1_state s0 = efes::upload_shadow(u);
  efes_sha1_state sh = s0;
  if (efes::replay_write(&sh, p, n) != EFES_OK) return false;  // Go panics: alone
  // Staged now, piece by piece (a Write larger than the room left in the chunk spans several), with
  // streaming stores compared with the leader's copy in the same pass.  Each piece is confirmed with
  // the Go state after it (its x[:nx] is what a later job continues from), the last one with the
  // single Write's state.
  efes_sha1_state ps = s0;
  size_t done = 0;
  while (done < n) {
    const size_t piece = (size_t)std::min<uint64_t>(n - done, efes::upload_room(u));
    bool same = false;
    uint64_t off = 0;
    if (efes::upload_stage_if_same(u, p + done, z->scratch + done, piece, &off, &same) != EFES_OK) {
      drop_pending(z);  // the fault is latched in the upload for the sync points
      return true;
    }
    if (!same) break;
    (void)efes::replay_write(&ps, p + done, piece);
    done += piece;
    z->conf = done;
    (void)efes::upload_confirm(u, done < n ? ps : sh);
  }
  if (done == n) {
    drop_pending(z);
    count_fused(n);
    return true;
  }
  if (done) {
    *whole = sh;
    *split_mid = true;
    p += done;
    n -= done;
  }
  return false;
}

// Write(p): Go's never fails except where it panics (nx > 64 -> EFES_ERR_STATE).  Other errors
// are latched for the next sync point.
int digest_write(Digest* d, const void* p0, size_t n0) {
  if (!d || (!p0 && n0)) return EFES_ERR_ARG;
  Call c(d);
  const uint8_t* p = static_cast<const uint8_t*>(p0);
  size_t n = n0;
  efes_sha1_state whole{};
  bool split_mid = false;  // the rest of a Write the pair confirmed in part
  if (c.z) {
    if (d->sha() ? follow(c, p, n, &whole, &split_mid) : lead(c, p, n)) return EFES_OK;
    c.split();  // the Writes diverged: both continue alone
  }
  if (d->latched) return d->latched == EFES_ERR_STATE ? EFES_ERR_STATE : EFES_OK;
  if (!split_mid && n > 0 && !d->u) {
    if (d->sha()) {
      if (try_bind(c, p, n) == Bind::kPending) {
        if (follow(c, p, n, &whole, &split_mid)) return EFES_OK;
        c.split();
        if (d->latched) return d->latched == EFES_ERR_STATE ? EFES_ERR_STATE : EFES_OK;
      }
    } else {
      // a CRC digest's first Write on a fresh upload waits for its MultiWriter partner
      size_t cap = 0;
      if (uint8_t* b = scratch_get(n, &cap)) {
        memcpy(b, p, n);
        d->defer = b;
        d->defer_cap = cap;
        d->defer_n = n;
        candidate(d, p, n);
        return EFES_OK;
      }
    }
  }
  int rc = acquire(d);
  if (rc == EFES_OK) rc = efes_upload_write(d->u, p, n);
  if (rc == EFES_OK && split_mid) efes::upload_set_shadow(d->u, whole);  // Go made ONE Write of it
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

template <class D>
void digest_free(D* d) {
  if (!d) return;
  {
    Call c(d, false);
    if (c.z) c.leave(false);
    drop(d);
  }
  delete d;
}

// The full Go state now (h from the device after every staged byte, x/nx/len replayed); parks.
int sha1_state_now(Call& c, efes_sha1_state* out) {
  efes_sha1* d = static_cast<efes_sha1*>(c.d);
  if (c.z) {
    if (c.z->open) c.split();
    else c.leave(true);  // the matched bytes are all of this digest's bytes
  }
  park(d);
  if (d->latched) return d->latched;
  *out = d->sbase;
  return EFES_OK;
}

// The CRC's parked value after every byte written (sync point of Sum32 / Sum / MarshalText).
int crc32_now(Call& c, uint32_t* out) {
  Digest* d = c.d;
  if (c.z) {
    if (c.z->open) c.split();  // the leader's last Write is its own: settle, hashing it for the CRC only
    else c.leave(true);
  }
  park(d);
  if (d->latched) return d->latched;
  *out = d->cbase.crc;
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

int efes_pair_stats_get(efes_pair_stats* out) {
  if (!out) return EFES_ERR_ARG;
  memset(out, 0, sizeof *out);
  for (const PairCounters& k : g_counters) {
    out->pairs += k.pairs.load(std::memory_order_relaxed);
    out->fused_writes += k.fused_writes.load(std::memory_order_relaxed);
    out->fused_bytes += k.fused_bytes.load(std::memory_order_relaxed);
    out->settles += k.settles.load(std::memory_order_relaxed);
  }
  return EFES_OK;
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
  Call c(d);
  efes_sha1_state cur;
  if (c.z) {
    cur = efes::upload_shadow(c.z->u);  // x after the matched Writes: all of this digest's
    c.leave(false);
  } else {
    cur = d->u ? efes::upload_shadow(d->u) : d->sbase;
    drop(d);
  }
  efes_sha1_state_init(&d->sbase);
  memcpy(d->sbase.x, cur.x, sizeof d->sbase.x);
  d->latched = EFES_OK;
}

int efes_sha1_size(void) { return 20; }
int efes_sha1_block_size(void) { return 64; }

int efes_sha1_write(efes_sha1* d, const void* p, size_t n) { return digest_write(d, p, n); }  // sha1.go:58-79

int efes_sha1_sum(efes_sha1* d, uint8_t out[20]) {  // sha1.go:82-87 (non-destructive)
  if (!d || !out) return EFES_ERR_ARG;
  Call c(d);
  uint8_t s[24];
  int rc;
  if (c.z && !c.z->open) {
    // the pair's Sum job (folded into the last chunk's fused job) computes both Sums; the
    // follower takes its own and leaves the upload to the leader (whose Sum is its parked CRC)
    rc = efes_upload_sum(c.z->u, s);
    if (rc == EFES_OK) memcpy(out, s, 20);
    else if (rc != EFES_ERR_STATE) d->latched = rc;  // checkSum's panic leaves the digest usable
    c.leave(true);
    return rc == EFES_OK && d->latched ? d->latched : rc;
  }
  if (c.z) c.split();
  rc = acquire(d);
  if (rc) return rc;
  rc = efes_upload_sum(d->u, s);
  if (rc == EFES_OK) memcpy(out, s, 20);
  else if (rc != EFES_ERR_STATE) d->latched = rc;  // checkSum's panic leaves the digest usable
  park(d);
  return rc == EFES_OK && d->latched ? d->latched : rc;
}

int efes_sha1_marshal_text(efes_sha1* d, char out[200]) {  // sha1_efes.go:25-38
  if (!d || !out) return EFES_ERR_ARG;
  Call c(d);
  efes_sha1_state st;
  const int rc = sha1_state_now(c, &st);
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
  Call c(d);
  return sha1_state_now(c, out);
}

int efes_sha1_set_state(efes_sha1* d, const efes_sha1_state* in) {
  if (!d || !in) return EFES_ERR_ARG;
  Call c(d);
  if (c.z) c.leave(false);
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
  Call c(d, false);
  if (c.z) c.leave(false);
  drop(d);
  d->cbase.crc = 0;
  d->latched = EFES_OK;
}

int efes_crc32_size(void) { return 4; }
int efes_crc32_block_size(void) { return 1; }

int efes_crc32_write(efes_crc32* d, const void* p, size_t n) { return digest_write(d, p, n); }  // crc32.go:76-86

int efes_crc32_sum32(efes_crc32* d, uint32_t* out) {  // crc32.go:88
  if (!d || !out) return EFES_ERR_ARG;
  Call c(d);
  return crc32_now(c, out);
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
  Call c(d, false);
  if (c.z) c.leave(false);
  drop(d);
  d->cbase = s;
  d->latched = EFES_OK;
  return EFES_OK;
}

}  // extern "C"
