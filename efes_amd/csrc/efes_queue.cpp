// efes_queue.cpp -- batching dispatcher for concurrent uploads.
//
// The reference hashes each upload in its own request goroutine (server.go:130): every
// io.Copy buffer goes through MultiWriter(file, CRC32, Sha1) (filereceiver.go:208-209) and
// the digest is read at the end of the PATCH (Sum, filereceiver.go:99-100) or saved to the
// .info file (MarshalText, filereceiver.go:226).  On the GPU one launch must carry many
// uploads, so an efes_upload is the device-resident (SHA-1, CRC-32) pair of one upload, its
// Write copies into pinned, device-mapped staging and returns (the kernel reads the staged
// chunks in place over PCIe: no H2D copy), and a dispatcher thread per queue turns the
// staged chunks of all uploads into one kernel launch (at most one chunk per upload per
// launch, so each upload's chain stays in order on the queue's stream) while callers keep
// staging.  Sync points (flush / state / sum) wait for that upload's bytes only.
//
// Tail-buffer bytes x/nx/len are replayed on the host per Write (efes::replay_write), so an
// exported state is byte-identical to what Go's MarshalText would write after the same
// Write calls, stale bytes included; h and crc come from the device.
//
// The per-upload state slots live in pinned, device-mapped host memory: the kernels read and
// write an upload's 104 + 4 bytes of state once per job over PCIe, and the sync points read
// them in place.  Sum is a zero-length FINALIZE job of the same dispatcher (so the Sums of many
// requests share launches with everyone's chunks) writing the 24-byte digest pair into the
// slot.  No sync point issues a copy or a launch of its own.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include <emmintrin.h>

#include "efes_internal.hpp"

using efes::DeviceGuard;

namespace {
// State slot of one upload (pinned, device-mapped): sha1 state 104 | crc 4 | pad | sum 24 | status 4.
constexpr size_t kDevStateBytes = 256;
constexpr size_t kOffCrc = 104, kOffSum = 112, kOffStatus = 136;
constexpr uint32_t kNoChunk = 0xffffffffu;  // a Pending that is a Sum (FINALIZE, no bytes)
}  // namespace

struct efes_upload {
  efes_queue* q = nullptr;
  uint32_t hashes = EFES_HASH_SHA1 | EFES_HASH_CRC32;
  uint32_t dslot = 0;            // device state slot
  int32_t cur = -1;              // staging chunk being filled (-1: none)
  uint64_t fill = 0;             // bytes in `cur`
  uint64_t reserved = 0;         // bytes the last efes_upload_reserve granted (0: no reservation)
  uint64_t inflight = 0;         // chunks queued or running
  uint64_t queued = 0;           // of which still in q->pending (not in a launch yet)
  bool in_batch = false;         // has a chunk in the batch being assembled
  bool fold_sum = false;         // Sum requested: the last queued chunk's job also writes the Sum
  std::atomic<int> latched{EFES_OK};  // first device / state error (set by the dispatcher too)
  efes_sha1_state shadow{};      // Go's x/nx/len after every Write (h from the device)
  std::condition_variable done;  // inflight dropped (signalled on every retired job)
};

struct Pending {
  efes_upload* u;
  uint32_t slot;  // staging chunk, or kNoChunk for a Sum
  uint64_t len;
};

using Clock = std::chrono::steady_clock;

struct Batch {
  hipEvent_t ev = nullptr;
  std::vector<Pending> items;
  int jobs_half = 0;
  int mode = 0;                // kernel shape it was launched with (efes::pcie_mode)
  uint64_t max_len = 0;        // its longest job: the launch's time follows it
  Clock::time_point start{};   // when it started running: its submit time on an idle stream, else the
                               // retire time of the launch ahead of it (set then)
  bool start_known = false;    // submitted onto an idle stream: `start` is its submit time
};

struct efes_queue {
  efes_ctx* ctx = nullptr;
  uint64_t chunk = 0;
  uint32_t nchunks = 0, max_uploads = 0;
  uint64_t ahead = 0;              // per-upload cap on queued + running chunks while chunks are scarce
  uint8_t* h_slab = nullptr;       // pinned, device-mapped staging, nchunks x chunk
  uint8_t* z_slab = nullptr;       // the device address of h_slab: kernels read it over PCIe
  uint8_t* h_states = nullptr;     // max_uploads x kDevStateBytes, pinned + device-mapped
  uint8_t* z_states = nullptr;     // the device address of h_states
  efes_job* h_jobs = nullptr;      // pinned, 2 halves x nchunks
  efes_job* d_jobs = nullptr;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::condition_variable work, freed;
  std::vector<uint32_t> free_chunks, free_states;
  std::deque<Pending> pending;
  std::deque<Batch> running;
  int next_half = 0;
  bool stop = false;
  int fault = EFES_OK;
  uint64_t n_launches = 0, n_jobs = 0, n_bytes = 0;  // efes_queue_get_stats
  uint64_t n_attempts = 0, inject_at = 0;  // test hook (efes_debug_fault_after): launch k faults
  // max_uploads may exceed the chunks only with a reclaim hook (efes::queue_create_reclaiming):
  // when writers wait for a chunk, none is free and nothing is queued, the dispatcher calls it --
  // without mu, holding no lock of the owner layer -- to have idle uploads hand their partly
  // filled chunks over, so no writer waits on chunks that nobody would hand over.
  bool (*reclaim)(void*, uint32_t want) = nullptr;
  void* reclaim_arg = nullptr;
  uint32_t chunk_waiters = 0;      // writers blocked in take_chunk
  uint64_t n_reclaims = 0;
  bool starving() const { return reclaim && chunk_waiters > 0 && free_chunks.empty(); }
  // hipEventBlockingSync: the dispatcher sleeps in retire instead of polling the event, so it does
  // not keep a host core busy beside the request threads (receiver within noise either way:
  // profiles/r03_receiver/ab_sync_*.log).
  static constexpr unsigned ev_flags = hipEventDisableTiming | hipEventBlockingSync;
  // Just-in-time assembly (round 6): while one launch runs, the next one is assembled only shortly
  // before the running one is expected to end (DESIGN_NOTES.md §5 "One PATCH's latency under load"),
  // so chunks staged meanwhile -- a new PATCH's first chunk above all -- still make that launch instead
  // of waiting for the one after it.  The expected end comes from the launch's longest job and a
  // learned time per byte of each kernel shape (EWMA over retired launches).
  double ns_per_byte[16] = {};
  // Extra margin learned from gaps: when the launch a just-in-time wait was timed on had already
  // finished by the time the next one was submitted (the dispatcher woke late: a busy CPU quota), the
  // GPU idled; the margin then grows (x2 + 250 us, at most one launch) and shrinks by 1/8 per launch
  // that was on time.
  std::chrono::nanoseconds jit_extra{0};
  bool jit_waited = false;  // the batch being assembled was timed by a just-in-time wait
  std::thread th;

  void run();
  void retire(Batch& b, std::unique_lock<std::mutex>& lk);
};

// Launches shorter than this are not timed for the per-byte model (launch overhead dominates them).
constexpr uint64_t kJitMinBytes = 64u << 10;
// How early the next launch is assembled before the running one's expected end: the host's wake-up
// (late when the request threads keep every core of the quota busy), the assembly, the job-array copy
// and the launch itself, plus the model's error -- 400 us plus a tenth of the expected time.
constexpr auto kJitMargin = std::chrono::microseconds(400);

// Waits for the batch (without holding mu, so callers keep staging) and releases its chunks.
void efes_queue::retire(Batch& b, std::unique_lock<std::mutex>& lk) {  // mu held on entry and exit
  lk.unlock();
  const bool ok = hipEventSynchronize(b.ev) == hipSuccess;
  const Clock::time_point done = Clock::now();
  (void)hipEventDestroy(b.ev);
  lk.lock();
  if (ok && b.max_len >= kJitMinBytes && b.mode >= 0 && b.mode < 16) {  // the launch time per byte of its shape
    // A sample is the launch's time plus this thread's wake-up, which the request threads can delay by
    // milliseconds on a busy CPU quota: samples above 1.5 x the model are clipped there, so one late
    // wake-up moves it by 12.5 % at most (the margin covers that) while real slowdowns still get in.
    double ns = std::chrono::duration<double, std::nano>(done - b.start).count() / (double)b.max_len;
    double& r = ns_per_byte[b.mode];
    if (r > 0) ns = std::min(ns, 1.5 * r);
    r = r > 0 ? 0.75 * r + 0.25 * ns : ns;
  }
  if (!running.empty() && !running.front().start_known) running.front().start = done;  // queued behind it: starts now
  if (!ok && fault == EFES_OK) fault = EFES_ERR_DEVICE_FAULT;
  for (const Pending& p : b.items) {
    if (p.slot != kNoChunk) free_chunks.push_back(p.slot);
    if (!ok) p.u->latched = EFES_ERR_DEVICE_FAULT;
    --p.u->inflight;
    p.u->done.notify_all();  // wait_idle (inflight 0) and pace (inflight < ahead)
  }
  freed.notify_all();
}

void efes_queue::run() {
  DeviceGuard g(ctx->device);
  std::unique_lock<std::mutex> lk(mu);
  for (;;) {
    work.wait(lk, [&] { return stop || !pending.empty() || !running.empty() || starving(); });
    if (pending.empty()) {
      if (starving() && !stop) {
        // Writers wait for a chunk and none is free: every chunk not in a launch sits partly filled
        // in an upload.  Have the idle holders hand theirs over, so the next launch is assembled
        // while the running one finishes.
        ++n_reclaims;
        const uint32_t want = chunk_waiters;  // > 0 (starving)
        lk.unlock();
        const bool any = reclaim(reclaim_arg, want);
        lk.lock();
        if (any) continue;
        if (running.empty()) {  // holders busy, nothing to retire: look again soon
          work.wait_for(lk, std::chrono::microseconds(200));
          continue;
        }
      }
      if (running.empty()) {
        if (stop) return;
        continue;
      }
      Batch b = std::move(running.front());  // nothing new to launch: retire the oldest
      running.pop_front();
      retire(b, lk);
      continue;
    }
    if (running.size() >= 2) {  // two launches in flight: their job-array halves are busy
      Batch b = std::move(running.front());
      running.pop_front();
      retire(b, lk);
      continue;
    }
    // Just in time: wait until shortly before the running launch is expected to end.  Only for DEEP
    // launches (at most one job per SIMD: uploads in flight up to the SIMD count), whose time is one
    // chunk's chain and barely varies; the grouped shapes of heavier loads launch ahead as before (there
    // every upload has chunks waiting anyway, and a late wake-up would idle the GPU: profiles/r06_jit_ab/).
    if (running.size() == 1 && !stop && running.front().mode == EFES_MODE_DEEP) {
      const Batch& r = running.front();
      const double rate = ns_per_byte[EFES_MODE_DEEP];
      if (rate > 0 && r.max_len >= kJitMinBytes) {
        const auto dur = std::chrono::nanoseconds((int64_t)(rate * (double)r.max_len));
        const auto at = r.start + dur - kJitMargin - dur / 10 - jit_extra;
        if (Clock::now() < at) {
          jit_waited = true;
          work.wait_until(lk, at, [&] { return stop; });  // staging Writes do not cut the wait short
          continue;
        }
      }
    }
    // Assemble: FIFO order, at most one chunk per upload (a job must not race its own state).
    Batch b;
    b.jobs_half = next_half;
    next_half ^= 1;
    std::deque<Pending> later;
    while (!pending.empty()) {
      // one job-array half holds nchunks jobs: with more uploads than chunks (a reclaiming queue)
      // the Sums of many uploads could otherwise outnumber it; the rest waits, in order
      if (b.items.size() >= nchunks) {
        later.insert(later.end(), pending.begin(), pending.end());
        pending.clear();
        break;
      }
      Pending p = pending.front();
      pending.pop_front();
      if (p.u->in_batch) {
        later.push_back(p);
        continue;
      }
      p.u->in_batch = true;
      --p.u->queued;
      b.items.push_back(p);
    }
    pending.swap(later);
    for (const Pending& p : b.items) p.u->in_batch = false;
    efes_job* hj = h_jobs + (size_t)b.jobs_half * nchunks;
    efes_job* dj = d_jobs + (size_t)b.jobs_half * nchunks;
    for (size_t i = 0; i < b.items.size(); ++i) {
      const Pending& p = b.items[i];
      uint8_t* st = z_states + (size_t)p.u->dslot * kDevStateBytes;
      const bool sum = p.slot == kNoChunk;  // Sum: works on a copy (sha1.go:82-87), state unchanged (SUM_ONLY)
      // The upload's last queued chunk after a Sum request: Write + Sum in one job (the kernel
      // writes back the post-Write state and the Sum of a copy of it), one launch fewer.
      const bool fold = !sum && p.u->fold_sum && p.u->queued == 0;
      if (fold) p.u->fold_sum = false;
      efes_job& j = hj[i];
      j.data = sum ? nullptr : z_slab + (size_t)p.slot * chunk;
      j.length = sum ? 0 : p.len;
      j.sha1 = (p.u->hashes & EFES_HASH_SHA1) ? reinterpret_cast<efes_sha1_state*>(st) : nullptr;
      j.crc32 = (p.u->hashes & EFES_HASH_CRC32) ? reinterpret_cast<efes_crc32_state*>(st + kOffCrc) : nullptr;
      j.sum = sum || fold ? st + kOffSum : nullptr;
      j.status = reinterpret_cast<int32_t*>(st + kOffStatus);
      j.flags = sum ? EFES_JOB_FINALIZE | EFES_JOB_SUM_ONLY : fold ? EFES_JOB_FINALIZE : 0u;
      j._reserved = 0;
    }
    // test hook (efes_debug_fault_after): this launch reports a device fault instead of running
    const bool inject = inject_at && ++n_attempts == inject_at;
    // the launch a just-in-time wait was timed on (the only one running): did it finish before this one?
    const hipEvent_t timed_on = jit_waited && running.size() == 1 ? running.front().ev : nullptr;
    const auto timed_dur = timed_on ? std::chrono::nanoseconds((int64_t)(ns_per_byte[EFES_MODE_DEEP] *
                                                                         (double)running.front().max_len))
                                    : std::chrono::nanoseconds(0);
    jit_waited = false;
    const bool idle_stream = running.empty();
    lk.unlock();  // callers keep staging while this batch is copied and launched
    const bool late = timed_on && hipEventQuery(timed_on) == hipSuccess;  // already done: the GPU idles
    if (timed_on) efes::clear_last_error();                                // (hipErrorNotReady: on time)
    // No H2D copy of the data: the DEEP kernel reads the pinned chunks in place (4 KiB per
    // wave per super-step, prefetched a super-step ahead, so the PCIe latency is hidden behind
    // the chain).  Measured 2.5x the rate of staging copies (DESIGN_NOTES.md).
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = hipMemcpyAsync(dj, hj, sizeof(efes_job) * b.items.size(), hipMemcpyHostToDevice, stream);
    // DEEP (or grouped DEEP beyond one chunk per SIMD): efes::pcie_mode.
    const uint32_t nb = (uint32_t)b.items.size();
    b.mode = efes::pcie_mode(ctx, nb);
    for (const Pending& p : b.items) b.max_len = std::max<uint64_t>(b.max_len, p.len);
    int rc = e == hipSuccess ? EFES_OK : EFES_ERR_HIP;
    if (rc == EFES_OK && inject) rc = EFES_ERR_DEVICE_FAULT;  // as a faulted kernel
    if (rc == EFES_OK) rc = efes_hash_submit_mode(ctx, dj, nb, stream, b.mode);
    b.start = Clock::now();  // on an idle stream it starts now; else retire() sets it
    b.start_known = idle_stream || late;
    if (rc == EFES_OK && hipEventCreateWithFlags(&b.ev, ev_flags) != hipSuccess) rc = EFES_ERR_HIP;
    if (rc == EFES_OK && hipEventRecord(b.ev, stream) != hipSuccess) rc = EFES_ERR_HIP;
    lk.lock();
    if (timed_on && rc == EFES_OK)
      jit_extra = late ? std::min<std::chrono::nanoseconds>(2 * jit_extra + std::chrono::microseconds(250), timed_dur)
                       : jit_extra - jit_extra / 8;
    if (rc != EFES_OK) {
      if (b.ev) (void)hipEventDestroy(b.ev);
      if (fault == EFES_OK) fault = rc;
      for (const Pending& p : b.items) {
        if (p.slot != kNoChunk) free_chunks.push_back(p.slot);
        p.u->latched = rc;
        --p.u->inflight;
        p.u->done.notify_all();
      }
      freed.notify_all();
      continue;
    }
    ++n_launches;
    n_jobs += b.items.size();
    for (const Pending& p : b.items) n_bytes += p.len;
    running.push_back(std::move(b));
  }
}

namespace {

int enqueue_current(efes_upload* u, std::unique_lock<std::mutex>&, bool even_empty = false) {  // q->mu held
  efes_queue* q = u->q;
  if (u->cur < 0 || (u->fill == 0 && !even_empty)) return EFES_OK;
  q->pending.push_back(Pending{u, (uint32_t)u->cur, u->fill});
  ++u->inflight;
  ++u->queued;
  u->cur = -1;
  u->fill = 0;
  q->work.notify_one();
  return EFES_OK;
}

// A staging chunk for `u` to fill (q->mu held): waits for a free one.
int take_chunk(efes_upload* u, std::unique_lock<std::mutex>& lk) {
  efes_queue* q = u->q;
  if (!q->fault && q->free_chunks.empty()) {
    ++q->chunk_waiters;  // the dispatcher may have to reclaim partly filled chunks (starving())
    q->work.notify_one();
    q->freed.wait(lk, [&] { return q->fault || !q->free_chunks.empty(); });
    --q->chunk_waiters;
  }
  if (q->fault) return u->latched = q->fault;
  u->cur = (int32_t)q->free_chunks.back();
  q->free_chunks.pop_back();
  return EFES_OK;
}

// Back-pressure after a full chunk is handed over (q->mu held): while chunks are scarce, the
// writer waits for its upload to have fewer than `ahead` chunks queued or running.  An upload
// gains nothing from more (its chain takes one chunk per launch: one in the running launch, one
// in the launch queued behind it, one pending for the launch after), while a fast writer that
// grabs every free chunk leaves the other uploads nothing to put in the next launches.
// "Scarce" = no more free chunks than
// uploads OPEN now (each may need one to go on), not than the queue's capacity: the shared digest
// queue has max_uploads = chunks - 1, so a capacity test paced every digest always -- and its
// writers then slept and woke once per 64 KiB chunk (drainer at 512 files: 17-19 GiB/s paced from
// the first chunk, 24-26 with room to run ahead; profiles/r03_drain/drain_pace.log).
constexpr uint64_t kAhead = 3;
void pace(efes_upload* u, std::unique_lock<std::mutex>& lk) {
  efes_queue* q = u->q;
  const size_t open = (size_t)q->max_uploads - q->free_states.size();
  if (q->ahead && q->free_chunks.size() <= open)
    u->done.wait(lk, [&] { return q->fault || u->inflight < q->ahead; });
}

// memcpy into a staging chunk with non-temporal stores: the chunk is read next by the GPU over
// PCIe, not by this core, so the copy skips the read-for-ownership of every destination line and
// leaves the caller's cache alone (one DRAM write per byte instead of a read and a write).
// Ends with sfence: the stores are visible before the chunk is handed to the dispatcher.
void copy_to_staging(uint8_t* dst, const uint8_t* src, size_t n) {
  if (n < 4096) {
    memcpy(dst, src, n);
    return;
  }
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
  memcpy(dst, src, head);
  dst += head;
  src += head;
  n -= head;
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
  }
  memcpy(dst + i, src + i, n - i);
  _mm_sfence();
}

// copy_to_staging that also compares src with ref (same length) in the same pass; returns whether
// they are equal.  The copy is complete either way.
bool copy_to_staging_if_same(uint8_t* dst, const uint8_t* src, const uint8_t* ref, size_t n) {
  if (n < 4096) {
    memcpy(dst, src, n);
    return memcmp(src, ref, n) == 0;
  }
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
  bool same = memcmp(src, ref, head) == 0;
  memcpy(dst, src, head);
  dst += head;
  src += head;
  ref += head;
  n -= head;
  __m128i diff = _mm_setzero_si128();
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
    diff = _mm_or_si128(diff, _mm_or_si128(_mm_xor_si128(a, _mm_loadu_si128(reinterpret_cast<const __m128i*>(ref + i))),
                                           _mm_xor_si128(b, _mm_loadu_si128(reinterpret_cast<const __m128i*>(ref + i + 16)))));
    diff = _mm_or_si128(diff, _mm_or_si128(_mm_xor_si128(c, _mm_loadu_si128(reinterpret_cast<const __m128i*>(ref + i + 32))),
                                           _mm_xor_si128(d, _mm_loadu_si128(reinterpret_cast<const __m128i*>(ref + i + 48)))));
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
  }
  same = same && memcmp(src + i, ref + i, n - i) == 0;
  memcpy(dst + i, src + i, n - i);
  _mm_sfence();
  return same && _mm_movemask_epi8(_mm_cmpeq_epi8(diff, _mm_setzero_si128())) == 0xFFFF;
}

int wait_idle(efes_upload* u) {
  efes_queue* q = u->q;
  std::unique_lock<std::mutex> lk(q->mu);
  enqueue_current(u, lk);
  u->done.wait(lk, [&] { return u->inflight == 0; });
  return u->latched;
}

}  // namespace

extern "C" {

int efes_queue_create(efes_ctx* ctx, uint64_t chunk_bytes, uint32_t max_chunks, uint32_t max_uploads,
                      efes_queue** out) {
  // Every open upload may hold one partly filled chunk; with max_uploads < max_chunks at least
  // one chunk is always free or queued, so a writer waiting for a chunk always makes progress.
  if (!ctx || !out || max_chunks < 2 || max_uploads == 0 || max_uploads >= max_chunks) return EFES_ERR_ARG;
  return efes::queue_create_reclaiming(ctx, chunk_bytes, max_chunks, max_uploads, nullptr, nullptr, out);
}

}  // extern "C"

int efes::queue_create_reclaiming(efes_ctx* ctx, uint64_t chunk_bytes, uint32_t max_chunks, uint32_t max_uploads,
                                  bool (*reclaim)(void*, uint32_t), void* reclaim_arg, efes_queue** out) {
  if (!ctx || !out || max_chunks < 2 || max_uploads == 0 || (max_uploads >= max_chunks && !reclaim))
    return EFES_ERR_ARG;
  *out = nullptr;
  efes_queue* q = new (std::nothrow) efes_queue;
  if (!q) return EFES_ERR_NOMEM;
  q->ctx = ctx;
  q->chunk = chunk_bytes ? (chunk_bytes + 63) & ~uint64_t(63) : (uint64_t)1 << 20;
  q->nchunks = max_chunks;
  q->max_uploads = max_uploads;
  q->reclaim = reclaim;
  q->reclaim_arg = reclaim_arg;
  q->ahead = kAhead;
  DeviceGuard g(ctx->device);
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&q->h_slab), q->chunk * max_chunks, hipHostMallocMapped);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&q->z_slab), q->h_slab, 0);
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void**>(&q->h_states), kDevStateBytes * max_uploads, hipHostMallocMapped);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&q->z_states), q->h_states, 0);
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void**>(&q->h_jobs), 2 * sizeof(efes_job) * max_chunks, hipHostMallocDefault);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&q->d_jobs), 2 * sizeof(efes_job) * max_chunks);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    efes_queue_destroy(q);
    efes::clear_last_error();  // the caller may retry smaller (create_digest_queue): not a later launch's error
    return EFES_ERR_HIP;
  }
  for (uint32_t i = max_chunks; i-- > 0;) q->free_chunks.push_back(i);
  for (uint32_t i = max_uploads; i-- > 0;) q->free_states.push_back(i);
  try {
    q->th = std::thread([q] { q->run(); });
  } catch (...) {
    efes_queue_destroy(q);
    return EFES_ERR_NOMEM;
  }
  *out = q;
  return EFES_OK;
}

extern "C" {

void efes_queue_destroy(efes_queue* q) {
  if (!q) return;
  if (q->th.joinable()) {
    {
      std::lock_guard<std::mutex> lk(q->mu);
      q->stop = true;
    }
    q->work.notify_all();
    q->th.join();
  }
  DeviceGuard g(q->ctx->device);
  if (q->stream) (void)hipStreamSynchronize(q->stream);
  if (q->h_slab) (void)hipHostFree(q->h_slab);
  if (q->h_states) (void)hipHostFree(q->h_states);
  if (q->h_jobs) (void)hipHostFree(q->h_jobs);
  if (q->d_jobs) (void)hipFree(q->d_jobs);
  if (q->stream) (void)hipStreamDestroy(q->stream);
  delete q;
}

int efes_upload_open(efes_queue* q, uint32_t hashes, const efes_sha1_state* sha1, const efes_crc32_state* crc,
                     efes_upload** out) {
  bool no_slot = false;
  return efes::upload_open_slot(q, hashes, sha1, crc, out, &no_slot);
}

int efes_debug_fault_after(efes_ctx* ctx, uint64_t k) {
  if (!ctx) return EFES_ERR_ARG;
  efes_queue* q;
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->fault_after = k;  // for the digest queue if it is created later (efes_stream.cpp)
    q = ctx->digests;
  }
  if (q) efes::queue_set_fault_after(q, k);
  return EFES_OK;
}

int efes_queue_get_stats(efes_queue* q, efes_queue_stats* out) {
  if (!q || !out) return EFES_ERR_ARG;
  std::lock_guard<std::mutex> lk(q->mu);
  out->launches = q->n_launches;
  out->jobs = q->n_jobs;
  out->bytes = q->n_bytes;
  out->free_uploads = (uint32_t)q->free_states.size();
  out->max_uploads = q->max_uploads;
  return EFES_OK;
}

}  // extern "C"

int64_t efes::queue_free_slots(efes_queue* q) {
  std::lock_guard<std::mutex> lk(q->mu);
  return q->fault ? -1 : (int64_t)q->free_states.size();
}

void efes::queue_set_fault_after(efes_queue* q, uint64_t k) {
  std::lock_guard<std::mutex> lk(q->mu);
  q->inject_at = k;
  q->n_attempts = 0;
}

int efes::upload_open_slot(efes_queue* q, uint32_t hashes, const efes_sha1_state* sha1, const efes_crc32_state* crc,
                           efes_upload** out, bool* no_slot) {
  *no_slot = false;
  if (!q || !out || !hashes || (hashes & ~(EFES_HASH_SHA1 | EFES_HASH_CRC32))) return EFES_ERR_ARG;
  *out = nullptr;
  efes_upload* u = new (std::nothrow) efes_upload;
  if (!u) return EFES_ERR_NOMEM;
  u->q = q;
  u->hashes = hashes;
  {
    std::lock_guard<std::mutex> lk(q->mu);
    if (q->free_states.empty()) {
      delete u;
      *no_slot = true;
      return EFES_ERR_NOMEM;
    }
    u->dslot = q->free_states.back();
    q->free_states.pop_back();
  }
  if (sha1) {
    u->shadow = *sha1;
  } else {
    memset(&u->shadow, 0, sizeof u->shadow);
    efes_sha1_state_init(&u->shadow);  // NewSha1 (sha1.go:48-52)
  }
  // the slot is not in use by any kernel (its previous upload closed after its last job)
  uint8_t* st = q->h_states + (size_t)u->dslot * kDevStateBytes;
  memset(st, 0, kDevStateBytes);
  memcpy(st, &u->shadow, sizeof u->shadow);
  const uint32_t c = crc ? crc->crc : 0u;  // NewCRC32IEEE
  memcpy(st + kOffCrc, &c, 4);
  *out = u;
  return EFES_OK;
}

extern "C" {

int efes_upload_write(efes_upload* u, const void* p, size_t n) {
  if (!u || (!p && n)) return EFES_ERR_ARG;
  if (u->latched) return u->latched;
  u->reserved = 0;  // the bytes go where a reservation pointed
  const bool full_tail = u->shadow.nx == 64;
  const int rc = efes::replay_write(&u->shadow, static_cast<const uint8_t*>(p), n);
  if (rc) return u->latched = rc;  // the Go Write would panic (nx > 64)
  efes_queue* q = u->q;
  if (n == 0 && full_tail && (u->hashes & EFES_HASH_SHA1)) {
    // Go compresses a full pending tail even on an empty Write (sha1.go:61-69); run a
    // zero-length job so the device state follows.
    std::unique_lock<std::mutex> lk(q->mu);
    enqueue_current(u, lk);  // hands a partly filled chunk over; an empty reserved one stays
    if (u->cur < 0)
      if (int rc = take_chunk(u, lk)) return rc;
    u->fill = 0;
    enqueue_current(u, lk, true);
    return EFES_OK;
  }
  const uint8_t* src = static_cast<const uint8_t*>(p);
  // `cur`/`fill` belong to the thread that owns this upload, so filling the current chunk
  // takes no lock; the queue lock is taken only to get a chunk and to hand a full one over.
  while (n > 0) {
    if (u->cur < 0) {
      std::unique_lock<std::mutex> lk(q->mu);
      if (int rc = take_chunk(u, lk)) return rc;
      u->fill = 0;
    }
    const uint64_t take = std::min<uint64_t>(n, q->chunk - u->fill);
    copy_to_staging(q->h_slab + (size_t)u->cur * q->chunk + u->fill, src, take);
    u->fill += take;
    src += take;
    n -= take;
    if (u->fill == q->chunk) {
      std::unique_lock<std::mutex> lk(q->mu);
      enqueue_current(u, lk);
      pace(u, lk);
    }
  }
  return EFES_OK;
}

int efes_upload_reserve(efes_upload* u, size_t min_bytes, void** p, size_t* n) {
  if (!u || !p || !n) return EFES_ERR_ARG;
  if (u->latched) return u->latched;
  efes_queue* q = u->q;
  const uint64_t want = std::max<uint64_t>(1, std::min<uint64_t>(min_bytes, q->chunk));
  u->reserved = 0;
  if (u->cur >= 0 && q->chunk - u->fill < want) {  // too little room left: hand the chunk over
    std::unique_lock<std::mutex> lk(q->mu);
    enqueue_current(u, lk);
    pace(u, lk);  // the same per-upload back-pressure as a chunk filled by write/commit
  }
  if (u->cur < 0) {
    std::unique_lock<std::mutex> lk(q->mu);
    if (int rc = take_chunk(u, lk)) return rc;
    u->fill = 0;
  }
  *p = q->h_slab + (size_t)u->cur * q->chunk + u->fill;
  *n = (size_t)(q->chunk - u->fill);
  u->reserved = *n;
  return EFES_OK;
}

int efes_upload_commit(efes_upload* u, size_t k) {
  if (!u) return EFES_ERR_ARG;
  if (u->latched) return u->latched;
  if (k == 0) return efes_upload_write(u, nullptr, 0);  // Write(empty): sha1.go:61-69 still runs
  efes_queue* q = u->q;
  // only bytes the last reserve granted, once: a stale pointer would hash stale staging bytes
  if (u->cur < 0 || k > u->reserved || k > q->chunk - u->fill) return EFES_ERR_ARG;
  u->reserved = 0;
  const uint8_t* src = q->h_slab + (size_t)u->cur * q->chunk + u->fill;
  const int rc = efes::replay_write(&u->shadow, src, k);
  if (rc) return u->latched = rc;  // the Go Write would panic (nx > 64)
  u->fill += k;
  if (u->fill == q->chunk) {
    std::unique_lock<std::mutex> lk(q->mu);
    enqueue_current(u, lk);
    pace(u, lk);
  }
  return EFES_OK;
}

int efes_upload_flush(efes_upload* u) {
  if (!u) return EFES_ERR_ARG;
  return wait_idle(u);
}

int efes_upload_state(efes_upload* u, efes_sha1_state* sha1, efes_crc32_state* crc) {
  if (!u) return EFES_ERR_ARG;
  int rc = wait_idle(u);  // after this no job of the upload is in flight: the slot is final
  if (rc) return rc;
  const uint8_t* st = u->q->h_states + (size_t)u->dslot * kDevStateBytes;
  int32_t status;
  memcpy(&status, st + kOffStatus, 4);
  if (status != EFES_OK) return u->latched = status;
  if (sha1) {
    *sha1 = u->shadow;  // x/nx/len: Go's, from the replay
    memcpy(sha1->h, st, sizeof sha1->h);
  }
  if (crc) memcpy(&crc->crc, st + kOffCrc, 4);
  return EFES_OK;
}

int efes_upload_sum(efes_upload* u, uint8_t out[24]) {
  if (!u || !out) return EFES_ERR_ARG;
  if (u->latched) return u->latched;
  efes_queue* q = u->q;
  {
    // Through the dispatcher, after the upload's staged bytes: folded into the job of its last
    // chunk when that chunk is not in a launch yet, else a zero-length FINALIZE job.
    std::unique_lock<std::mutex> lk(q->mu);
    enqueue_current(u, lk);
    if (u->queued > 0) {  // only data chunks can be queued: a Sum returns after its job ran
      u->fold_sum = true;
    } else {
      q->pending.push_back(Pending{u, kNoChunk, 0});
      ++u->inflight;
      ++u->queued;
      q->work.notify_one();
    }
    u->done.wait(lk, [&] { return u->inflight == 0; });
    u->fold_sum = false;  // (a failed launch retires the chunk without running it)
  }
  if (u->latched) return u->latched;
  uint8_t* st = q->h_states + (size_t)u->dslot * kDevStateBytes;
  int32_t status;
  memcpy(&status, st + kOffStatus, 4);
  if (status != EFES_OK) {
    // EFES_ERR_STATE: checkSum panics (sha1.go:108) on a copy, so the digest itself stays
    // usable; clear the slot's status (no job of this upload is in flight) so a later
    // efes_upload_state / MarshalText does not latch this Sum's failure.
    const int32_t ok = EFES_OK;
    memcpy(st + kOffStatus, &ok, 4);
    return status;
  }
  memcpy(out, st + kOffSum, 24);
  return EFES_OK;
}

}  // extern "C"

namespace efes {
efes_sha1_state upload_shadow(const efes_upload* u) { return u->shadow; }

// ---- fused digest pairs (efes_internal.hpp; used by efes_stream.cpp) ----------------------------
// The caller owns the upload as its writer (cur/fill need no lock, as in efes_upload_write).
uint64_t upload_room(const efes_upload* u) {
  const uint64_t c = u->q->chunk;
  return u->cur >= 0 && u->fill < c ? c - u->fill : c;
}

void upload_set_shadow(efes_upload* u, const efes_sha1_state& shadow) { u->shadow = shadow; }

void upload_keep(efes_upload* u, uint32_t hashes) {
  std::lock_guard<std::mutex> lk(u->q->mu);
  u->hashes = hashes;
  if (!(hashes & EFES_HASH_SHA1)) {  // a CRC-only upload replays a NewSha1 state (never a panic state)
    memset(&u->shadow, 0, sizeof u->shadow);
    efes_sha1_state_init(&u->shadow);
  }
}

int upload_stage_if_same(efes_upload* u, const void* p, const void* ref, size_t n, uint64_t* off, bool* same) {
  *same = false;
  if (u->latched) return u->latched;
  efes_queue* q = u->q;
  if (u->cur >= 0 && u->fill + n > q->chunk) {  // no room: hand the (matched) chunk over first
    std::unique_lock<std::mutex> lk(q->mu);
    enqueue_current(u, lk);
    pace(u, lk);
  }
  if (u->cur < 0) {
    std::unique_lock<std::mutex> lk(q->mu);
    if (int rc = take_chunk(u, lk)) return rc;
    u->fill = 0;
  }
  // bytes past `fill` are never handed over, so a mismatch leaves nothing behind
  *same = copy_to_staging_if_same(q->h_slab + (size_t)u->cur * q->chunk + u->fill, static_cast<const uint8_t*>(p),
                                  static_cast<const uint8_t*>(ref), n);
  if (*same) {
    *off = u->fill;
    u->fill += n;
  }
  return EFES_OK;
}

int upload_confirm(efes_upload* u, const efes_sha1_state& shadow) {
  u->shadow = shadow;
  efes_queue* q = u->q;
  if (u->cur >= 0 && u->fill == q->chunk) {
    std::unique_lock<std::mutex> lk(q->mu);
    enqueue_current(u, lk);
    pace(u, lk);
  }
  return u->latched;
}

bool upload_partial(const efes_upload* u) { return u->cur >= 0 && u->fill > 0; }

bool upload_handover(efes_upload* u) {
  std::unique_lock<std::mutex> lk(u->q->mu);
  if (u->cur < 0 || u->fill == 0) return false;
  enqueue_current(u, lk);
  return true;
}

uint64_t queue_reclaims(efes_queue* q) {
  std::lock_guard<std::mutex> lk(q->mu);
  return q->n_reclaims;
}

}  // namespace efes

extern "C" {

void efes_upload_close(efes_upload* u) {
  if (!u) return;
  efes_queue* q = u->q;
  {
    std::unique_lock<std::mutex> lk(q->mu);
    if (u->cur >= 0) {  // staged but never flushed: drop it
      q->free_chunks.push_back((uint32_t)u->cur);
      u->cur = -1;
      q->freed.notify_all();
    }
    u->done.wait(lk, [&] { return u->inflight == 0; });  // kernels may still use the state slot
    q->free_states.push_back(u->dslot);
  }
  delete u;
}

}  // extern "C"
