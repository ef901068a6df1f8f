// efes_ingest.cpp -- host-resident ingest: messages that start in host memory.
//
// The reference hashes bytes as they come off a socket (filereceiver.go:208-209, io.Copy of
// the PATCH body through MultiWriter(file, CRC32, Sha1)), i.e. the data path starts in host
// memory.  efes_hash_host() streams a batch of host-resident messages through HBM in
// segments: segment s of every message is copied H2D (pinned hipMemcpyAsync on a copy stream)
// into one of two device slots while segment s-1 is hashed on the context stream; the SHA-1 /
// CRC-32 states stay on the device between segments (exactly the per-PATCH resume of
// filereceiver.go:182-226), and only states and 24-byte sums come back.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "efes_internal.hpp"

using efes::DeviceGuard;

namespace {

struct HipBuf {  // device allocation released on scope exit
  void* p = nullptr;
  ~HipBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t n) { return hipMalloc(&p, n ? n : 1); }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

struct PinnedBuf {  // pinned host allocation released on scope exit
  void* p = nullptr;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t alloc(size_t n) { return hipHostMalloc(&p, n ? n : 1, hipHostMallocDefault); }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

struct Event {
  hipEvent_t e = nullptr;
  ~Event() {
    if (e) (void)hipEventDestroy(e);
  }
};

// Copies segment [off, off+len) of the active jobs into their slots: consecutive jobs whose
// host addresses advance by a constant stride become one hipMemcpy2DAsync (one call for a
// whole packed batch); anything else falls back to one hipMemcpyAsync per job.
hipError_t copy_segment(const std::vector<const uint8_t*>& src, const std::vector<uint64_t>& len, uint8_t* dst_base,
                        uint64_t seg, hipStream_t s) {
  const size_t n = src.size();
  size_t i = 0;
  while (i < n) {
    size_t j = i + 1;
    if (j < n && len[j] == len[i]) {
      const intptr_t stride = src[j] - src[i];
      while (j + 1 < n && len[j + 1] == len[i] && src[j + 1] - src[j] == stride) ++j;
      if (stride > 0 && (uint64_t)stride >= len[i]) {
        ++j;
        hipError_t e = hipMemcpy2DAsync(dst_base + i * seg, seg, src[i], (size_t)stride, len[i], j - i,
                                        hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return e;
        i = j;
        continue;
      }
      j = i + 1;
    }
    if (len[i]) {
      hipError_t e = hipMemcpyAsync(dst_base + i * seg, src[i], len[i], hipMemcpyHostToDevice, s);
      if (e != hipSuccess) return e;
    }
    i = j;
  }
  return hipSuccess;
}

}  // namespace

extern "C" {

int efes_host_alloc(efes_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out) return EFES_ERR_ARG;
  DeviceGuard g(ctx->device);
  return hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocMapped) == hipSuccess ? EFES_OK : EFES_ERR_HIP;
}

int efes_host_free(efes_ctx* ctx, void* p) {
  if (!ctx) return EFES_ERR_ARG;
  DeviceGuard g(ctx->device);
  return hipHostFree(p) == hipSuccess ? EFES_OK : EFES_ERR_HIP;
}

// EFES_HOST_ZERO_COPY: the data is pinned, device-mapped host memory (efes_host_alloc); one DEEP
// (or grouped-DEEP, efes::pcie_mode) launch reads it in place over PCIe (coalesced 4 KiB per wave, prefetched a super-step ahead
// of the chain) -- no staging, no segments.
static int hash_host_mapped(efes_ctx* ctx, const efes_job* jobs, uint32_t n, efes_host_stats* stats) {
  std::vector<efes_job> hj(jobs, jobs + n);
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    total += jobs[i].length;
    if (!jobs[i].length) continue;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, jobs[i].data) != hipSuccess || !attr.devicePointer) return EFES_ERR_ARG;
    hj[i].data = attr.devicePointer;  // device address of this exact host byte
  }
  HipBuf d_states, d_crcs, d_sums, d_status, d_jobs;
  hipError_t e = d_states.alloc(sizeof(efes_sha1_state) * n);
  if (e == hipSuccess) e = d_crcs.alloc(sizeof(efes_crc32_state) * n);
  if (e == hipSuccess) e = d_sums.alloc(24ull * n);
  if (e == hipSuccess) e = d_status.alloc(sizeof(int32_t) * n);
  if (e == hipSuccess) e = d_jobs.alloc(sizeof(efes_job) * n);
  if (e != hipSuccess) return EFES_ERR_HIP;
  std::vector<efes_sha1_state> hs(n);
  std::vector<efes_crc32_state> hc(n);
  std::vector<uint8_t> hsum(24ull * n);
  std::vector<int32_t> hst(n, EFES_OK);
  for (uint32_t i = 0; i < n; ++i) {
    if (jobs[i].sha1) hs[i] = *jobs[i].sha1;
    else memset(&hs[i], 0, sizeof hs[i]);
    hc[i].crc = jobs[i].crc32 ? jobs[i].crc32->crc : 0u;
    hj[i].sha1 = jobs[i].sha1 ? d_states.as<efes_sha1_state>() + i : nullptr;
    hj[i].crc32 = jobs[i].crc32 ? d_crcs.as<efes_crc32_state>() + i : nullptr;
    hj[i].sum = (jobs[i].flags & EFES_JOB_FINALIZE) ? d_sums.as<uint8_t>() + 24ull * i : nullptr;
    hj[i].status = d_status.as<int32_t>() + i;
  }
  hipStream_t s = ctx->stream;
  e = hipMemcpyAsync(d_states.p, hs.data(), sizeof(efes_sha1_state) * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(d_crcs.p, hc.data(), sizeof(efes_crc32_state) * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(d_status.p, hst.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(d_jobs.p, hj.data(), sizeof(efes_job) * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return EFES_ERR_HIP;
  const auto t0 = std::chrono::steady_clock::now();
  int rc = efes_hash_submit_mode(ctx, d_jobs.as<efes_job>(), n, s, efes::pcie_mode(ctx, n));
  if (rc) return rc;
  e = hipMemcpyAsync(hs.data(), d_states.p, sizeof(efes_sha1_state) * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(hc.data(), d_crcs.p, sizeof(efes_crc32_state) * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(hsum.data(), d_sums.p, 24ull * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(hst.data(), d_status.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return EFES_ERR_DEVICE_FAULT;
  for (uint32_t i = 0; i < n; ++i) {
    if (jobs[i].sha1) *jobs[i].sha1 = hs[i];
    if (jobs[i].crc32) *jobs[i].crc32 = hc[i];
    if (jobs[i].sum && (jobs[i].flags & EFES_JOB_FINALIZE)) memcpy(jobs[i].sum, hsum.data() + 24ull * i, 24);
    if (jobs[i].status) *jobs[i].status = hst[i];
  }
  if (stats) {
    stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    stats->bytes = total;
    stats->segments = 1;
  }
  return EFES_OK;
}

int efes_hash_host(efes_ctx* ctx, const efes_job* jobs, uint32_t n, uint64_t segment_bytes, efes_host_stats* stats) {
  if (!ctx || (!jobs && n) || n > EFES_MAX_JOBS) return EFES_ERR_ARG;
  if (stats) memset(stats, 0, sizeof *stats);
  if (n == 0) return EFES_OK;
  for (uint32_t i = 0; i < n; ++i)
    if ((jobs[i].flags & ~(EFES_JOB_FINALIZE | EFES_JOB_INIT)) || (!jobs[i].data && jobs[i].length) ||
        ((jobs[i].flags & EFES_JOB_FINALIZE) && !jobs[i].sum))
      return EFES_ERR_ARG;
  if (segment_bytes == EFES_HOST_ZERO_COPY) {
    DeviceGuard g(ctx->device);
    return hash_host_mapped(ctx, jobs, n, stats);
  }
  // 256 KiB: short segments keep the hash of the last one (the exposed tail) small; measured
  // 50.8 GiB/s against 45.4 at 1 MiB for 1024 x 4 MiB (H2D ceiling 57.6 GB/s, mb_h2d.hip).
  const uint64_t seg = segment_bytes ? (segment_bytes + 63) & ~uint64_t(63) : (uint64_t)256 << 10;
  uint64_t nseg = 1;
  for (uint32_t i = 0; i < n; ++i) nseg = std::max<uint64_t>(nseg, (jobs[i].length + seg - 1) / seg);

  DeviceGuard g(ctx->device);
  // Device side: n states, crcs, sums, status; two data slots of n x seg bytes; two job arrays.
  HipBuf d_states, d_crcs, d_sums, d_status, d_ring, d_jobs;
  PinnedBuf h_states, h_crcs, h_sums, h_status, h_jobs;
  hipError_t e = d_states.alloc(sizeof(efes_sha1_state) * n);
  if (e == hipSuccess) e = d_crcs.alloc(sizeof(efes_crc32_state) * n);
  if (e == hipSuccess) e = d_sums.alloc(24ull * n);
  if (e == hipSuccess) e = d_status.alloc(sizeof(int32_t) * n);
  if (e == hipSuccess) e = d_ring.alloc(2 * seg * n);
  if (e == hipSuccess) e = d_jobs.alloc(2 * sizeof(efes_job) * n);
  if (e == hipSuccess) e = h_states.alloc(sizeof(efes_sha1_state) * n);
  if (e == hipSuccess) e = h_crcs.alloc(sizeof(efes_crc32_state) * n);
  if (e == hipSuccess) e = h_sums.alloc(24ull * n);
  if (e == hipSuccess) e = h_status.alloc(sizeof(int32_t) * n);
  if (e == hipSuccess) e = h_jobs.alloc(2 * sizeof(efes_job) * n);
  if (e != hipSuccess) return EFES_ERR_HIP;

  // The context's copy stream: a hardware queue of its own, so the copies never wait behind the
  // hashing on a shared queue; made once per context (every CU-masked stream holds a queue, and
  // the GPU's queue slots are few).  One efes_hash_host at a time per context uses it.
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->copy && efes::own_queue_stream(ctx, &ctx->copy) != hipSuccess) ctx->copy = nullptr;
    if (!ctx->copy) return EFES_ERR_HIP;
  }
  std::unique_lock<std::mutex> copy_lk(ctx->copy_mu);
  struct CopyStream {  // drained on every exit, before the buffers above are freed
    hipStream_t s;
    ~CopyStream() { (void)hipStreamSynchronize(s); }
  } copy{ctx->copy};
  Event copied[2], hashed[2];
  e = hipSuccess;
  for (int k = 0; k < 2 && e == hipSuccess; ++k) {
    e = hipEventCreateWithFlags(&copied[k].e, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&hashed[k].e, hipEventDisableTiming);
  }
  if (e != hipSuccess) return EFES_ERR_HIP;
  hipStream_t comp = ctx->stream;

  // Initial states (not read by the kernel for EFES_JOB_INIT jobs).
  for (uint32_t i = 0; i < n; ++i) {
    efes_sha1_state* hs = h_states.as<efes_sha1_state>() + i;
    if (jobs[i].sha1) *hs = *jobs[i].sha1;
    else memset(hs, 0, sizeof *hs);
    h_crcs.as<efes_crc32_state>()[i].crc = jobs[i].crc32 ? jobs[i].crc32->crc : 0u;
    h_status.as<int32_t>()[i] = EFES_OK;
  }
  e = hipMemcpyAsync(d_states.p, h_states.p, sizeof(efes_sha1_state) * n, hipMemcpyHostToDevice, copy.s);
  if (e == hipSuccess) e = hipMemcpyAsync(d_crcs.p, h_crcs.p, sizeof(efes_crc32_state) * n, hipMemcpyHostToDevice, copy.s);
  if (e == hipSuccess) e = hipMemcpyAsync(d_status.p, h_status.p, sizeof(int32_t) * n, hipMemcpyHostToDevice, copy.s);
  if (e == hipSuccess) e = hipMemsetAsync(d_sums.p, 0, 24ull * n, copy.s);
  if (e != hipSuccess) return EFES_ERR_HIP;

  const auto t0 = std::chrono::steady_clock::now();  // the pipeline proper (allocations excluded)
  std::vector<const uint8_t*> src;
  std::vector<uint64_t> len;
  uint64_t total = 0;
  for (uint64_t s = 0; s < nseg; ++s) {
    const int slot = (int)(s & 1);
    if (s >= 2 && hipEventSynchronize(hashed[slot].e) != hipSuccess) return EFES_ERR_DEVICE_FAULT;
    efes_job* hj = h_jobs.as<efes_job>() + (size_t)slot * n;
    efes_job* dj = d_jobs.as<efes_job>() + (size_t)slot * n;
    uint8_t* ring = d_ring.as<uint8_t>() + (size_t)slot * seg * n;
    src.clear();
    len.clear();
    uint32_t active = 0;
    for (uint32_t i = 0; i < n; ++i) {
      const uint64_t L = jobs[i].length, off = s * seg;
      if (off >= L && !(s == 0 && L == 0)) continue;  // this job is done
      const uint64_t m = std::min<uint64_t>(seg, L - off);
      const bool last = off + m == L;
      efes_job& j = hj[active];
      j.data = ring + (size_t)active * seg;
      j.length = m;
      j.sha1 = jobs[i].sha1 ? d_states.as<efes_sha1_state>() + i : nullptr;
      j.crc32 = jobs[i].crc32 ? d_crcs.as<efes_crc32_state>() + i : nullptr;
      j.sum = last && (jobs[i].flags & EFES_JOB_FINALIZE) ? d_sums.as<uint8_t>() + 24ull * i : nullptr;
      j.status = d_status.as<int32_t>() + i;
      j.flags = (s == 0 ? (jobs[i].flags & EFES_JOB_INIT) : 0u) | (j.sum ? EFES_JOB_FINALIZE : 0u);
      j._reserved = 0;
      src.push_back(static_cast<const uint8_t*>(jobs[i].data) + off);
      len.push_back(m);
      total += m;
      ++active;
    }
    e = copy_segment(src, len, ring, seg, copy.s);
    if (e == hipSuccess) e = hipMemcpyAsync(dj, hj, sizeof(efes_job) * active, hipMemcpyHostToDevice, copy.s);
    if (e == hipSuccess) e = hipEventRecord(copied[slot].e, copy.s);
    if (e == hipSuccess) e = hipStreamWaitEvent(comp, copied[slot].e, 0);
    if (e != hipSuccess) return EFES_ERR_HIP;
    const int rc = efes_hash_submit(ctx, dj, active, comp);
    if (rc != EFES_OK) return rc;
    if (hipEventRecord(hashed[slot].e, comp) != hipSuccess) return EFES_ERR_HIP;
  }
  e = hipMemcpyAsync(h_states.p, d_states.p, sizeof(efes_sha1_state) * n, hipMemcpyDeviceToHost, comp);
  if (e == hipSuccess) e = hipMemcpyAsync(h_crcs.p, d_crcs.p, sizeof(efes_crc32_state) * n, hipMemcpyDeviceToHost, comp);
  if (e == hipSuccess) e = hipMemcpyAsync(h_sums.p, d_sums.p, 24ull * n, hipMemcpyDeviceToHost, comp);
  if (e == hipSuccess) e = hipMemcpyAsync(h_status.p, d_status.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, comp);
  if (e == hipSuccess) e = hipStreamSynchronize(comp);
  if (e != hipSuccess) return EFES_ERR_DEVICE_FAULT;
  for (uint32_t i = 0; i < n; ++i) {
    if (jobs[i].sha1) *jobs[i].sha1 = h_states.as<efes_sha1_state>()[i];
    if (jobs[i].crc32) *jobs[i].crc32 = h_crcs.as<efes_crc32_state>()[i];
    if (jobs[i].sum && (jobs[i].flags & EFES_JOB_FINALIZE)) memcpy(jobs[i].sum, h_sums.as<uint8_t>() + 24ull * i, 24);
    if (jobs[i].status) *jobs[i].status = h_status.as<int32_t>()[i];
  }
  if (stats) {
    stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    stats->bytes = total;
    stats->segments = (uint32_t)nseg;
  }
  return EFES_OK;
}

}  // extern "C"
