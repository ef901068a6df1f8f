// efes_internal.hpp -- shared between the kernels (efes_kernels.hip) and the C ABI (efes_api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <condition_variable>
#include <list>
#include <mutex>

#include "../../include/efes_hash.h"
#include "../../include/efes_testing.h"

namespace efes {

// CRC-32/IEEE tables resident in HBM, copied into LDS by every workgroup.
//   slice8: the slicing-by-8 table of crc32.go:138-149 (slice8[0] == IEEETable).
//   shift[k][b][v]: the raw (un-inverted, reflected) CRC register v<<(8b) advanced over
//   (64 << k) zero bytes, i.e. multiplication by x^(8*64*2^k) mod P.  The register map
//   is GF(2)-linear, so advancing any register is the XOR of its four byte lookups.
//   Used to combine per-block CRCs (crc(A||B) = shift(crc(A), |B|) ^ crc(B)).
constexpr int kShiftLevels = 7;  // 64 B .. 4 KiB
struct Tables {
  uint32_t slice8[8][256];
  uint32_t shift[kShiftLevels][4][256];
};

void build_tables(Tables* t);  // host

// Position tables for the grouped kernels' block CRC: pos[p][b] = raw CRC register (from 0)
// after a 64-byte block whose only nonzero byte is b at position p.  The register map is
// GF(2)-linear, so a block's raw CRC is the XOR of its 64 bytes' entries -- 64 independent LDS
// lookups instead of slicing-by-8's chain of 8 dependent steps.  On the device the context's
// allocation holds Tables immediately followed by PosTables (64 KiB).
struct PosTables {
  uint32_t pos[64][256];
};
void build_pos_tables(const Tables* t, PosTables* p);  // host

// Go's sha1digest.Write bookkeeping of x/nx/len (sha1.go:58-79) without the compressions:
// the host replays it so exported states carry Go's exact tail bytes (efes_api.cpp).
int replay_write(efes_sha1_state* s, const uint8_t* p, size_t n);

// The host-replayed Go state (x/nx/len; h as opened) of an upload (efes_queue.cpp).
efes_sha1_state upload_shadow(const efes_upload* u);
// The context's shared queue for the Go-surface digests, created on first use
// (efes_stream.cpp); nullptr and *rc set on failure.
efes_queue* stream_queue(efes_ctx* ctx, int* rc);
// efes_upload_open that reports a full state-slot table as *no_slot (and EFES_ERR_NOMEM) so the
// digest layer can evict an idle digest and retry instead of failing (efes_queue.cpp).
int upload_open_slot(efes_queue* q, uint32_t hashes, const efes_sha1_state* sha1, const efes_crc32_state* crc32,
                     efes_upload** out, bool* no_slot);
// Free upload slots of q, or -1 once q has latched a device fault (placement skips it).
int64_t queue_free_slots(efes_queue* q);
// Test hook behind efes_debug_fault_after: q's k-th launch from now reports a device fault.
void queue_set_fault_after(efes_queue* q, uint64_t k);
// efes_queue_create for an owner that can hand idle uploads' partly filled chunks over: then
// max_uploads may exceed max_chunks.  When writers wait for a chunk while every chunk sits partly
// filled in uploads (nothing queued or running), the dispatcher thread calls reclaim(arg) -- with
// no lock held -- which hands over what it can (upload_handover) and returns whether it did.  The
// digest queue (efes_stream.cpp).
int queue_create_reclaiming(efes_ctx* ctx, uint64_t chunk_bytes, uint32_t max_chunks, uint32_t max_uploads,
                            bool (*reclaim)(void*, uint32_t want), void* reclaim_arg, efes_queue** out);
uint64_t queue_reclaims(efes_queue* q);  // reclaim calls so far

// ---- fused digest pairs (efes_stream.cpp on efes_queue.cpp) ----------------------------------
// io.MultiWriter(f, CRC32, Sha1) (filereceiver.go:208) hands the same bytes to a CRC digest and
// then to a SHA-1 digest; the digest layer binds such a pair to ONE upload that keeps both hashes.
// The leader's (CRC) Write waits in a scratch buffer; the follower's (SHA-1) identical Write is
// staged and checked against it in one pass, which confirms it.
// u keeps only `hashes` from now on (a member of a fused pair left it).
void upload_keep(efes_upload* u, uint32_t hashes);
// Stages n <= chunk bytes into u's current chunk WITHOUT handing them over (a current chunk without
// room is handed over first), with streaming stores that check the bytes against `ref` in the same
// pass: they count as staged (fill advances, *off = their offset in the chunk) only when *same.  No
// host replay.
int upload_stage_if_same(efes_upload* u, const void* p, const void* ref, size_t n, uint64_t* off, bool* same);
// Bytes the current staging chunk can still take (a whole chunk when there is none or it is full).
uint64_t upload_room(const efes_upload* u);
// Replaces the host-replayed Go state (x/nx/len) with one that differs at most in the stale bytes
// x[nx:] (a Write hashed in pieces gets the single Write's replay back).
void upload_set_shadow(efes_upload* u, const efes_sha1_state& shadow);
// The follower matched the staged bytes: its replayed Go state; a full chunk is handed over.
int upload_confirm(efes_upload* u, const efes_sha1_state& shadow);
// Hands u's partly filled current chunk to the dispatcher (the caller owns u: no call on it runs);
// false when u holds none.
bool upload_handover(efes_upload* u);
// Whether u holds a partly filled chunk (the caller owns u, as for upload_handover).
bool upload_partial(const efes_upload* u);

// Streaming digests (efes_stream.cpp) that hold an upload of a context's digest queue, oldest
// first: the candidates for eviction when a digest needs a state slot and none is free.  An
// entry is a digest holding an upload alone, or a fused pair holding one for both members.
struct Digest;
struct Fused;
struct OpenRef {
  Digest* d;
  Fused* f;
};
struct DigestRegistry {
  std::mutex mu;
  std::list<OpenRef> open;
  std::condition_variable released;  // a digest gave its upload back
};

// Launchers (host side, defined in efes_kernels.hip).
hipError_t launch_deep(const efes_job* jobs, uint32_t njobs, const Tables* tabs, hipStream_t s);
// exclusive: one workgroup (one wave per SIMD) per CU, so a long job's lane is never slowed by
// other waves on its SIMD.
hipError_t launch_wide(const efes_job* jobs, uint32_t njobs, const Tables* tabs, hipStream_t s,
                       bool exclusive = false, int cus = 256);
// Grouped DEEP: 64/G jobs per wave, G in {4, 8, 16, 32} (64 = launch_deep).  exclusive: each
// workgroup reserves all LDS of its CU, so no other workgroup shares the CU's SIMDs.
hipError_t launch_group(const efes_job* jobs, uint32_t njobs, int G, const Tables* tabs, hipStream_t s,
                        bool exclusive = false);
// Grouped DEEP fed by producer waves on the CU's other SIMDs; each workgroup owns its CU.
// expand = false: EFES_MODE_FED4 (2 chain waves + 2 producers, 32 jobs per CU); true:
// EFES_MODE_FED4E (3 chain waves that expand the schedule + 1 producer, 48 jobs per CU).
hipError_t launch_fed(const efes_job* jobs, uint32_t njobs, const Tables* tabs, hipStream_t s, bool expand);
hipError_t launch_fill(void* dst, size_t bytes, uint64_t seed, hipStream_t s);

// Span CRC (efes_crc_span.hip): CRC-32 of one long buffer on the whole GPU.  Bytes per lane per
// row (64: half a 128-B cache line, measured fastest), lanes per workgroup, the workgroup cap (the host passes each
// workgroup's combine operator as a kernel argument), and the per-context operator table
// lane_op[k] = x^(8*kSpanLine*k) mod P (the row shift depends on the launch's workgroup count and is
// built by each workgroup from its operator).
constexpr int kSpanLine = 64;  // bytes per lane per row (round 2 A/B of 16, 32, 48, 64, 128: profiles/r02_span/)
constexpr int kSpanLanes = 1024;
constexpr int kSpanMaxGroups = 512;
struct SpanTables {
  uint32_t lane_op[kSpanLanes];
};
void build_span_tables(SpanTables* t);  // host
hipError_t launch_crc_span(const void* data, uint64_t length, uint32_t* crc, const Tables* tabs, const SpanTables* span,
                           int cus, hipStream_t s);

// Lanes per job of a grouped-DEEP mode (EFES_MODE_GROUPn -> n), 0 for other modes.
inline int group_of_mode(int mode) {
  switch (mode) {
    case EFES_MODE_GROUP4: return 4;
    case EFES_MODE_GROUP8: return 8;
    case EFES_MODE_GROUP16: return 16;
    case EFES_MODE_GROUP32: return 32;
    default: return 0;
  }
}

constexpr int kDeepWaves = 4;  // waves per DEEP workgroup: one per SIMD

// HIP keeps a failed call's error as the calling thread's last error until it is read, so a launcher
// that reports hipGetLastError() after its launch clears it first: an earlier failure on the same
// thread that was handled (a pinned allocation retried at half size, a LDS attribute that could not be
// raised) must not come back as this launch's error.
inline void clear_last_error() { (void)hipGetLastError(); }

// Makes `dev` current for the scope and restores the caller's device (C ABI calls may come
// from any host thread, efes_hash.h).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace efes

// One GPU: its CRC tables in HBM and its own stream (efes_ctx_create).
struct efes_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int cus = 256;                  // compute units (efes_plan_batch's capacity)
  // streams of a planned batch's parts (efes_hash_submit_plan), one per part: never `stream`,
  // so a planned batch does not queue behind NULL-stream work of the context
  hipStream_t side[EFES_PLAN_MAX_PARTS] = {};
  hipEvent_t ev_fork = nullptr, ev_join[EFES_PLAN_MAX_PARTS] = {};
  hipStream_t part_stream(uint32_t i) const { return side[i]; }
  std::mutex plan_mu;             // one planned submit at a time uses the side streams/events
  efes::Tables* d_tabs = nullptr;
  efes::SpanTables* d_span = nullptr;  // operators of the span CRC (efes_crc32_span)
  std::mutex mu;                  // guards the lazy creation of `digests` and `copy`
  efes_queue* digests = nullptr;  // shared queue of the streaming digests (efes_stream.cpp)
  hipStream_t copy = nullptr;     // efes_hash_host's H2D stream (own_queue_stream), created on first use
  std::mutex copy_mu;             // one efes_hash_host at a time on `copy`
  efes::DigestRegistry dreg;      // the digests holding an upload of `digests`
  uint64_t fault_after = 0;       // test hook (efes_debug_fault_after): the digest queue's k-th launch faults
};

namespace efes {

// A stream with a hardware queue of its own, for work that must run beside the process's other
// streams: HIP spreads ALL of a process's streams over GPU_MAX_HW_QUEUES (4) queues, so two
// ordinary streams may share one and serialize.  A stream created with a CU mask gets a queue of
// its own (the mask is a queue property); the mask is every CU, so placement is unchanged.
// Used for the planned batch's part streams and efes_hash_host's copy stream.  HIP creates CU-masked streams as blocking streams
// (hipStreamDefault): they also order against the legacy NULL stream, which adds ordering,
// never removes it.
hipError_t own_queue_stream(const efes_ctx* ctx, hipStream_t* out);

// Kernel shape for jobs whose bytes are read over PCIe in place (pinned, device-mapped host
// memory): the lowest-latency shape that keeps each job's reads long -- DEEP (4 KiB per job per
// super-step), then grouped DEEP with as many lanes per job as fit (G*64 contiguous bytes);
// never WIDE (scattered 64-B lane reads) nor FED4 (256 B per job, like GROUP4, at 32 jobs per CU).
// (Measured with 2048 uploads in flight: grouped 35.3-36.5 GiB/s vs 32.0-34.8 for DEEP only.)
inline int pcie_mode(const efes_ctx* ctx, uint32_t njobs) {
  const uint64_t simds = 4ull * (ctx ? (uint64_t)ctx->cus : 256ull), n = njobs;
  if (n <= simds) return EFES_MODE_DEEP;
  if (n <= 2 * simds) return EFES_MODE_GROUP32;
  if (n <= 4 * simds) return EFES_MODE_GROUP16;
  if (n <= 8 * simds) return EFES_MODE_GROUP8;
  return EFES_MODE_GROUP4;
}

}  // namespace efes
