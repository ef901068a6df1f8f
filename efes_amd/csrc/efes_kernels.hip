// efes_kernels.hip -- MI355X (gfx950) kernels for efes' per-chunk SHA-1 + CRC-32/IEEE.
//
// Semantics: every efes_job is one `Write(p)` of the reference's
//   sha1digest.Write  (/root/reference/sha1.go:58-79)  and
//   crc32digest.Write (/root/reference/crc32.go:76-86 -> slicingUpdate :153-169)
// into a device-resident state, optionally followed by Sum (sha1.go:82-120 checkSum,
// crc32.go:88-93).  Go panics (nx > 64 at Write, d.nx != 0 in checkSum) become
// EFES_ERR_STATE.  The tail buffer x is updated byte-for-byte as Go does, stale bytes
// included, so MarshalText (sha1_efes.go:25-38) of a device state equals Go's.
//
// Two kernel shapes (DESIGN_NOTES.md):
//   DEEP: one chain wavefront per job.  SHA-1 is a strict chain of 64-byte compressions, so a
//         job's speed is one wave's issue rate.  A producer wave on the same SIMD loads 64
//         consecutive blocks (4 KiB, coalesced), computes their CRC-32 partials (combined by a
//         6-level GF(2) shift tree) and expands each block's schedule W[i]+K[i]; the chain wave
//         copies its lane's block W+K from LDS into registers, the 80-round chain of block i
//         runs in lane i (5 VALU per round) and the chaining value steps to lane i+1 by DPP:
//         405 chain VALU + 5 DPP moves per block.
//   GROUPn: 64/n jobs per wavefront (n lanes each), the DEEP chain shared by the jobs.
//   WIDE: one lane per job (64 jobs per wave), schedule inline, CRC fused per lane.
//         Throughput shape for many concurrent jobs.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "efes_internal.hpp"
#include "sha1_device.hpp"

#ifdef EFES_CHECKED
// Debug build only (tools/debug_checked.py): every data load is range-checked against the
// job's [p, p+plen); a violation is printed and redirected to p so the kernel cannot fault.
#include <stdio.h>
#define EFES_RANGE(ptr, nbytes, lo, len, tag)                                                               \
  (((const uint8_t*)(ptr) < (const uint8_t*)(lo) ||                                                          \
    (const uint8_t*)(ptr) + (nbytes) > (const uint8_t*)(lo) + (len))                                         \
       ? (printf("EFES_CHECKED %s: ptr=%p n=%d lo=%p len=%llu blk=%d thr=%d\n", tag, (const void*)(ptr),        \
                 (int)(nbytes), (const void*)(lo), (unsigned long long)(len), (int)blockIdx.x, (int)threadIdx.x), \
          (decltype(ptr))(lo))                                                                              \
       : (ptr))
#else
#define EFES_RANGE(ptr, nbytes, lo, len, tag) (ptr)
#endif

namespace efes {

// ------------------------------------------------------------------ CRC-32 helpers
// Raw (register-level) reflected CRC: Go's update is ~raw(~crc, p) (crc32.go:123,127,155,165).
__device__ __forceinline__ uint32_t crc_byte(const uint32_t* __restrict__ t0, uint32_t crc, uint32_t b) {
  return t0[(crc ^ b) & 0xffu] ^ (crc >> 8);  // crc32.go:125
}

__device__ __forceinline__ uint32_t crc_shift(const uint32_t (&s)[4][256], uint32_t v) {
  return s[0][v & 0xffu] ^ s[1][(v >> 8) & 0xffu] ^ s[2][(v >> 16) & 0xffu] ^ s[3][v >> 24];
}

// Slicing-by-8 over 64 bytes held as 16 little-endian words (crc32.go:157-161).
__device__ __forceinline__ uint32_t crc_words_raw(const uint32_t (&t)[8][256], uint32_t crc, const uint32_t (&le)[16]) {
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const uint32_t hi = le[2 * s + 1];
    crc ^= le[2 * s];
    // eight lookups folded with three-input XORs (v_bitop3_b32 0x96): 4 VALU instead of 7
    const uint32_t a = __builtin_amdgcn_bitop3_b32(t[0][hi >> 24], t[1][(hi >> 16) & 0xffu], t[2][(hi >> 8) & 0xffu], 0x96);
    const uint32_t b = __builtin_amdgcn_bitop3_b32(t[3][hi & 0xffu], t[4][crc >> 24], t[5][(crc >> 16) & 0xffu], 0x96);
    crc = __builtin_amdgcn_bitop3_b32(a, b, t[6][(crc >> 8) & 0xffu] ^ t[7][crc & 0xffu], 0x96);
  }
  return crc;
}

// __builtin_amdgcn_readfirstlane returns int: go through uint32_t so the low half of a
// 64-bit value is zero-extended (a sign-extended low half corrupts pointers >= 2^31).
__device__ __forceinline__ uint32_t uniform32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  return (uint64_t)uniform32((uint32_t)v) | ((uint64_t)uniform32((uint32_t)(v >> 32)) << 32);
}

// Orders this wave's LDS stores before its later LDS loads from other lanes.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Big-endian word k (bytes 4k..4k+3) of a byte array in LDS.
__device__ __forceinline__ uint32_t be_word_lds(const uint8_t* b, int k) {
  return (uint32_t)b[4 * k] << 24 | (uint32_t)b[4 * k + 1] << 16 | (uint32_t)b[4 * k + 2] << 8 | b[4 * k + 3];
}

// Message bytes are always device global memory: address-space-1 pointers make the compiler
// emit global_load (counted by vmcnt only) instead of flat_load, which also counts in
// lgkmcnt and would make every LDS wait of the chain wait for the in-flight prefetch too.
#define EFES_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ const EFES_GLOBAL T* gptr(const T* p) {
  return (const EFES_GLOBAL T*)p;
}
__device__ __forceinline__ uint32_t ldg_u8(const uint8_t* p) { return *gptr(p); }

// Load 64 bytes at an arbitrary device address as 16 little-endian words.
// kAligned16: the address is 16-byte aligned (4 x global_load_dwordx4).
// Otherwise: 16 (or 17) naturally aligned dword loads funnel-shifted by v_alignbyte.  The
// 17th dword is loaded only when the block is misaligned, and then it holds a byte of the
// block, so it never touches a page the block does not touch.
template <bool kAligned16>
__device__ __forceinline__ void load_block_le(const uint8_t* src, uint32_t (&le)[16]) {
  if constexpr (kAligned16) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const EFES_GLOBAL v4u* s = gptr(reinterpret_cast<const v4u*>(src));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const v4u v = s[q];
      le[4 * q] = v.x; le[4 * q + 1] = v.y; le[4 * q + 2] = v.z; le[4 * q + 3] = v.w;
    }
  } else {
    const uintptr_t a = reinterpret_cast<uintptr_t>(src);
    const EFES_GLOBAL uint32_t* s = gptr(reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3));
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t d[17];
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = s[k];
    d[16] = sh ? s[16] : 0u;
#pragma unroll
    for (int k = 0; k < 16; ++k) le[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
  }
}

// ================================================================== DEEP kernel

constexpr int kGroupMaxJobs = 16;  // jobs per wave in the grouped DEEP kernel (G = 4)

// One job's running state between the phases of a DEEP wave (head -> bulk -> rest),
// parked in LDS while the wave's other jobs run their phases.
struct DeepMsg {
  uint32_t h[5];
  uint32_t crc_raw;
  const uint8_t* q;  // first bulk byte (p + pos)
  uint64_t pos;      // bytes consumed by the head
  uint64_t nbulk;    // whole blocks after the head
  uint64_t done;     // bulk blocks already hashed by the joint phase
  int64_t nx_new;
  uint32_t live;     // 0: no job, or Go panicked in the head
  uint32_t joint;    // takes part in the grouped kernel's current joint round
};

struct DeepLDS {
  Tables tab;                                    // 36 KiB
  PosTables pos;                                 // 64 KiB, follows tab (same order as in HBM)
  uint8_t xs[kDeepWaves][kGroupMaxJobs][64];     // each job's tail buffer x (sha1.go:31)
  uint8_t fin[kDeepWaves][192];                  // padding assembly for checkSum
  DeepMsg msg[kDeepWaves][kGroupMaxJobs];
};
static_assert(offsetof(DeepLDS, pos) == sizeof(Tables), "DeepLDS copies Tables+PosTables in one sweep");

struct DeepJob {
  const uint8_t* p;
  uint64_t plen;
  efes_sha1_state* st;
  efes_crc32_state* cs;
  uint8_t* sum;
  int32_t* status;
  uint32_t flags;
};

// Bulk blocks q[0 .. 64*nbulk) of one job by one wave alone (the one-job path, used for a
// grouped wave's left-over blocks through deep_rest).  The DEEP kernel proper splits this same super-step between a producer and a chain wave
// (pipe_produce / pipe_consume below).  Per super-step of up to 64 blocks (4 KiB, one coalesced
// load per lane, prefetched a super-step ahead): lane off+i holds block i, computes its raw
// CRC-32 (slicing-by-8, LDS tables) and expands its schedule W[t]+K[t] into its own 80 VGPRs.
// The block CRCs are merged by a 6-level GF(2) shift tree.  Then the wave runs the SHA-1
// chain 64 times with the SAME register names: in iteration i only lane off+i computes the
// real compression (its W+K registers hold block i) and the other lanes compute garbage in
// the same instructions, so the chain reads W+K straight from registers -- no LDS traffic.
// The chaining value moves from lane off+i to lane off+i+1 by DPP wave_shr:1 (5 v_mov_dpp
// per block).  Measured against W+K read back from LDS by ds_read_b128: 48.1 vs 52.7 ms per
// 1024 x 4 MiB (DESIGN_NOTES.md §4).
template <bool kAligned16>
__device__ void deep_bulk(const Tables& T, int lane, const uint8_t* q, uint64_t nbulk, bool do_sha, bool do_crc,
                          uint32_t (&h)[5], uint32_t& crc_raw) {
  uint32_t le[16];
  // Blocks are right-aligned in the lanes (lane 64-nb+i holds block i) so that the zero
  // CRCs of idle lanes lead the tree, and the last block of every super-step is in lane 63.
  uint64_t b0 = 0;
  int nb = (int)(nbulk < 64 ? nbulk : 64);
  {
    const int bi = lane - (64 - nb);
#pragma unroll
    for (int k = 0; k < 16; ++k) le[k] = 0;
    if (bi >= 0) load_block_le<kAligned16>(EFES_RANGE(q + 64 * (uint64_t)bi, 64, q, 64 * nbulk, "deep-bulk0"), le);
  }
  while (b0 < nbulk) {
    if (do_crc) {
      uint32_t r = crc_words_raw(T.slice8, 0u, le);  // raw CRC of this lane's block, register 0
#pragma unroll
      for (int k = 0; k < 6; ++k) {  // crc(A||B) = shift(crc(A), |B|) ^ crc(B), |B| = 64<<k bytes
        const uint32_t o = __shfl_xor(r, 1 << k);
        const bool right = (lane >> k) & 1;
        r = crc_shift(T.shift[k], right ? o : r) ^ (right ? r : o);
      }
      if (nb == 64) {
        crc_raw = crc_shift(T.shift[6], crc_raw);
      } else {
#pragma unroll
        for (int k = 0; k < 6; ++k)
          if ((nb >> k) & 1) crc_raw = crc_shift(T.shift[k], crc_raw);
      }
      crc_raw ^= r;
    }
    uint32_t x[80];  // this lane's block: W[t] + K[t], t = 0..79
    if (do_sha) {
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = bswap(le[k]);
      expand_wk(w, x);
    }
    // Prefetch the next super-step's blocks; they land while the chain runs.
    const uint64_t b1 = b0 + (uint64_t)nb;
    const int nb1 = (int)((nbulk - b1) < 64 ? (nbulk - b1) : 64);
    if (b1 < nbulk) {
      const int bj = lane - (64 - nb1);
#pragma unroll
      for (int k = 0; k < 16; ++k) le[k] = 0;
      if (bj >= 0) load_block_le<kAligned16>(EFES_RANGE(q + 64 * (b1 + (uint64_t)bj), 64, q, 64 * nbulk, "deep-bulk1"), le);
    }
    if (do_sha) {
      uint32_t hv[5] = {h[0], h[1], h[2], h[3], h[4]}, hs[5];
      auto block = [&]() {
        chain_block(hv, x, hs);  // sha1.go:193-197 folded in
#pragma unroll
        for (int k = 1; k < 6; ++k) hv[k % 5] = (uint32_t)__builtin_amdgcn_mov_dpp((int)hs[k % 5], 0x138, 0xf, 0xf, true);  // wave_shr:1, h0 (round 79's v_add3) last
      };
      const int nbu = (int)uniform32((uint32_t)nb);
      int j = 0;
      for (; j + 2 <= nbu; j += 2) { block(); block(); }  // unrolled by two: half the loop overhead
      if (j < nbu) block();
#pragma unroll
      for (int k = 0; k < 5; ++k) h[k] = (uint32_t)__builtin_amdgcn_readlane((int)hs[k], 63);
    }
    b0 = b1;
    nb = nb1;
  }
}

// Head of one Write (sha1.go:58-69): load the state, complete a pending x[:nx].  Returns the
// job's running state; live == 0 when Go would panic (status already written).
__device__ DeepMsg deep_head(const Tables& T, int lane, const DeepJob& J, uint8_t* xs) {
  const bool do_sha = J.st != nullptr, do_crc = J.cs != nullptr;
  DeepMsg M{};
  uint32_t (&h)[5] = M.h;
  int64_t nx = 0;
  const bool init = (J.flags & EFES_JOB_INIT) != 0;
  if (do_sha && init) {  // NewSha1(): zero value + Reset (sha1.go:36-52)
    h[0] = kIV0; h[1] = kIV1; h[2] = kIV2; h[3] = kIV3; h[4] = kIV4;
    if (lane < 16) reinterpret_cast<uint32_t*>(xs)[lane] = 0u;
  } else if (do_sha) {
#pragma unroll
    for (int k = 0; k < 5; ++k) h[k] = uniform32(J.st->h[k]);
    nx = (int64_t)uniform64((uint64_t)J.st->nx);
    if (lane < 16) reinterpret_cast<uint32_t*>(xs)[lane] = reinterpret_cast<const uint32_t*>(J.st->x)[lane];
  }
  uint32_t crc_raw = do_crc ? (init ? 0xFFFFFFFFu : ~uniform32(J.cs->crc)) : 0u;

  if (do_sha && nx > 64) {  // Go: copy(d.x[d.nx:], p) panics (sha1.go:62)
    if (lane == 0 && J.status) *J.status = EFES_ERR_STATE;
    return M;
  }
  const uint8_t* p = J.p;
  const uint64_t plen = J.plen;
  wave_lds_sync();

  // ---- complete the pending block x[:nx] (sha1.go:61-69)
  uint64_t pos = 0;
  int64_t nx_new = nx;
  if (do_sha && nx > 0) {
    const uint32_t room = (uint32_t)(64 - nx);
    const uint32_t nh = plen < room ? (uint32_t)plen : room;
    if ((uint32_t)lane < nh) xs[nx + lane] = ldg_u8(EFES_RANGE(p + lane, 1, p, plen, "deep-head"));
    wave_lds_sync();
    if ((uint32_t)nx + nh == 64) {
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = be_word_lds(xs, k);
      compress_inline(h, w);
      nx_new = 0;
    } else {
      nx_new = nx + nh;
    }
    pos = nh;
  }
  if (do_crc)
    for (uint64_t i = 0; i < pos; ++i) crc_raw = crc_byte(T.slice8[0], crc_raw, ldg_u8(EFES_RANGE(p + i, 1, p, plen, "deep-crchead")));
  M.crc_raw = crc_raw;
  M.q = p + pos;
  M.pos = pos;
  M.nbulk = (plen - pos) >> 6;
  M.done = 0;
  M.nx_new = nx_new;
  M.live = 1;
  return M;
}

// The rest of one Write after the head: bulk blocks [M.done, M.nbulk) (sha1.go:70-74), the
// tail (:75-77), Sum (:82-120) on a copy, and the write-back of state, crc, sum and status.
// kBulk = false: the caller has hashed every bulk block (M.done == M.nbulk) and T may hold only
// the slicing-by-8 table (FED kernel).
template <bool kBulk = true>
__device__ void deep_rest(const Tables& T, int lane, const DeepJob& J, uint8_t* xs, uint8_t* fb, DeepMsg M) {
  const bool do_sha = J.st != nullptr, do_crc = J.cs != nullptr;
  const bool fin = (J.flags & EFES_JOB_FINALIZE) != 0;
  int32_t status = EFES_OK;
  uint32_t (&h)[5] = M.h;
  uint32_t crc_raw = M.crc_raw;
  int64_t nx_new = M.nx_new;
  const uint8_t* p = J.p;
  const uint64_t plen = J.plen;
  const uint64_t pos = M.pos, nbulk = M.nbulk;
  uint64_t len = do_sha && !(J.flags & EFES_JOB_INIT) ? uniform64(J.st->len) : 0;

  // ---- bulk whole blocks not hashed yet (sha1.go:70-74)
  if (kBulk && nbulk > M.done) {
    const uint8_t* q = M.q + 64 * M.done;
    if ((reinterpret_cast<uintptr_t>(q) & 15) == 0)
      deep_bulk<true>(T, lane, q, nbulk - M.done, do_sha, do_crc, h, crc_raw);
    else
      deep_bulk<false>(T, lane, q, nbulk - M.done, do_sha, do_crc, h, crc_raw);
  }

  // ---- tail (sha1.go:75-77): x[:r] = rest; x[r:] keeps stale bytes
  const uint64_t tpos = pos + (nbulk << 6);
  const uint32_t r = (uint32_t)(plen - tpos);
  if (do_crc)
    for (uint32_t i = 0; i < r; ++i) crc_raw = crc_byte(T.slice8[0], crc_raw, ldg_u8(EFES_RANGE(p + tpos + i, 1, p, plen, "deep-crctail")));
  if (do_sha && r > 0) {
    if ((uint32_t)lane < r) xs[lane] = ldg_u8(EFES_RANGE(p + tpos + lane, 1, p, plen, "deep-tail"));
    nx_new = r;
  }
  wave_lds_sync();
  len += plen;  // sha1.go:60

  // ---- Sum (sha1.go:89-120) on a copy of the state
  uint32_t dig[5] = {0, 0, 0, 0, 0};
  bool have_sum = false;
  if (fin && do_sha) {
    const uint32_t nxf = nx_new > 0 ? (uint32_t)nx_new : 0u;  // Write skips a negative nx (sha1.go:61)
    const uint32_t lm = (uint32_t)(len & 63);
    const uint32_t padlen = lm < 56 ? 56 - lm : 120 - lm;     // sha1.go:94-98
    const uint32_t T = nxf + padlen + 8;
    if (T & 63) {
      status = EFES_ERR_STATE;  // sha1.go:107-109 panic("d.nx != 0")
    } else {
      const uint64_t bits = len << 3;
      for (uint32_t i = lane; i < T; i += 64) {
        uint32_t b;
        if (i < nxf) b = xs[i];
        else if (i == nxf) b = 0x80;
        else if (i >= T - 8) b = (uint32_t)(bits >> (56 - 8 * (i - (T - 8)))) & 0xffu;
        else b = 0;
        fb[i] = (uint8_t)b;
      }
      wave_lds_sync();
      uint32_t hf[5] = {h[0], h[1], h[2], h[3], h[4]};
      for (uint32_t blk = 0; blk < T / 64; ++blk) {
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = be_word_lds(fb + 64 * blk, k);
        compress_inline(hf, w);
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) dig[k] = hf[k];
      have_sum = true;
    }
  }

  // ---- write back (a Sum-only job leaves the states alone: Go's Sum works on a copy)
  const bool keep = (J.flags & EFES_JOB_SUM_ONLY) != 0;
  if (do_sha && !keep) {
    if (lane < 5) {
      uint32_t v = h[0];
#pragma unroll
      for (int k = 1; k < 5; ++k) v = lane == k ? h[k] : v;
      J.st->h[lane] = v;
    }
    if (lane < 16) reinterpret_cast<uint32_t*>(J.st->x)[lane] = reinterpret_cast<const uint32_t*>(xs)[lane];
    if (lane == 0) {
      J.st->nx = nx_new;
      J.st->len = len;
    }
  }
  if (do_crc && !keep && lane == 0) J.cs->crc = ~crc_raw;
  if (fin && J.sum && lane < 6) {
    uint32_t v;
    if (lane < 5) {
      v = dig[0];
#pragma unroll
      for (int k = 1; k < 5; ++k) v = lane == k ? dig[k] : v;
      v = have_sum ? v : 0u;
    } else {
      v = do_crc ? ~crc_raw : 0u;
    }
    reinterpret_cast<uint32_t*>(J.sum)[lane] = bswap(v);  // big-endian, as Sum appends
  }
  if (lane == 0 && J.status) *J.status = status;
}

// Job j's descriptor as wave-uniform values.
__device__ __forceinline__ DeepJob load_job(const efes_job* __restrict__ jobs, uint32_t j, int lane) {
  const efes_job* jb = jobs + j;
  DeepJob J;
  J.p = reinterpret_cast<const uint8_t*>(uniform64(reinterpret_cast<uint64_t>(jb->data)));
  J.plen = uniform64(jb->length);
  J.st = reinterpret_cast<efes_sha1_state*>(uniform64(reinterpret_cast<uint64_t>(jb->sha1)));
  J.cs = reinterpret_cast<efes_crc32_state*>(uniform64(reinterpret_cast<uint64_t>(jb->crc32)));
  J.sum = reinterpret_cast<uint8_t*>(uniform64(reinterpret_cast<uint64_t>(jb->sum)));
  J.status = reinterpret_cast<int32_t*>(uniform64(reinterpret_cast<uint64_t>(jb->status)));
  J.flags = uniform32(jb->flags);
#ifdef EFES_CHECKED
  if (lane == 0)
    printf("EFES_CHECKED job %u p=%p len=%llu st=%p cs=%p sum=%p status=%p flags=%u\n", j, (const void*)J.p,
           (unsigned long long)J.plen, (void*)J.st, (void*)J.cs, (void*)J.sum, (void*)J.status, J.flags);
#else
  (void)lane;
#endif
  return J;
}

// DeepMsg field read back from LDS as a wave-uniform value.
__device__ __forceinline__ DeepMsg uniform_msg(const DeepMsg& s) {
  DeepMsg M;
#pragma unroll
  for (int k = 0; k < 5; ++k) M.h[k] = uniform32(s.h[k]);
  M.crc_raw = uniform32(s.crc_raw);
  M.q = reinterpret_cast<const uint8_t*>(uniform64(reinterpret_cast<uint64_t>(s.q)));
  M.pos = uniform64(s.pos);
  M.nbulk = uniform64(s.nbulk);
  M.done = uniform64(s.done);
  M.nx_new = (int64_t)uniform64((uint64_t)s.nx_new);
  M.live = uniform32(s.live);
  M.joint = uniform32(s.joint);
  return M;
}

// ================================================================== DEEP kernel, producer/consumer
// Workgroup = 4 chain waves + 4 producer waves; wave w+4 always lands on the same SIMD as wave
// w (tools/microbench/mb_placement.hip), so each SIMD hosts one job's chain and its producer.
// The producer does everything of a super-step that is not the chain -- the coalesced load of
// 64 blocks, their CRC-32 and shift tree, the W+K expansion -- and hands W+K over through LDS
// (20 ds_write_b128 per lane); the chain wave (s_setprio 3) only copies its block's 80 words
// into registers (20 ds_read_b128 per lane per super-step) and runs the 64 chains.  The chain
// wave's instruction stream is then 405 + 5 per block plus ~30 per 64 blocks.
constexpr int kPipeJobs = 4;  // jobs per workgroup (one per SIMD)

struct PipeSlot {  // one job's hand-over area
  uint4 wk[20][64];  // [word quad][lane]: lane l's block W+K[4q..4q+3] -- conflict-free b128 access
  DeepMsg msg;       // the head's result (chain -> producer), then the final CRC (producer -> chain)
  int started;       // chain -> producer: msg holds the head's result
  int ready;         // producer -> chain: super-steps whose W+K has been written
  int taken;         // chain -> producer: super-steps whose W+K the chain has copied out
  int crc_done;      // producer -> chain: msg.crc_raw is the CRC after the bulk
};

struct PipeLDS {
  Tables tab;                                // 36 KiB
  PipeSlot slot[kPipeJobs];                  // 4 x 20 KiB
  uint8_t xs[kPipeJobs][64];
  uint8_t fin[kPipeJobs][192];
};

__device__ __forceinline__ int lds_acquire(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <int kSleep>
__device__ __forceinline__ void wait_at_least(const int* p, int v) {
  while (lds_acquire(p) < v) __builtin_amdgcn_s_sleep(kSleep);
}

// Producer side of deep_bulk: super-steps of up to 64 blocks, right-aligned in the lanes.
template <bool kAligned16>
__device__ void pipe_produce(const Tables& T, PipeSlot& P, int lane, const uint8_t* q, uint64_t nbulk, bool do_sha,
                             bool do_crc, uint32_t& crc_raw) {
  uint32_t le[16];
  uint64_t b0 = 0;
  int nb = (int)(nbulk < 64 ? nbulk : 64);
  {
    const int bi = lane - (64 - nb);
#pragma unroll
    for (int k = 0; k < 16; ++k) le[k] = 0;
    if (bi >= 0) load_block_le<kAligned16>(EFES_RANGE(q + 64 * (uint64_t)bi, 64, q, 64 * nbulk, "pipe-bulk0"), le);
  }
  for (int step = 0; b0 < nbulk; ++step) {
    if (do_crc) {
      uint32_t r = crc_words_raw(T.slice8, 0u, le);
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const uint32_t o = __shfl_xor(r, 1 << k);
        const bool right = (lane >> k) & 1;
        r = crc_shift(T.shift[k], right ? o : r) ^ (right ? r : o);
      }
      if (nb == 64) {
        crc_raw = crc_shift(T.shift[6], crc_raw);
      } else {
#pragma unroll
        for (int k = 0; k < 6; ++k)
          if ((nb >> k) & 1) crc_raw = crc_shift(T.shift[k], crc_raw);
      }
      crc_raw ^= r;
    }
    uint32_t x[80];
    if (do_sha) {
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = bswap(le[k]);
      expand_wk(w, x);
    }
    const uint64_t b1 = b0 + (uint64_t)nb;
    const int nb1 = (int)((nbulk - b1) < 64 ? (nbulk - b1) : 64);
    if (b1 < nbulk) {
      const int bj = lane - (64 - nb1);
#pragma unroll
      for (int k = 0; k < 16; ++k) le[k] = 0;
      if (bj >= 0) load_block_le<kAligned16>(EFES_RANGE(q + 64 * (b1 + (uint64_t)bj), 64, q, 64 * nbulk, "pipe-bulk1"), le);
    }
    if (do_sha) {
      wait_at_least<8>(&P.taken, step);  // the chain has copied super-step step-1 out
#pragma unroll
      for (int k = 0; k < 20; ++k) P.wk[k][lane] = make_uint4(x[4 * k], x[4 * k + 1], x[4 * k + 2], x[4 * k + 3]);
      lds_release(&P.ready, step + 1);
    }
    b0 = b1;
    nb = nb1;
  }
}

// Chain side: per super-step, copy this lane's block W+K out of LDS and run the nb chains.
__device__ void pipe_consume(PipeSlot& P, int lane, uint64_t nbulk, uint32_t (&h)[5]) {
  uint64_t b0 = 0;
  for (int step = 0; b0 < nbulk; ++step) {
    const int nb = (int)((nbulk - b0) < 64 ? (nbulk - b0) : 64);
    wait_at_least<1>(&P.ready, step + 1);
    uint32_t x[80];
#pragma unroll
    for (int k = 0; k < 20; ++k) {
      const uint4 v = P.wk[k][lane];
      x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
    }
    lds_release(&P.taken, step + 1);  // (release: the reads above complete first)
    uint32_t hv[5] = {h[0], h[1], h[2], h[3], h[4]}, hs[5];
    auto block = [&]() {
      chain_block(hv, x, hs);  // sha1.go:193-197 folded in
#pragma unroll
      for (int k = 1; k < 6; ++k) hv[k % 5] = (uint32_t)__builtin_amdgcn_mov_dpp((int)hs[k % 5], 0x138, 0xf, 0xf, true);  // wave_shr:1, h0 (round 79's v_add3) last
    };
    const int nbu = (int)uniform32((uint32_t)nb);
    int j = 0;
    for (; j + 2 <= nbu; j += 2) { block(); block(); }
    if (j < nbu) block();
#pragma unroll
    for (int k = 0; k < 5; ++k) h[k] = (uint32_t)__builtin_amdgcn_readlane((int)hs[k], 63);
    b0 += (uint64_t)nb;
  }
}

__global__ __launch_bounds__(128 * kPipeJobs, 1) void deep_kernel(const efes_job* __restrict__ jobs, uint32_t njobs,
                                                                  const Tables* __restrict__ tabs) {
  __shared__ __attribute__((aligned(16))) PipeLDS L;
  {
    const uint4* src = reinterpret_cast<const uint4*>(tabs);
    uint4* dst = reinterpret_cast<uint4*>(&L.tab);
    for (int i = threadIdx.x; i < (int)(sizeof(Tables) / 16); i += blockDim.x) dst[i] = src[i];
    if (threadIdx.x < kPipeJobs) {
      PipeSlot& P = L.slot[threadIdx.x];
      P.started = P.ready = P.taken = P.crc_done = 0;
    }
  }
  __syncthreads();
  const int wave = (int)uniform32(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int w = wave & (kPipeJobs - 1);
  const uint32_t j = blockIdx.x * kPipeJobs + (uint32_t)w;
  if (j >= njobs) return;
  PipeSlot& P = L.slot[w];
  const DeepJob J = load_job(jobs, j, lane);
  const bool do_sha = J.st != nullptr, do_crc = J.cs != nullptr;
  if (wave < kPipeJobs) {  // ---- chain wave
    __builtin_amdgcn_s_setprio(3);
    DeepMsg M = deep_head(L.tab, lane, J, L.xs[w]);
    if (lane == 0) P.msg = M;
    lds_release(&P.started, 1);
    if (!M.live) return;
    if (do_sha) pipe_consume(P, lane, M.nbulk, M.h);
    wait_at_least<1>(&P.crc_done, 1);
    M.crc_raw = uniform32(P.msg.crc_raw);
    M.done = M.nbulk;
    deep_rest(L.tab, lane, J, L.xs[w], L.fin[w], M);
  } else {  // ---- producer wave
    wait_at_least<4>(&P.started, 1);
    const DeepMsg M = uniform_msg(P.msg);
    if (!M.live) return;
    uint32_t crc_raw = M.crc_raw;
    if (M.nbulk) {
      if ((reinterpret_cast<uintptr_t>(M.q) & 15) == 0)
        pipe_produce<true>(L.tab, P, lane, M.q, M.nbulk, do_sha, do_crc, crc_raw);
      else
        pipe_produce<false>(L.tab, P, lane, M.q, M.nbulk, do_sha, do_crc, crc_raw);
    }
    if (lane == 0) P.msg.crc_raw = crc_raw;
    lds_release(&P.crc_done, 1);
  }
}

// The value of the last lane of each group of G lanes, in every lane of the group: a job's
// chaining value after a super-step, back to all its lanes.  G = 4 is one quad: a DPP
// quad_perm [3,3,3,3] move (no LDS round trip on the chain's critical path); wider groups use
// ds_bpermute.
template <int G>
__device__ __forceinline__ uint32_t group_last(uint32_t v, int lane) {
  if constexpr (G == 4) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xFF, 0xf, 0xf, true);
  return (uint32_t)__shfl((int)v, lane | (G - 1));
}

// ================================================================== grouped DEEP kernel
// k = 64/G jobs per wave, G lanes (= G consecutive blocks per super-step) per job.  For
// batches with more long jobs than SIMDs: the chain instructions are shared by the k jobs
// (lane m*G+i runs block i of job m), so a super-step of 410 G + ~700 instructions advances
// k jobs by G blocks each: (410 G + ~700)/64 instructions per block of issue work (DEEP: 422)
// at a per-job latency of 410 + ~700/G per block (WIDE: 740 at a slower issue rate).
// DESIGN_NOTES.md §4 "grouped DEEP".
//
// Phases per wave: the head of every job (sequential, state parked in LDS); joint rounds in
// which the jobs with >= G bulk blocks left advance together; then, per job, the rest
// (left-over bulk blocks through deep_bulk, tail, Sum, write-back).  Jobs are expected
// longest-first (efes_plan_batch) so the jobs of a wave have similar lengths.
// Raw CRC (register 0) of one 64-byte block: the XOR of 64 independent position-table lookups
// (PosTables), in four accumulation chains.
__device__ __forceinline__ uint32_t crc_block_pos(const uint32_t (&pos)[64][256], const uint32_t (&le)[16]) {
  uint32_t acc[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    const uint32_t v = le[w];
    const uint32_t x = __builtin_amdgcn_bitop3_b32(pos[4 * w][v & 0xffu], pos[4 * w + 1][(v >> 8) & 0xffu],
                                                   pos[4 * w + 2][(v >> 16) & 0xffu], 0x96);
    acc[w & 3] = __builtin_amdgcn_bitop3_b32(acc[w & 3], x, pos[4 * w + 3][v >> 24], 0x96);
  }
  return __builtin_amdgcn_bitop3_b32(acc[0], acc[1], acc[2], 0x96) ^ acc[3];
}

// kSha / kCrc are wave-uniform (any joining job needs the hash): with both, the CRC lookups and
// the schedule expansion share one basic block, so the lookups' latency hides behind VALU work.
template <int G, bool kAligned16, bool kSha, bool kCrc>
__device__ void group_bulk(const Tables& T, const PosTables& P, int lane, DeepMsg* msgs, uint64_t S) {
  constexpr int kLG = G == 4 ? 2 : G == 8 ? 3 : G == 16 ? 4 : 5;
  static_assert((1 << kLG) == G, "G must be 4, 8, 16 or 32");
  const int m = lane / G, i = lane % G;
  const DeepMsg& M = msgs[m];
  const bool live = M.live != 0 && M.joint != 0;
  const uint8_t* q = M.q + 64 * M.done;
  uint32_t hv[5] = {M.h[0], M.h[1], M.h[2], M.h[3], M.h[4]}, hs[5] = {0, 0, 0, 0, 0};
  uint32_t crc_raw = M.crc_raw;
  // One super-step: CRC + schedule of this lane's block `cur`, the prefetch of the next
  // super-step's block into `nxt` (exec-masked: a lane of a job outside this round loads
  // nothing; zeroed first so the compiler keeps the prefetch a whole chain ahead), the chain.
  auto super_step = [&](const uint32_t (&cur)[16], uint32_t (&nxt)[16], uint64_t st) {
    if constexpr (kCrc) {
      uint32_t r = crc_block_pos(P.pos, cur);  // raw CRC of this lane's block, register 0
#pragma unroll
      for (int k = 0; k < kLG; ++k) {  // crc(A||B) = shift(crc(A), |B|) ^ crc(B) within the job's G lanes
        const uint32_t o = __shfl_xor(r, 1 << k);
        const bool right = (lane >> k) & 1;
        r = crc_shift(T.shift[k], right ? o : r) ^ (right ? r : o);
      }
      crc_raw = crc_shift(T.shift[kLG], crc_raw) ^ r;  // running crc advanced over G*64 bytes
    }
    uint32_t x[80];
    if constexpr (kSha) {
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = bswap(cur[k]);
      expand_wk(w, x);
    }
    if (st + 1 < S) {
#pragma unroll
      for (int k = 0; k < 16; ++k) nxt[k] = 0;
      if (live) load_block_le<kAligned16>(q + 64 * ((st + 1) * G + (uint64_t)i), nxt);
    }
    if constexpr (kSha) {
      auto block = [&]() {
        chain_block(hv, x, hs);  // real in lane m*G+j of every job m at iteration j
#pragma unroll
        for (int k = 1; k < 6; ++k) hv[k % 5] = (uint32_t)__builtin_amdgcn_mov_dpp((int)hs[k % 5], 0x138, 0xf, 0xf, true);  // wave_shr:1, h0 (round 79's v_add3) last
      };
#pragma unroll
      for (int j = 0; j < G; j += 2) { block(); block(); }
      // the job's chaining value is in its last lane: back to all G lanes (its first one needs it)
#pragma unroll
      for (int k = 0; k < 5; ++k) hv[k] = group_last<G>(hs[k], lane);
    }
  };
  uint32_t A[16], B[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) A[k] = 0;
  if (live) load_block_le<kAligned16>(q + 64 * (uint64_t)i, A);
  for (uint64_t st = 0; st < S; st += 2) {  // two buffers, unrolled by two: no register copies of the prefetch
    super_step(A, B, st);
    if (st + 1 >= S) break;
    super_step(B, A, st + 1);
  }
  wave_lds_sync();
  if (live && i == 0) {  // joint jobs only
    DeepMsg& W = msgs[m];
#pragma unroll
    for (int k = 0; k < 5; ++k) W.h[k] = kSha ? hv[k] : W.h[k];
    W.crc_raw = crc_raw;
    W.done += S * G;
  }
  wave_lds_sync();
}

template <int G, bool kAligned16>
__device__ void group_bulk_any(const Tables& T, const PosTables& P, int lane, DeepMsg* msgs, uint64_t S, bool any_sha,
                               bool any_crc) {
  if (any_sha && any_crc) group_bulk<G, kAligned16, true, true>(T, P, lane, msgs, S);
  else if (any_sha) group_bulk<G, kAligned16, true, false>(T, P, lane, msgs, S);
  else group_bulk<G, kAligned16, false, true>(T, P, lane, msgs, S);
}


template <int G>
__global__ __launch_bounds__(64 * kDeepWaves, 1) void group_kernel(const efes_job* __restrict__ jobs, uint32_t njobs,
                                                                   const Tables* __restrict__ tabs) {
  constexpr int kJobs = 64 / G;
  static_assert(kJobs <= kGroupMaxJobs, "LDS holds kGroupMaxJobs jobs per wave");
  __shared__ __attribute__((aligned(16))) DeepLDS L;
  {
    const uint4* src = reinterpret_cast<const uint4*>(tabs);  // Tables then PosTables
    uint4* dst = reinterpret_cast<uint4*>(&L.tab);
    for (int i = threadIdx.x; i < (int)((sizeof(Tables) + sizeof(PosTables)) / 16); i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  const int wave = (int)uniform32(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t j0 = (blockIdx.x * kDeepWaves + (uint32_t)wave) * kJobs;
  if (j0 >= njobs) return;
  DeepMsg* msgs = L.msg[wave];

  // ---- heads (state parked in LDS)
  for (int m = 0; m < kJobs; ++m) {
    const uint32_t j = j0 + (uint32_t)m;
    DeepMsg M{};
    if (j < njobs) M = deep_head(L.tab, lane, load_job(jobs, j, lane), L.xs[wave][m]);
    wave_lds_sync();
    if (lane == 0) msgs[m] = M;
  }
  wave_lds_sync();

  // ---- joint rounds: while two or more jobs have >= G bulk blocks left, they advance together
  // by S*G blocks, S = the smallest of their floor(left/G) (so a wave lasts as long as its
  // longest job, whatever the mix of lengths); a job left alone finishes on the one-job path
  // (422 instructions per block instead of (410 G + ~700)/G).
  for (int round = 0; round < kJobs; ++round) {
    uint64_t S = ~0ull;
    int joiners = 0;
    bool any_sha = false, any_crc = false, all16 = true;
    for (int m = 0; m < kJobs; ++m) {
      const DeepMsg M = uniform_msg(msgs[m]);
      const uint64_t left = M.live ? (M.nbulk - M.done) / G : 0;
      if (left == 0) continue;
      ++joiners;
      S = left < S ? left : S;
      const DeepJob J = load_job(jobs, j0 + (uint32_t)m, lane);
      any_sha |= J.st != nullptr;
      any_crc |= J.cs != nullptr;
      all16 &= (reinterpret_cast<uintptr_t>(M.q + 64 * M.done) & 15) == 0;
    }
    if (joiners < 2) break;
    for (int m = 0; m < kJobs; ++m) {
      const DeepMsg M = uniform_msg(msgs[m]);
      if (lane == 0) msgs[m].joint = M.live && (M.nbulk - M.done) / G > 0 ? 1u : 0u;
    }
    wave_lds_sync();
    if (all16) group_bulk_any<G, true>(L.tab, L.pos, lane, msgs, S, any_sha, any_crc);
    else group_bulk_any<G, false>(L.tab, L.pos, lane, msgs, S, any_sha, any_crc);
  }

  // ---- per job: left-over blocks, tail, Sum, write-back
  for (int m = 0; m < kJobs; ++m) {
    const uint32_t j = j0 + (uint32_t)m;
    if (j >= njobs) break;
    const DeepMsg M = uniform_msg(msgs[m]);
    if (!M.live) continue;
    const DeepJob J = load_job(jobs, j, lane);
    deep_rest(L.tab, lane, J, L.xs[wave][m], L.fin[wave], M);
  }
}

// ================================================================== FED kernel: grouped DEEP fed from other SIMDs
// The grouped kernel's chain wave spends (410 G + ~665) instructions per super-step: the chain
// plus the loads, CRC and W+K expansion of its 64 blocks, all on one SIMD, so a job's latency is
// 410 + 665/G per block (GROUP4: 577).  Here a workgroup owns its CU (its LDS fills the CU) and
// splits that work across the CU's four SIMDs (one wave each): C chain waves holding 64/G jobs of
// G lanes each, and 4 - C producer waves.  Per super-step of a chain wave, its producer loads the
// 64 blocks (G consecutive blocks of each job, coalesced, prefetched a super-step ahead), computes
// their CRC-32 (position tables: 64 independent lookups per block, the G-lane shift tree, the fold
// into each job's running CRC) and the W+K expansion, and hands W+K over through LDS as the DEEP
// kernel does (20 ds_write_b128 per lane).  The chain wave copies its lane's 80 words out
// (20 ds_read_b128) and runs G chains: 410 + ~50/G instructions per block, DEEP's per-job latency.
// A producer serves its chain waves round-robin, polling their slots (measured: one item, i.e.
// one chain super-step, costs the producer ~3.9k cycles against the chain's ~6.9k at G = 4).
// Heads, left-over blocks (< G per job), tails and Sums run on the chain waves.
//   FED4 = <G 4, 2 chain waves + 2 producers>: 32 jobs per CU.
template <int G, int C>
struct FedCfg {
  static constexpr int kJobs = 64 / G;  // jobs per chain wave
  static constexpr int kProducers = 4 - C;
  static constexpr int kLG = G == 4 ? 2 : G == 8 ? 3 : 0;
  static_assert(kLG > 0 && C >= 1 && C <= 3, "G in {4, 8}, 1..3 chain waves");
};

// FED4E: the producer hands over the 16 message words W[0..15] (big-endian); the chain wave
// expands W[16..79] and adds K.  (Round 2 measured handing over more of the schedule: no gain.)
constexpr int kFedHand = 16;

struct FedSlot {
  uint4 wk[20][64];   // [word quad][lane], as PipeSlot
  uint64_t S;         // super-steps of the posted round
  uint32_t flags;     // bit 0: some joint job hashes SHA-1, bit 1: CRC-32, bit 2: all blocks 16-B aligned
  uint32_t req;       // chain -> producer: rounds posted
  uint32_t fin;       // chain -> producer: no more rounds
  uint32_t ready;     // producer -> chain: super-steps whose W+K is in wk (running count)
  uint32_t taken;     // chain -> producer: super-steps copied out of wk
  uint32_t crc_done;  // producer -> chain: rounds whose CRCs are back in the job's DeepMsg
};

// The LDS copy of the tables: the slicing-by-8 table and shift levels 0..3 (the tree and fold for
// G <= 8) -- a prefix of Tables, so deep_head / deep_rest<false> can take it as one -- and the
// position tables for the producer's CRC.
constexpr int kFedShift = 4;
struct FedTables {
  uint32_t slice8[8][256];
  uint32_t shift[kFedShift][4][256];
};
static_assert(offsetof(Tables, shift) == offsetof(FedTables, shift), "FedTables is a prefix of Tables");

template <int G, int C>
struct FedLDS {
  static constexpr int kJobs = FedCfg<G, C>::kJobs;
  FedTables tab;                // 24 KiB
  PosTables pos;                // 64 KiB
  FedSlot slot[C];              // 20 KiB each
  DeepMsg msg[C][kJobs];
  uint8_t xs[C][kJobs][64];
  uint8_t fin[C][192];
};

// Counters run modulo 2^32: "a has reached b".
__device__ __forceinline__ bool reached(uint32_t a, uint32_t b) { return (int32_t)(a - b) >= 0; }
__device__ __forceinline__ uint32_t lds_acq32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Release store issued HERE: the scheduling barrier keeps the compiler from sinking it below the
// (fully unrolled) work that follows, which would hold the other side up for that long.
__device__ __forceinline__ void lds_rel32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  __builtin_amdgcn_sched_barrier(0);
}

// One lane's block of a fed super-step (zeros for a lane whose job sits the round out).
__device__ __forceinline__ void fed_load(const uint8_t* src, bool live, bool a16, uint32_t (&le)[16]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) le[k] = 0;
  if (live) {
    if (a16) load_block_le<true>(src, le);
    else load_block_le<false>(src, le);
  }
}

// Producer-side state of one chain wave's current round.
struct FedFeed {
  const uint8_t* q;  // this lane's job: first byte of the round (M.q + 64 * (M.done + i))
  uint64_t S, st;    // super-steps of the round, produced so far
  uint32_t gstep;    // W+K super-steps handed to this chain wave, all rounds
  uint32_t round;    // rounds served
  uint32_t crc;      // this lane's job's running raw CRC
  uint32_t flags;
  bool live, active, done;
  uint32_t pre[16];  // the next super-step's block, in flight
};

template <int G, int C>
__device__ __forceinline__ void fed_start(FedLDS<G, C>& L, int c, int lane, FedFeed& F) {
  FedSlot& P = L.slot[c];
  F.S = uniform64(P.S);
  F.flags = uniform32(P.flags);
  const int m = lane / G, i = lane % G;
  const DeepMsg& M = L.msg[c][m];
  F.live = M.live != 0 && M.joint != 0;
  F.q = M.q + 64 * (M.done + (uint64_t)i);
  F.crc = M.crc_raw;
  F.st = 0;
  F.active = true;
  fed_load(F.q, F.live, (F.flags & 4u) != 0, F.pre);
}

// Produce super-step F.st of chain wave c into its (free) slot.  X: the chain wave expands the
// schedule itself, the producer hands over only the 16 message words (big-endian).
template <int G, int C, bool X>
__device__ __forceinline__ void fed_produce(FedLDS<G, C>& L, int c, int lane, FedFeed& F) {
  constexpr int kLG = FedCfg<G, C>::kLG;
  FedSlot& P = L.slot[c];
  const bool do_sha = (F.flags & 1u) != 0, do_crc = (F.flags & 2u) != 0, a16 = (F.flags & 4u) != 0;
  uint32_t cur[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) cur[k] = F.pre[k];
  if (F.st + 1 < F.S) fed_load(F.q + 64 * G * (F.st + 1), F.live, a16, F.pre);
  if (do_crc) {
    uint32_t r = crc_block_pos(L.pos.pos, cur);  // raw CRC of this lane's block (independent lookups)
#pragma unroll
    for (int k = 0; k < kLG; ++k) {  // the job's G blocks: crc(A||B) = shift(crc(A), |B|) ^ crc(B)
      const uint32_t o = __shfl_xor(r, 1 << k);
      const bool right = (lane >> k) & 1;
      r = crc_shift(L.tab.shift[k], right ? o : r) ^ (right ? r : o);
    }
    F.crc = crc_shift(L.tab.shift[kLG], F.crc) ^ r;  // running CRC advanced over G * 64 bytes
  }
  if (do_sha) {
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = bswap(cur[k]);
    if constexpr (X) {  // the first kFedHand raw schedule words; the chain wave expands the rest
      uint32_t r[kFedHand];
      expand_raw<kFedHand>(w, r);
#pragma unroll
      for (int k = 0; k < kFedHand / 4; ++k) P.wk[k][lane] = make_uint4(r[4 * k], r[4 * k + 1], r[4 * k + 2], r[4 * k + 3]);
    } else {
      uint32_t x[80];
      expand_wk(w, x);
#pragma unroll
      for (int k = 0; k < 20; ++k) P.wk[k][lane] = make_uint4(x[4 * k], x[4 * k + 1], x[4 * k + 2], x[4 * k + 3]);
    }
    lds_rel32(&P.ready, F.gstep + 1);
    ++F.gstep;  // counts handed-over super-steps only, as the chain's copy-outs do
  }
  if (++F.st == F.S) {  // round done: CRCs back to the jobs' messages
    const int m = lane / G;
    if (F.live && (lane % G) == 0 && do_crc) L.msg[c][m].crc_raw = F.crc;
    ++F.round;
    lds_rel32(&P.crc_done, F.round);
    F.active = false;
  }
}

// Producer p serves chain waves p, p + producers, ... (those of the C that exist: nchains).
template <int G, int C, bool X>
__device__ void fed_producer(FedLDS<G, C>& L, int lane, int p, uint32_t nchains) {
  constexpr int kP = FedCfg<G, C>::kProducers;
  FedFeed F[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    F[c].gstep = 0;
    F[c].round = 0;
    F[c].active = false;
    F[c].done = c % kP != p || (uint32_t)c >= nchains;
  }
  for (;;) {
    bool all_done = true, did = false;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (F[c].done) continue;
      all_done = false;
      FedSlot& P = L.slot[c];
      if (!F[c].active) {
        if (!reached(F[c].round, lds_acq32(&P.req))) {
          fed_start(L, c, lane, F[c]);
        } else {
          if (lds_acq32(&P.fin)) F[c].done = true;
          continue;
        }
      }
      if ((F[c].flags & 1u) && !reached(lds_acq32(&P.taken), F[c].gstep)) continue;  // slot still in use
      fed_produce<G, C, X>(L, c, lane, F[c]);
      did = true;
    }
    if (all_done) break;
    if (!did) __builtin_amdgcn_s_sleep(1);
  }
}

// Chain side of one round: S super-steps of G blocks for every joint job of the wave.
template <int G, bool X>
__device__ void fed_consume(FedSlot& P, int lane, const DeepMsg* msgs, uint64_t S, uint32_t& gstep, uint32_t (&hv)[5]) {
  const DeepMsg& M = msgs[lane / G];
#pragma unroll
  for (int k = 0; k < 5; ++k) hv[k] = M.h[k];
  uint32_t hs[5] = {0, 0, 0, 0, 0};
  for (uint64_t st = 0; st < S; ++st) {
    while (!reached(lds_acq32(&P.ready), gstep + 1)) __builtin_amdgcn_s_sleep(1);
    uint32_t x[80];
    if constexpr (X) {
      uint32_t w[kFedHand];
#pragma unroll
      for (int k = 0; k < kFedHand / 4; ++k) {
        const uint4 v = P.wk[k][lane];
        w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
      }
      lds_rel32(&P.taken, gstep + 1);  // the producer may overwrite the slot now
      expand_wk_from<kFedHand>(w, x);
    } else {
#pragma unroll
      for (int k = 0; k < 20; ++k) {
        const uint4 v = P.wk[k][lane];
        x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
      }
      lds_rel32(&P.taken, gstep + 1);  // the producer may overwrite the slot now
    }
    ++gstep;
    auto block = [&]() {
      chain_block(hv, x, hs);  // real in lane m*G+j of every job m at iteration j
#pragma unroll
      for (int k = 1; k < 6; ++k) hv[k % 5] = (uint32_t)__builtin_amdgcn_mov_dpp((int)hs[k % 5], 0x138, 0xf, 0xf, true);  // wave_shr:1, h0 (round 79's v_add3) last
    };
#pragma unroll
    for (int j = 0; j < G; ++j) block();
#pragma unroll
    for (int k = 0; k < 5; ++k) hv[k] = group_last<G>(hs[k], lane);
  }
}

template <int G, int C, bool X>
__global__ __launch_bounds__(256, 1) void fed_kernel(const efes_job* __restrict__ jobs, uint32_t njobs,
                                                     const Tables* __restrict__ tabs) {
  constexpr int kJobs = FedCfg<G, C>::kJobs;
  __shared__ __attribute__((aligned(16))) FedLDS<G, C> L;
  static_assert(sizeof(FedLDS<G, C>) <= 160 * 1024, "one FED workgroup per CU");
  {
    const uint4* src = reinterpret_cast<const uint4*>(tabs);  // Tables, then PosTables (efes_ctx_create)
    uint4* dst = reinterpret_cast<uint4*>(&L.tab);
    for (int i = threadIdx.x; i < (int)(sizeof(FedTables) / 16); i += blockDim.x) dst[i] = src[i];
    const uint4* psrc = reinterpret_cast<const uint4*>(tabs + 1);
    uint4* pdst = reinterpret_cast<uint4*>(&L.pos);
    for (int i = threadIdx.x; i < (int)(sizeof(PosTables) / 16); i += blockDim.x) pdst[i] = psrc[i];
    if (threadIdx.x < C) {
      FedSlot& P = L.slot[threadIdx.x];
      P.req = P.fin = P.ready = P.taken = P.crc_done = 0;
    }
  }
  __syncthreads();
  const int wave = (int)uniform32(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t base = blockIdx.x * (uint32_t)(C * kJobs);
  if (wave >= C) {  // ---- producer (a SIMD of its own)
    const uint32_t left = njobs - base;  // base < njobs for every launched workgroup
    fed_producer<G, C, X>(L, lane, wave - C, (left + kJobs - 1) / kJobs);
    return;
  }
  // ---- chain wave
  __builtin_amdgcn_s_setprio(3);
  const uint32_t j0 = base + (uint32_t)wave * kJobs;
  if (j0 >= njobs) return;  // no producer waits for this chain wave (nchains above)
  FedSlot& P = L.slot[wave];
  DeepMsg* msgs = L.msg[wave];
  const Tables& T = reinterpret_cast<const Tables&>(L.tab);  // slice8 only (deep_head, deep_rest<false>)
  for (int m = 0; m < kJobs; ++m) {  // heads (state parked in LDS)
    const uint32_t j = j0 + (uint32_t)m;
    DeepMsg M{};
    if (j < njobs) M = deep_head(T, lane, load_job(jobs, j, lane), L.xs[wave][m]);
    wave_lds_sync();
    if (lane == 0) msgs[m] = M;
  }
  wave_lds_sync();
  // Joint rounds as in group_kernel, but down to a single job: a lone job still runs at the fed
  // chain's latency, and afterwards every job has fewer than G bulk blocks left.
  uint32_t gstep = 0;
  for (uint32_t round = 0; round < (uint32_t)kJobs; ++round) {
    uint64_t S = ~0ull;
    int joiners = 0;
    bool any_sha = false, any_crc = false, all16 = true;
    for (int m = 0; m < kJobs; ++m) {
      const DeepMsg M = uniform_msg(msgs[m]);
      const uint64_t left = M.live ? (M.nbulk - M.done) / G : 0;
      if (left == 0) continue;
      ++joiners;
      S = left < S ? left : S;
      const DeepJob J = load_job(jobs, j0 + (uint32_t)m, lane);
      any_sha |= J.st != nullptr;
      any_crc |= J.cs != nullptr;
      all16 &= (reinterpret_cast<uintptr_t>(M.q + 64 * M.done) & 15) == 0;
    }
    if (joiners == 0) break;
    for (int m = 0; m < kJobs; ++m) {
      const DeepMsg M = uniform_msg(msgs[m]);
      if (lane == 0) msgs[m].joint = M.live && (M.nbulk - M.done) / G > 0 ? 1u : 0u;
    }
    if (lane == 0) {
      P.S = S;
      P.flags = (any_sha ? 1u : 0u) | (any_crc ? 2u : 0u) | (all16 ? 4u : 0u);
    }
    lds_rel32(&P.req, round + 1);  // release: the messages and S above are visible first
    uint32_t hv[5] = {0, 0, 0, 0, 0};
    if (any_sha) fed_consume<G, X>(P, lane, msgs, S, gstep, hv);
    while (!reached(lds_acq32(&P.crc_done), round + 1)) __builtin_amdgcn_s_sleep(1);
    const int m = lane / G;
    const bool joint = msgs[m].joint != 0;
    wave_lds_sync();
    if (joint && (lane % G) == 0) {
      DeepMsg& W = msgs[m];
#pragma unroll
      for (int k = 0; k < 5; ++k) W.h[k] = any_sha ? hv[k] : W.h[k];
      W.done += S * G;
    }
    wave_lds_sync();
  }
  lds_rel32(&P.fin, 1);
  for (int m = 0; m < kJobs; ++m) {  // per job: the < G left-over blocks, tail, Sum, write-back
    const uint32_t j = j0 + (uint32_t)m;
    if (j >= njobs) break;
    DeepMsg M = uniform_msg(msgs[m]);
    if (!M.live) continue;
    const DeepJob J = load_job(jobs, j, lane);
    for (; M.done < M.nbulk; ++M.done) {  // one block at a time, the same in every lane
      uint32_t le[16];
      load_block_le<false>(M.q + 64 * M.done, le);
      if (J.cs) M.crc_raw = crc_words_raw(T.slice8, M.crc_raw, le);
      if (J.st) {
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = bswap(le[k]);
        compress_inline(M.h, w);
      }
    }
    deep_rest<false>(T, lane, J, L.xs[wave][m], L.fin[wave], M);
  }
}

// ================================================================== WIDE kernel
// One lane per job.  Per-lane tail buffers live in LDS with a 68-byte stride (17 dwords:
// lanes touching the same byte index hit different banks).
//
// A workgroup holds every wave a SIMD will run in the launch: 4 x wps waves (wps = waves per SIMD,
// 1..3; wave w runs on SIMD w % 4), one workgroup per CU.  The SIMD issues from the oldest ready
// wave first, so of wps waves with equally long messages the oldest ran at nearly a lone wave's
// rate and ended first, and the last one ran alone -- at a lone wave's ~5.1 cycles per VALU
// instead of 4 -- for the last ~30 % of the launch (per-wave timeline, profiles/r03_wide_timeline:
// the SIMD busy 62 of 72.5 ms).  So the waves of a SIMD publish their progress in LDS and, once per
// loop iteration, the furthest behind takes the top priority and the furthest ahead the lowest
// (s_setprio): they advance together and end together.
constexpr int kWideWaves = 4;    // waves per workgroup per SIMD-wave (one per SIMD)
constexpr int kWideMaxWps = 3;   // waves per SIMD that fit (132 VGPRs)
constexpr int kXStride = 68;

// WIDE's CRC tables in LDS: the position tables (crc_issue below).
using WideCrcTab = uint32_t[64][256];

struct WideLDS {
  WideCrcTab crc;  // PosTables (64 KiB)
  uint32_t prog[kWideWaves * kWideMaxWps];  // blocks done by each wave of the workgroup
};
// The byte-wise head/tail: pos[63][b] (byte b, no byte after it) is IEEETable[b] (crc32.go:125).
__device__ __forceinline__ const uint32_t* wide_t0(const WideLDS& L) { return L.crc[63]; }
__device__ __forceinline__ const uint4* wide_tab_src(const Tables* tabs) {
  return reinterpret_cast<const uint4*>(tabs + 1);  // PosTables follow Tables (efes_ctx_create)
}

// The priority of wave w from its SIMD siblings' progress (w % 4, w % 4 + 4, ...): the furthest
// behind gets 3, the furthest ahead 0, the rest 1.  Wave-uniform; `b` = blocks this wave has done.
__device__ __forceinline__ void wide_pace(uint32_t* prog, uint32_t w, uint32_t nw, uint32_t b) {
  if (nw <= kWideWaves) return;  // one wave per SIMD: nothing to share
  __builtin_amdgcn_sched_barrier(0);
  if ((threadIdx.x & 63) == 0) __atomic_store_n(&prog[w], b, __ATOMIC_RELAXED);
  uint32_t lo = 0xffffffffu, hi = 0;
  for (uint32_t v = w & 3; v < nw; v += kWideWaves) {
    if (v == w) continue;
    const uint32_t o = __atomic_load_n(&prog[v], __ATOMIC_RELAXED);
    lo = o < lo ? o : lo;
    hi = o > hi ? o : hi;
  }
  lo = uniform32(lo);
  hi = uniform32(hi);
  if (b <= lo) __builtin_amdgcn_s_setprio(3);
  else if (b >= hi) __builtin_amdgcn_s_setprio(0);
  else __builtin_amdgcn_s_setprio(1);
  __builtin_amdgcn_sched_barrier(0);
}

// Byte i of the padded final stream x[:nxf] || 0x80 || 0.. || BE64(bits), length T.
__device__ __forceinline__ uint32_t fin_byte(const uint8_t* xl, uint32_t i, uint32_t nxf, uint32_t T, uint64_t bits) {
  if (i < nxf) return xl[i];
  if (i == nxf) return 0x80u;
  if (i >= T - 8) return (uint32_t)(bits >> (56 - 8 * (i - (T - 8)))) & 0xffu;
  return 0u;
}

// Whole blocks of one lane's message, software-pipelined: the next block is in flight while
// the current one is compressed (a lone uncoalesced 64-B load per lane would otherwise expose
// the full memory latency every block).  kSha/kCrc are wave-uniform template flags, so CRC
// lookups and SHA-1 rounds share one basic block; a lane that needs only one of the two
// computes both and never stores the other.  Lanes run their own trip counts; with jobs
// sorted by length the lanes of a wave finish together.

// The block's raw CRC from the position tables (pos[o][b]: the register after a 64-byte block
// whose only nonzero byte is b at offset o; efes_internal.hpp): crc32.go:153-169's slicing over
// the whole block at once.  The register is linear, so the new register is the XOR of 64
// lookups, and only the first four (bytes 0..3 XOR the old register, crc32.go:157) depend on the
// previous block.  Split in eight groups of eight bytes (LE words 2S, 2S+1): a group's lookups are
// issued first, the XORs that fold them into the running value come five SHA-1 rounds later.
// 97 VALU per block (64 lookup addresses, 1 + 32 XORs) against 112 for slicing-by-8's eight
// dependent steps (round 3 A/B, profiles/r03_wide_crc_ab/).
struct CrcPending {
  uint32_t v[8];
};
template <int S>
__device__ __forceinline__ void crc_issue(const WideCrcTab& t, uint32_t crc, const uint32_t (&le)[16], CrcPending& p) {
  const uint32_t lo = S == 0 ? crc ^ le[0] : le[2 * S];
  const uint32_t hi = le[2 * S + 1];
  constexpr int o = 8 * S;
  p.v[0] = t[o + 0][lo & 0xffu]; p.v[1] = t[o + 1][(lo >> 8) & 0xffu]; p.v[2] = t[o + 2][(lo >> 16) & 0xffu];
  p.v[3] = t[o + 3][lo >> 24]; p.v[4] = t[o + 4][hi & 0xffu]; p.v[5] = t[o + 5][(hi >> 8) & 0xffu];
  p.v[6] = t[o + 6][(hi >> 16) & 0xffu]; p.v[7] = t[o + 7][hi >> 24];
}
// Group S's eight values folded into the running value `acc` (group 0 starts it).
template <int S>
__device__ __forceinline__ uint32_t crc_combine(const CrcPending& p, uint32_t acc) {
  const uint32_t a = __builtin_amdgcn_bitop3_b32(p.v[0], p.v[1], p.v[2], 0x96);
  const uint32_t b = __builtin_amdgcn_bitop3_b32(p.v[3], p.v[4], p.v[5], 0x96);
  if constexpr (S == 0) return __builtin_amdgcn_bitop3_b32(a, b, p.v[6] ^ p.v[7], 0x96);
  const uint32_t c = __builtin_amdgcn_bitop3_b32(acc, a, b, 0x96);
  return __builtin_amdgcn_bitop3_b32(c, p.v[6], p.v[7], 0x96);
}

// 80 inline SHA-1 rounds with the 8 CRC groups of the same block woven in: group k's lookups are
// issued after round 10k+4 and combined after round 10k+9, so the LDS latency of the lookups is
// covered by SHA-1 rounds.  Scheduling barriers every five rounds keep the compiler from
// regrouping the CRC groups into back-to-back lookup/wait clusters.  `crc` is the register
// before the block until group 0 is issued, the running value after.
template <int R, bool kSha, bool kCrc>
struct WideRounds {
  __device__ __forceinline__ static void run(uint32_t (&s)[5], uint32_t (&w)[16], const WideCrcTab& t, uint32_t& crc,
                                             const uint32_t (&le)[16], CrcPending& p) {
    if constexpr (kSha) round_inline<R>(s, w);
    if constexpr (kCrc && R % 10 == 4) crc_issue<R / 10>(t, crc, le, p);
    if constexpr (kCrc && R % 10 == 9) {
      crc = crc_combine<R / 10>(p, crc);
      // Pins the fold here: the 64-term XOR is otherwise reassociated into one tree at the end of
      // the block, with all 64 lookups live at once (168 VGPRs and spills).
      asm volatile("" : "+v"(crc));
    }
    if constexpr (kSha && kCrc && R % 5 == 4) __builtin_amdgcn_sched_barrier(0);
    WideRounds<R + 1, kSha, kCrc>::run(s, w, t, crc, le, p);
  }
};
template <bool kSha, bool kCrc>
struct WideRounds<80, kSha, kCrc> {
  __device__ __forceinline__ static void run(uint32_t (&)[5], uint32_t (&)[16], const WideCrcTab&, uint32_t&,
                                             const uint32_t (&)[16], CrcPending&) {}
};

// One block of one lane's message; `live` lanes (b < their own block count) commit the result.
template <bool kSha, bool kCrc>
__device__ __forceinline__ void wide_step(const uint32_t (&le)[16], const WideCrcTab& t, uint32_t (&h)[5],
                                          uint32_t& crc_raw, bool live) {
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = bswap(le[k]);
  uint32_t s[5] = {h[0], h[1], h[2], h[3], h[4]};
  uint32_t c = crc_raw;
  CrcPending p;
  WideRounds<0, kSha, kCrc>::run(s, w, t, c, le, p);
  if constexpr (kSha) {
#pragma unroll
    for (int k = 0; k < 5; ++k) h[k] = live ? h[k] + s[k] : h[k];
  }
  if constexpr (kCrc) crc_raw = live ? c : crc_raw;
}

// Whole blocks of one lane's message: block b is hashed (SHA-1 rounds and CRC steps woven
// together) while the next blocks are in flight (three 16-word buffers, the loop unrolled so the
// buffers keep their registers).  Two phases:
//  * uniform: while every lane of the wave still has the blocks being hashed and prefetched
//    (b+5 < nmin, the wave's shortest message), loads are unconditional, a whole 128-B line (two
//    blocks) at a time, and every lane commits -- no per-lane selects (8 VALU per block fewer
//    than the ragged phase);
//  * ragged: up to the wave's longest message (`nmax`, uniform), so the loads stay
//    unconditional and the compiler's vmcnt waits exact; lanes past their own last block
//    load a harmless `dummy` block and do not commit.
// kSha/kCrc are wave-uniform template flags; a lane that needs only one of the two computes
// both and never stores the other.  Jobs sorted by length keep the lanes of a wave equally long.
template <bool kAligned16, bool kSha, bool kCrc>
__device__ __forceinline__ void wide_bulk(const uint8_t* q, uint64_t nbulk, uint64_t nmin, uint64_t nmax,
                                          const uint8_t* dummy, const WideCrcTab& t, uint32_t (&h)[5],
                                          uint32_t& crc_raw, uint32_t* prog, uint32_t w, uint32_t nw) {
  auto src = [&](uint64_t b) { return b < nbulk ? q + 64 * b : dummy; };
  uint32_t A[16], B[16], C[16];
  if (nmax == 0) return;
  load_block_le<kAligned16>(src(0), A);
  load_block_le<kAligned16>(src(1), B);
  uint64_t b = 0;
  // Uniform phase (blocks b..b+5 exist in every lane), a 128-B line at a time: the two blocks of a
  // line are loaded back to back (eight dwordx4), one block-time before the first is hashed.  A
  // lane's blocks loaded one at a time, a block apart (the A/B build below), fetched 14.5 % more
  // than the message from HBM (FETCH_SIZE x 2, calibrated on this access pattern with
  // tools/microbench/mb_wide_fetch: profiles/r04_fetch/): the second half of a line was often
  // evicted from L2 before the lane came back for it.  A holds the even block, B / C the odd one.
  for (; b + 5 < nmin; b += 4) {
    if (b % 32 == 0) wide_pace(prog, w, nw, (uint32_t)b);  // every 32 blocks (profiles/r05_wide_pace_ab/)
    const uint8_t* qb = q + 64 * b;
    wide_step<kSha, kCrc>(A, t, h, crc_raw, true);
    load_block_le<kAligned16>(qb + 128, A);
    load_block_le<kAligned16>(qb + 192, C);
    wide_step<kSha, kCrc>(B, t, h, crc_raw, true);
    wide_step<kSha, kCrc>(A, t, h, crc_raw, true);
    load_block_le<kAligned16>(qb + 256, A);
    load_block_le<kAligned16>(qb + 320, B);
    wide_step<kSha, kCrc>(C, t, h, crc_raw, true);
  }
  // ragged phase (A, B hold blocks b, b+1 or the dummy), paced at its start and every 6 blocks
  // (counted from the start: b enters at a multiple of 4, so b % 6 alone could skip every pace)
  for (const uint64_t b_ragged = b; b < nmax; b += 3) {
    if ((b - b_ragged) % 6 == 0) wide_pace(prog, w, nw, (uint32_t)b);
    load_block_le<kAligned16>(src(b + 2), C);
    wide_step<kSha, kCrc>(A, t, h, crc_raw, b < nbulk);
    if (b + 1 >= nmax) break;
    load_block_le<kAligned16>(src(b + 3), A);
    wide_step<kSha, kCrc>(B, t, h, crc_raw, b + 1 < nbulk);
    if (b + 2 >= nmax) break;
    load_block_le<kAligned16>(src(b + 4), B);
    wide_step<kSha, kCrc>(C, t, h, crc_raw, b + 2 < nbulk);
  }
}
template <bool kAligned16>
__device__ __forceinline__ void wide_bulk_any(const uint8_t* q, uint64_t nbulk, uint64_t nmin, uint64_t nmax,
                                              const uint8_t* dummy, bool any_sha, bool any_crc,
                                              const WideCrcTab& t, uint32_t (&h)[5], uint32_t& crc_raw,
                                              uint32_t* prog, uint32_t w, uint32_t nw) {
  if (any_sha && any_crc) wide_bulk<kAligned16, true, true>(q, nbulk, nmin, nmax, dummy, t, h, crc_raw, prog, w, nw);
  else if (any_sha) wide_bulk<kAligned16, true, false>(q, nbulk, nmin, nmax, dummy, t, h, crc_raw, prog, w, nw);
  else if (any_crc) wide_bulk<kAligned16, false, true>(q, nbulk, nmin, nmax, dummy, t, h, crc_raw, prog, w, nw);
}

// Wave-wide minimum of a per-lane 64-bit value over the lanes where `use` holds (uniform
// result; ~0 when no lane does).
__device__ __forceinline__ uint64_t wave_min64(uint64_t v, bool use) {
  v = use ? v : ~0ull;
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const uint64_t o = (uint64_t)__shfl_xor((unsigned long long)v, k);
    v = o < v ? o : v;
  }
  return uniform64(v);
}

// Wave-wide maximum of a per-lane 64-bit value (uniform result).
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const uint64_t o = (uint64_t)__shfl_xor((unsigned long long)v, k);
    v = o > v ? o : v;
  }
  return uniform64(v);
}


__global__ __launch_bounds__(64 * kWideWaves * kWideMaxWps, 1) void wide_kernel(const efes_job* __restrict__ jobs,
                                                                                uint32_t njobs,
                                                                                const Tables* __restrict__ tabs) {
  __shared__ __attribute__((aligned(16))) WideLDS L;
  extern __shared__ __attribute__((aligned(16))) uint8_t wide_xs[];  // blockDim.x x kXStride (launch_wide)
  {
    const uint4* src = wide_tab_src(tabs);
    uint4* dst = reinterpret_cast<uint4*>(L.crc);
    for (int i = threadIdx.x; i < (int)(sizeof(L.crc) / 16); i += blockDim.x) dst[i] = src[i];
    if (threadIdx.x < kWideWaves * kWideMaxWps) L.prog[threadIdx.x] = 0;
  }
  __syncthreads();
  const uint32_t wv = threadIdx.x / 64, nwv = blockDim.x / 64;
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = j < njobs;
  const efes_job jb = live ? jobs[j] : efes_job{};
  const uint8_t* p = reinterpret_cast<const uint8_t*>(jb.data);
  const uint64_t plen = jb.length;
  efes_sha1_state* st = jb.sha1;
  efes_crc32_state* cs = jb.crc32;
  const bool do_sha = live && st != nullptr, do_crc = live && cs != nullptr;
  const bool fin = live && (jb.flags & EFES_JOB_FINALIZE) != 0;
  uint8_t* xl = wide_xs + (size_t)threadIdx.x * kXStride;
  int32_t status = EFES_OK;

  uint32_t h[5] = {0, 0, 0, 0, 0};
  int64_t nx = 0;
  uint64_t len = 0;
  const bool init = live && (jb.flags & EFES_JOB_INIT) != 0;
  if (do_sha && init) {  // NewSha1() (sha1.go:36-52)
    h[0] = kIV0; h[1] = kIV1; h[2] = kIV2; h[3] = kIV3; h[4] = kIV4;
#pragma unroll
    for (int k = 0; k < 64; ++k) xl[k] = 0;
  } else if (do_sha) {
#pragma unroll
    for (int k = 0; k < 5; ++k) h[k] = st->h[k];
    nx = st->nx;
    len = st->len;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t v = reinterpret_cast<const uint32_t*>(st->x)[k];
      xl[4 * k] = (uint8_t)v; xl[4 * k + 1] = (uint8_t)(v >> 8); xl[4 * k + 2] = (uint8_t)(v >> 16); xl[4 * k + 3] = (uint8_t)(v >> 24);
    }
  }
  uint32_t crc_raw = do_crc ? (init ? 0xFFFFFFFFu : ~cs->crc) : 0u;
  const bool bad = do_sha && nx > 64;  // sha1.go:62 panic
  const bool go = live && !bad;

  // ---- head
  uint64_t pos = 0;
  int64_t nx_new = nx;
  if (go && do_sha && nx > 0) {
    const uint32_t room = (uint32_t)(64 - nx);
    const uint32_t nh = plen < room ? (uint32_t)plen : room;
    for (uint32_t i = 0; i < nh; ++i) xl[nx + i] = ldg_u8(p + i);
    if ((uint32_t)nx + nh == 64) {
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = be_word_lds(xl, k);
      compress_inline(h, w);
      nx_new = 0;
    } else {
      nx_new = nx + nh;
    }
    pos = nh;
  }
  if (go && do_crc)
    for (uint64_t i = 0; i < pos; ++i) crc_raw = crc_byte(wide_t0(L), crc_raw, ldg_u8(p + i));

  // ---- bulk: lanes iterate their own block counts (masked when done)
  const uint8_t* q = p + pos;
  const uint64_t nbulk = go ? (plen - pos) >> 6 : 0;
  const bool all16 = __all(!go || (reinterpret_cast<uintptr_t>(q) & 15) == 0);
  const bool any_sha = __any(do_sha), any_crc = __any(do_crc);  // wave-uniform
  const uint64_t nmax = wave_max64(nbulk);
  // the shortest message over ALL lanes (a lane without a job has nbulk 0: no uniform phase)
  const uint64_t nmin = wave_min64(nbulk, true);
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(tabs);  // 36 KiB of valid device memory
  if (all16) wide_bulk_any<true>(q, nbulk, nmin, nmax, dummy, any_sha, any_crc, L.crc, h, crc_raw, L.prog, wv, nwv);
  else wide_bulk_any<false>(q, nbulk, nmin, nmax, dummy, any_sha, any_crc, L.crc, h, crc_raw, L.prog, wv, nwv);
  if ((threadIdx.x & 63) == 0) __atomic_store_n(&L.prog[wv], 0xffffffffu, __ATOMIC_RELAXED);  // done: never the slowest

  // ---- tail
  const uint64_t tpos = pos + (nbulk << 6);
  const uint32_t r = go ? (uint32_t)(plen - tpos) : 0u;
  if (do_crc)
    for (uint32_t i = 0; i < r; ++i) crc_raw = crc_byte(wide_t0(L), crc_raw, ldg_u8(p + tpos + i));
  if (do_sha && r > 0) {
    for (uint32_t i = 0; i < r; ++i) xl[i] = ldg_u8(p + tpos + i);
    nx_new = r;
  }
  len += go ? plen : 0;

  // ---- Sum
  uint32_t dig[5] = {0, 0, 0, 0, 0};
  if (go && fin && do_sha) {
    const uint32_t nxf = nx_new > 0 ? (uint32_t)nx_new : 0u;
    const uint32_t lm = (uint32_t)(len & 63);
    const uint32_t padlen = lm < 56 ? 56 - lm : 120 - lm;
    const uint32_t T = nxf + padlen + 8;
    if (T & 63) {
      status = EFES_ERR_STATE;
    } else {
      const uint64_t bits = len << 3;
      uint32_t hf[5] = {h[0], h[1], h[2], h[3], h[4]};
      for (uint32_t blk = 0; blk < T / 64; ++blk) {
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const uint32_t i = 64 * blk + 4 * k;
          w[k] = fin_byte(xl, i, nxf, T, bits) << 24 | fin_byte(xl, i + 1, nxf, T, bits) << 16 |
                 fin_byte(xl, i + 2, nxf, T, bits) << 8 | fin_byte(xl, i + 3, nxf, T, bits);
        }
        compress_inline(hf, w);
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) dig[k] = hf[k];
    }
  }

  // ---- write back (a Sum-only job leaves the states alone: Go's Sum works on a copy)
  const bool keep = (jb.flags & EFES_JOB_SUM_ONLY) != 0;
  if (go) {
    if (do_sha && !keep) {
#pragma unroll
      for (int k = 0; k < 5; ++k) st->h[k] = h[k];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        reinterpret_cast<uint32_t*>(st->x)[k] = (uint32_t)xl[4 * k] | (uint32_t)xl[4 * k + 1] << 8 |
                                                (uint32_t)xl[4 * k + 2] << 16 | (uint32_t)xl[4 * k + 3] << 24;
      st->nx = nx_new;
      st->len = len;
    }
    if (do_crc && !keep) cs->crc = ~crc_raw;
    if (fin && jb.sum) {
#pragma unroll
      for (int k = 0; k < 5; ++k) reinterpret_cast<uint32_t*>(jb.sum)[k] = bswap(status == EFES_OK ? dig[k] : 0u);
      reinterpret_cast<uint32_t*>(jb.sum)[5] = bswap(do_crc ? ~crc_raw : 0u);
    }
  }
  if (live && jb.status) *jb.status = bad ? EFES_ERR_STATE : status;
}


// ================================================================== synthetic fill
__device__ __forceinline__ uint64_t splitmix(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void fill_kernel(uint64_t* __restrict__ dst, uint64_t nwords, uint64_t seed, uint8_t* tail_dst,
                            uint32_t tail_bytes) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += stride) dst[i] = splitmix(seed, i);
  if (blockIdx.x == 0 && threadIdx.x == 0 && tail_bytes) {
    const uint64_t z = splitmix(seed, nwords);
    for (uint32_t b = 0; b < tail_bytes; ++b) tail_dst[b] = (uint8_t)(z >> (8 * b));
  }
}

// ================================================================== launchers
hipError_t launch_deep(const efes_job* jobs, uint32_t njobs, const Tables* tabs, hipStream_t s) {
  if (njobs == 0) return hipSuccess;
  const uint32_t grid = (njobs + kPipeJobs - 1) / kPipeJobs;
  clear_last_error();
  hipLaunchKernelGGL(deep_kernel, dim3(grid), dim3(128 * kPipeJobs), 0, s, jobs, njobs, tabs);
  return hipGetLastError();
}

// LDS of one CU on gfx950; an exclusive launch asks for all of it per workgroup.
constexpr size_t kCuLds = 160 * 1024;

template <class K, class... A>
hipError_t launch_reserving(K kernel, dim3 grid, dim3 block, bool exclusive, hipStream_t s, const efes_job* jobs,
                            uint32_t njobs, const Tables* tabs, A... more) {
  size_t dyn = 0;
  if (exclusive) {
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kernel)) == hipSuccess && fa.sharedSizeBytes < kCuLds) {
      dyn = kCuLds - fa.sharedSizeBytes;
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)dyn) != hipSuccess)
        dyn = 0;  // cannot reserve: run shared
    }
  }
  clear_last_error();
  hipLaunchKernelGGL(kernel, grid, block, dyn, s, jobs, njobs, tabs, more...);
  return hipGetLastError();
}

hipError_t launch_group(const efes_job* jobs, uint32_t njobs, int G, const Tables* tabs, hipStream_t s, bool exclusive) {
  if (njobs == 0) return hipSuccess;
  const uint32_t per_block = kDeepWaves * (64u / (uint32_t)G);
  const dim3 grid((njobs + per_block - 1) / per_block), block(64 * kDeepWaves);
  switch (G) {
    case 4: return launch_reserving(group_kernel<4>, grid, block, exclusive, s, jobs, njobs, tabs);
    case 8: return launch_reserving(group_kernel<8>, grid, block, exclusive, s, jobs, njobs, tabs);
    case 16: return launch_reserving(group_kernel<16>, grid, block, exclusive, s, jobs, njobs, tabs);
    case 32: return launch_reserving(group_kernel<32>, grid, block, exclusive, s, jobs, njobs, tabs);
    case 64: return launch_reserving(deep_kernel, dim3((njobs + kPipeJobs - 1) / kPipeJobs), dim3(128 * kPipeJobs),
                                     exclusive, s, jobs, njobs, tabs);
    default: return hipErrorInvalidValue;
  }
}

// FED shape of a mode: lanes per job and chain waves per workgroup.
constexpr int kFed4G = 4, kFed4C = 2;

template <int G, int C, bool X = false>
hipError_t launch_fed_shape(const efes_job* jobs, uint32_t njobs, const Tables* tabs, hipStream_t s) {
  const uint32_t per = C * (64 / G);
  return launch_reserving(fed_kernel<G, C, X>, dim3((njobs + per - 1) / per), dim3(256), true, s, jobs, njobs, tabs);
}

hipError_t launch_fed(const efes_job* jobs, uint32_t njobs, const Tables* tabs, hipStream_t s, bool expand) {
  if (njobs == 0) return hipSuccess;
  if (expand) return launch_fed_shape<4, 3, true>(jobs, njobs, tabs, s);  // FED4E
  return launch_fed_shape<kFed4G, kFed4C>(jobs, njobs, tabs, s);          // FED4
}

hipError_t launch_wide(const efes_job* jobs, uint32_t njobs, const Tables* tabs, hipStream_t s, bool exclusive,
                       int cus) {
  if (njobs == 0) return hipSuccess;
  // waves per SIMD of the launch: a workgroup per CU holds all of its SIMDs' waves (wide_pace);
  // exclusive parts (one wave per SIMD on reserved CUs) use 4-wave groups.
  const uint64_t waves = (njobs + 63) / 64, simds = 4ull * (uint64_t)(cus > 0 ? cus : 256);
  const uint32_t wps = exclusive ? 1u : (uint32_t)std::min<uint64_t>(kWideMaxWps, (waves + simds - 1) / simds);
  const uint32_t per = 64 * kWideWaves * wps;
  const size_t xs = (size_t)per * kXStride;  // the lanes' tail buffers (dynamic LDS)
  // The kernel's static LDS, and the dynamic-LDS limit raised once to the rest of the CU's LDS
  // (per launch `dyn` decides what a workgroup takes).
  // Per device (the attribute is set on the current one; the caller holds a DeviceGuard).
  static std::mutex mu;
  static int8_t ok_dev[64] = {};  // 0 = not tried, 1 = raised, -1 = failed
  static size_t static_lds = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  bool big_ok = false;
  {
    std::lock_guard<std::mutex> lk(mu);
    int8_t& st = ok_dev[dev & 63];
    if (st == 0) {
      hipFuncAttributes fa{};
      st = -1;
      if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(wide_kernel)) == hipSuccess) {
        static_lds = fa.sharedSizeBytes;
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(wide_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kCuLds - static_lds)) == hipSuccess)
          st = 1;
      }
    }
    big_ok = st == 1;
  }
  // without the raised limit a workgroup gets 64 KiB of LDS in all (static: the CRC tables)
  if (!big_ok && sizeof(WideLDS) + xs > 64 * 1024) return hipErrorInvalidConfiguration;
  // exclusive: reserve the CU's whole LDS, so no other workgroup shares its SIMDs
  const size_t dyn = exclusive && big_ok ? kCuLds - static_lds : xs;
  clear_last_error();
  hipLaunchKernelGGL(wide_kernel, dim3((njobs + per - 1) / per), dim3(per), dyn, s, jobs, njobs, tabs);
  return hipGetLastError();
}

hipError_t launch_fill(void* dst, size_t bytes, uint64_t seed, hipStream_t s) {
  const uint64_t nwords = bytes / 8;
  const uint32_t tail = (uint32_t)(bytes % 8);
  uint64_t blocks = (nwords + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) blocks = 1;
  clear_last_error();
  hipLaunchKernelGGL(fill_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, reinterpret_cast<uint64_t*>(dst), nwords,
                     seed, reinterpret_cast<uint8_t*>(dst) + nwords * 8, tail);
  return hipGetLastError();
}

}  // namespace efes
