// efes_crc_span.hip -- CRC-32/IEEE of ONE long device buffer on the whole GPU.
//
// The reference's crc32digest.Write (crc32.go:76-86 -> slicingUpdate :153-169) is a serial byte
// loop; the fused upload kernels keep it serial per chunk because SHA-1 is serial anyway.  When
// only the CRC of one large object is wanted (an object re-checked after a drain or a copy,
// chunks of one object on several GPUs), CRC-32 is GF(2)-linear, so any split of the bytes can be
// CRC'd independently and merged:
//   raw(A||B) = Z^|B| raw(A) ^ raw(B),  Z^n(v) = v * x^(8n) mod P  (reflected representation)
// (the crc32_combine identity, efes_crc32_combine in efes_api.cpp), and Go's finalized update is
// crc' = ~(Z^n(~crc) ^ raw(p)) (crc32.go:123,127).
//
// Layout of one launch over n = head + 64*nline + rest bytes (kSpanLine = 64):
//   * span_prep_kernel (one lane): the <= 15 head bytes up to the first 16-byte boundary and the
//     < 64 rest bytes byte-wise (crc32.go:125); the state becomes ~Z^m(~crc_head) ^ raw(rest)
//     with m the bytes after the head -- every bulk contribution below is then XORed into it;
//   * span_kernel: rows of L = 1024 lines (64 KiB) are dealt round-robin -- workgroup w takes rows
//     w, w+G, w+2G, ... (G workgroups, one per CU), so the whole GPU sweeps the buffer front to back
//     -- and lane j takes line j of each of its rows (a wave's 64 lines of a row are 4 KiB, staged
//     into the wave's LDS slot by nontemporal LDS-DMA while the previous row is hashed).  Each
//     line's raw CRC comes from slicing-by-4 on lane-private copies of the tables in LDS (no bank
//     conflicts, one v_perm per lookup address) and is folded into the lane's accumulator,
//     acc = Z^(64LG)(acc) ^ raw(line) (a byte-sliced 4 x 256 table the workgroup builds from the
//     launch's stride operator).  At the end, lane j's accumulator is advanced over what follows
//     its last line -- the rest of that row (lane_op[L-1-j]) and everything after the row (op[w],
//     computed on the host), or for the partial last row lane_op[extra-1-j] and the rest bytes --
//     the lanes are XOR-reduced and the sum XORed into the state with one atomic per workgroup.
// Bound: HBM read (every byte once).  Round 5: 6.6-6.7 TB/s against 7.0-7.2 for LDS-DMA nt reads
// alone, with the engine clock power-limited to ~1.6 GHz while it runs (profiles/r05_span_ring/);
// sweeping rows round-robin rather than one contiguous range per workgroup keeps 6.3 TB/s on
// buffers whose allocation left the per-range layout at 5.9 (profiles/r05_span_alloc/).
// No SHA-1, no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "efes_internal.hpp"

namespace efes {

constexpr uint32_t kPolyReflected = 0xedb88320u;  // crc32.go:30 IEEE, reflected

// a * b mod P for polynomials in the reflected representation (bit 31 = x^0).  Branch-free, 32
// fixed steps (uniform control flow on the device).
__host__ __device__ inline uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    p ^= b & (0u - ((a >> (31 - i)) & 1u));
    b = (b >> 1) ^ (kPolyReflected & (0u - (b & 1u)));
  }
  return p;
}

// x^(8n) mod P: the operator that advances a raw CRC register over n zero bytes.
static uint32_t xpow8n(uint64_t n) {
  uint32_t x2n[32];            // x^(2^k) mod P; x^(2^32) = x for this primitive P, so k cycles mod 32
  x2n[0] = 1u << 30;           // x^1
  for (int k = 1; k < 32; ++k) x2n[k] = gf2_mulmod(x2n[k - 1], x2n[k - 1]);
  uint32_t p = 1u << 31;       // x^0
  for (int k = 3; n; n >>= 1, ++k)
    if (n & 1) p = gf2_mulmod(x2n[k & 31], p);
  return p;
}

void build_span_tables(SpanTables* t) {
  for (int k = 0; k < kSpanLanes; ++k) t->lane_op[k] = xpow8n((uint64_t)kSpanLine * (uint64_t)k);
}

struct SpanArgs {
  const uint8_t* bulk;  // 16-byte aligned, nline * kSpanLine bytes
  uint32_t* crc;        // the device state (finalized CRC), XOR target
  const Tables* tabs;   // slicing-by-8 tables (crc32.go:138-149)
  const SpanTables* span;
  uint64_t nline;
  uint32_t groups;
  uint32_t stride_op;           // x^(8 * 64 * L * groups): one workgroup's step from row to row
  uint32_t rest_op;             // x^(8 * rest)
  uint32_t _pad;
  uint32_t op[kSpanMaxGroups];  // x^(8 * bytes after workgroup w's last full row's line L-1) mod P
};
static_assert(sizeof(SpanArgs) <= 4096, "kernel argument segment");
static_assert(kSpanLine % 4 == 0, "whole words per line");

__global__ __launch_bounds__(64) void span_prep_kernel(const uint8_t* __restrict__ data, uint32_t head, uint32_t rest,
                                                       const uint8_t* __restrict__ rest_ptr, uint32_t after_head_op,
                                                       uint32_t* __restrict__ crc, const Tables* __restrict__ tabs) {
  if (threadIdx.x != 0) return;
  const uint32_t* t0 = tabs->slice8[0];
  uint32_t r = ~*crc;  // crc32.go:123
  for (uint32_t i = 0; i < head; ++i) r = t0[(r ^ data[i]) & 0xffu] ^ (r >> 8);  // crc32.go:125
  uint32_t tail = 0;   // raw CRC of the rest bytes from a zero register
  for (uint32_t i = 0; i < rest; ++i) tail = t0[(tail ^ rest_ptr[i]) & 0xffu] ^ (tail >> 8);
  // ~(Z^m(r) ^ raw(bulk||rest)): the bulk's contributions are XORed in by span_kernel.
  *crc = ~gf2_mulmod(after_head_op, r) ^ tail;
}

// LDS: the four slicing-by-4 tables (crc32.go:138-149's slicing8Table[0..3]) in one 64 KiB block --
// entry e of table t, copy c at byte e*256 + 64t + 4c, so table t sits in banks 16t..16t+15 -- and
// the read ring.  Lane j reads copy j mod 16, and its four lookups per word visit the tables in the
// rotated order t = (i + j/16) mod 4: in each lookup instruction the four 16-lane groups of a wave
// read four different tables, 64 different banks, so no instruction conflicts.  (Rounds 2-4 had
// every lane read the same table, which took 32 copies and 128 KiB for the same property.)  A
// lookup's address is still ONE v_perm_b32: byte 1 = the index byte of x, byte 0 = 64t + 4c from
// a lane constant, bytes 2-3 = 0.
constexpr int kSpanCopies = 16;
constexpr int kSpanWavesPerSimd = 4;  // one workgroup per CU
constexpr int kSpanWaves = kSpanLanes / 64;
constexpr int kLineWords = kSpanLine / 4;
static_assert(kSpanLine == 64, "one ring slot = 64 lines of 4 x 16 bytes");
// (The row shift keeps one copy: 2 or 4 copies measured no faster, DESIGN_NOTES.md.)
struct SpanLDS {
  uint32_t row_shift[4][256];           // 4 KiB at LDS address 0 (a lookup: one SDWA shift, the table in the offset)
  uint32_t slice[256][4][kSpanCopies];  // 64 KiB at 4 KiB (the ds_read offset)
  // Wave v's slot holds its 64 lines of the current row, the pieces of each line rotated (fetch_row).
  uint32_t ring[kSpanWaves][64 * kLineWords];  // 64 KiB
  uint32_t wave_sum[kSpanWaves];
};

// The lane's line read straight into registers (the partial last row only).
__device__ __forceinline__ void load_line(const uint8_t* src, uint32_t (&w)[kLineWords]) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const __attribute__((address_space(1))) v4u* s = (const __attribute__((address_space(1))) v4u*)src;
#pragma unroll
  for (int q = 0; q < kLineWords / 4; ++q) {
    const v4u v = s[q];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
}

// The wave's 64 lines of one row (4 KiB) into its ring slot by LDS-DMA with the nontemporal policy.
// Instruction k moves the row's bytes 1024k..1024k+1023 (lines 16k..16k+15, coalesced) and lane l
// of it lands at slot + 1024k + 16l.  Which 16 bytes lane l fetches is the swizzle (below): within
// each 64-byte line the four pieces are rotated by (line / 4) mod 4, so that when every lane then
// reads piece m of its own line, 16 neighbouring lanes hit 16 different 16-byte bank groups (the
// plain layout, a 64-byte stride, conflicts 4-way).  Fetching piece-major instead (instruction k =
// piece k of every line) avoids the conflict too but scatters each instruction over 4 KiB, which
// reads at 3.7 TB/s with the nontemporal policy (profiles/r05_span_ring/).
// The streamed bytes are read once, so they bypass the caches' retention (round 5: LDS-DMA nt
// reads at 7.0-7.2 TB/s where register loads top out at 6.2-6.3, profiles/r05_span_nt/).  Issued
// from inline assembly so the compiler does not see an LDS write in flight: it would otherwise
// wait for the DMA before every table lookup (the slot is only read after the explicit wait in
// span_kernel).  The lgkmcnt wait orders the slot's previous reads before the overwrite; M0 is the
// slot's LDS byte address (one wait state between writing M0 and the DMA).  LLVM reserves M0: a "m0"
// clobber is not honoured (clang warns and emits the same code), so the contract that nothing else
// in span_kernel keeps a value in M0 is checked on the compiled ISA by tests/test_span_isa.py.
//   slot unit (16 B) u = 4*line + ((piece + line/4) mod 4)
//   lane l of instruction k: unit 64k + l -> line 16k + l/4, piece ((l mod 4) - l/16) mod 4
__device__ __forceinline__ uint32_t fetch_offset(uint32_t lane) {
  return 64u * (lane >> 2) + 16u * (((lane & 3u) - (lane >> 4)) & 3u);
}
__device__ __forceinline__ uint32_t read_offset(uint32_t lane, int m) {
  return 64u * lane + 16u * (((uint32_t)m + (lane >> 2)) & 3u);
}
__device__ __forceinline__ void fetch_row(const uint8_t* src, uint32_t slot) {  // src: row chunk + fetch_offset
#pragma unroll
  for (int k = 0; k < kLineWords / 4; ++k)
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt"
        :
        : "v"(src + 1024 * k), "s"(slot + 1024u * k)
        : "memory");  // M0: no other user in span_kernel (tests/test_span_isa.py)
}

// Raw CRC (from a zero register) of one line: slicing-by-4 (the 4-byte form of crc32.go:157-161).
// lb: byte i = the lane's 64t + 4c for its i-th lookup; sel[i]: the v_perm selector for it (byte 0
// <- lb byte i, byte 1 <- x byte 3 - t, bytes 2-3 <- 0x00; selectors 0-3 pick the second operand's
// bytes, 4-7 the first's, 12 a zero).
__device__ __forceinline__ uint32_t line_raw(const SpanLDS& L, uint32_t lb, const uint32_t (&sel)[4],
                                             const uint32_t (&w)[kLineWords]) {
  const char* base = reinterpret_cast<const char*>(&L.slice);
  auto look = [&](uint32_t x, int i) {
    return *reinterpret_cast<const uint32_t*>(base + __builtin_amdgcn_perm(x, lb, sel[i]));
  };
  uint32_t x = w[0], crc = 0;  // x = crc ^ the next word (crc32.go:157's crc ^= ...)
#pragma unroll
  for (int s = 0; s < kLineWords; ++s) {
    const uint32_t p = __builtin_amdgcn_bitop3_b32(look(x, 0), look(x, 1), look(x, 2), 0x96);
    if (s + 1 < kLineWords)
      x = __builtin_amdgcn_bitop3_b32(p, look(x, 3), w[s + 1], 0x96);  // 6 VALU per 4 bytes
    else
      crc = p ^ look(x, 3);
  }
  return crc;
}

// Z^(64L)(v) ^ raw: the row shift of v (four lookups) folded with the next line's raw CRC.
__device__ __forceinline__ uint32_t row_advance(const uint32_t (&s)[4][256], uint32_t v, uint32_t raw) {
  const uint32_t p = __builtin_amdgcn_bitop3_b32(s[0][v & 0xffu], s[1][(v >> 8) & 0xffu], s[2][(v >> 16) & 0xffu], 0x96);
  return __builtin_amdgcn_bitop3_b32(p, s[3][v >> 24], raw, 0x96);
}

__global__ __launch_bounds__(kSpanLanes, kSpanWavesPerSimd) void span_kernel(const SpanArgs a) {
  __shared__ __attribute__((aligned(16))) SpanLDS L;
  {  // tables into LDS: each slicing entry kSpanCopies times (4 per ds_write_b128), the row shift once
    uint4* dst = reinterpret_cast<uint4*>(&L.slice);
    for (uint32_t i = threadIdx.x; i < sizeof(L.slice) / 16; i += kSpanLanes) {
      const uint32_t word = 4 * i;  // entry word >> 6, table (word >> 4) & 3
      const uint32_t v = a.tabs->slice8[(word >> 4) & 3u][word >> 6];
      dst[i] = make_uint4(v, v, v, v);
    }
    // the row shift for this launch's stride (groups rows): entry v of byte b = stride_op * (v << 8b)
    L.row_shift[threadIdx.x >> 8][threadIdx.x & 255u] = gf2_mulmod(a.stride_op, (threadIdx.x & 255u) << (8 * (threadIdx.x >> 8)));
  }
  // Rows of L lines are dealt round-robin: workgroup w takes rows w, w + G, w + 2G, ... (G =
  // groups), so the whole GPU sweeps the buffer front to back; the partial last row (extra lines)
  // goes to its round-robin owner.
  const uint32_t w = blockIdx.x, j = threadIdx.x, wave = j / 64, lane = j % 64;
  const uint64_t G = a.groups, rtot = a.nline / kSpanLanes;
  const uint32_t extra = (uint32_t)(a.nline % kSpanLanes);
  const uint64_t rows = rtot > w ? (rtot - 1 - w) / G + 1 : 0;  // full rows of this workgroup
  const bool partial = (rtot % G) == w && j < extra;            // this lane's line of the partial row
  const uint8_t* p = a.bulk + ((uint64_t)w * kSpanLanes + j) * kSpanLine;
  constexpr uint64_t kRow = (uint64_t)kSpanLine * kSpanLanes;
  const uint64_t kStride = kRow * G;
  uint32_t lb = 0, sel[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t t = (uint32_t)(i + (int)(j / 16)) & 3u;
    lb |= (64u * t + 4u * (j % kSpanCopies)) << (8 * i);
    sel[i] = 0x0C0C0000u | ((4u + 3u - t) << 8) | (uint32_t)i;
  }
  const uint32_t slot = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)&L.ring[wave][0]);
  __syncthreads();

  uint32_t acc = 0;
  if (rows) {
    // One row in flight per wave: the DMA of row g+1 lands while row g is hashed from registers.
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const char* mine = reinterpret_cast<const char*>(&L.ring[wave][0]);
    const uint8_t* src = p - kSpanLine * lane + fetch_offset(lane);
    fetch_row(src, slot);
    for (uint64_t g = 0; g < rows; ++g) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's row g is in its slot
      uint32_t line[kLineWords];
#pragma unroll
      for (int k = 0; k < kLineWords / 4; ++k) {
        const v4u v = *reinterpret_cast<const v4u*>(mine + read_offset(lane, k));
        line[4 * k] = v.x; line[4 * k + 1] = v.y; line[4 * k + 2] = v.z; line[4 * k + 3] = v.w;
      }
      if (g + 1 < rows) fetch_row(src + (g + 1) * kStride, slot);
      acc = row_advance(L.row_shift, acc, line_raw(L, lb, sel, line));
    }
  }
  uint32_t c = 0;
  if (partial) {  // the partial last row (row rtot = w + rows * G): followed by extra - 1 - j lines and rest
    uint32_t E[kLineWords];
    load_line(a.bulk + (rtot * kSpanLanes + j) * kSpanLine, E);
    acc = row_advance(L.row_shift, acc, line_raw(L, lb, sel, E));
    c = gf2_mulmod(a.rest_op, gf2_mulmod(a.span->lane_op[extra - 1 - j], acc));
  } else if (rows) {  // last line: row w + (rows-1) G, followed by L-1-j lines, then op[w]
    c = gf2_mulmod(a.op[w], gf2_mulmod(a.span->lane_op[kSpanLanes - 1 - j], acc));
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) c ^= __shfl_xor(c, off, 64);
  if ((j & 63) == 0) L.wave_sum[j / 64] = c;
  __syncthreads();
  if (j == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int v = 0; v < kSpanLanes / 64; ++v) t ^= L.wave_sum[v];
    atomicXor(a.crc, t);
  }
}

hipError_t launch_crc_span(const void* data, uint64_t length, uint32_t* crc, const Tables* tabs, const SpanTables* span,
                           int cus, hipStream_t s) {
  const uint8_t* d = static_cast<const uint8_t*>(data);
  const uint64_t head = length < (uint64_t)((16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15)
                            ? length
                            : (uint64_t)((16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15);
  const uint64_t m = length - head, nline = m / kSpanLine, rest = m % kSpanLine;
  const uint8_t* bulk = d + head;
  clear_last_error();
  hipLaunchKernelGGL(span_prep_kernel, dim3(1), dim3(64), 0, s, d, (uint32_t)head, (uint32_t)rest,
                     bulk + nline * kSpanLine, xpow8n(m), crc, tabs);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || nline == 0) return e;
  // Workgroups: as many as are resident at once (kSpanWavesPerSimd / 4 per CU), at least 4 rows
  // per lane.
  uint64_t groups = (nline + 4ull * kSpanLanes - 1) / (4ull * kSpanLanes);
  const uint64_t per_cu = kSpanWavesPerSimd / 4, resident = (uint64_t)(cus > 0 ? cus : 256) * per_cu;
  const uint64_t cap = resident < kSpanMaxGroups ? resident : (uint64_t)kSpanMaxGroups;
  if (groups > cap) groups = cap;
  if (groups > nline) groups = nline;
  if (groups == 0) groups = 1;
  SpanArgs a{};
  a.bulk = bulk;
  a.crc = crc;
  a.tabs = tabs;
  a.span = span;
  a.nline = nline;
  a.groups = (uint32_t)groups;
  a.stride_op = xpow8n((uint64_t)kSpanLine * kSpanLanes * groups);
  a.rest_op = xpow8n(rest);
  // op[w]: after workgroup w's last full row r_last come (rtot - 1 - r_last) = (rtot - 1 - w) mod G
  // full rows, the extra lines and the rest bytes.
  const uint64_t rtot = nline / kSpanLanes, extra = nline % kSpanLanes;
  const uint32_t base = xpow8n((uint64_t)kSpanLine * extra + rest), zrow = xpow8n((uint64_t)kSpanLine * kSpanLanes);
  uint32_t pw[kSpanMaxGroups];  // zrow^d
  pw[0] = 1u << 31;
  for (uint64_t d = 1; d < groups; ++d) pw[d] = gf2_mulmod(zrow, pw[d - 1]);
  for (uint64_t w = 0; w < groups; ++w)
    a.op[w] = w < rtot ? gf2_mulmod(base, pw[(rtot - 1 - w) % groups]) : 0u;
  clear_last_error();
  hipLaunchKernelGGL(span_kernel, dim3((uint32_t)groups), dim3(kSpanLanes), 0, s, a);
  return hipGetLastError();
}

}  // namespace efes
