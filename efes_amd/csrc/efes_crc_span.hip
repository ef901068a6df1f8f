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
//   * span_kernel: workgroup w owns a contiguous range of 64-byte lines; lane j takes lines j,
//     j+L, j+2L, ... (a wave reads 4 KiB per row), computes each line's raw CRC by slicing-by-4
//     from lane-private copies of the tables in LDS (no bank conflicts, one v_perm per lookup
//     address) and folds it into its accumulator, acc = Z^(64L)(acc) ^ raw(line) (a byte-sliced
//     4 x 256 table).  At the end, lane j's accumulator is advanced over the lines of the range
//     after its last line (one GF(2) product with lane_op[k] = x^(8*64*k)), the lanes are
//     XOR-reduced, the sum is advanced over the bytes after the range (op[w], computed on the
//     host) and XORed into the state with one atomic per workgroup.
// Bound: HBM read (every byte once); measured at ~93 % of a pure read kernel (DESIGN_NOTES.md §4 "Span
// CRC").  No SHA-1, no MFMA.
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
  const uint32_t row = xpow8n((uint64_t)kSpanLine * kSpanLanes);  // one workgroup row: L lines
  for (int b = 0; b < 4; ++b)
    for (uint32_t v = 0; v < 256; ++v) t->row_shift[b][v] = gf2_mulmod(row, v << (8 * b));
  for (int k = 0; k < kSpanLanes; ++k) t->lane_op[k] = xpow8n((uint64_t)kSpanLine * (uint64_t)k);
}

struct SpanArgs {
  const uint8_t* bulk;  // 16-byte aligned, nline * kSpanLine bytes
  uint32_t* crc;        // the device state (finalized CRC), XOR target
  const Tables* tabs;   // slicing-by-8 tables (crc32.go:138-149)
  const SpanTables* span;
  uint64_t nline;
  uint32_t groups;
  uint32_t _pad;
  uint32_t op[kSpanMaxGroups];  // x^(8 * bytes after workgroup w's range) mod P
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

// LDS: the four slicing-by-4 tables (crc32.go:138-149's slicing8Table[0..3]) with every entry
// stored 32 times side by side, lane j reading copy j mod 32, so a ds_read_b32 serves each 32-lane
// group in one LDS cycle with no bank conflict (random indices into one table conflict ~3.5-way).
// Layout (bytes): region r (tables 2r, 2r+1) at r*64 KiB, entry e at e*256 within it, table 2r+tt
// at tt*128, copy c at c*4 -- so a lookup's address is ONE v_perm_b32 (byte 1 = the index byte,
// byte 0 = 4c, byte 2 = r, byte 3 = 0) and the table's 128 goes in the ds_read offset.
// (Measured and not kept: 16 copies in one 64 KiB region with two workgroups per CU -- 2-way
// conflicts, 32 waves per CU -- ran at the same rate; DESIGN_NOTES.md §4 "Span CRC".)
constexpr int kSpanCopies = 32;
constexpr int kSpanWavesPerSimd = 4;  // one workgroup per CU
// (The row shift keeps one copy: 2 or 4 copies measured no faster, DESIGN_NOTES.md.)
struct SpanLDS {
  uint32_t slice[2][256][2][kSpanCopies];  // 128 KiB at LDS address 0
  uint32_t row_shift[4][256];              // 4 KiB
  uint32_t wave_sum[kSpanLanes / 64];
};

constexpr int kLineWords = kSpanLine / 4;
constexpr int kSpanBuf = 2;  // lines in flight per lane (round 2 A/B, profiles/r02_span/)

__device__ __forceinline__ void load_line(const uint8_t* src, uint32_t (&w)[kLineWords]) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const __attribute__((address_space(1))) v4u* s = (const __attribute__((address_space(1))) v4u*)src;
#pragma unroll
  for (int q = 0; q < kLineWords / 4; ++q) {
    const v4u v = s[q];  // (a nontemporal load measured no faster, round 2)
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
}

// v_perm_b32 selector: byte 0 <- lane byte 0 (4c), byte 1 <- x byte k, byte 2 <- lane byte 2 (r),
// byte 3 <- 0x00 (selector 12).  Selectors 0-3 pick the second operand's bytes, 4-7 the first's.
constexpr uint32_t perm_sel(int k) { return 0x0C020000u | ((4u + (uint32_t)k) << 8); }

__device__ __forceinline__ uint32_t lds_word(const SpanLDS& L, uint32_t byte_addr, uint32_t off) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(&L.slice) + byte_addr + off);
}
constexpr uint32_t kOff0 = 0, kOff1 = 128, kOff2 = 0, kOff3 = 128;  // table offsets within their region

// Raw CRC (from a zero register) of one line: slicing-by-4 (the 4-byte form of crc32.go:157-161),
// the lookups into this lane's copy.  l0 / l1: the lane's address bytes for region 0 / 1.
__device__ __forceinline__ uint32_t line_raw(const SpanLDS& L, uint32_t l0, uint32_t l1,
                                             const uint32_t (&w)[kLineWords]) {
  uint32_t x = w[0], crc = 0;  // x = crc ^ the next word (crc32.go:157's crc ^= ...)
#pragma unroll
  for (int s = 0; s < kLineWords; ++s) {
    const uint32_t t0 = lds_word(L, __builtin_amdgcn_perm(x, l0, perm_sel(3)), kOff0);  // tab[0][x >> 24]
    const uint32_t t1 = lds_word(L, __builtin_amdgcn_perm(x, l0, perm_sel(2)), kOff1);  // tab[1][x >> 16 & 0xff]
    const uint32_t t2 = lds_word(L, __builtin_amdgcn_perm(x, l1, perm_sel(1)), kOff2);  // tab[2][x >> 8 & 0xff]
    const uint32_t t3 = lds_word(L, __builtin_amdgcn_perm(x, l1, perm_sel(0)), kOff3);  // tab[3][x & 0xff]
    const uint32_t p = __builtin_amdgcn_bitop3_b32(t0, t1, t2, 0x96);
    if (s + 1 < kLineWords)
      x = __builtin_amdgcn_bitop3_b32(p, t3, w[s + 1], 0x96);  // 6 VALU per 4 bytes
    else
      crc = p ^ t3;
  }
  return crc;
}

__device__ __forceinline__ uint32_t row_advance(const uint32_t (&s)[4][256], uint32_t v) {
  return __builtin_amdgcn_bitop3_b32(s[0][v & 0xffu], s[1][(v >> 8) & 0xffu], s[2][(v >> 16) & 0xffu], 0x96) ^
         s[3][v >> 24];
}

__global__ __launch_bounds__(kSpanLanes, kSpanWavesPerSimd) void span_kernel(const SpanArgs a) {
  __shared__ __attribute__((aligned(16))) SpanLDS L;
  {  // tables into LDS: each slicing entry kSpanCopies times (4 per ds_write_b128), the row shift once
    uint4* dst = reinterpret_cast<uint4*>(&L.slice);
    for (uint32_t i = threadIdx.x; i < sizeof(L.slice) / 16; i += kSpanLanes) {
      const uint32_t word = 4 * i;  // region word >> 14, entry (word >> 6) & 255, table pair bit 5
      const uint32_t v = a.tabs->slice8[2 * (word >> 14) + ((word >> 5) & 1u)][(word >> 6) & 255u];
      dst[i] = make_uint4(v, v, v, v);
    }
    const uint4* s2 = reinterpret_cast<const uint4*>(a.span->row_shift);
    uint4* d2 = reinterpret_cast<uint4*>(L.row_shift);
    for (uint32_t i = threadIdx.x; i < sizeof(L.row_shift) / 16; i += kSpanLanes) d2[i] = s2[i];
  }
  const uint32_t w = blockIdx.x, j = threadIdx.x;
  const uint64_t q = a.nline / a.groups, r = a.nline % a.groups;
  const uint64_t count = q + (w < r ? 1 : 0);
  const uint64_t start = w < r ? w * (q + 1) : r * (q + 1) + (w - r) * q;
  const uint64_t rows = count / kSpanLanes;               // rows every lane takes part in
  const uint32_t extra = (uint32_t)(count % kSpanLanes);  // lanes j < extra take one more line
  const uint8_t* p = a.bulk + (start + j) * kSpanLine;
  constexpr uint64_t kRow = (uint64_t)kSpanLine * kSpanLanes;
  const uint32_t l0 = 4u * (j % kSpanCopies), l1 = l0 | (1u << 16);  // address bytes of regions 0 / 1
  __syncthreads();

  uint32_t acc = 0;
  if (rows) {
    // kSpanBuf lines in flight per lane: buffer k holds row g*kSpanBuf + k.  The loop body is
    // branch-free so the compiler's vmcnt waits stay exact (a conditional load made it wait for
    // every line): reloads past the last row re-read the last row (clamped address, never
    // committed), and the rows % kSpanBuf left over are already in buffers 0.. after the loop.
    // Scheduling barriers keep "chain of buffer k, reload buffer k" in order: left to itself the
    // compiler interleaves the chains and waits for all lines before issuing any reload.
    uint32_t buf[kSpanBuf][kLineWords];
    const uint64_t groups_of_rows = rows / kSpanBuf, last = rows - 1;
#pragma unroll
    for (int k = 0; k < kSpanBuf; ++k) load_line(p + ((uint64_t)k < last ? k : last) * kRow, buf[k]);
    for (uint64_t g = 0; g < groups_of_rows; ++g) {
#pragma unroll
      for (int k = 0; k < kSpanBuf; ++k) {
        const uint32_t rk = line_raw(L, l0, l1, buf[k]);
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t nxt = (g + 1) * kSpanBuf + k;
        load_line(p + (nxt < last ? nxt : last) * kRow, buf[k]);
        __builtin_amdgcn_sched_barrier(0);
        acc = row_advance(L.row_shift, acc) ^ rk;
      }
    }
#pragma unroll
    for (int k = 0; k < kSpanBuf - 1; ++k)
      if ((uint64_t)k < rows % kSpanBuf) acc = row_advance(L.row_shift, acc) ^ line_raw(L, l0, l1, buf[k]);
  }
  if (j < extra) {  // the partial last row
    uint32_t E[kLineWords];
    load_line(p + rows * kRow, E);
    acc = row_advance(L.row_shift, acc) ^ line_raw(L, l0, l1, E);
  }
  // Lane j's last line is followed, within the range, by (extra - 1 - j) mod L lines.
  const uint32_t after = (extra + kSpanLanes - 1 - j) % kSpanLanes;
  uint32_t c = (rows || j < extra) ? gf2_mulmod(a.span->lane_op[after], acc) : 0u;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) c ^= __shfl_xor(c, off, 64);
  if ((j & 63) == 0) L.wave_sum[j / 64] = c;
  __syncthreads();
  if (j == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int v = 0; v < kSpanLanes / 64; ++v) t ^= L.wave_sum[v];
    atomicXor(a.crc, gf2_mulmod(a.op[w], t));
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
  // op[w] = x^(8 * (bytes of the ranges after w + rest)); ranges hold q+1 lines (w < r) or q.
  const uint64_t q = nline / groups, r = nline % groups;
  const uint32_t step_q = xpow8n(kSpanLine * q), step_q1 = xpow8n(kSpanLine * (q + 1));
  uint32_t op = xpow8n(rest);
  for (uint64_t w = groups; w-- > 0;) {
    a.op[w] = op;
    op = gf2_mulmod(w < r ? step_q1 : step_q, op);  // w - 1 is followed by w's range as well
  }
  hipLaunchKernelGGL(span_kernel, dim3((uint32_t)groups), dim3(kSpanLanes), 0, s, a);
  return hipGetLastError();
}

}  // namespace efes
