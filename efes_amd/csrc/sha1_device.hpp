// sha1_device.hpp -- SHA-1 compression building blocks for gfx950 (CDNA4).
//
// Restates the compression function `block` of /root/reference/sha1.go:129-203
// (FIPS 180-4 SHA-1) in the shape that is cheapest to ISSUE on one CDNA4 wavefront:
// a lone wave issues about one VALU instruction per ~4.5 cycles and a dependent
// VALU op has ~8.5 cycles latency (measured, DESIGN_NOTES.md "Measured constants"), so the
// per-message rate is set by the instruction count of the chain.  Each round is
// exactly five VALU ops:
//     z  = e + WK[i]                      v_add_u32   (W[i] + K pre-added off-chain)
//     e' = rotl5(a) + F(b,c,d) + z        v_alignbit + v_bitop3 + v_add3_u32
//     b' = rotl30(b)                      v_alignbit
// with F = Ch/Parity/Maj as one `v_bitop3_b32` (LUT 0xCA / 0x96 / 0xE8), and the
// a..e renaming done at compile time (no moves).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace efes {

// sha1.go:122-127
constexpr uint32_t kK0 = 0x5A827999u, kK1 = 0x6ED9EBA1u, kK2 = 0x8F1BBCDCu, kK3 = 0xCA62C1D6u;
// sha1.go:21-25
constexpr uint32_t kIV0 = 0x67452301u, kIV1 = 0xEFCDAB89u, kIV2 = 0x98BADCFEu, kIV3 = 0x10325476u,
                   kIV4 = 0xC3D2E1F0u;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_rotateleft32(x, n); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// a + b + c as ONE v_add3_u32.  hipcc (ROCm 7.2) sometimes splits the 3-input add into two
// v_add_u32 inside large kernels (80 extra instructions per block on the chain), so the
// instruction is pinned here.  Not volatile: it stays freely schedulable.
__device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

template <int R>
__device__ __forceinline__ constexpr int round_lut() {
  // Ch for rounds 0-19 (sha1.go:147-163), Parity 20-39 and 60-79 (:164-172, :183-191),
  // Maj 40-59 (:173-182).  v_bitop3 truth-table index = 4*S0 + 2*S1 + S2.
  return R < 20 ? 0xCA : (R < 40 ? 0x96 : (R < 60 ? 0xE8 : 0x96));
}
template <int R>
__device__ __forceinline__ constexpr uint32_t round_k() {
  return R < 20 ? kK0 : (R < 40 ? kK1 : (R < 60 ? kK2 : kK3));
}

// One round on state s[5] with compile-time renaming: round R sees
// (a,b,c,d,e) = s[(5-R)%5], s[(6-R)%5], ... (sha1.go:152 `a, b, c, d, e = t, a, b30, c, d`).
template <int R>
__device__ __forceinline__ void round_wk(uint32_t (&s)[5], uint32_t wk) {
  constexpr int r = R % 5;
  constexpr int A = (5 - r) % 5, B = (6 - r) % 5, C = (7 - r) % 5, D = (8 - r) % 5, E = (9 - r) % 5;
  const uint32_t z = s[E] + wk;
  s[E] = add3(rotl(s[A], 5), __builtin_amdgcn_bitop3_b32(s[B], s[C], s[D], round_lut<R>()), z);
  s[B] = rotl(s[B], 30);
}

// ---- chain from pre-expanded W[i]+K[i] (80 words, 16-B aligned, wave-uniform address)
template <int Q>
struct ChainQuad {
  __device__ __forceinline__ static void run(uint32_t (&s)[5], const uint4* __restrict__ wk4) {
    const uint4 v = wk4[Q];
    round_wk<4 * Q + 0>(s, v.x);
    round_wk<4 * Q + 1>(s, v.y);
    round_wk<4 * Q + 2>(s, v.z);
    round_wk<4 * Q + 3>(s, v.w);
    ChainQuad<Q + 1>::run(s, wk4);
  }
};
template <>
struct ChainQuad<20> {
  __device__ __forceinline__ static void run(uint32_t (&)[5], const uint4* __restrict__) {}
};

// ---- chain from W[i]+K[i] held in this lane's own registers (80 VGPRs): rounds R..End-1.
template <int R, int End = 80>
struct ChainRegs {
  __device__ __forceinline__ static void run(uint32_t (&s)[5], const uint32_t (&wk)[80]) {
    round_wk<R>(s, wk[R]);
    ChainRegs<R + 1, End>::run(s, wk);
  }
};
template <int End>
struct ChainRegs<End, End> {
  __device__ __forceinline__ static void run(uint32_t (&)[5], const uint32_t (&)[80]) {}
};

// hs = hv + compress(hv, WK) (sha1.go:141-197) from W+K registers.  Round 79 writes a80 into
// s[0], and a80 + h0 is the new h0, so h0 is folded into that round's e + W + K (one v_add3 in
// place of a v_add there and the h0 add after it): 404 VALU per block instead of 405.
__device__ __forceinline__ void chain_block(const uint32_t (&hv)[5], const uint32_t (&wk)[80], uint32_t (&hs)[5]) {
  uint32_t s[5] = {hv[0], hv[1], hv[2], hv[3], hv[4]};
  ChainRegs<0, 79>::run(s, wk);
  // round 79 (R % 5 == 4): a, b, c, d, e = s[1], s[2], s[3], s[4], s[0]
  const uint32_t z = add3(s[0], wk[79], hv[0]);
  hs[0] = add3(rotl(s[1], 5), __builtin_amdgcn_bitop3_b32(s[2], s[3], s[4], round_lut<79>()), z);
  hs[1] = hv[1] + s[1];
  hs[2] = hv[2] + rotl(s[2], 30);
  hs[3] = hv[3] + s[3];
  hs[4] = hv[4] + s[4];
}

// h += compress(WK) -- sha1.go:141-197 with the schedule already expanded.
__device__ __forceinline__ void compress_wk(uint32_t (&h)[5], const uint4* __restrict__ wk4) {
  uint32_t s[5] = {h[0], h[1], h[2], h[3], h[4]};
  ChainQuad<0>::run(s, wk4);
  h[0] += s[0]; h[1] += s[1]; h[2] += s[2]; h[3] += s[3]; h[4] += s[4];
}

// ---- schedule expansion: W[0..15] (big-endian words) -> WK[0..79] = W[i] + K[i]
// sha1.go:154-156: W[i] = rotl1(W[i-3] ^ W[i-8] ^ W[i-14] ^ W[i-16]).
__device__ __forceinline__ void expand_wk(const uint32_t (&w)[16], uint32_t (&wk)[80]) {
  uint32_t x[80];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = w[i];
#pragma unroll
  for (int i = 16; i < 80; ++i)
    x[i] = rotl(__builtin_amdgcn_bitop3_b32(x[i - 3], x[i - 8], x[i - 14], 0x96) ^ x[i - 16], 1);
#pragma unroll
  for (int i = 0; i < 20; ++i) wk[i] = x[i] + kK0;
#pragma unroll
  for (int i = 20; i < 40; ++i) wk[i] = x[i] + kK1;
#pragma unroll
  for (int i = 40; i < 60; ++i) wk[i] = x[i] + kK2;
#pragma unroll
  for (int i = 60; i < 80; ++i) wk[i] = x[i] + kK3;
}

// ---- split expansion: the first N raw schedule words W[0..N-1] (N >= 16, a multiple of 4),
// then the rest of the schedule and + K from them.
template <int N>
__device__ __forceinline__ void expand_raw(const uint32_t (&w)[16], uint32_t (&x)[N]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = w[i];
#pragma unroll
  for (int i = 16; i < N; ++i)
    x[i] = rotl(__builtin_amdgcn_bitop3_b32(x[i - 3], x[i - 8], x[i - 14], 0x96) ^ x[i - 16], 1);
}
template <int N>
__device__ __forceinline__ void expand_wk_from(const uint32_t (&w)[N], uint32_t (&wk)[80]) {
  uint32_t x[80];
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = w[i];
#pragma unroll
  for (int i = N; i < 80; ++i)
    x[i] = rotl(__builtin_amdgcn_bitop3_b32(x[i - 3], x[i - 8], x[i - 14], 0x96) ^ x[i - 16], 1);
#pragma unroll
  for (int i = 0; i < 20; ++i) wk[i] = x[i] + kK0;
#pragma unroll
  for (int i = 20; i < 40; ++i) wk[i] = x[i] + kK1;
#pragma unroll
  for (int i = 40; i < 60; ++i) wk[i] = x[i] + kK2;
#pragma unroll
  for (int i = 60; i < 80; ++i) wk[i] = x[i] + kK3;
}

// ---- compression with the schedule computed inline (16-word ring in registers).
// Used for the few special blocks of a job (prefix/tail/padding) and by the
// lane-per-job WIDE kernel.
template <int R>
__device__ __forceinline__ void round_inline(uint32_t (&s)[5], uint32_t (&w)[16]) {
  uint32_t wi;
  if constexpr (R < 16) {
    wi = w[R];
  } else {
    wi = rotl(__builtin_amdgcn_bitop3_b32(w[(R - 3) & 15], w[(R - 8) & 15], w[(R - 14) & 15], 0x96) ^ w[R & 15], 1);
    w[R & 15] = wi;
  }
  constexpr int r = R % 5;
  constexpr int A = (5 - r) % 5, B = (6 - r) % 5, C = (7 - r) % 5, D = (8 - r) % 5, E = (9 - r) % 5;
  const uint32_t z = s[E] + wi + round_k<R>();
  s[E] = add3(rotl(s[A], 5), __builtin_amdgcn_bitop3_b32(s[B], s[C], s[D], round_lut<R>()), z);
  s[B] = rotl(s[B], 30);
}
template <int R>
struct InlineRounds {
  __device__ __forceinline__ static void run(uint32_t (&s)[5], uint32_t (&w)[16]) {
    round_inline<R>(s, w);
    InlineRounds<R + 1>::run(s, w);
  }
};
template <>
struct InlineRounds<80> {
  __device__ __forceinline__ static void run(uint32_t (&)[5], uint32_t (&)[16]) {}
};

// h += compress(w) where w holds the 16 big-endian message words (clobbered).
__device__ __forceinline__ void compress_inline(uint32_t (&h)[5], uint32_t (&w)[16]) {
  uint32_t s[5] = {h[0], h[1], h[2], h[3], h[4]};
  InlineRounds<0>::run(s, w);
  h[0] += s[0]; h[1] += s[1]; h[2] += s[2]; h[3] += s[3]; h[4] += s[4];
}

}  // namespace efes
