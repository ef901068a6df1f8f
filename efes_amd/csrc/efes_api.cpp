// efes_api.cpp -- C ABI of libefeshash (include/efes_hash.h): contexts, the batched
// device-resident submit (layer 1, kernels in efes_kernels.hip), device-memory helpers,
// the CRC tables, CRC combine, and the text codecs of sha1_efes.go / crc32_efes.go.
// Host-resident ingest is efes_ingest.cpp, the upload dispatcher efes_queue.cpp, and the
// Go-surface streaming digests efes_stream.cpp.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <new>
#include <vector>

#include "efes_internal.hpp"

using efes::Tables;


namespace {

int hip_err(hipError_t e) { return e == hipSuccess ? EFES_OK : EFES_ERR_HIP; }

using efes::DeviceGuard;

hipStream_t pick(efes_ctx* ctx, void* s) { return s ? static_cast<hipStream_t>(s) : ctx->stream; }

// ---- GF(2) helpers for the CRC shift tables ------------------------------------------
// A 32x32 GF(2) matrix is stored as its 32 columns (images of the unit vectors).
struct Gf2 {
  uint32_t col[32];
  uint32_t apply(uint32_t v) const {
    uint32_t r = 0;
    for (int i = 0; i < 32; ++i)
      if ((v >> i) & 1) r ^= col[i];
    return r;
  }
};
Gf2 compose(const Gf2& a, const Gf2& b) {  // a after b
  Gf2 r;
  for (int i = 0; i < 32; ++i) r.col[i] = a.apply(b.col[i]);
  return r;
}

// ---- byte codecs (sha1_efes.go, crc32_efes.go) -----------------------------------------
const char kHex[] = "0123456789abcdef";
int hexval(char c) {  // Go encoding/hex accepts both cases
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
void hex_encode(char* dst, const uint8_t* src, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    dst[2 * i] = kHex[src[i] >> 4];
    dst[2 * i + 1] = kHex[src[i] & 15];
  }
}
bool hex_decode(uint8_t* dst, const char* src, size_t nbytes) {
  for (size_t i = 0; i < nbytes; ++i) {
    const int hi = hexval(src[2 * i]), lo = hexval(src[2 * i + 1]);
    if (hi < 0 || lo < 0) return false;
    dst[i] = (uint8_t)(hi << 4 | lo);
  }
  return true;
}
void put_be32(uint8_t* b, uint32_t v) { b[0] = v >> 24; b[1] = v >> 16; b[2] = v >> 8; b[3] = (uint8_t)v; }
void put_be64(uint8_t* b, uint64_t v) { for (int i = 0; i < 8; ++i) b[i] = (uint8_t)(v >> (56 - 8 * i)); }
uint32_t get_be32(const uint8_t* b) { return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]; }
uint64_t get_be64(const uint8_t* b) { uint64_t v = 0; for (int i = 0; i < 8; ++i) v = v << 8 | b[i]; return v; }

}  // namespace

namespace efes {
// Go's sha1digest.Write bookkeeping of x/nx/len (sha1.go:58-79) without the compressions.
int replay_write(efes_sha1_state* s, const uint8_t* p, size_t n) {
  if (s->nx > 64) return EFES_ERR_STATE;  // copy(d.x[d.nx:], p) panics
  s->len += (uint64_t)n;
  if (s->nx > 0) {
    const size_t room = (size_t)(64 - s->nx);
    const size_t c = n < room ? n : room;
    memcpy(s->x + s->nx, p, c);
    s->nx += (int64_t)c;
    if (s->nx == 64) s->nx = 0;
    p += c;
    n -= c;
  }
  const size_t m = n & ~(size_t)63;
  p += m;
  n -= m;
  if (n > 0) {
    memcpy(s->x, p, n);
    s->nx = (int64_t)n;
  }
  return EFES_OK;
}
}  // namespace efes
using efes::replay_write;

// ======================================================================= tables
void efes::build_tables(Tables* t) {
  // crc32.go:106-118 simplePopulateTable(IEEE) and crc32.go:138-149 slicingMakeTable.
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t crc = i;
    for (int j = 0; j < 8; ++j) crc = (crc & 1) ? (crc >> 1) ^ 0xedb88320u : crc >> 1;
    t->slice8[0][i] = crc;
  }
  for (int i = 0; i < 256; ++i) {
    uint32_t crc = t->slice8[0][i];
    for (int j = 1; j < 8; ++j) {
      crc = t->slice8[0][crc & 0xff] ^ (crc >> 8);
      t->slice8[j][i] = crc;
    }
  }
  // One zero byte advances the raw register by s -> T0[s & 0xff] ^ (s >> 8) (crc32.go:125).
  Gf2 z;
  for (int i = 0; i < 32; ++i) {
    const uint32_t s = 1u << i;
    z.col[i] = t->slice8[0][s & 0xff] ^ (s >> 8);
  }
  Gf2 m = z;  // z^64: square six times
  for (int i = 0; i < 6; ++i) m = compose(m, m);
  for (int k = 0; k < efes::kShiftLevels; ++k) {  // level k advances 64<<k bytes
    for (int b = 0; b < 4; ++b)
      for (uint32_t v = 0; v < 256; ++v) t->shift[k][b][v] = m.apply(v << (8 * b));
    m = compose(m, m);
  }
}

void efes::build_pos_tables(const Tables* t, PosTables* out) {
  for (int p = 0; p < 64; ++p)
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t crc = 0;  // raw register, crc32.go:125 per byte
      for (int i = 0; i < 64; ++i) crc = t->slice8[0][(crc ^ (i == p ? b : 0u)) & 0xff] ^ (crc >> 8);
      out->pos[p][b] = crc;
    }
}

// A stream on a hardware queue of its own (efes_internal.hpp).
hipError_t efes::own_queue_stream(const efes_ctx* ctx, hipStream_t* out) {
  uint32_t all_cus[8];
  for (int w = 0; w < 8; ++w) {
    const int left = ctx->cus - 32 * w;
    all_cus[w] = left >= 32 ? 0xffffffffu : left > 0 ? (1u << left) - 1u : 0u;
  }
  return hipExtStreamCreateWithCUMask(out, (uint32_t)std::min(8, (ctx->cus + 31) / 32), all_cus);
}

// efes_amd/build.py passes -DEFES_BUILD_ID="<source_id()>"; other builds (A/B variants, sanitizer
// builds) report that they were not built from a recorded source set.
#ifndef EFES_BUILD_ID
#define EFES_BUILD_ID "unversioned"
#endif

// ======================================================================= C ABI
extern "C" {

const char* efes_strerror(int code) {
  switch (code) {
    case EFES_OK: return "ok";
    case EFES_ERR_INVALID_DIGEST: return "invalid digest";
    case EFES_ERR_STATE: return "invalid digest state (the reference would panic)";
    case EFES_ERR_HIP: return "HIP runtime error";
    case EFES_ERR_ARG: return "invalid argument";
    case EFES_ERR_NO_DEVICE: return "no usable gfx950 device";
    case EFES_ERR_NOMEM: return "out of host memory";
    case EFES_ERR_DEVICE_FAULT: return "device fault latched";
    default: return "unknown error";
  }
}

int efes_abi_version(void) { return EFES_ABI_VERSION; }

const char* efes_build_id(void) { return EFES_BUILD_ID; }

void efes_sha1_state_init(efes_sha1_state* s) {  // sha1.go:36-44 (x untouched, as Reset)
  s->h[0] = 0x67452301u; s->h[1] = 0xEFCDAB89u; s->h[2] = 0x98BADCFEu; s->h[3] = 0x10325476u; s->h[4] = 0xC3D2E1F0u;
  s->nx = 0;
  s->len = 0;
}

int efes_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    efes::clear_last_error();  // no runtime / no devices: a count of 0, not a later launch's error
    return 0;
  }
  return n > 0 ? n : 0;
}

int efes_ctx_create(int device, efes_ctx** out) {
  if (!out) return EFES_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return EFES_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return EFES_ERR_ARG;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return EFES_ERR_HIP;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return EFES_ERR_NO_DEVICE;  // code objects are gfx950-only
  efes_ctx* ctx = new (std::nothrow) efes_ctx;
  if (!ctx) return EFES_ERR_NOMEM;
  ctx->device = device;
  DeviceGuard g(device);
  // Tables followed by PosTables in one allocation (efes_internal.hpp)
  const size_t tab_bytes = sizeof(Tables) + sizeof(efes::PosTables);
  Tables* host = static_cast<Tables*>(malloc(tab_bytes));
  if (!host) { delete ctx; return EFES_ERR_NOMEM; }
  efes::build_tables(host);
  efes::build_pos_tables(host, reinterpret_cast<efes::PosTables*>(host + 1));
  ctx->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming);
  // The part streams of a planned batch are created by the first multi-part efes_hash_submit_plan
  // (efes_plan.cpp): each holds a hardware queue of its own, which a context that never plans
  // should not take from the process.
  for (int i = 0; i < EFES_PLAN_MAX_PARTS && e == hipSuccess; ++i)
    e = hipEventCreateWithFlags(&ctx->ev_join[i], hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&ctx->d_tabs), tab_bytes);
  if (e == hipSuccess) e = hipMemcpy(ctx->d_tabs, host, tab_bytes, hipMemcpyHostToDevice);
  free(host);
  if (e == hipSuccess) {
    efes::SpanTables* span = static_cast<efes::SpanTables*>(malloc(sizeof(efes::SpanTables)));
    if (!span) e = hipErrorOutOfMemory;
    if (span) efes::build_span_tables(span);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&ctx->d_span), sizeof(efes::SpanTables));
    if (e == hipSuccess) e = hipMemcpy(ctx->d_span, span, sizeof(efes::SpanTables), hipMemcpyHostToDevice);
    free(span);
  }
  if (e != hipSuccess) {
    efes_ctx_destroy(ctx);
    return EFES_ERR_HIP;
  }
  *out = ctx;
  return EFES_OK;
}

void efes_ctx_destroy(efes_ctx* ctx) {
  if (!ctx) return;
  if (ctx->digests) efes_queue_destroy(ctx->digests);  // free the context's digests first
  {
    DeviceGuard g(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (hipStream_t sd : ctx->side)
      if (sd) (void)hipStreamSynchronize(sd);
    if (ctx->copy) (void)hipStreamSynchronize(ctx->copy);
    if (ctx->d_tabs) (void)hipFree(ctx->d_tabs);
    if (ctx->d_span) (void)hipFree(ctx->d_span);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    for (hipEvent_t ev : ctx->ev_join)
      if (ev) (void)hipEventDestroy(ev);
    for (hipStream_t sd : ctx->side)
      if (sd) (void)hipStreamDestroy(sd);
    if (ctx->copy) (void)hipStreamDestroy(ctx->copy);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  }
  delete ctx;
}

int efes_ctx_device(const efes_ctx* ctx) { return ctx ? ctx->device : -1; }
void* efes_ctx_stream(efes_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }

int efes_auto_mode(const efes_ctx* ctx, uint32_t njobs) {
  // The lowest per-job latency that fits in one pass (DESIGN_NOTES.md §4): DEEP up to one job per
  // SIMD (46.5 ms per 4 MiB job); FED4 up to 32 jobs per CU (48.5 ms: DEEP's chain, fed from
  // two producer SIMDs -- below GROUP32/16/8's 49/52/57 ms at 2/4/8 jobs per SIMD); FED4E up to
  // 48 per CU (55.5 ms); grouped DEEP G = 4 (67 ms, 64 jobs per CU) up to 16 jobs per SIMD, i.e.
  // one GROUP4 wave per SIMD; WIDE beyond: a second GROUP4 wave on a SIMD doubles the launch
  // (134 ms), while WIDE lanes (~40 MB/s each) take 108 ms for any count up to a wave per SIMD
  // (measured 18 432-24 576 x 4 MiB: WIDE 668-883 GiB/s, GROUP4 534-715, tools/gpu_auto_band.sh).
  const uint64_t simds = 4ull * (ctx ? (uint64_t)ctx->cus : 256ull), n = njobs;
  if (n <= simds) return EFES_MODE_DEEP;
  if (n <= 8 * simds) return EFES_MODE_FED4;
  if (n <= 12 * simds) return EFES_MODE_FED4E;  // 55.5 ms, 48 jobs per CU
  if (n <= 16 * simds) return EFES_MODE_GROUP4;
  return EFES_MODE_WIDE;
}

int efes_hash_submit_mode(efes_ctx* ctx, const efes_job* jobs, uint32_t njobs, void* stream, int mode) {
  if (!ctx || (!jobs && njobs) || njobs > EFES_MAX_JOBS) return EFES_ERR_ARG;
  if (njobs == 0) return EFES_OK;
  if (mode == EFES_MODE_AUTO) mode = efes_auto_mode(ctx, njobs);
  DeviceGuard g(ctx->device);
  hipStream_t s = pick(ctx, stream);
  if (mode == EFES_MODE_DEEP) return hip_err(efes::launch_deep(jobs, njobs, ctx->d_tabs, s));
  if (mode == EFES_MODE_WIDE) return hip_err(efes::launch_wide(jobs, njobs, ctx->d_tabs, s, false, ctx->cus));
  if (mode == EFES_MODE_FED4 || mode == EFES_MODE_FED4E)
    return hip_err(efes::launch_fed(jobs, njobs, ctx->d_tabs, s, mode == EFES_MODE_FED4E));
  const int lanes = efes::group_of_mode(mode);
  if (lanes) return hip_err(efes::launch_group(jobs, njobs, lanes, ctx->d_tabs, s));
  return EFES_ERR_ARG;
}

int efes_hash_submit(efes_ctx* ctx, const efes_job* jobs, uint32_t njobs, void* stream) {
  return efes_hash_submit_mode(ctx, jobs, njobs, stream, EFES_MODE_AUTO);
}

int efes_sync(efes_ctx* ctx, void* stream) {
  if (!ctx) return EFES_ERR_ARG;
  DeviceGuard g(ctx->device);
  return hipStreamSynchronize(pick(ctx, stream)) == hipSuccess ? EFES_OK : EFES_ERR_DEVICE_FAULT;
}

int efes_device_alloc(efes_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out) return EFES_ERR_ARG;
  DeviceGuard g(ctx->device);
  return hip_err(hipMalloc(out, bytes ? bytes : 1));
}

int efes_device_free(efes_ctx* ctx, void* p) {
  if (!ctx) return EFES_ERR_ARG;
  DeviceGuard g(ctx->device);
  return hip_err(hipFree(p));
}

int efes_copy_to_device(efes_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream) {
  if (!ctx || (!dst && bytes) || (!src && bytes)) return EFES_ERR_ARG;
  DeviceGuard g(ctx->device);
  hipStream_t s = pick(ctx, stream);
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return hip_err(e);
}

int efes_copy_to_host(efes_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream) {
  if (!ctx || (!dst && bytes) || (!src && bytes)) return EFES_ERR_ARG;
  DeviceGuard g(ctx->device);
  hipStream_t s = pick(ctx, stream);
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return hip_err(e);
}

int efes_fill_synthetic(efes_ctx* ctx, void* dst, size_t bytes, uint64_t seed, void* stream) {
  if (!ctx || (!dst && bytes) || (reinterpret_cast<uintptr_t>(dst) & 7)) return EFES_ERR_ARG;
  if (!bytes) return EFES_OK;
  DeviceGuard g(ctx->device);
  return hip_err(efes::launch_fill(dst, bytes, seed, pick(ctx, stream)));
}

int efes_crc32_span(efes_ctx* ctx, const void* data, uint64_t length, efes_crc32_state* crc, void* stream) {
  if (!ctx || !crc || (!data && length) || (reinterpret_cast<uintptr_t>(crc) & 3)) return EFES_ERR_ARG;
  DeviceGuard g(ctx->device);
  return hip_err(efes::launch_crc_span(data, length, &crc->crc, ctx->d_tabs, ctx->d_span, ctx->cus, pick(ctx, stream)));
}

int efes_crc32_tables(uint32_t* out, size_t nwords) {
  const size_t need = sizeof(Tables) / 4, with_pos = need + sizeof(efes::PosTables) / 4;
  if (!out || nwords < need) return EFES_ERR_ARG;
  Tables* t = static_cast<Tables*>(malloc(sizeof(Tables) + sizeof(efes::PosTables)));
  if (!t) return EFES_ERR_NOMEM;
  efes::build_tables(t);
  const bool pos = nwords >= with_pos;  // room for the position tables too (WIDE / grouped kernels)
  if (pos) efes::build_pos_tables(t, reinterpret_cast<efes::PosTables*>(t + 1));
  memcpy(out, t, pos ? sizeof(Tables) + sizeof(efes::PosTables) : sizeof(Tables));
  free(t);
  return (int)(pos ? with_pos : need);
}

uint32_t efes_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  // Raw register update over B is affine: R(x, B) = Z^|B| x ^ R(0, B), Z = one zero byte
  // (crc32.go:125).  With crc(X) = ~R(~0, X) (crc32.go:123,127):
  //   crc(A||B) ^ crc(B) = Z^|B|(~crc(A)) ^ Z^|B|(~0) = Z^|B|(crc(A)).
  if (len2 == 0) return crc1;
  Gf2 z;
  for (int i = 0; i < 32; ++i) {
    const uint32_t s = 1u << i;
    uint32_t c = s;
    c = (c & 1) ? (c >> 1) ^ 0xedb88320u : c >> 1;  // one zero bit, eight times = one zero byte
    for (int k = 1; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0xedb88320u : c >> 1;
    z.col[i] = c;
  }
  uint32_t v = crc1;
  Gf2 p = z;  // Z^(2^k)
  for (uint64_t n = len2; n; n >>= 1) {
    if (n & 1) v = p.apply(v);
    p = compose(p, p);
  }
  return v ^ crc2;
}

// ---- text codecs --------------------------------------------------------------------------
void efes_sha1_state_marshal_text(const efes_sha1_state* s, char out[200]) {  // sha1_efes.go:25-38
  uint8_t b[100];
  for (int i = 0; i < 5; ++i) put_be32(b + 4 * i, s->h[i]);
  memcpy(b + 20, s->x, 64);
  put_be64(b + 84, (uint64_t)s->nx);
  put_be64(b + 92, s->len);
  hex_encode(out, b, 100);
}

int efes_sha1_state_unmarshal_text(efes_sha1_state* s, const char* text, size_t n) {  // sha1_efes.go:40-64
  if (!text || n != 200) return EFES_ERR_INVALID_DIGEST;
  uint8_t b[100];
  if (!hex_decode(b, text, 100)) return EFES_ERR_INVALID_DIGEST;
  for (int i = 0; i < 5; ++i) s->h[i] = get_be32(b + 4 * i);
  memcpy(s->x, b + 20, 64);
  s->nx = (int64_t)get_be64(b + 84);  // `nx > MaxInt` can never hold for a 64-bit int
  s->len = get_be64(b + 92);
  return EFES_OK;
}

void efes_crc32_state_marshal_text(const efes_crc32_state* s, char out[8]) {  // crc32_efes.go:18-24
  uint8_t b[4];
  put_be32(b, s->crc);
  hex_encode(out, b, 4);
}

int efes_crc32_state_unmarshal_text(efes_crc32_state* s, const char* text, size_t n) {  // crc32_efes.go:26-40
  if (!text || n != 8) return EFES_ERR_INVALID_DIGEST;
  uint8_t b[4];
  if (!hex_decode(b, text, 4)) return EFES_ERR_INVALID_DIGEST;
  s->crc = get_be32(b);
  return EFES_OK;
}

}  // extern "C"
