// efes_api.cpp -- C ABI of libefeshash (include/efes_hash.h).
//
// Layer 1 (efes_hash_submit) enqueues the gfx950 kernels of efes_kernels.hip.
// Layer 2 (efes_sha1_* / efes_crc32_*) mirrors the Go digests the reference streams
// uploads through: sha1digest (sha1.go:29-120, sha1_efes.go:25-64) and crc32digest
// (crc32.go:48-93, crc32_efes.go:18-40).  A streaming object stages the bytes of its
// Write calls and hashes them on the GPU in one job at the next Sum/MarshalText (or
// when the staging exceeds kFlushBytes).  Host code never compresses a block: it only
// replays Go's byte bookkeeping of the tail buffer (x, nx, len), so the device state
// plus that bookkeeping reproduces Go's state exactly, stale x bytes included.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <new>
#include <vector>

#include "efes_internal.hpp"

using efes::Tables;


namespace {

constexpr size_t kFlushBytes = 64u << 20;

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

// Device scratch of one streaming object: [job 56 | pad | sha1 state 104 | crc 4 | sum 24 | status 4].
struct DevScratch {
  uint8_t* base = nullptr;
  uint8_t* data = nullptr;
  size_t cap = 0;
  efes_job* job() { return reinterpret_cast<efes_job*>(base); }
  efes_sha1_state* sha1() { return reinterpret_cast<efes_sha1_state*>(base + 64); }
  efes_crc32_state* crc() { return reinterpret_cast<efes_crc32_state*>(base + 64 + 104); }
  uint8_t* sum() { return base + 64 + 104 + 8; }
  int32_t* status() { return reinterpret_cast<int32_t*>(base + 64 + 104 + 8 + 24); }
  static constexpr size_t kBytes = 256;
};

struct Staged {
  efes_ctx* ctx = nullptr;
  std::vector<uint8_t> pending;
  DevScratch dev;
  int latched = EFES_OK;

  int ensure(size_t need) {
    DeviceGuard g(ctx->device);
    if (!dev.base && hipMalloc(reinterpret_cast<void**>(&dev.base), DevScratch::kBytes) != hipSuccess) return EFES_ERR_HIP;
    if (need > dev.cap) {
      if (dev.data) (void)hipFree(dev.data);
      dev.data = nullptr;
      dev.cap = 0;
      size_t cap = 1 << 16;
      while (cap < need) cap <<= 1;
      if (hipMalloc(reinterpret_cast<void**>(&dev.data), cap) != hipSuccess) return EFES_ERR_HIP;
      dev.cap = cap;
    }
    return EFES_OK;
  }
  void release() {
    DeviceGuard g(ctx->device);
    if (dev.data) (void)hipFree(dev.data);
    if (dev.base) (void)hipFree(dev.base);
    dev = DevScratch{};
  }
  // Runs one job over `pending` with the given in-states; copies states (and sum) back.
  int run(efes_sha1_state* sha1, efes_crc32_state* crc, bool finalize, uint8_t sum_out[24]) {
    const size_t n = pending.size();
    int rc = ensure(n ? n : 1);
    if (rc) return rc;
    DeviceGuard g(ctx->device);
    hipStream_t s = ctx->stream;
    efes_job job{};
    job.data = dev.data;
    job.length = n;
    job.sha1 = sha1 ? dev.sha1() : nullptr;
    job.crc32 = crc ? dev.crc() : nullptr;
    job.sum = finalize ? dev.sum() : nullptr;
    job.status = dev.status();
    job.flags = finalize ? EFES_JOB_FINALIZE : 0u;
    uint8_t host[DevScratch::kBytes] = {};
    memcpy(host, &job, sizeof job);
    if (sha1) memcpy(host + 64, sha1, sizeof *sha1);
    if (crc) memcpy(host + 64 + 104, crc, sizeof *crc);
    hipError_t e = hipMemcpyAsync(dev.base, host, sizeof host, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && n) e = hipMemcpyAsync(dev.data, pending.data(), n, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = efes::launch_deep(dev.job(), 1, ctx->d_tabs, s);
    if (e == hipSuccess) e = hipMemcpyAsync(host, dev.base, sizeof host, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return latched = EFES_ERR_HIP;
    int32_t status;
    memcpy(&status, host + 64 + 104 + 8 + 24, 4);
    if (status != EFES_OK && status != EFES_ERR_STATE) return latched = EFES_ERR_DEVICE_FAULT;
    if (sha1) {
      efes_sha1_state out;
      memcpy(&out, host + 64, sizeof out);
      memcpy(sha1->h, out.h, sizeof out.h);  // x/nx/len come from the host replay
    }
    if (crc) memcpy(crc, host + 64 + 104, sizeof *crc);
    if (sum_out) memcpy(sum_out, host + 64 + 104 + 8, 24);
    pending.clear();
    return status;
  }
};

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

struct efes_sha1 {
  Staged stg;
  efes_sha1_state base{};    // state as of the last device flush (h authoritative)
  efes_sha1_state shadow{};  // Go's x/nx/len after every Write so far
};

struct efes_crc32 {
  Staged stg;
  efes_crc32_state st{};
};

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

void efes_sha1_state_init(efes_sha1_state* s) {  // sha1.go:36-44 (x untouched, as Reset)
  s->h[0] = 0x67452301u; s->h[1] = 0xEFCDAB89u; s->h[2] = 0x98BADCFEu; s->h[3] = 0x10325476u; s->h[4] = 0xC3D2E1F0u;
  s->nx = 0;
  s->len = 0;
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
  Tables* host = static_cast<Tables*>(malloc(sizeof(Tables)));
  if (!host) { delete ctx; return EFES_ERR_NOMEM; }
  efes::build_tables(host);
  hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&ctx->d_tabs), sizeof(Tables));
  if (e == hipSuccess) e = hipMemcpy(ctx->d_tabs, host, sizeof(Tables), hipMemcpyHostToDevice);
  free(host);
  if (e != hipSuccess) {
    efes_ctx_destroy(ctx);
    return EFES_ERR_HIP;
  }
  *out = ctx;
  return EFES_OK;
}

void efes_ctx_destroy(efes_ctx* ctx) {
  if (!ctx) return;
  {
    DeviceGuard g(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->d_tabs) (void)hipFree(ctx->d_tabs);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  }
  delete ctx;
}

int efes_ctx_device(const efes_ctx* ctx) { return ctx ? ctx->device : -1; }
void* efes_ctx_stream(efes_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }

int efes_hash_submit_mode(efes_ctx* ctx, const efes_job* jobs, uint32_t njobs, void* stream, int mode) {
  if (!ctx || (!jobs && njobs)) return EFES_ERR_ARG;
  if (njobs == 0) return EFES_OK;
  if (mode == EFES_MODE_AUTO) mode = njobs <= efes::kAutoDeepMaxJobs ? EFES_MODE_DEEP : EFES_MODE_WIDE;
  DeviceGuard g(ctx->device);
  hipStream_t s = pick(ctx, stream);
  if (mode == EFES_MODE_DEEP) return hip_err(efes::launch_deep(jobs, njobs, ctx->d_tabs, s));
  if (mode == EFES_MODE_WIDE) return hip_err(efes::launch_wide(jobs, njobs, ctx->d_tabs, s));
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

int efes_crc32_tables(uint32_t* out, size_t nwords) {
  const size_t need = sizeof(Tables) / 4;
  if (!out || nwords < need) return EFES_ERR_ARG;
  Tables* t = static_cast<Tables*>(malloc(sizeof(Tables)));
  if (!t) return EFES_ERR_NOMEM;
  efes::build_tables(t);
  memcpy(out, t, sizeof(Tables));
  free(t);
  return (int)need;
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

// ---- streaming SHA-1 -----------------------------------------------------------------------
static int sha1_alloc(efes_ctx* ctx, efes_sha1** out, bool reset) {
  if (!ctx || !out) return EFES_ERR_ARG;
  efes_sha1* d = new (std::nothrow) efes_sha1;
  if (!d) return EFES_ERR_NOMEM;
  d->stg.ctx = ctx;
  memset(&d->base, 0, sizeof d->base);
  if (reset) efes_sha1_state_init(&d->base);
  d->shadow = d->base;
  *out = d;
  return EFES_OK;
}

int efes_sha1_new(efes_ctx* ctx, efes_sha1** out) { return sha1_alloc(ctx, out, true); }
int efes_sha1_new_zero(efes_ctx* ctx, efes_sha1** out) { return sha1_alloc(ctx, out, false); }

void efes_sha1_free(efes_sha1* d) {
  if (!d) return;
  d->stg.release();
  delete d;
}

void efes_sha1_reset(efes_sha1* d) {
  if (!d) return;
  d->stg.pending.clear();
  efes_sha1_state_init(&d->base);  // Go's Reset leaves x as it is
  memcpy(d->base.x, d->shadow.x, 64);
  d->shadow = d->base;
}

int efes_sha1_size(void) { return 20; }
int efes_sha1_block_size(void) { return 64; }

static int sha1_flush(efes_sha1* d, bool finalize, uint8_t sum[24]) {
  if (d->stg.latched) return d->stg.latched;
  if (d->stg.pending.empty() && !finalize) return EFES_OK;
  efes_sha1_state st = d->base;
  const int rc = d->stg.run(&st, nullptr, finalize, sum);
  if (rc != EFES_OK && rc != EFES_ERR_STATE) return rc;
  memcpy(d->shadow.h, st.h, sizeof st.h);  // x/nx/len: the replay is authoritative
  d->base = d->shadow;
  return rc;
}

int efes_sha1_write(efes_sha1* d, const void* p, size_t n) {
  if (!d || (!p && n)) return EFES_ERR_ARG;
  if (d->stg.latched) return d->stg.latched;
  const int rc = replay_write(&d->shadow, static_cast<const uint8_t*>(p), n);
  if (rc) return rc;
  try {
    d->stg.pending.insert(d->stg.pending.end(), static_cast<const uint8_t*>(p), static_cast<const uint8_t*>(p) + n);
  } catch (...) {
    return EFES_ERR_NOMEM;
  }
  if (d->stg.pending.size() >= kFlushBytes) return sha1_flush(d, false, nullptr);
  return EFES_OK;
}

int efes_sha1_sum(efes_sha1* d, uint8_t out[20]) {
  if (!d || !out) return EFES_ERR_ARG;
  uint8_t sum[24];
  const int rc = sha1_flush(d, true, sum);
  if (rc) return rc;
  memcpy(out, sum, 20);
  return EFES_OK;
}

int efes_sha1_marshal_text(efes_sha1* d, char out[200]) {
  if (!d || !out) return EFES_ERR_ARG;
  const int rc = sha1_flush(d, false, nullptr);
  if (rc) return rc;
  efes_sha1_state_marshal_text(&d->base, out);
  return EFES_OK;
}

int efes_sha1_unmarshal_text(efes_sha1* d, const char* text, size_t n) {
  if (!d) return EFES_ERR_ARG;
  efes_sha1_state s;
  const int rc = efes_sha1_state_unmarshal_text(&s, text, n);
  if (rc) return rc;  // Go leaves the digest untouched on this path
  d->stg.pending.clear();
  d->base = d->shadow = s;
  return EFES_OK;
}

int efes_sha1_get_state(efes_sha1* d, efes_sha1_state* out) {
  if (!d || !out) return EFES_ERR_ARG;
  const int rc = sha1_flush(d, false, nullptr);
  if (rc) return rc;
  *out = d->base;
  return EFES_OK;
}

int efes_sha1_set_state(efes_sha1* d, const efes_sha1_state* in) {
  if (!d || !in) return EFES_ERR_ARG;
  d->stg.pending.clear();
  d->base = d->shadow = *in;
  return EFES_OK;
}

// ---- streaming CRC-32 ----------------------------------------------------------------------
int efes_crc32_new(efes_ctx* ctx, efes_crc32** out) {
  if (!ctx || !out) return EFES_ERR_ARG;
  efes_crc32* d = new (std::nothrow) efes_crc32;
  if (!d) return EFES_ERR_NOMEM;
  d->stg.ctx = ctx;
  d->st.crc = 0;
  *out = d;
  return EFES_OK;
}

void efes_crc32_free(efes_crc32* d) {
  if (!d) return;
  d->stg.release();
  delete d;
}

void efes_crc32_reset(efes_crc32* d) {
  if (!d) return;
  d->stg.pending.clear();
  d->st.crc = 0;
}

int efes_crc32_size(void) { return 4; }
int efes_crc32_block_size(void) { return 1; }

static int crc32_flush(efes_crc32* d) {
  if (d->stg.latched) return d->stg.latched;
  if (d->stg.pending.empty()) return EFES_OK;
  return d->stg.run(nullptr, &d->st, false, nullptr);
}

int efes_crc32_write(efes_crc32* d, const void* p, size_t n) {
  if (!d || (!p && n)) return EFES_ERR_ARG;
  if (d->stg.latched) return d->stg.latched;
  try {
    d->stg.pending.insert(d->stg.pending.end(), static_cast<const uint8_t*>(p), static_cast<const uint8_t*>(p) + n);
  } catch (...) {
    return EFES_ERR_NOMEM;
  }
  if (d->stg.pending.size() >= kFlushBytes) return crc32_flush(d);
  return EFES_OK;
}

int efes_crc32_sum32(efes_crc32* d, uint32_t* out) {
  if (!d || !out) return EFES_ERR_ARG;
  const int rc = crc32_flush(d);
  if (rc) return rc;
  *out = d->st.crc;
  return EFES_OK;
}

int efes_crc32_sum(efes_crc32* d, uint8_t out[4]) {
  uint32_t v;
  const int rc = efes_crc32_sum32(d, &v);
  if (rc) return rc;
  put_be32(out, v);
  return EFES_OK;
}

int efes_crc32_marshal_text(efes_crc32* d, char out[8]) {
  if (!d || !out) return EFES_ERR_ARG;
  const int rc = crc32_flush(d);
  if (rc) return rc;
  efes_crc32_state_marshal_text(&d->st, out);
  return EFES_OK;
}

int efes_crc32_unmarshal_text(efes_crc32* d, const char* text, size_t n) {
  if (!d) return EFES_ERR_ARG;
  efes_crc32_state s;
  const int rc = efes_crc32_state_unmarshal_text(&s, text, n);
  if (rc) return rc;
  d->stg.pending.clear();
  d->st = s;
  return EFES_OK;
}

}  // extern "C"
