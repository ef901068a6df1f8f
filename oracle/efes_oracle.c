/*
 * efes_oracle.c -- CPU restatement of putdotio/efes' hashing path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + "port" CPU baseline); see efes_oracle.h.
 * Every function follows the Go reference line by line; citations are
 * /root/reference/<file>:<line>.  Deliberately scalar and generic (no SHA-NI, no
 * PCLMUL), like the reference's vendored generic Go code.
 */
#include "efes_oracle.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---------------------------------------------------------------- SHA-1 */

/* sha1.go:19-26 */
#define CHUNK 64
#define INIT0 0x67452301u
#define INIT1 0xEFCDAB89u
#define INIT2 0x98BADCFEu
#define INIT3 0x10325476u
#define INIT4 0xC3D2E1F0u
/* sha1.go:122-127 */
#define K0 0x5A827999u
#define K1 0x6ED9EBA1u
#define K2 0x8F1BBCDCu
#define K3 0xCA62C1D6u

static inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* sha1.go:36-44 Reset */
void oracle_sha1_reset(oracle_sha1* d) {
    d->h[0] = INIT0;
    d->h[1] = INIT1;
    d->h[2] = INIT2;
    d->h[3] = INIT3;
    d->h[4] = INIT4;
    d->nx = 0;
    d->len = 0;
}

/* sha1.go:129-203 block: compresses every whole 64-byte chunk of p into d->h. */
void oracle_sha1_block(oracle_sha1* dig, const uint8_t* p, size_t n) {
    uint32_t w[16];
    uint32_t h0 = dig->h[0], h1 = dig->h[1], h2 = dig->h[2], h3 = dig->h[3], h4 = dig->h[4];
    while (n >= CHUNK) { /* sha1.go:133 */
        for (int i = 0; i < 16; i++) { /* sha1.go:136-139 big-endian load */
            int j = i * 4;
            w[i] = (uint32_t)p[j] << 24 | (uint32_t)p[j + 1] << 16 | (uint32_t)p[j + 2] << 8 | (uint32_t)p[j + 3];
        }
        uint32_t a = h0, b = h1, c = h2, d = h3, e = h4;
        int i = 0;
        for (; i < 16; i++) { /* sha1.go:147-153 */
            uint32_t f = (b & c) | ((~b) & d);
            uint32_t t = rotl32(a, 5) + f + e + w[i & 0xf] + K0;
            e = d; d = c; c = rotl32(b, 30); b = a; a = t;
        }
        for (; i < 20; i++) { /* sha1.go:154-163 */
            uint32_t tmp = w[(i - 3) & 0xf] ^ w[(i - 8) & 0xf] ^ w[(i - 14) & 0xf] ^ w[i & 0xf];
            w[i & 0xf] = rotl32(tmp, 1);
            uint32_t f = (b & c) | ((~b) & d);
            uint32_t t = rotl32(a, 5) + f + e + w[i & 0xf] + K0;
            e = d; d = c; c = rotl32(b, 30); b = a; a = t;
        }
        for (; i < 40; i++) { /* sha1.go:164-172 */
            uint32_t tmp = w[(i - 3) & 0xf] ^ w[(i - 8) & 0xf] ^ w[(i - 14) & 0xf] ^ w[i & 0xf];
            w[i & 0xf] = rotl32(tmp, 1);
            uint32_t f = b ^ c ^ d;
            uint32_t t = rotl32(a, 5) + f + e + w[i & 0xf] + K1;
            e = d; d = c; c = rotl32(b, 30); b = a; a = t;
        }
        for (; i < 60; i++) { /* sha1.go:173-182 */
            uint32_t tmp = w[(i - 3) & 0xf] ^ w[(i - 8) & 0xf] ^ w[(i - 14) & 0xf] ^ w[i & 0xf];
            w[i & 0xf] = rotl32(tmp, 1);
            uint32_t f = ((b | c) & d) | (b & c);
            uint32_t t = rotl32(a, 5) + f + e + w[i & 0xf] + K2;
            e = d; d = c; c = rotl32(b, 30); b = a; a = t;
        }
        for (; i < 80; i++) { /* sha1.go:183-191 */
            uint32_t tmp = w[(i - 3) & 0xf] ^ w[(i - 8) & 0xf] ^ w[(i - 14) & 0xf] ^ w[i & 0xf];
            w[i & 0xf] = rotl32(tmp, 1);
            uint32_t f = b ^ c ^ d;
            uint32_t t = rotl32(a, 5) + f + e + w[i & 0xf] + K3;
            e = d; d = c; c = rotl32(b, 30); b = a; a = t;
        }
        h0 += a; h1 += b; h2 += c; h3 += d; h4 += e; /* sha1.go:193-197 */
        p += CHUNK;
        n -= CHUNK;
    }
    dig->h[0] = h0; dig->h[1] = h1; dig->h[2] = h2; dig->h[3] = h3; dig->h[4] = h4;
}

/* sha1.go:58-79 Write.  Go never returns an error here, but `copy(d.x[d.nx:], p)`
 * panics when nx > 64 (slice bounds); that panic is ORACLE_ERR_PANIC.  A negative nx
 * is skipped by `if d.nx > 0` exactly as in Go. */
int oracle_sha1_write(oracle_sha1* d, const uint8_t* p, size_t n) {
    d->len += (uint64_t)n; /* sha1.go:60 */
    if (d->nx > 0) {       /* sha1.go:61-69 */
        if (d->nx > CHUNK) return ORACLE_ERR_PANIC;
        size_t room = (size_t)(CHUNK - d->nx);
        size_t c = n < room ? n : room;
        memcpy(d->x + d->nx, p, c);
        d->nx += (int64_t)c;
        if (d->nx == CHUNK) {
            oracle_sha1_block(d, d->x, CHUNK);
            d->nx = 0;
        }
        p += c;
        n -= c;
    }
    if (n >= CHUNK) { /* sha1.go:70-74 */
        size_t m = n & ~(size_t)(CHUNK - 1);
        oracle_sha1_block(d, p, m);
        p += m;
        n -= m;
    }
    if (n > 0) { /* sha1.go:75-77: only x[:n] is overwritten; x[n:] keeps stale bytes */
        memcpy(d->x, p, n);
        d->nx = (int64_t)n;
    }
    return ORACLE_OK;
}

/* sha1.go:82-87 Sum (on a copy) + sha1.go:89-120 checkSum. */
int oracle_sha1_sum(const oracle_sha1* d0, uint8_t out[20]) {
    oracle_sha1 d = *d0; /* sha1.go:84 d := *d0 */
    uint64_t len = d.len;
    uint8_t tmp[64];
    memset(tmp, 0, sizeof tmp);
    tmp[0] = 0x80;
    int rc;
    if (len % 64 < 56) /* sha1.go:94-98 */
        rc = oracle_sha1_write(&d, tmp, (size_t)(56 - len % 64));
    else
        rc = oracle_sha1_write(&d, tmp, (size_t)(64 + 56 - len % 64));
    if (rc) return rc;
    len <<= 3; /* sha1.go:101-105 */
    for (int i = 0; i < 8; i++) tmp[i] = (uint8_t)(len >> (56 - 8 * i));
    rc = oracle_sha1_write(&d, tmp, 8);
    if (rc) return rc;
    if (d.nx != 0) return ORACLE_ERR_PANIC; /* sha1.go:107-109 panic("d.nx != 0") */
    for (int i = 0; i < 5; i++) { /* sha1.go:111-117 */
        out[i * 4] = (uint8_t)(d.h[i] >> 24);
        out[i * 4 + 1] = (uint8_t)(d.h[i] >> 16);
        out[i * 4 + 2] = (uint8_t)(d.h[i] >> 8);
        out[i * 4 + 3] = (uint8_t)d.h[i];
    }
    return ORACLE_OK;
}

static const char hexdig[] = "0123456789abcdef";

static void hex_encode(char* dst, const uint8_t* src, size_t n) {
    for (size_t i = 0; i < n; i++) {
        dst[2 * i] = hexdig[src[i] >> 4];
        dst[2 * i + 1] = hexdig[src[i] & 15];
    }
}

/* Go's encoding/hex fromHexChar: accepts 0-9, a-f, A-F. */
static int hex_val(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

static int hex_decode(uint8_t* dst, const char* src, size_t nbytes) {
    for (size_t i = 0; i < nbytes; i++) {
        int hi = hex_val(src[2 * i]), lo = hex_val(src[2 * i + 1]);
        if (hi < 0 || lo < 0) return -1;
        dst[i] = (uint8_t)(hi << 4 | lo);
    }
    return 0;
}

static void put_be32(uint8_t* b, uint32_t v) { b[0] = v >> 24; b[1] = v >> 16; b[2] = v >> 8; b[3] = (uint8_t)v; }
static void put_be64(uint8_t* b, uint64_t v) { for (int i = 0; i < 8; i++) b[i] = (uint8_t)(v >> (56 - 8 * i)); }
static uint32_t get_be32(const uint8_t* b) { return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]; }
static uint64_t get_be64(const uint8_t* b) { uint64_t v = 0; for (int i = 0; i < 8; i++) v = v << 8 | b[i]; return v; }

/* sha1_efes.go:25-38 MarshalText: hex(BE h0..h4 || x[0:64] || BE int64 nx || BE uint64 len). */
void oracle_sha1_marshal_text(const oracle_sha1* d, char out[200]) {
    uint8_t b[100];
    for (int i = 0; i < 5; i++) put_be32(b + 4 * i, d->h[i]);
    memcpy(b + 20, d->x, 64);
    put_be64(b + 84, (uint64_t)d->nx);
    put_be64(b + 92, d->len);
    hex_encode(out, b, 100);
}

/* sha1_efes.go:40-64 UnmarshalText. */
int oracle_sha1_unmarshal_text(oracle_sha1* d, const char* text, size_t n) {
    if (n != 200) return ORACLE_ERR_INVALID_DIGEST; /* sha1_efes.go:41-43 */
    uint8_t b[100];
    if (hex_decode(b, text, 100)) return ORACLE_ERR_INVALID_DIGEST; /* :45-48 */
    for (int i = 0; i < 5; i++) d->h[i] = get_be32(b + 4 * i);     /* :50-54 */
    memcpy(d->x, b + 20, 64);                                       /* :55 */
    int64_t nx = (int64_t)get_be64(b + 84);                         /* :56-57 */
    /* :58 `if nx > int64(MaxInt)`: never true on a 64-bit int (amd64). */
    d->nx = nx;
    d->len = get_be64(b + 92); /* :62 */
    return ORACLE_OK;
}

/* ---------------------------------------------------------------- CRC-32 */

#define IEEE 0xedb88320u /* crc32.go:25 */
static uint32_t tab8[8][256]; /* crc32.go:130-131 slicing8Table; tab8[0] == IEEETable */
static pthread_once_t tab_once = PTHREAD_ONCE_INIT;

/* crc32.go:106-118 simplePopulateTable + crc32.go:138-149 slicingMakeTable */
static void make_tables(void) {
    for (int i = 0; i < 256; i++) {
        uint32_t crc = (uint32_t)i;
        for (int j = 0; j < 8; j++) crc = (crc & 1) ? (crc >> 1) ^ IEEE : crc >> 1;
        tab8[0][i] = crc;
    }
    for (int i = 0; i < 256; i++) {
        uint32_t crc = tab8[0][i];
        for (int j = 1; j < 8; j++) {
            crc = tab8[0][crc & 0xFF] ^ (crc >> 8);
            tab8[j][i] = crc;
        }
    }
}

void oracle_crc32_init_tables(void) { pthread_once(&tab_once, make_tables); } /* crc32.go:35-45 ieeeOnce */

const uint32_t* oracle_crc32_table(int k) {
    oracle_crc32_init_tables();
    return tab8[k & 7];
}

/* crc32.go:122-128 simpleUpdate */
uint32_t oracle_crc32_simple_update(uint32_t crc, const uint8_t* p, size_t n) {
    oracle_crc32_init_tables();
    crc = ~crc;
    for (size_t i = 0; i < n; i++) crc = tab8[0][(uint8_t)crc ^ p[i]] ^ (crc >> 8);
    return ~crc;
}

/* crc32.go:153-169 slicingUpdate */
uint32_t oracle_crc32_slicing_update(uint32_t crc, const uint8_t* p, size_t n) {
    oracle_crc32_init_tables();
    if (n >= 16) { /* slicing8Cutoff, crc32.go:131 */
        crc = ~crc;
        while (n > 8) {
            crc ^= (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
            crc = tab8[0][p[7]] ^ tab8[1][p[6]] ^ tab8[2][p[5]] ^ tab8[3][p[4]] ^ tab8[4][crc >> 24] ^
                  tab8[5][(crc >> 16) & 0xFF] ^ tab8[6][(crc >> 8) & 0xFF] ^ tab8[7][crc & 0xFF];
            p += 8;
            n -= 8;
        }
        crc = ~crc;
    }
    if (n == 0) return crc;
    return oracle_crc32_simple_update(crc, p, n);
}

void oracle_crc32_reset(oracle_crc32* d) { d->crc = 0; }                                                 /* crc32.go:74 */
void oracle_crc32_write(oracle_crc32* d, const uint8_t* p, size_t n) { d->crc = oracle_crc32_slicing_update(d->crc, p, n); } /* crc32.go:76-86 */
uint32_t oracle_crc32_sum32(const oracle_crc32* d) { return d->crc; }                                    /* crc32.go:88 */

/* crc32_efes.go:18-24 */
void oracle_crc32_marshal_text(const oracle_crc32* d, char out[8]) {
    uint8_t b[4];
    put_be32(b, d->crc);
    hex_encode(out, b, 4);
}

/* crc32_efes.go:26-40 */
int oracle_crc32_unmarshal_text(oracle_crc32* d, const char* text, size_t n) {
    if (n != 8) return ORACLE_ERR_INVALID_DIGEST;
    uint8_t b[4];
    if (hex_decode(b, text, 4)) return ORACLE_ERR_INVALID_DIGEST;
    d->crc = get_be32(b);
    oracle_crc32_init_tables(); /* crc32_efes.go:37 ieeeOnce.Do(ieeeInit) */
    return ORACLE_OK;
}

/* ---------------------------------------------------------------- Sha1File */

/* sha1file.go:16-21 NewSha1File */
void oracle_sha1file_init(oracle_sha1file* f, const uint8_t* data, int64_t size) {
    f->data = data;
    f->size = size;
    f->rs_pos = 0;
    f->position = 0;
    f->calculated = 0;
    oracle_sha1_reset(&f->digest);
}

/* An io.Reader over a byte slice: reads min(n, remaining) bytes; 0 at EOF. */
static int64_t mem_read(oracle_sha1file* f, uint8_t* p, int64_t n) {
    int64_t rem = f->size - f->rs_pos;
    if (rem <= 0) return 0;
    int64_t c = n < rem ? n : rem;
    memcpy(p, f->data + f->rs_pos, (size_t)c);
    f->rs_pos += c;
    return c;
}

/* sha1file.go:23-37 Read.  Returns bytes read, or ORACLE_ERR_SHA1FILE for
 * "missing data for sha1" (sha1file.go:25). */
int64_t oracle_sha1file_read(oracle_sha1file* f, uint8_t* p, int64_t n) {
    if (f->position > f->calculated) return ORACLE_ERR_SHA1FILE;
    int64_t prev = f->position;
    int64_t got = mem_read(f, p, n);
    f->position += got;
    if (f->position > f->calculated) {
        int64_t crop = f->calculated - prev;
        oracle_sha1_write(&f->digest, p + crop, (size_t)(got - crop));
        f->calculated += got - crop;
    }
    return got;
}

/* sha1file.go:39-49 Seek.  whence: 0 start, 1 current, 2 end.  *err = 0 ok,
 * 1 the underlying seek failed (negative position), 2 "seeking forward is not
 * supported" (the underlying reader HAS moved; f->position has not, as in Go). */
int64_t oracle_sha1file_seek(oracle_sha1file* f, int64_t offset, int whence, int* err) {
    int64_t base = whence == 0 ? 0 : (whence == 1 ? f->rs_pos : f->size);
    int64_t np = base + offset;
    *err = 0;
    if (np < 0) { *err = 1; return 0; }
    f->rs_pos = np;
    if (f->position < np) { *err = 2; return np; }
    f->position = np;
    return np;
}

int oracle_sha1file_sum(const oracle_sha1file* f, uint8_t out[20]) { return oracle_sha1_sum(&f->digest, out); }

/* ---------------------------------------------------------------- stream + baseline */

/* filereceiver.go:208-209: w := io.MultiWriter(f, CRC32, Sha1); io.Copy(w, r).
 * io.Copy moves at most copy_buf bytes per Write; the writers are called in order
 * (file, CRC32, SHA-1).  Then the headers take Sum of each (filereceiver.go:99-100). */
void oracle_hash_message(const uint8_t* p, size_t n, size_t copy_buf, uint8_t sha1_out[20], uint32_t* crc_out) {
    oracle_sha1 s;
    oracle_crc32 c;
    oracle_sha1_reset(&s);
    oracle_crc32_reset(&c);
    if (copy_buf == 0) copy_buf = 32 * 1024;
    for (size_t off = 0; off < n; off += copy_buf) {
        size_t m = n - off < copy_buf ? n - off : copy_buf;
        oracle_crc32_write(&c, p + off, m);
        oracle_sha1_write(&s, p + off, m);
    }
    oracle_sha1_sum(&s, sha1_out);
    *crc_out = c.crc;
}

typedef struct {
    const uint8_t* base;
    size_t stride;
    const uint64_t* lens;
    size_t nmsg;
    uint8_t* sha1_out;
    uint32_t* crc_out;
    atomic_size_t next;
} many_ctx;

static void* many_worker(void* arg) {
    many_ctx* m = (many_ctx*)arg;
    for (;;) {
        size_t i = atomic_fetch_add(&m->next, 1);
        if (i >= m->nmsg) break;
        oracle_hash_message(m->base + i * m->stride, (size_t)m->lens[i], 32 * 1024, m->sha1_out + 20 * i, m->crc_out + i);
    }
    return NULL;
}

double oracle_hash_many(const uint8_t* base, size_t stride, const uint64_t* lens, size_t nmsg, int nthreads,
                        uint8_t* sha1_out, uint32_t* crc_out) {
    oracle_crc32_init_tables();
    if (nthreads < 1) nthreads = 1;
    many_ctx m = {base, stride, lens, nmsg, sha1_out, crc_out, 0};
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, many_worker, &m);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    free(th);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

void oracle_fill_synthetic(uint8_t* p, size_t n, uint64_t seed) {
    const uint64_t gamma = 0x9E3779B97F4A7C15ull;
    size_t nw = n / 8;
    for (size_t i = 0; i < nw; i++) {
        uint64_t z = seed + (uint64_t)(i + 1) * gamma;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        memcpy(p + 8 * i, &z, 8); /* little-endian host */
    }
    if (n % 8) {
        uint64_t z = seed + (uint64_t)(nw + 1) * gamma;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        memcpy(p + 8 * nw, &z, n % 8);
    }
}
