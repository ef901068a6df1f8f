/*
 * efes_hash.h -- C ABI of the MI355X-native content-hashing path of efes.
 *
 * This library replaces the per-chunk SHA-1 + CRC-32/IEEE that putdotio/efes streams
 * every uploaded byte through.  Cited reference interfaces (/root/reference/<file>:<line>):
 *   sha1digest  (sha1.go:29-120), its text codec (sha1_efes.go:25-64),
 *   crc32digest (crc32.go:48-93), its text codec (crc32_efes.go:18-40),
 *   and the hot loop io.MultiWriter(f, CRC32, Sha1) + io.Copy (filereceiver.go:208-209).
 *
 * Two layers:
 *   1. Batched device-resident hot path (efes_hash_submit): every job is ONE `Write(p)`
 *      (sha1.go:58-79 and crc32.go:76-86) of a device buffer into a device-resident
 *      state, optionally followed by `Sum` (sha1.go:82-120, crc32.go:90-93).  All
 *      compression runs in hand-written gfx950 kernels.  Jobs are independent.
 *   2. Streaming digest objects mirroring the Go `hash.Hash` surface (efes_sha1_*,
 *      efes_crc32_*), staging host bytes and hashing them on the GPU through layer 1.
 *      Their MarshalText/UnmarshalText are byte-identical to the reference's, so
 *      `<path>.info` files (fileinfo.go:10-58) stay interchangeable.
 *
 * Plain C types only; every pointer documented "device" must be device memory of the
 * context's GPU (hipMalloc), "host" pointers are ordinary host memory.  Functions
 * return 0 (EFES_OK) or a negative efes error code; nothing panics or aborts.
 * All functions are thread-safe except concurrent use of ONE streaming object.
 */
#ifndef EFES_HASH_H
#define EFES_HASH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EFES_ABI_VERSION 7

/* ---- error codes ---------------------------------------------------------------- */
#define EFES_OK 0
#define EFES_ERR_INVALID_DIGEST (-1) /* sha1_efes.go:23 errInvalidDigest (bad text length / hex) */
#define EFES_ERR_STATE (-2)          /* state on which the Go code would panic: nx > 64 at Write
                                        (slice bounds, sha1.go:62) or d.nx != 0 in checkSum (sha1.go:107-109) */
#define EFES_ERR_HIP (-3)            /* a HIP runtime call failed (device fault, OOM, ...) */
#define EFES_ERR_ARG (-4)            /* invalid argument (NULL, bad flags, misaligned state) */
#define EFES_ERR_NO_DEVICE (-5)      /* no usable gfx950 device */
#define EFES_ERR_NOMEM (-6)          /* host allocation failed */
#define EFES_ERR_DEVICE_FAULT (-7)   /* an earlier asynchronous device error was latched */

const char* efes_strerror(int code);
int efes_abi_version(void);
/* The identity of the sources the library was built from (ABI 7): 16 hex digits of a SHA-256 over its
 * source and header files, compiled in by efes_amd/build.py ("unversioned" for any other build), so a
 * deployment -- and the GPU tests -- can check that the loaded library matches the sources beside it. */
const char* efes_build_id(void);

/* ---- state layouts (device- and host-side identical) ----------------------------- */

/* sha1.go:29-34 `sha1digest`: field order = MarshalText order (sha1_efes.go:26-34). */
typedef struct efes_sha1_state {
    uint32_t h[5];  /* running hash */
    uint8_t x[64];  /* tail buffer; bytes x[nx:64] are stale, exactly as in Go */
    uint32_t _pad;  /* keeps nx/len 8-byte aligned; ignored */
    int64_t nx;     /* bytes pending in x (Go int) */
    uint64_t len;   /* total bytes written (Go uint64, wraps) */
} efes_sha1_state; /* 104 bytes */

/* crc32.go:48-51 `crc32digest` (the table is always IEEE, crc32_efes.go:37-38). */
typedef struct efes_crc32_state {
    uint32_t crc; /* the finalized CRC-32/IEEE of everything written so far (Sum32) */
} efes_crc32_state;

/* sha1.go:36-44 Reset / sha1.go:48-52 NewSha1. */
void efes_sha1_state_init(efes_sha1_state* s);

/* ---- context ----------------------------------------------------------------------- */
typedef struct efes_ctx efes_ctx;

/* HIP devices visible to the process, of any architecture (ABI 7): 0 when there are none or the
 * runtime fails.  A binding opens every ordinal below it and SKIPS the ones efes_ctx_create refuses
 * (EFES_ERR_NO_DEVICE for a non-gfx950 card, EFES_ERR_HIP / EFES_ERR_NOMEM for one that fails to
 * initialise), so one bad GPU does not hide the GPUs after it (go/hash_gpu.go pool()). */
int efes_device_count(void);
/* Binds one GPU (HIP device ordinal), uploads the CRC tables, creates a stream.  EFES_ERR_ARG for an
 * ordinal outside [0, efes_device_count()), EFES_ERR_NO_DEVICE for a device that is not gfx950. */
int efes_ctx_create(int device, efes_ctx** out);
void efes_ctx_destroy(efes_ctx* ctx);
int efes_ctx_device(const efes_ctx* ctx);
/* The context's own stream (a hipStream_t), used when a call passes stream == NULL. */
void* efes_ctx_stream(efes_ctx* ctx);

/* ---- layer 1: batched device-resident jobs ----------------------------------------- */
#define EFES_JOB_FINALIZE 0x1u /* also write Sum of the post-Write state to `sum` */
#define EFES_JOB_INIT 0x2u     /* start from NewSha1() / NewCRC32IEEE() (sha1.go:48-52, crc32.go:68):
                                  the in-states are not read, only written (a fresh chunk) */
#define EFES_JOB_SUM_ONLY 0x4u /* with EFES_JOB_FINALIZE and length 0: Sum of the in-state on a copy
                                  (sha1.go:82-87 `d0 := *d`): the states are read, never written, so
                                  a pending full tail (nx == 64) stays pending as in Go */

/* One `Write(p)` (+ optional Sum) of len(p) = length bytes at device address `data`.
 * sha1 / crc32: device states updated in place; either may be NULL to skip that hash
 * (the MultiWriter of filereceiver.go:208 passes both).  sum (device, 24 bytes, only
 * with EFES_JOB_FINALIZE): SHA-1 Sum (20 B, sha1.go:82-87) then CRC-32 Sum (4 B BE,
 * crc32.go:90-93).  status (device, may be NULL): EFES_OK or EFES_ERR_STATE.
 * Jobs in one submit must not share a state. */
typedef struct efes_job {
    const void* data;
    uint64_t length;
    efes_sha1_state* sha1;
    efes_crc32_state* crc32;
    uint8_t* sum;
    int32_t* status;
    uint32_t flags;
    uint32_t _reserved;
} efes_job; /* 56 bytes */

/* Kernel shapes: DEEP = one wavefront per job (few, long jobs: per-job latency bound);
 * WIDE = one lane per job (many jobs: throughput bound).  AUTO picks by njobs.
 * GROUPn = grouped DEEP, 64/n jobs per wavefront with n lanes (n consecutive 64-B blocks
 * per step) each: for more long jobs than SIMDs (lower per-job latency than WIDE, fewer
 * instructions per byte than DEEP).  Jobs should be longest-first (efes_plan_batch).
 * AUTO picks by njobs (efes_auto_mode). */
#define EFES_MODE_AUTO 0
#define EFES_MODE_DEEP 1
#define EFES_MODE_WIDE 2
#define EFES_MODE_GROUP4 3
#define EFES_MODE_GROUP8 4
#define EFES_MODE_GROUP16 5
#define EFES_MODE_GROUP32 6
/* FED4: grouped DEEP (16 jobs of 4 lanes per chain wave) whose loads, CRC and schedule
 * expansion run on a producer wave on another SIMD of the same CU, so a job advances at DEEP's
 * per-block latency; 48 jobs per workgroup, each workgroup owns its CU.  For the longest jobs of
 * a mixed batch (efes_plan_batch), more of them than SIMDs. */
#define EFES_MODE_FED4 7
/* FED4E: FED4 with three chain waves and one producer per CU; the chain waves expand the
 * schedule themselves (the producer loads, CRCs and hands over the 16 message words): 48 jobs per
 * CU at a per-job latency between FED4's and GROUP4's. */
#define EFES_MODE_FED4E 8

/* Largest job count of one submit / plan / host batch (larger counts: EFES_ERR_ARG; split the
 * batch).  Keeps every grid size and lane index of the kernels within 32 bits. */
#define EFES_MAX_JOBS (1u << 30)

/* Enqueue njobs jobs (the job array itself in DEVICE memory) on `stream` (a
 * hipStream_t; NULL = the context stream).  Asynchronous; returns launch errors only. */
int efes_hash_submit(efes_ctx* ctx, const efes_job* jobs_device, uint32_t njobs, void* stream);
int efes_hash_submit_mode(efes_ctx* ctx, const efes_job* jobs_device, uint32_t njobs, void* stream, int mode);
/* The shape EFES_MODE_AUTO picks for njobs jobs of similar length (ctx may be NULL: one
 * MI355X): DEEP up to one job per SIMD, FED4 up to 32 per CU, FED4E up to 48 per CU, GROUP4 up to
 * 16 per SIMD (one wave each), WIDE beyond. */
int efes_auto_mode(const efes_ctx* ctx, uint32_t njobs);
/* Mixed-length batches (BASELINE configs[3], concurrent uploads of different sizes): the
 * makespan is set by the longest jobs (a SHA-1 chain per job), so a batch is cut, longest
 * first, into up to EFES_PLAN_MAX_PARTS consecutive parts that run CONCURRENTLY, each in its
 * own kernel shape: typically the longest jobs grouped-DEEP on CUs of their own (`exclusive`:
 * the launch reserves the CU's LDS so no other workgroup shares its SIMDs), the next ones
 * grouped-DEEP beside the rest, which run WIDE.
 * efes_plan_batch orders the jobs longest-first (order[i] = index into `lengths` of the job to
 * place at jobs_device[i]) and picks the cuts, shapes and exclusivity from an issue-time model
 * of the kernels calibrated on MI355X (DESIGN_NOTES.md §4); efes_hash_submit_plan launches a batch
 * laid out in that order: each part on a part stream of its own (created one after the other, so
 * usually -- HIP assigns hardware queues round-robin over all streams of the process, so not
 * certainly -- on distinct hardware queues), after the work queued on `stream`, which then waits
 * for all of them.  Planning is host-only (no device access; ctx
 * may be NULL: then the capacity of one MI355X, 256 CUs, is assumed). */
#define EFES_PLAN_MAX_PARTS 4
typedef struct efes_plan_part {
    uint32_t jobs;       /* consecutive jobs of this part (in plan order) */
    int32_t mode;        /* EFES_MODE_DEEP, EFES_MODE_GROUPn, EFES_MODE_FED4, EFES_MODE_FED4E or EFES_MODE_WIDE */
    uint32_t exclusive;  /* 1: each workgroup reserves its CU (one wave per SIMD); FED4/FED4E parts
                            ignore it: their workgroups always own their CU */
    uint32_t _reserved;
} efes_plan_part;
typedef struct efes_plan {
    uint32_t njobs;      /* jobs in the batch = sum of part[i].jobs */
    uint32_t nparts;     /* parts in use, 1..EFES_PLAN_MAX_PARTS (0 for an empty batch) */
    efes_plan_part part[EFES_PLAN_MAX_PARTS];
    double est_seconds;  /* the model's makespan estimate (informational) */
} efes_plan;
int efes_plan_batch(efes_ctx* ctx, const uint64_t* lengths, uint32_t n, uint32_t* order, efes_plan* plan);
int efes_hash_submit_plan(efes_ctx* ctx, const efes_job* jobs_device, const efes_plan* plan, void* stream);

/* Wait for `stream` (NULL = context stream); reports latched asynchronous errors. */
int efes_sync(efes_ctx* ctx, void* stream);

/* Device memory helpers for hosts without their own allocator (cgo). */
int efes_device_alloc(efes_ctx* ctx, size_t bytes, void** out);
int efes_device_free(efes_ctx* ctx, void* p);
int efes_copy_to_device(efes_ctx* ctx, void* dst_device, const void* src_host, size_t bytes, void* stream);
int efes_copy_to_host(efes_ctx* ctx, void* dst_host, const void* src_device, size_t bytes, void* stream);
/* Synthetic benchmark bytes: little-endian splitmix64 stream, z_i = mix(seed + (i+1)*0x9E3779B97F4A7C15). */
int efes_fill_synthetic(efes_ctx* ctx, void* dst_device, size_t bytes, uint64_t seed, void* stream);

/* ---- host-resident ingest -------------------------------------------------------------
 * The reference's path starts in host memory (a socket buffer, filereceiver.go:208-209).
 * efes_hash_host runs the jobs of a HOST array whose data/sha1/crc32/sum/status pointers are
 * all HOST memory: segment s (segment_bytes, rounded up to 64; 0 = 256 KiB) of every message is
 * copied H2D with hipMemcpyAsync on the context's copy stream (a hardware queue of its own) into
 * one of two device slots while segment s-1 is hashed on the context stream; concurrent calls on
 * one context take the copy stream in turn; states stay on the device between segments (the
 * per-PATCH resume of filereceiver.go:182-226); states, sums and status are copied back at
 * the end.  Equivalent to one Write per segment (so the stale bytes x[nx:64] are those of
 * segment-sized Writes, sha1.go:75-77).  Messages whose host addresses advance by a constant stride are copied with one
 * 2D copy per segment.  For the full PCIe rate the data should be pinned (efes_host_alloc).
 * Synchronous; stats (may be NULL) time the pipeline from the first copy to the last result. */
/* segment_bytes == EFES_HOST_ZERO_COPY: every data pointer is pinned, device-mapped host memory
 * (efes_host_alloc) and one launch reads it in place over PCIe: no staging copies, no segments
 * (EFES_ERR_ARG if a pointer is not device-accessible).  Stats time the launch and the result
 * copies. */
#define EFES_HOST_ZERO_COPY ((uint64_t)-1)
typedef struct efes_host_stats {
    double seconds;    /* wall time of the copy+hash pipeline */
    uint64_t bytes;    /* message bytes moved and hashed */
    uint32_t segments; /* pipeline steps */
    uint32_t _reserved;
} efes_host_stats;

int efes_hash_host(efes_ctx* ctx, const efes_job* jobs_host, uint32_t njobs, uint64_t segment_bytes,
                   efes_host_stats* stats);
int efes_host_alloc(efes_ctx* ctx, size_t bytes, void** out); /* pinned, device-mapped host memory */
int efes_host_free(efes_ctx* ctx, void* p);

/* ---- concurrent uploads: batching dispatcher ------------------------------------------
 * An efes_upload is the MultiWriter(CRC32, Sha1) of ONE upload (filereceiver.go:208) with
 * both states in HBM.  efes_upload_write copies into pinned staging (chunk_bytes pieces out
 * of max_chunks; it blocks only when all are in use) and returns; the queue's dispatcher
 * thread launches the staged chunks of ALL uploads together -- one job per upload per launch,
 * so each upload's chain stays in order -- while callers keep staging.  Sync points wait for
 * that upload's bytes only: flush; state (h/crc from the device, x/nx/len replayed on the host
 * per Write, so MarshalText of it is byte-identical to Go's after the same Writes); sum
 * (SHA-1 Sum || CRC Sum, non-destructive, sha1.go:82-87).  Uploads may be used from different
 * threads concurrently; one upload must not be written from two threads at once (each Go
 * digest belongs to one request goroutine, server.go:130).  max_uploads bounds open uploads
 * and must be < max_chunks (each open upload may hold one partly filled chunk). */
typedef struct efes_queue efes_queue;
typedef struct efes_upload efes_upload;
#define EFES_HASH_SHA1 0x1u  /* which digests an upload keeps (a MultiWriter of both is 0x3) */
#define EFES_HASH_CRC32 0x2u
int efes_queue_create(efes_ctx* ctx, uint64_t chunk_bytes, uint32_t max_chunks, uint32_t max_uploads,
                      efes_queue** out);
void efes_queue_destroy(efes_queue* q); /* finishes launched work; close uploads first */
/* hashes: EFES_HASH_SHA1 | EFES_HASH_CRC32; sha1 / crc32: initial states (host), NULL =
 * NewSha1() / NewCRC32IEEE().  Sums of a digest the upload does not keep read as zeros. */
int efes_upload_open(efes_queue* q, uint32_t hashes, const efes_sha1_state* sha1, const efes_crc32_state* crc32,
                     efes_upload** out);
int efes_upload_write(efes_upload* u, const void* p, size_t n);
/* Zero-copy staging (ABI 3): *p / *n = at least min(min_bytes, chunk_bytes) contiguous bytes of
 * the upload's pinned staging chunk (a partly filled chunk with less room is handed to the
 * dispatcher first; blocks while every chunk is in use).  Fill k <= *n of them -- read a request
 * body straight in, write the file from there -- and efes_upload_commit(u, k): the same as
 * efes_upload_write of those k bytes (one Write of k bytes, sha1.go:58-79) without the copy.
 * Bytes reserved but not committed are dropped; reserve again before the next commit (a commit
 * of more bytes than the last reserve granted, a second commit, or a commit after a write returns
 * EFES_ERR_ARG).  The pointer is valid only until the commit. */
int efes_upload_reserve(efes_upload* u, size_t min_bytes, void** p, size_t* n);
int efes_upload_commit(efes_upload* u, size_t k);
int efes_upload_flush(efes_upload* u);
int efes_upload_state(efes_upload* u, efes_sha1_state* sha1, efes_crc32_state* crc32);
int efes_upload_sum(efes_upload* u, uint8_t out[24]);
void efes_upload_close(efes_upload* u); /* drops bytes staged since the last sync point */
/* Counters of a queue (ABI 5): what its dispatcher launched, and its upload slots. */
typedef struct efes_queue_stats {
    uint64_t launches;      /* kernel launches */
    uint64_t jobs;          /* jobs in them (one per upload per launch, Sums included) */
    uint64_t bytes;         /* staged bytes hashed */
    uint32_t free_uploads;  /* upload (state) slots free now */
    uint32_t max_uploads;
} efes_queue_stats;
int efes_queue_get_stats(efes_queue* q, efes_queue_stats* out);

/* ---- layer 2: streaming digests mirroring the Go surface ----------------------------
 * Each object is an upload (above) of the context's shared digest queue that keeps only its
 * own hash, so unchanged Go code -- MultiWriter(f, CRC32, Sha1) in every request goroutine --
 * is batched across all concurrent requests: Write stages into pinned memory and returns,
 * Sum / Sum32 / MarshalText are the sync points.  The shared queue holds
 * EFES_DIGEST_STAGING_MIB (env, default 1024) of pinned staging in EFES_DIGEST_CHUNK_KIB (default
 * 256) chunks and EFES_DIGEST_SLOTS (default 65536) upload slots: a digest (a fused CRC + SHA-1 pair
 * is one) holds a slot from its first Write to its sync point; when writers wait for a chunk and
 * every chunk sits partly filled in idle uploads, the queue's dispatcher has those handed over.  A
 * Write blocks while all chunks are in flight.  EFES_DIGEST_SLOTS below the chunk count gives one
 * slot per chunk at most (no hand-over; a Write evicts instead, below).
 *
 * Go's Write never fails (sha1.go:58-79, crc32.go:76-86), and neither does this one for any
 * number of live digests:
 *   - a digest holds an upload slot only between its first Write and its next sync point: every
 *     Sum / Sum32 / MarshalText parks the state on the host and gives the slot back, the next
 *     Write takes one again (so digests that are never freed hold no queue resources);
 *   - a Write (or Sum) that finds every slot taken waits for a holder's sync point; it evicts the
 *     oldest holder that is not inside a call and has been idle for EFES_DIGEST_EVICT_MS (env,
 *     default 50; a stalled client, an abandoned digest) -- or, once it has itself waited that
 *     long, the oldest holder not inside a call -- hashing what that one staged and parking its
 *     state on the host; back-pressure, never EFES_ERR_NOMEM;
 *   - a device or HIP fault during a Write is latched and the Write returns EFES_OK: the next
 *     Sum / Sum32 / MarshalText reports it (MarshalText's error -> HTTP 500, filereceiver.go:94-96).
 * Write returns an error only for bad arguments and for the states on which Go's Write panics
 * (EFES_ERR_STATE: nx > 64, sha1.go:62).  The object itself is host memory, so freeing it late
 * (a Go finalizer) costs nothing scarce. */
typedef struct efes_sha1 efes_sha1;
typedef struct efes_crc32 efes_crc32;

/* Fused pairs (ABI 6).  io.MultiWriter(f, CRC32, Sha1) (filereceiver.go:208-209) hands every body
 * buffer to the CRC digest and then, unchanged, to the SHA-1 digest.  The library detects that
 * pattern and binds the two digests to ONE upload keeping both hashes, so each byte is staged once
 * and hashed by one fused job, as efes_upload_* does for a caller that asks for it:
 *   - a CRC digest's first Write after a sync point is held back (copied) as a candidate; a parked
 *     SHA-1 digest's Write with the same pointer and length binds to it, and the pair opens one
 *     upload (a candidate nobody binds is staged at the CRC digest's next call);
 *   - then each CRC Write is held back until the SHA-1 Write of the same (p, n) -- of any size --
 *     is staged and compared with it in one pass, which confirms it;
 *   - anything else (a Write to one digest only, other bytes, the CRC digest synced first, Reset /
 *     UnmarshalText / free of one, an eviction) splits the pair: every confirmed byte is in both
 *     states, an unconfirmed CRC Write in the CRC state only, and both go on alone.
 * Every digest therefore hashes exactly the bytes of its own Writes, in order, whatever the caller
 * does; only the speed depends on the pattern.  Process-wide counters: */
typedef struct efes_pair_stats {
    uint64_t pairs;         /* CRC + SHA-1 digests bound to one upload */
    uint64_t fused_writes;  /* SHA-1 Writes confirming the CRC Write (one staging copy, one job) */
    uint64_t fused_bytes;   /* their bytes */
    uint64_t settles;       /* pairs split (diverging Writes, evictions) */
} efes_pair_stats;
int efes_pair_stats_get(efes_pair_stats* out);

int efes_sha1_new(efes_ctx* ctx, efes_sha1** out);                       /* sha1.go:48-52 NewSha1 */
int efes_sha1_new_zero(efes_ctx* ctx, efes_sha1** out);                  /* `var d sha1digest` (zero value) */
void efes_sha1_free(efes_sha1* d);
void efes_sha1_reset(efes_sha1* d);                                      /* sha1.go:36-44 */
int efes_sha1_size(void);                                                /* sha1.go:54 (20) */
int efes_sha1_block_size(void);                                          /* sha1.go:56 (64) */
int efes_sha1_write(efes_sha1* d, const void* p, size_t n);              /* sha1.go:58-79 */
int efes_sha1_sum(efes_sha1* d, uint8_t out[20]);                        /* sha1.go:82-87 */
int efes_sha1_marshal_text(efes_sha1* d, char out[200]);                 /* sha1_efes.go:25-38 */
int efes_sha1_unmarshal_text(efes_sha1* d, const char* text, size_t n);  /* sha1_efes.go:40-64 */
int efes_sha1_get_state(efes_sha1* d, efes_sha1_state* out);
int efes_sha1_set_state(efes_sha1* d, const efes_sha1_state* in);

int efes_crc32_new(efes_ctx* ctx, efes_crc32** out);                     /* crc32.go:68 NewCRC32IEEE */

/* Multi-GPU digests (ABI 5).  A storage server is one process (server.go:130, one goroutine per
 * request), so one process's digests should use every GPU: a pool spreads them over its
 * contexts.  A pooled digest takes its upload slot, at every (re)open, on the context whose digest
 * queue has the most free slots (its state is on the host between sync points, so consecutive
 * PATCHes of one object may run on different GPUs; the byte order is kept by the caller).  The
 * contexts must outlive the pool, and the pool its digests. */
typedef struct efes_pool efes_pool;
int efes_pool_create(efes_ctx* const* ctxs, uint32_t n, efes_pool** out);
void efes_pool_destroy(efes_pool* p);
int efes_sha1_new_pool(efes_pool* p, efes_sha1** out);                   /* NewSha1 on the pool */
int efes_sha1_new_zero_pool(efes_pool* p, efes_sha1** out);              /* `var d sha1digest` on the pool */
int efes_crc32_new_pool(efes_pool* p, efes_crc32** out);                 /* NewCRC32IEEE on the pool */
/* Counters of the digest queue of the pool's i-th context (zeros before its first digest Write). */
int efes_pool_stats(efes_pool* p, uint32_t i, efes_queue_stats* out);
void efes_crc32_free(efes_crc32* d);
void efes_crc32_reset(efes_crc32* d);                                    /* crc32.go:74 */
int efes_crc32_size(void);                                               /* crc32.go:70 (4) */
int efes_crc32_block_size(void);                                         /* crc32.go:72 (1) */
int efes_crc32_write(efes_crc32* d, const void* p, size_t n);            /* crc32.go:76-86 */
int efes_crc32_sum32(efes_crc32* d, uint32_t* out);                      /* crc32.go:88 */
int efes_crc32_sum(efes_crc32* d, uint8_t out[4]);                       /* crc32.go:90-93 */
int efes_crc32_marshal_text(efes_crc32* d, char out[8]);                 /* crc32_efes.go:18-24 */
int efes_crc32_unmarshal_text(efes_crc32* d, const char* text, size_t n);/* crc32_efes.go:26-40 */

/* Host-side diagnostics (no device work): copies the CRC-32 tables the kernels use,
 * slice8[8][256] (crc32.go:138-149) then shift[7][4][256] (advance of the raw register
 * over 64<<k zero bytes, byte-sliced), then -- when nwords leaves room for them (9216 + 16384
 * words) -- the position tables pos[64][256] (the raw register after a 64-byte block whose only
 * nonzero byte is b at offset o, from register 0: the WIDE and grouped kernels' block CRC);
 * returns the word count written or EFES_ERR_ARG. */
int efes_crc32_tables(uint32_t* out, size_t nwords);

/* CRC-32 of A||B from crc(A), crc(B) and |B| (crc32.go is GF(2)-linear: the zlib
 * crc32_combine identity), so chunks of one object can be CRC'd out of order or on different
 * devices and merged on the host; len2 may be any size (O(log len2) 32x32 GF(2) products). */
uint32_t efes_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);

/* CRC-32 of ONE long device buffer on the whole GPU: the same result as
 * crc32.go's Write (76-86) of `length` bytes at `data` (device memory, any alignment) into the
 * device state *crc -- so chained calls compose like Writes and efes_crc32_combine merges pieces
 * hashed on different GPUs -- but computed segment-parallel instead of byte by byte: every 64-byte
 * block's raw CRC from position tables, merged by the GF(2)-linearity that efes_crc32_combine uses.
 * For an object's CRC alone (a re-check after a copy or drain); uploads keep the fused SHA-1 +
 * CRC-32 jobs above, whose speed SHA-1's serial chain sets.  Asynchronous on `stream` (NULL = the
 * context stream); calls that share a state must be ordered on one stream. */
int efes_crc32_span(efes_ctx* ctx, const void* data_device, uint64_t length, efes_crc32_state* crc_device,
                    void* stream);

/* Test hooks are declared in efes_testing.h: exported, but not part of the stable surface. */

/* Pure text codecs on plain states (no device work). */
void efes_sha1_state_marshal_text(const efes_sha1_state* s, char out[200]);
int efes_sha1_state_unmarshal_text(efes_sha1_state* s, const char* text, size_t n);
void efes_crc32_state_marshal_text(const efes_crc32_state* s, char out[8]);
int efes_crc32_state_unmarshal_text(efes_crc32_state* s, const char* text, size_t n);

#ifdef __cplusplus
}
#endif
#endif /* EFES_HASH_H */
