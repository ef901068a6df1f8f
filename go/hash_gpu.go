//go:build efesgpu

// hash_gpu.go -- the cgo binding of libefeshash.so (include/efes_hash.h) that replaces the pure-Go
// digests of putdotio/efes under the build tag `efesgpu` (INTEGRATION.md §2).
//
// Drop-in: copy this file (and, optionally, upload_gpu.go) into the reference's package directory
// next to `include/` and `efes_amd/lib/` of this repository, apply efesgpu_build_tags.patch (one
// `//go:build !efesgpu` line on sha1.go, sha1_efes.go, crc32.go and crc32_efes.go), and build the
// storage server with `CGO_ENABLED=1 go build -tags efesgpu` (INTEGRATION.md §1).  Without the tag the
// reference builds exactly as before.  It defines what the four excluded files defined and the rest of
// the package uses: the types sha1digest / crc32digest with their method sets (sha1.go:29-120,
// sha1_efes.go:25-64, crc32.go:48-93, crc32_efes.go:18-40), NewSha1 (sha1.go:48-52), NewCRC32IEEE
// (crc32.go:68) and errInvalidDigest (sha1_efes.go:23).  sha1file.go, fileinfo.go, filereceiver.go,
// write.go and the _efes_test.go files compile unchanged against it.
//
// No Go toolchain exists in the image this was written in: tests/test_abi.py checks this file as text
// (symbols it binds, handle ownership, KeepAlive after C calls, the device enumeration), and
// tests/c/efes_consumer_test.c / efes_lifecycle_test.c make the same C calls in the same order.

package main

/*
#cgo CFLAGS: -I${SRCDIR}/include
#cgo LDFLAGS: -L${SRCDIR}/efes_amd/lib -lefeshash -Wl,-rpath,${SRCDIR}/efes_amd/lib
#include "efes_hash.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"strconv"
	"sync"
	"sync/atomic"
	"unsafe"

	"github.com/cenkalti/log"
	"github.com/prometheus/client_golang/prometheus"
)

// sha1_efes.go:23, which this build excludes.
var errInvalidDigest = errors.New("invalid digest")

var (
	gpuOnce    sync.Once
	gpuLog     = log.NewLogger("gpu")
	gpuVisible int             // efes_device_count(): HIP devices the process sees
	gpuCtxs    []*C.efes_ctx   // one per GPU that opened
	gpuDevs    []int           // the HIP ordinal of gpuCtxs[i] (the `gpu` label of the gauges)
	gpuSkipped []string        // "ordinal: reason" of every GPU that did not open
	gpuPool    *C.efes_pool
	gpuReady   atomic.Bool // set once gpuCtxs / gpuPool are complete (read by the metrics collector)
)

// The storage server is ONE process (server.go:130: a goroutine per request), so the digests of all
// its requests share every GPU of the node: one context per GPU, one pool over them.  Each digest
// takes its upload slot on the GPU whose digest queue has the most free slots.  A GPU that does not
// open -- not gfx950 (EFES_ERR_NO_DEVICE), failing to initialise (EFES_ERR_HIP, EFES_ERR_NOMEM) -- is
// logged, counted and skipped: it must not hide the GPUs after it.
func pool() *C.efes_pool {
	gpuOnce.Do(func() {
		gpuVisible = int(C.efes_device_count())
		for dev := 0; dev < gpuVisible; dev++ {
			var c *C.efes_ctx
			if rc := C.efes_ctx_create(C.int(dev), &c); rc != C.EFES_OK {
				reason := C.GoString(C.efes_strerror(rc))
				gpuSkipped = append(gpuSkipped, fmt.Sprintf("%d: %s", dev, reason))
				gpuLog.Warningln("GPU", dev, "skipped:", reason)
				continue
			}
			gpuCtxs = append(gpuCtxs, c)
			gpuDevs = append(gpuDevs, dev)
		}
		if len(gpuCtxs) == 0 {
			panic(fmt.Sprintf("efes gpu: no usable gfx950 device among %d visible (%v)", gpuVisible, gpuSkipped))
		}
		gpuLog.Noticeln("digests on", len(gpuCtxs), "of", gpuVisible, "GPUs; ordinals", gpuDevs)
		// a Go slice of C pointers may be passed to C (it holds no Go pointers)
		if rc := C.efes_pool_create(&gpuCtxs[0], C.uint32_t(len(gpuCtxs)), &gpuPool); rc != C.EFES_OK {
			panic(fmt.Sprintf("efes gpu: %s", C.GoString(C.efes_strerror(rc))))
		}
		gpuReady.Store(true)
	})
	return gpuPool
}

// Write never fails, as sha1.go:58-79 / crc32.go:76-86 never do: the library blocks for an upload
// slot (evicting an idle digest) instead of running out, and latches device faults for the next Sum /
// MarshalText.  Its only error is the one Go's Write panics on (nx > 64, the slice bounds of
// sha1.go:62), so that is the only panic here.
func checkWrite(rc C.int) {
	switch rc {
	case C.EFES_OK:
	case C.EFES_ERR_STATE:
		panic("runtime error: slice bounds out of range") // sha1.go:62 with nx > 64
	default: // EFES_ERR_ARG: a nil handle, a bug in this file
		panic(fmt.Sprintf("efes gpu: %s", C.GoString(C.efes_strerror(rc))))
	}
}

// Sum cannot return an error in Go (hash.Hash), so a latched device fault panics there; net/http
// recovers a handler's panic per request.  The .info path (MarshalText, filereceiver.go:226) returns
// the error instead (-> HTTP 500, filereceiver.go:94-96).
func checkSum(rc C.int) {
	switch rc {
	case C.EFES_OK:
	case C.EFES_ERR_STATE: // checkSum's panic (sha1.go:107-109)
		panic("d.nx != 0")
	default:
		panic(fmt.Sprintf("efes gpu: %s", C.GoString(C.efes_strerror(rc))))
	}
}

// cbytes: the address of p's first byte for C (nil for an empty slice).  cgo pins p for the call.
func cbytes(p []byte) unsafe.Pointer {
	if len(p) == 0 {
		return nil
	}
	return unsafe.Pointer(&p[0])
}

// ---- sha1digest: sha1.go:29-34 -- same name, same method set ------------------------------------

type sha1digest struct{ c *C.efes_sha1 }

// open allocates d's handle IN d and sets the finalizer on d, the object that owns the handle.
// zero: the all-zero state of `var d sha1digest`; else NewSha1's (sha1.go:48-52).
func (d *sha1digest) open(zero bool) {
	if zero {
		checkWrite(C.efes_sha1_new_zero_pool(pool(), &d.c))
	} else {
		checkWrite(C.efes_sha1_new_pool(pool(), &d.c))
	}
	// The finalizer frees ~400 B of host memory and nothing scarce: a digest holds an upload slot only
	// between a Write and its next sync point, and the library evicts idle holders when the slots run
	// out, so garbage-collector timing never decides whether a Write can proceed.
	runtime.SetFinalizer(d, (*sha1digest).free)
}

func (d *sha1digest) free() { C.efes_sha1_free(d.c); d.c = nil }

// handle opens a zero digest's handle on first use (var d sha1digest; json's new(sha1digest)).
func (d *sha1digest) handle() *C.efes_sha1 {
	if d.c == nil {
		d.open(true)
	}
	return d.c
}

func NewSha1() *sha1digest { d := new(sha1digest); d.open(false); return d }

func (d *sha1digest) Size() int      { return int(C.efes_sha1_size()) }
func (d *sha1digest) BlockSize() int { return int(C.efes_sha1_block_size()) }

// sha1.go:36-44
func (d *sha1digest) Reset() {
	C.efes_sha1_reset(d.handle())
	runtime.KeepAlive(d)
}

// sha1.go:58-79.  p is only read during the call (copied into the pinned staging).  Empty Writes go
// to C too: a pending full x is compressed by them, as in Go.
func (d *sha1digest) Write(p []byte) (int, error) {
	rc := C.efes_sha1_write(d.handle(), cbytes(p), C.size_t(len(p)))
	runtime.KeepAlive(d)
	checkWrite(rc)
	return len(p), nil
}

// sha1.go:82-87: non-destructive, appends.
func (d *sha1digest) Sum(in []byte) []byte {
	var out [20]byte
	rc := C.efes_sha1_sum(d.handle(), (*C.uint8_t)(&out[0]))
	runtime.KeepAlive(d)
	checkSum(rc)
	return append(in, out[:]...)
}

// sha1_efes.go:25-38 -- byte-identical 200 hex chars (stale x bytes included).
func (d *sha1digest) MarshalText() ([]byte, error) {
	out := make([]byte, 200)
	rc := C.efes_sha1_marshal_text(d.handle(), (*C.char)(unsafe.Pointer(&out[0])))
	runtime.KeepAlive(d)
	if rc != C.EFES_OK {
		return nil, fmt.Errorf("efes gpu: %s", C.GoString(C.efes_strerror(rc))) // -> HTTP 500 (filereceiver.go:94-96)
	}
	return out, nil
}

// sha1_efes.go:40-64.  json.Unmarshal calls this on the new(sha1digest) it allocates for a nil
// *sha1digest field (fileinfo.go:43): handle() opens that object's own handle.
func (d *sha1digest) UnmarshalText(text []byte) error {
	rc := C.efes_sha1_unmarshal_text(d.handle(), (*C.char)(cbytes(text)), C.size_t(len(text)))
	runtime.KeepAlive(d)
	if rc != C.EFES_OK {
		return errInvalidDigest
	}
	return nil
}

// ---- crc32digest: crc32.go:48-93 -- same name, same method set ----------------------------------

type crc32digest struct{ c *C.efes_crc32 }

// NewCRC32IEEE's state and a zero crc32digest's are the same (crc 0).
func (d *crc32digest) open() {
	checkWrite(C.efes_crc32_new_pool(pool(), &d.c))
	runtime.SetFinalizer(d, (*crc32digest).free) // host memory only, as above
}

func (d *crc32digest) free() { C.efes_crc32_free(d.c); d.c = nil }

func (d *crc32digest) handle() *C.efes_crc32 {
	if d.c == nil {
		d.open()
	}
	return d.c
}

func NewCRC32IEEE() *crc32digest { d := new(crc32digest); d.open(); return d } // crc32.go:68

func (d *crc32digest) Size() int      { return int(C.efes_crc32_size()) }
func (d *crc32digest) BlockSize() int { return int(C.efes_crc32_block_size()) }

func (d *crc32digest) Reset() { // crc32.go:74
	C.efes_crc32_reset(d.handle())
	runtime.KeepAlive(d)
}

func (d *crc32digest) Write(p []byte) (int, error) { // crc32.go:76-86
	rc := C.efes_crc32_write(d.handle(), cbytes(p), C.size_t(len(p)))
	runtime.KeepAlive(d)
	checkWrite(rc)
	return len(p), nil
}

func (d *crc32digest) Sum32() uint32 { // crc32.go:88
	var v C.uint32_t
	rc := C.efes_crc32_sum32(d.handle(), &v)
	runtime.KeepAlive(d)
	checkSum(rc)
	return uint32(v)
}

func (d *crc32digest) Sum(in []byte) []byte { // crc32.go:90-93
	s := d.Sum32()
	return append(in, byte(s>>24), byte(s>>16), byte(s>>8), byte(s))
}

func (d *crc32digest) MarshalText() ([]byte, error) { // crc32_efes.go:18-24
	out := make([]byte, 8)
	rc := C.efes_crc32_marshal_text(d.handle(), (*C.char)(unsafe.Pointer(&out[0])))
	runtime.KeepAlive(d)
	if rc != C.EFES_OK {
		return nil, fmt.Errorf("efes gpu: %s", C.GoString(C.efes_strerror(rc)))
	}
	return out, nil
}

func (d *crc32digest) UnmarshalText(text []byte) error { // crc32_efes.go:26-40
	rc := C.efes_crc32_unmarshal_text(d.handle(), (*C.char)(cbytes(text)), C.size_t(len(text)))
	runtime.KeepAlive(d)
	if rc != C.EFES_OK {
		return errInvalidDigest
	}
	return nil
}

// ---- /metrics: the digest queues' load (server.go:95-97 serves promhttp.Handler()) --------------

func init() { prometheus.MustRegister(gpuCollector{}) }

type gpuCollector struct{}

var (
	mVisible  = prometheus.NewDesc("efes_gpu_devices_visible", "GPUs the process sees (efes_device_count).", nil, nil)
	mOpened   = prometheus.NewDesc("efes_gpu_devices_opened", "GPUs whose context opened and that hash digests; fewer than visible: see the log.", nil, nil)
	mInFlight = prometheus.NewDesc("efes_gpu_uploads_in_flight",
		"Upload slots held: digests (a fused CRC + SHA-1 pair is one) between a Write and their sync point.", []string{"gpu"}, nil)
	mSlots    = prometheus.NewDesc("efes_gpu_upload_slots", "Upload slots of the GPU's digest queue.", []string{"gpu"}, nil)
	mLaunches = prometheus.NewDesc("efes_gpu_launches_total", "Kernel launches of the GPU's digest queue.", []string{"gpu"}, nil)
	mJobs     = prometheus.NewDesc("efes_gpu_jobs_total", "Upload jobs in those launches.", []string{"gpu"}, nil)
	mBytes    = prometheus.NewDesc("efes_gpu_hashed_bytes_total", "Staged bytes hashed.", []string{"gpu"}, nil)
	mPairs    = prometheus.NewDesc("efes_gpu_fused_pairs_total", "CRC + SHA-1 digests bound to one upload.", nil, nil)
	mFused    = prometheus.NewDesc("efes_gpu_fused_bytes_total", "Bytes staged and hashed once for both digests.", nil, nil)
	mSettles  = prometheus.NewDesc("efes_gpu_pair_settles_total", "Fused pairs split (diverging Writes, evictions).", nil, nil)
)

func (gpuCollector) Describe(ch chan<- *prometheus.Desc) {
	for _, d := range []*prometheus.Desc{mVisible, mOpened, mInFlight, mSlots, mLaunches, mJobs, mBytes, mPairs, mFused, mSettles} {
		ch <- d
	}
}

// Collect reads the library's counters at scrape time (efes_pool_stats: zeros before a GPU's first
// digest Write; efes_pair_stats_get: process-wide).  A scrape never opens the GPUs itself: before the
// first digest (or in a role of the binary that never hashes, e.g. `tracker`) it reports nothing.
func (gpuCollector) Collect(ch chan<- prometheus.Metric) {
	if !gpuReady.Load() {
		return
	}
	ch <- prometheus.MustNewConstMetric(mVisible, prometheus.GaugeValue, float64(gpuVisible))
	ch <- prometheus.MustNewConstMetric(mOpened, prometheus.GaugeValue, float64(len(gpuCtxs)))
	p := gpuPool
	for i := range gpuCtxs {
		var st C.efes_queue_stats
		if C.efes_pool_stats(p, C.uint32_t(i), &st) != C.EFES_OK {
			continue
		}
		g := strconv.Itoa(gpuDevs[i])
		ch <- prometheus.MustNewConstMetric(mInFlight, prometheus.GaugeValue, float64(st.max_uploads-st.free_uploads), g)
		ch <- prometheus.MustNewConstMetric(mSlots, prometheus.GaugeValue, float64(st.max_uploads), g)
		ch <- prometheus.MustNewConstMetric(mLaunches, prometheus.CounterValue, float64(st.launches), g)
		ch <- prometheus.MustNewConstMetric(mJobs, prometheus.CounterValue, float64(st.jobs), g)
		ch <- prometheus.MustNewConstMetric(mBytes, prometheus.CounterValue, float64(st.bytes), g)
	}
	var ps C.efes_pair_stats
	if C.efes_pair_stats_get(&ps) == C.EFES_OK {
		ch <- prometheus.MustNewConstMetric(mPairs, prometheus.CounterValue, float64(ps.pairs))
		ch <- prometheus.MustNewConstMetric(mFused, prometheus.CounterValue, float64(ps.fused_bytes))
		ch <- prometheus.MustNewConstMetric(mSettles, prometheus.CounterValue, float64(ps.settles))
	}
}
