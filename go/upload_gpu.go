//go:build efesgpu

// upload_gpu.go -- optional entry points beside hash_gpu.go for callers that can do better than the
// unchanged digest surface (INTEGRATION.md §4 and §5).  Nothing in the reference calls them; a
// maintainer who wants them uses them from saveFile (filereceiver.go:208-226) or a re-check tool.
//
//   uploadWriter -- one io.MultiWriter(CRC32, Sha1) of filereceiver.go:208 as ONE device-resident
//                   upload (efes_upload_*): since ABI 6 the library already fuses the two digests of
//                   the unchanged surface, so this saves only the host-side pairing check;
//   CRC32Span    -- crc32digest.Write (crc32.go:76-86) of one object already in HBM, segment-parallel
//                   over the whole GPU (efes_crc32_span).

package main

/*
#include "efes_hash.h"
*/
import "C"

import (
	"fmt"
	"io"
	"os"
	"runtime"
	"sync"
	"unsafe"
)

// one MultiWriter(CRC32, Sha1) of filereceiver.go:208 as a single device-resident upload
type uploadWriter struct{ u *C.efes_upload }

var (
	queueOnce sync.Once
	queues    []*C.efes_queue
)

// One queue per GPU that opened (256 KiB staging chunks, up to 4096 uploads in flight each); an upload
// goes to the queue with the most free upload slots.  saveFile closes its writer at the end of every
// PATCH, so the slots bound the requests in flight (4096 per GPU), not the objects alive.
func uploadQueue() *C.efes_queue {
	queueOnce.Do(func() {
		pool()
		for _, c := range gpuCtxs {
			var q *C.efes_queue
			checkSum(C.efes_queue_create(c, 256<<10, 16384, 4096, &q))
			queues = append(queues, q)
		}
	})
	best, most := queues[0], C.uint32_t(0)
	for _, q := range queues {
		var st C.efes_queue_stats
		if C.efes_queue_get_stats(q, &st) == C.EFES_OK && st.free_uploads > most {
			best, most = q, st.free_uploads
		}
	}
	return best
}

// resume from the .info state of a partial upload (fileinfo.go:43-58), or start fresh (nil).  The
// writer owns its upload as a digest owns its handle (hash_gpu.go): allocated in w, finalizer on w,
// KeepAlive after every C call.  saveFile closes it at the end of the PATCH; the finalizer only
// catches a writer a panic left open.
func openUpload(sha *C.efes_sha1_state, crc *C.efes_crc32_state) *uploadWriter {
	w := new(uploadWriter)
	checkSum(C.efes_upload_open(uploadQueue(), C.EFES_HASH_SHA1|C.EFES_HASH_CRC32, sha, crc, &w.u))
	runtime.SetFinalizer(w, (*uploadWriter).Close)
	return w
}

func (w *uploadWriter) Write(p []byte) (int, error) { // staged and returned: hashed by the dispatcher
	rc := C.efes_upload_write(w.u, cbytes(p), C.size_t(len(p)))
	runtime.KeepAlive(w)
	checkSum(rc)
	return len(p), nil
}

func (w *uploadWriter) Sums() (sha1 [20]byte, crc [4]byte) { // filereceiver.go:99-100
	var out [24]byte
	rc := C.efes_upload_sum(w.u, (*C.uint8_t)(&out[0]))
	runtime.KeepAlive(w)
	checkSum(rc)
	copy(sha1[:], out[:20])
	copy(crc[:], out[20:])
	return
}

func (w *uploadWriter) State() (s C.efes_sha1_state, c C.efes_crc32_state) { // for the .info save (:226)
	rc := C.efes_upload_state(w.u, &s, &c)
	runtime.KeepAlive(w)
	checkSum(rc)
	return
}

func (w *uploadWriter) Close() {
	if w.u == nil {
		return
	}
	runtime.SetFinalizer(w, nil)
	C.efes_upload_close(w.u)
	w.u = nil
	runtime.KeepAlive(w)
}

// io.Copy(MultiWriter(f, w), r) with the body read straight into the upload's pinned staging
// (efes_upload_reserve / efes_upload_commit, ABI 3): the file is written from the same buffer, and a
// commit is one Write without the staging copy.  Measured on the C++ mirror, the plain Write above is
// the cheaper of the two on the host (INTEGRATION.md §4).
func (w *uploadWriter) fill(f *os.File, r io.Reader) (n int64, err error) {
	for {
		var p unsafe.Pointer
		var room C.size_t
		rc := C.efes_upload_reserve(w.u, 32<<10, &p, &room)
		runtime.KeepAlive(w)
		checkSum(rc)
		buf := unsafe.Slice((*byte)(p), min(int(room), 32<<10))
		nr, er := r.Read(buf)
		if nr > 0 {
			if _, ew := f.Write(buf[:nr]); ew != nil {
				return n, ew // MultiWriter order: the digests never see this buffer
			}
			rc = C.efes_upload_commit(w.u, C.size_t(nr))
			runtime.KeepAlive(w)
			checkSum(rc)
			n += int64(nr)
		}
		if er != nil {
			return n, nil // io.Copy's EOF / read error, ignored by saveFile (filereceiver.go:209)
		}
	}
}

// CRC32Span is crc32digest.Write of n device bytes at d into the device state st, on all CUs.  d is
// device memory of ctx's GPU (efes_device_alloc) holding the object, st a 4-byte device state.  One
// object over several GPUs: each GPU spans its piece from a zero state, then efes_crc32_combine of the
// 4-byte results in piece order.
func CRC32Span(ctx *C.efes_ctx, d unsafe.Pointer, n uint64, st *C.efes_crc32_state) error {
	if rc := C.efes_crc32_span(ctx, d, C.uint64_t(n), st, nil); rc != 0 {
		return fmt.Errorf("efes gpu: %s", C.GoString(C.efes_strerror(rc)))
	}
	return nil
}
