// efes_receiver.hpp -- the upload receiver of efes (the caller of the hashing path) restated in
// C++ above the C ABI of include/efes_hash.h.
//
// The reference is Go (no Go toolchain in this image), so the host side that a maintainer would
// keep in Go is mirrored here in C++, name for name, with the same argument meaning and the same
// error behaviour, so that the reference's own tests (filereceiver_test.go, sha1file_test.go,
// client_test.go's upload) can be replayed against it (tests/cpp/receiver_test.cpp):
//
//   fileinfo.go:10-62       FileInfo / Digest, the `<path>.info` JSON (json.Encoder / Decoder)
//   filereceiver.go:42-127  FileReceiver.ServeHTTP (POST / HEAD / PATCH / DELETE; no socket, no DB:
//                           the handler logic with db == nil, as filereceiver_test.go runs it)
//   filereceiver.go:148-236 createFile, deleteFile, saveFile, OffsetMismatchError
//   sha1file.go:9-53        Sha1File (hash-while-reading with crop-on-retry)
//   write.go:68-195         sendFile: the client side (PATCH per ChunkSize, HEAD + seek back on
//                           failure, local vs remote SHA-1), over a Transport
//
// Every byte is hashed on the GPU: saveFile streams the body through ONE upload of a batching
// queue (efes_upload_*, hashes SHA-1 | CRC-32) -- the MultiWriter(f, CRC32, Sha1) of
// filereceiver.go:208 with both digests fused into one pass -- so concurrent requests share
// kernel launches.  Sha1File uses the streaming sha1digest objects (efes_sha1_*).
//
// Go `error` values become efes::Error (code 0 = nil).  Where Go panics (a nil digest decoded
// from JSON null, a sha1digest state with nx > 64) the mirror returns an error instead.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <condition_variable>
#include <map>
#include <mutex>
#include <string>
#include <string_view>
#include <vector>

#include "efes_hash.h"

namespace efes {

// Host error codes beside the library's EFES_ERR_* (which keep their values).
enum : int {
  ERR_IO = -100,              // an os / syscall error (msg: "op path: errno text", as Go's *PathError)
  ERR_NOT_EXIST = -101,       // os.IsNotExist(err)
  ERR_OFFSET_MISMATCH = -102, // *OffsetMismatchError (filereceiver.go:229-236)
  ERR_JSON = -103,            // encoding/json syntax / type error
  ERR_EOF = -104,             // io.EOF
  ERR_NIL_DIGEST = -105,      // a null / missing digest in the .info JSON (Go: nil pointer, panics on Write)
  ERR_SHA1FILE = -106,        // sha1file.go:25 "missing data for sha1", :45 "seeking forward is not supported"
  ERR_SYNTAX = -107,          // strconv.ParseInt
  ERR_HTTP = -108,            // a non-2xx response (httperror.go: ServerError / ClientError / HTTPError)
  ERR_TRANSPORT = -109,       // the request did not complete (connection error)
  ERR_SHA1_MISMATCH = -110,   // write.go:112-115 local vs remote SHA-1
};

struct Error {
  int code = 0;
  std::string msg;
  int64_t given = 0, required = 0;  // ERR_OFFSET_MISMATCH only
  int status = 0;                   // ERR_HTTP: the response's status code
  explicit operator bool() const { return code != 0; }
  const std::string& str() const { return msg; }  // Go's err.Error()
};

Error make_error(int code, std::string msg);
Error errno_error(const char* op, const std::string& path, int err);  // *os.PathError
Error lib_error(int rc);                                             // an efes_* return code

// ---- io ----------------------------------------------------------------------------------------
// io.Reader: returns n (0 <= n <= cap) and sets *err (ERR_EOF at the end of the stream).
struct Reader {
  virtual ~Reader() = default;
  virtual size_t Read(uint8_t* p, size_t cap, Error* err) = 0;
};
// io.ReadSeeker (whence: 0 SeekStart, 1 SeekCurrent, 2 SeekEnd).
struct ReadSeeker : Reader {
  virtual int64_t Seek(int64_t offset, int whence, Error* err) = 0;
};
// bytes.NewBufferString / strings.Reader over a copy of `data`; `max_read` caps each Read (as a
// socket delivers at most what has arrived).
class BytesReader : public ReadSeeker {
 public:
  explicit BytesReader(std::string data, size_t max_read = SIZE_MAX) : d_(std::move(data)), max_(max_read) {}
  size_t Read(uint8_t* p, size_t cap, Error* err) override;
  int64_t Seek(int64_t offset, int whence, Error* err) override;

 private:
  std::string d_;
  size_t pos_ = 0, max_;
};
// An *os.File opened read-only.
class FileReader : public ReadSeeker {
 public:
  static Error Open(const std::string& path, FileReader** out);
  ~FileReader() override;
  size_t Read(uint8_t* p, size_t cap, Error* err) override;
  int64_t Seek(int64_t offset, int whence, Error* err) override;

 private:
  int fd_ = -1;
  std::string path_;
};

// ---- fileinfo.go -------------------------------------------------------------------------------
// FileInfo{Offset, Digest{Sha1 *sha1digest, CRC32 *crc32digest}} (fileinfo.go:10-18); the
// digests are held as plain states (nil pointers as has_* = false).
struct FileInfo {
  int64_t Offset = 0;
  efes_sha1_state Sha1{};
  efes_crc32_state CRC32{};
  bool has_sha1 = false, has_crc32 = false;
};
FileInfo newFileInfo();                                      // fileinfo.go:20-27 (NewSha1, NewCRC32IEEE)
std::string EncodeFileInfo(const FileInfo& fi);              // json.NewEncoder(f).Encode(fi) incl. '\n'
Error DecodeFileInfo(std::string_view text, FileInfo* fi);   // json.NewDecoder(f).Decode(&fi)
Error ReadFileInfo(const std::string& path, FileInfo* fi);   // fileinfo.go:29-35
Error ReadExistingFileInfo(const std::string& path, FileInfo* fi);  // fileinfo.go:37-45
Error SaveFileInfo(const std::string& path, const FileInfo& fi);    // fileinfo.go:47-58
Error DeleteFileInfo(const std::string& path);                      // fileinfo.go:60-62
extern const char* const fileInfoExt;                               // ".info" (fileinfo.go:8)

// ---- filereceiver.go ---------------------------------------------------------------------------
// The digests a finished upload reports (filereceiver.go:98-101): Sha1.Sum(nil), CRC32.Sum(nil).
struct DigestSums {
  uint8_t sha1[20];
  uint8_t crc32[4];
};

// A hashing backend for saveFile: one batching queue per GPU, shared by every request of the
// process (the role of the per-request digests of the reference, batched).  Each PATCH is hashed
// on the device with the most free request slots (the state travels through the .info file
// between PATCHes, so consecutive PATCHes of one upload may use different GPUs); max_uploads
// bounds the requests hashed at once per device, further requests wait for a slot.
class Hasher {
 public:
  static Error Create(efes_ctx* ctx, uint64_t chunk_bytes, uint32_t max_chunks, uint32_t max_uploads, Hasher** out);
  static Error Create(const std::vector<efes_ctx*>& ctxs, uint64_t chunk_bytes, uint32_t max_chunks,
                      uint32_t max_uploads, Hasher** out);  // one queue per context (GPU)
  ~Hasher();
  size_t devices() const { return q_.size(); }
  efes_queue* queue(size_t d = 0) const { return q_[d]; }
  size_t acquire();          // a request slot on the least-loaded device (blocks while all are busy)
  void release(size_t d);
  uint64_t served(size_t d) const;  // requests hashed on device d so far

 private:
  std::vector<efes_queue*> q_;
  std::vector<uint32_t> free_;
  std::vector<uint64_t> served_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
};

Error createFile(const std::string& path);                 // filereceiver.go:148-165
Error deleteFile(const std::string& path);                 // filereceiver.go:167-169
// filereceiver.go:171-227: returns the new offset; *done (with *sums) when offset == length.
// h == nullptr (no GPU context): every request that gets as far as hashing fails.
Error saveFile(Hasher* h, const std::string& path, int64_t offset, int64_t length, Reader& r,
               int64_t* new_offset, bool* done, DigestSums* sums);
std::string OffsetMismatchText(int64_t given, int64_t required);  // OffsetMismatchError.Error()

// Host CPU accounting of saveFile by phase (tools/bench_receiver, EnableSavePhases): the
// request threads' CPU nanoseconds (CLOCK_THREAD_CPUTIME_ID) summed over every request, per
// phase.  Off by default (one branch per phase); when on, one clock read and one relaxed atomic
// add per phase.
enum SavePhase {
  kPhaseCreate,   // createFile: os.Create + Close + the newFileInfo .info (filereceiver.go:148-165)
  kPhaseOpen,     // ReadFileInfo / OpenFile / Seek / upload slot + efes_upload_open
  kPhaseReserve,  // efes_upload_reserve (waits for a staging chunk, hands full ones over)
  kPhaseRead,     // r.Read into the staging buffer (the socket's copy)
  kPhaseWrite,    // write(2) of the buffer to the file
  kPhaseCommit,   // efes_upload_commit (Go's x/nx/len replay; hands a full chunk over)
  kPhaseSync,     // f.Sync() + Close
  kPhaseSum,      // efes_upload_sum / efes_upload_state: waiting for this upload's GPU jobs
  kPhaseInfo,     // DeleteFileInfo / SaveFileInfo at the end
  kPhases
};
void EnableSavePhases(bool on, bool wall_clock = false);  // wall_clock: CLOCK_MONOTONIC instead
// saveFile's body copy: io.Copy's 32 KiB buffer then efes_upload_write (true, the default and the
// cheaper on the host), or the body read straight into the upload's pinned staging
// (efes_upload_reserve / efes_upload_commit).  Process-wide; set it before serving requests.
void SetSaveFileCopyBuffer(bool on);
void SavePhaseTotals(uint64_t ns[kPhases]);
const char* SavePhaseName(int p);

// strconv.ParseInt(s, 10, 64)
Error ParseInt(std::string_view s, int64_t* out);
// filepath.Join(dir, p) (Clean of the joined path)
std::string JoinPath(const std::string& dir, const std::string& p);

// net/http request / response of the handler, without a socket.  Header names are
// case-insensitive (http.Header canonicalises them).
struct HeaderLess {
  bool operator()(const std::string& a, const std::string& b) const;
};
using Header = std::map<std::string, std::string, HeaderLess>;
struct Request {
  std::string Method, Path;
  Header Headers;
  Reader* Body = nullptr;  // nil body = empty
};
struct Response {
  int Code = 200;
  Header Headers;
  std::string Body;
};

// filereceiver.go:19-127 with db == nil (tempfileExists is true, filereceiver.go:130-132).
class FileReceiver {
 public:
  FileReceiver(std::string dir, Hasher* h) : dir_(std::move(dir)), h_(h) {}
  Response ServeHTTP(const Request& r);

 private:
  std::string dir_;
  Hasher* h_;
};

// ---- write.go: the client side of an upload (Client.sendFile) --------------------------------
struct Checksums {  // write.go:63-66
  std::string Sha1, CRC32;
};
// http.Client.Do: one request/response; *err set when the request did not complete.
struct Transport {
  virtual ~Transport() = default;
  virtual Response RoundTrip(const Request& r, Error* err) = 0;
};
// Requests to a FileReceiver of this process (no socket).
struct LocalTransport : Transport {
  explicit LocalTransport(FileReceiver* fr) : fr_(fr) {}
  Response RoundTrip(const Request& r, Error* err) override;

 private:
  FileReceiver* fr_;
};
struct ClientConfig {
  int64_t ChunkSize = 50ll << 20;  // config.go:80 Client.ChunkSize (50M); one PATCH per chunk (write.go:126)
  int MaxAttempts = 10;            // backoff.Retry's attempts (its sleeps are not modelled)
  bool Drainer = false;            // client.go:21: the drainer's client adds efes-drain: true (write.go:163-165)
};
// write.go:68-117 sendFile with send (120-144), patch (154-172), getOffset (174-185) and finishFile
// (188-195): the file read through Sha1File (hashed on the GPU while it is sent), one PATCH per
// ChunkSize, on failure HEAD the server's offset, seek back and resend (Sha1File hashes each
// byte once), then compare the local SHA-1 with the server's efes-file-sha1 header.
Error sendFile(Transport& t, efes_ctx* ctx, const std::string& path, ReadSeeker& rs, int64_t size,
               const ClientConfig& cfg, Checksums* out);

// ---- sha1file.go -------------------------------------------------------------------------------
class Sha1File : public ReadSeeker {
 public:
  static Error New(ReadSeeker* rs, efes_ctx* ctx, Sha1File** out);  // sha1file.go:16-21
  ~Sha1File() override;
  size_t Read(uint8_t* p, size_t cap, Error* err) override;         // sha1file.go:23-37
  int64_t Seek(int64_t offset, int whence, Error* err) override;    // sha1file.go:39-49
  Error Sum(uint8_t out[20]);                                       // sha1file.go:51-53

 private:
  ReadSeeker* rs_ = nullptr;
  int64_t position_ = 0, calculated_ = 0;
  efes_sha1* digest_ = nullptr;
  int latched_ = 0;  // a failed digest Write (Go's Write cannot fail): reported by Sum
};

std::string HexEncode(const uint8_t* p, size_t n);  // hex.EncodeToString

}  // namespace efes
