// efes_receiver.cpp -- see efes_receiver.hpp.  The C++ restatement of the Go code that calls the
// hashing path: fileinfo.go, filereceiver.go, sha1file.go (file:line cited per function).
#include "efes_receiver.hpp"

#include <errno.h>
#include <strings.h>
#include <fcntl.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <vector>

namespace efes {

const char* const fileInfoExt = ".info";  // fileinfo.go:8

// ---- errors ------------------------------------------------------------------------------------
Error make_error(int code, std::string msg) {
  Error e;
  e.code = code;
  e.msg = std::move(msg);
  return e;
}

Error errno_error(const char* op, const std::string& path, int err) {
  // *os.PathError: "op path: text", the syscall text lower-case as Go prints it
  std::string t = strerror(err);
  if (!t.empty() && t[0] >= 'A' && t[0] <= 'Z') t[0] = (char)(t[0] - 'A' + 'a');
  return make_error(err == ENOENT ? ERR_NOT_EXIST : ERR_IO, std::string(op) + " " + path + ": " + t);
}

Error lib_error(int rc) { return rc ? make_error(rc, efes_strerror(rc)) : Error{}; }

std::string HexEncode(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    s[2 * i] = d[p[i] >> 4];
    s[2 * i + 1] = d[p[i] & 15];
  }
  return s;
}

// ---- io ----------------------------------------------------------------------------------------
size_t BytesReader::Read(uint8_t* p, size_t cap, Error* err) {  // bytes.Buffer / strings.Reader
  *err = Error{};
  if (cap == 0) return 0;
  if (pos_ >= d_.size()) {
    *err = make_error(ERR_EOF, "EOF");
    return 0;
  }
  size_t n = std::min(std::min(cap, max_), d_.size() - pos_);
  memcpy(p, d_.data() + pos_, n);
  pos_ += n;
  return n;
}

int64_t BytesReader::Seek(int64_t offset, int whence, Error* err) {  // strings.Reader.Seek
  *err = Error{};
  int64_t abs;
  switch (whence) {
    case 0: abs = offset; break;
    case 1: abs = (int64_t)pos_ + offset; break;
    case 2: abs = (int64_t)d_.size() + offset; break;
    default: *err = make_error(ERR_IO, "strings.Reader.Seek: invalid whence"); return 0;
  }
  if (abs < 0) {
    *err = make_error(ERR_IO, "strings.Reader.Seek: negative position");
    return 0;
  }
  pos_ = (size_t)abs;
  return abs;
}

Error FileReader::Open(const std::string& path, FileReader** out) {  // os.Open
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return errno_error("open", path, errno);
  FileReader* f = new FileReader;
  f->fd_ = fd;
  f->path_ = path;
  *out = f;
  return Error{};
}

FileReader::~FileReader() {
  if (fd_ >= 0) ::close(fd_);
}

size_t FileReader::Read(uint8_t* p, size_t cap, Error* err) {  // (*os.File).Read
  *err = Error{};
  if (cap == 0) return 0;
  for (;;) {
    const ssize_t n = ::read(fd_, p, cap);
    if (n > 0) return (size_t)n;
    if (n == 0) {
      *err = make_error(ERR_EOF, "EOF");
      return 0;
    }
    if (errno != EINTR) {
      *err = errno_error("read", path_, errno);
      return 0;
    }
  }
}

int64_t FileReader::Seek(int64_t offset, int whence, Error* err) {  // (*os.File).Seek
  *err = Error{};
  const off_t r = ::lseek(fd_, (off_t)offset, whence);
  if (r < 0) {
    *err = errno_error("seek", path_, errno);
    return 0;
  }
  return (int64_t)r;
}

namespace {

Error write_full(int fd, const std::string& path, const uint8_t* p, size_t n, size_t* done) {  // (*os.File).Write
  *done = 0;
  while (*done < n) {
    const ssize_t w = ::write(fd, p + *done, n - *done);
    if (w < 0) {
      if (errno == EINTR) continue;
      return errno_error("write", path, errno);
    }
    *done += (size_t)w;
  }
  return Error{};
}

Error read_all(const std::string& path, std::string* out) {
  FileReader* f = nullptr;
  Error e = FileReader::Open(path, &f);
  if (e) return e;
  std::unique_ptr<FileReader> g(f);
  out->clear();
  uint8_t buf[4096];
  for (;;) {
    const size_t n = f->Read(buf, sizeof buf, &e);
    out->append(reinterpret_cast<char*>(buf), n);
    if (e.code == ERR_EOF) return Error{};
    if (e) return e;
  }
}

Error create_write(const std::string& path, const std::string& data) {  // os.Create + Write + Close
  const int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
  if (fd < 0) return errno_error("open", path, errno);
  size_t done;
  Error e = write_full(fd, path, reinterpret_cast<const uint8_t*>(data.data()), data.size(), &done);
  if (::close(fd) != 0 && !e) e = errno_error("close", path, errno);
  return e;
}

Error remove_path(const std::string& path) {  // os.Remove: unlink, else rmdir (os/file_unix.go)
  if (::unlink(path.c_str()) == 0) return Error{};
  int e = errno;
  if (::rmdir(path.c_str()) == 0) return Error{};
  if (errno != ENOTDIR) e = errno;
  return errno_error("remove", path, e);
}

Error mkdir_all(const std::string& path, mode_t mode) {  // os.MkdirAll
  struct stat st;
  if (::stat(path.c_str(), &st) == 0) {
    if (S_ISDIR(st.st_mode)) return Error{};
    return errno_error("mkdir", path, ENOTDIR);
  }
  const size_t slash = path.find_last_of('/');
  if (slash != std::string::npos && slash > 0) {
    Error e = mkdir_all(path.substr(0, slash), mode);
    if (e) return e;
  }
  if (::mkdir(path.c_str(), mode) != 0) {
    const int err = errno;
    if (::stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) return Error{};
    return errno_error("mkdir", path, err);
  }
  return Error{};
}

// ---- encoding/json, restricted to the FileInfo document ---------------------------------------
// json.Decoder.Decode(&fi) into a nil *FileInfo: the first JSON value of the stream; object
// keys match struct fields exactly or ASCII case-insensitively; unknown keys are skipped;
// a JSON null leaves a value unchanged (a pointer: nil); a TextUnmarshaler gets the unquoted
// string.  Nesting is limited like Go's (10000).
struct Json {
  std::string_view s;
  size_t i = 0;
  Error err;      // first syntax error (ends decoding)
  Error type_err; // first type / UnmarshalText error (Go keeps decoding, then returns it)

  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  bool syntax(const std::string& what) {
    if (!err) err = make_error(i >= s.size() ? ERR_EOF : ERR_JSON, i >= s.size() ? "unexpected EOF" : "invalid character in JSON: " + what);
    return false;
  }
  void type_error(const std::string& what) {
    if (!type_err) type_err = make_error(ERR_JSON, "json: cannot unmarshal " + what);
  }
  static int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  static void utf8(std::string* out, uint32_t cp) {
    if (cp < 0x80) {
      out->push_back((char)cp);
    } else if (cp < 0x800) {
      out->push_back((char)(0xC0 | (cp >> 6)));
      out->push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out->push_back((char)(0xE0 | (cp >> 12)));
      out->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      out->push_back((char)(0xF0 | (cp >> 18)));
      out->push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      out->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  bool u4(uint32_t* v) {
    if (i + 4 > s.size()) return syntax("short \\u escape");
    *v = 0;
    for (int k = 0; k < 4; ++k) {
      const int h = hexval(s[i + k]);
      if (h < 0) return syntax("in \\u hexadecimal character escape");
      *v = *v << 4 | (uint32_t)h;
    }
    i += 4;
    return true;
  }
  bool str(std::string* out) {  // s[i] == '"'
    ++i;
    out->clear();
    while (i < s.size()) {
      const unsigned char c = (unsigned char)s[i];
      if (c == '"') {
        ++i;
        return true;
      }
      if (c < 0x20) return syntax("control character in string literal");
      if (c != '\\') {
        out->push_back((char)c);
        ++i;
        continue;
      }
      if (++i >= s.size()) break;
      const char e = s[i++];
      switch (e) {
        case '"': case '\\': case '/': out->push_back(e); break;
        case 'b': out->push_back('\b'); break;
        case 'f': out->push_back('\f'); break;
        case 'n': out->push_back('\n'); break;
        case 'r': out->push_back('\r'); break;
        case 't': out->push_back('\t'); break;
        case 'u': {
          uint32_t v = 0;
          if (!u4(&v)) return false;
          if (v >= 0xD800 && v < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
            const size_t save = i;
            i += 2;
            uint32_t lo = 0;
            if (!u4(&lo)) return false;
            if (lo >= 0xDC00 && lo < 0xE000) {
              v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
            } else {
              i = save;
              v = 0xFFFD;
            }
          } else if (v >= 0xD800 && v < 0xE000) {
            v = 0xFFFD;
          }
          utf8(out, v);
          break;
        }
        default: --i; return syntax("in string escape code");
      }
    }
    return syntax("unterminated string");
  }
  bool lit(const char* w) {
    const size_t n = strlen(w);
    if (s.substr(i, n) != std::string_view(w, n)) return syntax("in literal");
    i += n;
    return true;
  }
  bool num(std::string_view* out) {  // -?(0|[1-9]d*)(.d+)?([eE][+-]?d+)?
    const size_t b = i;
    if (i < s.size() && s[i] == '-') ++i;
    if (i >= s.size()) return syntax("in numeric literal");
    if (s[i] == '0') {
      ++i;
    } else if (s[i] >= '1' && s[i] <= '9') {
      while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
    } else {
      return syntax("in numeric literal");
    }
    if (i < s.size() && s[i] == '.') {
      ++i;
      if (i >= s.size() || s[i] < '0' || s[i] > '9') return syntax("after decimal point in numeric literal");
      while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
    }
    if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
      ++i;
      if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
      if (i >= s.size() || s[i] < '0' || s[i] > '9') return syntax("in exponent of numeric literal");
      while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
    }
    *out = s.substr(b, i - b);
    return true;
  }
  // Any value, discarded.
  bool skip(int depth) {
    if (depth > 10000) return syntax("exceeded max depth");
    ws();
    if (i >= s.size()) return syntax("");
    const char c = s[i];
    if (c == '"') {
      std::string t;
      return str(&t);
    }
    if (c == '{' || c == '[') {
      const char close = c == '{' ? '}' : ']';
      ++i;
      ws();
      if (i < s.size() && s[i] == close) {
        ++i;
        return true;
      }
      for (;;) {
        if (c == '{') {
          ws();
          if (i >= s.size() || s[i] != '"') return syntax("looking for beginning of object key string");
          std::string k;
          if (!str(&k)) return false;
          ws();
          if (i >= s.size() || s[i] != ':') return syntax("after object key");
          ++i;
        }
        if (!skip(depth + 1)) return false;
        ws();
        if (i >= s.size()) return syntax("");
        if (s[i] == ',') {
          ++i;
          continue;
        }
        if (s[i] == close) {
          ++i;
          return true;
        }
        return syntax(c == '{' ? "after object key:value pair" : "after array element");
      }
    }
    if (c == 't') return lit("true");
    if (c == 'f') return lit("false");
    if (c == 'n') return lit("null");
    std::string_view n;
    return num(&n);
  }
  static const char* kind(char c) {
    switch (c) {
      case '"': return "string";
      case '{': return "object";
      case '[': return "array";
      case 't': case 'f': return "bool";
      default: return "number";
    }
  }
  static bool key_is(const std::string& k, const char* field) {  // exact, then ASCII case fold
    const size_t n = strlen(field);
    if (k.size() != n) return false;
    for (size_t j = 0; j < n; ++j) {
      char a = k[j], b = field[j];
      if (a >= 'A' && a <= 'Z') a = (char)(a - 'A' + 'a');
      if (b >= 'A' && b <= 'Z') b = (char)(b - 'A' + 'a');
      if (a != b) return false;
    }
    return true;
  }
  // Iterates an object's members: f(key) parses or skips the value.
  template <class F>
  bool object(int depth, F&& f) {  // s[i] == '{'
    if (depth > 10000) return syntax("exceeded max depth");
    ++i;
    ws();
    if (i < s.size() && s[i] == '}') {
      ++i;
      return true;
    }
    for (;;) {
      ws();
      if (i >= s.size() || s[i] != '"') return syntax("looking for beginning of object key string");
      std::string k;
      if (!str(&k)) return false;
      ws();
      if (i >= s.size() || s[i] != ':') return syntax("after object key");
      ++i;
      ws();
      if (i >= s.size()) return syntax("");
      if (!f(k)) return false;
      ws();
      if (i >= s.size()) return syntax("");
      if (s[i] == ',') {
        ++i;
        continue;
      }
      if (s[i] == '}') {
        ++i;
        return true;
      }
      return syntax("after object key:value pair");
    }
  }
  // A *sha1digest / *crc32digest field (TextUnmarshaler behind a pointer).
  template <class U>
  bool text_field(int depth, const char* go_type, bool* has, U&& unmarshal) {
    const char c = s[i];
    if (c == 'n') {
      if (!lit("null")) return false;
      *has = false;  // null into a pointer: nil
      return true;
    }
    if (c == '"') {
      std::string t;
      if (!str(&t)) return false;
      *has = true;  // a new zero digest, then UnmarshalText (encoding/json literalStore)
      const int rc = unmarshal(t);
      if (rc && !type_err) type_err = make_error(rc, efes_strerror(rc));
      return true;
    }
    type_error(std::string(kind(c)) + " into Go value of type " + go_type);
    return skip(depth);
  }
};

}  // namespace

// ---- fileinfo.go -------------------------------------------------------------------------------
FileInfo newFileInfo() {  // fileinfo.go:20-27
  FileInfo fi;
  fi.Offset = 0;
  memset(&fi.Sha1, 0, sizeof fi.Sha1);
  efes_sha1_state_init(&fi.Sha1);  // NewSha1 (sha1.go:48-52)
  fi.CRC32.crc = 0;                // NewCRC32IEEE (crc32.go:68)
  fi.has_sha1 = fi.has_crc32 = true;
  return fi;
}

std::string EncodeFileInfo(const FileInfo& fi) {  // fileinfo.go:53 json.NewEncoder(f).Encode(fi)
  std::string out = "{\"offset\":" + std::to_string(fi.Offset) + ",\"digest\":{\"sha1\":";
  if (fi.has_sha1) {
    char t[200];
    efes_sha1_state_marshal_text(&fi.Sha1, t);  // sha1_efes.go:25-38
    out += '"';
    out.append(t, 200);
    out += '"';
  } else {
    out += "null";
  }
  out += ",\"crc32\":";
  if (fi.has_crc32) {
    char t[8];
    efes_crc32_state_marshal_text(&fi.CRC32, t);  // crc32_efes.go:18-24
    out += '"';
    out.append(t, 8);
    out += '"';
  } else {
    out += "null";
  }
  out += "}}\n";  // Encode terminates each value with a newline
  return out;
}

Error DecodeFileInfo(std::string_view text, FileInfo* fi) {  // fileinfo.go:43 json.NewDecoder(f).Decode(&fi)
  Json j;
  j.s = text;
  j.ws();
  if (j.i >= text.size()) return make_error(ERR_EOF, "EOF");  // an empty stream: io.EOF
  FileInfo r;  // a new FileInfo: Offset 0, nil digests
  const char c = text[j.i];
  if (c == 'n') {
    if (!j.lit("null")) return j.err;
    // `var fi *FileInfo` stays nil; every caller would then dereference it (Go panics).
    return make_error(ERR_NIL_DIGEST, "null file info");
  }
  if (c != '{') {
    if (!j.skip(0)) return j.err;
    return make_error(ERR_JSON, std::string("json: cannot unmarshal ") + Json::kind(c) + " into Go value of type main.FileInfo");
  }
  const bool ok = j.object(1, [&](const std::string& k) {
    const char v = text[j.i];
    if (Json::key_is(k, "offset")) {
      if (v == 'n') return j.lit("null");  // null leaves Offset unchanged
      if (v == '"' || v == '{' || v == '[' || v == 't' || v == 'f') {
        j.type_error(std::string(Json::kind(v)) + " into Go struct field FileInfo.offset of type int64");
        return j.skip(1);
      }
      std::string_view n;
      if (!j.num(&n)) return false;
      int64_t x;
      if (ParseInt(n, &x)) {  // 3.0, 1e3, out of range: UnmarshalTypeError
        j.type_error("number " + std::string(n) + " into Go struct field FileInfo.offset of type int64");
      } else {
        r.Offset = x;
      }
      return true;
    }
    if (Json::key_is(k, "digest")) {
      if (v == 'n') return j.lit("null");  // a struct: unchanged
      if (v != '{') {
        j.type_error(std::string(Json::kind(v)) + " into Go struct field FileInfo.digest of type main.Digest");
        return j.skip(1);
      }
      return j.object(2, [&](const std::string& dk) {
        if (Json::key_is(dk, "sha1"))
          return j.text_field(3, "*main.sha1digest", &r.has_sha1, [&](const std::string& t) {
            memset(&r.Sha1, 0, sizeof r.Sha1);
            return efes_sha1_state_unmarshal_text(&r.Sha1, t.data(), t.size());  // sha1_efes.go:40-64
          });
        if (Json::key_is(dk, "crc32"))
          return j.text_field(3, "*main.crc32digest", &r.has_crc32, [&](const std::string& t) {
            r.CRC32.crc = 0;
            return efes_crc32_state_unmarshal_text(&r.CRC32, t.data(), t.size());  // crc32_efes.go:26-40
          });
        return j.skip(3);
      });
    }
    return j.skip(1);
  });
  if (!ok) return j.err;
  if (j.type_err) return j.type_err;
  *fi = r;
  return Error{};
}

Error ReadExistingFileInfo(const std::string& path, FileInfo* fi) {  // fileinfo.go:37-45
  std::string text;
  Error e = read_all(path + fileInfoExt, &text);
  if (e) return e;
  return DecodeFileInfo(text, fi);
}

Error ReadFileInfo(const std::string& path, FileInfo* fi) {  // fileinfo.go:29-35
  Error e = ReadExistingFileInfo(path, fi);
  if (e.code == ERR_NOT_EXIST) {
    *fi = newFileInfo();
    return Error{};
  }
  return e;
}

Error SaveFileInfo(const std::string& path, const FileInfo& fi) {  // fileinfo.go:47-58
  return create_write(path + fileInfoExt, EncodeFileInfo(fi));
}

Error DeleteFileInfo(const std::string& path) { return remove_path(path + fileInfoExt); }  // fileinfo.go:60-62

// ---- filereceiver.go ---------------------------------------------------------------------------
Error Hasher::Create(efes_ctx* ctx, uint64_t chunk_bytes, uint32_t max_chunks, uint32_t max_uploads, Hasher** out) {
  return Create(std::vector<efes_ctx*>{ctx}, chunk_bytes, max_chunks, max_uploads, out);
}

Error Hasher::Create(const std::vector<efes_ctx*>& ctxs, uint64_t chunk_bytes, uint32_t max_chunks,
                     uint32_t max_uploads, Hasher** out) {
  if (ctxs.empty()) return lib_error(EFES_ERR_ARG);
  std::unique_ptr<Hasher> h(new Hasher);
  for (efes_ctx* ctx : ctxs) {
    efes_queue* q = nullptr;
    const int rc = efes_queue_create(ctx, chunk_bytes, max_chunks, max_uploads, &q);
    if (rc) return lib_error(rc);  // ~Hasher destroys the queues made so far
    h->q_.push_back(q);
    h->free_.push_back(max_uploads);
    h->served_.push_back(0);
  }
  *out = h.release();
  return Error{};
}

Hasher::~Hasher() {
  for (efes_queue* q : q_) efes_queue_destroy(q);
}

size_t Hasher::acquire() {
  std::unique_lock<std::mutex> lk(mu_);
  size_t best = 0;
  cv_.wait(lk, [&] {
    for (size_t d = 0; d < free_.size(); ++d)  // most free slots; ties: the device that served fewer
      if (free_[d] > free_[best] || (free_[d] == free_[best] && served_[d] < served_[best])) best = d;
    return free_[best] > 0;
  });
  --free_[best];
  ++served_[best];
  return best;
}

void Hasher::release(size_t d) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    ++free_[d];
  }
  cv_.notify_one();
}

uint64_t Hasher::served(size_t d) const {
  std::lock_guard<std::mutex> lk(mu_);
  return served_[d];
}

std::string OffsetMismatchText(int64_t given, int64_t required) {  // filereceiver.go:234-236
  return "given offset (" + std::to_string(given) + ") does not match required offset (" + std::to_string(required) + ")";
}

static Error offset_mismatch(int64_t given, int64_t required) {  // &OffsetMismatchError{Given, Required}
  Error e = make_error(ERR_OFFSET_MISMATCH, OffsetMismatchText(given, required));
  e.given = given;
  e.required = required;
  return e;
}

Error createFile(const std::string& path) {  // filereceiver.go:148-165
  int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);  // os.Create
  if (fd < 0 && errno == ENOENT) {
    const size_t slash = path.find_last_of('/');
    Error e = mkdir_all(slash == std::string::npos ? std::string(".") : path.substr(0, slash ? slash : 1), 0700);
    if (e) return e;
    fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
  }
  if (fd < 0) return errno_error("open", path, errno);
  if (::close(fd) != 0) return errno_error("close", path, errno);
  return SaveFileInfo(path, newFileInfo());
}

Error deleteFile(const std::string& path) { return remove_path(path); }  // filereceiver.go:167-169

namespace {
// One request's slot in the Hasher and its fused (SHA-1, CRC-32) upload, released on every path.
struct UploadGuard {
  Hasher& h;
  efes_upload* u = nullptr;
  size_t dev = 0;
  bool held = false;
  explicit UploadGuard(Hasher& hh) : h(hh) {}
  ~UploadGuard() {
    if (u) efes_upload_close(u);
    if (held) h.release(dev);
  }
};
struct FdGuard {
  int fd = -1;
  ~FdGuard() {
    if (fd >= 0) ::close(fd);  // logCloseFile (filereceiver.go:198-203)
  }
};
}  // namespace

namespace {
std::atomic<bool> g_phases_on{false};
std::atomic<clockid_t> g_phase_clock{CLOCK_THREAD_CPUTIME_ID};
std::atomic<uint64_t> g_phase_ns[kPhases];
const char* const kPhaseNames[kPhases] = {"create", "open", "reserve", "read", "write", "commit", "sync", "sum",
                                          "info"};

// Charges the calling thread's CPU time (user + system) since the last mark to a phase (when
// enabled): with hundreds of request threads on 16 cores, wall time per phase would mostly be
// run-queue waits.
// EnableSavePhases(on, wall_clock = true) charges wall time instead (where a request WAITS: run
// queue, locks, pacing, its GPU chain).
uint64_t phase_ns() {
  struct timespec ts;
  clock_gettime(g_phase_clock.load(std::memory_order_relaxed), &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
// saveFile's copy path: io.Copy's own buffer + efes_upload_write (default), or the body read straight
// into the upload's pinned staging (efes_upload_reserve / commit).
std::atomic<bool> g_copy_buffer{true};

struct PhaseClock {
  bool on = g_phases_on.load(std::memory_order_relaxed);
  uint64_t t = on ? phase_ns() : 0;
  void mark(SavePhase p) {
    if (!on) return;
    const uint64_t now = phase_ns();
    g_phase_ns[p].fetch_add(now - t, std::memory_order_relaxed);
    t = now;
  }
};
}  // namespace

void EnableSavePhases(bool on, bool wall_clock) {
  g_phase_clock.store(wall_clock ? CLOCK_MONOTONIC : CLOCK_THREAD_CPUTIME_ID, std::memory_order_relaxed);
  for (auto& v : g_phase_ns) v.store(0, std::memory_order_relaxed);
  g_phases_on.store(on, std::memory_order_relaxed);
}
void SetSaveFileCopyBuffer(bool on) { g_copy_buffer.store(on, std::memory_order_relaxed); }

void SavePhaseTotals(uint64_t ns[kPhases]) {
  for (int p = 0; p < kPhases; ++p) ns[p] = g_phase_ns[p].load(std::memory_order_relaxed);
}
const char* SavePhaseName(int p) { return p >= 0 && p < kPhases ? kPhaseNames[p] : "?"; }

Error saveFile(Hasher* h, const std::string& path, int64_t offset, int64_t length, Reader& r, int64_t* new_offset,
               bool* done, DigestSums* sums) {  // filereceiver.go:171-227
  *new_offset = 0;
  *done = false;
  FileInfo fi;
  PhaseClock pc;
  // A receiver without a GPU context (h == nullptr) fails every request that would hash, before
  // touching the file: there is no CPU fallback.  Offset mismatches are still reported first.
  if (offset == 0) {
    if (!h) return lib_error(EFES_ERR_NO_DEVICE);
    Error e = createFile(path);  // a PATCH at 0 needs no prior POST (filereceiver.go:175)
    if (e) return e;
    fi = newFileInfo();
    pc.mark(kPhaseCreate);
  } else {
    Error e = ReadFileInfo(path, &fi);
    if (e) return e;
    if (offset != fi.Offset) return offset_mismatch(offset, fi.Offset);
    if (!h) return lib_error(EFES_ERR_NO_DEVICE);
  }
  FdGuard f;
  f.fd = ::open(path.c_str(), O_WRONLY | O_CLOEXEC);  // os.OpenFile(path, os.O_WRONLY, 0600)
  if (f.fd < 0) {
    if (errno == ENOENT) {
      (void)DeleteFileInfo(path);
      return offset_mismatch(offset, 0);
    }
    return errno_error("open", path, errno);
  }
  if (::lseek(f.fd, (off_t)offset, SEEK_SET) < 0) return errno_error("seek", path, errno);

  // w := io.MultiWriter(f, fi.Digest.CRC32, fi.Digest.Sha1) (filereceiver.go:208).  Go would
  // panic writing into a nil digest; refuse the request instead.
  if (!fi.has_sha1 || !fi.has_crc32) return make_error(ERR_NIL_DIGEST, "nil digest in " + path + fileInfoExt);
  UploadGuard g(*h);
  g.dev = h->acquire();
  g.held = true;
  int rc = efes_upload_open(h->queue(g.dev), EFES_HASH_SHA1 | EFES_HASH_CRC32, &fi.Sha1, &fi.CRC32, &g.u);
  if (rc) return lib_error(rc);
  pc.mark(kPhaseOpen);

  // n, _ := io.Copy(w, r) (filereceiver.go:209): 32 KiB buffers; a read error ends the copy
  // and is ignored, so the bytes read so far still advance the state.  The buffer IS the
  // upload's pinned staging (efes_upload_reserve): the body is read straight into it, the file
  // written from it, and the commit hashes it in place -- one host copy fewer than a Write.
  constexpr size_t kCopyBuf = 32 << 10;
  int64_t n = 0;
  // io.Copy's own 32 KiB buffer (cache-hot: the body is read into it and the file written from it),
  // then one Write into the upload's staging with streaming stores (efes_upload_write): 0.45-0.47
  // request-thread CPU-s per GiB against 0.56-0.58 for reading the body straight into the pinned
  // staging (efes_upload_reserve/commit), whose cold lines cost a read-for-ownership each and
  // then serve the file write from farther away (profiles/r03_receiver/ab_copybuf.log).
  // SetSaveFileCopyBuffer(false) selects the reserve/commit path.
  const bool staged_copy = g_copy_buffer.load(std::memory_order_relaxed);
  if (staged_copy) {
    static thread_local uint8_t cbuf[kCopyBuf];
    for (;;) {
      Error er;
      const size_t nr = r.Read(cbuf, kCopyBuf, &er);
      pc.mark(kPhaseRead);
      if (nr > 0) {
        size_t nw = 0;
        Error ew = write_full(f.fd, path, cbuf, nr, &nw);
        pc.mark(kPhaseWrite);
        if (ew) {
          n += (int64_t)nw;
          break;
        }
        rc = efes_upload_write(g.u, cbuf, nr);  // CRC32.Write, Sha1.Write: staged with streaming stores
        if (rc) return lib_error(rc);
        pc.mark(kPhaseCommit);
        n += (int64_t)nr;
      }
      if (er) break;
    }
  }
  for (; !staged_copy;) {
    void* sp = nullptr;
    size_t room = 0;
    rc = efes_upload_reserve(g.u, kCopyBuf, &sp, &room);
    if (rc) return lib_error(rc);  // the .info keeps its old offset
    pc.mark(kPhaseReserve);
    uint8_t* buf = static_cast<uint8_t*>(sp);
    Error er;
    const size_t nr = r.Read(buf, std::min(room, kCopyBuf), &er);
    pc.mark(kPhaseRead);
    if (nr > 0) {
      size_t nw = 0;
      Error ew = write_full(f.fd, path, buf, nr, &nw);
      pc.mark(kPhaseWrite);
      if (ew) {  // MultiWriter stops at the file: the digests never see this buffer
        n += (int64_t)nw;
        break;
      }
      rc = efes_upload_commit(g.u, nr);  // CRC32.Write, Sha1.Write
      if (rc) return lib_error(rc);
      pc.mark(kPhaseCommit);
      n += (int64_t)nr;
    }
    if (er) break;
  }
  if (::fsync(f.fd) != 0) return errno_error("sync", path, errno);  // f.Sync()
  const int fd = f.fd;
  f.fd = -1;
  if (::close(fd) != 0) return errno_error("close", path, errno);
  pc.mark(kPhaseSync);

  fi.Offset = offset + n;
  *new_offset = fi.Offset;
  if (fi.Offset == length) {  // filereceiver.go:220-224: finished; the digests go to the headers
    uint8_t s[24];
    rc = efes_upload_sum(g.u, s);  // Sha1.Sum(nil) || CRC32.Sum(nil) (filereceiver.go:99-100)
    if (rc) return lib_error(rc);
    pc.mark(kPhaseSum);
    memcpy(sums->sha1, s, 20);
    memcpy(sums->crc32, s + 20, 4);
    *done = true;
    Error e = DeleteFileInfo(path);
    pc.mark(kPhaseInfo);
    return e;
  }
  rc = efes_upload_state(g.u, &fi.Sha1, &fi.CRC32);  // MarshalText's input after the Writes
  if (rc) return lib_error(rc);
  pc.mark(kPhaseSum);
  Error e = SaveFileInfo(path, fi);  // filereceiver.go:226
  pc.mark(kPhaseInfo);
  return e;
}

// ---- strconv / filepath / net/http -------------------------------------------------------------
Error ParseInt(std::string_view s, int64_t* out) {  // strconv.ParseInt(s, 10, 64)
  const std::string q = "strconv.ParseInt: parsing \"" + std::string(s) + "\": ";
  if (s.empty()) return make_error(ERR_SYNTAX, q + "invalid syntax");
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i == s.size()) return make_error(ERR_SYNTAX, q + "invalid syntax");
  uint64_t v = 0;
  bool range = false;
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if (c < '0' || c > '9') return make_error(ERR_SYNTAX, q + "invalid syntax");
    if (v > (UINT64_MAX - 9) / 10) range = true;
    if (!range) v = v * 10 + (uint64_t)(c - '0');
  }
  const uint64_t lim = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
  if (range || v > lim) return make_error(ERR_SYNTAX, q + "value out of range");
  *out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return Error{};
}

static std::string clean_path(const std::string& p) {  // path/filepath.Clean (Unix)
  if (p.empty()) return ".";
  const bool rooted = p[0] == '/';
  std::vector<std::string> parts;
  size_t i = 0;
  while (i < p.size()) {
    while (i < p.size() && p[i] == '/') ++i;
    size_t j = i;
    while (j < p.size() && p[j] != '/') ++j;
    const std::string el = p.substr(i, j - i);
    i = j;
    if (el.empty() || el == ".") continue;
    if (el == "..") {
      if (!parts.empty() && parts.back() != "..") {
        parts.pop_back();
      } else if (!rooted) {
        parts.push_back("..");
      }
      continue;
    }
    parts.push_back(el);
  }
  std::string out = rooted ? "/" : "";
  for (size_t k = 0; k < parts.size(); ++k) {
    if (k) out += '/';
    out += parts[k];
  }
  return out.empty() ? "." : out;
}

std::string JoinPath(const std::string& dir, const std::string& p) {  // filepath.Join
  if (dir.empty() && p.empty()) return "";
  if (dir.empty()) return clean_path(p);
  if (p.empty()) return clean_path(dir);
  return clean_path(dir + "/" + p);
}

bool HeaderLess::operator()(const std::string& a, const std::string& b) const {
  return strcasecmp(a.c_str(), b.c_str()) < 0;
}

static std::string header_get(const Header& h, const char* k) {  // http.Header.Get
  auto it = h.find(k);
  return it == h.end() ? std::string() : it->second;
}

static void http_error(Response* w, const std::string& msg, int code) {  // net/http.Error
  w->Headers["Content-Type"] = "text/plain; charset=utf-8";
  w->Headers["X-Content-Type-Options"] = "nosniff";
  w->Code = code;
  w->Body = msg + "\n";
}

static void internal_server_error(Response* w, const std::string& message, const Error& err) {  // filereceiver.go:34-40
  http_error(w, message + ": " + err.str(), 500);
}

Response FileReceiver::ServeHTTP(const Request& r) {  // filereceiver.go:42-127
  Response w;
  const std::string path = JoinPath(dir_, r.Path);
  if (r.Method == "POST") {
    Error e = createFile(path);
    if (e) internal_server_error(&w, "cannot create file", e);
  } else if (r.Method == "HEAD") {
    FileInfo fi;
    Error e = ReadFileInfo(path, &fi);
    if (e) {
      internal_server_error(&w, "cannot get offset", e);
      return w;
    }
    w.Headers["efes-file-offset"] = std::to_string(fi.Offset);
  } else if (r.Method == "PATCH") {
    int64_t offset;
    if (ParseInt(header_get(r.Headers, "efes-file-offset"), &offset)) {
      http_error(&w, "invalid header: efes-file-offset", 400);
      return w;
    }
    int64_t length = -1;
    const std::string lh = header_get(r.Headers, "efes-file-length");
    if (!lh.empty() && ParseInt(lh, &length)) {
      http_error(&w, "invalid header: efes-file-length", 400);
      return w;
    }
    // efes-drain / tempfileExists: db == nil -> the tempfile exists (filereceiver.go:73-83, 130-132)
    BytesReader empty("");
    Reader& body = r.Body ? *r.Body : empty;
    int64_t new_offset = 0;
    bool done = false;
    DigestSums sums;
    Error e = saveFile(h_, path, offset, length, body, &new_offset, &done, &sums);
    if (e.code == ERR_OFFSET_MISMATCH) {  // filereceiver.go:85-93
      w.Headers["Content-Type"] = "text/plain; charset=utf-8";
      w.Headers["X-Content-Type-Options"] = "nosniff";
      w.Headers["efes-file-offset"] = std::to_string(e.required);
      w.Code = 409;
      w.Body = e.str();
      return w;
    }
    if (e) {
      internal_server_error(&w, "cannot save file", e);
      return w;
    }
    if (done) {
      w.Headers["efes-file-sha1"] = HexEncode(sums.sha1, 20);
      w.Headers["efes-file-crc32"] = HexEncode(sums.crc32, 4);
    }
    w.Headers["efes-file-offset"] = std::to_string(new_offset);
  } else if (r.Method == "DELETE") {
    FileInfo fi;
    Error e = ReadExistingFileInfo(path, &fi);
    if (e.code == ERR_NOT_EXIST) {
      http_error(&w, "offset file does not exist", 404);
      return w;
    }
    if (e) {
      internal_server_error(&w, "cannot read offset file", e);
      return w;
    }
    if ((e = DeleteFileInfo(path))) {
      internal_server_error(&w, "cannot delete offset file", e);
      return w;
    }
    if ((e = deleteFile(path))) internal_server_error(&w, "cannot delete file", e);
  } else {
    http_error(&w, "Method Not Allowed", 405);
  }
  return w;
}

// ---- write.go ----------------------------------------------------------------------------------
Response LocalTransport::RoundTrip(const Request& r, Error* err) {
  *err = Error{};
  return fr_->ServeHTTP(r);
}

namespace {

struct ReadCounter : Reader {  // readcounter.go:8-27
  Reader& r;
  int64_t count = 0;
  explicit ReadCounter(Reader& rr) : r(rr) {}
  size_t Read(uint8_t* p, size_t cap, Error* err) override {
    const size_t n = r.Read(p, cap, err);
    count += (int64_t)n;
    return n;
  }
};

struct LimitReader : Reader {  // io.LimitReader
  Reader& r;
  int64_t left;
  LimitReader(Reader& rr, int64_t n) : r(rr), left(n) {}
  size_t Read(uint8_t* p, size_t cap, Error* err) override {
    *err = Error{};
    if (left <= 0) {
      *err = make_error(ERR_EOF, "EOF");
      return 0;
    }
    const size_t n = r.Read(p, std::min<size_t>(cap, (size_t)left), err);
    left -= (int64_t)n;
    return n;
  }
};

Error check_response(const Response& w) {  // httperror.go:10-22
  if (w.Code / 100 == 2) return Error{};
  Error e = make_error(ERR_HTTP, std::to_string(w.Code) + ": " + w.Body);
  e.status = w.Code;
  return e;
}

// write.go:154-172 (efes-drain when the client is the drainer's, client.go:21 / write.go:163-165)
Error patch(Transport& t, const std::string& path, Reader* body, int64_t offset, int64_t size, bool drainer,
            Response* w) {
  Request r;
  r.Method = "PATCH";
  r.Path = path;
  r.Headers["efes-file-offset"] = std::to_string(offset);
  if (size > -1) r.Headers["efes-file-length"] = std::to_string(size);
  if (drainer) r.Headers["efes-drain"] = "true";
  r.Body = body;
  Error e;
  *w = t.RoundTrip(r, &e);
  if (e) return e;
  return check_response(*w);
}

Error get_offset(Transport& t, const std::string& path, int64_t* off) {  // write.go:174-185
  Request r;
  r.Method = "HEAD";
  r.Path = path;
  Error e;
  Response w = t.RoundTrip(r, &e);
  if (e) return e;
  return ParseInt(w.Headers["efes-file-offset"], off);
}

Checksums checksums_from(Response& w) {  // write.go:146-151
  return Checksums{w.Headers["efes-file-sha1"], w.Headers["efes-file-crc32"]};
}

// write.go:120-144: PATCHes of ChunkSize until the size is reached, or an empty one (then finish).
Error send(Transport& t, const std::string& path, Reader& r, int64_t offset, int64_t size, const ClientConfig& cfg,
           Checksums* out) {
  ReadCounter rc(r);
  int64_t current = offset;
  for (;;) {
    LimitReader chunk_reader(rc, cfg.ChunkSize);
    const int64_t request_offset = current;
    Response w;
    Error e = patch(t, path, &chunk_reader, request_offset, size, cfg.Drainer, &w);
    if (e) return e;
    current = offset + rc.count;
    if (current == size) {  // EOF reached: the server has deleted the offset file
      *out = checksums_from(w);
      return Error{};
    }
    if (current == request_offset) {  // nothing sent: the file was read to its end (write.go:188-195)
      e = patch(t, path, nullptr, request_offset, request_offset, cfg.Drainer, &w);
      if (e) return e;
      *out = checksums_from(w);
      return Error{};
    }
  }
}

bool hex_decode(const std::string& h, std::string* out) {
  if (h.size() % 2) return false;
  out->clear();
  for (size_t i = 0; i < h.size(); i += 2) {
    int v = 0;
    for (int k = 0; k < 2; ++k) {
      const char c = h[i + k];
      const int d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
      if (d < 0) return false;
      v = v * 16 + d;
    }
    out->push_back((char)v);
  }
  return true;
}

}  // namespace

Error sendFile(Transport& t, efes_ctx* ctx, const std::string& path, ReadSeeker& rs, int64_t size,
               const ClientConfig& cfg, Checksums* out) {  // write.go:68-117
  Sha1File* sfp = nullptr;
  Error e = Sha1File::New(&rs, ctx, &sfp);
  if (e) return e;
  std::unique_ptr<Sha1File> sf(sfp);
  Checksums cs;
  std::string remote;
  bool first = true;
  for (int attempt = 0;; ++attempt) {  // backoff.Retry(op, bo)
    int64_t offset = 0;
    e = Error{};
    if (first) {
      first = false;
    } else {  // resume where the server is (write.go:84-96)
      e = get_offset(t, path, &offset);
      if (!e) {
        Error se;
        sf->Seek(offset, 0, &se);
        e = se;
      }
    }
    if (!e) e = send(t, path, *sf, offset, size, cfg, &cs);
    if (!e && !hex_decode(cs.Sha1, &remote)) e = make_error(ERR_SYNTAX, "encoding/hex: invalid byte in " + cs.Sha1);
    if (!e) break;
    if (e.code == ERR_HTTP && e.status == 404) return e;  // backoff.Permanent (write.go:98-100)
    if (attempt + 1 >= cfg.MaxAttempts) return e;
  }
  uint8_t local[20];
  e = sf->Sum(local);
  if (e) return e;
  if (remote != std::string(reinterpret_cast<char*>(local), 20))
    return make_error(ERR_SHA1_MISMATCH, "local sha1 (" + HexEncode(local, 20) + ") does not match remote sha1 (" +
                                             cs.Sha1 + ")");
  *out = cs;
  return Error{};
}

// ---- sha1file.go -------------------------------------------------------------------------------
Error Sha1File::New(ReadSeeker* rs, efes_ctx* ctx, Sha1File** out) {  // sha1file.go:16-21
  efes_sha1* d = nullptr;
  const int rc = efes_sha1_new(ctx, &d);
  if (rc) return lib_error(rc);
  Sha1File* f = new Sha1File;
  f->rs_ = rs;
  f->digest_ = d;
  *out = f;
  return Error{};
}

Sha1File::~Sha1File() { efes_sha1_free(digest_); }

size_t Sha1File::Read(uint8_t* p, size_t cap, Error* err) {  // sha1file.go:23-37
  *err = Error{};
  if (position_ > calculated_) {
    *err = make_error(ERR_SHA1FILE, "missing data for sha1");
    return 0;
  }
  const int64_t prev = position_;
  const size_t n = rs_->Read(p, cap, err);
  position_ += (int64_t)n;
  if (position_ > calculated_) {
    const int64_t crop = calculated_ - prev;  // only the bytes not hashed before (a retry re-reads)
    const size_t c = n - (size_t)crop;
    const int rc = efes_sha1_write(digest_, p + crop, c);  // f.digest.Write(c)
    if (rc && !latched_) latched_ = rc;
    calculated_ += (int64_t)c;
  }
  return n;
}

int64_t Sha1File::Seek(int64_t offset, int whence, Error* err) {  // sha1file.go:39-49
  const int64_t np = rs_->Seek(offset, whence, err);
  if (*err) return np;
  if (position_ < np) {
    *err = make_error(ERR_SHA1FILE, "seeking forward is not supported");
    return np;
  }
  position_ = np;
  return np;
}

Error Sha1File::Sum(uint8_t out[20]) {  // sha1file.go:51-53
  if (latched_) return lib_error(latched_);
  return lib_error(efes_sha1_sum(digest_, out));
}

}  // namespace efes
