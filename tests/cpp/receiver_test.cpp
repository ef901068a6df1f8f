// receiver_test.cpp -- the reference's own tests of the upload receiver, replayed against the
// C++ mirror (efes_amd/host/efes_receiver.hpp) with every digest checked against the CPU oracle.
// Test infrastructure: built by __graft_entry__.build() (links libefesreceiver.so,
// libefeshash.so and oracle/liboracle.so); run by tests/test_receiver.py.
//
//   receiver_test cpu <tmpdir>                      no device work: the .info JSON codec, strconv /
//                                                   filepath helpers, POST / HEAD / DELETE and the
//                                                   PATCH paths that end before hashing (400, 409)
//   receiver_test gpu <tmpdir> [threads] [uploads]  filereceiver_test.go (all six tests) with the
//                                                   digest headers asserted, sha1file_test.go over a
//                                                   real file, concurrent resumable uploads through
//                                                   ServeHTTP (every .info byte-compared with Go's),
//                                                   and the error paths of saveFile
//
// Prints "receiver_test <mode> ok ..." and exits 0, or names the first failure and exits 1.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../efes_amd/host/efes_receiver.hpp"
#include "../../oracle/efes_oracle.h"

using namespace efes;

static std::atomic<int> g_fail{0};
static std::mutex g_mu;
static int g_checks = 0;

#define CHECK(cond, ...)                              \
  do {                                                \
    std::lock_guard<std::mutex> lk_(g_mu);            \
    ++g_checks;                                       \
    if (!(cond)) {                                    \
      if (!g_fail) {                                  \
        fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
        fprintf(stderr, __VA_ARGS__);                 \
        fprintf(stderr, "\n");                        \
      }                                               \
      g_fail = 1;                                     \
    }                                                 \
  } while (0)

static std::string slurp(const std::string& p, bool* ok = nullptr) {
  FILE* f = fopen(p.c_str(), "rb");
  if (ok) *ok = f != nullptr;
  if (!f) return "";
  std::string s;
  char b[4096];
  size_t n;
  while ((n = fread(b, 1, sizeof b, f)) > 0) s.append(b, n);
  fclose(f);
  return s;
}

static bool exists(const std::string& p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0;
}

// What Go's json.Encoder writes for a FileInfo with these oracle digests (fileinfo.go:53).
static std::string go_info(int64_t offset, const oracle_sha1& s, const oracle_crc32& c) {
  char st[200], ct[8];
  oracle_sha1_marshal_text(&s, st);
  oracle_crc32_marshal_text(&c, ct);
  return "{\"offset\":" + std::to_string(offset) + ",\"digest\":{\"sha1\":\"" + std::string(st, 200) +
         "\",\"crc32\":\"" + std::string(ct, 8) + "\"}}\n";
}

static oracle_sha1 o_new_sha1() {  // NewSha1: a zero sha1digest, then Reset (sha1.go:48-52)
  oracle_sha1 s;
  memset(&s, 0, sizeof s);
  oracle_sha1_reset(&s);
  return s;
}

static std::string hexs(const uint8_t* p, size_t n) { return HexEncode(p, n); }

// ---- the handler calls of filereceiver_test.go:103-165 ----------------------------------------
struct Client {
  FileReceiver* fr;
  std::string path = "/dir/file.txt";  // filereceiver_test.go:14 testPath

  Response call(const char* method, Reader* body = nullptr, Header h = {}) {
    Request r;
    r.Method = method;
    r.Path = path;
    r.Headers = std::move(h);
    r.Body = body;
    return fr->ServeHTTP(r);
  }
  void create() {  // testCreate
    Response w = call("POST");
    CHECK(w.Code == 200, "POST %s: %d %s", path.c_str(), w.Code, w.Body.c_str());
  }
  void del() {  // testDelete
    Response w = call("DELETE");
    CHECK(w.Code == 200, "DELETE %s: %d %s", path.c_str(), w.Code, w.Body.c_str());
  }
  void offset(int64_t want) {  // testOffset
    Response w = call("HEAD");
    CHECK(w.Code == 200, "HEAD %s: %d %s", path.c_str(), w.Code, w.Body.c_str());
    int64_t got = -1;
    CHECK(!ParseInt(w.Headers["efes-file-offset"], &got) && got == want, "HEAD %s offset %s want %lld", path.c_str(),
          w.Headers["efes-file-offset"].c_str(), (long long)want);
  }
  Response send(int64_t off, int64_t length, const std::string& data, size_t max_read = SIZE_MAX) {  // testSend
    BytesReader b(data, max_read);
    Header h;
    h["efes-file-offset"] = std::to_string(off);
    if (length >= 0) h["efes-file-length"] = std::to_string(length);
    return call("PATCH", &b, h);
  }
  void send_ok(int64_t off, int64_t length, const std::string& data) {
    Response w = send(off, length, data);
    CHECK(w.Code == 200, "PATCH %s at %lld: %d %s", path.c_str(), (long long)off, w.Code, w.Body.c_str());
  }
};

static std::string fresh_dir(const std::string& root, const char* name) {  // os.MkdirTemp
  const std::string d = root + "/" + name;
  std::string cmd = "rm -rf '" + d + "'";
  if (system(cmd.c_str()) != 0) CHECK(false, "rm %s", d.c_str());
  mkdir(d.c_str(), 0700);
  return d;
}

// =================================================================================================
// CPU tests: no device work
// =================================================================================================
static void test_parse_int() {
  int64_t v = 0;
  CHECK(!ParseInt("0", &v) && v == 0, "0");
  CHECK(!ParseInt("+5", &v) && v == 5, "+5");
  CHECK(!ParseInt("-5", &v) && v == -5, "-5");
  CHECK(!ParseInt("9223372036854775807", &v) && v == INT64_MAX, "max");
  CHECK(!ParseInt("-9223372036854775808", &v) && v == INT64_MIN, "min");
  CHECK(!ParseInt("007", &v) && v == 7, "leading zeros");
  Error e = ParseInt("9223372036854775808", &v);
  CHECK(e && e.msg.find("value out of range") != std::string::npos, "range: %s", e.msg.c_str());
  CHECK(ParseInt("99999999999999999999999", &v).msg.find("out of range") != std::string::npos, "huge");
  for (const char* bad : {"", "+", "-", " 1", "1 ", "1.0", "0x10", "1_000", "1e3", "abc"}) {
    e = ParseInt(bad, &v);
    CHECK(e && e.msg == std::string("strconv.ParseInt: parsing \"") + bad + "\": invalid syntax", "'%s': %s", bad,
          e.msg.c_str());
  }
}

static void test_join_path() {  // filepath.Join(f.dir, r.URL.Path) (filereceiver.go:43)
  CHECK(JoinPath("/srv/dev1", "/dir/file.txt") == "/srv/dev1/dir/file.txt", "join");
  CHECK(JoinPath("/srv/dev1/", "//a/./b//c/") == "/srv/dev1/a/b/c", "clean");
  CHECK(JoinPath("/srv/dev1", "/a/../b") == "/srv/dev1/b", "dotdot");
  CHECK(JoinPath("/srv", "/../../x") == "/x", "above root: %s", JoinPath("/srv", "/../../x").c_str());
  CHECK(JoinPath("rel", "../..") == "..", "relative: %s", JoinPath("rel", "../..").c_str());
  CHECK(JoinPath("", "") == "", "empty");
  CHECK(JoinPath("/", "") == "/", "root");
}

static void test_offset_mismatch_text() {  // filereceiver.go:234-236
  CHECK(OffsetMismatchText(1, 0) == "given offset (1) does not match required offset (0)", "text");
}

static void test_json() {
  // newFileInfo() as Go encodes it: NewSha1 (IV, zero tail), NewCRC32IEEE (0)
  const std::string fresh = std::string("{\"offset\":0,\"digest\":{\"sha1\":\"") +
                            "67452301efcdab8998badcfe10325476c3d2e1f0" + std::string(128, '0') + std::string(32, '0') +
                            "\",\"crc32\":\"00000000\"}}\n";
  CHECK(EncodeFileInfo(newFileInfo()) == fresh, "fresh .info:\n%s", EncodeFileInfo(newFileInfo()).c_str());

  // a mid-stream state (nx != 0, stale tail bytes) from the oracle, through the codec and back
  oracle_sha1 s = o_new_sha1();
  oracle_crc32 c;
  oracle_crc32_reset(&c);
  std::vector<uint8_t> data(1000);
  oracle_fill_synthetic(data.data(), data.size(), 5);
  for (size_t o = 0; o < data.size(); o += 77) {
    const size_t n = std::min<size_t>(77, data.size() - o);
    oracle_sha1_write(&s, data.data() + o, n);
    oracle_crc32_write(&c, data.data() + o, n);
  }
  const std::string want = go_info(1000, s, c);
  FileInfo fi;
  Error e = DecodeFileInfo(want, &fi);
  CHECK(!e && fi.Offset == 1000 && fi.has_sha1 && fi.has_crc32, "decode: %s", e.msg.c_str());
  CHECK(EncodeFileInfo(fi) == want, "re-encode differs:\n%s\n%s", EncodeFileInfo(fi).c_str(), want.c_str());
  CHECK(fi.Sha1.nx == s.nx && fi.Sha1.len == s.len && !memcmp(fi.Sha1.x, s.x, 64) && !memcmp(fi.Sha1.h, s.h, 20),
        "state");
  CHECK(fi.CRC32.crc == c.crc, "crc");

  char st[200], ct[8];
  oracle_sha1_marshal_text(&s, st);
  oracle_crc32_marshal_text(&c, ct);
  const std::string sh(st, 200), ch(ct, 8);
  // encoding/json accepts: any whitespace, case-insensitive keys, unknown keys, escapes, and
  // ignores what follows the first value of the stream
  const std::string loose = " \n{ \"Digest\" : { \"CRC32\":\"" + ch + "\", \"extra\": [1, {\"a\": null}, \"x\"], \"SHA1\": \"" +
                            sh + "\" } ,\"unknown\":{\"offset\":5},\"OFFSET\" : 1000 } trailing";
  e = DecodeFileInfo(loose, &fi);
  CHECK(!e && EncodeFileInfo(fi) == want, "loose JSON: %s", e.msg.c_str());
  std::string esc = want;
  esc.replace(esc.find(sh), 1, std::string("\\u00") + HexEncode(reinterpret_cast<const uint8_t*>(sh.data()), 1));
  e = DecodeFileInfo(esc, &fi);
  CHECK(!e && EncodeFileInfo(fi) == want, "\\u escape: %s", e.msg.c_str());
  e = DecodeFileInfo("{\"offset\":1,\"offset\":7,\"digest\":{\"sha1\":\"" + sh + "\",\"crc32\":\"" + ch + "\"}}", &fi);
  CHECK(!e && fi.Offset == 7, "duplicate key: last wins");

  // errors
  std::string bad = want;
  bad[bad.find(sh) + 3] = 'g';
  e = DecodeFileInfo(bad, &fi);
  CHECK(e.code == EFES_ERR_INVALID_DIGEST && e.msg == "invalid digest", "bad hex: %d %s", e.code, e.msg.c_str());
  bad = want;
  bad.erase(bad.find(sh), 2);
  CHECK(DecodeFileInfo(bad, &fi).code == EFES_ERR_INVALID_DIGEST, "short sha1 text");
  bad = want;
  bad.replace(bad.find(ch), 8, "0000000");
  CHECK(DecodeFileInfo(bad, &fi).code == EFES_ERR_INVALID_DIGEST, "short crc32 text");
  CHECK(DecodeFileInfo("{\"offset\":3.0}", &fi).code == ERR_JSON, "float offset");
  CHECK(DecodeFileInfo("{\"offset\":\"3\"}", &fi).code == ERR_JSON, "string offset");
  CHECK(DecodeFileInfo("{\"offset\":99999999999999999999}", &fi).code == ERR_JSON, "offset range");
  CHECK(DecodeFileInfo("{\"digest\":{\"sha1\":5}}", &fi).code == ERR_JSON, "number digest");
  CHECK(DecodeFileInfo("[]", &fi).code == ERR_JSON, "array");
  CHECK(DecodeFileInfo("", &fi).code == ERR_EOF, "empty file: io.EOF");
  CHECK(DecodeFileInfo("  \n", &fi).code == ERR_EOF, "blank file: io.EOF");
  CHECK(DecodeFileInfo("{\"offset\":3", &fi), "truncated");
  CHECK(DecodeFileInfo("{\"offset\":3,}", &fi).code == ERR_JSON, "trailing comma");
  CHECK(DecodeFileInfo("{offset:3}", &fi).code == ERR_JSON, "unquoted key");
  CHECK(DecodeFileInfo("{\"offset\":01}", &fi), "leading zero number");
  CHECK(DecodeFileInfo("{\"a\":\"\x01\"}", &fi).code == ERR_JSON, "control character");
  CHECK(DecodeFileInfo("null", &fi).code == ERR_NIL_DIGEST, "null document");
  std::string deep(20000, '[');
  CHECK(DecodeFileInfo("{\"x\":" + deep, &fi), "nesting limit");
  // null digests decode to nil pointers (encode back as null), missing ones stay nil
  e = DecodeFileInfo("{\"offset\":4,\"digest\":{\"sha1\":null,\"crc32\":\"" + ch + "\"}}", &fi);
  CHECK(!e && !fi.has_sha1 && fi.has_crc32 && fi.Offset == 4, "null sha1");
  CHECK(EncodeFileInfo(fi).find("\"sha1\":null") != std::string::npos, "null re-encoded");
  e = DecodeFileInfo("{\"offset\":4}", &fi);
  CHECK(!e && !fi.has_sha1 && !fi.has_crc32, "missing digests");
}

static void test_fileinfo_files(const std::string& root) {
  const std::string d = fresh_dir(root, "fileinfo");
  const std::string p = d + "/sub/dir/17.dat";
  FileInfo fi;
  Error e = ReadFileInfo(p, &fi);  // no .info: a new FileInfo (fileinfo.go:31-33)
  CHECK(!e && EncodeFileInfo(fi) == EncodeFileInfo(newFileInfo()), "ReadFileInfo of a missing file");
  e = ReadExistingFileInfo(p, &fi);
  CHECK(e.code == ERR_NOT_EXIST && e.msg == "open " + p + ".info: no such file or directory", "%s", e.msg.c_str());
  e = createFile(p);  // MkdirAll(dir, 0700) then Create, and a fresh .info (filereceiver.go:148-165)
  CHECK(!e && exists(p), "createFile: %s", e.msg.c_str());
  struct stat st;
  CHECK(stat((d + "/sub/dir").c_str(), &st) == 0 && (st.st_mode & 0777) == 0700, "MkdirAll mode");
  CHECK(slurp(p + ".info") == EncodeFileInfo(newFileInfo()), ".info of a created file");
  fi.Offset = 12345;
  CHECK(!SaveFileInfo(p, fi), "SaveFileInfo");
  FileInfo back;
  CHECK(!ReadExistingFileInfo(p, &back) && back.Offset == 12345, "read back");
  CHECK(!DeleteFileInfo(p) && !exists(p + ".info"), "DeleteFileInfo");
  e = DeleteFileInfo(p);
  CHECK(e.code == ERR_NOT_EXIST && e.msg == "remove " + p + ".info: no such file or directory", "%s", e.msg.c_str());
  FILE* f = fopen((p + ".info").c_str(), "w");
  fclose(f);  // an empty .info: json.Decode gives io.EOF
  CHECK(ReadFileInfo(p, &fi).code == ERR_EOF, "empty .info");
}

// The HTTP methods that do no hashing (a FileReceiver without a Hasher).
static void test_handler_cpu(const std::string& root) {
  const std::string dir = fresh_dir(root, "handler_cpu");
  FileReceiver fr(dir, nullptr);
  Client c{&fr};
  c.offset(0);  // TestFileReceiver's opening steps (filereceiver_test.go:38-40)
  c.create();
  c.offset(0);
  CHECK(exists(dir + "/dir/file.txt") && exists(dir + "/dir/file.txt.info"), "POST created file and .info");
  c.del();
  c.offset(0);
  CHECK(!exists(dir + "/dir/file.txt") && !exists(dir + "/dir/file.txt.info"), "DELETE removed both");
  Response w = c.call("DELETE");  // filereceiver.go:105-107
  CHECK(w.Code == 404 && w.Body == "offset file does not exist\n", "DELETE twice: %d %s", w.Code, w.Body.c_str());
  w = c.call("GET");
  CHECK(w.Code == 405 && w.Body == "Method Not Allowed\n", "GET: %d", w.Code);

  // TestFileReceiverInvalidOffset (filereceiver_test.go:86-101): 409 before any hashing
  w = c.call("PATCH", nullptr, Header{{"efes-file-offset", "1"}});
  CHECK(w.Code == 409 && w.Headers["efes-file-offset"] == "0" &&
            w.Body == "given offset (1) does not match required offset (0)",
        "invalid offset: %d %s", w.Code, w.Body.c_str());
  CHECK(w.Headers["Content-Type"] == "text/plain; charset=utf-8" && w.Headers["X-Content-Type-Options"] == "nosniff",
        "409 headers");
  w = c.call("PATCH");  // no offset header
  CHECK(w.Code == 400 && w.Body == "invalid header: efes-file-offset\n", "missing offset: %d", w.Code);
  w = c.call("PATCH", nullptr, Header{{"EFES-FILE-OFFSET", "x"}});
  CHECK(w.Code == 400, "bad offset (header names are case-insensitive)");
  w = c.call("PATCH", nullptr, Header{{"efes-file-offset", "0"}, {"efes-file-length", "3.5"}});
  CHECK(w.Code == 400 && w.Body == "invalid header: efes-file-length\n", "bad length: %d", w.Code);
  // a corrupt .info: HEAD fails with 500 and Go's message
  c.create();
  FILE* f = fopen((dir + "/dir/file.txt.info").c_str(), "w");
  fputs("{\"offset\":3,\"digest\":{\"sha1\":\"zz\",\"crc32\":\"00000000\"}}\n", f);
  fclose(f);
  w = c.call("HEAD");
  CHECK(w.Code == 500 && w.Body == "cannot get offset: invalid digest\n", "corrupt .info HEAD: %d %s", w.Code,
        w.Body.c_str());
  w = c.send(3, -1, "x");
  CHECK(w.Code == 500 && w.Body == "cannot save file: invalid digest\n", "corrupt .info PATCH: %d %s", w.Code,
        w.Body.c_str());
  // no GPU context behind the receiver: a PATCH that reaches saveFile fails loudly (no CPU fallback)
  w = c.send(0, -1, "x");
  CHECK(w.Code == 500 && w.Body == "cannot save file: no usable gfx950 device\n", "no hasher: %d %s", w.Code,
        w.Body.c_str());
}

// =================================================================================================
// GPU tests
// =================================================================================================
static efes_ctx* g_ctx;
static Hasher* g_hasher;

static void check_done(Response w, const std::string& data, const char* what) {
  uint8_t sha[20];
  uint32_t crc;
  oracle_hash_message(reinterpret_cast<const uint8_t*>(data.data()), data.size(), 32768, sha, &crc);
  char c[9];
  snprintf(c, sizeof c, "%08x", crc);
  CHECK(w.Code == 200, "%s: %d %s", what, w.Code, w.Body.c_str());
  CHECK(w.Headers["efes-file-sha1"] == hexs(sha, 20), "%s: efes-file-sha1 %s want %s", what,
        w.Headers["efes-file-sha1"].c_str(), hexs(sha, 20).c_str());
  CHECK(w.Headers["efes-file-crc32"] == c, "%s: efes-file-crc32 %s want %s", what, w.Headers["efes-file-crc32"].c_str(), c);
}

static void test_file_receiver(const std::string& root) {  // filereceiver_test.go:34-101
  {  // TestFileReceiver
    const std::string dir = fresh_dir(root, "TestFileReceiver");
    FileReceiver fr(dir, g_hasher);
    Client c{&fr};
    c.offset(0);
    c.create();
    c.offset(0);
    c.send_ok(0, -1, "foo");
    c.offset(3);
    oracle_sha1 s = o_new_sha1();
    oracle_crc32 k;
    oracle_crc32_reset(&k);
    oracle_sha1_write(&s, reinterpret_cast<const uint8_t*>("foo"), 3);
    oracle_crc32_write(&k, reinterpret_cast<const uint8_t*>("foo"), 3);
    CHECK(slurp(dir + "/dir/file.txt.info") == go_info(3, s, k), "TestFileReceiver .info after foo:\n%s",
          slurp(dir + "/dir/file.txt.info").c_str());
    c.send_ok(3, -1, "bar");
    c.offset(6);
    oracle_sha1_write(&s, reinterpret_cast<const uint8_t*>("bar"), 3);
    oracle_crc32_write(&k, reinterpret_cast<const uint8_t*>("bar"), 3);
    CHECK(slurp(dir + "/dir/file.txt.info") == go_info(6, s, k), "TestFileReceiver .info after bar");
    CHECK(slurp(dir + "/dir/file.txt") == "foobar", "file contents");
    c.del();
    c.offset(0);
  }
  {  // TestFileReceiverNoCreate
    const std::string dir = fresh_dir(root, "TestFileReceiverNoCreate");
    FileReceiver fr(dir, g_hasher);
    Client c{&fr};
    c.send_ok(0, -1, "baz");
    c.offset(3);
    c.del();
    c.offset(0);
  }
  {  // TestFileReceiverNoDelete: the last PATCH deletes the .info itself and reports the digests
    const std::string dir = fresh_dir(root, "TestFileReceiverNoDelete");
    FileReceiver fr(dir, g_hasher);
    Client c{&fr};
    c.create();
    Response w = c.send(0, 3, "baz");
    check_done(w, "baz", "NoDelete");
    CHECK(w.Headers["efes-file-sha1"] == "bbe960a25ea311d21d40669e93df2003ba9b90a2" &&
              w.Headers["efes-file-crc32"] == "78240498",
          "baz KAT");
    CHECK(!exists(dir + "/dir/file.txt.info"), ".info deleted on the last PATCH");
    c.offset(0);
  }
  {  // TestFileReceiverZeroByte
    const std::string dir = fresh_dir(root, "TestFileReceiverZeroByte");
    FileReceiver fr(dir, g_hasher);
    Client c{&fr};
    c.create();
    c.send_ok(0, -1, "");
    c.offset(0);
    c.del();
    Response w;
    c.create();  // a zero-byte upload with its length finishes at once: SHA-1 / CRC-32 of ""
    w = c.send(0, 0, "");
    check_done(w, "", "zero-byte");
    CHECK(w.Headers["efes-file-sha1"] == "da39a3ee5e6b4b0d3255bfef95601890afd80709", "empty KAT");
  }
  {  // TestFileReceiverSingleRequest
    const std::string dir = fresh_dir(root, "TestFileReceiverSingleRequest");
    FileReceiver fr(dir, g_hasher);
    Client c{&fr};
    Response w = c.send(0, 3, "foo");
    check_done(w, "foo", "SingleRequest");
    CHECK(w.Headers["efes-file-sha1"] == "0beec7b5ea3f0fdbc95d0dd47f3c5bc275da8a33" &&
              w.Headers["efes-file-crc32"] == "8c736521" && w.Headers["efes-file-offset"] == "3",
          "foo KAT");
    c.offset(0);
  }
  {  // TestFileReceiverInvalidOffset
    const std::string dir = fresh_dir(root, "TestFileReceiverInvalidOffset");
    FileReceiver fr(dir, g_hasher);
    Client c{&fr};
    Response w = c.call("PATCH", nullptr, Header{{"efes-file-offset", "1"}});
    CHECK(w.Code == 409, "InvalidOffset: %d", w.Code);
  }
  {  // "foo" + "bar" finishing with the length: the TestFileReceiver object's digests
    const std::string dir = fresh_dir(root, "foobar");
    FileReceiver fr(dir, g_hasher);
    Client c{&fr};
    c.send_ok(0, 6, "foo");
    Response w = c.send(3, 6, "bar");
    check_done(w, "foobar", "foo+bar");
    CHECK(w.Headers["efes-file-sha1"] == "8843d7f92416211de9ebb963ff4ce28125932878" &&
              w.Headers["efes-file-crc32"] == "9ef61f95",
          "foobar KAT");
    w = c.send(3, 6, "bar");  // a retry after the upload finished: the offset restarts at 0
    CHECK(w.Code == 409 && w.Headers["efes-file-offset"] == "0", "retry after finish: %d", w.Code);
  }
}

// An io.Reader that fails after `limit` bytes (a dropped connection): io.Copy ignores the
// error (filereceiver.go:209), so the bytes read so far still count.
struct FailingReader : Reader {
  BytesReader in;
  size_t left;
  FailingReader(std::string d, size_t limit) : in(std::move(d), 1000), left(limit) {}
  size_t Read(uint8_t* p, size_t cap, Error* err) override {
    if (left == 0) {
      *err = make_error(ERR_IO, "read tcp: connection reset by peer");
      return 0;
    }
    const size_t n = in.Read(p, std::min(cap, left), err);
    left -= n;
    return n;
  }
};

static void test_save_file_errors(const std::string& root) {
  const std::string dir = fresh_dir(root, "errors");
  FileReceiver fr(dir, g_hasher);
  Client c{&fr};
  std::string data(5000, 'q');
  for (size_t i = 0; i < data.size(); ++i) data[i] = (char)(i * 131 + 7);
  {  // a body that breaks after 2500 bytes: state and offset advance by 2500, the request succeeds
    FailingReader fr2(data, 2500);
    Request r;
    r.Method = "PATCH";
    r.Path = c.path;
    r.Headers["efes-file-offset"] = "0";
    r.Body = &fr2;
    Response w = fr.ServeHTTP(r);
    CHECK(w.Code == 200 && w.Headers["efes-file-offset"] == "2500", "broken body: %d %s", w.Code,
          w.Headers["efes-file-offset"].c_str());
    oracle_sha1 s = o_new_sha1();
    oracle_crc32 k;
    oracle_crc32_reset(&k);
    for (size_t o = 0; o < 2500; o += 1000) {  // the reader's 1000-byte reads are the Writes
      const size_t n = std::min<size_t>(1000, 2500 - o);
      oracle_sha1_write(&s, reinterpret_cast<const uint8_t*>(data.data()) + o, n);
      oracle_crc32_write(&k, reinterpret_cast<const uint8_t*>(data.data()) + o, n);
    }
    CHECK(slurp(dir + "/dir/file.txt.info") == go_info(2500, s, k), "broken body .info");
    Response w2 = c.send(2500, 5000, data.substr(2500), 1000);  // the client resumes
    check_done(w2, data, "resume after broken body");
  }
  {  // the file vanished between PATCHes: 409 with offset 0 and the .info removed (filereceiver.go:190-193)
    c.send_ok(0, -1, "abc");
    unlink((dir + "/dir/file.txt").c_str());
    Response w = c.send(3, -1, "def");
    CHECK(w.Code == 409 && w.Headers["efes-file-offset"] == "0", "vanished file: %d", w.Code);
    CHECK(!exists(dir + "/dir/file.txt.info"), "vanished file: .info removed");
  }
  {  // a .info whose state Go would panic on (nx > 64): the request fails, the .info is kept
    c.send_ok(0, -1, "abc");
    FileInfo fi;
    CHECK(!ReadExistingFileInfo(dir + "/dir/file.txt", &fi), "read");
    fi.Sha1.nx = 65;
    CHECK(!SaveFileInfo(dir + "/dir/file.txt", fi), "save");
    const std::string before = slurp(dir + "/dir/file.txt.info");
    Response w = c.send(3, -1, "def");
    CHECK(w.Code == 500 && w.Body.rfind("cannot save file: ", 0) == 0, "nx > 64: %d %s", w.Code, w.Body.c_str());
    CHECK(slurp(dir + "/dir/file.txt.info") == before, "nx > 64: .info unchanged");
    // nil digests (JSON null) refuse the request instead of panicking
    fi.Sha1.nx = 3;
    fi.has_sha1 = false;
    CHECK(!SaveFileInfo(dir + "/dir/file.txt", fi), "save");
    w = c.send(3, -1, "def");
    CHECK(w.Code == 500, "nil digest: %d", w.Code);
  }
}

// sha1file_test.go:10-64 over a real file, plus the two errors of sha1file.go
static void test_sha1file(const std::string& root) {
  const std::string content = "the quick brown fox jumps over the lazy dog\n";
  const std::string p = root + "/test-sha1-file";
  FILE* f = fopen(p.c_str(), "wb");
  fwrite(content.data(), 1, content.size(), f);
  fclose(f);
  FileReader* fr = nullptr;
  CHECK(!FileReader::Open(p, &fr), "open");
  Sha1File* sf = nullptr;
  CHECK(!Sha1File::New(fr, g_ctx, &sf), "NewSha1File");
  auto seek_and_read = [&](int64_t seek, size_t read, const std::string& want) {  // testSeekAndRead
    Error e;
    const int64_t m = sf->Seek(seek, 0, &e);
    CHECK(!e && m == seek, "seek %lld: %s", (long long)seek, e.msg.c_str());
    std::vector<uint8_t> b(read);
    const size_t n = sf->Read(b.data(), read, &e);
    CHECK(!e && n == read, "read %zu: got %zu %s", read, n, e.msg.c_str());
    CHECK(std::string(b.begin(), b.end()) == want, "content at %lld", (long long)seek);
  };
  seek_and_read(0, 9, content.substr(0, 9));
  seek_and_read(2, 3, content.substr(2, 3));   // do not pass sf.calculated
  seek_and_read(2, 7, content.substr(2, 7));   // read exactly up to sf.calculated
  seek_and_read(2, 9, content.substr(2, 9));   // read beyond sf.calculated
  seek_and_read(11, content.size() - 11, content.substr(11));  // the rest
  uint8_t d[20];
  CHECK(!sf->Sum(d) && hexs(d, 20) == "5d2781d78fa5a97b7bafa849fe933dfc9dc93eba", "TestSha1File KAT: %s",
        hexs(d, 20).c_str());
  Error e;
  sf->Seek(40, 0, &e);
  uint8_t b[4];
  sf->Read(b, 4, &e);
  CHECK(!e, "read within calculated");
  delete sf;
  delete fr;

  // forward seeks and reads past `calculated` fail as in Go
  BytesReader br(content);
  CHECK(!Sha1File::New(&br, g_ctx, &sf), "NewSha1File");
  sf->Seek(5, 0, &e);
  CHECK(e && e.msg == "seeking forward is not supported", "forward seek: %s", e.msg.c_str());
  sf->Read(b, 4, &e);  // the underlying reader moved, Sha1File's position did not
  CHECK(!e, "read after refused seek");
  delete sf;
  BytesReader br2(content);
  CHECK(!Sha1File::New(&br2, g_ctx, &sf), "NewSha1File");
  uint8_t big[64];
  sf->Read(big, 10, &e);
  sf->Seek(3, 0, &e);
  sf->Read(big, 4, &e);  // position 7 <= calculated 10
  CHECK(!e, "re-read");
  delete sf;
}

static uint64_t rnd(uint64_t* s) {
  *s ^= *s >> 12;
  *s ^= *s << 25;
  *s ^= *s >> 27;
  return *s * 0x2545F4914F6CDD1Dull;
}

// ---- write.go sendFile against the receiver: client-side Sha1File and server-side saveFile both
// on the GPU, with the connection failing mid-request ------------------------------------------
// A transport that, for some PATCHes, delivers only the first k body bytes to the server (which
// keeps them: io.Copy's error is ignored, filereceiver.go:209), loses up to `lost` more bytes in
// flight (read from the client's Sha1File, never delivered) and reports a connection error.
struct FlakyTransport : Transport {
  FileReceiver* fr;
  uint64_t s;
  int fail_percent;
  long failures = 0;
  FlakyTransport(FileReceiver* f, uint64_t seed, int pct) : fr(f), s(seed | 1), fail_percent(pct) {}
  uint64_t next() {
    s ^= s >> 12; s ^= s << 25; s ^= s >> 27;
    return s * 0x2545F4914F6CDD1Dull;
  }
  struct Cut : Reader {  // the first k bytes, then a broken connection
    Reader& r;
    size_t left;
    Cut(Reader& rr, size_t k) : r(rr), left(k) {}
    size_t Read(uint8_t* p, size_t cap, Error* err) override {
      if (left == 0) {
        *err = make_error(ERR_TRANSPORT, "read: connection reset by peer");
        return 0;
      }
      const size_t n = r.Read(p, std::min(cap, left), err);
      left -= n;
      return n;
    }
  };
  Response RoundTrip(const Request& r, Error* err) override {
    *err = Error{};
    if (r.Method != "PATCH" || !r.Body || (int)(next() % 100) >= fail_percent) return fr->ServeHTTP(r);
    ++failures;
    Cut cut(*r.Body, (size_t)(next() % 100000));
    Request q = r;
    q.Body = &cut;
    fr->ServeHTTP(q);  // the server keeps what arrived
    std::vector<uint8_t> lost(next() % 70000);  // in flight when the connection broke
    Error e;
    if (!lost.empty()) r.Body->Read(lost.data(), lost.size(), &e);
    *err = make_error(ERR_TRANSPORT, "write: broken pipe");
    return Response{};
  }
};

static void expect_checksums(const Checksums& cs, const std::string& data, const char* what) {
  uint8_t sha[20];
  uint32_t crc;
  oracle_hash_message(reinterpret_cast<const uint8_t*>(data.data()), data.size(), 32768, sha, &crc);
  char c[9];
  snprintf(c, sizeof c, "%08x", crc);
  CHECK(cs.Sha1 == hexs(sha, 20) && cs.CRC32 == c, "%s: checksums %s %s want %s %s", what, cs.Sha1.c_str(),
        cs.CRC32.c_str(), hexs(sha, 20).c_str(), c);
}

static void test_client_send_file(const std::string& root) {
  {  // TestClient's content (client_test.go:158-171) through sendFile, known and unknown size
    const std::string dir = fresh_dir(root, "client");
    FileReceiver fr(dir, g_hasher);
    LocalTransport t(&fr);
    const std::string fox = "the quick brown fox jumps over the lazy dog\n";
    for (int64_t size : {(int64_t)fox.size(), (int64_t)-1}) {
      BytesReader rs(fox);
      Checksums cs;
      ClientConfig cfg;
      cfg.ChunkSize = 16;  // three PATCHes
      Error e = sendFile(t, g_ctx, "/0/000/1.fid", rs, size, cfg, &cs);
      CHECK(!e, "sendFile(size %lld): %s", (long long)size, e.msg.c_str());
      CHECK(cs.Sha1 == "5d2781d78fa5a97b7bafa849fe933dfc9dc93eba" && cs.CRC32 == "28c3debf", "fox KAT via sendFile: %s %s",
            cs.Sha1.c_str(), cs.CRC32.c_str());
      CHECK(slurp(dir + "/0/000/1.fid") == fox, "uploaded content");
    }
    {  // the drainer's client (drain.go:124 through write.go:163-165): every PATCH says efes-drain
      struct Recording : Transport {
        LocalTransport inner;
        int patches = 0, drain = 0, heads = 0;
        explicit Recording(FileReceiver* f) : inner(f) {}
        Response RoundTrip(const Request& r, Error* err) override {
          if (r.Method == "PATCH") {
            ++patches;
            auto it = r.Headers.find("Efes-Drain");
            if (it != r.Headers.end() && it->second == "true") ++drain;
          } else if (r.Method == "HEAD") {
            ++heads;
          }
          return inner.RoundTrip(r, err);
        }
      } rec(&fr);
      for (bool drainer : {true, false}) {
        rec.patches = rec.drain = rec.heads = 0;
        BytesReader rs(fox);
        Checksums cs;
        ClientConfig cfg;
        cfg.ChunkSize = 10;
        cfg.Drainer = drainer;
        Error e = sendFile(rec, g_ctx, "/0/000/2.fid", rs, (int64_t)fox.size(), cfg, &cs);
        CHECK(!e && cs.Sha1 == "5d2781d78fa5a97b7bafa849fe933dfc9dc93eba", "drainer=%d sendFile: %s", (int)drainer,
              e.msg.c_str());
        CHECK(rec.patches == 5 && rec.heads == 0 && rec.drain == (drainer ? 5 : 0),
              "drainer=%d: %d PATCHes, %d with efes-drain, %d HEADs", (int)drainer, rec.patches, rec.drain, rec.heads);
      }
    }
    BytesReader rs(fox);
    Checksums cs;
    struct NotFound : Transport {  // 404 is permanent (write.go:98-100)
      Response RoundTrip(const Request&, Error* err) override {
        *err = Error{};
        Response w;
        w.Code = 404;
        w.Body = "tempfile does not exist\n";
        return w;
      }
    } nf;
    Error e = sendFile(nf, g_ctx, "/x.fid", rs, (int64_t)fox.size(), ClientConfig{}, &cs);
    CHECK(e.code == ERR_HTTP && e.status == 404, "404: %d %s", e.code, e.msg.c_str());
  }
  // random objects over a connection that breaks in a third of the PATCHes, 8 clients at once
  const std::string dir = fresh_dir(root, "client_flaky");
  std::atomic<long> failures{0}, objects{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      FileReceiver fr(dir, g_hasher);
      FlakyTransport ft(&fr, 0x1234567ull * (uint64_t)(t + 1), 33);
      uint64_t s = 77 + (uint64_t)t;
      for (int u = 0; u < 5 && !g_fail; ++u) {
        const size_t len = (rnd(&s) % 5 == 0) ? rnd(&s) % 100 : rnd(&s) % (3u << 20);
        std::string obj(len, '\0');
        oracle_fill_synthetic(reinterpret_cast<uint8_t*>(&obj[0]), len, rnd(&s));
        BytesReader rs(obj, 1 + rnd(&s) % 40000);
        ClientConfig cfg;
        cfg.ChunkSize = (int64_t)(1 + rnd(&s) % (1u << 20));
        cfg.MaxAttempts = 1000;
        const int64_t size = rnd(&s) % 3 ? (int64_t)len : -1;
        const std::string path = "/c" + std::to_string(t) + "/" + std::to_string(u) + ".fid";
        Checksums cs;
        Error e = sendFile(ft, g_ctx, path, rs, size, cfg, &cs);
        CHECK(!e, "flaky sendFile %s (len %zu, chunk %lld): %s", path.c_str(), len, (long long)cfg.ChunkSize,
              e.msg.c_str());
        if (!e) expect_checksums(cs, obj, path.c_str());
        CHECK(slurp(dir + path) == obj, "%s: server file content", path.c_str());
        ++objects;
      }
      failures += ft.failures;
    });
  for (auto& x : th) x.join();
  printf("sendFile: %ld objects over a flaky connection, %ld broken PATCHes resumed\n", objects.load(), failures.load());
  CHECK(failures > 10, "the flaky transport broke PATCHes");
}

// Concurrent resumable uploads through ServeHTTP, each thread with its own objects; every
// intermediate .info is compared byte for byte with what Go would write after the same Writes.
struct Up {
  int id;
  long patches = 0, bytes = 0;
};


static void upload_worker(const std::string& dir, int uploads, Up* a, Hasher* hasher) {
  FileReceiver fr(dir, hasher);
  uint64_t s = 0x9E3779B97F4A7C15ull ^ (uint64_t)(a->id + 1) * 0xD1B54A32D192ED03ull;
  for (int u = 0; u < uploads && !g_fail; ++u) {
    Client c{&fr};
    c.path = "/dev" + std::to_string(a->id % 3) + "/0/000/" + std::to_string(a->id * 1000 + u) + ".fid";
    const size_t len = (rnd(&s) % 4 == 0) ? rnd(&s) % 200 : rnd(&s) % (3u << 20);
    std::string obj(len, '\0');
    oracle_fill_synthetic(reinterpret_cast<uint8_t*>(&obj[0]), len, rnd(&s));
    const bool with_length = rnd(&s) % 2;
    oracle_sha1 os = o_new_sha1();
    oracle_crc32 oc;
    oracle_crc32_reset(&oc);
    if (rnd(&s) % 2) c.create();
    size_t off = 0;
    do {
      size_t n = (rnd(&s) % 3 == 0) ? rnd(&s) % 70000 : (size_t)(1 + rnd(&s) % (1u << 20));
      if (n > len - off) n = len - off;
      const size_t max_read = (rnd(&s) % 3 == 0) ? 1 + rnd(&s) % 5000 : SIZE_MAX;  // socket read sizes
      Response w = c.send((int64_t)off, with_length ? (int64_t)len : -1, obj.substr(off, n), max_read);
      for (size_t q = 0; q < n;) {  // the Writes io.Copy made: min(32 KiB, read size, rest)
        const size_t m = std::min(std::min<size_t>(32768, max_read), n - q);
        oracle_sha1_write(&os, reinterpret_cast<const uint8_t*>(obj.data()) + off + q, m);
        oracle_crc32_write(&oc, reinterpret_cast<const uint8_t*>(obj.data()) + off + q, m);
        q += m;
      }
      off += n;
      a->patches++;
      CHECK(w.Code == 200 && w.Headers["efes-file-offset"] == std::to_string(off), "upload %s PATCH at %zu: %d %s",
            c.path.c_str(), off, w.Code, w.Body.c_str());
      const std::string info = dir + c.path + ".info";
      if (with_length && off == len) {
        check_done(w, obj, c.path.c_str());
        CHECK(!exists(info), "%s: .info left after the last PATCH", c.path.c_str());
      } else {
        bool ok;
        const std::string got = slurp(info, &ok);
        CHECK(ok && got == go_info((int64_t)off, os, oc), "%s .info at %zu:\n got  %s want %s", c.path.c_str(), off,
              got.c_str(), go_info((int64_t)off, os, oc).c_str());
      }
    } while (off < len && !g_fail);
    CHECK(slurp(dir + c.path) == obj, "%s: file contents", c.path.c_str());
    if (!with_length) {  // no length header: the client DELETEs (write.go's createClose path)
      c.offset((int64_t)len);
      c.del();
    }
    a->bytes += (long)len;
  }
}

static void test_concurrent_uploads(const std::string& root, int threads, int uploads, Hasher* hasher,
                                    const char* name) {
  const std::string dir = fresh_dir(root, name);
  std::vector<Up> args(threads);
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) {
    args[t].id = t;
    th.emplace_back(upload_worker, dir, uploads, &args[t], hasher);
  }
  long patches = 0, bytes = 0;
  for (int t = 0; t < threads; ++t) {
    th[t].join();
    patches += args[t].patches;
    bytes += args[t].bytes;
  }
  printf("%s: %d threads x %d uploads, %ld PATCHes, %ld bytes, PATCHes per device:", name, threads, uploads, patches,
         bytes);
  for (size_t d = 0; d < hasher->devices(); ++d) printf(" %llu", (unsigned long long)hasher->served(d));
  printf("\n");
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s cpu|gpu <tmpdir> [threads] [uploads] [copybuf|reserve]\n", argv[0]);
    return 2;
  }
  const std::string mode = argv[1], root = argv[2];
  oracle_crc32_init_tables();
  if (mode == "cpu") {
    test_parse_int();
    test_join_path();
    test_offset_mismatch_text();
    test_json();
    test_fileinfo_files(root);
    test_handler_cpu(root);
  } else if (mode == "gpu") {
    const int threads = argc > 3 ? atoi(argv[3]) : 16;
    const int uploads = argc > 4 ? atoi(argv[4]) : 4;
    if (argc > 5 && !strcmp(argv[5], "reserve")) SetSaveFileCopyBuffer(false);  // efes_upload_reserve/commit
    int rc = efes_ctx_create(0, &g_ctx);
    if (rc) {
      fprintf(stderr, "efes_ctx_create: %s\n", efes_strerror(rc));
      return 1;
    }
    Error e = Hasher::Create(g_ctx, 256 << 10, 512, 64, &g_hasher);
    if (e) {
      fprintf(stderr, "Hasher::Create: %s\n", e.msg.c_str());
      return 1;
    }
    test_file_receiver(root);
    if (!g_fail) test_save_file_errors(root);
    if (!g_fail) test_sha1file(root);
    if (!g_fail) test_client_send_file(root);
    if (!g_fail) test_concurrent_uploads(root, threads, uploads, g_hasher, "uploads");
    delete g_hasher;
    // Several GPUs in one process: one queue per context, each PATCH on the least-loaded one
    // (two contexts on device 0 stand in for two GPUs on a one-GPU box).
    efes_ctx* ctx2 = nullptr;
    if (!g_fail && (rc = efes_ctx_create(0, &ctx2)) == 0) {
      Hasher* multi = nullptr;
      Error me = Hasher::Create(std::vector<efes_ctx*>{g_ctx, ctx2}, 256 << 10, 512, 32, &multi);
      CHECK(!me, "multi-device Hasher: %s", me.msg.c_str());
      if (multi) {
        test_concurrent_uploads(root, threads, uploads, multi, "uploads over 2 queues");
        CHECK(multi->served(0) > 0 && multi->served(1) > 0, "both devices served PATCHes");
        delete multi;
      }
      efes_ctx_destroy(ctx2);
    } else if (!g_fail) {
      CHECK(false, "second context: %s", efes_strerror(rc));
    }
    efes_ctx_destroy(g_ctx);
  } else {
    fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  }
  if (g_fail) return 1;
  printf("receiver_test %s ok (%d checks)\n", mode.c_str(), g_checks);
  return 0;
}
