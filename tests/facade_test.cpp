// facade_test.cpp -- the reference's packed-serialization tests (capnproto c++/src/capnp/
// serialize-packed-test.c++) restated against the cpk_capnp façade (include/cpk_capnp.h), i.e.
// the reference API running on the MI355X codec.  Fixtures are the reference's own testdata
// files and KATs, committed under tests/golden/.
//
//   cpk_facade_test <tests/golden dir>        exit 0 = all checks passed
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "cpk_capnp.h"

using namespace cpk_capnp;

static int g_fail = 0, g_pass = 0;
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (cond) {                                            \
      g_pass++;                                            \
    } else {                                               \
      g_fail++;                                            \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                        \
      fprintf(stderr, "\n");                               \
    }                                                      \
  } while (0)

static std::vector<byte> read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<byte>(std::istreambuf_iterator<char>(f), {});
}

// Unpacked message file (stream framing) -> segments over its words.
static std::vector<ArrayPtr<const word>> segments_of(const std::vector<byte>& msg) {
  const uint32_t* t = reinterpret_cast<const uint32_t*>(msg.data());
  const uint32_t n = t[0] + 1;
  const word* w = reinterpret_cast<const word*>(msg.data());
  size_t at = n / 2 + 1;
  std::vector<ArrayPtr<const word>> segs;
  for (uint32_t i = 0; i < n; i++) {
    segs.push_back(ArrayPtr<const word>(w + at, t[i + 1]));
    at += t[i + 1];
  }
  return segs;
}

static bool same(ArrayPtr<const byte> a, const std::vector<byte>& b) {
  return a.size() == b.size() && (a.size() == 0 || memcmp(a.begin(), b.data(), a.size()) == 0);
}

static std::vector<byte> hex(const char* s) {
  std::vector<byte> v;
  for (; s[0] && s[1]; s += 2) {
    unsigned x;
    sscanf(s, "%2x", &x);
    v.push_back((byte)x);
  }
  return v;
}

// serialize-packed-test.c++:203-220 style: one chunk through PackedOutputStream, and back.
static void kat_chunks(const std::string& dir) {
  std::ifstream f(dir + "/kats.txt");
  std::string u, p;
  int n = 0;
  while (f >> u >> p) {
    if (u == "-") u.clear();
    if (p == "-") p.clear();
    std::vector<byte> unpacked = hex(u.c_str()), packed = hex(p.c_str());
    VectorOutputStream out;
    _::PackedOutputStream pk(out);
    pk.write(unpacked.data(), unpacked.size());
    CHECK(same(out.getArray(), packed), "KAT %d pack", n);
    if (!unpacked.empty()) {
      // serialize-packed-test.c++:85-101: and back through PackedInputStream
      ArrayInputStream ain(ArrayPtr<const byte>(packed.data(), packed.size()));
      _::PackedInputStream pin(ain);
      std::vector<byte> back(unpacked.size());
      pin.InputStream::read(back.data(), back.size());
      CHECK(back == unpacked, "KAT %d PackedInputStream::read", n);
      CHECK(ain.tryGetReadBuffer().size() == 0, "KAT %d read consumed the input", n);
      ArrayInputStream ain2(ArrayPtr<const byte>(packed.data(), packed.size()));
      _::PackedInputStream pin2(ain2);
      pin2.skip(unpacked.size());
      CHECK(ain2.tryGetReadBuffer().size() == 0, "KAT %d PackedInputStream::skip", n);
    }
    n++;
  }
  CHECK(n >= 10, "KATs read: %d", n);
}

// testdata/binary <-> testdata/packed, testdata/segmented <-> testdata/segmented-packed
// (capnp-test.sh golden files).
static void fixtures(const std::string& dir, const char* unpacked_name, const char* packed_name) {
  std::vector<byte> msg = read_file(dir + "/" + unpacked_name);
  std::vector<byte> packed = read_file(dir + "/" + packed_name);
  auto segs = segments_of(msg);
  VectorOutputStream out;
  writePackedMessage(out, ArrayPtr<const ArrayPtr<const word>>(segs.data(), segs.size()));
  CHECK(same(out.getArray(), packed), "%s: writePackedMessage bytes (%zu vs %zu)", packed_name,
        out.getArray().size(), packed.size());

  ArrayInputStream in(ArrayPtr<const byte>(packed.data(), packed.size()));
  PackedMessageReader reader(in);
  CHECK(reader.segmentCount() == segs.size(), "%s: segment count", packed_name);
  bool eq = true;
  for (size_t i = 0; i < segs.size(); i++) {
    auto s = reader.getSegment((unsigned)i);
    eq = eq && s.size() == segs[i].size() && memcmp(s.begin(), segs[i].begin(), 8 * s.size()) == 0;
  }
  CHECK(eq, "%s: PackedMessageReader segments", packed_name);
  CHECK(in.tryGetReadBuffer().size() == 0, "%s: reader consumed the whole message", packed_name);
  CHECK(computeUnpackedSizeInWords(ArrayPtr<const byte>(packed.data(), packed.size())) ==
            msg.size() / 8,
        "%s: computeUnpackedSizeInWords", packed_name);
}

// The reader's segments against a message's segments.
static bool same_message(PackedMessageReader& r, const std::vector<ArrayPtr<const word>>& segs) {
  if (r.segmentCount() != segs.size()) return false;
  for (size_t i = 0; i < segs.size(); i++) {
    auto s = r.getSegment((unsigned)i);
    if (s.size() != segs[i].size() || memcmp(s.begin(), segs[i].begin(), 8 * s.size()) != 0)
      return false;
  }
  return r.getSegment((unsigned)segs.size()).size() == 0;
}

// serialize-packed-test.c++:348-371: two messages back to back in one stream, the second read
// after the first; also with a scratch space and through a file descriptor.
static void two_messages(const std::string& dir) {
  std::vector<byte> a = read_file(dir + "/binary"), b = read_file(dir + "/segmented");
  auto sa = segments_of(a), sb = segments_of(b);
  VectorOutputStream out;
  writePackedMessage(out, ArrayPtr<const ArrayPtr<const word>>(sa.data(), sa.size()));
  writePackedMessage(out, ArrayPtr<const ArrayPtr<const word>>(sb.data(), sb.size()));
  auto all = out.getArray();
  ArrayInputStream in(all);
  {
    std::vector<word> scratch(8);
    PackedMessageReader r1(in, ReaderOptions(), ArrayPtr<word>(scratch.data(), scratch.size()));
    CHECK(same_message(r1, sa), "first message");
  }
  {
    PackedMessageReader r2(in);
    CHECK(same_message(r2, sb), "second message");
  }
  CHECK(in.tryGetReadBuffer().size() == 0, "stream drained");

  // lazy segments (serialize.c++:264-302): the multi-segment message first, only segment 0
  // looked at -- the destructor skips the rest, so the next message reads cleanly
  {
    VectorOutputStream o2;
    writePackedMessage(o2, ArrayPtr<const ArrayPtr<const word>>(sb.data(), sb.size()));
    writePackedMessage(o2, ArrayPtr<const ArrayPtr<const word>>(sa.data(), sa.size()));
    ArrayInputStream in2(o2.getArray());
    {
      std::vector<word> scratch(b.size() / 8);  // large enough: segments land in it
      PackedMessageReader r1(in2, ReaderOptions(), ArrayPtr<word>(scratch.data(), scratch.size()));
      auto s0 = r1.getSegment(0);
      CHECK(s0.size() == sb[0].size() && memcmp(s0.begin(), sb[0].begin(), 8 * s0.size()) == 0 &&
                (const void*)s0.begin() == (const void*)scratch.data(),
            "lazy: segment 0 in the caller's scratch");
    }
    PackedMessageReader r2(in2);
    CHECK(same_message(r2, sa), "lazy: next message after the destructor's skip");
    CHECK(in2.tryGetReadBuffer().size() == 0, "lazy: stream drained");
  }

  // through a pipe: the reader refills across small buffers
  int fds[2];
  if (pipe(fds) == 0) {
    writePackedMessageToFd(fds[1], ArrayPtr<const ArrayPtr<const word>>(sb.data(), sb.size()));
    writePackedMessageToFd(fds[1], ArrayPtr<const ArrayPtr<const word>>(sa.data(), sa.size()));
    close(fds[1]);
    {
      PackedFdMessageReader f1(fds[0]);
      CHECK(same_message(f1, sb), "fd: first message");
    }
    close(fds[0]);
  }
  // serialize-packed.h:82-83: the OwnFd overload closes the descriptor with the reader
  if (pipe(fds) == 0) {
    writePackedMessageToFd(fds[1], ArrayPtr<const ArrayPtr<const word>>(sa.data(), sa.size()));
    close(fds[1]);
    {
      PackedFdMessageReader f2{OwnFd(fds[0])};
      CHECK(same_message(f2, sa), "OwnFd: message");
    }
    CHECK(fcntl(fds[0], F_GETFD) == -1, "OwnFd: descriptor closed with the reader");
  }
}

// Error behaviour: the reference's exceptions (serialize-packed-test.c++:297-346).
static void errors(const std::string& dir) {
  std::vector<byte> packed = read_file(dir + "/packed");
  for (size_t cut : {(size_t)0, (size_t)1, packed.size() / 2, packed.size() - 1}) {
    ArrayInputStream in(ArrayPtr<const byte>(packed.data(), cut));
    bool threw = false;
    cpk_status st = CPK_OK;
    try {
      PackedMessageReader r(in);
    } catch (const Exception& e) {
      threw = true;
      st = e.status();
    }
    CHECK(threw && st == CPK_ERR_PREMATURE_EOF, "truncated at %zu -> premature EOF (got %d)",
          cut, (int)st);
  }
  // a zero run that overshoots the message (table says 1 word, the run says 3)
  {
    std::vector<byte> bad = {0x10, 0x01, 0x00, 0x02};  // table: 1 segment of 1 word; then 00 02
    ArrayInputStream in(ArrayPtr<const byte>(bad.data(), bad.size()));
    cpk_status st = CPK_OK;
    try {
      PackedMessageReader r(in);
    } catch (const Exception& e) {
      st = e.status();
    }
    CHECK(st == CPK_ERR_RUN_OVERSHOOT, "run overshoot (got %d)", (int)st);
  }
  // traversal limit (serialize.c++:235)
  {
    std::vector<byte> msg = read_file(dir + "/binary");
    auto segs = segments_of(msg);
    VectorOutputStream out;
    writePackedMessage(out, ArrayPtr<const ArrayPtr<const word>>(segs.data(), segs.size()));
    ArrayInputStream in(out.getArray());
    ReaderOptions opt;
    opt.traversalLimitInWords = 4;
    cpk_status st = CPK_OK;
    try {
      PackedMessageReader r(in, opt);
    } catch (const Exception& e) {
      st = e.status();
    }
    CHECK(st == CPK_ERR_MESSAGE_TOO_LARGE, "traversal limit (got %d)", (int)st);
  }
  // writing an empty message
  {
    VectorOutputStream out;
    cpk_status st = CPK_OK;
    try {
      writePackedMessage(out, ArrayPtr<const ArrayPtr<const word>>());
    } catch (const Exception& e) {
      st = e.status();
    }
    CHECK(st == CPK_ERR_EMPTY_MESSAGE, "empty message (got %d)", (int)st);
  }
  // computeUnpackedSizeInWords on truncated input: "invalid packed data"
  {
    std::vector<byte> t = {0xff, 1, 2, 3};
    cpk_status st = CPK_OK;
    try {
      computeUnpackedSizeInWords(ArrayPtr<const byte>(t.data(), t.size()));
    } catch (const Exception& e) {
      st = e.status();
    }
    CHECK(st == CPK_ERR_INVALID_PACKED, "invalid packed data (got %d)", (int)st);
  }
  // ArrayOutputStream capacity
  {
    std::vector<byte> small(4);
    ArrayOutputStream out(ArrayPtr<byte>(small.data(), small.size()));
    std::vector<byte> msg = read_file(dir + "/binary");
    auto segs = segments_of(msg);
    cpk_status st = CPK_OK;
    try {
      writePackedMessage(out, ArrayPtr<const ArrayPtr<const word>>(segs.data(), segs.size()));
    } catch (const Exception& e) {
      st = e.status();
    }
    CHECK(st == CPK_ERR_CAPACITY, "ArrayOutputStream capacity (got %d)", (int)st);
  }
}

// _::PackedInputStream on its own (serialize-packed.c++:34-299): reads split at record
// boundaries, refills across small buffers, and its exceptions.
static void input_stream(const std::string& dir) {
  std::vector<byte> msg = read_file(dir + "/binary"), packed = read_file(dir + "/packed");
  {  // two reads split at a word boundary the records respect: the segment table, then the rest
    ArrayInputStream ain(ArrayPtr<const byte>(packed.data(), packed.size()));
    _::PackedInputStream pin(ain);
    std::vector<byte> back(msg.size());
    pin.InputStream::read(back.data(), 8);
    pin.InputStream::read(back.data() + 8, back.size() - 8);
    CHECK(back == msg, "PackedInputStream: table, then segments");
    CHECK(ain.tryGetReadBuffer().size() == 0, "PackedInputStream: input consumed");
  }
  int fds[2];
  if (pipe(fds) == 0) {  // 7-byte stream buffers: every read spans refills
    if (write(fds[1], packed.data(), packed.size()) != (ssize_t)packed.size()) g_fail++;
    close(fds[1]);
    FdBufferedInputStream fin(fds[0], 7);
    _::PackedInputStream pin(fin);
    std::vector<byte> back(msg.size());
    pin.InputStream::read(back.data(), back.size());
    CHECK(back == msg, "PackedInputStream over 7-byte buffers");
    close(fds[0]);
  }
  auto expect = [](const char* hexin, size_t minB, size_t maxB, cpk_status want, size_t got_bytes,
                   const char* what) {
    std::vector<byte> in = hex(hexin);
    ArrayInputStream ain(ArrayPtr<const byte>(in.data(), in.size()));
    _::PackedInputStream pin(ain);
    std::vector<word> out(maxB / 8 + 1);
    cpk_status st = CPK_OK;
    size_t n = 0;
    try {
      n = pin.tryRead(out.data(), minB, maxB);
    } catch (const Exception& e) {
      st = e.status();
    }
    CHECK(st == want && (st != CPK_OK || n == got_bytes), "%s: status %d bytes %zu", what,
          (int)st, n);
  };
  expect("", 8, 8, CPK_OK, 0, "empty input reads nothing");
  expect("0001", 8, 8, CPK_ERR_RUN_OVERSHOOT, 0, "zero run crossing the read");
  expect("ff0102", 8, 8, CPK_ERR_PREMATURE_EOF, 0, "truncated record");
  expect("0000", 8, 16, CPK_OK, 8, "input ends at a record boundary past minBytes");
  expect("0000", 16, 16, CPK_ERR_PREMATURE_EOF, 0, "input ends before minBytes");
}

// A stream that hands out fixed-size buffers (the buffer boundaries fall every `chunk` bytes
// of the stream, like a buffered reader over a socket delivering that much at a time).
class ChunkedInput : public BufferedInputStream {
 public:
  ChunkedInput(const std::vector<byte>& d, size_t chunk) : d_(d), chunk_(chunk) {}
  ArrayPtr<const byte> tryGetReadBuffer() override {
    const size_t end = std::min(d_.size(), (pos_ / chunk_ + 1) * chunk_);
    return ArrayPtr<const byte>(d_.data() + pos_, end - pos_);
  }
  size_t tryRead(void* buffer, size_t minBytes, size_t maxBytes) override {
    (void)minBytes;
    const size_t n = std::min(maxBytes, d_.size() - pos_);
    memcpy(buffer, d_.data() + pos_, n);
    pos_ += n;
    return n;
  }
  void skip(size_t bytes) override {
    if (bytes > d_.size() - pos_) throw Exception(CPK_ERR_PREMATURE_EOF, "ChunkedInput::skip");
    pos_ += bytes;
  }
  size_t pos() const { return pos_; }

 private:
  const std::vector<byte>& d_;
  size_t chunk_, pos_ = 0;
};

// The reference's PackedInputStream::tryRead stopping rules (serialize-packed.c++:34-183),
// restated over the same chunked stream as a model: returns the bytes produced and leaves
// *pos where the reference leaves the stream; throws the reference's failure as a cpk_status.
static size_t model_try_read(const std::vector<byte>& d, size_t chunk, size_t* pos, size_t minB,
                             size_t maxB) {
  auto chunk_end = [&](size_t p) { return std::min(d.size(), (p / chunk + 1) * chunk); };
  size_t in = *pos, end = chunk_end(in), out = 0;
  if (in == end) return 0;
  auto refresh = [&]() {  // REFRESH_BUFFER
    in = end;
    end = chunk_end(in);
    if (in == end) throw CPK_ERR_PREMATURE_EOF;
  };
  for (;;) {
    unsigned tag;
    if (end - in < 10) {
      if (out >= minB) {
        *pos = in;
        return out;
      }
      if (end == in) {
        refresh();
        continue;
      }
      tag = d[in++];
      for (int i = 0; i < 8; i++) {
        if (tag & (1u << i)) {
          if (in == end) refresh();
          in++;
        }
        out++;
      }
      if (in == end && (tag == 0 || tag == 0xff)) refresh();
    } else {
      tag = d[in++];
      in += __builtin_popcount(tag);
      out += 8;
    }
    if (tag == 0 || tag == 0xff) {
      const size_t run = 8 * (size_t)d[in++];
      if (run > maxB - out) throw CPK_ERR_RUN_OVERSHOOT;
      if (tag == 0 || end - in >= run) {
        if (tag == 0xff) in += run;
        out += run;
      } else {
        // the rest of the run is read straight from the stream, then a new buffer is required
        const size_t rest = run - (end - in);
        if (rest > d.size() - end) throw CPK_ERR_PREMATURE_EOF;
        in = end + rest;
        out += run;
        if (out == maxB) {
          *pos = in;
          return maxB;
        }
        end = chunk_end(in);
        if (in == end) throw CPK_ERR_PREMATURE_EOF;  // getReadBuffer() at the end of the stream
        continue;
      }
    }
    if (out == maxB) {
      *pos = in;
      return maxB;
    }
  }
}

// The façade's PackedInputStream against the model: same byte counts, same stream position,
// same failures, for every buffer size and (min, max) shape, reading the stream to its end.
static void stream_model(const std::string& dir) {
  for (const char* name : {"packed", "segmented-packed"}) {
    const std::vector<byte> packed = read_file(dir + "/" + name);
    const std::vector<byte> msg = read_file(dir + (strcmp(name, "packed") ? "/segmented" : "/binary"));
    for (size_t chunk : {1, 2, 7, 9, 10, 11, 16, 64, 100, 4096}) {
      for (int shape = 0; shape < 5; shape++) {
        ChunkedInput ci(packed, chunk);
        _::PackedInputStream pin(ci);
        size_t mpos = 0, done = 0;
        bool ok = true;
        for (int call = 0; call < 4096 && ok; call++) {
          const size_t left = msg.size() - done;
          size_t minB, maxB;
          switch (shape) {
            case 0: minB = maxB = left; break;                    // read()
            case 1: minB = 8; maxB = left; break;                 // as much as is buffered
            case 2: minB = 0; maxB = left; break;                 // whatever is at hand
            case 3: minB = maxB = std::min<size_t>(left, 24); break;  // word triples
            default: minB = 8; maxB = std::min<size_t>(left, 200); break;
          }
          if (maxB == 0) break;
          int want = 0, got = 0;
          size_t nm = 0, nf = 0;
          try {
            nm = model_try_read(packed, chunk, &mpos, minB, maxB);
          } catch (cpk_status e) {
            want = e;
          }
          std::vector<byte> buf(maxB);
          try {
            nf = pin.tryRead(buf.data(), minB, maxB);
          } catch (const Exception& e) {
            got = e.status();
          }
          ok = want == got && (want || (nm == nf && mpos == ci.pos() &&
                                        memcmp(buf.data(), msg.data() + done, nf) == 0));
          CHECK(ok, "%s chunk %zu shape %d call %d: model %zu B (err %d, pos %zu) vs facade %zu B (err %d, pos %zu)",
                name, chunk, shape, call, nm, want, mpos, nf, got, ci.pos());
          if (want || (nm == 0 && minB == 0 && mpos == packed.size())) break;
          done += nf;
          if (nf == 0 && minB == 0) break;
        }
      }
    }
  }
  // PackedInputStream::skip over small buffers consumes exactly the skipped records
  {
    const std::vector<byte> packed = read_file(dir + "/packed"), msg = read_file(dir + "/binary");
    ChunkedInput ci(packed, 7);
    _::PackedInputStream pin(ci);
    std::vector<byte> first(8);
    pin.InputStream::read(first.data(), 8);
    pin.skip(msg.size() - 8);
    CHECK(ci.pos() == packed.size() && memcmp(first.data(), msg.data(), 8) == 0,
          "skip over 7-byte buffers");
  }
  // tryRead(min < max) on a pipe whose writer stays open: returns what is there (:71-76)
  // instead of waiting for bytes that may never come
  int fds[2];
  if (pipe(fds) == 0) {
    const std::vector<byte> packed = read_file(dir + "/packed"), msg = read_file(dir + "/binary");
    if (write(fds[1], packed.data(), packed.size()) != (ssize_t)packed.size()) g_fail++;
    alarm(60);  // a hang fails the run instead of blocking it
    FdBufferedInputStream fin(fds[0]);
    _::PackedInputStream pin(fin);
    std::vector<byte> buf(msg.size() + 4096);
    const size_t n = pin.tryRead(buf.data(), 8, buf.size());
    alarm(0);
    size_t mpos = 0;
    const size_t nm = model_try_read(packed, 65536, &mpos, 8, buf.size());
    CHECK(n == nm && n >= 8 && memcmp(buf.data(), msg.data(), n) == 0,
          "pipe left open: tryRead(8, %zu) returned %zu (model %zu)", buf.size(), n, nm);
    close(fds[1]);
    close(fds[0]);
  }
}

// Config C1: samples/addressbook.c++ -- writeAddressBook packs with writePackedMessageToFd
// (:75), printAddressBook reads with PackedFdMessageReader (:79).  tests/golden/addressbook.bin
// is the sample's message, addressbook.packed the reference's bytes for it.
static void addressbook(const std::string& dir) {
  std::vector<byte> msg = read_file(dir + "/addressbook.bin");
  std::vector<byte> ref = read_file(dir + "/addressbook.packed");
  CHECK(msg.size() == 288 && ref.size() == 151, "addressbook fixtures present");
  if (msg.size() != 288) return;
  auto segs = segments_of(msg);
  int fds[2];
  if (pipe(fds) != 0) return;
  writePackedMessageToFd(fds[1], ArrayPtr<const ArrayPtr<const word>>(segs.data(), segs.size()));
  std::vector<byte> got(ref.size() + 16);
  const ssize_t n = read(fds[0], got.data(), got.size());
  got.resize(n > 0 ? (size_t)n : 0);
  CHECK(got == ref, "addressbook: writePackedMessageToFd bytes == reference (%zd B)", n);
  // the reader side of the sample: the same bytes back through a pipe
  writePackedMessageToFd(fds[1], ArrayPtr<const ArrayPtr<const word>>(segs.data(), segs.size()));
  close(fds[1]);
  {
    PackedFdMessageReader reader(fds[0]);
    CHECK(reader.segmentCount() == 1, "addressbook: one segment");
    auto s0 = reader.getSegment(0);
    CHECK(s0.size() == segs[0].size() && memcmp(s0.begin(), segs[0].begin(), s0.size() * 8) == 0,
          "addressbook: PackedFdMessageReader segment 0");
  }
  close(fds[0]);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "tests/golden";
  try {
    kat_chunks(dir);
    fixtures(dir, "binary", "packed");
    fixtures(dir, "segmented", "segmented-packed");
    two_messages(dir);
    errors(dir);
    input_stream(dir);
    stream_model(dir);
    addressbook(dir);
  } catch (const Exception& e) {
    fprintf(stderr, "unexpected exception: %s\n", e.what());
    return 2;
  }
  printf("facade: %d passed, %d failed\n", g_pass, g_fail);
  return g_fail ? 1 : 0;
}
