// cpk-convert -- the packed / flat-packed front-end of `capnp convert` on the device codec
// (compiler/capnp.c++:773-800 loop, :1027-1076 readers, :1096-1134
// writers).
//
//   cpk-convert <from>:<to> [--quiet] < input > output
//   formats: binary | packed | flat | flat-packed
//
// What the reference does per format, and what runs here:
//   read  binary       InputStreamMessageReader, one message after another (capnp.c++:1036-1039)
//                      -> host walk of the segment tables (the unpacked framing is not on the
//                      packed path; it is O(messages) header reads)
//   read  packed       PackedMessageReader, one after another (:1040-1043)
//                      -> cpk_split_packed_stream: the whole stream decoded and split on device
//   read  flat         all input as one segment, straggler bytes chopped (:1044-1061)
//   read  flat-packed  computeUnpackedSizeInWords + PackedInputStream::read, no bytes may be
//                      left (:1063-1076) -> cpk_unpacked_size + cpk_unpack_chunks
//   write binary       writeMessage (:1097-1103): table + segments
//   write packed       writePackedMessage (:1104-1111) -> cpk_pack_messages, the whole batch in
//                      one launch sequence
//   write flat         the single segment (:1112-1118)
//   write flat-packed  one PackedOutputStream::write of the segment (:1119-1127) -> cpk_pack_chunks
//
// Layout: the reference copies every message into a fresh MallocMessageBuilder (setRoot, or
// copyToUnchecked for flat) before writing it.  That is a pointer-tree copy (builders/readers,
// out of scope); this tool keeps each message's segments as they are.  For a
// message in the canonical single-segment layout the reference writes (every testdata file, and
// the reference's own convert tests capnp-test.sh:69-70) the output is the same; a multi-segment
// message converted to flat / flat-packed, which would need the re-layout, is refused.
// Traversal limits are lifted as in capnp.c++:1029-1031.  On a bad message the messages before it
// are written, the reference's message goes to stderr and the exit status is 1.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cpk.h"

namespace {

enum class Fmt { kBinary, kPacked, kFlat, kFlatPacked, kBad };

Fmt parse_fmt(const std::string& s) {
  if (s == "binary") return Fmt::kBinary;
  if (s == "packed") return Fmt::kPacked;
  if (s == "flat") return Fmt::kFlat;
  if (s == "flat-packed") return Fmt::kFlatPacked;
  return Fmt::kBad;
}

[[noreturn]] void die(int code, const std::string& msg) {
  fprintf(stderr, "cpk-convert: %s\n", msg.c_str());
  exit(code);
}

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) die(2, std::string(what) + ": " + hipGetErrorString(e));
}

void check(cpk_status s, const char* what) {
  if (s != CPK_OK) die(2, std::string(what) + ": " + cpk_status_string(s));
}

std::vector<uint8_t> read_all(int fd) {
  std::vector<uint8_t> buf;
  size_t n = 0;
  buf.resize(1 << 16);
  for (;;) {
    if (n == buf.size()) buf.resize(buf.size() * 2);
    const ssize_t r = ::read(fd, buf.data() + n, buf.size() - n);
    if (r < 0) die(2, "read failed");
    if (r == 0) break;
    n += (size_t)r;
  }
  buf.resize(n);
  return buf;
}

void write_all(const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  while (n > 0) {
    const ssize_t r = ::write(STDOUT_FILENO, b, n);
    if (r <= 0) die(2, "write failed");
    b += r;
    n -= (size_t)r;
  }
}

// Device buffer owned for the tool's lifetime.
template <typename T>
struct Dev {
  T* p = nullptr;
  explicit Dev(size_t n) { check_hip(hipMalloc(&p, (n ? n : 1) * sizeof(T)), "hipMalloc"); }
  ~Dev() { (void)hipFree(p); }
  Dev(const Dev&) = delete;
  Dev& operator=(const Dev&) = delete;
};

template <typename T>
void h2d(T* d, const T* h, size_t n) {
  if (n) check_hip(hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy");
}
template <typename T>
void d2h(T* h, const T* d, size_t n) {
  if (n) check_hip(hipMemcpy(h, d, n * sizeof(T), hipMemcpyDeviceToHost), "hipMemcpy");
}

// A batch of flat messages (segment table + segments each) back to back.
struct Batch {
  std::vector<uint64_t> words;
  std::vector<uint64_t> off{0};  // message i = words[off[i], off[i+1])
  int32_t stop = CPK_OK;         // why reading stopped early (CPK_OK: the input was consumed)
  size_t count() const { return off.size() - 1; }
};

const cpk_limits kNoLimit = {~0ull};

// writeMessage framing read back (serialize.c++:202-242, limits lifted): one message after
// another while input remains.
Batch read_binary(const std::vector<uint8_t>& in) {
  Batch b;
  const size_t nw = in.size() / 8;
  b.words.resize(nw);
  if (nw) memcpy(b.words.data(), in.data(), nw * 8);
  size_t pos = 0;  // bytes
  while (pos < in.size()) {
    if (in.size() - pos < 8) {
      b.stop = CPK_ERR_PREMATURE_EOF;
      break;
    }
    const uint64_t w0 = b.words[pos / 8];
    if ((uint32_t)w0 >= 511) {  // serialize.c++:214-221 (segCount-1 < 511)
      b.stop = CPK_ERR_TOO_MANY_SEGMENTS;
      break;
    }
    const uint32_t nseg = (uint32_t)w0 + 1;
    const uint64_t table_words = (nseg + 2) / 2;
    if ((in.size() - pos) / 8 < table_words) {
      b.stop = CPK_ERR_PREMATURE_EOF;
      break;
    }
    const uint32_t* t32 = reinterpret_cast<const uint32_t*>(in.data() + pos);
    uint64_t total = table_words;
    for (uint32_t s = 0; s < nseg; s++) total += t32[1 + s];
    if ((in.size() - pos) / 8 < total) {
      b.stop = CPK_ERR_PREMATURE_EOF;
      break;
    }
    pos += total * 8;
    b.off.push_back(pos / 8);
  }
  b.words.resize(b.off.back());
  return b;
}

// PackedMessageReader one after another (serialize-packed-test.c++:348-371 shape): the whole
// stream split and decoded on the device.
Batch read_packed(cpk_ctx* ctx, const std::vector<uint8_t>& in) {
  Batch b;
  if (in.empty()) return b;
  const uint64_t n = in.size();
  Dev<uint8_t> d_in(n);
  h2d(d_in.p, in.data(), n);
  // Capacity: computeUnpackedSizeInWords of the whole stream (runs never cross a message, so
  // the stream is one valid tag sequence); a truncated tail still decodes what precedes it.
  uint64_t cap = 0;
  {
    Dev<uint64_t> d_off(2), d_w(1);
    Dev<int32_t> d_st(1);
    const uint64_t off[2] = {0, n};
    h2d(d_off.p, off, 2);
    check(cpk_unpacked_size(ctx, d_in.p, n, d_off.p, 1, d_w.p, d_st.p, nullptr), "size");
    check(cpk_sync(ctx, nullptr), "size");
    int32_t st = 0;
    d2h(&cap, d_w.p, 1);
    d2h(&st, d_st.p, 1);
    if (st != CPK_OK) cap = n * 128 + 64;  // a zero run: 256 words per 2 bytes
  }
  const uint64_t max_msgs = n / 2 + 1;  // a message packs to >= 2 bytes
  Dev<uint64_t> d_words(cap), d_woff(max_msgs + 1), d_ioff(max_msgs + 1), d_n(1);
  Dev<int32_t> d_st(max_msgs + 1);
  check(cpk_split_packed_stream(ctx, d_in.p, n, d_words.p, cap, max_msgs, d_woff.p, d_ioff.p,
                                d_st.p, d_n.p, &kNoLimit, nullptr),
        "split");
  check(cpk_sync(ctx, nullptr), "split");
  uint64_t nm = 0;
  d2h(&nm, d_n.p, 1);
  b.off.resize(nm + 1);
  d2h(b.off.data(), d_woff.p, nm + 1);
  d2h(&b.stop, d_st.p + nm, 1);
  b.off[0] = 0;
  b.words.resize(b.off[nm]);
  d2h(b.words.data(), d_words.p, b.words.size());
  return b;
}

// One segment: the flat words (straggler bytes chopped, capnp.c++:1047-1054), as a message with
// a one-segment table.
Batch single_segment(const uint64_t* w, uint64_t nw) {
  Batch b;
  b.words.resize(1 + nw);
  b.words[0] = (uint64_t)nw << 32;  // segCount-1 = 0, size = nw (serialize.c++:311-330)
  if (nw) memcpy(b.words.data() + 1, w, nw * 8);
  b.off.push_back(1 + nw);
  return b;
}

Batch read_flat(const std::vector<uint8_t>& in) {
  std::vector<uint64_t> w(in.size() / 8);
  if (!w.empty()) memcpy(w.data(), in.data(), w.size() * 8);
  return single_segment(w.data(), w.size());
}

Batch read_flat_packed(cpk_ctx* ctx, const std::vector<uint8_t>& in) {
  const uint64_t n = in.size();
  Dev<uint8_t> d_in(n);
  h2d(d_in.p, in.data(), n);
  Dev<uint64_t> d_off(2), d_w(1), d_woff(2);
  Dev<int32_t> d_st(1);
  const uint64_t off[2] = {0, n};
  h2d(d_off.p, off, 2);
  check(cpk_unpacked_size(ctx, d_in.p, n, d_off.p, 1, d_w.p, d_st.p, nullptr), "size");
  check(cpk_sync(ctx, nullptr), "size");
  uint64_t nw = 0;
  int32_t st = 0;
  d2h(&nw, d_w.p, 1);
  d2h(&st, d_st.p, 1);
  if (st != CPK_OK) {
    Batch b;
    b.stop = st;
    return b;
  }
  const uint64_t woff[2] = {0, nw};
  h2d(d_woff.p, woff, 2);
  Dev<uint64_t> d_words(nw);
  check(cpk_unpack_chunks(ctx, d_in.p, n, d_off.p, d_woff.p, 1, d_words.p, nw, d_st.p, nullptr),
        "unpack");
  check(cpk_sync(ctx, nullptr), "unpack");
  d2h(&st, d_st.p, 1);
  if (st != CPK_OK) {
    Batch b;
    b.stop = st;
    return b;
  }
  std::vector<uint64_t> w(nw);
  d2h(w.data(), d_words.p, nw);
  return single_segment(w.data(), nw);
}

void write_binary(const Batch& b) { write_all(b.words.data(), b.off.back() * 8); }

void write_packed(cpk_ctx* ctx, const Batch& b) {
  const uint64_t nm = b.count(), nw = b.off.back();
  if (nm == 0) return;
  const uint64_t cap = cpk_packed_bound(nw, nw + 2 * nm);
  Dev<uint64_t> d_words(nw), d_off(nm + 1), d_out_off(nm + 1);
  Dev<uint8_t> d_out(cap);
  Dev<int32_t> d_st(nm);
  h2d(d_words.p, b.words.data(), nw);
  h2d(d_off.p, b.off.data(), nm + 1);
  check(cpk_pack_messages(ctx, d_words.p, nw, d_off.p, nm, d_out.p, cap, d_out_off.p, d_st.p,
                          nullptr),
        "pack");
  check(cpk_sync(ctx, nullptr), "pack");
  std::vector<uint64_t> oo(nm + 1);
  d2h(oo.data(), d_out_off.p, nm + 1);
  std::vector<uint8_t> out(oo[nm]);
  d2h(out.data(), d_out.p, out.size());
  write_all(out.data(), out.size());
}

// flat / flat-packed output: each message must be one segment (the re-layout that would merge
// several is outside the codec).  Returns the segment ranges (word offsets into b.words).
std::vector<uint64_t> segment_ranges(const Batch& b) {
  std::vector<uint64_t> r{0};
  for (size_t i = 0; i < b.count(); i++) {
    const uint64_t w0 = b.words[b.off[i]];
    if ((uint32_t)w0 != 0)
      die(1, "message " + std::to_string(i) +
                 " has several segments; flat output needs the single-segment re-layout "
                 "(MallocMessageBuilder::setRoot), which this tool does not do");
    r.push_back(b.off[i] + 1);  // start of segment 0
    r.push_back(b.off[i + 1]);
  }
  return r;
}

void write_flat(const Batch& b) {
  const auto r = segment_ranges(b);
  for (size_t i = 1; i + 1 < r.size(); i += 2)
    write_all(b.words.data() + r[i], (r[i + 1] - r[i]) * 8);
}

void write_flat_packed(cpk_ctx* ctx, const Batch& b) {
  const auto r = segment_ranges(b);
  const uint64_t nm = b.count();
  if (nm == 0) return;
  // the segments gathered back to back, one chunk each
  std::vector<uint64_t> w, coff{0};
  for (size_t i = 1; i + 1 < r.size(); i += 2) {
    w.insert(w.end(), b.words.begin() + r[i], b.words.begin() + r[i + 1]);
    coff.push_back(w.size());
  }
  const uint64_t nw = w.size();
  const uint64_t cap = cpk_packed_bound(nw, nm);
  Dev<uint64_t> d_words(nw), d_coff(nm + 1), d_oo(nm + 1);
  Dev<uint8_t> d_out(cap);
  h2d(d_words.p, w.data(), nw);
  h2d(d_coff.p, coff.data(), nm + 1);
  check(cpk_pack_chunks(ctx, d_words.p, nw, d_coff.p, nm, d_out.p, cap, d_oo.p, nullptr), "pack");
  check(cpk_sync(ctx, nullptr), "pack");
  std::vector<uint64_t> oo(nm + 1);
  d2h(oo.data(), d_oo.p, nm + 1);
  std::vector<uint8_t> out(oo[nm]);
  d2h(out.data(), d_out.p, out.size());
  write_all(out.data(), out.size());
}

void usage() {
  fprintf(stderr,
          "usage: cpk-convert <from>:<to> [--quiet]\n"
          "  Converts Cap'n Proto messages from stdin to stdout between the wire formats\n"
          "  binary, packed, flat and flat-packed on the GPU codec (capnp convert without a\n"
          "  schema; message layout is preserved, see the file comment).\n");
}

}  // namespace

int main(int argc, char** argv) {
  std::string spec;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    if (a == "--quiet") continue;  // the reference's plausibility warnings are not restated
    if (a == "-h" || a == "--help") {
      usage();
      return 0;
    }
    if (!spec.empty()) {
      usage();
      return 2;
    }
    spec = a;
  }
  const size_t colon = spec.find(':');
  if (colon == std::string::npos) {
    usage();
    return 2;
  }
  const Fmt from = parse_fmt(spec.substr(0, colon)), to = parse_fmt(spec.substr(colon + 1));
  if (from == Fmt::kBad || to == Fmt::kBad) die(2, "unknown format in '" + spec + "'");

  const std::vector<uint8_t> in = read_all(STDIN_FILENO);
  cpk_ctx* ctx = nullptr;
  check(cpk_init(0, &ctx), "init");

  Batch b;
  switch (from) {
    case Fmt::kBinary: b = read_binary(in); break;
    case Fmt::kPacked: b = read_packed(ctx, in); break;
    case Fmt::kFlat: b = read_flat(in); break;
    case Fmt::kFlatPacked: b = read_flat_packed(ctx, in); break;
    case Fmt::kBad: break;
  }
  switch (to) {
    case Fmt::kBinary: write_binary(b); break;
    case Fmt::kPacked: write_packed(ctx, b); break;
    case Fmt::kFlat: write_flat(b); break;
    case Fmt::kFlatPacked: write_flat_packed(ctx, b); break;
    case Fmt::kBad: break;
  }
  cpk_destroy(ctx);
  if (b.stop != CPK_OK) {
    fprintf(stderr,
            "*** ERROR CONVERTING PREVIOUS MESSAGE ***\n"
            "The following error occurred while converting the message above.\n"
            "This probably means the input data is invalid/corrupted.\n"
            "Exception description: %s\n"
            "*** END ERROR ***\n",
            cpk_status_string(b.stop));
    return 1;
  }
  return 0;
}
