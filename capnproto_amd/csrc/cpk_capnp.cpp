// cpk_capnp.cpp -- the reference's packed-serialization API (include/cpk_capnp.h) over the C ABI.
// Host plumbing only: every pack / unpack goes to the device through cpk.h.
#include "../../include/cpk_capnp.h"

#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <exception>
#include <utility>

namespace cpk_capnp {

namespace {

int g_device = -1;

struct CtxHolder {
  cpk_ctx* ctx = nullptr;
  int device = -1;
  ~CtxHolder() {
    if (ctx) cpk_destroy(ctx);
  }
};

thread_local CtxHolder t_ctx;

[[noreturn]] void fail(cpk_status st, const char* where) { throw Exception(st, where); }

void check(cpk_status st, const char* where) {
  if (st != CPK_OK) fail(st, where);
}

// The flat form of a message: segment table (serialize.c++:311-330) then the segments.
std::vector<uint64_t> flatten(ArrayPtr<const ArrayPtr<const word>> segments) {
  const size_t n = segments.size();
  const size_t table_words = n / 2 + 1;
  size_t total = table_words;
  for (auto& s : segments) total += s.size();
  std::vector<uint64_t> flat(total, 0);
  uint32_t* t = reinterpret_cast<uint32_t*>(flat.data());
  t[0] = (uint32_t)(n - 1);
  for (size_t i = 0; i < n; i++) t[i + 1] = (uint32_t)segments[i].size();
  size_t at = table_words;
  for (auto& s : segments) {
    if (s.size()) memcpy(flat.data() + at, s.begin(), s.size() * 8);
    at += s.size();
  }
  return flat;
}

}  // namespace

Exception::Exception(cpk_status status, const std::string& where)
    : std::runtime_error(std::string(cpk_status_string(status)) +
                         (where.empty() ? "" : " [" + where + "]")),
      status_(status) {}

void setDevice(int device) { g_device = device; }

cpk_ctx* threadContext() {
  int dev = g_device;
  if (dev < 0) {
    const char* e = getenv("CPK_DEVICE");
    dev = e ? atoi(e) : 0;
  }
  if (t_ctx.ctx && t_ctx.device == dev) return t_ctx.ctx;
  if (t_ctx.ctx) {
    cpk_destroy(t_ctx.ctx);
    t_ctx.ctx = nullptr;
  }
  cpk_ctx* c = nullptr;
  check(cpk_init(dev, &c), "cpk_init");
  t_ctx.ctx = c;
  t_ctx.device = dev;
  return c;
}

// ---- streams ---------------------------------------------------------------------------------
void OutputStream::write(ArrayPtr<const ArrayPtr<const byte>> pieces) {
  for (auto& p : pieces) write(p.begin(), p.size());
}

size_t InputStream::read(void* buffer, size_t minBytes, size_t maxBytes) {
  const size_t n = tryRead(buffer, minBytes, maxBytes);
  if (n < minBytes) fail(CPK_ERR_PREMATURE_EOF, "InputStream::read");
  return n;
}

void InputStream::skip(size_t bytes) {
  char scratch[8192];
  while (bytes > 0) {
    const size_t amount = std::min(bytes, sizeof(scratch));
    read(scratch, amount);
    bytes -= amount;
  }
}

void ArrayOutputStream::write(const void* buffer, size_t size) {
  if (buffer == array_.begin() + fill_) {  // written in place through getWriteBuffer()
    if (size > array_.size() - fill_) fail(CPK_ERR_CAPACITY, "ArrayOutputStream");
    fill_ += size;
    return;
  }
  if (size > array_.size() - fill_) fail(CPK_ERR_CAPACITY, "ArrayOutputStream");
  if (size) memcpy(array_.begin() + fill_, buffer, size);
  fill_ += size;
}

ArrayPtr<byte> VectorOutputStream::getWriteBuffer() {
  spare_.resize(std::max<size_t>(4096, bytes_.capacity() - bytes_.size()));
  return ArrayPtr<byte>(spare_.data(), spare_.size());
}

void VectorOutputStream::write(const void* buffer, size_t size) {
  const byte* b = static_cast<const byte*>(buffer);
  bytes_.insert(bytes_.end(), b, b + size);
}

size_t ArrayInputStream::tryRead(void* buffer, size_t minBytes, size_t maxBytes) {
  (void)minBytes;
  const size_t n = std::min(maxBytes, array_.size());
  if (n) memcpy(buffer, array_.begin(), n);
  array_ = array_.slice(n, array_.size());
  return n;
}

void ArrayInputStream::skip(size_t bytes) {
  if (bytes > array_.size()) fail(CPK_ERR_PREMATURE_EOF, "ArrayInputStream::skip");
  array_ = array_.slice(bytes, array_.size());
}

OwnFd& OwnFd::operator=(OwnFd&& o) noexcept {
  if (this != &o) {
    if (fd_ >= 0) ::close(fd_);
    fd_ = o.fd_;
    o.fd_ = -1;
  }
  return *this;
}

OwnFd::~OwnFd() {
  if (fd_ >= 0) ::close(fd_);
}

FdBufferedInputStream::FdBufferedInputStream(int fd, size_t bufferSize)
    : fd_(fd), buf_(bufferSize) {}

FdBufferedInputStream::FdBufferedInputStream(OwnFd fd, size_t bufferSize)
    : owned_(std::move(fd)), fd_(owned_.get()), buf_(bufferSize) {}

ArrayPtr<const byte> FdBufferedInputStream::tryGetReadBuffer() {
  if (begin_ == end_) {
    begin_ = end_ = 0;
    for (;;) {
      const ssize_t n = ::read(fd_, buf_.data(), buf_.size());
      if (n < 0 && errno == EINTR) continue;
      if (n < 0) fail(CPK_ERR_PREMATURE_EOF, "read(fd)");
      end_ = (size_t)n;
      break;
    }
  }
  return ArrayPtr<const byte>(buf_.data() + begin_, end_ - begin_);
}

size_t FdBufferedInputStream::tryRead(void* buffer, size_t minBytes, size_t maxBytes) {
  byte* out = static_cast<byte*>(buffer);
  size_t got = 0;
  while (got < minBytes) {
    auto b = tryGetReadBuffer();
    if (b.size() == 0) break;
    const size_t n = std::min(b.size(), maxBytes - got);
    memcpy(out + got, b.begin(), n);
    begin_ += n;
    got += n;
  }
  return got;
}

void FdBufferedInputStream::skip(size_t bytes) {
  while (bytes > 0) {
    auto b = tryGetReadBuffer();
    if (b.size() == 0) fail(CPK_ERR_PREMATURE_EOF, "skip(fd)");
    const size_t n = std::min(b.size(), bytes);
    begin_ += n;
    bytes -= n;
  }
}

void FdOutputStream::write(const void* buffer, size_t size) {
  const byte* p = static_cast<const byte*>(buffer);
  while (size > 0) {
    const ssize_t n = ::write(fd_, p, size);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) fail(CPK_ERR_INVALID_ARGUMENT, "write(fd)");
    p += n;
    size -= (size_t)n;
  }
}

// ---- pack ------------------------------------------------------------------------------------
void _::PackedOutputStream::write(const void* buffer, size_t size) {
  // serialize-packed.c++:309-313: the input must be whole words.
  if (size % 8 != 0) fail(CPK_ERR_INVALID_ARGUMENT, "PackedOutputStream::write: not word-sized");
  const uint64_t nwords = size / 8;
  if (nwords == 0) return;
  std::vector<uint64_t> words(nwords);
  memcpy(words.data(), buffer, size);
  const uint64_t off[2] = {0, nwords};
  std::vector<uint8_t> out(cpk_packed_bound(nwords, 1) + 16);
  uint64_t out_off[2] = {0, 0};
  check(cpk_pack_chunks_host(threadContext(), words.data(), nwords, off, 1, out.data(), out.size(),
                             out_off),
        "PackedOutputStream::write");
  inner_.write(out.data(), out_off[1]);
}

void writePackedMessage(OutputStream& output, ArrayPtr<const ArrayPtr<const word>> segments) {
  // serialize.c++:333 "Tried to serialize uninitialized message."
  if (segments.size() == 0) fail(CPK_ERR_EMPTY_MESSAGE, "writePackedMessage");
  std::vector<uint64_t> flat = flatten(segments);
  const uint64_t off[2] = {0, flat.size()};
  // every piece (table, each segment) is a chunk: bound over n + 1 chunks
  std::vector<uint8_t> out(cpk_packed_bound(flat.size(), segments.size() + 1) + 16);
  uint64_t out_off[2] = {0, 0};
  int32_t status = 0;
  check(cpk_pack_messages_host(threadContext(), flat.data(), flat.size(), off, 1, out.data(),
                               out.size(), out_off, &status),
        "writePackedMessage");
  if (status != CPK_OK) fail((cpk_status)status, "writePackedMessage");
  output.write(out.data(), out_off[1]);
}

void writePackedMessage(BufferedOutputStream& output,
                        ArrayPtr<const ArrayPtr<const word>> segments) {
  writePackedMessage(static_cast<OutputStream&>(output), segments);
}

void writePackedMessageToFd(int fd, ArrayPtr<const ArrayPtr<const word>> segments) {
  FdOutputStream out(fd);
  writePackedMessage(out, segments);
}

// ---- unpack ----------------------------------------------------------------------------------
namespace {

// Byte length and word count of the record at v[q] (doc/encoding.md:296-349), for the few
// boundaries in a buffer's last 9 bytes that the device does not report one by one.
size_t rec_len(const byte* v, size_t q) {
  const unsigned tag = v[q];
  const size_t run = (tag == 0 || tag == 0xff) ? 1 : 0;
  return 1 + (size_t)__builtin_popcount(tag) + run + (tag == 0xff ? 8 * (size_t)v[q + 9] : 0);
}
uint64_t rec_words(const byte* v, size_t q) {
  const unsigned tag = v[q];
  return 1 + (tag == 0 ? v[q + 1] : (tag == 0xff ? v[q + 9] : 0));
}

}  // namespace

size_t _::PackedInputStream::readWords(uint64_t* dst, size_t minw, size_t maxw) {
  // serialize-packed.c++:34-183.  Each pass hands the device one stream buffer V (with the
  // start of a record the previous buffer cut in front of it) and gets back where the read
  // stops in V: max words out, a run crossing max (overshoot), or the start of the record V
  // cuts.  The reference also returns at the first record boundary with fewer than 10 bytes left
  // in V once min words are out (:71-76); those boundaries are checked here from the device's
  // word counts.
  cpk_ctx* ctx = threadContext();
  ArrayPtr<const byte> buf = inner_.tryGetReadBuffer();
  if (buf.size() == 0) return 0;  // :48-51: nothing at all to read
  std::vector<byte> carry;         // bytes of V already taken from the stream (a cut record)
  size_t out = 0;
  for (;;) {
    const byte* v = buf.begin();
    size_t vlen = buf.size();
    const size_t carried = carry.size();
    if (carried) {
      carry.insert(carry.end(), buf.begin(), buf.end());
      v = carry.data();
      vlen = carry.size();
    }
    const uint64_t want = maxw - out;
    // a record yields at least one word per 10 bytes, so max words never need more than
    // 10 * want + 10 bytes (and then no boundary lies in V's last 9 bytes)
    const size_t look = want < vlen / 10 ? (size_t)(10 * want + 10) : vlen;
    uint64_t w = 0, c = 0;
    const cpk_status st =
        cpk_unpack_prefix_host(ctx, v, look, dst ? dst + out : nullptr, want, &w, &c);
    if (st != CPK_OK && st != CPK_ERR_PREMATURE_EOF && st != CPK_ERR_RUN_OVERSHOOT)
      fail(st, "PackedInputStream");
    if (look < vlen && st == CPK_ERR_PREMATURE_EOF) fail(CPK_ERR_INTERNAL, "PackedInputStream");
    auto consume = [&](size_t q) { inner_.skip(q - carried); };
    const size_t s = vlen > 9 ? vlen - 9 : 0;  // boundaries at >= s leave < 10 bytes
    if (look == vlen && c >= s && out + w >= minw) {
      // the boundaries in [s, c]: walk from the record holding byte s (found by the device)
      uint64_t b0 = 0, wb0 = 0;
      if (s > 0) {
        const cpk_status st0 = cpk_unpack_prefix_host(ctx, v, s, nullptr, want, &wb0, &b0);
        if (st0 != CPK_OK && st0 != CPK_ERR_PREMATURE_EOF)
          fail(st0 == CPK_ERR_RUN_OVERSHOOT ? CPK_ERR_INTERNAL : st0, "PackedInputStream");
      }
      uint64_t q = b0, wq = wb0;
      if (q < s) {
        wq += rec_words(v, q);
        q += rec_len(v, q);
      }
      while (q <= c) {
        // a raw run that crossed into this buffer and ends with it: the reference asks the
        // stream for more before it looks at the boundary (:157-168)
        const bool crossed = q == vlen && carried && v[0] == 0xff && 9 < carried && v[9] != 0 &&
                             rec_len(v, 0) == vlen;
        if (out + wq >= minw && !crossed) {
          consume(q);
          return out + wq;
        }
        if (q == c) break;
        wq += rec_words(v, q);
        q += rec_len(v, q);
      }
    }
    if (st == CPK_OK) {
      consume(c);
      return maxw;
    }
    if (st == CPK_ERR_RUN_OVERSHOOT) fail(st, "PackedInputStream");
    // V ends inside the record at c (or at c itself): keep its bytes and read on
    out += w;
    if (carried) {
      carry.erase(carry.begin(), carry.begin() + (ptrdiff_t)c);
    } else {
      carry.assign(buf.begin() + c, buf.end());
    }
    inner_.skip(buf.size());
    buf = inner_.tryGetReadBuffer();
    if (buf.size() == 0) fail(CPK_ERR_PREMATURE_EOF, "PackedInputStream");  // :57
  }
}

size_t _::PackedInputStream::tryRead(void* buffer, size_t minBytes, size_t maxBytes) {
  if (maxBytes == 0) return 0;
  if (minBytes % 8 != 0 || maxBytes % 8 != 0)
    fail(CPK_ERR_INVALID_ARGUMENT, "PackedInputStream reads must be word-aligned.");
  if (minBytes > maxBytes) minBytes = maxBytes;
  return 8 * readWords(static_cast<uint64_t*>(buffer), minBytes / 8, maxBytes / 8);
}

void _::PackedInputStream::skip(size_t bytes) {
  // serialize-packed.c++:185-299: the same parse with nothing stored -- the device parses with no
  // output buffer at all (cpk_unpack_prefix_host with no destination)
  if (bytes == 0) return;
  if (bytes % 8 != 0) fail(CPK_ERR_INVALID_ARGUMENT, "PackedInputStream reads must be word-aligned.");
  if (readWords(nullptr, bytes / 8, bytes / 8) < bytes / 8)
    fail(CPK_ERR_PREMATURE_EOF, "PackedInputStream");
}

PackedMessageReader::PackedMessageReader(BufferedInputStream& in, ReaderOptions options,
                                         ArrayPtr<word> scratch)
    : MessageReader(options), _::PackedInputStream(in) {
  // serialize.c++:202-270
  uint32_t first[2];
  InputStream::read(first, 8);
  uint32_t segmentCount = first[0] + 1;
  const uint32_t segment0Size = first[1];
  size_t totalWords = segment0Size;
  if (first[0] >= 511) fail(CPK_ERR_TOO_MANY_SEGMENTS, "PackedMessageReader");  // :217
  std::vector<uint32_t> moreSizes(segmentCount & ~1u);
  if (segmentCount > 1) {
    InputStream::read(moreSizes.data(), moreSizes.size() * 4);
    for (uint32_t i = 0; i < segmentCount - 1; i++) totalWords += moreSizes[i];
  }
  if (totalWords > options.traversalLimitInWords)  // :235
    fail(CPK_ERR_MESSAGE_TOO_LARGE, "PackedMessageReader");
  if (scratch.size() < totalWords) {
    owned_.resize(totalWords);
    scratch = ArrayPtr<word>(owned_.data(), owned_.size());
  }
  segment0_ = ArrayPtr<const word>(scratch.begin(), segment0Size);
  size_t offset = segment0Size;
  for (uint32_t i = 0; i + 1 < segmentCount; i++) {
    moreSegments_.push_back(ArrayPtr<const word>(scratch.begin() + offset, moreSizes[i]));
    offset += moreSizes[i];
  }
  if (segmentCount == 1) {
    InputStream::read(scratch.begin(), totalWords * 8);
  } else {
    readPos_ = reinterpret_cast<byte*>(scratch.begin());
    readPos_ += InputStream::read(readPos_, segment0Size * 8, totalWords * 8);
  }
}

PackedMessageReader::~PackedMessageReader() noexcept(false) {
  // serialize.c++:272-281: leave the stream after the message
  if (readPos_ == nullptr) return;
  const byte* allEnd = reinterpret_cast<const byte*>(moreSegments_.back().end());
  if (std::uncaught_exceptions() > 0) {
    try {
      skip((size_t)(allEnd - readPos_));
    } catch (...) {
    }
  } else {
    skip((size_t)(allEnd - readPos_));
  }
}

ArrayPtr<const word> PackedMessageReader::getSegment(unsigned id) {
  // serialize.c++:283-302
  if (id > moreSegments_.size()) return nullptr;
  ArrayPtr<const word> segment = id == 0 ? segment0_ : moreSegments_[id - 1];
  if (readPos_ != nullptr) {
    const byte* segmentEnd = reinterpret_cast<const byte*>(segment.end());
    if (readPos_ < segmentEnd) {
      const byte* allEnd = reinterpret_cast<const byte*>(moreSegments_.back().end());
      readPos_ += InputStream::read(readPos_, (size_t)(segmentEnd - readPos_),
                                    (size_t)(allEnd - readPos_));
    }
  }
  return segment;
}

PackedFdMessageReader::PackedFdMessageReader(int fd, ReaderOptions options,
                                             ArrayPtr<word> scratchSpace)
    : FdBufferedInputStream(fd),
      PackedMessageReader(static_cast<FdBufferedInputStream&>(*this), options, scratchSpace) {}

PackedFdMessageReader::PackedFdMessageReader(OwnFd fd, ReaderOptions options,
                                             ArrayPtr<word> scratchSpace)
    : FdBufferedInputStream(std::move(fd)),
      PackedMessageReader(static_cast<FdBufferedInputStream&>(*this), options, scratchSpace) {}

size_t computeUnpackedSizeInWords(ArrayPtr<const byte> packedBytes) {
  uint64_t words = 0;
  check(cpk_unpacked_size_host(threadContext(), packedBytes.begin(), packedBytes.size(), &words),
        "computeUnpackedSizeInWords");
  return words;
}

}  // namespace cpk_capnp
