// cpk_capnp.cpp -- the reference's packed-serialization API (include/cpk_capnp.h) over the C ABI.
// Host plumbing only: every pack / unpack goes to the device through cpk.h.
#include "../../include/cpk_capnp.h"

#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>

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

void InputStream::read(void* buffer, size_t bytes) {
  const size_t n = tryRead(buffer, bytes, bytes);
  if (n < bytes) fail(CPK_ERR_PREMATURE_EOF, "InputStream::read");
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

FdBufferedInputStream::FdBufferedInputStream(int fd, size_t bufferSize)
    : fd_(fd), buf_(bufferSize) {}

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
size_t _::PackedInputStream::tryRead(void* buffer, size_t minBytes, size_t maxBytes) {
  // serialize-packed.c++:34-51
  if (maxBytes == 0) return 0;
  if (minBytes % 8 != 0 || maxBytes % 8 != 0)
    fail(CPK_ERR_INVALID_ARGUMENT, "PackedInputStream reads must be word-aligned.");
  if (minBytes > maxBytes) minBytes = maxBytes;
  cpk_ctx* ctx = threadContext();
  uint64_t* dst = static_cast<uint64_t*>(buffer);
  std::vector<byte> acc;  // bytes already taken from the stream (the read spans buffers)
  for (;;) {
    ArrayPtr<const byte> buf = inner_.tryGetReadBuffer();
    if (acc.empty() && buf.size() == 0) return 0;  // :48-51: nothing at all to read
    const byte* data = buf.begin();
    size_t avail = buf.size();
    if (!acc.empty()) {
      acc.insert(acc.end(), buf.begin(), buf.end());
      data = acc.data();
      avail = acc.size();
    }
    const size_t before = acc.empty() ? 0 : acc.size() - buf.size();
    uint64_t used = 0;
    cpk_status st = cpk_unpack_words_host(ctx, data, avail, dst, maxBytes / 8, &used);
    if (st == CPK_ERR_PREMATURE_EOF && buf.size() > 0) {
      // the records continue past what is buffered: take these bytes and refill
      if (acc.empty()) acc.assign(buf.begin(), buf.end());
      inner_.skip(buf.size());
      continue;
    }
    if (st == CPK_ERR_PREMATURE_EOF) {
      // the input has ended: what it holds is enough if it ends at a record boundary with at
      // least minBytes of output (:65-80, the early return once out >= outMin)
      uint64_t have = 0;
      if (cpk_unpacked_size_host(ctx, data, avail, &have) == CPK_OK && have * 8 >= minBytes &&
          have * 8 < maxBytes) {
        check(cpk_unpack_words_host(ctx, data, avail, dst, have, &used), "PackedInputStream");
        inner_.skip(used - before);
        return have * 8;
      }
      fail(CPK_ERR_PREMATURE_EOF, "PackedInputStream");
    }
    check(st, "PackedInputStream");
    inner_.skip(used - before);
    return maxBytes;
  }
}

void _::PackedInputStream::skip(size_t bytes) {
  // serialize-packed.c++:185-299: the same parse without a destination -- decoded into scratch
  // in one piece, since a run may not cross `bytes` but may cross any smaller piece
  if (bytes == 0) return;
  if (bytes % 8 != 0) fail(CPK_ERR_INVALID_ARGUMENT, "PackedInputStream reads must be word-aligned.");
  std::vector<uint64_t> scratch(bytes / 8);
  if (tryRead(scratch.data(), bytes, bytes) < bytes) fail(CPK_ERR_PREMATURE_EOF, "PackedInputStream");
}

PackedMessageReader::PackedMessageReader(BufferedInputStream& in, ReaderOptions options,
                                         ArrayPtr<word> scratch)
    : options_(options) {
  cpk_ctx* ctx = threadContext();
  cpk_limits lim;
  lim.traversal_limit_words = options.traversalLimitInWords;
  std::vector<byte> acc;  // bytes already taken from the stream (the message spans buffers)
  word* dst = scratch.begin();
  size_t cap = scratch.size();
  for (;;) {
    ArrayPtr<const byte> buf = in.tryGetReadBuffer();
    const byte* data = buf.begin();
    size_t avail = buf.size();
    if (!acc.empty()) {
      acc.insert(acc.end(), buf.begin(), buf.end());
      data = acc.data();
      avail = acc.size();
    }
    if (avail == 0) fail(CPK_ERR_PREMATURE_EOF, "PackedMessageReader");
    uint64_t nwords = 0, used = 0;
    cpk_status st = cpk_read_packed_message_host(ctx, data, avail,
                                                 reinterpret_cast<uint64_t*>(dst), cap, &nwords,
                                                 &used, &lim);
    if (st == CPK_ERR_CAPACITY) {
      // serialize.c++:244-249: scratch too small -> the reader owns the space
      owned_.resize(nwords);
      dst = owned_.data();
      cap = nwords;
      st = cpk_read_packed_message_host(ctx, data, avail, reinterpret_cast<uint64_t*>(dst), cap,
                                        &nwords, &used, &lim);
    }
    if (st == CPK_ERR_PREMATURE_EOF && buf.size() > 0) {
      // the message continues past what is buffered: take these bytes and refill
      if (acc.empty()) acc.assign(buf.begin(), buf.end());
      in.skip(buf.size());
      continue;
    }
    check(st, "PackedMessageReader");
    // leave the stream right after the message
    const size_t before = acc.empty() ? 0 : acc.size() - buf.size();
    in.skip(used - before);
    flat_ = ArrayPtr<const word>(dst, nwords);
    break;
  }
  // segments from the table (serialize.c++:210-260)
  const uint32_t* t = reinterpret_cast<const uint32_t*>(flat_.begin());
  const uint32_t nseg = t[0] + 1;
  size_t at = nseg / 2 + 1;
  for (uint32_t i = 0; i < nseg; i++) {
    const size_t n = t[i + 1];
    segments_.push_back(ArrayPtr<const word>(flat_.begin() + at, n));
    at += n;
  }
}

ArrayPtr<const word> PackedMessageReader::getSegment(unsigned id) const {
  if (id >= segments_.size()) return nullptr;
  return segments_[id];
}

PackedFdMessageReader::PackedFdMessageReader(int fd, ReaderOptions options,
                                             ArrayPtr<word> scratchSpace)
    : FdBufferedInputStream(fd),
      PackedMessageReader(static_cast<FdBufferedInputStream&>(*this), options, scratchSpace) {}

size_t computeUnpackedSizeInWords(ArrayPtr<const byte> packedBytes) {
  uint64_t words = 0;
  check(cpk_unpacked_size_host(threadContext(), packedBytes.begin(), packedBytes.size(), &words),
        "computeUnpackedSizeInWords");
  return words;
}

}  // namespace cpk_capnp
