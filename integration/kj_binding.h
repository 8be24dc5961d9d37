// kj_binding.h -- the reference-side binding: what a code base built against capnproto adds to
// route its packed-message calls to the MI355X codec.  Header-only; include it
// next to <capnp/serialize-packed.h> and link libcpk_hip.so.  It adapts kj streams to the
// façade's stream types (include/cpk_capnp.h) with no copies, and gives the reference's entry
// points (serialize-packed.h:65-124) the same names in namespace cpk_kj:
//
//   capnp::writePackedMessage(out, builder)      -> cpk_kj::writePackedMessage(out, builder)
//   capnp::writePackedMessageToFd(fd, builder)   -> cpk_kj::writePackedMessageToFd(fd, builder)
//   (both for kj::BufferedOutputStream and for an unbuffered kj::OutputStream)
//   capnp::PackedMessageReader reader(in, opts)  -> cpk_kj::PackedMessageReader reader(in, opts)
//   capnp::PackedFdMessageReader message(fd)     -> cpk_kj::PackedFdMessageReader message(fd)
//   (fd as int, borrowed, or as kj::OwnFd, owned)
//   capnp::computeUnpackedSizeInWords(bytes)     -> cpk_kj::computeUnpackedSizeInWords(bytes)
//
// cpk_kj::PackedMessageReader IS a capnp::MessageReader, so getRoot<T>() works unchanged.
// Failures arrive as cpk_capnp::Exception (same descriptions as the reference's kj::Exception).
// Checked to compile against the reference's own headers by tests/test_integration.py.
#pragma once

#include <capnp/message.h>
#include <kj/io.h>

#include <vector>

#include "cpk_capnp.h"

namespace cpk_kj {

// kj::BufferedOutputStream as the façade's BufferedOutputStream.
class KjOut final : public cpk_capnp::BufferedOutputStream {
 public:
  explicit KjOut(kj::BufferedOutputStream& k) : k_(k) {}
  cpk_capnp::ArrayPtr<cpk_capnp::byte> getWriteBuffer() override {
    auto b = k_.getWriteBuffer();
    return {b.begin(), b.size()};
  }
  void write(const void* p, size_t n) override {
    k_.write(kj::arrayPtr(static_cast<const kj::byte*>(p), n));
  }
  using cpk_capnp::OutputStream::write;

 private:
  kj::BufferedOutputStream& k_;
};

// kj::BufferedInputStream as the façade's BufferedInputStream.
class KjIn final : public cpk_capnp::BufferedInputStream {
 public:
  explicit KjIn(kj::BufferedInputStream& k) : k_(k) {}
  cpk_capnp::ArrayPtr<const cpk_capnp::byte> tryGetReadBuffer() override {
    auto b = k_.tryGetReadBuffer();
    return {b.begin(), b.size()};
  }
  size_t tryRead(void* p, size_t minBytes, size_t maxBytes) override {
    return k_.tryRead(kj::arrayPtr(static_cast<kj::byte*>(p), maxBytes), minBytes);
  }
  void skip(size_t n) override { k_.skip(n); }

 private:
  kj::BufferedInputStream& k_;
};

// serialize-packed.h:32-62, the stream-level codec (used by the reference's tests and by `capnp
// convert`'s flat-packed paths, compiler/capnp.c++:1066-1071, :1130-1132): kj streams in and out,
// the device codec in between.
namespace _ {

class PackedOutputStream final : public kj::OutputStream {
 public:
  explicit PackedOutputStream(kj::BufferedOutputStream& inner) : out_(inner), packed_(out_) {}
  void write(kj::ArrayPtr<const kj::byte> data) override {
    packed_.write(data.begin(), data.size());
  }
  // kj/io.c++:109-113: one write() -- one chunk -- per piece
  void write(kj::ArrayPtr<const kj::ArrayPtr<const kj::byte>> pieces) override {
    for (auto& p : pieces) write(p);
  }

 private:
  KjOut out_;
  cpk_capnp::_::PackedOutputStream packed_;
};

class PackedInputStream final : public kj::InputStream {
 public:
  explicit PackedInputStream(kj::BufferedInputStream& inner) : in_(inner), packed_(in_) {}
  size_t tryRead(kj::ArrayPtr<kj::byte> buffer, size_t minBytes) override {
    return packed_.tryRead(buffer.begin(), minBytes, buffer.size());
  }
  void skip(size_t bytes) override { packed_.skip(bytes); }

 private:
  KjIn in_;
  cpk_capnp::_::PackedInputStream packed_;
};

}  // namespace _

// capnp::word and cpk_capnp::word are both eight opaque bytes.
static_assert(sizeof(capnp::word) == sizeof(cpk_capnp::word), "word size");

inline std::vector<cpk_capnp::ArrayPtr<const cpk_capnp::word>> segments_of(
    kj::ArrayPtr<const kj::ArrayPtr<const capnp::word>> segs) {
  std::vector<cpk_capnp::ArrayPtr<const cpk_capnp::word>> v;
  v.reserve(segs.size());
  for (auto& s : segs)
    v.emplace_back(reinterpret_cast<const cpk_capnp::word*>(s.begin()), s.size());
  return v;
}

// serialize-packed.h:92-98, :114-124
inline void writePackedMessage(kj::BufferedOutputStream& output,
                               kj::ArrayPtr<const kj::ArrayPtr<const capnp::word>> segments) {
  auto v = segments_of(segments);
  KjOut out(output);
  cpk_capnp::writePackedMessage(
      out, cpk_capnp::ArrayPtr<const cpk_capnp::ArrayPtr<const cpk_capnp::word>>(v.data(),
                                                                                 v.size()));
}
inline void writePackedMessage(kj::BufferedOutputStream& output, capnp::MessageBuilder& builder) {
  writePackedMessage(output, builder.getSegmentsForOutput());
}
// serialize-packed.h:94-98, :118-120 (serialize-packed.c++:466-475): an unbuffered kj stream.  The
// reference packs straight into a kj::BufferedOutputStream when the stream is one, else through
// an 8 KiB buffer; here the façade's OutputStream overload does the buffering (one device call
// per message, then one write() of the packed bytes).
class KjPlainOut final : public cpk_capnp::OutputStream {
 public:
  explicit KjPlainOut(kj::OutputStream& k) : k_(k) {}
  void write(const void* p, size_t n) override {
    k_.write(kj::arrayPtr(static_cast<const kj::byte*>(p), n));
  }
  using cpk_capnp::OutputStream::write;

 private:
  kj::OutputStream& k_;
};
inline void writePackedMessage(kj::OutputStream& output,
                               kj::ArrayPtr<const kj::ArrayPtr<const capnp::word>> segments) {
  KJ_IF_SOME(buffered, kj::dynamicDowncastIfAvailable<kj::BufferedOutputStream>(output)) {
    writePackedMessage(buffered, segments);
  } else {
    auto v = segments_of(segments);
    KjPlainOut out(output);
    cpk_capnp::writePackedMessage(
        out, cpk_capnp::ArrayPtr<const cpk_capnp::ArrayPtr<const cpk_capnp::word>>(v.data(),
                                                                                   v.size()));
  }
}
inline void writePackedMessage(kj::OutputStream& output, capnp::MessageBuilder& builder) {
  writePackedMessage(output, builder.getSegmentsForOutput());
}

inline void writePackedMessageToFd(int fd,
                                   kj::ArrayPtr<const kj::ArrayPtr<const capnp::word>> segments) {
  auto v = segments_of(segments);
  cpk_capnp::writePackedMessageToFd(
      fd, cpk_capnp::ArrayPtr<const cpk_capnp::ArrayPtr<const cpk_capnp::word>>(v.data(),
                                                                                v.size()));
}
inline void writePackedMessageToFd(int fd, capnp::MessageBuilder& builder) {
  writePackedMessageToFd(fd, builder.getSegmentsForOutput());
}

// serialize-packed.h:65-71 as a capnp::MessageReader: segments are read (lazily, as the
// reference does) by the façade reader; getRoot<T>() and the rest come from MessageReader.
class PackedMessageReader : public capnp::MessageReader {
 public:
  PackedMessageReader(kj::BufferedInputStream& in,
                      capnp::ReaderOptions options = capnp::ReaderOptions(),
                      kj::ArrayPtr<capnp::word> scratch = nullptr)
      : capnp::MessageReader(options),
        in_(in),
        reader_(in_, toCpk(options),
                cpk_capnp::ArrayPtr<cpk_capnp::word>(
                    reinterpret_cast<cpk_capnp::word*>(scratch.begin()), scratch.size())) {}
  kj::ArrayPtr<const capnp::word> getSegment(uint id) override {
    auto s = reader_.getSegment(id);
    return kj::arrayPtr(reinterpret_cast<const capnp::word*>(s.begin()), s.size());
  }

 private:
  static cpk_capnp::ReaderOptions toCpk(const capnp::ReaderOptions& o) {
    cpk_capnp::ReaderOptions r;
    r.traversalLimitInWords = o.traversalLimitInWords;
    r.nestingLimit = o.nestingLimit;
    return r;
  }
  KjIn in_;
  cpk_capnp::PackedMessageReader reader_;
};

namespace _ {
// The descriptor side of PackedFdMessageReader: kj::FdInputStream (owning the fd or not) and the
// reference's own BufferedInputStreamWrapper over it, constructed before the reader that reads
// through them (serialize-packed.c++:444-456).
struct FdInput {
  kj::FdInputStream fdIn;
  kj::BufferedInputStreamWrapper buffered;
  explicit FdInput(int fd) : fdIn(fd), buffered(fdIn) {}
  explicit FdInput(kj::OwnFd fd) : fdIn(kj::mv(fd)), buffered(fdIn) {}
};
}  // namespace _

// serialize-packed.h:73-89: read a packed message from a file descriptor, borrowing it (int) or
// owning it (kj::OwnFd), as samples/addressbook.c++:79 does (`PackedFdMessageReader message(fd)`).
class PackedFdMessageReader final : private _::FdInput, public PackedMessageReader {
 public:
  PackedFdMessageReader(int fd, capnp::ReaderOptions options = capnp::ReaderOptions(),
                        kj::ArrayPtr<capnp::word> scratch = nullptr)
      : _::FdInput(fd), PackedMessageReader(buffered, options, scratch) {}
  PackedFdMessageReader(kj::OwnFd fd, capnp::ReaderOptions options = capnp::ReaderOptions(),
                        kj::ArrayPtr<capnp::word> scratch = nullptr)
      : _::FdInput(kj::mv(fd)), PackedMessageReader(buffered, options, scratch) {}
};

// serialize-packed.h:107
inline size_t computeUnpackedSizeInWords(kj::ArrayPtr<const kj::byte> packedBytes) {
  return cpk_capnp::computeUnpackedSizeInWords(
      cpk_capnp::ArrayPtr<const cpk_capnp::byte>(packedBytes.begin(), packedBytes.size()));
}

}  // namespace cpk_kj
