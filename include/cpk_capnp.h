// cpk_capnp.h -- the reference's packed-serialization API (capnproto c++/src/capnp/
// serialize-packed.h:32-124 and the kj/io.h stream contracts it is written against), over the
// MI355X codec's C ABI (cpk.h).  Same class / function names, argument meaning and failure
// behaviour: the reference throws kj::Exception with a fixed description; this façade throws
// cpk_capnp::Exception carrying the same description (cpk_status_string) and the cpk_status.
//
// Everything here is host C++; every byte of packing / unpacking runs in the HIP kernels behind
// libcpk_hip.so.  There is no CPU fallback: without a GPU the first call throws
// Exception(CPK_ERR_NO_DEVICE).
//
// Namespace cpk_capnp stands in for capnp (and the few kj types the API names).  A code base
// that uses capnp::writePackedMessage / capnp::PackedMessageReader switches by including this
// header and replacing the namespace.
#ifndef CPK_CAPNP_H_
#define CPK_CAPNP_H_

#include <cstddef>
#include <cstdint>
#include <future>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "cpk.h"

namespace cpk_capnp {

typedef unsigned char byte;

// capnp::word (common.h:344): eight opaque bytes.
struct word {
  uint64_t content;
};
static_assert(sizeof(word) == 8, "word is 8 bytes");

// kj::ArrayPtr subset.
template <typename T>
class ArrayPtr {
 public:
  ArrayPtr() : ptr_(nullptr), size_(0) {}
  ArrayPtr(decltype(nullptr)) : ptr_(nullptr), size_(0) {}
  ArrayPtr(T* p, size_t n) : ptr_(p), size_(n) {}
  template <typename U>
  ArrayPtr(const ArrayPtr<U>& o) : ptr_(o.begin()), size_(o.size()) {}
  ArrayPtr(std::vector<typename std::remove_const<T>::type>& v) : ptr_(v.data()), size_(v.size()) {}
  T* begin() const { return ptr_; }
  T* end() const { return ptr_ + size_; }
  size_t size() const { return size_; }
  T& operator[](size_t i) const { return ptr_[i]; }
  ArrayPtr slice(size_t a, size_t b) const { return ArrayPtr(ptr_ + a, b - a); }

 private:
  T* ptr_;
  size_t size_;
};

// kj::Exception (FAILED) as thrown by KJ_REQUIRE / KJ_FAIL_REQUIRE on the packed path.
class Exception : public std::runtime_error {
 public:
  Exception(cpk_status status, const std::string& where);
  cpk_status status() const { return status_; }

 private:
  cpk_status status_;
};

// ---- kj/io.h stream contracts ----------------------------------------------------------------
class OutputStream {
 public:
  virtual ~OutputStream() = default;
  virtual void write(const void* buffer, size_t size) = 0;
  void write(ArrayPtr<const byte> bytes) { write(bytes.begin(), bytes.size()); }
  // kj/io.c++:109-113: one write() per piece (PackedOutputStream does not override it, so runs
  // never cross a piece).
  virtual void write(ArrayPtr<const ArrayPtr<const byte>> pieces);
};

class BufferedOutputStream : public OutputStream {
 public:
  virtual ArrayPtr<byte> getWriteBuffer() = 0;
};

class InputStream {
 public:
  virtual ~InputStream() noexcept(false) = default;  // kj/io.h: readers may throw on close
  virtual size_t tryRead(void* buffer, size_t minBytes, size_t maxBytes) = 0;
  // kj/io.c++:53: "Premature EOF" when fewer than minBytes arrive; returns the bytes read.
  size_t read(void* buffer, size_t minBytes, size_t maxBytes);
  void read(void* buffer, size_t bytes) { read(buffer, bytes, bytes); }
  virtual void skip(size_t bytes);
};

class BufferedInputStream : public InputStream {
 public:
  // Whatever is buffered (empty = end of stream); refills when the buffer is exhausted.
  virtual ArrayPtr<const byte> tryGetReadBuffer() = 0;
};

// kj/io.h:210-230, io.c++:267-286: writes into a caller-owned array; "backing array was not large enough for
// the data" (CPK_ERR_CAPACITY) when it overflows.
class ArrayOutputStream : public BufferedOutputStream {
 public:
  explicit ArrayOutputStream(ArrayPtr<byte> array) : array_(array), fill_(0) {}
  ArrayPtr<byte> getArray() { return array_.slice(0, fill_); }
  ArrayPtr<byte> getWriteBuffer() override { return array_.slice(fill_, array_.size()); }
  void write(const void* buffer, size_t size) override;
  using OutputStream::write;

 private:
  ArrayPtr<byte> array_;
  size_t fill_;
};

// kj/io.h:232-254, io.c++:290-326: growing vector.
class VectorOutputStream : public BufferedOutputStream {
 public:
  explicit VectorOutputStream(size_t initialCapacity = 4096) { bytes_.reserve(initialCapacity); }
  ArrayPtr<const byte> getArray() const { return ArrayPtr<const byte>(bytes_.data(), bytes_.size()); }
  void clear() { bytes_.clear(); }
  ArrayPtr<byte> getWriteBuffer() override;
  void write(const void* buffer, size_t size) override;
  using OutputStream::write;

 private:
  std::vector<byte> bytes_;
  std::vector<byte> spare_;
};

// kj/io.h:195-208, io.c++:243-263.
class ArrayInputStream : public BufferedInputStream {
 public:
  explicit ArrayInputStream(ArrayPtr<const byte> array) : array_(array) {}
  ArrayPtr<const byte> tryGetReadBuffer() override { return array_; }
  size_t tryRead(void* buffer, size_t minBytes, size_t maxBytes) override;
  void skip(size_t bytes) override;

 private:
  ArrayPtr<const byte> array_;
};

// File descriptors (kj::FdInputStream / FdOutputStream + the buffered wrappers of kj/io.c++:
// 145-239), used by PackedFdMessageReader / writePackedMessageToFd.
// kj::OwnFd (kj/io.h): a file descriptor closed when the owner goes away.  Move-only.
class OwnFd {
 public:
  OwnFd() : fd_(-1) {}
  explicit OwnFd(int fd) : fd_(fd) {}
  OwnFd(OwnFd&& o) noexcept : fd_(o.fd_) { o.fd_ = -1; }
  OwnFd& operator=(OwnFd&& o) noexcept;
  OwnFd(const OwnFd&) = delete;
  OwnFd& operator=(const OwnFd&) = delete;
  ~OwnFd();
  int get() const { return fd_; }
  int release() {
    const int f = fd_;
    fd_ = -1;
    return f;
  }

 private:
  int fd_;
};

class FdBufferedInputStream : public BufferedInputStream {
 public:
  explicit FdBufferedInputStream(int fd, size_t bufferSize = 65536);
  explicit FdBufferedInputStream(OwnFd fd, size_t bufferSize = 65536);
  ArrayPtr<const byte> tryGetReadBuffer() override;
  size_t tryRead(void* buffer, size_t minBytes, size_t maxBytes) override;
  void skip(size_t bytes) override;

 private:
  OwnFd owned_;
  int fd_;
  std::vector<byte> buf_;
  size_t begin_ = 0, end_ = 0;
};

class FdOutputStream : public OutputStream {
 public:
  explicit FdOutputStream(int fd) : fd_(fd) {}
  void write(const void* buffer, size_t size) override;
  using OutputStream::write;

 private:
  int fd_;
};

// ---- capnp ----------------------------------------------------------------------------------
// message.h:54-73 (the limits the packed reader enforces).
struct ReaderOptions {
  uint64_t traversalLimitInWords = 8 * 1024 * 1024;
  int nestingLimit = 64;
};

// Device the calling thread's codec context uses (default 0; env CPK_DEVICE).  Each thread owns
// one cpk_ctx, created on first use (a cpk_ctx is single-threaded, cpk.h).
void setDevice(int device);
cpk_ctx* threadContext();

// message.h:95-130 MessageReader, the part the packed path fills in: segments by id (null past
// the last one) and the options the message was read with.
class MessageReader {
 public:
  explicit MessageReader(ReaderOptions options) : options_(options) {}
  virtual ~MessageReader() noexcept(false) = default;
  virtual ArrayPtr<const word> getSegment(unsigned id) = 0;
  const ReaderOptions& getOptions() const { return options_; }

 private:
  ReaderOptions options_;
};

namespace _ {  // private

// serialize-packed.h:49-63.  Each write() is one chunk, packed by the device.
class PackedOutputStream : public OutputStream {
 public:
  explicit PackedOutputStream(BufferedOutputStream& inner) : inner_(inner) {}
  void write(const void* buffer, size_t size) override;
  using OutputStream::write;

 private:
  BufferedOutputStream& inner_;
};

// serialize-packed.h:37-47 (serialize-packed.c++:34-299).  Decodes packed input from `inner`
// on the device, whole records per call, with the reference's stopping rules: tryRead fills
// up to maxBytes (whole words) and returns early only at a record boundary that leaves fewer
// than 10 bytes in the current stream buffer once minBytes are out (:71-76) -- so it never
// blocks for input it does not need; "Premature end of packed input." when the input ends
// before minBytes or inside a record; "Packed input did not end cleanly on a segment boundary."
// when a run crosses maxBytes.  skip(bytes) consumes exactly `bytes` unpacked bytes with the
// same checks and copies nothing back from the device.  Each stream buffer is sent to the
// device once (plus the few bytes of a record it cuts), so a read is O(bytes).
class PackedInputStream : public InputStream {
 public:
  explicit PackedInputStream(BufferedInputStream& inner) : inner_(inner) {}
  size_t tryRead(void* buffer, size_t minBytes, size_t maxBytes) override;
  size_t tryRead(ArrayPtr<byte> dst, size_t minBytes) {  // the newer kj signature
    return tryRead(dst.begin(), minBytes, dst.size());
  }
  void skip(size_t bytes) override;

 private:
  // minWords..maxWords words into dst (NULL: decoded on the device and dropped); returns words
  size_t readWords(uint64_t* dst, size_t minWords, size_t maxWords);
  BufferedInputStream& inner_;
};

}  // namespace _

// serialize-packed.h:65-71: a PackedInputStream read by InputStreamMessageReader
// (serialize.c++:202-302).  The constructor reads the segment table and segment 0; later
// segments are read lazily by getSegment (:283-302), and the destructor skips whatever was not
// read so the stream is left right after the message (:272-281).  Segments go into
// scratchSpace when it is large enough, else into space the reader owns (:244-249).
class PackedMessageReader : public MessageReader, private _::PackedInputStream {
 public:
  PackedMessageReader(BufferedInputStream& inputStream, ReaderOptions options = ReaderOptions(),
                      ArrayPtr<word> scratchSpace = nullptr);
  virtual ~PackedMessageReader() noexcept(false);
  PackedMessageReader(const PackedMessageReader&) = delete;
  PackedMessageReader& operator=(const PackedMessageReader&) = delete;
  size_t segmentCount() const { return 1 + moreSegments_.size(); }
  // MessageReader::getSegment (message.h:100): null past the last segment.
  ArrayPtr<const word> getSegment(unsigned id) override;

 private:
  std::vector<word> owned_;
  ArrayPtr<const word> segment0_;
  std::vector<ArrayPtr<const word>> moreSegments_;
  byte* readPos_ = nullptr;  // next byte of a lazily read multi-segment message
};

// serialize-packed.h:73-89: reads from a file descriptor (borrowed, or owned and closed with
// the reader).
class PackedFdMessageReader : private FdBufferedInputStream, public PackedMessageReader {
 public:
  PackedFdMessageReader(int fd, ReaderOptions options = ReaderOptions(),
                        ArrayPtr<word> scratchSpace = nullptr);
  PackedFdMessageReader(OwnFd fd, ReaderOptions options = ReaderOptions(),
                        ArrayPtr<word> scratchSpace = nullptr);
};

// serialize-packed.h:91-104 (MessageBuilder overloads :114-124 pass getSegmentsForOutput()).
void writePackedMessage(BufferedOutputStream& output,
                        ArrayPtr<const ArrayPtr<const word>> segments);
void writePackedMessage(OutputStream& output, ArrayPtr<const ArrayPtr<const word>> segments);
void writePackedMessageToFd(int fd, ArrayPtr<const ArrayPtr<const word>> segments);

// serialize-packed.h:114-124: the MessageBuilder overloads -- any builder whose
// getSegmentsForOutput() yields the segment list (arena.c++:300-329).
template <typename Builder>
auto writePackedMessage(BufferedOutputStream& output, Builder& builder)
    -> decltype(builder.getSegmentsForOutput(), void()) {
  writePackedMessage(output, builder.getSegmentsForOutput());
}
template <typename Builder>
auto writePackedMessage(OutputStream& output, Builder& builder)
    -> decltype(builder.getSegmentsForOutput(), void()) {
  writePackedMessage(output, builder.getSegmentsForOutput());
}
template <typename Builder>
auto writePackedMessageToFd(int fd, Builder& builder)
    -> decltype(builder.getSegmentsForOutput(), void()) {
  writePackedMessageToFd(fd, builder.getSegmentsForOutput());
}

// serialize-packed.h:107.
size_t computeUnpackedSizeInWords(ArrayPtr<const byte> packedBytes);

// ---- async message streams (serialize-async.h:42-108) with packed framing ------------------
// std::future stands in for kj::Promise and std::unique_ptr for kj::Own.  File descriptors
// attached to messages (the fdSpace / fds overloads, SCM_RIGHTS over capability streams) are not
// carried: they are no part of the packed path.
class MessageStream {
 public:
  virtual ~MessageStream() = default;
  // serialize-async.h:54-57: the next message, or null at a clean end of the stream (the input
  // ends before the message's first byte).  scratchSpace must outlive the returned reader.
  virtual std::future<std::unique_ptr<MessageReader>> tryReadMessage(
      ReaderOptions options = ReaderOptions(), ArrayPtr<word> scratchSpace = nullptr) = 0;
  // serialize-async.c++:518-529: like tryReadMessage, but "Premature EOF." at the end.
  virtual std::future<std::unique_ptr<MessageReader>> readMessage(
      ReaderOptions options = ReaderOptions(), ArrayPtr<word> scratchSpace = nullptr) = 0;
  // serialize-async.h:78-83.  The segments must stay valid until the future is ready.
  virtual std::future<void> writeMessage(ArrayPtr<const ArrayPtr<const word>> segments) = 0;
  // serialize-async.h:88-93: a batch of messages, written back to back in one go.
  virtual std::future<void> writeMessages(
      ArrayPtr<const ArrayPtr<const ArrayPtr<const word>>> messages) = 0;
  template <typename Builder>
  auto writeMessage(Builder& builder) -> decltype(builder.getSegmentsForOutput(),
                                                  std::future<void>()) {
    return writeMessage(builder.getSegmentsForOutput());
  }
  // serialize-async.h:95: SO_SNDBUF of the underlying socket, if it is one.
  virtual std::optional<int> getSendBufferSize() = 0;
  // serialize-async.h:105: shut down the write end (after every write already started).
  virtual std::future<void> end() = 0;
};

// The packed counterpart of AsyncIoMessageStream (serialize-async.h:110-133) over a socket, pipe
// or file descriptor: what a writePackedMessage / PackedMessageReader pair exchanges, with each
// call running on the stream's own reader or writer thread (reads in order, writes in order,
// the two directions independent).  Reads decode on the device exactly as PackedMessageReader
// does, taking from the stream only the bytes of the message; a batch write packs every message
// of the batch in one device call and issues one write(2).
class PackedMessageStream final : public MessageStream {
 public:
  explicit PackedMessageStream(int fd, size_t bufferSizeInWords = 8192);
  explicit PackedMessageStream(OwnFd fd, size_t bufferSizeInWords = 8192);
  ~PackedMessageStream() override;  // waits for the operations already started
  PackedMessageStream(const PackedMessageStream&) = delete;
  PackedMessageStream& operator=(const PackedMessageStream&) = delete;

  std::future<std::unique_ptr<MessageReader>> tryReadMessage(
      ReaderOptions options = ReaderOptions(), ArrayPtr<word> scratchSpace = nullptr) override;
  std::future<std::unique_ptr<MessageReader>> readMessage(
      ReaderOptions options = ReaderOptions(), ArrayPtr<word> scratchSpace = nullptr) override;
  std::future<void> writeMessage(ArrayPtr<const ArrayPtr<const word>> segments) override;
  std::future<void> writeMessages(
      ArrayPtr<const ArrayPtr<const ArrayPtr<const word>>> messages) override;
  using MessageStream::writeMessage;
  std::optional<int> getSendBufferSize() override;
  std::future<void> end() override;

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

}  // namespace cpk_capnp

#endif  // CPK_CAPNP_H_
