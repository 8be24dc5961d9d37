// cpk_stream_async.cpp -- PackedMessageStream (include/cpk_capnp.h): the MessageStream interface
// of serialize-async.h:42-108 with packed framing, over a socket / pipe / file descriptor.
//
// Each direction has its own worker thread (and so its own cpk_ctx, cpk.h: one context per host
// thread), which runs the calls of that direction in the order they were made: a read waits for
// the reads before it, a write for the writes before it, and a read never waits for a write.
// The futures returned to the caller stand in for kj::Promise.
//
//   reads   PackedMessageReader over the stream's buffered fd (serialize-async.c++:84-97 for the
//           EOF rule): no byte before the message's first -> null; otherwise the segment table,
//           then every segment, decoded on the device and taken from the stream up to the
//           message's last record -- the next message's bytes stay buffered for the next read.
//   writes  writeMessages (serialize-async.c++:302-349) packs the whole batch -- each message's
//           table and segments as separate chunks, exactly writePackedMessage's bytes -- in ONE
//           device call (cpk_pack_messages_host) and writes it with one write loop.
#include <errno.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>

#include "../../include/cpk_capnp.h"

namespace cpk_capnp {

namespace {

// Runs submitted tasks one after another on its own thread; the destructor lets the queued
// tasks finish, then joins.
class Serial {
 public:
  Serial() : th_([this] { run(); }) {}
  ~Serial() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  template <class F>
  auto submit(F f) -> std::future<decltype(f())> {
    using R = decltype(f());
    auto task = std::make_shared<std::packaged_task<R()>>(std::move(f));
    std::future<R> fut = task->get_future();
    {
      std::lock_guard<std::mutex> lk(m_);
      q_.push_back([task] { (*task)(); });
    }
    cv_.notify_one();
    return fut;
  }

 private:
  void run() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        job = std::move(q_.front());
        q_.pop_front();
      }
      job();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
  std::thread th_;
};

[[noreturn]] void fail(cpk_status st, const char* where) { throw Exception(st, where); }

// One message's segment list, copied at submission (the segment words themselves are read when
// the write runs, as the reference's "parameters must remain valid" contract allows).
typedef std::vector<ArrayPtr<const word>> SegList;

}  // namespace

struct PackedMessageStream::Impl {
  OwnFd owned;
  int fd;
  FdBufferedInputStream in;
  bool write_closed = false;
  // declared last: destroyed (joined) first, while the stream state their tasks use still exists
  Serial reader, writer;

  Impl(int f, size_t bufferWords) : fd(f), in(f, std::max<size_t>(bufferWords, 1) * 8) {}
  Impl(OwnFd f, size_t bufferWords)
      : owned(std::move(f)), fd(owned.get()), in(fd, std::max<size_t>(bufferWords, 1) * 8) {}

  std::unique_ptr<MessageReader> read_one(ReaderOptions options, ArrayPtr<word> scratch) {
    // serialize-async.c++:86-95: end of stream before the first word -> no message
    if (in.tryGetReadBuffer().size() == 0) return nullptr;
    auto r = std::make_unique<PackedMessageReader>(in, options, scratch);
    // the whole message now (the lazy reads of serialize.c++:283-302 would otherwise reach into
    // the stream after the next message has been read from it)
    r->getSegment((unsigned)(r->segmentCount() - 1));
    return r;
  }

  void write_batch(const std::vector<SegList>& msgs) {
    // serialize-async.c++:304 / serialize.c++:333
    if (msgs.empty()) fail(CPK_ERR_INVALID_ARGUMENT, "Tried to serialize zero messages.");
    std::vector<uint64_t> off(1, 0);
    uint64_t bound = 0;
    for (const SegList& segs : msgs) {
      if (segs.empty()) fail(CPK_ERR_EMPTY_MESSAGE, "MessageStream::writeMessages");
      uint64_t words = segs.size() / 2 + 1;
      for (auto& s : segs) words += s.size();
      off.push_back(off.back() + words);
      bound += cpk_packed_bound(words, segs.size() + 1);
    }
    // the flat messages back to back: table (serialize.c++:311-330), then the segments
    std::vector<uint64_t> flat(off.back(), 0);
    for (size_t m = 0; m < msgs.size(); m++) {
      const SegList& segs = msgs[m];
      uint64_t* w = flat.data() + off[m];
      uint32_t* t = reinterpret_cast<uint32_t*>(w);
      t[0] = (uint32_t)(segs.size() - 1);
      for (size_t i = 0; i < segs.size(); i++) t[i + 1] = (uint32_t)segs[i].size();
      uint64_t at = segs.size() / 2 + 1;
      for (auto& s : segs) {
        if (s.size()) memcpy(w + at, s.begin(), s.size() * 8);
        at += s.size();
      }
    }
    std::vector<uint8_t> out(bound + 16);
    std::vector<uint64_t> out_off(msgs.size() + 1, 0);
    std::vector<int32_t> status(msgs.size(), 0);
    const cpk_status st =
        cpk_pack_messages_host(threadContext(), flat.data(), flat.size(), off.data(), msgs.size(),
                               out.data(), out.size(), out_off.data(), status.data());
    if (st != CPK_OK) fail(st, "MessageStream::writeMessages");
    for (int32_t s : status)
      if (s != CPK_OK) fail((cpk_status)s, "MessageStream::writeMessages");
    if (write_closed) fail(CPK_ERR_INVALID_ARGUMENT, "write after end()");
    FdOutputStream(fd).write(out.data(), out_off.back());
  }
};

PackedMessageStream::PackedMessageStream(int fd, size_t bufferSizeInWords)
    : impl_(new Impl(fd, bufferSizeInWords)) {}

PackedMessageStream::PackedMessageStream(OwnFd fd, size_t bufferSizeInWords)
    : impl_(new Impl(std::move(fd), bufferSizeInWords)) {}

PackedMessageStream::~PackedMessageStream() = default;

std::future<std::unique_ptr<MessageReader>> PackedMessageStream::tryReadMessage(
    ReaderOptions options, ArrayPtr<word> scratchSpace) {
  Impl* im = impl_.get();
  return im->reader.submit([im, options, scratchSpace] { return im->read_one(options, scratchSpace); });
}

std::future<std::unique_ptr<MessageReader>> PackedMessageStream::readMessage(
    ReaderOptions options, ArrayPtr<word> scratchSpace) {
  Impl* im = impl_.get();
  return im->reader.submit([im, options, scratchSpace] {
    auto r = im->read_one(options, scratchSpace);
    if (!r) fail(CPK_ERR_PREMATURE_EOF, "Premature EOF.");  // serialize-async.c++:518-529
    return r;
  });
}

std::future<void> PackedMessageStream::writeMessage(ArrayPtr<const ArrayPtr<const word>> segments) {
  Impl* im = impl_.get();
  std::vector<SegList> one(1, SegList(segments.begin(), segments.end()));
  return im->writer.submit([im, one] { im->write_batch(one); });
}

std::future<void> PackedMessageStream::writeMessages(
    ArrayPtr<const ArrayPtr<const ArrayPtr<const word>>> messages) {
  Impl* im = impl_.get();
  std::vector<SegList> batch;
  batch.reserve(messages.size());
  for (auto& m : messages) batch.emplace_back(m.begin(), m.end());
  return im->writer.submit([im, batch] { im->write_batch(batch); });
}

std::optional<int> PackedMessageStream::getSendBufferSize() {
  // serialize-async.c++:457-477: SO_SNDBUF, none when the descriptor is not a socket
  int size = 0;
  socklen_t len = sizeof(size);
  if (getsockopt(impl_->fd, SOL_SOCKET, SO_SNDBUF, &size, &len) != 0 || len != sizeof(size))
    return std::nullopt;
  return size;
}

std::future<void> PackedMessageStream::end() {
  // serialize-async.c++:479-482 (AsyncIoStream::shutdownWrite): a socket's write half is shut
  // down; a descriptor that is not a socket (a pipe's write end) is closed when the stream owns it
  Impl* im = impl_.get();
  return im->writer.submit([im] {
    im->write_closed = true;
    if (shutdown(im->fd, SHUT_WR) == 0) return;
    if (errno == ENOTSOCK) {
      if (im->owned.get() >= 0) im->owned = OwnFd();
      return;
    }
    fail(CPK_ERR_INVALID_ARGUMENT, "shutdown(fd)");
  });
}

}  // namespace cpk_capnp
