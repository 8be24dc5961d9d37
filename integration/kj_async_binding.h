// kj_async_binding.h -- the packed codec behind the reference's ASYNC message interface:
// cpk_kj::PackedMessageStream is a capnp::MessageStream (serialize-async.h:42-108) over a
// kj::AsyncIoStream, the packed counterpart of capnp::AsyncIoMessageStream (:110-133).  It is
// what an event-loop code base (an RPC transport, a log shipper) drops in where it would write
// writePackedMessage / read PackedMessageReader on a socket: every message is packed and unpacked
// by libcpk_hip.so; kj's event loop only moves bytes.  Header-only, built against the reference's
// kj-async and capnp headers; run on the GPU box by
// tests/test_gpu_async_binding.py through integration/kj_async_binding_test.c++.
//
//   tryReadMessage  reads from the stream into a byte buffer, asks the device for one message
//                   (cpk_read_packed_message_host); CPK_ERR_PREMATURE_EOF means "read more and
//                   retry".  After a failed attempt the next one waits until the buffered bytes
//                   have doubled, unless a stream read comes back short (the peer paused: the
//                   message may be complete, and a request/response peer sends nothing more
//                   until it is read) or the stream ends.  A message streamed without pauses
//                   costs O(log size) device attempts and O(size) bytes uploaded, however the
//                   socket fragments it; each pause of the peer inside a message adds one.  Bytes past the message stay
//                   buffered for the next call (back-to-back messages, one stream read).  A clean
//                   end before the first byte is kj::none; an end inside a message is
//                   DISCONNECTED "Premature EOF." (serialize-async.c++:92, :525).  The flat
//                   words land in scratchSpace when it is large enough, else in an array the
//                   reader owns (serialize.c++:244-249).
//   writeMessage    one device pack (the façade's writePackedMessage), one stream write.
//   writeMessages   the whole batch gathered flat and packed in ONE device call
//                   (cpk_pack_messages_host), one stream write.
//   getSendBufferSize  the reference's AsyncIoMessageStream answer for the same stream
//                   (serialize-async.c++:457-486); end  shutdownWrite, as it does.
// File descriptors attached to messages are not carried (no part of the packed path): a write
// with fds is refused, reads return no fds.
#pragma once

#include <capnp/serialize-async.h>
#include <kj/async-io.h>
#include <kj/debug.h>
#include <sys/socket.h>

#include <cstring>
#include <vector>

#include "kj_binding.h"

namespace cpk_kj {

// The flat words of one message (segment table + segments, serialize.c++:161-190) as a
// capnp::MessageReader; owns its words unless they live in the caller's scratch space.
class FlatWordsMessageReader final : public capnp::MessageReader {
 public:
  FlatWordsMessageReader(kj::Array<capnp::word> owned, kj::ArrayPtr<const capnp::word> words,
                         capnp::ReaderOptions options)
      : capnp::MessageReader(options), owned_(kj::mv(owned)) {
    const uint32_t* t = reinterpret_cast<const uint32_t*>(words.begin());
    // (the device read rejected such a header already; this reader allocates from it, so it checks
    // again: serialize.c++:217, and the UINT_MAX case of serialize-test.c++:533-543)
    KJ_REQUIRE(words.size() > 0 && t[0] < 511, "Message has too many segments.");
    const size_t nseg = size_t(t[0]) + 1;
    KJ_REQUIRE(nseg / 2 + 1 <= words.size(), "segment table disagrees with the words");
    size_t off = nseg / 2 + 1;
    segs_ = kj::heapArray<kj::ArrayPtr<const capnp::word>>(nseg);
    for (size_t i = 0; i < nseg; i++) {
      KJ_REQUIRE(off + t[1 + i] <= words.size(), "segment table disagrees with the words");
      segs_[i] = words.slice(off, off + t[1 + i]);
      off += t[1 + i];
    }
  }
  kj::ArrayPtr<const capnp::word> getSegment(uint id) override {
    return id < segs_.size() ? segs_[id] : nullptr;
  }

 private:
  kj::Array<capnp::word> owned_;
  kj::Array<kj::ArrayPtr<const capnp::word>> segs_;
};

inline void throw_status(cpk_status st) {
  KJ_FAIL_REQUIRE(cpk_status_string(st), int(st));
}

class PackedMessageStream final : public capnp::MessageStream {
 public:
  explicit PackedMessageStream(kj::AsyncIoStream& stream, size_t bufferSizeInWords = 8192)
      : stream_(stream), readSize_(bufferSizeInWords * sizeof(capnp::word)) {}

  kj::Promise<kj::Maybe<capnp::MessageReaderAndFds>> tryReadMessage(
      kj::ArrayPtr<kj::OwnFd> fdSpace, capnp::ReaderOptions options = capnp::ReaderOptions(),
      kj::ArrayPtr<capnp::word> scratchSpace = nullptr) override {
    (void)fdSpace;
    return readLoop(options, scratchSpace);
  }

  kj::Promise<void> writeMessage(kj::ArrayPtr<const int> fds,
                                 kj::ArrayPtr<const kj::ArrayPtr<const capnp::word>> segments)
      override {
    KJ_REQUIRE(fds.size() == 0, "file descriptors are not carried by the packed stream");
    kj::VectorOutputStream out;
    writePackedMessage(out, segments);  // kj_binding.h: one device pack
    return writeBytes(kj::heapArray(out.getArray()));
  }

  kj::Promise<void> writeMessages(
      kj::ArrayPtr<kj::ArrayPtr<const kj::ArrayPtr<const capnp::word>>> messages) override {
    if (messages.size() == 0) return kj::READY_NOW;
    // Gather every message flat (table + segments), then pack the batch in one device call.
    std::vector<uint64_t> off(messages.size() + 1, 0);
    uint64_t chunks = 0;
    for (size_t i = 0; i < messages.size(); i++) {
      KJ_REQUIRE(messages[i].size() > 0, "Tried to serialize uninitialized message.");
      uint64_t w = messages[i].size() / 2 + 1;
      for (auto& s : messages[i]) w += s.size();
      off[i + 1] = off[i] + w;
      chunks += messages[i].size() + 1;
    }
    std::vector<uint64_t> flat(off.back(), 0);
    for (size_t i = 0; i < messages.size(); i++) {
      uint32_t* t = reinterpret_cast<uint32_t*>(flat.data() + off[i]);
      t[0] = uint32_t(messages[i].size() - 1);
      uint64_t w = off[i] + messages[i].size() / 2 + 1;
      for (size_t s = 0; s < messages[i].size(); s++) {
        const auto& seg = messages[i][s];
        t[1 + s] = uint32_t(seg.size());
        if (seg.size()) memcpy(flat.data() + w, seg.begin(), seg.size() * sizeof(capnp::word));
        w += seg.size();
      }
    }
    const uint64_t cap = cpk_packed_bound(off.back(), chunks);
    auto bytes = kj::heapArray<kj::byte>(cap);
    std::vector<uint64_t> out_off(messages.size() + 1);
    std::vector<int32_t> status(messages.size());
    cpk_status st = cpk_pack_messages_host(cpk_capnp::threadContext(), flat.data(), off.back(),
                                           off.data(), messages.size(), bytes.begin(), cap,
                                           out_off.data(), status.data());
    if (st != CPK_OK) throw_status(st);
    for (auto s : status)
      if (s != CPK_OK) throw_status(cpk_status(s));
    return writeBytes(kj::heapArray(bytes.slice(0, out_off.back())));
  }

  kj::Maybe<int> getSendBufferSize() override {
    // the reference's own answer for this stream (SO_SNDBUF on a socket, none otherwise):
    // AsyncIoMessageStream::getSendBufferSize, serialize-async.c++:484-486
    return capnp::AsyncIoMessageStream(stream_).getSendBufferSize();
  }

  kj::Promise<void> end() override {
    stream_.shutdownWrite();
    return kj::READY_NOW;
  }

  using capnp::MessageStream::tryReadMessage;
  using capnp::MessageStream::writeMessage;

  // Bytes read from the stream but not yet consumed by a message.
  size_t buffered() const { return end_ - begin_; }

 private:
  kj::Promise<void> writeBytes(kj::Array<kj::byte> bytes) {
    auto p = stream_.write(bytes.asPtr());
    return p.attach(kj::mv(bytes));
  }

  // One device attempt at the buffered bytes: the message, or kj::none when more input is needed.
  kj::Maybe<kj::Own<capnp::MessageReader>> tryDecode(capnp::ReaderOptions options,
                                                      kj::ArrayPtr<capnp::word> scratch) {
    cpk_limits lim{options.traversalLimitInWords};
    const uint8_t* src = buf_.data() + begin_;
    const uint64_t avail = end_ - begin_;
    uint64_t nw = 0, used = 0;
    kj::Array<capnp::word> owned;
    uint64_t* dst = reinterpret_cast<uint64_t*>(scratch.begin());
    uint64_t cap = scratch.size();
    if (cap == 0) {
      // a first guess; when the message is larger the device reports its exact size
      // (CPK_ERR_CAPACITY with *words_out) and the second attempt fits
      cap = std::max<uint64_t>(64, std::min<uint64_t>(avail, 1 << 20));
      owned = kj::heapArray<capnp::word>(cap);
      dst = reinterpret_cast<uint64_t*>(owned.begin());
    }
    cpk_status st = cpk_read_packed_message_host(cpk_capnp::threadContext(), src, avail, dst, cap,
                                                 &nw, &used, &lim);
    if (st == CPK_ERR_CAPACITY) {
      owned = kj::heapArray<capnp::word>(nw);
      dst = reinterpret_cast<uint64_t*>(owned.begin());
      st = cpk_read_packed_message_host(cpk_capnp::threadContext(), src, avail, dst, nw, &nw,
                                        &used, &lim);
    }
    if (st == CPK_ERR_PREMATURE_EOF) return kj::none;
    if (st != CPK_OK) throw_status(st);
    begin_ += used;
    kj::ArrayPtr<const capnp::word> words(reinterpret_cast<const capnp::word*>(dst), nw);
    return kj::Own<capnp::MessageReader>(
        kj::heap<FlatWordsMessageReader>(kj::mv(owned), words, options));
  }

  kj::Promise<kj::Maybe<capnp::MessageReaderAndFds>> readLoop(capnp::ReaderOptions options,
                                                               kj::ArrayPtr<capnp::word> scratch,
                                                               bool paused = true) {
    if (end_ > begin_ && (paused || end_ - begin_ >= retryAt_)) {
      KJ_IF_SOME(r, tryDecode(options, scratch)) {
        retryAt_ = failedAt_ = 0;
        return kj::Maybe<capnp::MessageReaderAndFds>(capnp::MessageReaderAndFds{kj::mv(r), nullptr});
      }
      failedAt_ = end_ - begin_;
      retryAt_ = 2 * failedAt_;  // next attempt once the buffered bytes have doubled
    }
    // Need more input: compact, then read at least as much as is already buffered.
    if (begin_ > 0) {
      memmove(buf_.data(), buf_.data() + begin_, end_ - begin_);
      end_ -= begin_;
      begin_ = 0;
    }
    const size_t want = std::max(readSize_, end_);
    if (buf_.size() < end_ + want) buf_.resize(end_ + want);
    return stream_.tryRead(buf_.data() + end_, 1, want)
        .then([this, options, scratch, want](size_t n) mutable -> kj::Promise<kj::Maybe<capnp::MessageReaderAndFds>> {
          if (n == 0) {
            if (end_ == begin_) return kj::Maybe<capnp::MessageReaderAndFds>(kj::none);
            if (end_ - begin_ != failedAt_) {
              // the stream ended before the buffer doubled: one last attempt at what there is
              KJ_IF_SOME(r, tryDecode(options, scratch)) {
                retryAt_ = failedAt_ = 0;
                return kj::Maybe<capnp::MessageReaderAndFds>(
                    capnp::MessageReaderAndFds{kj::mv(r), nullptr});
              }
            }
            kj::throwRecoverableException(KJ_EXCEPTION(DISCONNECTED, "Premature EOF."));
            return kj::Maybe<capnp::MessageReaderAndFds>(kj::none);
          }
          end_ += n;
          return readLoop(options, scratch, n < want);  // a short read: the peer paused
        });
  }

  kj::AsyncIoStream& stream_;
  size_t readSize_;
  std::vector<uint8_t> buf_;
  size_t begin_ = 0, end_ = 0;
  size_t retryAt_ = 0;   // buffered bytes needed before the next device attempt
  size_t failedAt_ = 0;  // buffered bytes at the last failed attempt
};

}  // namespace cpk_kj
