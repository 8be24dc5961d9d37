// kj_async_binding_test.c++ -- the reference's async message interface (capnp::MessageStream,
// serialize-async.h:42-108) with packed framing, through integration/kj_async_binding.h, on the
// reference's own kj event loop (kj::setupAsyncIo) and the device codec.  Built by
// oracle/Makefile.ref against the reference's kj / kj-async / capnp objects WITHOUT its
// serialize-packed.o; run on the GPU box by tests/test_gpu_async_binding.py.
//
// The flows follow serialize-async-test.c++ (a message written on one end of a socket pair is
// read on the other; several messages back to back; EOF rules) with the reference's fixtures as
// the messages and their packed files as the expected wire bytes:
//   1. writeMessage of binary / segmented / addressbook.bin over a socketpair: the raw bytes the
//      peer receives == packed / segmented-packed / addressbook.packed;
//   2. the fixture's packed bytes written raw in fragments (1, 7, 64 B and whole) are read back by
//      tryReadMessage, segments == the reference's FlatArrayMessageReader; into scratch space;
//   3. writeMessages of all three in one batch, read back as three messages, then end() and a
//      clean EOF (kj::none); a message cut short then EOF -> DISCONNECTED "Premature EOF.";
//   4. the same over an in-memory kj::newTwoWayPipe (getSendBufferSize none; socket > 0);
//   5. a traversal limit below the message size -> "Message is too large.".
//
//   kj_async_binding_test <tests/golden dir>     -> prints "async binding ok: N checks", exit 0
#include <capnp/serialize.h>
#include <kj/async-io.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "kj_async_binding.h"

namespace {

int checks = 0;

void step(const std::string& what) { std::fprintf(stderr, "[step] %s\n", what.c_str()); }

void check(bool ok, const std::string& what) {
  ++checks;
  if (!ok) {
    std::fprintf(stderr, "FAILED: %s\n", what.c_str());
    std::exit(1);
  }
}

std::vector<kj::byte> read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  check(bool(f), "open " + path);
  return std::vector<kj::byte>(std::istreambuf_iterator<char>(f), {});
}

struct Fixture {
  std::string name;
  kj::Array<capnp::word> words;
  std::vector<kj::byte> packed;
  kj::Own<capnp::FlatArrayMessageReader> reader;
  std::vector<kj::ArrayPtr<const capnp::word>> segs;
  Fixture(const std::string& dir, const std::string& src, const std::string& dst) : name(src) {
    auto bytes = read_file(dir + "/" + src);
    packed = read_file(dir + "/" + dst);
    words = kj::heapArray<capnp::word>(bytes.size() / 8);
    memcpy(words.begin(), bytes.data(), bytes.size());
    reader = kj::heap<capnp::FlatArrayMessageReader>(words.asPtr());
    for (uint i = 0;; i++) {
      auto s = reader->getSegment(i);
      if (s == nullptr) break;
      segs.push_back(s);
    }
  }
  kj::ArrayPtr<const kj::ArrayPtr<const capnp::word>> pieces() const {
    return kj::arrayPtr(segs.data(), segs.size());
  }
};

void same_segments(capnp::MessageReader& r, const Fixture& f, const std::string& what) {
  for (uint i = 0; i < f.segs.size(); i++) {
    auto s = r.getSegment(i);
    check(s.size() == f.segs[i].size() &&
              memcmp(s.begin(), f.segs[i].begin(), s.size() * sizeof(capnp::word)) == 0,
          what + ": " + f.name + " segment " + std::to_string(i));
  }
  check(r.getSegment(f.segs.size()) == nullptr, what + ": " + f.name + " segment count");
}

// Raw bytes from a stream until `n` have arrived (or EOF).
std::vector<kj::byte> read_raw(kj::AsyncIoStream& s, size_t n, kj::WaitScope& ws) {
  std::vector<kj::byte> v(n);
  size_t got = 0;
  while (got < n) {
    size_t k = s.tryRead(v.data() + got, 1, n - got).wait(ws);
    if (k == 0) break;
    got += k;
  }
  v.resize(got);
  return v;
}

void run(kj::AsyncIoStream& a, kj::AsyncIoStream& b, const std::vector<Fixture>& fx,
         kj::WaitScope& ws, const std::string& kind) {
  cpk_kj::PackedMessageStream sa(a), sb(b);

  // 1. writeMessage -> raw wire bytes
  step(kind + ": writeMessage");
  for (auto& f : fx) {
    auto w = sa.writeMessage(f.pieces());
    auto got = read_raw(b, f.packed.size(), ws);
    w.wait(ws);
    check(got == f.packed, kind + ": writeMessage bytes of " + f.name);
  }

  // 2. raw packed bytes in fragments -> tryReadMessage
  step(kind + ": fragments");
  for (size_t frag : {size_t(1), size_t(7), size_t(64), size_t(1) << 30}) {
    for (auto& f : fx) {
      auto wr = kj::evalLater([&a, &f, frag]() -> kj::Promise<void> {
        kj::Promise<void> p = kj::READY_NOW;
        for (size_t o = 0; o < f.packed.size(); o += frag) {
          const size_t k = std::min(frag, f.packed.size() - o);
          p = p.then([&a, &f, o, k]() { return a.write(kj::arrayPtr(f.packed.data() + o, k)); });
        }
        return p;
      });
      auto r = sb.readMessage().wait(ws);
      wr.wait(ws);
      same_segments(*r, f, kind + ": fragments of " + std::to_string(frag));
    }
  }
  check(sb.buffered() == 0, kind + ": nothing left buffered");
  {
    // into caller scratch space (serialize.c++:244-249)
    auto& f = fx[0];
    std::vector<capnp::word> scratch(f.words.size() + 8);
    auto w = a.write(kj::arrayPtr(f.packed.data(), f.packed.size()));
    auto r = sb.readMessage(capnp::ReaderOptions(), kj::arrayPtr(scratch.data(), scratch.size()))
                 .wait(ws);
    w.wait(ws);
    same_segments(*r, f, kind + ": scratch");
    check(r->getSegment(0).begin() >= scratch.data() &&
              r->getSegment(0).end() <= scratch.data() + scratch.size(),
          kind + ": segment 0 lives in the scratch space");
  }

  // 3. writeMessages (one device pack) -> three reads; then end() -> clean EOF
  step(kind + ": writeMessages");
  {
    std::vector<kj::ArrayPtr<const kj::ArrayPtr<const capnp::word>>> batch;
    for (auto& f : fx) batch.push_back(f.pieces());
    auto w = sa.writeMessages(kj::arrayPtr(batch.data(), batch.size()));
    for (auto& f : fx) {
      auto r = sb.readMessage().wait(ws);
      same_segments(*r, f, kind + ": writeMessages batch");
    }
    w.wait(ws);
  }
  {
    // a batch's wire bytes are the fixtures' packed files back to back
    std::vector<kj::ArrayPtr<const kj::ArrayPtr<const capnp::word>>> batch;
    std::vector<kj::byte> want;
    for (auto& f : fx) {
      batch.push_back(f.pieces());
      want.insert(want.end(), f.packed.begin(), f.packed.end());
    }
    auto w = sa.writeMessages(kj::arrayPtr(batch.data(), batch.size()));
    auto got = read_raw(b, want.size(), ws);
    w.wait(ws);
    check(got == want, kind + ": writeMessages bytes");
  }
  {
    // 5. traversal limit
    step(kind + ": traversal limit");
    auto& f = fx[0];
    capnp::ReaderOptions small;
    small.traversalLimitInWords = 1;
    cpk_kj::PackedMessageStream sc(b);
    auto w = a.write(kj::arrayPtr(f.packed.data(), f.packed.size()));
    bool threw = false;
    KJ_IF_SOME(e, kj::runCatchingExceptions([&]() { sc.readMessage(small).wait(ws); })) {
      threw = e.getDescription().contains("Message is too large");
    }
    w.wait(ws);
    check(threw, kind + ": traversal limit -> Message is too large.");
  }
  {
    // a message cut short, then end of stream -> "Premature EOF."
    step(kind + ": premature EOF");
    // (an in-memory pipe's write completes only once the peer reads, so the write and the end()
    // after it run while the reader waits)
    auto& f = fx[1];
    auto w = a.write(kj::arrayPtr(f.packed.data(), f.packed.size() / 2)).then([&sa]() {
      return sa.end();
    });
    cpk_kj::PackedMessageStream sd(b);
    bool threw = false;
    KJ_IF_SOME(e, kj::runCatchingExceptions([&]() { sd.readMessage().wait(ws); })) {
      threw = e.getType() == kj::Exception::Type::DISCONNECTED &&
              e.getDescription().contains("Premature EOF");
    }
    w.wait(ws);
    check(threw, kind + ": cut message -> DISCONNECTED Premature EOF.");
  }
}

void clean_eof(kj::AsyncIoStream& a, kj::AsyncIoStream& b, const Fixture& f, kj::WaitScope& ws,
               const std::string& kind) {
  step(kind + ": clean EOF");
  cpk_kj::PackedMessageStream sa(a), sb(b);
  auto w = sa.writeMessage(f.pieces());
  auto r = sb.tryReadMessage().wait(ws);
  w.wait(ws);
  KJ_IF_SOME(m, r) { same_segments(*m, f, kind + ": tryReadMessage"); }
  else check(false, kind + ": tryReadMessage returned a message");
  sa.end().wait(ws);
  auto eof = sb.tryReadMessage().wait(ws);
  check(eof == kj::none, kind + ": clean EOF -> none");
}

// serialize-test.c++:533-543 on the async reader the advisory is about
// (security-advisories/2026-03-12-0-segment-count-overflow.md): a first word of
// ff ff ff ff 00 00 00 00 (packed 0f ff ff ff ff) is "Message has too many segments.".
void uint_max_segment_count(kj::AsyncIoStream& a, kj::AsyncIoStream& b, kj::WaitScope& ws,
                            const std::string& kind) {
  step(kind + ": UINT_MAX segment count");
  static const kj::byte bytes[] = {0x0f, 0xff, 0xff, 0xff, 0xff};
  // (not waited for before the read: an in-memory pipe's write completes only as it is read)
  auto w = a.write(kj::arrayPtr(bytes, sizeof(bytes))).eagerlyEvaluate(nullptr);
  cpk_kj::PackedMessageStream sb(b);
  bool threw = false;
  KJ_IF_SOME(e, kj::runCatchingExceptions([&]() { sb.readMessage().wait(ws); })) {
    threw = e.getDescription().contains("Message has too many segments.");
  }
  w.wait(ws);
  check(threw, kind + ": UINT_MAX segment count rejected (Message has too many segments.)");
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <tests/golden dir>\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  std::vector<Fixture> fx;
  fx.emplace_back(dir, "binary", "packed");
  fx.emplace_back(dir, "segmented", "segmented-packed");
  fx.emplace_back(dir, "addressbook.bin", "addressbook.packed");

  auto io = kj::setupAsyncIo();
  auto& ws = io.waitScope;
  {
    auto sock = io.provider->newTwoWayPipe();  // an OS socket pair
    cpk_kj::PackedMessageStream s(*sock.ends[0]);
    KJ_IF_SOME(n, s.getSendBufferSize()) { check(n > 0, "socket: SO_SNDBUF > 0"); }
    else check(false, "socket: getSendBufferSize returns a size");
    run(*sock.ends[0], *sock.ends[1], fx, ws, "socket");
  }
  {
    auto sock = io.provider->newTwoWayPipe();
    clean_eof(*sock.ends[0], *sock.ends[1], fx[2], ws, "socket");
  }
  {
    auto mem = kj::newTwoWayPipe();  // in-memory
    cpk_kj::PackedMessageStream s(*mem.ends[0]);
    check(s.getSendBufferSize() == kj::none, "in-memory pipe: no send buffer size");
    run(*mem.ends[0], *mem.ends[1], fx, ws, "in-memory");
  }
  {
    auto mem = kj::newTwoWayPipe();
    clean_eof(*mem.ends[0], *mem.ends[1], fx[0], ws, "in-memory");
  }
  {
    auto sock = io.provider->newTwoWayPipe();
    uint_max_segment_count(*sock.ends[0], *sock.ends[1], ws, "socket");
  }
  {
    auto mem = kj::newTwoWayPipe();
    uint_max_segment_count(*mem.ends[0], *mem.ends[1], ws, "in-memory");
  }
  std::printf("async binding ok: %d checks (socket pair + in-memory pipe, %zu fixtures)\n",
              checks, fx.size());
  return 0;
}
