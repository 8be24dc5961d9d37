// stream_test.cpp -- PackedMessageStream (include/cpk_capnp.h): the MessageStream interface of
// serialize-async.h:42-133 with packed framing, on the MI355X codec, over socket pairs and
// pipes.  Restates the shape of serialize-async-test.c++ (messages written on one end read back
// on the other, EOF as null, "Premature EOF." from readMessage, batched writes) and pins the wire
// bytes against writePackedMessage and the reference's fixtures (tests/golden).
//
//   cpk_stream_test <tests/golden dir>        exit 0 = all checks passed
#include <fcntl.h>
#include <stdio.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <fstream>
#include <algorithm>
#include <iterator>
#include <random>
#include <string>
#include <thread>
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

// A message: owned segment words.
struct Msg {
  std::vector<std::vector<word>> segs;
  std::vector<ArrayPtr<const word>> ptrs() const {
    std::vector<ArrayPtr<const word>> p;
    for (auto& s : segs) p.emplace_back(s.data(), s.size());
    return p;
  }
};

// Unpacked message file (stream framing) -> Msg.
static Msg msg_of(const std::vector<byte>& f) {
  Msg m;
  const uint32_t* t = reinterpret_cast<const uint32_t*>(f.data());
  const uint32_t n = t[0] + 1;
  const word* w = reinterpret_cast<const word*>(f.data());
  size_t at = n / 2 + 1;
  for (uint32_t i = 0; i < n; i++) {
    m.segs.emplace_back(w + at, w + at + t[i + 1]);
    at += t[i + 1];
  }
  return m;
}

// Struct-like words: small ints, zeros, pointers, text (runs of every kind appear).
static Msg random_msg(std::mt19937_64& rng, int nseg, size_t max_words) {
  Msg m;
  for (int s = 0; s < nseg; s++) {
    std::vector<word> seg(1 + rng() % max_words);
    for (auto& w : seg) {
      const uint64_t r = rng();
      switch (r % 5) {
        case 0: w.content = 0; break;
        case 1: w.content = r >> 40; break;
        case 2: w.content = (r >> 8) | 0x0101010101010101ull; break;  // no zero byte
        case 3: w.content = (r & 0xffff) << 32; break;
        default: w.content = r; break;
      }
      if (rng() % 7 == 0) {  // a zero stretch
        w.content = 0;
      }
    }
    m.segs.push_back(seg);
  }
  return m;
}

static bool same(MessageReader& r, const Msg& m) {
  for (size_t i = 0; i < m.segs.size(); i++) {
    auto s = r.getSegment((unsigned)i);
    if (s.size() != m.segs[i].size()) return false;
    if (s.size() && memcmp(s.begin(), m.segs[i].data(), s.size() * 8) != 0) return false;
  }
  return r.getSegment((unsigned)m.segs.size()).size() == 0;
}

static std::vector<byte> packed_bytes(const Msg& m) {
  VectorOutputStream out;
  auto p = m.ptrs();
  writePackedMessage(out, ArrayPtr<const ArrayPtr<const word>>(p.data(), p.size()));
  auto a = out.getArray();
  return std::vector<byte>(a.begin(), a.end());
}

// Messages written on one end of a socket pair come back on the other, in order; end() makes
// the next read null (serialize-async-test.c++ "MessageStream"), and readMessage then throws.
static void socket_round_trip(const std::string& dir) {
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return;
  std::vector<Msg> msgs = {msg_of(read_file(dir + "/binary")), msg_of(read_file(dir + "/segmented")),
                           msg_of(read_file(dir + "/addressbook.bin"))};
  std::mt19937_64 rng(20261016);
  for (int i = 0; i < 5; i++) msgs.push_back(random_msg(rng, 1 + i % 3, 3000));
  PackedMessageStream a{OwnFd(sv[0])}, b{OwnFd(sv[1])};
  // the read is requested before anything is written: it waits on the reader thread
  auto first = b.tryReadMessage();
  CHECK(first.wait_for(std::chrono::milliseconds(50)) == std::future_status::timeout,
        "a read with no data pending does not complete");
  std::vector<std::vector<ArrayPtr<const word>>> ptrs;
  for (auto& m : msgs) ptrs.push_back(m.ptrs());
  std::vector<std::future<void>> writes;
  for (auto& p : ptrs)
    writes.push_back(a.writeMessage(ArrayPtr<const ArrayPtr<const word>>(p.data(), p.size())));
  auto r0 = first.get();
  CHECK(r0 && same(*r0, msgs[0]), "socket: message 0");
  for (size_t i = 1; i < msgs.size(); i++) {
    auto r = b.readMessage().get();
    CHECK(r && same(*r, msgs[i]), "socket: message %zu", i);
  }
  for (auto& w : writes) w.get();
  CHECK(a.getSendBufferSize().has_value() && *a.getSendBufferSize() > 0, "socket SO_SNDBUF");
  a.end().get();
  auto eof = b.tryReadMessage().get();
  CHECK(!eof, "tryReadMessage after end() is null");
  bool threw = false;
  try {
    b.readMessage().get();
  } catch (const Exception& e) {
    threw = e.status() == CPK_ERR_PREMATURE_EOF;
  }
  CHECK(threw, "readMessage at EOF: Premature EOF.");
}

// writeMessages: one batch, one device call -- the bytes on the wire are writePackedMessage's for
// each message back to back, and the reader splits them again.
static void batch_write(const std::string& dir) {
  int p[2];
  if (pipe(p) != 0) return;
  std::mt19937_64 rng(7);
  std::vector<Msg> msgs;
  for (int i = 0; i < 40; i++) msgs.push_back(random_msg(rng, 1 + i % 4, 700));
  msgs.push_back(msg_of(read_file(dir + "/segmented")));
  std::vector<byte> expect;
  for (auto& m : msgs) {
    auto b = packed_bytes(m);
    expect.insert(expect.end(), b.begin(), b.end());
  }
  std::vector<std::vector<ArrayPtr<const word>>> ptrs;
  for (auto& m : msgs) ptrs.push_back(m.ptrs());
  std::vector<ArrayPtr<const ArrayPtr<const word>>> batch;
  for (auto& q : ptrs) batch.emplace_back(q.data(), q.size());
  {
    PackedMessageStream w{OwnFd(p[1])};
    CHECK(!w.getSendBufferSize().has_value(), "pipe: no SO_SNDBUF");
    // drain the pipe concurrently (the batch exceeds the pipe buffer)
    std::vector<byte> got;
    std::thread drain([&] {
      byte buf[65536];
      for (;;) {
        const ssize_t n = read(p[0], buf, sizeof(buf));
        if (n <= 0) break;
        got.insert(got.end(), buf, buf + n);
      }
    });
    w.writeMessages(ArrayPtr<const ArrayPtr<const ArrayPtr<const word>>>(batch.data(), batch.size()))
        .get();
    w.end().get();  // closes the owned write end: the drain sees EOF
    drain.join();
    CHECK(got == expect, "writeMessages bytes == writePackedMessage per message (%zu vs %zu B)",
          got.size(), expect.size());
    // and back through a reading stream
    int q[2];
    if (pipe(q) != 0) return;
    std::thread feed([&] {
      size_t at = 0;
      while (at < got.size()) {
        const ssize_t n = write(q[1], got.data() + at, std::min<size_t>(got.size() - at, 1000));
        if (n <= 0) break;
        at += (size_t)n;
      }
      close(q[1]);
    });
    PackedMessageStream r{OwnFd(q[0]), 64};  // a 512-byte read buffer: messages cross refills
    for (size_t i = 0; i < msgs.size(); i++) {
      auto m = r.tryReadMessage().get();
      CHECK(m && same(*m, msgs[i]), "batch: message %zu read back", i);
    }
    CHECK(!r.tryReadMessage().get(), "batch: clean end");
    feed.join();
  }
  close(p[0]);
}

// The reference's packed fixtures on the wire are read as the reference's messages; a stream cut
// inside a message is "Premature end of packed input."; empty writes are refused.
static void fixtures_and_errors(const std::string& dir) {
  const std::vector<std::pair<const char*, const char*>> cases = {{"packed", "binary"},
                                                                   {"segmented-packed", "segmented"}};
  for (auto& c : cases) {
    std::vector<byte> wire = read_file(dir + "/" + c.first);
    Msg m = msg_of(read_file(dir + "/" + c.second));
    int p[2];
    if (pipe(p) != 0) return;
    if (write(p[1], wire.data(), wire.size()) != (ssize_t)wire.size()) return;
    close(p[1]);
    PackedMessageStream r{OwnFd(p[0])};
    auto got = r.tryReadMessage().get();
    CHECK(got && same(*got, m), "fixture %s read through the stream", c.first);
    CHECK(!r.tryReadMessage().get(), "fixture %s: end", c.first);
  }
  {
    std::vector<byte> wire = read_file(dir + "/segmented-packed");
    int p[2];
    if (pipe(p) != 0) return;
    if (write(p[1], wire.data(), wire.size() / 2) != (ssize_t)(wire.size() / 2)) return;
    close(p[1]);
    PackedMessageStream r{OwnFd(p[0])};
    bool threw = false;
    try {
      r.tryReadMessage().get();
    } catch (const Exception& e) {
      threw = e.status() == CPK_ERR_PREMATURE_EOF;
    }
    CHECK(threw, "stream cut inside a message: premature end");
  }
  {
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return;
    PackedMessageStream a{OwnFd(sv[0])};
    bool threw = false;
    try {
      a.writeMessage(ArrayPtr<const ArrayPtr<const word>>()).get();
    } catch (const Exception& e) {
      threw = e.status() == CPK_ERR_EMPTY_MESSAGE;
    }
    CHECK(threw, "writeMessage of no segments: uninitialized message");
    threw = false;
    try {
      a.writeMessages(ArrayPtr<const ArrayPtr<const ArrayPtr<const word>>>()).get();
    } catch (const Exception& e) {
      threw = true;
    }
    CHECK(threw, "writeMessages of no messages refused");
    close(sv[1]);
  }
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "tests/golden";
  try {
    threadContext();  // no device: fail here, before any stream thread waits on a peer
  } catch (const Exception& e) {
    fprintf(stderr, "%s\n", e.what());
    return 2;
  }
  try {
    socket_round_trip(dir);
    batch_write(dir);
    fixtures_and_errors(dir);
  } catch (const Exception& e) {
    fprintf(stderr, "unexpected exception: %s\n", e.what());
    return 2;
  }
  printf("stream: %d passed, %d failed\n", g_pass, g_fail);
  return g_fail ? 1 : 0;
}
