// kj_binding_test.c++ -- reference callers run through the binding (integration/kj_binding.h)
// with the device codec underneath.  Built by oracle/Makefile.ref against the reference's own
// kj / capnp objects WITHOUT the reference's serialize-packed.o, so every packed or unpacked byte
// here comes from libcpk_hip.so; run on the GPU box by tests/test_gpu_binding.py.
//
//   1. the expectPacksTo loop of serialize-packed-test.c++:90-195 over its KATs (:202-221, kept as
//      tests/golden/kats.txt): computeUnpackedSizeInWords, PackedOutputStream::write into a
//      kj::VectorOutputStream, PackedInputStream::read from a kj::ArrayInputStream, reads through
//      fragmented buffers (preferredReadSize 1, 2, 4, ...), skip(), five back-to-back copies;
//   2. writePackedMessage / PackedMessageReader over the reference's fixtures (testdata/binary ->
//      packed, segmented -> segmented-packed), segments compared with capnp::FlatArrayMessageReader;
//   3. the addressbook flow of samples/addressbook.c++:47-79: writePackedMessageToFd into a pipe,
//      PackedFdMessageReader message(fd) (borrowed int fd, then an owned kj::OwnFd after a
//      MallocMessageBuilder write), writePackedMessage over an unbuffered kj::OutputStream,
//      PackedMessageReader over kj::FdInputStream, getRoot<AnyPointer>() walked to the two people
//      the sample writes (ids 123 / 456, names, emails, phone counts);
//   4. the RoundTrip tests of serialize-packed-test.c++:225-585 restated schema-free (AnyPointer):
//      forced segment counts 1/2/3/7/10 (its TestMessageBuilder), lazy one-byte reads and scratch
//      space, two messages from one stream, the all-zero message in at most 7 bytes, and a
//      5023-byte text field (raw runs over 255 words).
//
//   kj_binding_test <tests/golden dir>     -> prints "binding ok: N checks", exit 0
#include <capnp/any.h>
#include <capnp/serialize.h>
#include <kj/io.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <sstream>
#include <string>
#include <vector>

#include "kj_binding.h"

namespace {

int checks = 0;

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

std::vector<kj::byte> unhex(const std::string& s) {
  std::vector<kj::byte> v;
  if (s == "-") return v;
  for (size_t i = 0; i + 1 < s.size(); i += 2) v.push_back((kj::byte)std::stoul(s.substr(i, 2), 0, 16));
  return v;
}

// A BufferedInputStream over bytes that hands them out at most `preferred` at a time (the
// fragmented reads of TestPipe, serialize-packed-test.c++:33-88).
class FragmentedInput final : public kj::BufferedInputStream {
 public:
  FragmentedInput(kj::ArrayPtr<const kj::byte> data, size_t preferred)
      : data_(data), preferred_(preferred) {}
  kj::ArrayPtr<const kj::byte> tryGetReadBuffer() override {
    const size_t n = std::min(preferred_, data_.size() - pos_);
    return data_.slice(pos_, pos_ + n);
  }
  size_t tryRead(kj::ArrayPtr<kj::byte> buffer, size_t minBytes) override {
    size_t n = 0;
    while (n < minBytes && pos_ < data_.size()) {
      const size_t k = std::min({preferred_, data_.size() - pos_, buffer.size() - n});
      memcpy(buffer.begin() + n, data_.begin() + pos_, k);
      pos_ += k;
      n += k;
    }
    return n;
  }
  void skip(size_t bytes) override { pos_ += bytes; }
  size_t remaining() const { return data_.size() - pos_; }

 private:
  kj::ArrayPtr<const kj::byte> data_;
  size_t preferred_;
  size_t pos_ = 0;
};

kj::Array<kj::byte> pack_chunks(const std::vector<kj::byte>& unpacked, int copies) {
  kj::VectorOutputStream out;
  {
    cpk_kj::_::PackedOutputStream packed(out);
    for (int i = 0; i < copies; i++) packed.write(kj::arrayPtr(unpacked.data(), unpacked.size()));
  }
  return kj::heapArray(out.getArray());
}

// serialize-packed-test.c++:90-195 (expectPacksTo) for one KAT
void expect_packs_to(const std::vector<kj::byte>& unpacked, const std::vector<kj::byte>& packed,
                     const std::string& name) {
  const size_t U = unpacked.size();
  check(cpk_kj::computeUnpackedSizeInWords(kj::arrayPtr(packed.data(), packed.size())) == U / 8,
        name + ": computeUnpackedSizeInWords");
  auto got = pack_chunks(unpacked, 1);
  check(got.size() == packed.size() && memcmp(got.begin(), packed.data(), packed.size()) == 0,
        name + ": pack");
  {
    kj::ArrayInputStream in(kj::arrayPtr(packed.data(), packed.size()));
    cpk_kj::_::PackedInputStream pin(in);
    std::vector<kj::byte> back(U);
    pin.read(kj::arrayPtr(back.data(), U));
    check(back == unpacked, name + ": unpack");
    check(in.tryGetReadBuffer().size() == 0, name + ": unpack consumed the input");
  }
  for (size_t pref = 1; pref <= 2 * packed.size() + 1; pref *= 2) {
    FragmentedInput in(kj::arrayPtr(packed.data(), packed.size()), pref);
    cpk_kj::_::PackedInputStream pin(in);
    std::vector<kj::byte> back(U);
    pin.read(kj::arrayPtr(back.data(), U));
    check(back == unpacked, name + ": fragmented unpack " + std::to_string(pref));
    check(in.remaining() == 0, name + ": fragmented unpack consumed " + std::to_string(pref));
  }
  {
    kj::ArrayInputStream in(kj::arrayPtr(packed.data(), packed.size()));
    cpk_kj::_::PackedInputStream pin(in);
    pin.skip(U);
    check(in.tryGetReadBuffer().size() == 0, name + ": skip");
  }
  {
    // five back-to-back writes, read back as five words-long reads
    auto five = pack_chunks(unpacked, 5);
    std::vector<kj::byte> want;
    for (int i = 0; i < 5; i++) want.insert(want.end(), packed.begin(), packed.end());
    check(five.size() == want.size() && memcmp(five.begin(), want.data(), want.size()) == 0,
          name + ": five copies packed");
    kj::ArrayInputStream in(kj::arrayPtr(five.begin(), five.size()));
    cpk_kj::_::PackedInputStream pin(in);
    for (int i = 0; i < 5; i++) {
      std::vector<kj::byte> back(U);
      pin.read(kj::arrayPtr(back.data(), U));
      check(back == unpacked, name + ": five copies, copy " + std::to_string(i));
    }
  }
}

// segments of an unpacked (framed) message, as the reference reads them
struct Flat {
  std::vector<capnp::word> words;
  kj::Own<capnp::FlatArrayMessageReader> reader;
  std::vector<kj::ArrayPtr<const capnp::word>> segs;
  explicit Flat(const std::vector<kj::byte>& bytes) : words(bytes.size() / 8) {
    memcpy(words.data(), bytes.data(), bytes.size());
    reader = kj::heap<capnp::FlatArrayMessageReader>(kj::arrayPtr(words.data(), words.size()));
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

void check_same_segments(capnp::MessageReader& r, const Flat& f, const std::string& name) {
  for (uint i = 0; i < f.segs.size(); i++) {
    auto s = r.getSegment(i);
    check(s.size() == f.segs[i].size() &&
              memcmp(s.begin(), f.segs[i].begin(), s.size() * sizeof(capnp::word)) == 0,
          name + ": segment " + std::to_string(i));
  }
}

void fixture(const std::string& dir, const std::string& src, const std::string& dst) {
  auto unpacked = read_file(dir + "/" + src);
  auto packed = read_file(dir + "/" + dst);
  Flat f(unpacked);
  kj::VectorOutputStream out;
  cpk_kj::writePackedMessage(out, f.pieces());
  auto got = out.getArray();
  check(got.size() == packed.size() && memcmp(got.begin(), packed.data(), packed.size()) == 0,
        src + " -> " + dst + ": writePackedMessage");
  kj::ArrayInputStream in(kj::arrayPtr(packed.data(), packed.size()));
  {
    cpk_kj::PackedMessageReader reader(in);
    check_same_segments(reader, f, dst + ": PackedMessageReader");
  }
  check(in.tryGetReadBuffer().size() == 0, dst + ": reader consumed the message");
}

// samples/addressbook.capnp: AddressBook { people @0 :List(Person) }; Person { id @0 :UInt32,
// name @1 :Text, email @2 :Text, phones @3 :List(PhoneNumber), employment union } -- id in the
// data section, name / email / phones the first three pointers.
void addressbook(const std::string& dir) {
  auto unpacked = read_file(dir + "/addressbook.bin");
  auto packed = read_file(dir + "/addressbook.packed");
  Flat f(unpacked);
  int fds[2];
  check(pipe(fds) == 0, "pipe");
  cpk_kj::writePackedMessageToFd(fds[1], f.pieces());  // samples/addressbook.c++:75
  close(fds[1]);
  std::vector<kj::byte> wire;
  {
    kj::byte buf[4096];
    ssize_t n;
    while ((n = ::read(fds[0], buf, sizeof buf)) > 0) wire.insert(wire.end(), buf, buf + n);
    close(fds[0]);
  }
  check(wire == packed, "addressbook: writePackedMessageToFd bytes == the sample's");
  // samples/addressbook.c++:79 (PackedFdMessageReader message(fd)), over a second pipe
  check(pipe(fds) == 0, "pipe 2");
  check(::write(fds[1], packed.data(), packed.size()) == (ssize_t)packed.size(), "pipe write");
  close(fds[1]);
  {
    cpk_kj::PackedFdMessageReader message(fds[0]);
    check_same_segments(message, f, "addressbook: PackedFdMessageReader");
    auto book = message.getRoot<capnp::AnyPointer>().getAs<capnp::AnyStruct>();
    auto people = book.getPointerSection()[0].getAs<capnp::AnyList>().as<capnp::List<capnp::AnyStruct>>();
    check(people.size() == 2, "addressbook: two people");
    const uint32_t ids[2] = {123, 456};
    const char* names[2] = {"Alice", "Bob"};
    const char* emails[2] = {"alice@example.com", "bob@example.com"};
    const uint phones[2] = {1, 2};
    for (uint i = 0; i < 2; i++) {
      auto p = people[i];
      auto data = p.getDataSection();
      uint32_t id;
      memcpy(&id, data.begin(), 4);
      check(id == ids[i], "addressbook: person id");
      auto ptrs = p.getPointerSection();
      // pointer section: name, email, phones, then the employment union's school (Alice)
      check(std::string(ptrs[0].getAs<capnp::Text>().cStr()) == names[i], "addressbook: name");
      check(std::string(ptrs[1].getAs<capnp::Text>().cStr()) == emails[i], "addressbook: email");
      check(ptrs[2].getAs<capnp::AnyList>().size() == phones[i], "addressbook: phones");
    }
  }
  close(fds[0]);
  // the sample's shape with a MessageBuilder (samples/addressbook.c++:47-79): the message built
  // in a capnp::MallocMessageBuilder (a copy of the fixture's root), writePackedMessageToFd(fd,
  // builder), then PackedFdMessageReader over an owned descriptor (kj::OwnFd)
  capnp::MallocMessageBuilder builder;
  builder.setRoot(f.reader->getRoot<capnp::AnyPointer>());
  auto bsegs = builder.getSegmentsForOutput();
  check(pipe(fds) == 0, "pipe 3");
  cpk_kj::writePackedMessageToFd(fds[1], builder);
  close(fds[1]);
  {
    cpk_kj::PackedFdMessageReader message{kj::OwnFd(fds[0])};
    for (uint i = 0; i < bsegs.size(); i++) {
      auto s = message.getSegment(i);
      check(s.size() == bsegs[i].size() &&
                memcmp(s.begin(), bsegs[i].begin(), s.size() * sizeof(capnp::word)) == 0,
            "addressbook: builder -> fd -> PackedFdMessageReader(OwnFd) segment");
    }
    auto people = message.getRoot<capnp::AnyPointer>().getAs<capnp::AnyStruct>()
                      .getPointerSection()[0].getAs<capnp::AnyList>();
    check(people.size() == 2, "addressbook: builder round trip, two people");
  }
  // writePackedMessage over an unbuffered kj::OutputStream (serialize-packed.h:94-98): same bytes
  // as the buffered path
  {
    kj::VectorOutputStream vec;
    class Unbuffered final : public kj::OutputStream {
     public:
      explicit Unbuffered(kj::VectorOutputStream& v) : v_(v) {}
      void write(kj::ArrayPtr<const kj::byte> data) override { v_.write(data); }
     private:
      kj::VectorOutputStream& v_;
    } plain(vec);
    cpk_kj::writePackedMessage(static_cast<kj::OutputStream&>(plain), f.pieces());
    auto got = vec.getArray();
    check(got.size() == packed.size() && memcmp(got.begin(), packed.data(), packed.size()) == 0,
          "addressbook: writePackedMessage(kj::OutputStream&) bytes == the sample's");
    kj::VectorOutputStream vec2;
    cpk_kj::writePackedMessage(static_cast<kj::OutputStream&>(vec2), builder);
    kj::ArrayInputStream in(vec2.getArray());
    cpk_kj::PackedMessageReader r(in);
    check(r.getSegment(0).size() == bsegs[0].size(),
          "addressbook: writePackedMessage(kj::OutputStream& buffered, builder)");
  }
}

// ---- serialize-packed-test.c++:225-585, schema-free --------------------------------------------
// The reference's round trips build TestAllTypes (test.capnp) messages; here the same shapes are
// built through capnp::AnyPointer / AnyStruct: a root struct with data, text, blobs, nested
// structs and lists (many separately allocated objects), an all-zero struct, and a 5023-byte
// text field (raw runs past the 255-word cap).

// serialize-packed-test.c++:225-254 TestMessageBuilder: minimum-size segments until the desired
// count, then one large segment (so a message of enough objects has exactly that many segments).
class SegmentCountBuilder final : public capnp::MallocMessageBuilder {
 public:
  explicit SegmentCountBuilder(uint n)
      : capnp::MallocMessageBuilder(0, capnp::AllocationStrategy::FIXED_SIZE), left_(n) {}
  kj::ArrayPtr<capnp::word> allocateSegment(uint minimumSize) override {
    if (left_ <= 1) {
      if (left_ == 1) --left_;
      else over_ = true;
      return capnp::MallocMessageBuilder::allocateSegment(capnp::SUGGESTED_FIRST_SEGMENT_WORDS);
    }
    --left_;
    return capnp::MallocMessageBuilder::allocateSegment(minimumSize);
  }
  bool exact() const { return left_ == 0 && !over_; }

 private:
  uint left_;
  bool over_ = false;
};

// the stand-in for initTestMessage (test-util.c++): more than ten separately allocated objects
void fill_message(capnp::MessageBuilder& b) {
  auto root = b.getRoot<capnp::AnyPointer>().initAsAnyStruct(6, 8);
  auto data = root.getDataSection();
  for (size_t i = 0; i < data.size(); i++) data[i] = (kj::byte)((i % 3) ? i * 37 + 1 : 0);
  auto ptrs = root.getPointerSection();
  ptrs[0].setAs<capnp::Text>("foo");
  ptrs[1].setAs<capnp::Text>("a text field long enough to make a raw run of several words");
  const kj::byte blob[] = {0, 1, 2, 0, 0, 0, 0, 0, 7, 8, 9, 10, 11, 12, 13, 0, 0, 0, 0, 0, 0, 0, 0,
                           0, 255, 254, 0, 0, 0, 0, 0, 1};
  ptrs[2].setAs<capnp::Data>(kj::arrayPtr(blob, sizeof blob));
  auto s1 = ptrs[3].initAsAnyStruct(2, 2);
  s1.getDataSection()[0] = 5;
  s1.getPointerSection()[0].setAs<capnp::Text>("nested");
  auto s2 = s1.getPointerSection()[1].initAsAnyStruct(1, 1);
  s2.getDataSection()[3] = 0x80;
  s2.getPointerSection()[0].setAs<capnp::Text>("deeper");
  auto ls = ptrs[4].initAsListOfAnyStruct(2, 1, 5);
  for (uint i = 0; i < 5; i++) {
    ls[i].getDataSection()[i] = (kj::byte)(i + 1);
    ls[i].getPointerSection()[0].setAs<capnp::Text>(i % 2 ? "odd" : "even element");
  }
  auto l8 = ptrs[5].initAs<capnp::List<uint64_t>>(20);
  for (uint i = 0; i < 20; i++) l8.set(i, i % 4 == 0 ? 0 : 0x0101010101010101ull * i + i);
  ptrs[6].setAs<capnp::Text>("bar");
  ptrs[7].setAs<capnp::Text>("baz");
}

// the segments of a builder read back through a PackedMessageReader from `in`
void check_builder_segments(capnp::MessageReader& r, capnp::MessageBuilder& b,
                            const std::string& name) {
  auto segs = b.getSegmentsForOutput();
  for (uint i = 0; i < segs.size(); i++) {
    auto s = r.getSegment(i);
    check(s.size() == segs[i].size() &&
              memcmp(s.begin(), segs[i].begin(), s.size() * sizeof(capnp::word)) == 0,
          name + ": segment " + std::to_string(i));
  }
  check(r.getSegment(segs.size()) == nullptr, name + ": segment count");
}

// one RoundTrip* test: writePackedMessage, computeUnpackedSizeInWords against
// computeSerializedSizeInWords, then a PackedMessageReader over a whole buffer, over a buffer
// handed out one byte at a time (the Lazy tests: TestPipe(1)) and with a scratch space (the
// ScratchSpace tests)
std::vector<kj::byte> round_trip(capnp::MessageBuilder& b, const std::string& name) {
  kj::VectorOutputStream out;
  cpk_kj::writePackedMessage(out, b);
  auto bytes = out.getArray();
  std::vector<kj::byte> packed(bytes.begin(), bytes.end());
  check(capnp::computeSerializedSizeInWords(b) ==
            cpk_kj::computeUnpackedSizeInWords(kj::arrayPtr(packed.data(), packed.size())),
        name + ": computeUnpackedSizeInWords == computeSerializedSizeInWords");
  {
    kj::ArrayInputStream in(kj::arrayPtr(packed.data(), packed.size()));
    cpk_kj::PackedMessageReader r(in);
    check_builder_segments(r, b, name);
  }
  {
    FragmentedInput in(kj::arrayPtr(packed.data(), packed.size()), 1);
    cpk_kj::PackedMessageReader r(in);
    check_builder_segments(r, b, name + " lazy");
    check(in.remaining() == 0, name + " lazy: consumed");
  }
  {
    kj::ArrayInputStream in(kj::arrayPtr(packed.data(), packed.size()));
    capnp::word scratch[1024];
    cpk_kj::PackedMessageReader r(in, capnp::ReaderOptions(), kj::arrayPtr(scratch, 1024));
    check_builder_segments(r, b, name + " scratch");
  }
  return packed;
}

void reference_round_trips() {
  // RoundTrip, RoundTripOddSegmentCount (7), RoundTripEvenSegmentCount (10), and 2 and 3
  for (uint n : {1u, 2u, 3u, 7u, 10u}) {
    SegmentCountBuilder b(n);
    fill_message(b);
    check(b.exact() && b.getSegmentsForOutput().size() == n,
          "segment count " + std::to_string(n) + " forced");
    round_trip(b, "RoundTrip " + std::to_string(n) + " segments");
  }
  // RoundTripTwoMessages: two messages back to back on one stream, two readers in turn
  {
    SegmentCountBuilder b1(1), b2(1);
    fill_message(b1);
    auto r2 = b2.getRoot<capnp::AnyPointer>().initAsAnyStruct(0, 1);
    r2.getPointerSection()[0].setAs<capnp::Text>("Second message.");
    kj::VectorOutputStream out;
    cpk_kj::writePackedMessage(out, b1);
    cpk_kj::writePackedMessage(out, b2);
    auto bytes = out.getArray();
    check(capnp::computeSerializedSizeInWords(b1) + capnp::computeSerializedSizeInWords(b2) ==
              cpk_kj::computeUnpackedSizeInWords(bytes),
          "RoundTripTwoMessages: computeUnpackedSizeInWords");
    kj::ArrayInputStream in(bytes);
    {
      cpk_kj::PackedMessageReader r(in);
      check_builder_segments(r, b1, "RoundTripTwoMessages: first");
    }
    {
      cpk_kj::PackedMessageReader r(in);
      auto t = r.getRoot<capnp::AnyPointer>().getAs<capnp::AnyStruct>().getPointerSection()[0];
      check(std::string(t.getAs<capnp::Text>().cStr()) == "Second message.",
            "RoundTripTwoMessages: second");
    }
    check(in.tryGetReadBuffer().size() == 0, "RoundTripTwoMessages: consumed");
  }
  // RoundTripAllZero (1 segment): "Segment table packs to 2 bytes. Root pointer packs to 3 bytes.
  // Content packs to 2 bytes (zero span)" -- at most 7 bytes; then the 3- and 2-segment shapes
  // with two nested all-zero structs (initStructField().initStructField())
  {
    SegmentCountBuilder b(1);
    b.getRoot<capnp::AnyPointer>().initAsAnyStruct(6, 20);
    auto packed = round_trip(b, "RoundTripAllZero");
    check(packed.size() <= 7, "RoundTripAllZero: at most 7 bytes (" +
                                  std::to_string(packed.size()) + ")");
  }
  for (uint n : {3u, 2u}) {
    SegmentCountBuilder b(n);
    auto root = b.getRoot<capnp::AnyPointer>().initAsAnyStruct(6, 20);
    root.getPointerSection()[0].initAsAnyStruct(6, 20).getPointerSection()[0].initAsAnyStruct(6, 20);
    check(b.exact() && b.getSegmentsForOutput().size() == n,
          "all-zero segment count " + std::to_string(n) + " forced");
    round_trip(b, "RoundTripAllZero " + std::to_string(n) + " segments");
  }
  // RoundTripHugeString: a 5023-byte text field of 'x' (raw runs over 255 words), 1, 3 and 2
  // segments
  for (uint n : {1u, 3u, 2u}) {
    std::string huge(5023, 'x');
    SegmentCountBuilder b(n);
    auto root = b.getRoot<capnp::AnyPointer>().initAsAnyStruct(6, 20);
    root.getPointerSection()[0].setAs<capnp::Text>(huge.c_str());
    // (the 2- and 3-segment shapes: objects after the text spill into further segments)
    if (n > 1) root.getPointerSection()[1].initAsAnyStruct(1, 1).getPointerSection()[0]
                   .setAs<capnp::Text>("after");
    check(!(n > 1) || b.exact(), "huge string segment count " + std::to_string(n));
    round_trip(b, "RoundTripHugeString " + std::to_string(n) + " segments");
    kj::VectorOutputStream out;
    cpk_kj::writePackedMessage(out, b);
    kj::ArrayInputStream in(out.getArray());
    cpk_kj::PackedMessageReader r(in);
    auto t = r.getRoot<capnp::AnyPointer>().getAs<capnp::AnyStruct>().getPointerSection()[0];
    check(std::string(t.getAs<capnp::Text>().cStr()) == huge, "RoundTripHugeString text");
  }
}

// serialize-test.c++:533-543: a segment count of UINT_MAX + 1 is "Message has too many segments."
// (security-advisories/2026-03-12-0-segment-count-overflow.md).  Its first word
// ff ff ff ff 00 00 00 00 packs to the record 0f ff ff ff ff.
void uint_max_segment_count() {
  const kj::byte bytes[] = {0x0f, 0xff, 0xff, 0xff, 0xff};
  kj::ArrayInputStream in(kj::arrayPtr(bytes, sizeof(bytes)));
  bool threw = false;
  try {
    cpk_kj::PackedMessageReader r(in);
  } catch (const cpk_capnp::Exception& e) {
    threw = std::string(e.what()).find("Message has too many segments.") != std::string::npos;
  }
  check(threw, "UINT_MAX segment count: PackedMessageReader throws \"Message has too many segments.\"");
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <tests/golden dir>\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  std::ifstream kats(dir + "/kats.txt");
  check(bool(kats), "kats.txt");
  std::string line;
  int k = 0;
  while (std::getline(kats, line)) {
    std::istringstream ls(line);
    std::string u, p;
    if (!(ls >> u >> p)) continue;
    expect_packs_to(unhex(u), unhex(p), "kat " + std::to_string(k++));
  }
  check(k >= 11, "all KATs read");
  fixture(dir, "binary", "packed");
  fixture(dir, "segmented", "segmented-packed");
  addressbook(dir);
  reference_round_trips();
  uint_max_segment_count();
  std::printf("binding ok: %d checks (%d KATs, 2 fixtures, addressbook, the RoundTrip tests of "
              "serialize-packed-test.c++:225-585, the UINT_MAX segment count)\n", checks, k);
  return 0;
}
