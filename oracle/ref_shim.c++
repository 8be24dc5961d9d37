// ref_shim.c++ -- C-ABI shim over the REAL reference packed codec.  TEST INFRASTRUCTURE ONLY.
//
// Our own file; it is compiled together with the reference's unmodified sources (read in place
// under /root/reference) by oracle/Makefile.ref into oracle/_ref/libcpk_ref.so.  It exposes the
// reference's writePackedMessage / PackedOutputStream / PackedMessageReader / PackedInputStream::skip
// / computeUnpackedSizeInWords to ctypes so that tests/ can pin oracle/cpk_oracle.c (and through
// it the HIP path) against the reference itself, and bench.py can time the reference CPU codec as
// the cpu_baseline ("kind": "reference").  Nothing in capnp_amd/ loads this library.
#include <capnp/serialize-packed.h>
#include <capnp/serialize.h>
#include <kj/debug.h>
#include <kj/io.h>

#include <stdint.h>
#include <string.h>

namespace {

// Status codes == include/cpk.h cpk_status.
enum {
  OK = 0, PREMATURE_EOF = 1, RUN_OVERSHOOT = 2, TOO_MANY_SEGMENTS = 3, MESSAGE_TOO_LARGE = 4,
  INVALID_PACKED = 5, CAPACITY = 8, OTHER = 99
};

char g_last_error[512];

int map_exception(const kj::Exception& e) {
  auto desc = e.getDescription();
  size_t n = desc.size() < sizeof(g_last_error) - 1 ? desc.size() : sizeof(g_last_error) - 1;
  memcpy(g_last_error, desc.begin(), n);
  g_last_error[n] = 0;
  const char* d = g_last_error;
  if (strstr(d, "Premature EOF") || strstr(d, "Premature end of packed input")) return PREMATURE_EOF;
  if (strstr(d, "did not end cleanly on a segment boundary")) return RUN_OVERSHOOT;
  if (strstr(d, "too many segments")) return TOO_MANY_SEGMENTS;
  if (strstr(d, "too large")) return MESSAGE_TOO_LARGE;
  if (strstr(d, "invalid packed data")) return INVALID_PACKED;
  if (strstr(d, "not large enough")) return CAPACITY;
  return OTHER;
}

}  // namespace

extern "C" {

const char* ref_last_error() { return g_last_error; }

// PackedOutputStream::write(one piece) into an ArrayOutputStream.
int ref_pack_chunk(const uint64_t* words, uint64_t nwords, uint8_t* out, uint64_t cap,
                   uint64_t* out_len) {
  g_last_error[0] = 0;
  try {
    kj::ArrayOutputStream aos(kj::arrayPtr(reinterpret_cast<kj::byte*>(out), cap));
    capnp::_::PackedOutputStream packed(aos);
    packed.write(kj::arrayPtr(reinterpret_cast<const kj::byte*>(words), nwords * 8));
    *out_len = aos.getArray().size();
    return OK;
  } catch (const kj::Exception& e) {
    return map_exception(e);
  }
}

// writePackedMessage(BufferedOutputStream&, segments) -- the benchmark's ArrayOutputStream shape.
int ref_pack_segments(const uint64_t* const* segs, const uint32_t* seg_words, uint32_t nseg,
                      uint8_t* out, uint64_t cap, uint64_t* out_len) {
  g_last_error[0] = 0;
  try {
    kj::Vector<kj::ArrayPtr<const capnp::word>> v(nseg);
    for (uint32_t s = 0; s < nseg; s++)
      v.add(kj::arrayPtr(reinterpret_cast<const capnp::word*>(segs[s]), seg_words[s]));
    kj::ArrayOutputStream aos(kj::arrayPtr(reinterpret_cast<kj::byte*>(out), cap));
    capnp::writePackedMessage(aos, v.asPtr());
    *out_len = aos.getArray().size();
    return OK;
  } catch (const kj::Exception& e) {
    return map_exception(e);
  }
}

// writePackedMessage(OutputStream&, segments) through a non-buffered stream: exercises the
// 8 KiB stack buffer + BufferedOutputStreamWrapper path (serialize-packed.c++:466-475).
namespace {
struct SinkStream final : public kj::OutputStream {
  uint8_t* out; uint64_t cap; uint64_t len = 0; bool overflow = false;
  void write(kj::ArrayPtr<const kj::byte> data) override {
    if (len + data.size() > cap) { overflow = true; return; }
    memcpy(out + len, data.begin(), data.size());
    len += data.size();
  }
};
}  // namespace

int ref_pack_segments_unbuffered(const uint64_t* const* segs, const uint32_t* seg_words,
                                 uint32_t nseg, uint8_t* out, uint64_t cap, uint64_t* out_len) {
  g_last_error[0] = 0;
  try {
    kj::Vector<kj::ArrayPtr<const capnp::word>> v(nseg);
    for (uint32_t s = 0; s < nseg; s++)
      v.add(kj::arrayPtr(reinterpret_cast<const capnp::word*>(segs[s]), seg_words[s]));
    SinkStream sink;
    sink.out = out; sink.cap = cap;
    capnp::writePackedMessage(static_cast<kj::OutputStream&>(sink), v.asPtr());
    if (sink.overflow) return CAPACITY;
    *out_len = sink.len;
    return OK;
  } catch (const kj::Exception& e) {
    return map_exception(e);
  }
}

// PackedMessageReader(ArrayInputStream) reading every segment.  Writes the flat message
// (table rebuilt from the reader's segment sizes, then segments); reports consumed bytes.
int ref_read_message(const uint8_t* in, uint64_t len, uint64_t traversal_limit_words,
                     uint64_t* out, uint64_t out_cap_words, uint64_t* consumed,
                     uint64_t* out_words, uint32_t* nseg_out) {
  g_last_error[0] = 0;
  kj::ArrayInputStream ais(kj::arrayPtr(reinterpret_cast<const kj::byte*>(in), len));
  *out_words = 0;
  *nseg_out = 0;
  try {
    capnp::ReaderOptions opts;
    opts.traversalLimitInWords = traversal_limit_words;
    if (out_cap_words < 257) return CAPACITY;
    {
      // Scratch space = the caller's array past a 257-word table area, so every segment
      // (even an empty one) has a non-null begin(); getSegment(id) returns a null ArrayPtr
      // only for id past the declared count (serialize.c++:283-286).
      capnp::PackedMessageReader reader(
          ais, opts, kj::arrayPtr(reinterpret_cast<capnp::word*>(out + 257), out_cap_words - 257));
      uint32_t nseg = 0;
      uint64_t total = 0;
      uint64_t sizes[512];
      const capnp::word* begins[512];
      for (; nseg < 512; nseg++) {
        auto seg = reader.getSegment(nseg);
        if (seg.begin() == nullptr) break;
        sizes[nseg] = seg.size();
        begins[nseg] = seg.begin();
        total += seg.size();
      }
      uint64_t table_words = nseg / 2 + 1;
      if (table_words + total > out_cap_words) return CAPACITY;
      // Segments are contiguous in scratch starting at out+257; slide them down behind the table.
      if (nseg > 0) memmove(out + table_words, begins[0], total * 8);
      memset(out, 0, table_words * 8);
      uint32_t* t32 = reinterpret_cast<uint32_t*>(out);
      t32[0] = nseg - 1;
      for (uint32_t s = 0; s < nseg; s++) t32[s + 1] = (uint32_t)sizes[s];
      *out_words = table_words + total;
      *nseg_out = nseg;
    }
    *consumed = len - ais.tryGetReadBuffer().size();
    return OK;
  } catch (const kj::Exception& e) {
    *consumed = len - ais.tryGetReadBuffer().size();
    return map_exception(e);
  }
}

// PackedInputStream::read of exactly nwords words (flat-packed path, capnp.c++:1066-1071).
int ref_unpack_exact(const uint8_t* in, uint64_t len, uint64_t* out, uint64_t nwords,
                     uint64_t* consumed) {
  g_last_error[0] = 0;
  kj::ArrayInputStream ais(kj::arrayPtr(reinterpret_cast<const kj::byte*>(in), len));
  try {
    capnp::_::PackedInputStream pis(ais);
    pis.read(kj::arrayPtr(reinterpret_cast<kj::byte*>(out), nwords * 8));
    *consumed = len - ais.tryGetReadBuffer().size();
    return OK;
  } catch (const kj::Exception& e) {
    *consumed = len - ais.tryGetReadBuffer().size();
    return map_exception(e);
  }
}

// PackedInputStream::skip over nwords words.
int ref_skip_words(const uint8_t* in, uint64_t len, uint64_t nwords, uint64_t* consumed) {
  g_last_error[0] = 0;
  kj::ArrayInputStream ais(kj::arrayPtr(reinterpret_cast<const kj::byte*>(in), len));
  try {
    capnp::_::PackedInputStream pis(ais);
    pis.skip(nwords * 8);
    *consumed = len - ais.tryGetReadBuffer().size();
    return OK;
  } catch (const kj::Exception& e) {
    *consumed = len - ais.tryGetReadBuffer().size();
    return map_exception(e);
  }
}

int ref_unpacked_size(const uint8_t* in, uint64_t len, uint64_t* words) {
  g_last_error[0] = 0;
  try {
    *words = capnp::computeUnpackedSizeInWords(
        kj::arrayPtr(reinterpret_cast<const kj::byte*>(in), len));
    return OK;
  } catch (const kj::Exception& e) {
    return map_exception(e);
  }
}

// Batch timing entry points (cpu_baseline): pack n flat single/multi-segment messages laid out
// back to back (table + segments), with writePackedMessage(ArrayOutputStream&, segments); unpack
// with ArrayInputStream + PackedMessageReader, touching every segment.  The benchmark/ harness
// shape (capnproto-common.h:82-101).  Returns 0 or the first failing status.
int ref_pack_batch(const uint64_t* words, const uint64_t* msg_word_off, uint64_t n, uint8_t* out,
                   uint64_t cap, uint64_t* msg_out_off) {
  uint64_t o = 0;
  try {
    for (uint64_t m = 0; m < n; m++) {
      const uint64_t* w = words + msg_word_off[m];
      const uint32_t* t32 = reinterpret_cast<const uint32_t*>(w);
      uint32_t nseg = t32[0] + 1;
      uint64_t pos = nseg / 2 + 1;
      kj::ArrayPtr<const capnp::word> segs[512];
      if (nseg > 512) return OTHER;
      for (uint32_t s = 0; s < nseg; s++) {
        segs[s] = kj::arrayPtr(reinterpret_cast<const capnp::word*>(w + pos), t32[s + 1]);
        pos += t32[s + 1];
      }
      msg_out_off[m] = o;
      kj::ArrayOutputStream aos(kj::arrayPtr(reinterpret_cast<kj::byte*>(out + o), cap - o));
      capnp::writePackedMessage(aos, kj::arrayPtr(segs, nseg));
      o += aos.getArray().size();
    }
    msg_out_off[n] = o;
    return OK;
  } catch (const kj::Exception& e) {
    return map_exception(e);
  }
}

int ref_unpack_batch(const uint8_t* packed, const uint64_t* msg_in_off, uint64_t n,
                     uint64_t* words, uint64_t words_cap, uint64_t* msg_word_off) {
  uint64_t o = 0;
  try {
    for (uint64_t m = 0; m < n; m++) {
      kj::ArrayInputStream ais(kj::arrayPtr(reinterpret_cast<const kj::byte*>(packed + msg_in_off[m]),
                                            msg_in_off[m + 1] - msg_in_off[m]));
      // Read straight into the caller's array as scratch space (no heap allocation), the way a
      // server reusing a buffer would.
      capnp::PackedMessageReader reader(
          ais, capnp::ReaderOptions(),
          kj::arrayPtr(reinterpret_cast<capnp::word*>(words + o), words_cap - o));
      msg_word_off[m] = o;
      uint64_t total = 0;
      for (uint32_t s = 0;; s++) {
        auto seg = reader.getSegment(s);
        if (seg.begin() == nullptr) break;
        total += seg.size();
      }
      o += total;
    }
    msg_word_off[n] = o;
    return OK;
  } catch (const kj::Exception& e) {
    return map_exception(e);
  }
}

}  // extern "C"
