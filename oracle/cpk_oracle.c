/* cpk_oracle.c -- CPU restatement of Cap'n Proto's packed codec.  TEST INFRASTRUCTURE ONLY.
 *
 * Restates, function by function, c++/src/capnp/serialize-packed.c++ (the reference's scalar
 * loops), c++/src/capnp/serialize.c++ (framing) and the kj/io.c++ stream contracts those loops
 * run on.  It is the checker for the HIP path (tests/, smoke(), bench.py cpu_baseline) and is
 * never linked into capnp_amd/.  Pinning: tests/test_oracle.py checks it against the
 * reference's golden files + KATs and against oracle/_ref/libcpk_ref.so (the reference itself,
 * compiled from /root/reference by oracle/Makefile.ref) on fuzzed inputs.
 */
#include "cpk_oracle.h"

#include <string.h>

#include "../include/cpk.h"

static inline unsigned zero_bytes(uint64_t w) {
  unsigned c = 0;
  for (int b = 0; b < 8; b++) c += ((w >> (8 * b)) & 0xff) == 0;
  return c;
}

/* serialize-packed.c++:307-431.  One call == one OutputStream::write(piece).  The output
 * bytes do not depend on the inner stream's buffer sizes (the slow buffer at :317-328 and the
 * direct write at :418-425 only move the same bytes), so we append to a flat array. */
size_t cpko_pack_chunk(const uint64_t* in, size_t nwords, uint8_t* out) {
  uint8_t* o = out;
  size_t i = 0;
  while (i < nwords) {
    uint64_t w = in[i++];
    uint8_t* tag_pos = o++;
    uint8_t tag = 0;
    /* :332-350 -- tag bit n <=> byte n non-zero; non-zero bytes follow in order. */
    for (int b = 0; b < 8; b++) {
      uint8_t v = (uint8_t)(w >> (8 * b));
      if (v != 0) {
        tag |= (uint8_t)(1u << b);
        *o++ = v;
      }
    }
    *tag_pos = tag;
    if (tag == 0) {
      /* :352-374 -- count of further all-zero words, capped at 255 and at the chunk end. */
      size_t lim = nwords - i;
      if (lim > 255) lim = 255;
      size_t n = 0;
      while (n < lim && in[i + n] == 0) n++;
      *o++ = (uint8_t)n;
      i += n;
    } else if (tag == 0xff) {
      /* :376-426 -- count of further words with fewer than two zero bytes (:403), capped at
       * 255 and at the chunk end, then those words raw. */
      size_t lim = nwords - i;
      if (lim > 255) lim = 255;
      size_t n = 0;
      while (n < lim && zero_bytes(in[i + n]) < 2) n++;
      *o++ = (uint8_t)n;
      memcpy(o, in + i, n * 8);
      o += n * 8;
      i += n;
    }
  }
  return (size_t)(o - out);
}

/* writeMessage (serialize.c++:332-357): table = {segCount-1, sizes..., pad}, one piece; then
 * one piece per segment; PackedOutputStream inherits OutputStream::write(pieces) which loops
 * write(piece) (kj/io.c++:109-113), so each piece is packed on its own. */
size_t cpko_pack_segments(const uint64_t* const* segs, const uint32_t* seg_words, uint32_t nseg,
                          uint8_t* out) {
  size_t table_words = nseg / 2 + 1;
  uint64_t table[257];
  uint64_t* t = table;
  if (table_words > 257) return 0; /* > 512 segments: not needed by the tests */
  memset(t, 0, table_words * 8);
  uint32_t* t32 = (uint32_t*)t;
  t32[0] = nseg - 1;
  for (uint32_t s = 0; s < nseg; s++) t32[s + 1] = seg_words[s];
  size_t n = cpko_pack_chunk(t, table_words, out);
  for (uint32_t s = 0; s < nseg; s++) n += cpko_pack_chunk(segs[s], seg_words[s], out + n);
  return n;
}

/* Reads the segment table of a flat message in place.  Returns 1 and fills nseg/table_words
 * when the table is consistent with nwords. */
static int parse_flat_table(const uint64_t* words, size_t nwords, uint32_t* nseg_out,
                            size_t* table_words_out) {
  if (nwords == 0) return 0;
  const uint32_t* t32 = (const uint32_t*)words;
  uint64_t nseg = (uint64_t)t32[0] + 1; /* may be 2^32: serialize.c++:107-137 overflow note */
  uint64_t table_words = nseg / 2 + 1;
  if (table_words > nwords) return 0;
  uint64_t total = table_words;
  for (uint64_t s = 0; s < nseg; s++) total += t32[s + 1];
  if (total != nwords) return 0;
  *nseg_out = (uint32_t)nseg;
  *table_words_out = (size_t)table_words;
  return 1;
}

size_t cpko_pack_flat_message(const uint64_t* words, size_t nwords, uint8_t* out, int32_t* status) {
  uint32_t nseg;
  size_t tw;
  if (!parse_flat_table(words, nwords, &nseg, &tw)) {
    *status = CPK_ERR_BAD_FRAMING;
    return cpko_pack_chunk(words, nwords, out);
  }
  *status = CPK_OK;
  const uint32_t* t32 = (const uint32_t*)words;
  size_t n = cpko_pack_chunk(words, tw, out);
  size_t pos = tw;
  for (uint32_t s = 0; s < nseg; s++) {
    n += cpko_pack_chunk(words + pos, t32[s + 1], out + n);
    pos += t32[s + 1];
  }
  return n;
}

/* PackedInputStream::read(dst, nbytes) over ArrayInputStream -- tryRead
 * serialize-packed.c++:34-183 with minBytes == maxBytes, then InputStream::read's
 * "Premature EOF" check (kj/io.c++:51-59).  Over an array input every buffer-seam path of
 * tryRead sees the same bytes; what remains observable is the first failure:
 *   - input exhausted at or inside a record (incl. a missing run-count byte, :99-101, and a
 *     raw run longer than the input, :151-158) -> PREMATURE_EOF;
 *   - run count * 8 > bytes still wanted (:128-131, :140-143) -> RUN_OVERSHOOT, checked after
 *     the count byte is available and before the raw bytes are. */
static int32_t unpack_exact_bytes(const uint8_t* in, size_t len, size_t* pos_io, uint8_t* out,
                                  size_t nbytes, int write) {
  size_t pos = *pos_io;
  size_t o = 0;
  while (o < nbytes) {
    if (pos >= len) { *pos_io = pos; return CPK_ERR_PREMATURE_EOF; }
    uint8_t tag = in[pos++];
    uint8_t w[8];
    for (int b = 0; b < 8; b++) {
      if (tag & (1u << b)) {
        if (pos >= len) { *pos_io = pos; return CPK_ERR_PREMATURE_EOF; }
        w[b] = in[pos++];
      } else {
        w[b] = 0;
      }
    }
    if (write) memcpy(out + o, w, 8);
    o += 8;
    if (tag == 0 || tag == 0xff) {
      if (pos >= len) { *pos_io = pos; return CPK_ERR_PREMATURE_EOF; }
      size_t run = (size_t)in[pos++] * 8;
      if (run > nbytes - o) { *pos_io = pos; return CPK_ERR_RUN_OVERSHOOT; }
      if (tag == 0) {
        if (write) memset(out + o, 0, run);
      } else {
        if (len - pos < run) { *pos_io = len; return CPK_ERR_PREMATURE_EOF; }
        if (write) memcpy(out + o, in + pos, run);
        pos += run;
      }
      o += run;
    }
  }
  *pos_io = pos;
  return CPK_OK;
}

int32_t cpko_unpack_exact(const uint8_t* in, size_t len, size_t* pos, uint64_t* out, size_t nwords) {
  return unpack_exact_bytes(in, len, pos, (uint8_t*)out, nwords * 8, 1);
}

/* PackedInputStream::skip (serialize-packed.c++:185-299): the same parse with no stores; its
 * failures are the same two checks (:200, :254, :265). */
int32_t cpko_skip_words(const uint8_t* in, size_t len, size_t* pos, size_t nwords) {
  return unpack_exact_bytes(in, len, pos, NULL, nwords * 8, 0);
}

/* InputStreamMessageReader(PackedInputStream) -- serialize.c++:202-270 (+ getSegment :283-302
 * reading everything).  The lazy multi-segment reads all target the same outEnd (end of all
 * segments), so reading every segment is one exact read of totalWords. */
int32_t cpko_read_message(const uint8_t* in, size_t len, uint64_t traversal_limit_words,
                          uint64_t* out, size_t out_cap_words, size_t* consumed,
                          size_t* out_words) {
  size_t pos = 0;
  uint64_t first;
  *out_words = 0;
  int32_t st = unpack_exact_bytes(in, len, &pos, (uint8_t*)&first, 8, 1); /* :207 */
  if (st != CPK_OK) { *consumed = pos; return st; }
  uint32_t seg_count_m1 = (uint32_t)first;
  uint32_t seg0 = (uint32_t)(first >> 32);
  if (seg_count_m1 >= 511) { *consumed = pos; return CPK_ERR_TOO_MANY_SEGMENTS; } /* :217 */
  uint32_t nseg = seg_count_m1 + 1;
  size_t table_words = nseg / 2 + 1;
  uint64_t table[256];
  table[0] = first;
  if (nseg > 1) { /* :224-230 -- (segCount & ~1) * 4 bytes */
    st = unpack_exact_bytes(in, len, &pos, (uint8_t*)(table + 1), (size_t)(nseg & ~1u) * 4, 1);
    if (st != CPK_OK) { *consumed = pos; return st; }
  }
  const uint32_t* t32 = (const uint32_t*)table;
  uint64_t total = seg0;
  for (uint32_t s = 1; s < nseg; s++) total += t32[s + 1];
  if (total > traversal_limit_words) { *consumed = pos; return CPK_ERR_MESSAGE_TOO_LARGE; } /* :235 */
  if (table_words + total > out_cap_words) {
    /* The reference would heap-allocate (serialize.c++:244-249) and go on reading, so a decode
     * failure still wins over our capacity report: parse without storing. */
    st = unpack_exact_bytes(in, len, &pos, NULL, (size_t)total * 8, 0);
    *consumed = pos;
    return st != CPK_OK ? st : CPK_ERR_CAPACITY;
  }
  /* Header accepted: the message's flat size is now fixed (the batch ABI reserves it even when
   * a segment read fails later). */
  *out_words = table_words + total;
  memcpy(out, table, table_words * 8);
  st = unpack_exact_bytes(in, len, &pos, (uint8_t*)(out + table_words), (size_t)total * 8, 1);
  *consumed = pos;
  return st;
}

/* computeUnpackedSizeInWords -- serialize-packed.c++:482-508, including its exact bounds
 * checks (`end - ptr >= count` at :491 admits a record whose last data byte is missing; the
 * loop then simply ends). */
int32_t cpko_unpacked_size(const uint8_t* in, size_t len, uint64_t* words) {
  const uint8_t* ptr = in;
  const uint8_t* end = in + len;
  uint64_t total = 0;
  while (ptr < end) {
    unsigned tag = *ptr;
    size_t count = (size_t)__builtin_popcount(tag);
    total += 1;
    if (!((size_t)(end - ptr) >= count)) return CPK_ERR_INVALID_PACKED;
    ptr += count + 1;
    if (tag == 0) {
      if (!(ptr < end)) return CPK_ERR_INVALID_PACKED;
      total += *ptr++;
    } else if (tag == 0xff) {
      if (!(ptr < end)) return CPK_ERR_INVALID_PACKED;
      size_t w = *ptr++;
      total += w;
      size_t bytes = w * 8;
      if (!((size_t)(end - ptr) >= bytes)) return CPK_ERR_INVALID_PACKED;
      ptr += bytes;
    }
  }
  *words = total;
  return CPK_OK;
}

uint64_t cpko_packed_bound(uint64_t words, uint64_t chunks) {
  return words * 8 + (words + 1) / 2 + 2 * chunks;
}

int32_t cpko_pack_batch(const uint64_t* words, const uint64_t* msg_word_off, uint64_t n,
                        uint8_t* out, uint64_t* msg_out_off, int32_t* status) {
  uint64_t o = 0;
  int32_t first_bad = CPK_OK;
  for (uint64_t m = 0; m < n; m++) {
    msg_out_off[m] = o;
    int32_t st;
    o += cpko_pack_flat_message(words + msg_word_off[m], msg_word_off[m + 1] - msg_word_off[m],
                                out + o, &st);
    if (status) status[m] = st;
    if (st != CPK_OK && first_bad == CPK_OK) first_bad = st;
  }
  msg_out_off[n] = o;
  return first_bad;
}

int32_t cpko_unpack_batch(const uint8_t* packed, const uint64_t* msg_in_off, uint64_t n,
                          uint64_t* words, uint64_t words_cap, uint64_t* msg_word_off,
                          int32_t* status, uint64_t traversal_limit_words) {
  uint64_t o = 0;
  int32_t first_bad = CPK_OK;
  for (uint64_t m = 0; m < n; m++) {
    msg_word_off[m] = o;
    size_t consumed = 0, nw = 0;
    size_t len = msg_in_off[m + 1] - msg_in_off[m];
    int32_t st = cpko_read_message(packed + msg_in_off[m], len, traversal_limit_words, words + o,
                                   (size_t)(words_cap - o), &consumed, &nw);
    if (st == CPK_OK && consumed != len) st = CPK_ERR_TRAILING_BYTES;
    if (status) status[m] = st;
    if (st != CPK_OK && first_bad == CPK_OK) first_bad = st;
    o += nw;
  }
  msg_word_off[n] = o;
  return first_bad;
}

uint64_t cpko_splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

/* Host restatement of the benchmark generator (capnproto_amd/csrc/cpk_gen.hip: gen_word,
 * gen_kernel, gen_sizes_kernel) -- the synthetic workloads of SURVEY.md 8(d).  Test
 * infrastructure: lets tests/ and tools/make_manifest.py rebuild any message of a bench config
 * on the host, so the reference's packed bytes can be pinned for the full-size configs. */
static uint64_t text_word(uint64_t h) {
  uint64_t w = 0;
  for (int b = 0; b < 8; b++) w |= (uint64_t)(0x20 + ((h >> (8 * b)) & 0xff) % 95) << (8 * b);
  return w;
}

static uint64_t gen_word(int profile, uint64_t seed, uint64_t msg, uint64_t idx) {
  const uint64_t mkey = cpko_splitmix64(seed ^ (msg * 0xD1B54A32D192ED03ull));
  if (profile == 3) profile = (int)(mkey % 3);
  const uint64_t h = cpko_splitmix64(mkey + idx * 0x9E3779B97F4A7C15ull);
  if (profile == 2) return text_word(h);
  if (profile == 1) {
    const uint64_t blk = idx / 340, p = idx % 340;
    const uint64_t nz = 4 + cpko_splitmix64(mkey ^ (blk * 0xA24BAED4963EE407ull)) % 73;
    if (p >= nz) return 0;
    if (h >> 63) return (h & 0xfc) | ((h >> 8) & 0xff) << 32 | ((h >> 16) & 0xffff) << 48;
    return h & 0xffffff;
  }
  const uint32_t r = (uint32_t)((h >> 56) % 100);
  if (r < 45) {
    const int k = 1 + (int)((h >> 48) % 3);
    return h & ((1ull << (8 * k)) - 1);
  }
  if (r < 65) return (h & 0xffff) | (((h >> 16) & 0xffff) << 32);
  if (r < 80) return 0;
  if (r < 90) return (h & 0xff) | ((h >> 8) & 0xff) << 32 | ((h >> 16) & 0xff) << 48;
  return text_word(cpko_splitmix64(h));
}

void cpko_gen_offsets(uint64_t seed, uint64_t first_msg, uint64_t stride, uint64_t nmsgs,
                      uint32_t nseg, uint64_t seg_words, uint64_t* off) {
  const uint64_t tw = nseg / 2 + 1;
  uint64_t o = 0;
  if (stride == 0) stride = 1;
  for (uint64_t m = 0; m < nmsgs; m++) {
    off[m] = o;
    if (seg_words) {
      o += tw + (uint64_t)nseg * seg_words;
    } else {
      const uint64_t k =
          3 + cpko_splitmix64(seed ^ ((first_msg + m * stride) * 0x94D049BB133111EBull)) % 9;
      o += tw + (1ull << k);
    }
  }
  off[nmsgs] = o;
}

void cpko_gen_messages(int profile, uint64_t seed, uint64_t first_msg, uint64_t stride,
                       uint64_t nmsgs, uint32_t nseg, const uint64_t* off, uint64_t* words) {
  const uint64_t tw = nseg / 2 + 1;
  if (stride == 0) stride = 1;
  for (uint64_t m = 0; m < nmsgs; m++) {
    uint64_t* w = words + (off[m] - off[0]);
    const uint64_t body = (off[m + 1] - off[m]) - tw;
    const uint64_t seg = body / nseg;
    uint32_t* t32 = (uint32_t*)w;
    for (uint64_t i = 0; i < 2 * tw; i++) {
      uint32_t v = 0;
      if (i == 0) v = nseg - 1;
      else if (i <= nseg) v = (uint32_t)(i < nseg ? seg : body - seg * (nseg - 1));
      t32[i] = v;
    }
    const uint64_t g = first_msg + m * stride;
    for (uint64_t i = 0; i < body; i++) w[tw + i] = gen_word(profile, seed, g, i);
  }
}
