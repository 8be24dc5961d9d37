/* cpk_oracle.h -- CPU restatement of the reference packed codec.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this; the
 * product (capnp_amd/, libcpk_hip.so) never does.  Parity is pinned two ways (see
 * tests/test_oracle.py): against the reference's own golden files
 * (c++/testdata/{binary,packed,segmented,segmented-packed,flat,packedflat}) and KATs
 * (serialize-packed-test.c++:202-221), and against the real reference compiled from its
 * sources by oracle/Makefile.ref (oracle/_ref/libcpk_ref.so) on fuzzed inputs.
 *
 * Status codes are include/cpk.h's cpk_status values.
 */
#ifndef CPK_ORACLE_H_
#define CPK_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* PackedOutputStream::write(one piece) -- serialize-packed.c++:307-431.
 * nwords words at `in`; appends to out, returns bytes written. */
size_t cpko_pack_chunk(const uint64_t* in, size_t nwords, uint8_t* out);

/* writePackedMessage(segments) -- serialize-packed.c++:460-464 -> writeMessage
 * serialize.c++:332-357 (table piece, then one piece per segment). */
size_t cpko_pack_segments(const uint64_t* const* segs, const uint32_t* seg_words, uint32_t nseg,
                          uint8_t* out);

/* Same as cpko_pack_segments for a flat message (table followed by segments, the layout of
 * messageToFlatArray serialize.c++:161-190).  Returns bytes written; *status = CPK_OK or
 * CPK_ERR_BAD_FRAMING (then the message is packed as one chunk). */
size_t cpko_pack_flat_message(const uint64_t* words, size_t nwords, uint8_t* out, int32_t* status);

/* InputStreamMessageReader over PackedInputStream over ArrayInputStream(in[0..len)) --
 * serialize-packed.c++:437-440, serialize.c++:202-302, tryRead :34-183.  Reads the table and
 * every segment; writes the flat message (table + segments) to out (capacity out_cap_words).
 * Returns status; *consumed = packed bytes consumed, *out_words = words written. */
int32_t cpko_read_message(const uint8_t* in, size_t len, uint64_t traversal_limit_words,
                          uint64_t* out, size_t out_cap_words, size_t* consumed,
                          size_t* out_words);

/* Unpack exactly nwords words from in[*pos..len) with PackedInputStream::read semantics
 * (runs may not overshoot nwords).  Advances *pos. */
int32_t cpko_unpack_exact(const uint8_t* in, size_t len, size_t* pos, uint64_t* out, size_t nwords);

/* PackedInputStream::skip -- serialize-packed.c++:185-299. */
int32_t cpko_skip_words(const uint8_t* in, size_t len, size_t* pos, size_t nwords);

/* computeUnpackedSizeInWords -- serialize-packed.c++:482-508. */
int32_t cpko_unpacked_size(const uint8_t* in, size_t len, uint64_t* words);

/* Bound on packed bytes (see include/cpk.h cpk_packed_bound). */
uint64_t cpko_packed_bound(uint64_t words, uint64_t chunks);

/* Batch helpers used by the CPU baseline / tests: pack or unpack n flat messages laid out
 * back to back.  Return CPK_OK or the first failing status. */
int32_t cpko_pack_batch(const uint64_t* words, const uint64_t* msg_word_off, uint64_t n,
                        uint8_t* out, uint64_t* msg_out_off, int32_t* status);
int32_t cpko_unpack_batch(const uint8_t* packed, const uint64_t* msg_in_off, uint64_t n,
                          uint64_t* words, uint64_t words_cap, uint64_t* msg_word_off,
                          int32_t* status, uint64_t traversal_limit_words);

/* Deterministic synthetic generator shared with the HIP generator (capnp_amd/csrc/gen.hip):
 * SplitMix64 per (seed, message, word).  See SURVEY.md 8(d). */
uint64_t cpko_splitmix64(uint64_t x);

/* Host restatement of the benchmark generator (capnproto_amd/csrc/cpk_gen.hip), same arguments
 * as cpk_gen_offsets / cpk_gen_messages (include/cpk.h).  off has nmsgs + 1 entries; words
 * receives messages first_msg, first_msg + stride, ... with off[0] mapped to words[0]. */
void cpko_gen_offsets(uint64_t seed, uint64_t first_msg, uint64_t stride, uint64_t nmsgs,
                      uint32_t nseg, uint64_t seg_words, uint64_t* off);
void cpko_gen_messages(int profile, uint64_t seed, uint64_t first_msg, uint64_t stride,
                       uint64_t nmsgs, uint32_t nseg, const uint64_t* off, uint64_t* words);

#ifdef __cplusplus
}
#endif
#endif
