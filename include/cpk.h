/* cpk.h -- C ABI of the MI355X-native Cap'n Proto *packed* wire codec (libcpk_hip.so).
 *
 * This is the drop-in boundary under the reference's packed stream / message API
 * (capnproto c++/src/capnp/serialize-packed.h:32-124).  Each entry point below names the
 * reference function it replaces.  All arguments are plain pointers and sizes: `d_*` pointers
 * are device (HBM) allocations, `h_*` pointers host memory, `stream` is a hipStream_t passed as
 * void* (NULL = the default stream).  No C++ exception crosses this boundary.
 *
 * Ownership mirrors serialize-packed.h:46,60 (streams borrow, never own): the caller owns every
 * buffer; a cpk_ctx owns only its device scratch.  Threading: a cpk_ctx is single-threaded; any
 * number of contexts may be used in parallel (one per device / host thread).
 *
 * Asynchrony: the device entry points only enqueue work on `stream` and return CPK_OK when the
 * launch succeeded.  Per-message results land in caller-owned d_status arrays; batch-level
 * failures found on the device (output capacity exceeded, internal protocol timeout) are kept in
 * the context's error word and returned by cpk_sync().
 *
 * Wire format (doc/encoding.md:296-349): each 8-byte word becomes a tag byte (bit i <=> byte i
 * non-zero) followed by its non-zero bytes.  Tag 0x00 is followed by a count N <= 255 of further
 * all-zero words; tag 0xff by a count N <= 255 of further words copied raw.  Runs never cross a
 * chunk: a chunk is one OutputStream::write() piece -- the segment table, then each segment
 * (serialize.c++:332-357 -> kj/io.c++:109-113).
 */
#ifndef CPK_H_
#define CPK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CPK_ABI_VERSION 2

typedef enum cpk_status {
  CPK_OK = 0,
  /* Input ended before the message did: kj/io.c++:53 "Premature EOF" (InputStream::read) and
   * serialize-packed.c++:57 "Premature end of packed input." */
  CPK_ERR_PREMATURE_EOF = 1,
  /* serialize-packed.c++:128-131, :140-143 "Packed input did not end cleanly on a segment
   * boundary." -- a zero or raw run overshoots the words being read. */
  CPK_ERR_RUN_OVERSHOOT = 2,
  /* serialize.c++:217 "Message has too many segments." (segment count > 512) */
  CPK_ERR_TOO_MANY_SEGMENTS = 3,
  /* serialize.c++:235-242 "Message is too large." (> ReaderOptions::traversalLimitInWords) */
  CPK_ERR_MESSAGE_TOO_LARGE = 4,
  /* serialize-packed.c++:491-502 "invalid packed data" (computeUnpackedSizeInWords) */
  CPK_ERR_INVALID_PACKED = 5,
  /* pack input: a flat message's segment table disagrees with its word count (the message is
   * then packed as a single chunk so offsets stay defined) */
  CPK_ERR_BAD_FRAMING = 6,
  /* unpack batch: the message ended before its [in_off[i], in_off[i+1]) byte range did */
  CPK_ERR_TRAILING_BYTES = 7,
  /* kj/io.c++:281-282 "backing array was not large enough" -- output capacity too small */
  CPK_ERR_CAPACITY = 8,
  CPK_ERR_INVALID_ARGUMENT = 9,
  CPK_ERR_HIP = 10,
  /* serialize.c++:333 "Tried to serialize uninitialized message." (zero segments / words) */
  CPK_ERR_EMPTY_MESSAGE = 11,
  /* internal: a device-side wait gave up (bounded spin); never expected */
  CPK_ERR_INTERNAL = 12,
  CPK_ERR_NO_DEVICE = 13
} cpk_status;

/* Reference message text for a status ("" for CPK_OK). */
const char* cpk_status_string(int32_t status);
int cpk_abi_version(void);

/* ReaderOptions (capnp/message.h:51-84): traversal_limit_words defaults to 8 Mi words
 * (message.h:54).  The 512-segment cap is fixed by serialize.c++:217. */
typedef struct cpk_limits {
  uint64_t traversal_limit_words;
} cpk_limits;

typedef struct cpk_ctx cpk_ctx;

/* One context per (device, host thread).  Scratch grows on demand; cpk_reserve pre-sizes it so
 * that later calls allocate nothing (required before capturing calls into a hipGraph).  Device
 * scratch for a batch of W words in T = ceil(W / 2048) pack tiles: a byte arena of 4 KiB per
 * pack tile (2 W bytes, at most 8 GiB), ~41 B per pack tile and 1 bit per word; for unpack ~44 B
 * per 4 KiB of packed input (~570 B with the split message decode, CPK_UNPACK_SPLIT=1: chain 0's
 * record-start bits, 512 B) and a few tens of bytes per message; for the stream split, 8 B per
 * output word (the record-head map). */
cpk_status cpk_init(int device, cpk_ctx** out);
cpk_status cpk_destroy(cpk_ctx* ctx);
cpk_status cpk_reserve(cpk_ctx* ctx, uint64_t max_words, uint64_t max_packed_bytes,
                       uint64_t max_items);
/* hipStreamSynchronize(stream), then return (and clear) the first device-side batch error since
 * the previous cpk_sync: CPK_OK, CPK_ERR_CAPACITY or CPK_ERR_INTERNAL. */
cpk_status cpk_sync(cpk_ctx* ctx, void* stream);

/* Worst-case packed bytes for `words` words in `chunks` chunks: 8*words + ceil(words/2) +
 * 2*chunks (a lone F word costs 10 B and cannot be followed by another raw-eligible word
 * without joining its run; doc/encoding.md:328-329).  Use it to size packed buffers. */
uint64_t cpk_packed_bound(uint64_t words, uint64_t chunks);

/* ------------------------------------------------------------------------------------------
 * PACK (device-resident)
 *
 * a1 + a6: PackedOutputStream::write once per piece (serialize-packed.c++:307-431 via
 * kj/io.c++:109-113).  Chunk c is d_words[chunk_word_off[c] .. chunk_word_off[c+1]);
 * chunk_word_off has nchunks+1 non-decreasing entries, [0] == 0 and [nchunks] == total_words
 * (empty chunks allowed).  The packed chunks are concatenated into d_out;
 * d_chunk_out_off[c] (nchunks+1 entries) receives each chunk's packed start and the total. */
cpk_status cpk_pack_chunks(cpk_ctx* ctx, const uint64_t* d_words, uint64_t total_words,
                           const uint64_t* d_chunk_word_off, uint64_t nchunks,
                           uint8_t* d_out, uint64_t out_capacity, uint64_t* d_chunk_out_off,
                           void* stream);

/* a5 + a7: writePackedMessage(BufferedOutputStream&, segments) for a batch
 * (serialize-packed.c++:460-464 over writeMessage serialize.c++:332-357).  Message i is the flat
 * serialized message d_words[msg_word_off[i] .. msg_word_off[i+1]) -- segment table then
 * segments, the layout messageToFlatArray produces (serialize.c++:161-190); msg_word_off has
 * nmsgs+1 entries, [0] == 0, [nmsgs] == total_words.  The table is read in place to find the
 * chunk boundaries.  d_msg_out_off (nmsgs+1 entries) receives each message's packed start and
 * the total; d_status (may be NULL) CPK_OK, CPK_ERR_BAD_FRAMING or CPK_ERR_EMPTY_MESSAGE. */
cpk_status cpk_pack_messages(cpk_ctx* ctx, const uint64_t* d_words, uint64_t total_words,
                             const uint64_t* d_msg_word_off, uint64_t nmsgs,
                             uint8_t* d_out, uint64_t out_capacity, uint64_t* d_msg_out_off,
                             int32_t* d_status, void* stream);

/* a7 without a host gather: writePackedMessage(output, builder.getSegmentsForOutput())
 * (serialize-packed.h:92-98, serialize-packed.c++:460-464) with the segments left where the
 * message builder keeps them (BuilderArena::getSegmentsForOutput, arena.c++:300-329).
 * h_seg_ptrs[i] is a DEVICE pointer to segment i and h_seg_words[i] its size in words (host
 * arrays of nseg entries, read during the call).  The segment table (serialize.c++:311-330) and
 * the segments are gathered into the context's device staging and packed as nseg + 1 chunks into
 * d_out; *d_out_bytes (device u64) receives the packed size.  Asynchronous on `stream`; output
 * capacity overflow is reported by cpk_sync.  nseg == 0 is CPK_ERR_EMPTY_MESSAGE
 * (serialize.c++:333). */
cpk_status cpk_pack_segments(cpk_ctx* ctx, const uint64_t* const* h_seg_ptrs,
                             const uint64_t* h_seg_words, uint64_t nseg, uint8_t* d_out,
                             uint64_t out_capacity, uint64_t* d_out_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * UNPACK (device-resident)
 *
 * a2 + a8: PackedMessageReader over an array, for a batch (serialize-packed.c++:437-440 ->
 * InputStreamMessageReader serialize.c++:202-302 -> PackedInputStream::tryRead
 * serialize-packed.c++:34-183).  Message i's packed bytes are
 * d_packed[msg_in_off[i] .. msg_in_off[i+1]) (nmsgs+1 entries, [nmsgs] == total_bytes).  The
 * flat unpacked message (table + segments) is written to d_words at d_msg_word_off[i], which
 * this call computes (nmsgs+1 entries: exclusive scan of each message's table-declared size, 0
 * for a message whose header is rejected).  d_status[i] is the reference's first failure for
 * message i (PREMATURE_EOF, RUN_OVERSHOOT, TOO_MANY_SEGMENTS, MESSAGE_TOO_LARGE), or
 * TRAILING_BYTES when the range holds more than one message, or CAPACITY when the message does
 * not fit words_capacity.  limits may be NULL (reference defaults). */
cpk_status cpk_unpack_messages(cpk_ctx* ctx, const uint8_t* d_packed, uint64_t total_bytes,
                               const uint64_t* d_msg_in_off, uint64_t nmsgs,
                               uint64_t* d_words, uint64_t words_capacity,
                               uint64_t* d_msg_word_off, int32_t* d_status,
                               const cpk_limits* limits, void* stream);

/* f1: stream boundary discovery.  d_packed[0, nbytes) holds packed
 * messages back to back with unknown boundaries -- a file or socket buffer written by repeated
 * writePackedMessage, read back by constructing one PackedMessageReader after another on the
 * same stream (serialize-packed-test.c++:348-371).  The device decodes the stream into d_words
 * (the flat messages back to back: table + segments each) and finds every message from the
 * segment tables (serialize.c++:202-242), checking each the way that reader would.
 * Outputs, all device, written asynchronously on `stream`:
 *   *d_nmsgs                       n = messages read cleanly (at most max_msgs);
 *   d_msg_word_off[0..n]           word offsets in d_words ([n] = end of message n-1);
 *   d_msg_in_off[0..n]             packed byte offsets ([n] = bytes the n messages used);
 *   d_status[0..n]                 CPK_OK for each message; [n] = why reading stopped: CPK_OK
 *                                  (the input ended cleanly, or max_msgs), else the reference's
 *                                  failure for the next message (PREMATURE_EOF, RUN_OVERSHOOT,
 *                                  TOO_MANY_SEGMENTS, MESSAGE_TOO_LARGE) or CPK_ERR_CAPACITY
 *                                  when it does not fit words_capacity.
 * The three arrays need max_msgs + 1 entries.  limits may be NULL (reference defaults).
 * nbytes < 2^40 (CPK_ERR_INVALID_ARGUMENT otherwise: record positions share a word with the
 * call's generation). */
cpk_status cpk_split_packed_stream(cpk_ctx* ctx, const uint8_t* d_packed, uint64_t nbytes,
                                   uint64_t* d_words, uint64_t words_capacity, uint64_t max_msgs,
                                   uint64_t* d_msg_word_off, uint64_t* d_msg_in_off,
                                   int32_t* d_status, uint64_t* d_nmsgs, const cpk_limits* limits,
                                   void* stream);

/* a4: computeUnpackedSizeInWords (serialize-packed.c++:482-508) for n independent buffers
 * d_packed[in_off[i] .. in_off[i+1]).  d_words_out[i] = total words; d_status[i] = CPK_OK or
 * CPK_ERR_INVALID_PACKED (then d_words_out[i] = 0). */
cpk_status cpk_unpacked_size(cpk_ctx* ctx, const uint8_t* d_packed, uint64_t total_bytes,
                             const uint64_t* d_in_off, uint64_t n, uint64_t* d_words_out,
                             int32_t* d_status, void* stream);

/* a2 (flat-packed, capnp.c++:1063-1076): PackedInputStream::read of exactly
 * word_off[i+1]-word_off[i] words from each single-chunk buffer d_packed[in_off[i] ..
 * in_off[i+1]) into d_words[word_off[i] ..).  Runs may not overshoot a buffer's word count
 * (RUN_OVERSHOOT); a buffer that ends early is PREMATURE_EOF; unread bytes TRAILING_BYTES. */
cpk_status cpk_unpack_chunks(cpk_ctx* ctx, const uint8_t* d_packed, uint64_t total_bytes,
                             const uint64_t* d_in_off, const uint64_t* d_word_off, uint64_t n,
                             uint64_t* d_words, uint64_t words_capacity, int32_t* d_status,
                             void* stream);

/* Batch exchange (multi-GPU): copies n byte ranges
 * d_src[d_src_off[i], +d_len[i]) to d_dst[d_dst_off[i], ...) on the device -- the placement of
 * each shard's packed messages at their global offsets when the shards are not contiguous
 * message ranges (round-robin: message k of the global batch at position k of the one packed
 * stream, as serialize-packed-test.c++:348-371 reads messages back to back).  Ranges must not
 * overlap in d_dst.  No reference counterpart (the reference has one process, one stream). */
cpk_status cpk_copy_ranges(cpk_ctx* ctx, const uint8_t* d_src, const uint64_t* d_src_off,
                           const uint64_t* d_dst_off, const uint64_t* d_len, uint64_t n,
                           uint8_t* d_dst, void* stream);

/* ------------------------------------------------------------------------------------------
 * Host-buffer convenience: the path the reference actually sits on (a socket or file buffer).
 * These stage through the context's device buffers and include the H2D and D2H copies.
 * Synchronous.  Offsets arrays are host arrays with the same meaning as above. */
cpk_status cpk_pack_messages_host(cpk_ctx* ctx, const uint64_t* h_words, uint64_t total_words,
                                  const uint64_t* h_msg_word_off, uint64_t nmsgs,
                                  uint8_t* h_out, uint64_t out_capacity, uint64_t* h_msg_out_off,
                                  int32_t* h_status);
cpk_status cpk_unpack_messages_host(cpk_ctx* ctx, const uint8_t* h_packed, uint64_t total_bytes,
                                    const uint64_t* h_msg_in_off, uint64_t nmsgs,
                                    uint64_t* h_words, uint64_t words_capacity,
                                    uint64_t* h_msg_word_off, int32_t* h_status,
                                    const cpk_limits* limits);

/* ------------------------------------------------------------------------------------------
 * Stream readers (serialize-packed.c++:437-458 PackedMessageReader over a BufferedInputStream;
 * serialize-packed-test.c++:348-371 reads two messages from one stream).
 * Like cpk_unpack_messages, plus d_msg_in_end[i] = the absolute packed byte offset where
 * message i actually ends -- the bytes the reader consumed from its stream.  A message whose
 * [in_off[i], in_off[i+1]) range holds more bytes than it uses still reports
 * CPK_ERR_TRAILING_BYTES in d_status (with d_msg_in_end set): for a stream reader that is
 * success, the remaining bytes belong to the next message. */
cpk_status cpk_read_packed_messages(cpk_ctx* ctx, const uint8_t* d_packed, uint64_t total_bytes,
                                   const uint64_t* d_msg_in_off, uint64_t nmsgs,
                                   uint64_t* d_words, uint64_t words_capacity,
                                   uint64_t* d_msg_word_off, int32_t* d_status,
                                   uint64_t* d_msg_in_end, const cpk_limits* limits,
                                   void* stream);
/* One message from the front of a host buffer (what PackedMessageReader's constructor reads):
 * decodes on the device, returns the flat words (table + segments) in h_words, their count in
 * *words_out and the packed bytes used in *consumed_out.  CPK_ERR_PREMATURE_EOF when the buffer
 * ends inside the message (a stream caller reads more and retries); CPK_ERR_CAPACITY (with
 * *words_out set) when h_words is too small. */
cpk_status cpk_read_packed_message_host(cpk_ctx* ctx, const uint8_t* h_packed,
                                       uint64_t avail_bytes, uint64_t* h_words,
                                       uint64_t words_capacity, uint64_t* words_out,
                                       uint64_t* consumed_out, const cpk_limits* limits);
/* PackedOutputStream::write (serialize-packed.c++:307-431) of host chunks: chunk i =
 * h_words[h_chunk_word_off[i] .. h_chunk_word_off[i+1]), each packed on its own. */
cpk_status cpk_pack_chunks_host(cpk_ctx* ctx, const uint64_t* h_words, uint64_t total_words,
                                const uint64_t* h_chunk_word_off, uint64_t nchunks, uint8_t* h_out,
                                uint64_t out_capacity, uint64_t* h_chunk_out_off);
/* PackedInputStream::tryRead at a record boundary (serialize-packed.c++:34-183): decodes exactly
 * nwords words from the front of a host buffer into h_words and returns the packed bytes they
 * used in *consumed_out.  CPK_ERR_PREMATURE_EOF when the buffer ends first (a stream caller
 * reads more and retries); CPK_ERR_RUN_OVERSHOOT when a run crosses the nwords boundary ("Packed
 * input did not end cleanly on a segment boundary."). */
cpk_status cpk_unpack_words_host(cpk_ctx* ctx, const uint8_t* h_packed, uint64_t avail_bytes,
                                 uint64_t* h_words, uint64_t nwords, uint64_t* consumed_out);
/* The device step of PackedInputStream::tryRead / skip (serialize-packed.c++:34-183, :185-299)
 * over whatever one stream buffer holds: decodes whole records from the front of
 * h_packed[0, avail_bytes) until max_words words are out (CPK_OK), a zero or raw run would cross
 * max_words (CPK_ERR_RUN_OVERSHOOT), or the buffer ends first (CPK_ERR_PREMATURE_EOF).  In all
 * three cases *consumed_out / *words_out are the record boundary where the read stopped -- for
 * the two failures the start of the record that did not fit -- and the words decoded before it,
 * which land in h_words (h_words NULL: a skip -- the records are parsed and checked with no
 * output buffer at all, nothing stored on the device either).  The stream
 * caller keeps the unconsumed bytes in front of the next buffer and calls again. */
cpk_status cpk_unpack_prefix_host(cpk_ctx* ctx, const uint8_t* h_packed, uint64_t avail_bytes,
                                  uint64_t* h_words, uint64_t max_words, uint64_t* words_out,
                                  uint64_t* consumed_out);
/* computeUnpackedSizeInWords (serialize-packed.c++:482-508) of one host buffer. */
cpk_status cpk_unpacked_size_host(cpk_ctx* ctx, const uint8_t* h_packed, uint64_t nbytes,
                                  uint64_t* words_out);

/* ------------------------------------------------------------------------------------------
 * Synthetic workloads (benchmarks and tests).  Fills d_words with nmsgs flat
 * messages whose word offsets are given in d_msg_word_off (nmsgs+1 entries, e.g. from
 * cpk_gen_offsets).  Message i of the call is global message first_msg + i * msg_stride
 * (msg_stride 0 is taken as 1; round-robin sharding passes first_msg = rank, msg_stride =
 * world).  Every word is a function of (seed, global message id, word index) only, so all
 * GPUs and the host restatement (oracle) build identical bytes without transfers.
 *   profile 0 "flat"    -- flat-struct mix (45% small ints, 20% u32 pairs, 15% zero, 10%
 *                          pointers, 10% ASCII text)
 *   profile 1 "pointer" -- pointer-heavy: zero stretches of 264..336 words between short runs of
 *                          pointers / small ints
 *   profile 2 "text"    -- ASCII text (no zero byte)
 *   profile 3 "mixed"   -- per-message choice of 0/1/2 by hash */
cpk_status cpk_gen_messages(cpk_ctx* ctx, int profile, uint64_t seed, uint64_t first_msg,
                            uint64_t msg_stride, uint64_t nmsgs, uint32_t nseg,
                            const uint64_t* d_msg_word_off,
                            uint64_t* d_words, void* stream);
/* Message sizes for the generator: message i has nseg segments of seg_words words each, or,
 * when seg_words == 0, one segment of 2^k words with k uniform in [3, 11] by hash (config C5).
 * Writes d_msg_word_off (nmsgs+1 entries) on the device and returns the total word count. */
cpk_status cpk_gen_offsets(cpk_ctx* ctx, uint64_t seed, uint64_t first_msg,
                           uint64_t msg_stride, uint64_t nmsgs, uint32_t nseg, uint64_t seg_words, uint64_t* d_msg_word_off,
                           uint64_t* total_words_out, void* stream);

/* ------------------------------------------------------------------------------------------
 * Measurement hooks (bench.py).  When enabled, every pack / unpack call brackets its tile
 * kernels with HIP events on the call's stream: timer 0 the pack kernels after the framing
 * launch (tile kernel, scan of the tile byte counts, placement -- or the direct kernel alone),
 * timer 1 the unpack kernels after the header launch, timer 2 the unpack tile kernel alone;
 * timers 3..7 are unused.  cpk_timing_read synchronises the events, returns the summed
 * milliseconds and
 * launch counts of timers 0 and 1 since the last read, and clears every timer;
 * cpk_timing_read_all does the same for all CPK_TIMERS timers. */
#define CPK_TIMERS 8
cpk_status cpk_timing_enable(cpk_ctx* ctx, int on);
cpk_status cpk_timing_read(cpk_ctx* ctx, double* pack_ms, uint64_t* pack_launches,
                           double* unpack_ms, uint64_t* unpack_launches);
cpk_status cpk_timing_read_all(cpk_ctx* ctx, double* ms /* CPK_TIMERS */,
                               uint64_t* launches /* CPK_TIMERS */);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* CPK_H_ */
