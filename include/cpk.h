/* cpk.h -- C ABI of the MI355X-native Cap'n Proto *packed* wire codec (libcpk_hip.so).
 *
 * This is the drop-in boundary under the reference's packed stream/message API
 * (capnproto c++/src/capnp/serialize-packed.h:32-107).  Every entry point takes plain
 * pointers and sizes; device pointers are HBM allocations (hipMalloc or torch tensors),
 * `stream` is a hipStream_t passed as void* (NULL = the default stream).  No C++ exception
 * crosses this boundary: failures come back as cpk_status, per-message failures as int32
 * codes in a caller-owned status array (same enum).
 *
 * Ownership (mirrors serialize-packed.h:46,60 -- streams borrow, never own): the caller owns
 * every buffer; a cpk_ctx owns only its scratch (look-back flags, tile maps, scans).
 * Threading: one cpk_ctx per (device, host thread); any number of contexts may run in parallel.
 *
 * Wire format recap (doc/encoding.md:296-349): the input is a sequence of 8-byte words.  Each
 * word becomes a tag byte (bit i set <=> byte i non-zero) followed by its non-zero bytes.  Tag
 * 0x00 is followed by a count N<=255 of further all-zero words; tag 0xff by a count N<=255 of
 * further words with at most one zero byte, copied raw.  Runs never cross a chunk: a "chunk" is
 * one OutputStream::write() piece -- the segment table, then each segment
 * (serialize.c++:332-357 -> kj/io.c++:109-113).
 */
#ifndef CPK_H_
#define CPK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CPK_ABI_VERSION 1

typedef enum cpk_status {
  CPK_OK = 0,
  /* kj/io.c++:53 / :118 "Premature EOF" -- packed input ended before the message did.
   * (PackedInputStream's own "Premature end of packed input." at serialize-packed.c++:57 is
   * unreachable behind BufferedInputStream::getReadBuffer's check; pinned by oracle/_ref.) */
  CPK_ERR_PREMATURE_EOF = 1,
  /* serialize-packed.c++:128-131, :140-143 */
  CPK_ERR_RUN_OVERSHOOT = 2,
  /* serialize.c++:217 "Message has too many segments." (segment count > 512) */
  CPK_ERR_TOO_MANY_SEGMENTS = 3,
  /* serialize.c++:235-242 "Message is too large." (> ReaderOptions::traversalLimitInWords) */
  CPK_ERR_MESSAGE_TOO_LARGE = 4,
  /* serialize-packed.c++:491-502 "invalid packed data" (computeUnpackedSizeInWords) */
  CPK_ERR_INVALID_PACKED = 5,
  /* pack input: a flat message's segment table disagrees with its word count */
  CPK_ERR_BAD_FRAMING = 6,
  /* unpack batch: the message parse finished before its [in_off[i], in_off[i+1]) range did */
  CPK_ERR_TRAILING_BYTES = 7,
  /* kj/io.c++:281-282 "backing array was not large enough" -- output capacity too small */
  CPK_ERR_CAPACITY = 8,
  CPK_ERR_INVALID_ARGUMENT = 9,
  CPK_ERR_HIP = 10,
  /* serialize.c++:333 "Tried to serialize uninitialized message." (zero segments) */
  CPK_ERR_EMPTY_MESSAGE = 11,
  /* internal: the device look-back gave up waiting (should never happen; bounded spin) */
  CPK_ERR_INTERNAL = 12,
  CPK_ERR_NO_DEVICE = 13
} cpk_status;

/* Reference message text for a status ("" for CPK_OK). */
const char* cpk_status_string(int32_t status);

/* ReaderOptions (capnp/message.h:51-84).  traversal_limit_words default 8 Mi words
 * (message.h:54); the 512-segment cap is fixed by serialize.c++:217. */
typedef struct cpk_limits {
  uint64_t traversal_limit_words;
} cpk_limits;

typedef struct cpk_ctx cpk_ctx;

/* One context per device.  Allocates no large buffers up front; scratch grows on demand. */
cpk_status cpk_init(int device, cpk_ctx** out);
cpk_status cpk_destroy(cpk_ctx* ctx);
int        cpk_abi_version(void);
/* Device synchronisation helper (hipStreamSynchronize); the batch calls are asynchronous. */
cpk_status cpk_stream_sync(cpk_ctx* ctx, void* stream);

/* Worst-case packed bytes for `words` words split into `chunks` chunks:
 *   8*words + ceil(words/2) + 2*chunks  (an F word costs 10 B but must be followed by a
 *   cheaper word unless the chunk ends).  Use it to size d_out. */
uint64_t cpk_packed_bound(uint64_t words, uint64_t chunks);

/* ------------------------------------------------------------------------------------------
 * a1 + a6: PackedOutputStream::write per piece (serialize-packed.c++:307-431, kj/io.c++:109-113).
 * Packs `nchunks` independent word chunks d_words[chunk_word_off[c] .. chunk_word_off[c+1]) and
 * concatenates the packed bytes in chunk order into d_out.  d_chunk_out_off[c] receives each
 * chunk's packed start, d_chunk_out_off[nchunks] the total.  chunk_word_off must be
 * non-decreasing (empty chunks allowed).  Asynchronous on `stream`. */
cpk_status cpk_pack_chunks(cpk_ctx* ctx, const uint64_t* d_words, const uint64_t* d_chunk_word_off,
                           uint64_t nchunks, uint8_t* d_out, uint64_t out_capacity,
                           uint64_t* d_chunk_out_off, void* stream);

/* a5 + a7: writePackedMessage for a batch (serialize-packed.c++:460-464 over
 * serialize.c++:332-357).  Message i is the flat serialized message
 * d_words[msg_word_off[i] .. msg_word_off[i+1]) -- segment table then segments, i.e. the
 * layout messageToFlatArray (serialize.c++:161-190) produces.  The table is read in place to
 * find the chunk boundaries.  d_msg_out_off[i] receives message i's packed start (nmsgs+1
 * entries); d_status[i] its status (CPK_OK / BAD_FRAMING / TOO_MANY_SEGMENTS).  A message
 * with bad framing is packed as one chunk so offsets stay defined. */
cpk_status cpk_pack_messages(cpk_ctx* ctx, const uint64_t* d_words, const uint64_t* d_msg_word_off,
                             uint64_t nmsgs, uint8_t* d_out, uint64_t out_capacity,
                             uint64_t* d_msg_out_off, int32_t* d_status, void* stream);

/* a2 + a8: PackedMessageReader over an array for a batch (serialize-packed.c++:437-440 ->
 * serialize.c++:202-302, PackedInputStream::tryRead serialize-packed.c++:34-183).  Message i's
 * packed bytes are d_packed[msg_in_off[i] .. msg_in_off[i+1]).  The flat unpacked message
 * (table + segments) is written to d_words at d_msg_word_off[i] (computed here: nmsgs+1
 * entries, exclusive scan of each message's table-declared size, or of 0 for a message whose
 * header is rejected).  words_capacity is checked against the total.  Statuses per message
 * follow the reference's first failure (PREMATURE_EOF, RUN_OVERSHOOT, TOO_MANY_SEGMENTS,
 * MESSAGE_TOO_LARGE) plus TRAILING_BYTES when the range holds more than one message.
 * limits may be NULL (reference defaults). */
cpk_status cpk_unpack_messages(cpk_ctx* ctx, const uint8_t* d_packed, const uint64_t* d_msg_in_off,
                               uint64_t nmsgs, uint64_t* d_words, uint64_t words_capacity,
                               uint64_t* d_msg_word_off, int32_t* d_status,
                               const cpk_limits* limits, void* stream);

/* a4: computeUnpackedSizeInWords (serialize-packed.c++:482-508) for n independent buffers
 * d_packed[in_off[i] .. in_off[i+1]).  d_words_out[i] = total words, d_status[i] = CPK_OK or
 * CPK_ERR_INVALID_PACKED. */
cpk_status cpk_unpacked_size(cpk_ctx* ctx, const uint8_t* d_packed, const uint64_t* d_in_off,
                             uint64_t n, uint64_t* d_words_out, int32_t* d_status, void* stream);

/* flat-packed (capnp.c++:1063-1076, :1126-1134): unpack n single-chunk buffers with no
 * segment table.  Word offsets come from cpk_unpacked_size; each buffer must decode to
 * exactly that many words (computeUnpackedSizeInWords + PackedInputStream::read). */
cpk_status cpk_unpack_chunks(cpk_ctx* ctx, const uint8_t* d_packed, const uint64_t* d_in_off,
                             uint64_t n, uint64_t* d_words, uint64_t words_capacity,
                             uint64_t* d_word_off, int32_t* d_status, void* stream);

/* a3: PackedInputStream::skip semantics (serialize-packed.c++:185-299): given one packed
 * buffer, advance over `skip_words` unpacked words and report the packed byte position
 * reached.  Synchronous; returns PREMATURE_EOF / RUN_OVERSHOOT like the reference. */
cpk_status cpk_skip_words(cpk_ctx* ctx, const uint8_t* d_packed, uint64_t packed_len,
                          uint64_t skip_words, uint64_t* packed_pos_out, void* stream);

/* ------------------------------------------------------------------------------------------
 * Host-buffer convenience (pinned or pageable host memory in and out).  These include the
 * H2D and D2H copies -- the path the reference actually sits on (a socket or file buffer).
 * Synchronous. */
cpk_status cpk_pack_messages_host(cpk_ctx* ctx, const uint64_t* h_words, const uint64_t* h_msg_word_off,
                                  uint64_t nmsgs, uint8_t* h_out, uint64_t out_capacity,
                                  uint64_t* h_msg_out_off, int32_t* h_status);
cpk_status cpk_unpack_messages_host(cpk_ctx* ctx, const uint8_t* h_packed, const uint64_t* h_msg_in_off,
                                    uint64_t nmsgs, uint64_t* h_words, uint64_t words_capacity,
                                    uint64_t* h_msg_word_off, int32_t* h_status,
                                    const cpk_limits* limits);
cpk_status cpk_pack_chunks_host(cpk_ctx* ctx, const uint64_t* h_words, const uint64_t* h_chunk_word_off,
                                uint64_t nchunks, uint8_t* h_out, uint64_t out_capacity,
                                uint64_t* h_chunk_out_off);
cpk_status cpk_unpacked_size_host(cpk_ctx* ctx, const uint8_t* h_packed, uint64_t len,
                                  uint64_t* words_out);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* CPK_H_ */
