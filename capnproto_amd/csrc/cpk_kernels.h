// cpk_kernels.h -- internal launch interface between the C-ABI layer (cpk_api.cpp) and the HIP
// kernels.  Not installed; include/cpk.h is the public boundary.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cpk {

constexpr uint64_t kPackTileWords = 2048;       // words per workgroup tile (cpk_pack.hip)
constexpr uint64_t kPackScratchBytes = 10 * kPackTileWords;  // a tile's packed bytes, worst case
// pack tiles of at most this many packed bytes may leave them in the byte arena (cpk_pack.hip),
// so the arena never needs more than this per tile
constexpr uint32_t kPackArenaTile = 4096;
constexpr uint64_t kUnpackTileBytes = 4096;     // packed bytes per unpack tile (>= 2050)

struct PackTileArgs {
  const uint64_t* words;       // batch of words (all chunks back to back)
  uint64_t nwords;
  uint64_t* chunk_bits;        // bit i set <=> word i starts a chunk (word 0 always); zero at
                               // rest: each tile clears the words of its own 2048 words
  uint8_t* tile_starts;        // byte t set <=> tile t's first word starts a chunk (read and
                               // cleared by tile t - 1)
  uint64_t ntiles;
  uint8_t* out;
  uint64_t out_capacity;
  // optional: output byte offset of each word position pos[0..npos] (sorted)
  const uint64_t* pos;
  uint64_t npos;               // index of the last entry (pos has npos + 1 entries)
  const uint64_t* tile_first;  // per tile: first i with pos[i] >= tile start
  uint64_t* pos_out;
  uint64_t* total_out;         // optional: total packed bytes
  // scratch
  uint32_t* state;             // ntiles exit budgets (0x80000000 | raw << 8 | budget), zeroed
  uint64_t* tile_bytes;        // ntiles packed bytes per tile
  uint8_t* arena;              // byte arena (16-byte aligned pieces) for the tiles whose offset is
  uint64_t arena_cap;          // not known in time, arena_cap bytes
  unsigned long long* arena_next;  // bytes of the arena taken so far (zeroed)
  uint64_t* tpiece;            // per tile: its arena piece (~0: written straight out or not at all)
  uint64_t* gdesc;             // placement group descriptors (zeroed)
  uint32_t* thole;             // byte of a tile's provisional count (~0: none)
  uint32_t* tpatch;            // the next tile's final value for it (0x100 | v; 0: none)
  uint32_t* err;
  // single-tile batches: the framing launch's work done by the tile kernel itself (frame_mode 1:
  // message batch, frame_off = message word offsets, statuses to frame_status; 2: chunk
  // offsets; 0: framed by the framing launch)
  uint32_t frame_mode;
  uint32_t* err_host;          // single-tile batch: where to copy the error word at the end (or NULL)
  const uint64_t* frame_off;
  uint64_t frame_n;
  int32_t* frame_status;
  uint64_t* desc;              // tile descriptors (AGG | bytes, INCL | inclusive prefix), zeroed
};

// tiles -> out when the tile's offset is known in time, else a piece of the byte arena
// (tile_bytes, thole, tpatch, desc, tpiece); then placement: offsets from a scan of the tile byte
// counts (kPlaceGroup tiles per workgroup), arena pieces -> out
hipError_t launch_pack_tiles(const PackTileArgs& a, hipStream_t stream);
hipError_t launch_pack_place(const PackTileArgs& a, hipStream_t stream);
constexpr uint64_t kPackPlaceGroup = 64;
inline uint64_t pack_place_groups(uint64_t ntiles) {
  return (ntiles + kPackPlaceGroup - 1) / kPackPlaceGroup;
}
// tile_first (first i with pos[i] >= tile start, per tile) as extra blocks of a prologue
// kernel: one launch fewer per call.  ntiles == 0: no such job.
struct TileFirstJob {
  const uint64_t* pos;
  uint64_t npos, ntiles, T;
  uint64_t* out;
  uint64_t* outpos = nullptr;  // optional: pos[out[t]] (~0 past the end)
  // optional: zero zero_words u64 at `zero` in further blocks of the same launch (scratch the
  // kernels after the prologue expect zeroed: one launch fewer)
  uint64_t* zero = nullptr;
  uint64_t zero_words = 0;
};
// The chunk-start bitmap (OR-ed into zeroed bits, and into tstarts for the first word of a
// pack tile of kPackTileWords words), tile_first and the zeroing of TileFirstJob::zero in one
// launch.
hipError_t launch_message_bits(const uint64_t* words, const uint64_t* off, uint64_t n,
                               uint64_t N, uint64_t* bits, uint8_t* tstarts, int32_t* status,
                               const TileFirstJob& tf, hipStream_t stream);
hipError_t launch_chunk_bits(const uint64_t* off, uint64_t n, uint64_t N, uint64_t* bits,
                             uint8_t* tstarts, const TileFirstJob& tf, hipStream_t stream);

struct UnpackArgs {
  const uint8_t* packed;        // batch of packed bytes
  uint64_t nbytes;
  const uint64_t* in_off;       // nmsgs + 1 byte offsets
  uint64_t nmsgs;
  const uint64_t* tile_first;   // per tile: first m with in_off[m] >= tile start
  const uint64_t* word_off;     // nmsgs + 1 word offsets (NULL in size-only mode)
  const int32_t* hdr_status;    // header verdicts (NULL: all OK)
  uint64_t* words;
  uint64_t words_capacity;
  int32_t* status;
  uint64_t* size_out;           // mode 2
  uint64_t* in_end;             // optional: packed byte where each message actually ends
  uint64_t* rec_pos;            // optional: packed byte of the record whose head is word i,
                                // tagged with the call's generation (rec_tag below)
  const uint64_t* rec_gen;      // with rec_pos: the call's generation (device word; the tag is
                                // gen << kRecGenShift)
  uint32_t mode;                // 0 messages, 1 exact-size chunks (flat-packed), 2 size only
  uint64_t ntiles;
  uint64_t* desc;               // ntiles tile descriptors (cpk_unpack.hip), zeroed
  uint32_t* x0p;                // ntiles chain-0 exits (0x80000000 | exit), zeroed
  uint32_t* err;
  unsigned long long* stamps;   // diagnostic build only (env CPK_STAMPS), else NULL
  uint32_t debug_skip;          // diagnostic (env CPK_DEBUG_SKIP): 4 no chain-0 walks, 8 no look-back,
                                // 16 no record batches, 32 no lists; return after 64 staging and
                                // message window, 128 chain 0, 256 entry and look-back; 512 at once
  const uint64_t* tile_firstpos;  // in_off[tile_first[t]]: the first message start >= tile start
  uint64_t* hdr_desc;           // the header launch's scan descriptors (zero at rest): cleared
  uint64_t hdr_nblocks;         // by the tile kernel once the headers are done (0: none)
  // a single-tile message batch of at most kUnpackFuseMsgs messages: the header launch's work
  // (headers, word offsets, statuses) done by the tile kernel itself (0: header launch ran)
  uint64_t* desc2;              // flat stream decode only (else NULL): per tile, zeroed, its
                                // exit and words for a second candidate entry (cpk_unpack.hip)
  uint32_t hdr_fuse;
  uint32_t* err_host;           // fused batch: where to copy the error word at the end (or NULL)
  uint64_t hdr_limit;
  uint64_t* hdr_word_off;
  int32_t* hdr_status_out;
  uint32_t prio;                // batches of very long messages: raised wave priority (cpk_unpack.hip)
  // The split message decode (cpk_unpack.hip, "Split decode"): phase 0 one pass (chain, look-back
  // and expansion per tile); 1 the index launch (chain 0 per tile, published with its record-start
  // bits); 2 the expansion launch (after the resolve launch).
  uint32_t phase;
  uint64_t* tbits;              // ntiles * 64: each tile's base-chain record starts (1 bit per byte)
  uint32_t* tegs;               // ntiles: each tile's guessed entry
  const uint64_t* texcl;        // ntiles: words of the tile's first message before the tile
  const uint32_t* gate;         // non-zero: the resolve launch could not place every tile
};
constexpr uint64_t kUnpackFuseMsgs = 256;

// The resolve launch of the split message decode: every tile's words before it in its first
// message, from the index launch's descriptors (a segmented scan over 64-tile groups; tiles whose
// guessed entry was wrong re-traced from the true one).
struct ResolveArgs {
  const uint8_t* packed;
  uint64_t nbytes;
  uint64_t ntiles;
  const uint64_t* desc;         // the index launch's tile descriptors
  const uint32_t* x0p;          // ... and base-chain exits
  const uint64_t* tbits;        // ... and record-start bits
  const uint64_t* tile_firstpos;
  uint64_t* gdesc;              // per 64-tile group look-back descriptors (zeroed)
  unsigned int* ticket;         // group tickets (zeroed)
  uint64_t* texcl;
  uint32_t* gate;               // set when a tile's true exit is not its base-chain exit (zeroed)
  uint32_t* err;
};
constexpr uint64_t kResolveGroup = 64;
__host__ __device__ inline uint64_t resolve_groups(uint64_t ntiles) { return (ntiles + kResolveGroup - 1) / kResolveGroup; }
hipError_t launch_unpack_resolve(const ResolveArgs& r, hipStream_t stream);

// The stream split's record-head map holds (gen << kRecGenShift) | packed byte for a record head,
// anything else elsewhere: an entry counts only with the call's generation, so the map is filled
// (0xff bytes: generation 0xffffff, never a call's) only when its layout changes or the
// generation counter wraps, not on every call (the fill of a 3.55 GiB stream's map: 0.61 ms).
constexpr int kRecGenShift = 40;
constexpr uint64_t kRecPosMask = (1ull << kRecGenShift) - 1;
constexpr uint64_t kRecGenMax = 1ull << 23;

// Unpack stages (launch_unpack_stage): the one-pass tile kernel, or the split decode's index and
// expansion launches (the resolve launch between them is launch_unpack_resolve).
constexpr int kUnpackTiles = 0;
constexpr int kUnpackIndex = 1;
constexpr int kUnpackExpand = 2;

uint32_t debug_skip();

// Diagnostic stamp buffers: kStampRows rows of kStampSlots u64 (a block adds into row
// blockIdx % kStampRows, so the atomics of the waves stay apart); cpk_debug_stamps sums rows.
constexpr int kStampSlots = 16;
constexpr int kStampRows = 256;

// Diagnostic stamp buffers (env CPK_STAMPS=1): [1] unpack counters.
unsigned long long* debug_stamps(int which);

// Headers + their word offsets in one launch (decoupled look-back over header blocks whose
// descriptors `desc` -- header_scan_blocks(n) u64 -- are zero on entry and cleared again by the
// tile kernel through UnpackArgs::hdr_desc); word_off gets n + 1 entries.
uint64_t header_scan_blocks(uint64_t n);
hipError_t launch_unpack_header(const uint8_t* packed, uint64_t P, const uint64_t* in_off,
                                uint64_t n,
                                uint64_t limit, uint64_t* word_off, int32_t* hdr_status,
                                int32_t* status, uint64_t* desc, uint32_t* err,
                                const TileFirstJob& tf, hipStream_t stream);
hipError_t launch_unpack_stage(int stage, const UnpackArgs& a, hipStream_t stream);
hipError_t launch_unpack_init(uint32_t mode, const uint64_t* in_off, const uint64_t* word_off,
                              uint64_t n, int32_t* status, uint64_t* size_out,
                              const TileFirstJob& tf, hipStream_t stream);

// Stream boundary discovery (cpk_stream.hip).  meta (device, 4 u64): [0] packed byte and [1]
// word where the flat decode of the stream stopped, [2] its cpk_status; the walk follows the
// segment tables from word 0 over the decoded words.
// Fills nbytes at p (8-byte aligned) with value: the codec's scratch zeroing.
hipError_t launch_fill(void* p, uint64_t nbytes, uint8_t value, hipStream_t stream);
// Streaming 16-byte-per-lane copy (diagnostic: the bench's measured copy ceiling).
hipError_t launch_copy(void* dst, const void* src, uint64_t nbytes, uint32_t blocks,
                       hipStream_t stream);
hipError_t launch_set_u64x4(uint64_t* dst, uint64_t v0, uint64_t v1, uint64_t v2, uint64_t v3,
                            hipStream_t stream);
// The message chain over the decoded words, block-parallel (cpk_stream.hip); scratch holds
// split_scratch_bytes(words_capacity).
uint64_t split_scratch_bytes(uint64_t words_capacity);
// The split's generation (device word genw): the next one, or 1 when `force` (a new map layout)
// or on wrap-around, which also sets *fill; then the map is filled where *fill says so.
hipError_t launch_split_gen(uint64_t* genw, uint32_t* fill, bool force, uint64_t* rec_pos,
                            uint64_t nbytes, hipStream_t stream);
hipError_t launch_split_walk(const uint8_t* packed, uint64_t nbytes, const uint64_t* words,
                             const uint64_t* rec_pos, const uint64_t* rec_gen,
                             const uint64_t* meta, uint64_t max_msgs,
                             uint64_t limit, uint64_t words_capacity, void* scratch,
                             uint64_t* msg_word_off, uint64_t* msg_in_off, int32_t* status,
                             uint64_t* nmsgs, hipStream_t stream);

// n byte ranges src[src_off[i], +len[i]) -> dst[dst_off[i], ...) (the multi-GPU gather).
hipError_t launch_copy_ranges(const uint8_t* src, const uint64_t* src_off,
                              const uint64_t* dst_off, const uint64_t* len, uint64_t n,
                              uint8_t* dst, hipStream_t stream);

hipError_t launch_gather_segments(const uint64_t* meta, uint32_t nseg, uint64_t total,
                                  uint64_t* out, hipStream_t stream);

hipError_t launch_gen(int profile, uint64_t seed, uint64_t first_msg, uint64_t stride,
                      uint64_t nmsgs,
                      uint32_t nseg, const uint64_t* off, uint64_t* words, hipStream_t stream);
hipError_t launch_gen_sizes(uint64_t seed, uint64_t first_msg, uint64_t stride, uint64_t nmsgs,
                            uint32_t nseg,
                            uint64_t seg_words, uint64_t* sizes, hipStream_t stream);

uint64_t scan_tiles(uint64_t n);
// out[0..n] = exclusive prefix sums of in[0..n), out[n] = total.  counter/desc zeroed before.
hipError_t launch_exclusive_scan(const uint64_t* in, uint64_t n, uint64_t* out, uint32_t* counter,
                                 uint64_t* desc, uint32_t* err, hipStream_t stream);

}  // namespace cpk
