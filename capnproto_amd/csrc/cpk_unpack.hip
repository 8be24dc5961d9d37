// cpk_unpack.hip -- MI355X (gfx950) kernels for Cap'n Proto's packed decoding.
//
// Functional spec: PackedInputStream::tryRead (capnproto c++/src/capnp/serialize-packed.c++:
// 34-183) driven by InputStreamMessageReader (serialize.c++:202-302): read the first word, check
// the segment count (< 512), read the rest of the table, check the traversal limit, then read
// all segments.  A record is a tag byte, its non-zero bytes, and for tags 0x00 / 0xff a count
// byte (plus 8*count raw bytes for 0xff); a run may not overshoot the words being read.
//
// Record starts form a chain (next = p + record length) that restarts at every message start.
// The batch of packed bytes is cut into 4 KiB tiles, one wave each; P is read once.
//   1. header_kernel        one thread per message: decodes the first word and the rest of the
//                           segment table with the reference's checks; yields the flat size.
//   2. scan                 message word offsets (cpk_scan.hip).
//   3. unpack_tiles_kernel  per tile: "chain 0", the chain entered at the tile's first byte, from
//                           speculative walks of the 64-byte sub-tiles and a lane fixed point;
//                           its exit is published at once.  The tile's optimistic entry is where
//                           the predecessor's chain 0 leads; its chain from there (traced until
//                           it meets chain 0) gives an aggregate that a look-back over the
//                           predecessors confirms or corrects (a tile holding a message start is
//                           inclusive at once).  Then the records are expanded one lane per
//                           record, 64 consecutive records at a time (coalesced stores), zero and
//                           raw runs written by the wave.
//   (The lane fixed point that settles chain 0 converges in at most 64 rounds -- once lanes
//   0..k-1 hold their true entries lane k's is right -- so no tile is ever left unsettled and
//   there is no serial fallback decoder; a tile that did hit the cap would raise an internal
//   error rather than write words.)
#include <limits.h>

#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {

#ifdef CPK_DIAG
// diagnostic build only (-DCPK_DIAG): per-phase step counters, read by cpk_debug_diag
__device__ unsigned long long g_diag[32];
// per-tile timeline of the first kTimelineTiles tiles: wall-clock stamps (100 MHz) at the phase
// boundaries the clock counters use, then the wave's hardware id; read by cpk_debug_timeline
constexpr int kTimelineTiles = 1 << 16;
__device__ unsigned long long g_timeline[kTimelineTiles * 8];
#endif

namespace {

// The kernel's arguments re-read from the kernarg segment (an opaque copy of its address): the
// rare per-record paths (a record that ends or breaks its message) use these, so the many
// pointers they touch are not hoisted into SGPRs for the whole tile (the kernel spilled SGPRs
// to VGPR lanes and reloaded them with v_readlane inside the record loops).  Every kernel of this
// file takes UnpackArgs as its only argument.
typedef const __attribute__((address_space(4))) UnpackArgs KUnpackArgs;
__device__ __forceinline__ const UnpackArgs& kua() {
  KUnpackArgs* p = (KUnpackArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *(const UnpackArgs*)p;  // (the compiler infers the constant address space back)
}

constexpr int kB = (int)kUnpackTileBytes;  // 4096
constexpr int kPad = 16;
constexpr int kDead = 1 << 24;  // chain ran into the end of the batch



#ifdef CPK_DIAG
// (every 16th workgroup only: a few global atomics per tile from every tile contend enough to
// distort the timings they measure)
__device__ __forceinline__ void diag_add(int k, uint64_t v) {
  if (lane_id() == 0 && (blockIdx.x & 15) == 0) atomicAdd(&g_diag[k], (unsigned long long)v);
}
// wave-level trip count (max over lanes) and lane-step total of a per-lane count n
__device__ __forceinline__ void diag_trips(int k, int n) {
  const uint32_t mx = readlane32(wave_incl_max32((uint32_t)n), 63);
  const uint32_t sm = readlane32(wave_incl_sum32((uint32_t)n), 63);
  diag_add(k, mx);
  diag_add(k + 1, sm);
}
#define CPK_DIAG_ONLY(x) x
#else
#define CPK_DIAG_ONLY(x)
#endif
#ifndef CPK_MERGE_CAP
#define CPK_MERGE_CAP 8
#endif
constexpr int kMergeCap = CPK_MERGE_CAP;               // entry-walk records before the jump walk

// status codes (include/cpk.h)
constexpr int32_t kOK = 0, kEOF = 1, kOvershoot = 2, kTooMany = 3, kTooLarge = 4, kInvalid = 5;
constexpr int32_t kTrailing = 7, kCap = 8;
constexpr int32_t kSizeDone = 100;  // mode 2: last record of the buffer

__device__ __forceinline__ uint64_t load_u64_unaligned(const uint8_t* p) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

// PackedInputStream::read of exactly n words from b[p..end) (serialize-packed.c++:65-177 with
// minBytes == maxBytes); f(index, word) receives every word.  Same failure order as the
// reference: missing bytes -> PREMATURE_EOF, run past n -> RUN_OVERSHOOT (checked once the count
// byte is present, before the raw bytes).
template <class F>
__device__ int32_t decode_exact(const uint8_t* b, uint64_t& p, uint64_t end, uint64_t n, F f) {
  uint64_t o = 0;
  while (o < n) {
    if (p >= end) return kEOF;
    const uint32_t tag = b[p++];
    uint64_t w = 0;
    for (int i = 0; i < 8; i++) {
      if ((tag >> i) & 1) {
        if (p >= end) return kEOF;
        w |= (uint64_t)b[p++] << (8 * i);
      }
    }
    f(o, w);
    o++;
    if (tag == 0 || tag == 0xff) {
      if (p >= end) return kEOF;
      const uint64_t c = b[p++];
      if (c > n - o) return kOvershoot;
      if (tag == 0) {
        for (uint64_t k = 0; k < c; k++) f(o + k, 0);
      } else {
        if (end - p < 8 * c) return kEOF;
        for (uint64_t k = 0; k < c; k++) f(o + k, load_u64_unaligned(b + p + 8 * k));
        p += 8 * c;
      }
      o += c;
    }
  }
  return kOK;
}

// 1. Message headers (serialize.c++:202-242): the flat size of message m in words (segment
// table + segments), 0 when the header fails (its status says why).
// (v0, v1: the message's first 16 packed bytes, read by the caller when end - p >= 16)
__device__ __forceinline__ uint64_t header_words_v(const uint8_t* __restrict__ packed, uint64_t p,
                                                   uint64_t end, uint64_t v0, uint64_t v1,
                                                   uint64_t limit, int32_t* st_out) {
  uint64_t first = 0;
  int32_t st;
  if (end - p >= 16) {
    // the first word's record (<= 10 bytes) from one 16-byte read: decode_exact's steps for
    // one word, with every byte present (a run record's count must be 0 -- it may not cross
    // word 1 -- so its raw bytes are never needed)
    auto byte_at = [&](uint32_t k) -> uint32_t {
      return (uint32_t)((k < 8 ? v0 >> (8 * k) : v1 >> (8 * (k - 8))) & 0xff);
    };
    const uint32_t tag = (uint32_t)(v0 & 0xff);
    uint32_t k = 1;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if ((tag >> i) & 1) first |= (uint64_t)byte_at(k++) << (8 * i);
    }
    st = kOK;
    if (tag == 0 || tag == 0xff) {
      if (byte_at(k) > 0) st = kOvershoot;
      k++;
    }
    p += k;
  } else {
    st = decode_exact(packed, p, end, 1, [&](uint64_t, uint64_t w) { first = w; });
  }
  uint64_t words = 0;
  if (st == kOK) {
    const uint32_t segm1 = (uint32_t)first;
    if (segm1 >= 511) {
      st = kTooMany;
    } else {
      const uint32_t nseg = segm1 + 1;
      uint64_t total = first >> 32;
      if (nseg > 1) {
        st = decode_exact(packed, p, end, (nseg & ~1u) / 2, [&](uint64_t i, uint64_t w) {
          if (2 + 2 * i <= nseg) total += (uint32_t)w;
          if (3 + 2 * i <= nseg) total += (uint32_t)(w >> 32);
        });
      }
      if (st == kOK) {
        if (total > limit) st = kTooLarge;
        else words = nseg / 2 + 1 + total;
      }
    }
  }
  *st_out = st;
  return words;
}
__device__ __forceinline__ uint64_t header_words(const uint8_t* __restrict__ packed,
                                                 const uint64_t* __restrict__ in_off, uint64_t m,
                                                 uint64_t limit, int32_t* st_out) {
  const uint64_t p = in_off[m];
  const uint64_t end = in_off[m + 1];
  uint64_t v0 = 0, v1 = 0;
  if (end - p >= 16) {
    __builtin_memcpy(&v0, packed + p, 8);
    __builtin_memcpy(&v1, packed + p + 8, 8);
  }
  return header_words_v(packed, p, end, v0, v1, limit, st_out);
}

// One launch for the headers and their word offsets: blocks [0, nsb) each take kHdrBlock
// messages (4 per thread), decode their headers and scan the flat sizes into word_off with a
// single-pass decoupled look-back over the blocks (blocks in launch order; a block only waits
// on lower ones).  The look-back descriptors are zero at rest: the tile kernel of the same call
// clears them once every header block is done (UnpackArgs::hdr_desc).  Blocks past nsb compute
// tile_first and zero the tile kernel's scratch (TileFirstJob).
// Headers per thread: 1 for batches of up to kHdrSmall messages (each thread's two dependent
// loads are the launch's latency: C2 10.1 -> 5.9 us), 4 above (fewer look-back blocks: C3 66.6 ->
// 56.3 us).
// (One block of 16 headers per thread for batches of up to 4096, no look-back: C2's header
// launch 5.9 -> 34.7 us -- one CU decoding every header -- so not that.)
constexpr uint64_t kHdrSmall = 1ull << 16;
__host__ __device__ constexpr int hdr_per(uint64_t n) { return n <= kHdrSmall ? 1 : 4; }
template <int kHdrPerThread>
__global__ __launch_bounds__(256) void header_kernel(
    const uint8_t* __restrict__ packed, uint64_t P, const uint64_t* __restrict__ in_off,
    uint64_t n, uint64_t limit, uint64_t* __restrict__ word_off, int32_t* __restrict__ hdr_status,
    int32_t* __restrict__ status, uint64_t* desc, uint32_t* err, TileFirstJob tf,
    uint32_t nsb) {
  if (run_tile_first(tf, nsb)) return;
  __shared__ uint64_t s_wave[4];
  __shared__ uint64_t s_excl;
  const uint64_t b = blockIdx.x;
  const int l = lane_id();
  const int wv = (int)(threadIdx.x >> 6);
  constexpr uint64_t kHdrBlock = 256 * kHdrPerThread;
  const uint64_t m0 = b * kHdrBlock + (uint64_t)kHdrPerThread * threadIdx.x;
  uint64_t w[kHdrPerThread];
  uint64_t sum = 0;
  // every message's offsets, then every message's first 16 bytes, all in flight before any is
  // used (clamped indices and addresses, no branch: a load under a branch is waited for at the
  // join) -- two round trips per thread whatever kHdrPerThread is (C5's header launch 218 -> 206
  // us)
  uint64_t hp[kHdrPerThread], he[kHdrPerThread], v0[kHdrPerThread], v1[kHdrPerThread];
#pragma unroll
  for (int k = 0; k < kHdrPerThread; k++) {
    const uint64_t m = m0 + k < n ? m0 + k : n - 1;
    hp[k] = in_off[m];
    he[k] = in_off[m + 1];
  }
  const bool wide = P >= 16;  // (uniform: else no message has 16 bytes)
#pragma unroll
  for (int k = 0; k < kHdrPerThread; k++) {
    const uint64_t q = (wide && he[k] - hp[k] >= 16) ? hp[k] : 0;
    v0[k] = 0;
    v1[k] = 0;
    if (wide) {
      __builtin_memcpy(&v0[k], packed + q, 8);
      __builtin_memcpy(&v1[k], packed + q + 8, 8);
    }
  }
#pragma unroll
  for (int k = 0; k < kHdrPerThread; k++) {
    const uint64_t m = m0 + k;
    w[k] = 0;
    if (m < n) {
      int32_t st;
      w[k] = header_words_v(packed, hp[k], he[k], v0[k], v1[k], limit, &st);
      hdr_status[m] = st;
      status[m] = st;
    }
    sum += w[k];
  }
  const uint64_t incl = wave_incl_sum64(sum);
  if (l == 63) s_wave[wv] = incl;
  __syncthreads();
  uint64_t before = 0, agg = 0;
#pragma unroll
  for (int v = 0; v < 4; v++) {
    const uint64_t x = s_wave[v];
    if (v < wv) before += x;
    agg += x;
  }
  if (wv == 0) {
    uint64_t excl = 0;
    if (b == 0) {
      if (l == 0) store_agent(desc, kDescIncl | agg);
    } else {
      if (l == 0) store_agent(desc + b, kDescAgg | agg);
      excl = lookback<8>(desc, b, err);
      if (l == 0) store_agent(desc + b, kDescIncl | (excl + agg));
    }
    if (l == 0) s_excl = excl;
  }
  __syncthreads();
  uint64_t o = s_excl + before + incl - sum;
#pragma unroll
  for (int k = 0; k < kHdrPerThread; k++) {
    const uint64_t m = m0 + k;
    if (m < n) word_off[m] = o;
    o += w[k];
    if (m + 1 == n) word_off[n] = o;
  }
}

// Byte length of a record from its tag and its count byte (tag 0x00: + count byte; 0xff: +
// count byte + 8*count raw bytes).
__device__ __forceinline__ int rec_len(uint32_t tag, uint32_t cnt) {
  // (tag - 1 >= 0xfe: tag 0x00 or 0xff, in 32-bit arithmetic -- no 16-bit byte compares)
  const uint32_t run = tag - 1u >= 0xfeu ? 2u : 1u;
  return (int)(__popc(tag) + run + ((tag == 0xffu ? cnt : 0u) << 3));
}

// Staged tile bytes: tile byte p at d[p], zero past the batch end, kPad bytes past the tile, so
// every byte a walk step reads (p, p + 1, p + 9) is in LDS.
__device__ __forceinline__ const uint8_t* ix(const uint8_t* d, int p) { return d + p; }

// Record length at tile position p given the staged rows (no clipping).
__device__ __forceinline__ int record_len(const uint8_t* d, int p) {
  const uint8_t* q = ix(d, p);
  return rec_len(q[0], q[9]);
}

struct SubTile {
  int s, end, vend;  // sub-tile [s, end); walks stop at vend = min(end, batch end)
  uint64_t msw;      // message-start bits of the sub-tile
  int nms_after;     // first message start >= end (tile-relative; may be >= kB)
  bool no_starts;    // wave-uniform: no message start in any sub-tile of the tile
  int pend;          // batch end, tile-relative
};

// First message start after position q of the sub-tile (q >= st.s): the next chain clip.
__device__ __forceinline__ int next_start_after(const SubTile& st, int q) {
  const int k = q - st.s + 1;
  const uint64_t after = k < 64 ? (st.msw >> k) : 0;
  return after ? q + 1 + lowest_bit(after) : st.nms_after;
}

// Length of the record whose tag is t and whose byte 9 past the tag is c9.  (An LDS table of
// lengths by tag measured slower: one more dependent LDS round trip per walk step, and its reads
// collide in banks.)
__device__ __forceinline__ int step_len(uint32_t t, uint32_t c9) { return rec_len(t, c9); }

// Walks from p (inside the sub-tile) marking record starts until the chain leaves the sub-tile
// or reaches a position of `stop`.  Record ends are clipped at the next message start nm, which
// only moves when the chain reaches it (rare), so the step itself carries no message logic.
// Returns the position reached.  (Sub-tiles are 64-byte aligned in the tile: bit p & 63.)
__device__ __forceinline__ int walk(const uint8_t* d, const SubTile& st, int p, uint64_t stop,
                                    uint64_t* marks, uint64_t* runs = nullptr, int* nstep = nullptr) {
  uint64_t m = 0, rm = 0;
  if (st.no_starts) {
    // no message start in the tile: the only clip is the first start after the sub-tile, where
    // the walk ends anyway (most tiles of large messages)
    while (p < st.vend) {
      if (nstep) ++*nstep;
      uint32_t e = d[p];
      const uint32_t c9 = d[p + 9];
      asm("" : "+v"(e));  // a plain 32-bit value: 32-bit compares, no 16-bit byte arithmetic
      const uint64_t bit = 1ull << (p & 63);
      m |= bit;
      if (e - 1u >= 0xfeu) rm |= bit;
      const int np = p + step_len(e, c9);
      p = np < st.nms_after ? np : st.nms_after;
      if (p < st.vend && ((stop >> (p & 63)) & 1)) break;
    }
    *marks = m;
    if (runs) *runs = rm;
    return p >= st.pend ? kDead : p;
  }
  int nm = next_start_after(st, p);
  while (p < st.vend) {
    if (nstep) ++*nstep;
    uint32_t e = d[p];
    const uint32_t c9 = d[p + 9];
    asm("" : "+v"(e));
    const uint64_t bit = 1ull << (p & 63);
    m |= bit;
    if (e - 1u >= 0xfeu) rm |= bit;
    int np = p + step_len(e, c9);
    if (np >= nm) {
      np = nm;
      nm = np < st.end ? next_start_after(st, np) : st.nms_after;
    }
    p = np;
    if (p < st.vend && ((stop >> (p & 63)) & 1)) break;
  }
  *marks = m;
  if (runs) *runs = rm;
  if (p >= st.pend) return kDead;
  return p;
}

// Lane-entry fixed point for a tile entry E.  In: the speculative chain of the lane's sub-tile
// (chain, exit sx).  In/out: e (entries).  Out: true record-start mask of the lane and its exit.
// A lane's entry is the largest exit of the earlier lanes that hold a record start (a lane
// covered by a longer record passes nothing on), never below its own start: a wrong far jump of
// one speculative chain is then corrected in the next round instead of being carried from lane
// to lane.  Returns false when the iteration cap is hit (the caller flags the tile).
__device__ __forceinline__ bool settle(const uint8_t* d, const SubTile& st, uint64_t chain,
                                       int sx, int E, int& e, uint64_t& tm, int& out,
                                       uint64_t& runm, int* iters = nullptr) {
  // round 0, every lane entered at its own start, needs no walk: the speculative chain itself
  // (a sub-tile past the batch end passes nothing on)
  bool pass = e >= st.end || e >= st.pend;
  out = pass ? (e >= st.pend ? kDead : e) : sx;
  tm = pass ? 0ull : chain;
  for (int iter = 0; iter < 96; iter++) {
    if (iters) iters[0] = iter + 1;
#ifdef CPK_DIAG
    if (iter && iters) diag_trips(3, iters[1] - iters[2]), iters[2] = iters[1];
#endif
    // the largest exit of the earlier lanes (wave_shr:1 of the inclusive max: no LDS trip)
    const uint32_t incl = wave_incl_max32(pass ? 0u : (uint32_t)out);
    const int prev = (int)wave_shr1_32(incl);
    int en = lane_id() == 0 ? E : (prev > E ? prev : E);
    if (lane_id() > 0 && en < st.s) en = st.s;
    if (!ballot(en != e)) return true;
    e = en;
    pass = e >= st.end || e >= st.pend;
    if (pass) {
      out = e >= st.pend ? kDead : e;
      tm = 0;
    } else if ((chain >> (e - st.s)) & 1) {
      out = sx;
      tm = chain & ~mask_lt(e - st.s);
    } else {
      uint64_t wm, wr;
#ifdef CPK_DIAG
      int ns = 0;
      const int p = walk(d, st, e, chain, &wm, &wr, &ns);
      if (iters) iters[1] += ns;
#else
      const int p = walk(d, st, e, chain, &wm, &wr);
#endif
      runm |= wr;
      if (p != kDead && p < st.vend) {
        out = sx;
        tm = wm | (chain & ~mask_lt(p - st.s));
      } else {
        out = p;
        tm = wm;
      }
    }
  }
  return false;
}

// Positions j of the lane's sub-tile [s, s + 64) with d[s + j] == d[s + j + 9] == 0xff: the head
// of a raw record of 255 words (or two 0xff bytes 9 apart).
__device__ __forceinline__ uint64_t ff_heads(const uint8_t* d, int s) {
  const uint32_t* const w = (const uint32_t*)(d + s);
  uint64_t m = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t y = ~w[k];  // 0xff bytes -> zero bytes
    uint32_t f = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y) & 0x80808080u;
    while (f) {
      const int b = __builtin_ctz(f) >> 3;
      f &= f - 1;
      if (d[s + 4 * k + b + 9] == 0xff) m |= 1ull << (4 * k + b);
    }
  }
  return m;
}

// Positions j of the lane's sub-tile [s, s + 64) whose byte is 0x00 or 0xff: the run records'
// tags among any record starts there (the split decode's expansion launch rebuilds the run mask
// of chain 0 from these instead of walking the chain again).
__device__ __forceinline__ uint64_t run_bytes(const uint8_t* d, int s) {
  const uint32_t* const w = (const uint32_t*)(d + s);
  uint64_t m = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t x = w[k], y = ~x;
    const uint32_t z = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
    const uint32_t f = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y) & 0x80808080u;
    // bits 7, 15, 23, 31 -> 0..3 (one multiply gathers them into bits 21-24)
    const uint32_t nib = ((((z | f) >> 7) * 0x204081u) >> 21) & 15u;
    m |= (uint64_t)nib << (4 * k);
  }
  return m;
}

struct Rec {
  uint32_t tag;
  int hb;       // tag + data bytes
  uint32_t cnt; // run count (0 unless tag 0x00 / 0xff and the count byte is in range)
  bool run;
};

__device__ __forceinline__ Rec read_rec(const uint8_t* d, int p) {
  Rec r;
  r.tag = d[p];
  r.hb = 1 + __popc(r.tag);
  r.run = r.tag == 0 || r.tag == 0xff;
  r.cnt = r.run ? d[p + r.hb] : 0;
  return r;
}

// 8 bytes at any LDS offset q: three aligned dword reads + byte funnel shifts.
__device__ __forceinline__ uint64_t read8(const uint8_t* d, int q) {
  const uint32_t* w = (const uint32_t*)(d + (q & ~3));
  const uint32_t sh = q & 3;
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
  const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
  return ((uint64_t)hi << 32) | lo;
}

// v_perm selector that deposits the first popc(n) bytes of its source into the byte lanes of
// nibble n (byte i <- source byte rank_i when bit i is set, else 0): the inverse of the tag
// compaction (serialize-packed.c++:105-119).
__device__ __forceinline__ uint32_t deposit_sel(uint32_t n) {
  uint32_t sel = 0, r = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const bool b = (n >> i) & 1;
    sel |= (b ? r : 0x0cu) << (8 * i);
    r += b;
  }
  return sel;
}

// Expands a record's word from the staged bytes following its tag (two v_perm_b32).
__device__ __forceinline__ uint64_t expand_word(const uint8_t* d, int p, uint32_t tag,
                                                uint32_t lut) {
  const uint64_t data = read8(d, p + 1);
  const uint32_t tl = tag & 15, th = tag >> 4;
  const uint32_t sl = shfl32(lut, (int)tl), sh = shfl32(lut, (int)th);
  const uint32_t lo = __builtin_amdgcn_perm((uint32_t)(data >> 32), (uint32_t)data, sl);
  const uint64_t d2 = data >> (8 * __popc(tl));
  const uint32_t hi = __builtin_amdgcn_perm((uint32_t)(d2 >> 32), (uint32_t)d2, sh);
  return ((uint64_t)hi << 32) | lo;
}

struct MsgInfo {
  uint64_t base, total, end;  // word offset, flat words, packed end (absolute byte)
  bool ok, fits;
};

// Message m's metadata.
__device__ __forceinline__ MsgInfo msg_info(const UnpackArgs& a, uint64_t m) {
  MsgInfo mi;
  if (!a.word_off) {  // size-only mode
    mi.base = 0;
    mi.total = ~0ull >> 2;
    mi.end = a.in_off[m + 1];
    mi.ok = true;
    mi.fits = false;
    return mi;
  }
  mi.base = a.word_off[m];
  mi.total = a.word_off[m + 1] - mi.base;
  mi.end = a.in_off[m + 1];
  mi.ok = a.hdr_status ? a.hdr_status[m] == kOK : true;
  mi.fits = mi.base + mi.total <= a.words_capacity;
  return mi;
}

// Checks + main word for one record (lane).  wb = words of the message before this record.
// Returns the record's terminal status (or -1), and the run still to be written (run_n words
// at run_dst, raw source run_src or zeros).
struct RunJob {
  uint64_t dst, src;
  uint32_t n;
  bool raw;
  uint64_t end;  // absolute packed byte after this record (terminal records: message end)
  uint64_t bw;   // words of the message decoded at `end`
};

// The terminal record of message m: its end (stream readers), and, for the prefix reads of
// PackedInputStream (size_out given in mode 1), where a failing read stops too -- the start of
// the record that ends the input early or overshoots -- with the words decoded up to there.
__device__ __forceinline__ void report_end(const UnpackArgs& a_unused, uint64_t m, int32_t st,
                                           const RunJob& job) {
  (void)a_unused;
  const UnpackArgs& a = kua();
  if (!a.in_end) return;
  const bool prefix = a.mode == 1 && a.size_out;
  if (st == kOK || st == kTrailing || st == kCap || (prefix && (st == kEOF || st == kOvershoot)))
    a.in_end[m] = job.end;
  if (prefix) a.size_out[m] = job.bw;
}

__device__ __forceinline__ int32_t handle_record(const UnpackArgs& a_unused, const uint8_t* d,
                                                 int p, uint64_t pabs, uint64_t wb,
                                                 const MsgInfo& mi, RunJob* job, uint64_t word) {
  (void)a_unused;
  const UnpackArgs& a = kua();
  job->n = 0;
  job->dst = job->src = 0;
  job->raw = false;
  const Rec r = read_rec(d, p);
  const uint64_t mend = mi.end;
  if (a.mode == 2) {
    // computeUnpackedSizeInWords (serialize-packed.c++:487-505) bounds checks, incl. its
    // `end - ptr >= count` test that admits a record whose last data byte is missing.
    if (mend - pabs < (uint64_t)(r.hb - 1)) return kInvalid;
    uint64_t ptr = pabs + r.hb;
    if (r.run) {
      if (!(ptr < mend)) return kInvalid;
      ptr += 1;
      if (r.tag == 0xff) {
        if (mend - ptr < 8ull * r.cnt) return kInvalid;
        ptr += 8ull * r.cnt;
      }
    }
    return ptr >= mend ? kSizeDone : -1;  // terminal: words = wb + 1 + count (caller)
  }
  if (!mi.ok || wb >= mi.total) return -1;
  int32_t st = -1;
  const bool trunc1 = pabs + r.hb > mend;
  const bool trunc2 = !trunc1 && r.run && pabs + r.hb >= mend;
  uint64_t end = pabs + r.hb;
  uint32_t cnt = (trunc1 || trunc2) ? 0 : r.cnt;
  bool trunc3 = false, over = false;
  if (trunc1 || trunc2) {
    st = kEOF;
  } else if (r.run) {
    end += 1;
    if (wb + 1 + cnt > mi.total) {
      over = true;
      st = kOvershoot;
    } else if (r.tag == 0xff) {
      end += 8ull * cnt;
      if (end > mend) {
        trunc3 = true;
        st = kEOF;
      }
    }
  }
  job->end = end;
  job->bw = wb + 1 + cnt;
  if (st < 0) {
    if (wb + 1 + cnt == mi.total) st = end < mend ? kTrailing : kOK;
    else if (end >= mend) st = kEOF;
  }
  if (trunc1 || trunc2 || trunc3 || over) {  // the read stops before this record
    job->end = pabs;
    job->bw = wb;
  }
  if (st == kOK && !mi.fits) st = kCap;
  if (mi.fits && !trunc1) {
    if (a.words) a.words[mi.base + wb] = word;  // (NULL: a skip, nothing stored)
    if (a.rec_pos) a.rec_pos[mi.base + wb] = pabs | (*a.rec_gen << kRecGenShift);
    uint64_t n = cnt;
    if (over) n = mi.total - wb - 1;
    if (trunc3) {
      const uint64_t avail = (mend - (pabs + r.hb + 1)) / 8;
      n = n < avail ? n : avail;
    }
    if (n) {
      job->n = (uint32_t)n;
      job->dst = mi.base + wb + 1;
      job->raw = r.tag == 0xff;
      job->src = pabs + r.hb + 1;
    }
  }
  return st;
}

// Writes the pending runs of a batch with the whole wave (coalesced).
// d: the wave's LDS copy of packed bytes [dbase, dbase + dlen): a raw run whose bytes lie inside
// it is copied from there (no global round trip per run; dlen 0: always from global memory).
__device__ __forceinline__ void run_jobs(const UnpackArgs& a, const RunJob& job,
                                         const uint8_t* d = nullptr, uint64_t dbase = 0,
                                         uint32_t dlen = 0) {
  uint64_t pend = a.words ? ballot(job.n != 0) : 0ull;  // (no words: a skip)
  const int l = lane_id();
  while (pend) {
    const int j = lowest_bit(pend);
    pend &= pend - 1;
    const uint32_t n = readlane32(job.n, j);
    const uint64_t dst = readlane64(job.dst, j);
    const uint64_t src = readlane64(job.src, j);
    const bool raw = readlane32(job.raw, j);
    if (!raw) {
      for (uint32_t k = l; k < n; k += 64) a.words[dst + k] = 0;
      continue;
    }
    if (src >= dbase && src - dbase + 8ull * n + 4 <= dlen) {
      const uint32_t o0 = (uint32_t)(src - dbase);
      const uint32_t* const d32 = (const uint32_t*)d;
      for (uint32_t k = l; k < n; k += 64) {
        const uint32_t o = o0 + 8 * k, q = o >> 2, sh = o & 3;
        const uint32_t q0 = d32[q], q1 = d32[q + 1], q2 = d32[q + 2];
        const uint32_t lo = __builtin_amdgcn_alignbyte(q1, q0, sh);
        const uint32_t hi = __builtin_amdgcn_alignbyte(q2, q1, sh);
        a.words[dst + k] = ((uint64_t)hi << 32) | lo;
      }
      continue;
    }
    // raw run: every load of a 256-word block is issued before its stores (one round trip per
    // block instead of one per 64 words), each from a clamped index inside the run's bytes;
    // the words are unaligned 8-byte loads (the target's unaligned access mode)
    for (uint32_t k0 = 0; k0 < n; k0 += 256) {
      uint64_t v[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t k = k0 + 64 * i + l;
        __builtin_memcpy(&v[i], a.packed + src + 8ull * (k < n ? k : n - 1), 8);
      }
      // unconditional stores: a lane past the run end loaded word n - 1 (clamped) and writes
      // that same value to it again -- a skipped store would leave its load outstanding, and
      // the next batch would wait for it before reusing the register
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t k = k0 + 64 * i + l;
        a.words[dst + (k < n ? k : n - 1)] = v[i];
      }
    }
  }
}

// A raw run crossing into the next tile (text: runs of up to 2 KiB): its words ending at most
// kRunSplit bytes into the next tile are written by the run's own tile (from its staged bytes
// and kPad), the rest by the next tile, which stages those bytes itself (run_tail) -- rather
// than every crossing run being read whole again from global memory, from another XCD's L2.
constexpr uint32_t kRunSplit = (uint32_t)kPad - 4u;
constexpr uint32_t kShortRunGeneral = 4;  // runs of at most this many words: their own lane
// Runs of a batch: a short run (at most kShortRunGeneral words, zero or raw from the staged tile --
// most runs of dense data, where a zero or raw stretch rarely lasts) is written by its own lane,
// all such lanes together, one word per step; longer runs and raw runs outside the staged bytes
// go through run_jobs (the whole wave per run, coalesced).
__device__ __forceinline__ void run_jobs_batch(const UnpackArgs& a, RunJob job, const uint8_t* d,
                                               uint64_t dbase, uint32_t dlen) {
  if (a.words) {
    const bool in_lds = !job.raw || (job.src >= dbase && job.src - dbase + 8ull * job.n + 4 <= dlen);
    const bool sh = job.n != 0 && job.n <= kShortRunGeneral && in_lds;
    if (ballot(sh)) {
      const uint32_t n = sh ? job.n : 0u;
      const uint32_t o0 = (uint32_t)(job.src - dbase);
      const uint32_t* const d32 = (const uint32_t*)d;
#pragma unroll
      for (uint32_t k = 0; k < kShortRunGeneral; k++) {
        if (!ballot(k < n)) break;
        if (k < n) {
          uint64_t v = 0;
          if (job.raw) {
            const uint32_t o = o0 + 8 * k, q = o >> 2, s3 = o & 3;
            const uint32_t q0 = d32[q], q1 = d32[q + 1], q2 = d32[q + 2];
            v = ((uint64_t)__builtin_amdgcn_alignbyte(q2, q1, s3) << 32) |
                __builtin_amdgcn_alignbyte(q1, q0, s3);
          }
          a.words[job.dst + k] = v;
        }
      }
      if (sh) job.n = 0;
    }
  }
  run_jobs(a, job, d, dbase, dlen);
}

// Per-tile window of message metadata: lane i describes message mw + i.
struct MsgWin {
  int64_t mw;        // message of lane 0 (may be -1 / past the end: empty entries)
  uint64_t start;    // in_off[m]          (~0 for missing entries)
  uint64_t end;      // in_off[m + 1]
  uint64_t base;     // word_off[m]
  uint64_t total;    // word_off[m + 1] - word_off[m]
  uint32_t ok;       // header accepted
};

// Lanes from nl on load lane 0's entry again (the same lines, not more of them) and hold the
// defaults of a missing entry.
__device__ __forceinline__ void load_win(const UnpackArgs& a, int64_t mw, MsgWin& w,
                                         int nl = 64) {
  // every load unconditional, from a clamped index (entries past the batch select their defaults
  // afterwards): loads under branches each got their own wait, three round trips in a row
  const int64_t m = mw + lane_id();
  const bool v = m >= 0 && (uint64_t)m < a.nmsgs && lane_id() < nl;
  const uint64_t mc = v ? (uint64_t)m : (mw >= 0 && (uint64_t)mw < a.nmsgs ? (uint64_t)mw : 0);
  const uint64_t mn = mc + 1 <= a.nmsgs ? mc + 1 : a.nmsgs;
  const uint64_t* const wo = a.word_off ? a.word_off : a.in_off;
  const int32_t* const hs = a.hdr_status ? a.hdr_status : (const int32_t*)a.in_off;
  const uint64_t s0 = a.in_off[mc], e0 = a.in_off[mn];
  const uint64_t b0 = wo[mc], b1 = wo[mn];
  const int32_t h = hs[mc];
  w.mw = mw;
  w.start = v ? s0 : ~0ull;
  w.end = v ? e0 : ~0ull;
  w.base = v && a.word_off ? b0 : 0;
  w.total = !v ? 0 : (a.word_off ? b1 - b0 : ~0ull >> 2);
  w.ok = v && (a.hdr_status ? h == kOK : true);
}

// Starts only (index_kernel needs no more of the window).
__device__ __forceinline__ void load_starts(const UnpackArgs& a, int64_t mw, MsgWin& w) {
  const int64_t m = mw + lane_id();
  w.mw = mw;
  w.start = (m >= 0 && (uint64_t)m < a.nmsgs) ? a.in_off[m] : ~0ull;
  w.end = ~0ull;
  w.base = 0;
  w.total = 0;
  w.ok = 0;
}

// Packed bytes [A - kPre, A + kB + kPad) of the batch (zero outside it) in 16-byte pieces per
// lane: loaded into registers first (stage_load) so that other independent loads can be issued
// before the wave waits for them, then written to LDS (stage_store; d[-kPre] is byte A - kPre).
// The kPre bytes before the tile are the predecessor's last bytes: the walk through them guesses
// the tile's entry.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kPre = 64;
constexpr int kStageVecs = (kPre + kB + kPad + 1023) / 1024;
struct Staged {
  u32x4 v[kStageVecs];
};

__device__ __forceinline__ void stage_store(const Staged& sg, uint8_t* d) {
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < kStageVecs; k++) {
    const int o = 16 * (64 * k + l);
    if (o < kPre + kB + kPad) *(u32x4*)(d - kPre + o) = sg.v[k];
  }
  lane_handoff();  // other lanes read these bytes next
}

__device__ __forceinline__ void stage_load(const UnpackArgs& a, uint64_t A, Staged& sg) {
  const int l = lane_id();
  const uint64_t P = a.nbytes;
  const bool aligned = ((uintptr_t)a.packed & 15) == 0;
#pragma unroll
  for (int k = 0; k < kStageVecs; k++) {
    const int o = 16 * (64 * k + l);
    sg.v[k] = (u32x4){0, 0, 0, 0};
    if (o < kPre + kB + kPad) {
      // bytes [b, b + 16) of the batch, b = A - kPre + o (may be negative: tile 0's prefix)
      const int64_t b = (int64_t)A - kPre + o;
      u32x4 v = {0, 0, 0, 0};
      if (aligned && b >= 0 && (uint64_t)b + 16 <= P) {
        v = *(const u32x4*)(a.packed + b);
      } else {
        uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;
        for (int i = 0; i < 16; i++) {
          const bool inb = b + i >= 0 && (uint64_t)(b + i) < P;
          const uint32_t bv = inb ? (uint32_t)a.packed[b + i] : 0u;
          const uint32_t sv = bv << (8 * (i & 3));
          if (i < 4) q0 |= sv;
          else if (i < 8) q1 |= sv;
          else if (i < 12) q2 |= sv;
          else q3 |= sv;
        }
        v = (u32x4){q0, q1, q2, q3};
      }
      sg.v[k] = v;
    }
  }
}

// Message-start bitmap of tile [A, A + kB) into ms[64] (bit = tile-relative byte; the batch end
// counts as a start when it falls inside the tile).  Returns one past the last message starting
// in the tile; *nms_after = first message start at or after the tile end (tile-relative, capped
// at the batch end).  first != NULL: full windows, the first one (lane 0 = message mfirst-1)
// returned; else message starts only.
__device__ __forceinline__ uint64_t tile_msg_starts(const UnpackArgs& a, uint64_t A,
                                                    uint64_t mfirst, uint64_t* ms,
                                                    int* nms_after, MsgWin* first) {
  const int l = lane_id();
  const uint64_t P = a.nbytes;
  ms[l] = 0;
  MsgWin w2;
  // the first window is 8 entries (a tile holds a few messages; the lines of 64 entries are
  // fetched again by the tiles of other XCDs sharing them), all 64 when 7 messages start in it
  int nl = first ? 8 : 64;
  if (first) {
    load_win(a, (int64_t)mfirst - 1, w2, nl);
    *first = w2;
  } else {
    load_starts(a, (int64_t)mfirst - 1, w2);
  }
  uint64_t mlast;
  for (;;) {
    const bool in = l > 0 && l < nl && w2.start >= A && w2.start < A + kB;
    if (in) {
      const uint64_t r = w2.start - A;
      atomicOr((unsigned long long*)&ms[r >> 6], 1ull << (r & 63));
    }
    const uint64_t inm = ballot(in);
    if (inm != (nl == 64 ? (~0ull << 1) : (((1ull << nl) - 1) & ~1ull))) {
      mlast = (uint64_t)(w2.mw + 1 + __popcll(inm));
      if (nms_after) {
        // message mlast is the window lane after the last one in the tile (a missing entry
        // reads ~0): no extra round trip to in_off
        const uint64_t nx = readlane64(w2.start, (int)(mlast - (uint64_t)w2.mw));
        *nms_after = (int)((nx < P ? nx : P) - A);
      }
      break;
    }
    if (nl < 64) {  // the first window again, whole
      nl = 64;
      load_win(a, w2.mw, w2);
      *first = w2;
      continue;
    }
    // 63 starts in this window: continue with the next
    if (first) load_win(a, w2.mw + 63, w2);
    else load_starts(a, w2.mw + 63, w2);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (P - A < (uint64_t)kB) {
    const int pe = (int)(P - A);
    atomicOr((unsigned long long*)&ms[pe >> 6], 1ull << (pe & 63));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return mlast;
}

// Sub-tile geometry of this lane: [64l, 64l + 64), message starts, the first message start
// after the sub-tile (suffix minimum over the lanes).
__device__ __forceinline__ SubTile make_subtile(uint64_t A, uint64_t P, uint64_t msw,
                                                int nms_tile_after) {
  const int l = lane_id();
  SubTile st;
  st.s = 64 * l;
  st.end = st.s + 64;
  st.pend = (P - A) < (uint64_t)kDead ? (int)(P - A) : kDead;
  st.vend = st.end < st.pend ? st.end : st.pend;
  st.msw = msw;
  // the next lane holding a message start, and its first one
  const uint64_t hs = ballot(st.msw != 0);
  st.no_starts = hs == 0;
  const uint64_t above = hs & ~mask_le(l);
  const int fs = st.msw ? st.s + lowest_bit(st.msw) : 0x7fffffff;
  const int nxt = (int)shfl32((uint32_t)fs, above ? lowest_bit(above) : l);
  st.nms_after = above ? nxt : nms_tile_after;
  return st;
}

// v_perm selectors depositing the bytes that follow a tag into the word: byte i <- data byte
// rank_i when bit i of the tag is set, else 0 (the inverse of serialize-packed.c++:332-350).
__device__ __forceinline__ uint64_t make_dep(uint32_t tag) {
  uint64_t sel = 0;
  uint32_t r = 0;
  for (int i = 0; i < 8; i++) {
    const bool b = (tag >> i) & 1;
    sel |= (uint64_t)(b ? r : 0x0cu) << (8 * i);
    r += b;
  }
  return sel;
}

// ---------------------------------------------------------------------------------------------
// 3. The tile kernel: one wave per 4 KiB packed tile, four waves per workgroup, tiles in
//    workgroup order (a tile only ever waits on lower tiles, which are running or done).
//
// Tile descriptors (desc[t], zero until published).  A tile's exit is the first position of its
// chain at or past the tile end; its words are those of its records (message starts excepted,
// below).  States:
//   AGG   the tile's exit and words for its guessed entry, with that entry: the guess is where the
//         chain through the 64 bytes before the tile lands in it (chains synchronise within a
//         few records), so it needs nothing from the predecessor tile -- no wait before the AGG;
//   INCL  its true exit and the inclusive words of the message at the tile end.
// An AGG is right when its entry is where its predecessor's (right) exit leads: the look-back
// checks that on neighbouring descriptors.  A guess can be wrong (a raw run longer than the
// kPre bytes: they parse as garbage records), and a wrong AGG would hold every later tile's
// look-back until its own look-back published INCL -- tile after tile, serially, where guesses
// fail often (C4: 5 % of the tiles, 4.2 -> 19.9 ms).  So a tile also finalises its AGG from the
// entry its predecessor's base-chain exit gives (x0p[t - 1]; that chain ran the predecessor's
// whole tile, so it is wrong about as rarely as the old chain-0 guesses): right away if x0p is
// published by then, else when its look-back first has to wait anyway.  A look-back meeting a
// wrong tentative AGG waits for the final one (not for an INCL); a wrong final one, for the INCL.
// A tile holding a message start publishes INCL at once: its exit and the words after its last
// start do not depend on its entry.
// (The flat stream decode keeps the scheme its composed look-back is built on: the optimistic
// entry is where the predecessor's chain 0 leads (x0p[t - 1]), and the ok bit says the exit is the
// tile's chain-0 exit, so the next tile's optimistic entry is its true one.)
constexpr uint64_t kOkBit = 1ull << 61;
constexpr int kExitShift = 48;                       // bits 48-60: exit - kB
constexpr int kEntryShift = 35;                      // bits 35-47: an AGG's guessed entry
constexpr uint64_t kWordsMask = (1ull << kEntryShift) - 1;  // (a message of < 2^35 words)
constexpr uint32_t kExitDead = 0x1fff;               // the chain ran past the batch end

__device__ __forceinline__ uint64_t make_desc(uint64_t state, uint32_t exit, uint32_t x0,
                                              uint64_t words, uint32_t entry = 0) {
  const uint32_t e = exit >= (uint32_t)kDead ? kExitDead : exit - (uint32_t)kB;
  return state | (exit == x0 ? kOkBit : 0ull) | ((uint64_t)e << kExitShift) |
         ((uint64_t)(entry & 0x1fffu) << kEntryShift) | (words & kWordsMask);
}
__device__ __forceinline__ uint32_t desc_exit(uint64_t d) {
  const uint32_t e = (uint32_t)(d >> kExitShift) & 0x1fffu;
  return e == kExitDead ? (uint32_t)kDead : e + (uint32_t)kB;
}
__device__ __forceinline__ uint32_t desc_entry(uint64_t d) {
  return (uint32_t)(d >> kEntryShift) & 0x1fffu;
}
constexpr uint64_t kFinalBit = 1ull << 61;  // (message decode: the bit the flat decode's ok uses)
__device__ __forceinline__ uint64_t make_agg(uint32_t exit, uint64_t words, uint32_t entry,
                                             bool final) {
  return (make_desc(kDescAgg, exit, ~0u, words, entry) & ~kOkBit) | (final ? kFinalBit : 0ull);
}

// Entry of a tile from its predecessor's exit (predecessor-relative), clipped at the tile's first
// message start (every chain restarts there).
__device__ __forceinline__ uint32_t entry_from_exit(uint32_t xp, uint32_t fms) {
  const uint32_t E = xp >= (uint32_t)kDead ? (uint32_t)kB : xp - (uint32_t)kB;
  return E < fms ? E : fms;
}

// Words of the records in mask m of the sub-tile at s (a run record adds its count).
__device__ __forceinline__ uint32_t mask_words(const uint8_t* d, int s, uint64_t m, uint64_t runs) {
  uint32_t w = __popcll(m);
  uint64_t r = m & runs;
  while (r) {
    const int b = lowest_bit(r);
    r &= r - 1;
    const uint8_t* q = d + s + b;
    w += q[1 + __popc(q[0])];
  }
  return w;
}

// Chains beside chain 0 that enter_chain's jump walk follows: chain k of a sub-tile starts at
// its first byte neither chain 0 nor chains 1 .. k-1 start a record at (text parsed as records
// runs as several interleaved chains).  Stream split with the lane-0 walk capped at 48 records:
// 16.0 / 14.3 / 13.6 ms with 1 / 2 / 3 chains; capped at 16: 13.5 ms with 3, 13.3 with 4, 15.7
// with 6 (registers: C2 unpack_tiles 225 -> 257 us); 4 chains capped at 8: 13.2 ms.  The message
// decode is unchanged within noise (C2 / C4 unpack_tiles 225 / 4370 -> 220 / 4351 us).
#ifndef CPK_ENTER_CHAINS
#define CPK_ENTER_CHAINS 4
#endif
constexpr int kEnterChains = CPK_ENTER_CHAINS;
// The chain entered at tile byte E (0 < E < fms) replaces chain 0's record starts before the
// point where it meets chain 0.  Lane 0 walks it record by record (one LDS round trip per
// record) for up to kMergeCap records; a chain still running beside chain 0 then (interleaved
// chains that meet late, or never) is continued by all lanes in step, jumping along the
// sub-tiles' other chains (kEnterChains of them) where it meets one of them.  Returns
// the lane's true record-start mask; *exit is chain 0's exit when the chains meet (or the walk
// reaches the first message start, where every chain restarts), else where the entry's chain
// leaves the tile.  *runs gains the run records of the walked starts.
__device__ uint64_t enter_chain(const uint8_t* d, uint64_t* aux, const SubTile& st, uint64_t tm0,
                                int E, int fms, uint32_t x0, uint32_t* exit, uint64_t* runs) {
  const int l = lane_id();
  uint64_t* const fix = aux + 64;
  aux[l] = tm0;
  fix[l] = 0;
  lane_handoff();
  int p = E, cur = E >> 6, steps = 0;
  uint64_t fm = 0;
  bool done = true;
  if (l == 0) {
    // the reads of a step are independent (one LDS round trip per record); the walked starts of
    // a sub-tile collect in a register until the walk leaves it
    while (p < fms && p < kB && steps < kMergeCap) {
      const uint64_t mk = aux[p >> 6];
      const uint32_t le = d[p], c9 = d[p + 9];
      asm volatile("" ::"v"(le), "v"(c9));
      if ((mk >> (p & 63)) & 1) break;
      if ((p >> 6) != cur) {
        fix[cur] = fm;
        fm = 0;
        cur = p >> 6;
      }
      fm |= 1ull << (p & 63);
      p += step_len(le, c9);
      steps++;
    }
    done = steps < kMergeCap;
  }
  CPK_DIAG_ONLY(diag_add(6, 1); diag_add(7, readlane32((uint32_t)steps, 0)); diag_add(8, !readlane32(done, 0)));
  if (!readlane32(done, 0)) {
    p = (int)readlane32((uint32_t)p, 0);
    cur = (int)readlane32((uint32_t)cur, 0);
    fm = readlane64(fm, 0);
    const uint64_t vm = st.vend <= st.s ? 0ull : (st.vend >= st.s + 64 ? ~0ull
                                                                     : mask_lt(st.vend - st.s));
    // (the chains' records are clipped at the first message start after the tile, as chain 0's
    // are; each is walked until it meets chain 0 or an earlier one)
    uint64_t ch[kEnterChains];
    int xc[kEnterChains];
    uint64_t taken = tm0, left = ~tm0 & vm;
#pragma unroll
    for (int c = 0; c < kEnterChains; c++) {
      ch[c] = 0;
      xc[c] = kDead;
      if (left) xc[c] = walk(d, st, st.s + lowest_bit(left), taken, &ch[c]);
      taken |= ch[c];
      left &= ~ch[c];
    }
    for (int k = 0; k < 2 * kB && p < fms && p < kB; k++) {
      const int j = p >> 6, b = p & 63;
      if ((readlane64(tm0, j) >> b) & 1) break;
      if (j != cur) {
        if (l == 0) fix[cur] = fm;
        fm = 0;
        cur = j;
      }
      bool jumped = false;
#pragma unroll
      for (int c = 0; c < kEnterChains; c++) {
        const uint64_t Cj = readlane64(ch[c], j);
        if (!jumped && ((Cj >> b) & 1)) {
          fm |= Cj & ~mask_lt(b);
          p = (int)readlane32((uint32_t)xc[c], j);
          jumped = true;
        }
      }
      if (!jumped) {
        fm |= 1ull << b;
        p += step_len(d[p], d[p + 9]);
      }
    }
  }
  if (l == 0) fix[cur] = fm;
  p = (int)readlane32((uint32_t)p, 0);
  lane_handoff();
  const int m = p < fms ? p : fms;  // chain 0 holds from here on
  const int s = 64 * l;
  const uint64_t below = m <= s ? 0ull : (m >= s + 64 ? ~0ull : mask_lt(m - s));
  const uint64_t fl = fix[l];
  lane_handoff();
  // run records among the walked starts
  uint64_t fr = fl & ~*runs, rr = 0;
  while (fr) {
    const int b = lowest_bit(fr);
    fr &= fr - 1;
    const uint32_t tg = d[s + b];
    if (tg == 0 || tg == 0xff) rr |= 1ull << b;
  }
  *runs |= rr;
  if (p < fms && p < kB) {
    *exit = x0;  // met chain 0
  } else if (fms < kB) {
    *exit = x0;  // restarted at the first message start
  } else {
    // left the tile on its own; its last record clipped at the next message start (as walk())
    const int q = p < st.nms_after ? p : st.nms_after;
    *exit = q >= st.pend ? (uint32_t)kDead : (uint32_t)q;
  }
  return (tm0 & ~below) | fl;
}

// Entry at or past the first message start: no record before it (the predecessor's last record
// reaches past it), chain 0 from there on; an entry past the tile (the predecessor's chain ran
// past the batch end) leaves no record at all.
__device__ __forceinline__ uint64_t clip_below(uint64_t tm0, uint32_t fms, int s, uint32_t* exit) {
  if (fms >= (uint32_t)kB) *exit = (uint32_t)kDead;
  const uint64_t below = fms <= (uint32_t)s ? 0ull
                                            : (fms >= (uint32_t)s + 64 ? ~0ull : mask_lt(fms - s));
  return tm0 & ~below;
}

// Exclusive prefix of tile t -- words of the message at the tile start before this tile -- and
// (*xprev) the true exit of tile t - 1, from the descriptors of tiles t - 1, t - 2, ...: up to the
// nearest INCL, every AGG on the way must be right -- its entry the one its predecessor's exit
// (as published, and itself right) leads to.  The farthest AGG that is not makes every nearer one
// wrong: the wave waits for that tile to publish its final AGG (if this one was its guess) or its
// INCL, and starts over.  Waits are only ever for lower tiles; before its first wait the wave runs
// on_wait (the tile finalises its own AGG).  The first window of each pass is 16 tiles (one
// 128-byte line of descriptors: the nearest INCL is usually a few tiles back, and these
// agent-scope reads go past the L2), later ones 64.
template <class OnWait>
__device__ uint64_t lookback_tiles(const UnpackArgs& a, uint64_t t, uint32_t* xprev,
                                   OnWait on_wait) {
  const int l = lane_id();
  int64_t base = (int64_t)t - 1;  // nearest tile of the window
  uint64_t acc = 0;
  uint32_t xfirst = (uint32_t)kB;
  uint32_t spins = 0;
  int width = 16;
  uint64_t carry = 0;  // descriptor of the previous window's farthest tile (an AGG) to check
  bool has_carry = false;
  for (;;) {
    const int64_t idx = base - l;
    const bool in = l < width;
    CPK_DIAG_ONLY(diag_add(22, 1); const uint64_t lt0 = wall_clock64());
    // before tile 0: an inclusive zero whose exit enters tile 0 at byte 0
    const uint64_t dv = !in ? 0ull : (idx >= 0 ? load_agent(a.desc + idx) : kDescIncl);
#ifdef CPK_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (width == 16) diag_add(15, wall_clock64() - lt0);  // the first window's read, 10 ns ticks
#endif
    const uint64_t stt = dv & kDescFlags;
    const uint64_t sb = ballot(in && stt == kDescIncl);
    const int k = sb ? lowest_bit(sb) : 64;
    const uint64_t nb = ballot(in && stt == 0);
    const int nl = nb ? lowest_bit(nb) : 64;
    const uint64_t* wait_on = nullptr;
    int want = 0;  // 0: published, 1: final AGG or INCL, 2: INCL
    if (nl < k) {
      wait_on = a.desc + (base - nl);
    } else {
      const int kk = k < width ? k : width - 1;
      // entry each tile's predecessor (the next lane) leads to; an AGG tile has no message start
      const uint32_t ent = entry_from_exit(desc_exit(dv), (uint32_t)kB);
      const uint32_t pent = shfl32(ent, l + 1 < 64 ? l + 1 : 63);
      const uint64_t fb = ballot(l < kk && desc_entry(dv) != pent);
      if (has_carry && desc_entry(carry) != readlane32(ent, 0)) {
        wait_on = a.desc + (base + 1);
        want = (carry & kFinalBit) ? 2 : 1;
      } else if (fb) {
        const int j = highest_bit(fb);
        wait_on = a.desc + (base - j);
        want = (readlane64(dv, j) & kFinalBit) ? 2 : 1;
      } else {
        if (base == (int64_t)t - 1) xfirst = desc_exit(readlane64(dv, 0));
        acc += wave_sum64(l <= kk ? (dv & kWordsMask) : 0ull);
        if (k < width) break;
        carry = readlane64(dv, width - 1);
        has_carry = true;
        base -= width;
        width = 64;
        continue;
      }
    }
    on_wait();
    // one lane polls the blocking descriptor (sleeping between polls), then the window is read
    // again from the nearest tile (after a wrong AGG, from tile t - 1)
    CPK_DIAG_ONLY(diag_add(want ? 24 : 23, 1); const uint32_t sp0 = uniform32(spins));
    if (l == 0) {
      for (;;) {
        const uint64_t v = load_agent(wait_on);
        const uint64_t f = v & kDescFlags;
        if (want == 0 ? f != 0 : (f == kDescIncl || (want == 1 && (v & kFinalBit)))) break;
        if (++spins >= kSpinLimit) break;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    spins = uniform32(spins);
    CPK_DIAG_ONLY(diag_add(25, spins - sp0));
    if (spins >= kSpinLimit) {
      raise_error(a.err, kErrInternal);
      break;
    }
    if (want) {
      base = (int64_t)t - 1;
      acc = 0;
      width = 16;
      has_carry = false;
    }
  }
  *xprev = xfirst;
  return acc;
}

// Flat stream decode (the stream split): each tile t also publishes desc2[t], its exit and words
// for a second candidate entry -- the one the predecessor's AGG exit gives, when that is not the
// optimistic one (a predecessor without the ok bit: its chain-0 exit, which the optimistic entry
// came from, is then likely not its true exit, and its AGG exit is, when its own entry was
// right).  desc2: 0 until published; kD2None: no second candidate; else AGG | ok | exit (as
// desc) | the candidate entry (bits 21-33) | the tile's words (bits 0-20: at most 4096 records
// of at most 256 words).
constexpr uint64_t kD2None = 1;
constexpr int kD2EntryShift = 21;
constexpr uint64_t kD2WordsMask = (1ull << kD2EntryShift) - 1;

__device__ __forceinline__ uint64_t wait_nonzero64(const uint64_t* p, uint32_t* err) {
  uint64_t v = 0;
  if (lane_id() == 0) {
    for (uint32_t i = 0; i < kSpinLimit; i++) {
      v = load_agent(p);
      if (v) break;
      __builtin_amdgcn_s_sleep(1);
    }
    if (!v) raise_error(err, kErrInternal);
  }
  return readlane64(v, 0);
}

constexpr int kFlatWindows = 16;

// Flat look-back by composition.  A tile's true entry is one of two candidates
// when the look-back can resolve it: a (E1, the entry the predecessor's chain-0 exit gives: the
// tile's AGG holds its exit and words) or b (E2, its desc2 candidate).  So each tile is a transfer
// function from {a, b} to the state its exit gives the next tile ({a, b} or fail) plus words, and
// runs of tiles compose: a wave composes a window of 64 tiles in six shuffle steps, windows compose
// in turn, and the look-back reads window after window until an INCL -- the serial resolution (one
// lane step per tile) and its one-window limit (no INCL within 64 tiles: wait for the INCL 64
// back, so the INCL frontier moved 64 tiles per hop) are gone.  A tile whose entry matches neither
// candidate is waited for (its INCL; rare: 0.3 % of the tiles of the bench stream).
__device__ __forceinline__ uint32_t flat_cls(uint32_t E, uint32_t E1, uint32_t E2, uint32_t v2) {
  return E == E1 ? 0u : ((v2 && E == E2) ? 1u : 2u);
}
__device__ __forceinline__ uint32_t flat_entry(uint32_t x) {
  return x >= (uint32_t)kDead ? (uint32_t)kB : x - (uint32_t)kB;
}
// one lane polls p until (value & mask) == want (want 0: until non-zero); false: spin limit
__device__ bool flat_wait(const uint64_t* p, uint64_t mask, uint64_t want, uint32_t* spins,
                          uint32_t* err) {
  if (lane_id() == 0) {
    for (;;) {
      const uint64_t v = load_agent(p);
      if (want ? (v & mask) == want : v != 0) break;
      if (++*spins >= kSpinLimit) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  *spins = uniform32(*spins);
  if (*spins >= kSpinLimit) {
    raise_error(err, kErrInternal);
    return false;
  }
  return true;
}

// PUB: every tile's AGG, second candidate and chain-0 exit are published before the launch (the
// split flat decode's second launch): a window's three reads go out together, the last two as
// plain loads (nothing changes them during the launch), one round trip per window instead of two.
template <bool PUB>
__device__ uint64_t lookback_flat_scan(const UnpackArgs& a, uint64_t t, uint32_t* xprev) {
  const int l = lane_id();
  uint32_t spins = 0;
  for (;;) {  // (a pass; a wait starts the next -- and counts against the spin limit, so a
              // wait that makes no progress cannot loop for ever)
    if (++spins >= kSpinLimit) {
      raise_error(a.err, kErrInternal);
      *xprev = (uint32_t)kB;
      return 0;
    }
    // composite of the windows read so far, nearest first: far-edge state -> tile t-1's exit
    // (a: its AGG exit, b: its desc2 exit)
    uint32_t Gs[2] = {0u, 1u};
    uint64_t Gw[2] = {0, 0};
    uint32_t c1 = 0, c2 = 0, cv = 0;  // the nearer window's far tile's candidates
    uint32_t exA0 = 0, exB0 = 0;
    const uint64_t* wait_p = nullptr;
    uint64_t wait_mask = 0, wait_want = 0;
    int w = 0;
    while (w < kFlatWindows) {
      const int64_t base = (int64_t)t - 1 - 64 * w;
      const int64_t u = base - l;
      // before tile 0: an inclusive zero whose exit enters tile 0 at byte 0
      const uint64_t dv = u >= 0 ? load_agent(a.desc + u) : (kDescIncl | kOkBit);
      uint64_t d2p = kD2None;
      uint32_t xqp = 0;
      if (PUB) {
        d2p = u >= 0 ? a.desc2[u] : kD2None;
        xqp = u >= 1 ? a.x0p[u - 1] : 0u;
      }
      const uint64_t stt = dv & kDescFlags;
      const uint64_t ib = ballot(stt == kDescIncl);
      const int k = ib ? lowest_bit(ib) : 64;
      const uint64_t nb = ballot(l < k && stt == 0);
      if (nb) {  // a descriptor not published yet: wait for it, then read this window again
        CPK_DIAG_ONLY(diag_add(27, 1));
        if (!flat_wait(a.desc + (base - lowest_bit(nb)), 0, 0, &spins, a.err)) break;
        continue;
      }
      const bool agg = l < k;  // (AGG: published, not INCL)
      const uint64_t d2 = agg ? (PUB ? d2p : load_agent(a.desc2 + u)) : kD2None;
      const uint32_t xq = agg ? ((PUB ? xqp : load_agent32(a.x0p + u - 1)) & 0x7fffffffu) : 0u;
      const uint64_t n2 = ballot(agg && d2 == 0);
      if (n2) {
        CPK_DIAG_ONLY(diag_add(27, 1));
        if (!flat_wait(a.desc2 + (base - lowest_bit(n2)), 0, 0, &spins, a.err)) break;
        continue;
      }
      const uint32_t E1 = flat_entry(xq);
      const uint32_t v2 = (agg && d2 != kD2None) ? 1u : 0u;
      const uint32_t E2 = v2 ? (uint32_t)((d2 >> kD2EntryShift) & 0x1fffu) : 0u;
      const uint32_t exA = desc_exit(dv), exB = v2 ? desc_exit(d2) : exA;
      // the successor's candidates: lane l - 1's; lane 0: the nearer window's far tile's, or in
      // window 0 (successor: tile t) the exits themselves, so the state says which exit
      const int ps = l > 0 ? l - 1 : 0;
      uint32_t sE1 = shfl32(E1, ps), sE2 = shfl32(E2, ps), sv = shfl32(v2, ps);
      if (l == 0) {
        sE1 = w == 0 ? flat_entry(exA) : c1;
        sE2 = w == 0 ? flat_entry(exB) : c2;
        sv = w == 0 ? v2 : cv;
      }
      if (w == 0) {
        exA0 = readlane32(exA, 0);
        exB0 = readlane32(exB, 0);
      }
      // the lane's transfer function (lanes >= k: not composed)
      const uint32_t fa = flat_cls(flat_entry(exA), sE1, sE2, sv);
      const uint32_t fb = v2 ? flat_cls(flat_entry(exB), sE1, sE2, sv) : 2u;
      const uint32_t fwa = (uint32_t)(dv & kWordsMask), fwb = (uint32_t)(d2 & kD2WordsMask);
      uint32_t sa = fa, sb = fb, wa = fwa, wb = fwb;
      // compose lanes [0, k): lane l ends with tiles l .. k-1 (the predecessor side applied first)
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int q = l + o < 64 ? l + o : 63;
        const uint32_t psa = shfl32(sa, q), psb = shfl32(sb, q);
        const uint32_t pwa = shfl32(wa, q), pwb = shfl32(wb, q);
        if (l + o < k) {
          const uint32_t na = psa == 2u ? 2u : (psa == 0u ? sa : sb);
          const uint32_t nwa = pwa + (psa == 0u ? wa : wb);
          const uint32_t nb2 = psb == 2u ? 2u : (psb == 0u ? sa : sb);
          const uint32_t nwb = pwb + (psb == 0u ? wa : wb);
          sa = na;
          wa = nwa;
          sb = nb2;
          wb = nwb;
        }
      }
      const uint32_t Fs[2] = {k ? readlane32(sa, 0) : 0u, k ? readlane32(sb, 0) : 1u};
      const uint32_t Fw[2] = {k ? readlane32(wa, 0) : 0u, k ? readlane32(wb, 0) : 0u};
      if (k < 64) {
        const uint64_t dk = readlane64(dv, k);
        if (k == 0 && w == 0) {  // tile t - 1 holds an INCL
          *xprev = desc_exit(dk);
          return dk & kWordsMask;
        }
        // the INCL's exit in the states of the tile after it
        const uint32_t kE1 = k ? readlane32(E1, k - 1) : c1;
        const uint32_t kE2 = k ? readlane32(E2, k - 1) : c2;
        const uint32_t kv = k ? readlane32(v2, k - 1) : cv;
        const uint32_t s0 = flat_cls(flat_entry(desc_exit(dk)), kE1, kE2, kv);
        const uint32_t s1 = s0 == 2u ? 2u : Fs[s0];
        const uint32_t s2 = s1 == 2u ? 2u : Gs[s1];
        if (s2 != 2u) {
          CPK_DIAG_ONLY(diag_add(29, w + 1));
          *xprev = s2 == 0u ? exA0 : exB0;
          return (dk & kWordsMask) + Fw[s0] + Gw[s1];
        }
        // an entry that matches neither candidate: wait for that tile's INCL
        if (s0 == 2u) {
          wait_p = a.desc + (k ? base - (k - 1) : base + 1);  // (the tile after the INCL)
        } else if (s1 == 2u) {
          // in this window: the state entering lane l is lane l + 1's composite applied to s0
          const int q = l + 1 < 64 ? l + 1 : 63;
          const uint32_t qa = shfl32(sa, q), qb = shfl32(sb, q);
          const uint32_t in = l + 1 >= k ? s0 : (s0 == 2u ? 2u : (s0 == 0u ? qa : qb));
          const uint32_t out = in == 2u ? 2u : (in == 0u ? fa : fb);
          const uint64_t fl = ballot(l < k && in != 2u && out == 2u);
          wait_p = a.desc + (base - (fl ? highest_bit(fl) : 0));
        } else {
          wait_p = a.desc + (base + 1);  // (in a nearer window: its far tile)
        }
        wait_mask = kDescFlags;
        wait_want = kDescIncl;
        break;
      }
      // no INCL in this window: G := G after F; this window's far tile's candidates carry over
      uint32_t ns[2];
      uint64_t nw[2];
#pragma unroll
      for (int s = 0; s < 2; s++) {
        ns[s] = Fs[s] == 2u ? 2u : Gs[Fs[s]];
        nw[s] = Fw[s] + (Fs[s] == 2u ? 0ull : Gw[Fs[s]]);
      }
      Gs[0] = ns[0];
      Gs[1] = ns[1];
      Gw[0] = nw[0];
      Gw[1] = nw[1];
      c1 = readlane32(E1, 63);
      c2 = readlane32(E2, 63);
      cv = readlane32(v2, 63);
      w++;
    }
    if (!wait_p) {  // no INCL within kFlatWindows windows: the farthest tile read
      wait_p = a.desc + ((int64_t)t - 64 * kFlatWindows);
      wait_mask = kDescFlags;
      wait_want = kDescIncl;
    }
    CPK_DIAG_ONLY(diag_add(26, 1); diag_add(28, w));
    if (spins >= kSpinLimit || !flat_wait(wait_p, wait_mask, wait_want, &spins, a.err)) {
      *xprev = (uint32_t)kB;
      return 0;
    }
  }
}

// General expansion (any batch the lean path below does not take: modes 1 and 2, messages beyond
// the 64-entry window, rejected headers, output too small, empty messages): one lane per record,
// record positions by binary search over the lane masks, each record's message from the window,
// every record through handle_record (the reference's checks in the reference's order).  Kept out
// of line: its registers are not the lean path's.
__device__ __forceinline__ void expand_general(uint64_t A, const uint8_t* d,
                                                         uint32_t lut, uint64_t tm, uint64_t excl,
                                                         MsgWin win, uint64_t mfirst,
                                                         uint64_t msw) {
  const UnpackArgs& a = kua();  // (the kernel's arguments stay in the kernarg segment)
  const int l = lane_id();
  const uint32_t cnt_all = __popcll(tm);
  const uint32_t Rall_incl = wave_incl_sum32(cnt_all);
  const uint32_t nrec = readlane32(Rall_incl, 63);
  const uint32_t R = Rall_incl - cnt_all;
  int64_t mcur = (int64_t)mfirst - 1;
  uint64_t nxt_start = readlane64(win.start, 1);
  uint64_t sum = 0;
  uint32_t base_key = 0;
  for (uint32_t b0 = 0; b0 < nrec; b0 += 64) {
    const uint32_t r = b0 + l;
    const bool act = r < nrec;
    const uint32_t rq = act ? r : 0;
    // record position: lane j holding record r, then the (r - R_j)-th set bit of its mask
    int j = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1) {
      const int c = j + step;
      const uint32_t Rc = shfl32(R, c <= 63 ? c : 63);
      if (c <= 63 && Rc <= rq) j = c;
    }
    const uint32_t Rj = shfl32(R, j);
    uint64_t mj = shfl64(tm, j);
    int k = (int)(rq - Rj), pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
      const uint64_t low = mj & ((1ull << w) - 1);
      const int c = __popcll(low);
      if (k >= c) {
        k -= c;
        mj >>= w;
        pos += w;
      } else {
        mj = low;
      }
    }
    const int p = act ? 64 * j + pos : 0;
    const uint64_t pabs = A + p;
    const Rec rc = read_rec(d, p);
    const uint32_t w = act ? 1 + rc.cnt : 0;
    // every lane takes part in the shuffle (an inactive source lane would read as 0)
    const uint64_t msrc = shfl64(msw, p >> 6);
    const bool is_ms = act && ((msrc >> (p & 63)) & 1);
    const uint32_t inc = wave_incl_sum32(w);
    const uint64_t Sx = sum + inc - w;
    const uint32_t key = is_ms ? (uint32_t)(Sx + 1) : 0;
    uint32_t km = wave_incl_max32(key);
    if (km < base_key) km = base_key;
    const uint64_t wb = km ? Sx - (km - 1) : excl + Sx;
    const uint32_t lastl = (nrec - b0 < 64 ? nrec - b0 : 64) - 1;
    const uint64_t maxp = readlane64(pabs, (int)lastl);
    int64_t m = mcur;
    if (maxp >= nxt_start) {
      bool found = false;
      for (;;) {
        int c = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1) {
          const uint64_t probe = shfl64(win.start, c + step <= 63 ? c + step : 63);
          if (c + step <= 63 && probe <= pabs) c += step;
        }
        const bool beyond = act && c == 63 && readlane64(win.start, 63) <= pabs;
        if (!found && !beyond) m = win.mw + c;
        found = found || !beyond;
        if (!ballot(beyond)) break;
        load_win(a, win.mw + 63, win);
      }
      mcur = (int64_t)readlane64((uint64_t)m, (int)lastl);
      if (mcur - win.mw >= 63) load_win(a, mcur, win);
      nxt_start = readlane64(win.start, (int)(mcur - win.mw) + 1);
    }
    const int64_t wl64 = m - win.mw;
    const bool inwin = wl64 >= 0 && wl64 < 64;
    const int wl = inwin ? (int)wl64 : 0;
    MsgInfo mi;
    mi.base = shfl64(win.base, wl);
    mi.total = shfl64(win.total, wl);
    mi.end = shfl64(win.end, wl);
    mi.ok = shfl32(win.ok, wl) != 0;
    if (!inwin && act && m >= 0 && (uint64_t)m < a.nmsgs) mi = msg_info(a, (uint64_t)m);
    mi.fits = a.word_off ? (mi.base + mi.total <= a.words_capacity) : false;
    const uint64_t word = expand_word(d, p, rc.tag, lut);
    RunJob job;
    job.n = 0;
    if (act && m >= 0 && (uint64_t)m < a.nmsgs) {
      const int32_t st = handle_record(a, d, p, pabs, wb, mi, &job, word);
      if (a.mode == 2) {
        if (mi.ok) {
          if (st == kInvalid) {
            a.status[m] = kInvalid;
            a.size_out[m] = 0;
          } else if (st == kSizeDone) {
            a.status[m] = kOK;
            a.size_out[m] = wb + 1 + (rc.run ? rc.cnt : 0);
          }
        }
      } else if (st >= 0) {
        a.status[m] = st;
        report_end(a, (uint64_t)m, st, job);
      }
    }
    run_jobs_batch(a, job, d, A, (uint32_t)(kB + kPad));
    base_key = readlane32(km, 63);
    sum += readlane32(inc, 63);
  }
}

// A record that ends or breaks its message in the lean expansion: the reference's checks
// (handle_record), its status and end, and its run (out of line: rare).
__device__ __forceinline__ void lean_special(const uint8_t* d, int p, uint64_t A,
                                                       uint64_t wb, uint64_t mbase,
                                                       uint64_t mtotal, uint64_t mend, int64_t m,
                                                       uint64_t word, bool act) {
  const UnpackArgs& a = kua();
  RunJob job;
  job.n = 0;
  if (act) {
    MsgInfo mi;
    mi.base = mbase;
    mi.total = mtotal;
    mi.end = mend;
    mi.ok = true;
    mi.fits = true;
    const int32_t st = handle_record(a, d, p, A + (uint32_t)p, wb, mi, &job, word);
    if (st >= 0) {
      kua().status[m] = st;
      report_end(a, (uint64_t)m, st, job);
    }
  }
  run_jobs(a, job, d, A, (uint32_t)(kB + kPad));
}

// A record that ends its message exactly -- its last word the message's last, its last byte the
// message's last -- is the reference's clean end (handle_record: kOK, the header launch's status
// stands): the lean batch writes it like any other record.  Not when the call reports where each
// message ends (in_end), nor for a raw run whose bytes leave the staged ones (handle_record writes
// such a run whole: the next tile's run_tail skips runs that end a message).
__device__ __forceinline__ bool clean_end(const UnpackArgs& a, bool words_end, bool bytes_end,
                                          bool raw, uint32_t rb, uint32_t cnt) {
  return words_end && bytes_end && !a.in_end && (!raw || rb + 8u * cnt + 4u <= (uint32_t)(kB + kPad));
}

// Lean expansion (mode 0; every message touching the tile in the window, accepted, fitting the
// output; no empty message in the tile; at most kB/8 records per quarter tile).  Record lists
// per quarter tile in LDS, one lane per record, 64 consecutive records per batch, coalesced
// 8-byte stores.  Tile-relative 32-bit arithmetic; the current message's word pointer is
// wave-uniform.  A batch with no message start whose records cannot reach the message's end --
// by words or by bytes (a record is at most 2050 bytes): one uniform check -- runs with no
// per-record message logic; the records of other batches find their message by the start bits
// and a max-scan, and those that end or break their message go through handle_record.  The
// first word of every zero or raw run is written by the record's own lane with the record (most
// runs of dense data are one word); the rest of a run by the whole wave.
__device__ __forceinline__ void expand_lean(const UnpackArgs& a, uint64_t A, const uint8_t* d,
                                            uint64_t* aux, const uint64_t* dep_tab, uint64_t tm,
                                            uint64_t excl, const MsgWin& win, uint64_t msw) {
  const int l = lane_id();
  // No vector load of the phases before is outstanding here (the look-back's were all used).  An
  // explicit vmcnt(0) tells the compiler so: without it, it waits for vmcnt(0) -- which on gfx950
  // counts stores too, so every store of the expansion so far -- before the loops below reuse
  // such a load's register, once per record batch.
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0); expcnt, lgkmcnt not waited
  const bool starts = ballot(msw != 0) != 0;
  // 16 record-start (and message-start) bits per lane and quarter: u16 number 64h + l of the
  // sub-tile masks is bits [16(l % 4), +16) of sub-tile 16h + l/4, i.e. tile bytes 1024h + 16l..
  aux[l] = tm;
  aux[64 + l] = msw;
  lane_handoff();
  // (two quarters per register: an array indexed by the quarter would live in scratch)
  const uint16_t* const a16 = (const uint16_t*)aux;
  const uint32_t tq01 = a16[l] | ((uint32_t)a16[64 + l] << 16);
  const uint32_t tq23 = a16[128 + l] | ((uint32_t)a16[192 + l] << 16);
  const uint32_t mq01 = a16[256 + l] | ((uint32_t)a16[320 + l] << 16);
  const uint32_t mq23 = a16[384 + l] | ((uint32_t)a16[448 + l] << 16);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the lists overwrite aux)
  uint16_t* const list = (uint16_t*)aux;
  uint32_t mcount = 0;  // message starts so far
  // the current message (window lane mcount) and its words before the next batch
  uint64_t cbase = readlane64(win.base, 0), ctot = readlane64(win.total, 0);
  uint64_t cend = readlane64(win.end, 0);
  uint64_t mw0 = excl;
  const uint32_t* const d32 = (const uint32_t*)d;
  constexpr uint32_t kStaged = (uint32_t)(kB + kPad);
  for (int h = 0; h < ((a.debug_skip & 32) ? 0 : 4); h++) {
    const uint32_t hs = 16u * ((uint32_t)h & 1u);
    uint32_t bits = ((h < 2 ? tq01 : tq23) >> hs) & 0xffffu;
    const uint32_t c = __popc(bits);
    const uint32_t Rin = wave_incl_sum32(c);
    const uint32_t nh = readlane32(Rin, 63);
    const uint32_t pbase = 1024u * (uint32_t)h + 16u * (uint32_t)l;
    uint16_t* lp = list + (Rin - c);
    if (starts) {
      // (the message-start flag in bit 12 of each entry)
      const uint32_t msp = ((h < 2 ? mq01 : mq23) >> hs) & 0xffffu;
      while (bits) {
        const uint32_t b = (uint32_t)__builtin_ctz(bits);
        bits &= bits - 1;
        *lp++ = (uint16_t)((pbase + b) | (((msp >> b) & 1u) << 12));
      }
    } else {
      while (bits) {
        const uint32_t b = (uint32_t)__builtin_ctz(bits);
        bits &= bits - 1;
        *lp++ = (uint16_t)(pbase + b);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (uint32_t b0 = 0; b0 < ((a.debug_skip & 16) ? 0u : nh); b0 += 64) {
      const uint32_t rr = b0 + l;
      const bool act = rr < nh;
      // branch-free body: an inactive lane reads the last entry again (LDS stays in bounds) and
      // is masked by selects
      const uint32_t e = list[act ? rr : nh - 1];
      const uint32_t p = e & 0xfffu;
      const bool is_ms = act && (e & 0x1000u);
      // bytes p .. p + 12: tag, up to 8 data bytes, count byte
      const uint32_t q = p >> 2, sh = p & 3u;
      const uint32_t q0 = d32[q], q1 = d32[q + 1], q2 = d32[q + 2], q3 = d32[q + 3];
      const uint32_t rb = p + 10u;  // a raw run's first word: bytes p + 10 .. p + 17
      const uint32_t b0w = __builtin_amdgcn_alignbyte(q1, q0, sh);  // bytes p .. p+3
      const uint32_t b1w = __builtin_amdgcn_alignbyte(q2, q1, sh);  // p+4 .. p+7
      const uint32_t b2w = __builtin_amdgcn_alignbyte(q3, q2, sh);  // p+8 .. p+11
      const uint32_t tag = b0w & 0xffu;
      const uint64_t sel = dep_tab[tag];
      const uint32_t dlo = __builtin_amdgcn_alignbyte(b1w, b0w, 1);  // data bytes 0..3
      const uint32_t dhi = __builtin_amdgcn_alignbyte(b2w, b1w, 1);  // data bytes 4..7
      const bool z = tag == 0, f = tag == 0xffu;
      uint32_t cnt = z ? ((b0w >> 8) & 0xffu) : 0u;
      cnt = f ? ((b2w >> 8) & 0xffu) : cnt;
      const uint32_t w = act ? 1u + cnt : 0u;
      // words of the batch before the record: a batch of single-word records (no run) needs no
      // scan -- the active lanes are a prefix
      const uint64_t runs = ballot(act && cnt != 0);
      uint32_t o = (uint32_t)l, btot = (uint32_t)__popcll(ballot(act));
      if (runs) {
        const uint32_t inc = wave_incl_sum32(w);
        o = inc - w;
        btot = readlane32(inc, 63);
      }
      const uint64_t msb = ballot(is_ms);
      const uint32_t wlo = __builtin_amdgcn_perm(dhi, dlo, (uint32_t)sel);
      const uint32_t whi = __builtin_amdgcn_perm(dhi, dlo, (uint32_t)(sel >> 32));
      const uint64_t word = ((uint64_t)whi << 32) | wlo;
      // a raw run's first word (only a batch with a raw run of words reads it)
      uint64_t rw = 0;
      if (ballot(f && cnt != 0)) {
        const uint32_t rq = rb >> 2, rs = rb & 3u;
        const uint32_t rqc = rq < kStaged / 4 - 2 ? rq : kStaged / 4 - 3;
        const uint32_t r0 = d32[rqc], r1 = d32[rqc + 1], r2 = d32[rqc + 2];
        rw = f ? (((uint64_t)__builtin_amdgcn_alignbyte(r2, r1, rs) << 32) |
                  __builtin_amdgcn_alignbyte(r1, r0, rs))
               : 0ull;
      }
      // the run's first word is in the staged bytes (always for a zero run)
      const bool inl = !f || rb + 12u <= kStaged;  // (its three dwords unclamped)
      uint64_t* wp;  // the record's word
      bool special = false;
      int wl = (int)mcount;
      uint64_t wb = 0;
      uint32_t kml = 0;
      if (msb == 0) {
        // the batch continues the current message: a uniform word pointer
        wp = a.words + (cbase + mw0) + o;
        const uint32_t maxp = readlane32(p, 63);  // (inactive lanes repeat the last record)
        if (mw0 + btot >= ctot || A + maxp + 2050 >= cend) {
          const uint32_t len = 1u + __popc(tag) + ((z || f) ? 1u : 0u) + (f ? 8u * cnt : 0u);
          wb = mw0 + o;
          special = act && (wb + w >= ctot || A + p + len >= cend) &&
                    !clean_end(a, wb + w == ctot, A + p + len == cend, f, rb, cnt);
        }
      } else {
        // message starts in the batch: the latest start at or before each record (key-max scan)
        const uint32_t key = is_ms ? o + 1u : 0u;
        const uint32_t km = wave_incl_max32(key);
        kml = readlane32(km, 63);
        wl = (int)(mcount + (uint32_t)__popcll(msb & mask_le(l)));
        const uint64_t mbase = shfl64(win.base, wl);
        wb = km ? (uint64_t)(o - (km - 1u)) : mw0 + o;
        wp = a.words + mbase + wb;
        const uint64_t mtot = shfl64(win.total, wl), mend = shfl64(win.end, wl);
        const uint32_t len = 1u + __popc(tag) + ((z || f) ? 1u : 0u) + (f ? 8u * cnt : 0u);
        special = act && (wb + w >= mtot || A + p + len >= mend) &&
                  !clean_end(a, wb + w == mtot, A + p + len == mend, f, rb, cnt);
      }
      const bool put = act && !special;
      if (put) {
        wp[0] = word;
        if (cnt != 0 && inl) wp[1] = rw;
        if (a.rec_pos) a.rec_pos[wp - a.words] = (A + p) | (*a.rec_gen << kRecGenShift);
      }
      if (ballot(special)) {
        const uint64_t mbase = msb ? shfl64(win.base, wl) : cbase;
        const uint64_t mtot = msb ? shfl64(win.total, wl) : ctot;
        const uint64_t mend = msb ? shfl64(win.end, wl) : cend;
        lean_special(d, (int)p, A, wb, mbase, mtot, mend, win.mw + wl, word, special);
      }
      // the rest of the runs (the words after the first, or a raw run whose first word is past
      // the staged bytes): the whole wave per run, from the staged bytes when they hold it
      uint64_t lm = ballot(put && (cnt > 1u || (cnt != 0 && !inl)));
      while (lm) {
        const int j = lowest_bit(lm);
        lm &= lm - 1;
        const uint32_t k0 = readlane32(inl ? 1u : 0u, j);
        const uint32_t nj = readlane32(cnt, j);
        uint64_t* const dst = (uint64_t*)readlane64((uint64_t)(wp + 1), j);
        const uint32_t sj = readlane32(rb, j);
        if (!readlane32(f ? 1u : 0u, j)) {
          for (uint32_t k = k0 + l; k < nj; k += 64) dst[k] = 0;
        } else if (sj + 8u * nj + 4u <= kStaged) {
          for (uint32_t k = k0 + l; k < nj; k += 64) {
            const uint32_t ob = sj + 8u * k, qq = ob >> 2, s3 = ob & 3u;
            const uint32_t x0 = d32[qq], x1 = d32[qq + 1], x2 = d32[qq + 2];
            dst[k] = ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, s3) << 32) |
                     __builtin_amdgcn_alignbyte(x1, x0, s3);
          }
        } else {
          // a raw run leaving the staged bytes: its words whose bytes are staged (ending at most
          // kRunSplit bytes into the next tile) from LDS; the rest the next tile writes from its
          // own staged bytes (run_tail) -- this record neither ends nor breaks its message
          const uint32_t kin = sj + 12u <= kStaged ? (kStaged - 4u - sj) / 8u : 0u;
          const uint32_t ke = nj < kin ? nj : kin;
          for (uint32_t k = k0 + l; k < ke; k += 64) {
            const uint32_t ob = sj + 8u * k, qq = ob >> 2, s3 = ob & 3u;
            const uint32_t x0 = d32[qq], x1 = d32[qq + 1], x2 = d32[qq + 2];
            dst[k] = ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, s3) << 32) |
                     __builtin_amdgcn_alignbyte(x1, x0, s3);
          }
        }
      }
      if (msb == 0) {
        mw0 += btot;
      } else {
        mcount += (uint32_t)__popcll(msb);
        mw0 = btot - (kml - 1u);
        cbase = readlane64(win.base, (int)mcount);
        ctot = readlane64(win.total, (int)mcount);
        cend = readlane64(win.end, (int)mcount);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// The words of the raw run this tile's entry E lies behind (the predecessor's last record, a
// raw run when E > kRunSplit) that end more than kRunSplit bytes into the tile: the predecessor
// left them (lean expansion) or wrote them too (same values).  Not for a run that ends or breaks
// its message, whose record handle_record writes whole, nor for a message the lean path would
// not take (header refused, output too small).
__device__ __forceinline__ void run_tail(const UnpackArgs& a, uint64_t A, const uint8_t* d,
                                         uint32_t E, uint64_t excl, const MsgWin& win) {
  const int l = lane_id();
  const uint64_t mbase = readlane64(win.base, 0), mtot = readlane64(win.total, 0);
  const uint64_t mend = readlane64(win.end, 0);
  const uint32_t n = (E - kRunSplit + 7u) / 8u;  // words ending past byte kRunSplit
  if (!readlane32(win.ok, 0) || mbase + mtot > a.words_capacity || excl >= mtot ||
      A + E >= mend || excl < n)
    return;
  const uint32_t* const d32 = (const uint32_t*)d;
  for (uint32_t j = (uint32_t)l; j < n; j += 64) {
    const uint32_t ob = E - 8u * j - 8u, qq = ob >> 2, s3 = ob & 3u;  // bytes [ob, ob + 8)
    const uint32_t x0 = d32[qq], x1 = d32[qq + 1], x2 = d32[qq + 2];
    a.words[mbase + excl - 1u - j] = ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, s3) << 32) |
                                     __builtin_amdgcn_alignbyte(x1, x0, s3);
  }
}

// Expansion of a tile in the middle of a message: no message start in the tile, and neither the
// words of its records nor their bytes can reach the message's end (most tiles of long
// messages).  Then no record can end or break its message, and the record batches need none of
// expand_lean's per-record message logic: one wave-uniform word pointer, one store per record, the
// runs' other words by the wave.  (Same stores as expand_lean for such a tile.)
// FLAT (the split flat decode): each record's packed byte goes to the record-head map too, and a
// raw run leaving the staged bytes is written whole here (its far words from global memory: the
// flat decode has no run_tail).
template <bool FLAT>
__device__ __forceinline__ void expand_simple(const UnpackArgs& a, uint64_t A, const uint8_t* d,
                                              uint64_t* aux, const uint64_t* dep_tab, uint64_t tm,
                                              uint64_t* wp, uint64_t* rp, uint64_t gen_tag) {
  const int l = lane_id();
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): as expand_lean
  aux[l] = tm;
  lane_handoff();
  const uint16_t* const a16 = (const uint16_t*)aux;
  const uint32_t tq01 = a16[l] | ((uint32_t)a16[64 + l] << 16);
  const uint32_t tq23 = a16[128 + l] | ((uint32_t)a16[192 + l] << 16);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the lists overwrite aux)
  uint16_t* const list = (uint16_t*)aux;
  const uint32_t* const d32 = (const uint32_t*)d;
  constexpr uint32_t kStaged = (uint32_t)(kB + kPad);
  for (int h = 0; h < 4; h++) {
    const uint32_t hs = 16u * ((uint32_t)h & 1u);
    uint32_t bits = ((h < 2 ? tq01 : tq23) >> hs) & 0xffffu;
    const uint32_t c = __popc(bits);
    const uint32_t Rin = wave_incl_sum32(c);
    const uint32_t nh = readlane32(Rin, 63);
    const uint32_t pbase = 1024u * (uint32_t)h + 16u * (uint32_t)l;
    uint16_t* lp = list + (Rin - c);
    while (bits) {
      const uint32_t b = (uint32_t)__builtin_ctz(bits);
      bits &= bits - 1;
      *lp++ = (uint16_t)(pbase + b);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (uint32_t b0 = 0; b0 < nh; b0 += 64) {
      const uint32_t rr = b0 + l;
      const bool act = rr < nh;
      const uint32_t p = list[act ? rr : nh - 1];
      const uint32_t q = p >> 2, sh = p & 3u;
      const uint32_t q0 = d32[q], q1 = d32[q + 1], q2 = d32[q + 2], q3 = d32[q + 3];
      const uint32_t b0w = __builtin_amdgcn_alignbyte(q1, q0, sh);  // bytes p .. p+3
      const uint32_t b1w = __builtin_amdgcn_alignbyte(q2, q1, sh);  // p+4 .. p+7
      const uint32_t b2w = __builtin_amdgcn_alignbyte(q3, q2, sh);  // p+8 .. p+11
      const uint32_t tag = b0w & 0xffu;
      const uint64_t sel = dep_tab[tag];
      const uint32_t dlo = __builtin_amdgcn_alignbyte(b1w, b0w, 1);
      const uint32_t dhi = __builtin_amdgcn_alignbyte(b2w, b1w, 1);
      const bool z = tag == 0, f = tag == 0xffu;
      uint32_t cnt = z ? ((b0w >> 8) & 0xffu) : 0u;
      cnt = f ? ((b2w >> 8) & 0xffu) : cnt;
      const uint64_t runs = ballot(act && cnt != 0);
      uint32_t o = (uint32_t)l, btot = (uint32_t)__popcll(ballot(act));
      if (runs) {
        const uint32_t w = act ? 1u + cnt : 0u;
        const uint32_t inc = wave_incl_sum32(w);
        o = inc - w;
        btot = readlane32(inc, 63);
      }
      const uint32_t wlo = __builtin_amdgcn_perm(dhi, dlo, (uint32_t)sel);
      const uint32_t whi = __builtin_amdgcn_perm(dhi, dlo, (uint32_t)(sel >> 32));
      if (act) wp[o] = ((uint64_t)whi << 32) | wlo;
      if (FLAT && act) rp[o] = (A + p) | gen_tag;
      if (runs) {
        // a run's first word with its record (a raw run's from the staged bytes when they hold
        // it), the rest by the whole wave -- as expand_lean
        const uint32_t rb = p + 10u;  // a raw run's first word: bytes p + 10 .. p + 17
        const bool inl = !f || rb + 12u <= kStaged;
        uint64_t rw = 0;
        if (ballot(f && cnt != 0)) {
          const uint32_t rq = rb >> 2, rs = rb & 3u;
          const uint32_t rqc = rq < kStaged / 4 - 2 ? rq : kStaged / 4 - 3;
          const uint32_t r0 = d32[rqc], r1 = d32[rqc + 1], r2 = d32[rqc + 2];
          rw = f ? (((uint64_t)__builtin_amdgcn_alignbyte(r2, r1, rs) << 32) |
                    __builtin_amdgcn_alignbyte(r1, r0, rs))
                 : 0ull;
        }
        if (act && cnt != 0 && inl) wp[o + 1] = rw;
        uint64_t lm = ballot(act && (cnt > 1u || (cnt != 0 && !inl)));
        while (lm) {
          const int j = lowest_bit(lm);
          lm &= lm - 1;
          const uint32_t k0 = readlane32(inl ? 1u : 0u, j);
          const uint32_t nj = readlane32(cnt, j);
          uint64_t* const dst = wp + readlane32(o, j) + 1;
          const uint32_t sj = readlane32(rb, j);
          if (!readlane32(f ? 1u : 0u, j)) {
            for (uint32_t k = k0 + l; k < nj; k += 64) dst[k] = 0;
          } else {
            // (a raw run leaving the staged bytes: its words ending at most kRunSplit bytes into
            // the next tile; the next tile writes the rest, run_tail)
            const uint32_t kin = sj + 8u * nj + 4u <= kStaged
                                     ? nj
                                     : (sj + 12u <= kStaged ? (kStaged - 4u - sj) / 8u : 0u);
            const uint32_t ke = nj < kin ? nj : kin;
            for (uint32_t k = k0 + l; k < ke; k += 64) {
              const uint32_t ob = sj + 8u * k, qq = ob >> 2, s3 = ob & 3u;
              const uint32_t x0 = d32[qq], x1 = d32[qq + 1], x2 = d32[qq + 2];
              dst[k] = ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, s3) << 32) |
                       __builtin_amdgcn_alignbyte(x1, x0, s3);
            }
            if (FLAT)
              for (uint32_t k = (ke > k0 ? ke : k0) + l; k < nj; k += 64) {
                uint64_t v;
                __builtin_memcpy(&v, a.packed + A + sj + 8ull * k, 8);
                dst[k] = v;
              }
          }
        }
      }
      wp += btot;
      if (FLAT) rp += btot;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// Expansion of a tile's records given its true record-start masks (lane = sub-tile) and excl,
// the words of the tile's first message before the tile: the lean path when the tile's window
// allows it, else the general one.
template <bool FLAT = false>
__device__ __forceinline__ void expand_records(const UnpackArgs& a, uint64_t A, const uint8_t* d,
                                               uint64_t* aux, const uint64_t* dep_tab, uint64_t tm,
                                               uint64_t excl, MsgWin& win, uint64_t mfirst,
                                               uint64_t mlast, uint64_t msw,
                                               uint64_t tile_words = ~0ull) {
  const int l = lane_id();
  // a tile in the middle of one accepted message (no start in it; its words and bytes short of
  // the message's end; the message fits the output); FLAT: the split flat decode's tiles in the
  // middle of the stream.  (Taken in the one-pass flat decode too it measured slower: 9.55 ->
  // 10.8 ms -- that kernel's bound was its look-back, and the path's registers cost it spills.)
  if ((FLAT ? (a.rec_pos != nullptr) : (a.mode == 0 && !a.rec_pos)) && a.words && a.word_off &&
      tile_words != ~0ull && ballot(msw != 0) == 0) {
    const uint64_t cbase = readlane64(win.base, 0), ctot = readlane64(win.total, 0);
    const uint64_t cend = readlane64(win.end, 0);
    if (readlane32(win.ok, 0) && cbase + ctot <= a.words_capacity && excl + tile_words < ctot &&
        A + (uint64_t)kB + 2050u < cend) {
      expand_simple<FLAT>(a, A, d, aux, dep_tab, tm, a.words + cbase + excl,
                          FLAT ? a.rec_pos + cbase + excl : nullptr,
                          FLAT ? (*a.rec_gen << kRecGenShift) : 0ull);
      return;
    }
  }
  bool fast = a.mode == 0 && mlast - (mfirst - 1) <= 63 && a.word_off && a.words;
  if (fast) {
    const int64_t m = win.mw + l;
    const bool inrange = m >= 0 && (uint64_t)m < mlast;
    const bool bad = inrange && (!win.ok || win.base + win.total > a.words_capacity);
    const uint64_t nxs = shfl64(win.start, l < 63 ? l + 1 : 63);
    const bool dup = inrange && l < 63 && (uint64_t)(m + 1) < mlast && nxs == win.start;
    fast = ballot(bad || dup) == 0;
  }
  if (fast) {
    // list capacity per quarter tile (records shorter than 2 bytes exist only where message
    // starts clip them)
    const uint32_t cq = __popcll(tm);
    const uint32_t Rq = wave_incl_sum32(cq);
    const uint32_t q1 = readlane32(Rq, 15), q2 = readlane32(Rq, 31), q3 = readlane32(Rq, 47);
    const uint32_t nrec = readlane32(Rq, 63);
    constexpr uint32_t kList = kB / 8;
    if (q1 > kList || q2 - q1 > kList || q3 - q2 > kList || nrec - q3 > kList) fast = false;
  }
  if (fast) expand_lean(a, A, d, aux, dep_tab, tm, excl, win, msw);
  else expand_general(A, d, deposit_sel((uint32_t)l & 15), tm, excl, win, mfirst, msw);
}

#ifndef CPK_PREWALK
#define CPK_PREWALK 64  // bytes of unmarked walk before each sub-tile (0: none; at most 64)
#endif
#ifndef CPK_UNPACK_WPE
#define CPK_UNPACK_WPE 7  // 72 VGPRs: 7 waves per SIMD (LDS allows 7); 6 at the unconstrained 80
#endif
// FLAT: the flat stream decode's second-candidate descriptors and look-back are compiled in (a
// variant of its own: their registers cost the other variant spills).
// PHASE: 0 one pass; 1 an index launch (stage, chain 0, descriptors and the base chain's
// record-start bits; no look-back, no expansion); 2 its second launch (the base chain from the
// bits).  For message batches ("Split decode" below, the measured alternative CPK_UNPACK_SPLIT=1)
// the tile's prefix then comes from the resolve launch between the two.  For the flat decode
// (FLAT, the stream split's default) the index launch publishes every tile's chain-0 exit, AGG
// and second candidate, and the second launch looks back over descriptors that are all
// published (lookback_flat_scan<true>: one round trip per window, waits only for INCLs).
template <bool FLAT, int PHASE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CPK_UNPACK_WPE))) void
unpack_tiles_kernel(UnpackArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_data[4][kPre + kB + kPad];
  // per wave 1 KiB: message starts while they are found, then chain 0 and the walked starts
  // while the entry's chain is traced, then the record list of a quarter tile
  __shared__ uint64_t lds_aux[4][kB / 32];
  __shared__ uint64_t dep_tab[256];
  const int l = lane_id();
  const int wv = (int)uniform32(threadIdx.x >> 6);  // wave-uniform (keeps tile math scalar)
  if (PHASE != 1) dep_tab[threadIdx.x] = make_dep(threadIdx.x);
  if (PHASE == 0 && a.hdr_fuse) {
    // a single-tile batch of few messages: the header launch's work first, one message per
    // thread (serialize.c++:202-242 via header_words), the word offsets by one block scan
    __shared__ uint64_t s_hw[4];
    const uint64_t m = threadIdx.x;
    uint64_t w = 0;
    if (m < a.nmsgs) {
      int32_t hst;
      w = header_words(a.packed, a.in_off, m, a.hdr_limit, &hst);
      a.hdr_status_out[m] = hst;
      a.status[m] = hst;
    }
    const uint64_t inc = wave_incl_sum64(w);
    if (l == 63) s_hw[wv] = inc;
    __syncthreads();
    uint64_t before = 0;
    for (int v = 0; v < wv; v++) before += s_hw[v];
    const uint64_t o = before + inc - w;
    if (m < a.nmsgs) a.hdr_word_off[m] = o;
    if (m + 1 == a.nmsgs) a.hdr_word_off[a.nmsgs] = o + w;
    // (waves 1-3 leave at the tile check below: their stores, which may go to pinned host
    // memory, are complete before wave 0 publishes the call's error word for the host)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const uint64_t t = (uint64_t)blockIdx.x * 4 + wv;
  if (t >= a.ntiles) return;
  // the expansion launch of a split decode whose resolve launch could not place every tile runs
  // the one-pass look-back instead (wave-uniform)
  const bool gated = PHASE == 2 && !FLAT && uniform32(*(const volatile uint32_t*)a.gate) != 0;
  if (a.debug_skip & 512) return;  // diagnostic: the launch alone
  // batches of very long messages (whose look-backs reach back to the previous occupancy round):
  // the phases later tiles wait on (chain 0, the entry, the descriptors) ahead of other waves'
  // expansions in the SIMD's issue arbitration (C4 unpack_tiles 4.51 -> 4.21 ms; no gain on C2)
  if (PHASE == 0 && a.prio) __builtin_amdgcn_s_setprio(2);
  CPK_DIAG_ONLY(uint64_t ck[7]; uint64_t wk[7]; uint64_t wflat = 0; ck[0] = clock64(); wk[0] = wall_clock64());
  // the header launch is done: its scan descriptors go back to zero for the next call
  if (PHASE != 2)
    for (uint64_t i = t + a.ntiles * (uint64_t)l; i < a.hdr_nblocks; i += 64 * a.ntiles)
      a.hdr_desc[i] = 0;
  uint8_t* const d = lds_data[wv] + kPre;
  uint64_t* const aux = lds_aux[wv];
  const uint64_t P = a.nbytes;
  const uint64_t A = t * kB;
  Staged stg;
  stage_load(a, A, stg);
  const uint64_t mfirst = a.hdr_fuse ? 0 : uniform64(a.tile_first[t]);
  stage_store(stg, d);
  MsgWin win;
  int nms_tile_after;
  const uint64_t mlast = tile_msg_starts(a, A, mfirst, aux, &nms_tile_after, &win);
  const uint64_t msw = aux[l];
  lane_handoff();
  const SubTile st = make_subtile(A, P, msw, nms_tile_after);
  CPK_DIAG_ONLY(ck[1] = clock64(); wk[1] = wall_clock64());
  if (a.debug_skip & 64) {  // diagnostic: staging + message window only
    if (l == 0 && st.msw == 0) a.x0p[t] = 0x80000000u | (uint32_t)ballot(st.msw != 0);
    return;
  }

  // first message start (the batch end counts), tile-relative; kB if none
  const uint64_t msl = ballot(st.msw != 0);
  const int fl = lowest_bit(msl);
  const uint32_t fms = msl ? (uint32_t)(64 * fl + lowest_bit(readlane64(st.msw, fl))) : (uint32_t)kB;
  uint64_t runm = 0, tm0 = 0;
  uint32_t Eg = 0, x0 = 0;
  bool settled = true;
  int q0 = 0;  // where the tile's base chain starts
  if constexpr (PHASE == 2 && !FLAT) {
    // chain 0 as the index launch left it (its run records are rebuilt only where needed)
    tm0 = a.tbits[t * 64 + l];
    Eg = t > 0 ? uniform32(a.tegs[t]) : 0u;
    x0 = uniform32(a.x0p[t]) & 0x7fffffffu;
  } else if constexpr (PHASE == 2 && FLAT) {
    // the split flat decode: the base chain as the index launch left it (from byte 0, or from
    // the raw-record head that replaced it), its run records from the staged bytes
    tm0 = a.tbits[t * 64 + l];
    q0 = (int)uniform32(a.tegs[t]);
    x0 = uniform32(a.x0p[t]) & 0x7fffffffu;
    runm = run_bytes(d, st.s);
  } else {
  // ---- chain 0 (entered at the tile's first byte): speculative walks, then the lane fixed point
  uint64_t chain = 0;
  int sx = kDead;
  // Each lane's speculative chain starts CPK_PREWALK bytes before its sub-tile (at the last
  // message start there, if any) and walks unmarked up to it: chains synchronise within a few
  // records, so the chain then usually enters the sub-tile where the true one does, and the
  // fixed point below has little left to re-walk.
  // Lane 0 does the same through the kPre bytes before the tile (the predecessor's last bytes,
  // from its last message start there if any): where it lands is the tile's guessed entry Eg,
  // the start of the tile's base chain (the flat stream decode keeps chain 0, from byte 0).
  const bool guess = !FLAT && t > 0;
  int e0 = st.s;
#if CPK_PREWALK > 0
  {
    uint64_t pm = shfl64(st.msw, l > 0 ? l - 1 : 0);
    if (l == 0) {
      const uint64_t s0 = readlane64(win.start, 0);  // message mfirst - 1: the last start before A
      pm = (s0 != ~0ull && s0 + kPre >= A && s0 < A) ? 1ull << (s0 + kPre - A) : 0ull;
    }
    if ((l > 0 || guess) && st.s < st.pend && !(a.debug_skip & 4)) {
      const uint64_t wn = pm & ~mask_lt(64 - CPK_PREWALK);
      int q = wn ? st.s - 64 + highest_bit(wn) : st.s - CPK_PREWALK;
      while (q < st.s) q += step_len(d[q], d[q + 9]);
      // (a message start in the sub-tile before the landing point restarts the chain there)
      const int fm = st.msw ? st.s + lowest_bit(st.msw) : 0x7fffffff;
      e0 = q < fm ? q : fm;
      // (the base chain starts at or before the tile's first message start, where every chain
      // restarts, and inside the tile)
      if (l == 0 && e0 > (int)fms) e0 = (int)fms;
    }
  }
#endif
  Eg = guess ? (uint32_t)readlane32((uint32_t)e0, 0) : 0u;
#ifdef CPK_DIAG
  int dn = 0, dit[3] = {0, 0, 0};
  if (e0 < st.pend && !(a.debug_skip & 4)) sx = walk(d, st, e0, 0, &chain, &runm, &dn);
  diag_add(0, 1);
  diag_trips(1, dn);
  int* const diag_it = dit;
#else
  if (e0 < st.pend && !(a.debug_skip & 4)) sx = walk(d, st, e0, 0, &chain, &runm);
  int* const diag_it = nullptr;
#endif
  if (e0 >= st.pend) sx = kDead;
  int e = e0;
  int out = st.end;
  settled = (a.debug_skip & 4) ? true : settle(d, st, chain, sx, (int)Eg, e, tm0, out, runm, diag_it);
  CPK_DIAG_ONLY(diag_add(5, dit[0]));
  x0 = readlane32((uint32_t)out, 63);
  // Flat streams (stream split): inside long raw stretches (text) the chain from the tile's first
  // byte parses raw bytes as records and rarely finds the true chain within the tile, so its exit
  // -- the next tile's optimistic entry -- is wrong tile after tile and the entries resolve one
  // tile per look-back hop.  There, a raw record head with a full count (0xff, 8 bytes, 0xff) off
  // that chain is a better guess: when the chain through it never meets chain 0, it stands in for
  // chain 0 (any chain of the tile serves as the base the entry's chain is traced onto; its exit
  // is only ever a guess the look-back checks).
  if (FLAT && a.rec_pos && st.no_starts && t > 0 && settled && !(a.debug_skip & 4)) {
    const uint64_t ffm = ff_heads(d, st.s) & ~tm0;
    const uint64_t fl = ballot(ffm != 0);
    if (fl) {
      const int ql = lowest_bit(fl);
      const int q = 64 * ql + lowest_bit(readlane64(ffm, ql));
      int eF = e0, outF = st.end;
      uint64_t tmF = 0, runF = runm;
      CPK_DIAG_ONLY(diag_add(12, 1));
      if (settle(d, st, chain, sx, q, eF, tmF, outF, runF) && ballot((tmF & tm0) != 0) == 0) {
        CPK_DIAG_ONLY(diag_add(13, 1));
        tm0 = tmF;
        runm = runF;
        x0 = readlane32((uint32_t)outF, 63);
        q0 = q;
      }
    }
  }
  if (l == 0 && !(FLAT && PHASE == 2)) store_agent32(a.x0p + t, 0x80000000u | x0);
  if constexpr (PHASE == 1) {
    // the expansion launch's chain 0 (coalesced: 512 bytes per tile) and where it starts
    a.tbits[t * 64 + l] = tm0;
    if (l == 0) a.tegs[t] = FLAT ? (uint32_t)q0 : Eg;
  }
  }
  CPK_DIAG_ONLY(ck[2] = ck[3] = ck[4] = ck[5] = clock64(); wk[2] = wk[3] = wk[4] = wk[5] = wall_clock64());
  if (a.debug_skip & 128) return;  // diagnostic: + chain-0 walks and settle
  if (!settled) {
    // unreachable (the fixed point settles in at most 64 rounds): refuse the batch, write nothing
    if (l == 0) raise_error(a.err, kErrInternal);
    win.ok = 0;
  }

  // a message starting in the tile: exit and words after the last start are entry-independent
  const uint64_t msin = tm0 & st.msw;
  const int lastms = highest_bit(msin);
  const uint64_t hm = ballot(lastms >= 0);
  const bool has_start = hm != 0;
  CPK_DIAG_ONLY(diag_add(11, has_start));
  // (the expansion launch rebuilds chain 0's run records only where words are counted again)
  if (gated) runm = run_bytes(d, st.s);
  if (has_start && PHASE != 2) {
    const int lm = highest_bit(hm);
    const uint64_t from = l > lm ? ~0ull : (l == lm ? ~mask_lt(lastms) : 0ull);
    const uint32_t wl = mask_words(d, st.s, tm0 & from, runm);
    const uint64_t wpost = readlane32(wave_incl_sum32(wl), 63);
    if (l == 0) store_agent(a.desc + t, make_desc(kDescIncl, x0, x0, wpost));
  }

  // ---- the tile's entry and the words before it ------------------------------------------
  uint64_t tm = tm0, excl = 0;
  uint32_t Ein = 0;  // the tile's true entry
  uint64_t tile_words = ~0ull;  // words of the tile's records (a tile without a message start)
  if (t == 0 || fms == 0) {
    if (!has_start && PHASE != 2) {  // (tile 0 without a message start: bytes before the first message)
      const uint64_t w = readlane32(wave_incl_sum32(mask_words(d, st.s, tm0, runm)), 63);
      if (l == 0) store_agent(a.desc + t, make_desc(kDescIncl, x0, x0, w));
    }
  } else if constexpr (!FLAT) {
    // the guessed entry's AGG, at once (a tile with a message start published its INCL already;
    // the expansion launch's tiles find the index launch's)
    uint32_t xE = x0;
    uint64_t runs = runm, w = 0;
    if (!has_start && (PHASE != 2 || gated)) {
      w = readlane32(wave_incl_sum32(mask_words(d, st.s, tm0, runm)), 63);
      if (PHASE != 2 && l == 0) store_agent(a.desc + t, make_agg(x0, w, Eg, false));
    }
    CPK_DIAG_ONLY(ck[3] = clock64(); wk[3] = wall_clock64());
    // the final AGG: for the entry the predecessor's base-chain exit gives
    bool fin = has_start;
    uint32_t Eo = Eg, xO = x0;
    uint64_t tmO = tm0, runsO = runm, wO = w;
    auto finalize = [&](bool block) {
      if (fin) return;
      uint32_t xp = 0;
      if (block) {
        xp = wait_nonzero32(a.x0p + t - 1, a.err);
      } else {
        if (l == 0) xp = load_agent32(a.x0p + t - 1);
        xp = readlane32(xp, 0);
        if (!xp) return;
      }
      Eo = entry_from_exit(xp & 0x7fffffffu, fms);
      if (Eo != Eg) {
        runsO = runm;
        xO = x0;
        if (Eo < fms)
          tmO = enter_chain(d, aux, st, tm0, (int)Eo, (int)fms, x0, &xO, &runsO);
        else
          tmO = clip_below(tm0, fms, st.s, &xO);
        wO = readlane32(wave_incl_sum32(mask_words(d, st.s, tmO, runsO)), 63);
      }
      if (l == 0) store_agent(a.desc + t, make_agg(xO, wO, Eo, true));
      fin = true;
    };
    if constexpr (PHASE == 1) {
      // the index launch: the final AGG too when the predecessor's exit is out already (else the
      // resolve launch traces the entry); no look-back, no expansion
      finalize(false);
      return;
    }
    uint32_t xprev = (uint32_t)kB + Eg;
    if (PHASE == 2 && !gated) {
      // resolved: every tile's true exit is its base-chain exit (the resolve launch checked it)
      excl = a.texcl[t];
      xprev = uniform32(a.x0p[t - 1]) & 0x7fffffffu;
    } else {
      if (PHASE == 0) finalize(false);
      CPK_DIAG_ONLY(ck[4] = clock64(); wk[4] = wall_clock64());
      if (!(a.debug_skip & 8)) excl = lookback_tiles(a, t, &xprev, [&]() { finalize(true); });
    }
    CPK_DIAG_ONLY(ck[5] = clock64(); wk[5] = wall_clock64());
    const uint32_t E = entry_from_exit(xprev, fms);
    Ein = E;
    CPK_DIAG_ONLY(diag_add(9, E != Eg); diag_add(10, fin && Eo != Eg); diag_add(14, fin && E != Eo));
    if (E == Eg) {
    } else if (fin && E == Eo) {
      tm = tmO;
      runs = runsO;
      xE = xO;
      w = wO;
    } else {
      // neither guess: the predecessor's chain does not lead where they did
      if (E < fms)
        tm = enter_chain(d, aux, st, tm0, (int)E, (int)fms, x0, &xE, &runs);
      else
        tm = clip_below(tm0, fms, st.s, &xE);
      if (!has_start && (PHASE != 2 || gated))
        w = readlane32(wave_incl_sum32(mask_words(d, st.s, tm, runs)), 63);
    }
    if (!has_start && (PHASE != 2 || gated) && l == 0)
      store_agent(a.desc + t, make_desc(kDescIncl, xE, x0, excl + w));
    if (!has_start && (PHASE != 2 || gated)) tile_words = w;
    if (a.stamps && l == 0 && t < 1024) {  // diagnostic dump (CPK_STAMPS=1)
      a.stamps[4 * t] = E | ((uint64_t)Eg << 32);
      a.stamps[4 * t + 1] = xE | ((uint64_t)x0 << 32);
      a.stamps[4 * t + 2] = excl;
      a.stamps[4 * t + 3] = w | ((uint64_t)fms << 32) | ((uint64_t)has_start << 63);
    }
  } else {
    // optimistic entry: where the predecessor's chain 0 leads (a tile with a message start
    // publishes its descriptor already, so it goes straight to the look-back)
    // (the split flat decode's second launch: published by the index launch)
    const uint32_t xp = has_start ? 0u
                        : (PHASE == 2 ? uniform32(a.x0p[t - 1])
                                      : wait_nonzero32(a.x0p + t - 1, a.err)) & 0x7fffffffu;
    CPK_DIAG_ONLY(ck[3] = ck[4] = ck[5] = clock64(); wk[3] = wk[4] = wk[5] = wall_clock64());
    const uint32_t Eopt = has_start ? ~0u : entry_from_exit(xp, fms);
    uint32_t xE = x0;
    uint64_t runs = runm;
    uint64_t w = 0;
    if (PHASE != 2) {  // (the split decode's second launch: the index launch published these)
    if (has_start) {
    } else if (Eopt != (uint32_t)q0 && Eopt < fms)
      tm = enter_chain(d, aux, st, tm0, (int)Eopt, (int)fms, x0, &xE, &runs);
    else if (Eopt >= fms)
      tm = clip_below(tm0, fms, st.s, &xE);
    if (!has_start) {
      w = readlane32(wave_incl_sum32(mask_words(d, st.s, tm, runs)), 63);
      if (l == 0) store_agent(a.desc + t, make_desc(kDescAgg, xE, x0, w));
      CPK_DIAG_ONLY(diag_add(14, xE != x0));
    }
    if (FLAT && !has_start) {
      // flat stream: the exit and words for the entry the predecessor's AGG exit gives
      CPK_DIAG_ONLY(const uint64_t wa0 = wall_clock64());
      const uint64_t dp = wait_nonzero64(a.desc + t - 1, a.err);
      // (diagnostic) AGG published, predecessor's AGG seen: ticks after the tile's start
      CPK_DIAG_ONLY(wflat = (wa0 - wk[0]) | ((wall_clock64() - wk[0]) << 32));
      const uint32_t E2 = entry_from_exit(desc_exit(dp), fms);
      uint64_t d2 = kD2None;
      if (E2 != Eopt && E2 <= (uint32_t)kB) {
        uint64_t runs2 = runm, tm2;
        uint32_t xE2 = x0;
        if (E2 != (uint32_t)q0 && E2 < fms)
          tm2 = enter_chain(d, aux, st, tm0, (int)E2, (int)fms, x0, &xE2, &runs2);
        else if (E2 >= fms)
          tm2 = clip_below(tm0, fms, st.s, &xE2);
        else
          tm2 = tm0;
        const uint64_t w2 = readlane32(wave_incl_sum32(mask_words(d, st.s, tm2, runs2)), 63);
        d2 = (make_desc(kDescAgg, xE2, x0, 0) & ~kWordsMask) | ((uint64_t)E2 << kD2EntryShift) |
             (w2 & kD2WordsMask);
      }
      if (l == 0) store_agent(a.desc2 + t, d2);
    }
    }
    if constexpr (PHASE == 1) return;  // the split decode's index launch: published, done
    uint32_t xprev = xp;
    CPK_DIAG_ONLY(ck[4] = clock64(); wk[4] = wall_clock64());
    if (!(a.debug_skip & 8)) {
      excl = lookback_flat_scan<PHASE == 2>(a, t, &xprev);
    }
    CPK_DIAG_ONLY(ck[5] = clock64(); wk[5] = wall_clock64());
    const uint32_t E = entry_from_exit(xprev, fms);
    CPK_DIAG_ONLY(diag_add(9, E != Eopt); diag_add(10, Eopt > 0 && Eopt < fms));
    if (PHASE == 2 || E != Eopt) {
      // the predecessor's chain did not lead where its chain 0 does (or, in the split decode's
      // second launch, the entry's chain is traced here for the first time)
      runs = runm;
      xE = x0;
      if (E != (uint32_t)q0 && E < fms)
        tm = enter_chain(d, aux, st, tm0, (int)E, (int)fms, x0, &xE, &runs);
      else if (E >= fms)
        tm = clip_below(tm0, fms, st.s, &xE);
      else
        tm = tm0;
      if (!has_start) w = readlane32(wave_incl_sum32(mask_words(d, st.s, tm, runs)), 63);
    }
    if (!has_start) {
      if (l == 0) store_agent(a.desc + t, make_desc(kDescIncl, xE, x0, excl + w));
      if (PHASE == 2) tile_words = w;
    }
    if (a.stamps && l == 0 && t < 1024) {  // diagnostic dump (CPK_STAMPS=1)
      a.stamps[4 * t] = E | ((uint64_t)Eopt << 32);
      a.stamps[4 * t + 1] = xE | ((uint64_t)x0 << 32);
      a.stamps[4 * t + 2] = excl;
      a.stamps[4 * t + 3] = w | ((uint64_t)fms << 32) | ((uint64_t)has_start << 63);
    }
  }

  // ---- expansion -------------------------------------------------------------------------
  if constexpr (PHASE == 1) return;
  if (a.debug_skip & 256) return;  // diagnostic: + the entry and the look-back
  if (PHASE == 0 && a.prio) __builtin_amdgcn_s_setprio(0);
  if (!FLAT && a.mode == 0 && a.words && Ein > kRunSplit) run_tail(a, A, d, Ein, excl, win);
  expand_records<FLAT && PHASE == 2>(a, A, d, aux, dep_tab, tm, excl, win, mfirst, mlast, msw,
                                     tile_words);
  // a fused single-tile batch: this wave is the whole call -- its error word for the host, last:
  // its stores done, then a system-scope release
  if (a.err_host) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (l == 0) {
      __threadfence_system();
      __hip_atomic_store(a.err_host, load_agent32(a.err), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
#ifdef CPK_DIAG
  ck[6] = clock64();
  wk[6] = wall_clock64();
  for (int k = 0; k < 6; k++) diag_add(16 + k, ck[k + 1] - ck[k]);
  if (l == 0 && t < (uint64_t)kTimelineTiles) {
    for (int k = 0; k < 7; k++) g_timeline[8 * t + k] = wk[k];
    g_timeline[8 * t + 7] = FLAT ? wflat : __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
  }
#endif
}

// ---------------------------------------------------------------------------------------------
// Split decode (message batches, cpk_unpack_messages): the one-pass tile kernel above spends a
// quarter of a tile's life in its look-back, waiting for predecessors that are still walking
// their own chain 0.  Split into three launches, no tile ever waits on another tile:
//   index    (PHASE 1) stage, chain 0 and the tile's descriptor (AGG with its guessed entry, or
//            INCL when a message starts in it) exactly as the one-pass kernel publishes them,
//            plus chain 0's record-start bits (512 B per tile) and the guessed entry;
//   resolve  (below) every tile's true entry is where its predecessor's base-chain exit leads --
//            true as long as every tile's exit is its base-chain exit, which this launch checks
//            -- so each tile's words follow from its own descriptor (or, when its guessed entry was
//            not that one, from its chain re-traced from the true entry) and the words before
//            every tile are one segmented scan (decoupled look-back over 64-tile groups);
//   expand   (PHASE 2) stage, chain 0 from the bits, the entry from the predecessor's exit, the
//            expansion.
// A tile whose true exit is not its base-chain exit (chains that do not meet within a tile) sets
// the gate, and the expansion launch then runs the one-pass look-back on the index launch's
// descriptors instead -- the same results, the one-pass kernel's speed.
__global__ __launch_bounds__(256) void unpack_resolve_kernel(ResolveArgs r) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_data[4][kB + kPad + 16];
  __shared__ uint64_t lds_aux[4][128];
  __shared__ unsigned int s_ticket;
  const int l = lane_id();
  const int wv = (int)uniform32(threadIdx.x >> 6);
  // groups in ticket order: a group waits only on groups whose workgroups took their tickets
  // before its own (running or done), whatever else shares the device
  const uint64_t g = (uint64_t)wg_ticket(r.ticket, &s_ticket) * 4 + (uint64_t)wv;
  const uint64_t ngroups = resolve_groups(r.ntiles);
  if (g >= ngroups) return;
  const uint64_t P = r.nbytes;
  const uint64_t t = g * kResolveGroup + (uint64_t)l;
  const bool valid = t < r.ntiles;
  const uint64_t tc = valid ? t : r.ntiles - 1;
  // (the index launch is complete: plain loads)
  const uint64_t dv = r.desc[tc];
  const uint32_t x0 = r.x0p[tc] & 0x7fffffffu;
  const uint32_t xp = tc > 0 ? (r.x0p[tc - 1] & 0x7fffffffu) : 0u;
  const uint64_t A = tc * kB;
  // an AGG tile holds no message start; its first "start" is the batch end, if inside it
  const uint32_t fmsn = (P - A) < (uint64_t)kB ? (uint32_t)(P - A) : (uint32_t)kB;
  const uint64_t stt = dv & kDescFlags;
  uint64_t v = 0;
  uint32_t reset = 0, bad = 0, fix = 0;
  const uint32_t E = entry_from_exit(xp, fmsn);
  if (valid) {
    if (stt == kDescIncl) {
      v = dv & kWordsMask;  // words after the last message start in the tile
      reset = 1;
    } else if (stt == kDescAgg) {
      if (desc_entry(dv) == E) {
        v = dv & kWordsMask;
        bad = desc_exit(dv) != x0;  // (a final AGG whose chain never met chain 0)
      } else {
        fix = 1;
      }
    } else {
      bad = 1;  // (unreachable: the index launch publishes every tile)
    }
  }
  // tiles whose guessed entry is not the true one: the chain from the true entry, traced onto
  // chain 0 in LDS (as the one-pass kernel's finalisation does)
  uint64_t fixes = ballot(fix != 0);
  uint8_t* const d = lds_data[wv];
  uint64_t* const aux = lds_aux[wv];
  const bool aligned = ((uintptr_t)r.packed & 15) == 0;
  while (fixes) {
    const int j = lowest_bit(fixes);
    fixes &= fixes - 1;
    const uint64_t tj = g * kResolveGroup + (uint64_t)j;
    const uint64_t Aj = tj * kB;
    const uint32_t Ej = readlane32(E, j), x0j = readlane32(x0, j), fj = readlane32(fmsn, j);
#pragma unroll
    for (int k = 0; k < 5; k++) {
      const int o = 16 * (64 * k + l);
      if (o < kB + kPad) {
        const uint64_t b = Aj + (uint64_t)o;
        u32x4 q = {0, 0, 0, 0};
        if (aligned && b + 16 <= P) {
          q = *(const u32x4*)(r.packed + b);
        } else {
          uint32_t w4[4] = {0, 0, 0, 0};
          for (int i = 0; i < 16; i++)
            if (b + i < P) w4[i >> 2] |= (uint32_t)r.packed[b + i] << (8 * (i & 3));
          q = (u32x4){w4[0], w4[1], w4[2], w4[3]};
        }
        *(u32x4*)(d + o) = q;
      }
    }
    lane_handoff();
    const uint64_t tm0 = r.tbits[tj * 64 + (uint64_t)l];
    uint64_t runs = run_bytes(d, 64 * l);
    const uint64_t pe = P - Aj;  // the batch end, tile-relative (a start when inside the tile)
    const uint64_t msw = (pe < (uint64_t)kB && (int)(pe >> 6) == l) ? 1ull << (pe & 63) : 0ull;
    const uint64_t fp = r.tile_firstpos[tj];
    const uint64_t na = (fp < P ? fp : P) - Aj;
    const SubTile st = make_subtile(Aj, P, msw, na < (uint64_t)kDead ? (int)na : kDead);
    uint32_t xO = x0j;
    uint64_t tmO;
    if (Ej < fj)
      tmO = enter_chain(d, aux, st, tm0, (int)Ej, (int)fj, x0j, &xO, &runs);
    else
      tmO = clip_below(tm0, fj, st.s, &xO);
    const uint64_t wO = readlane32(wave_incl_sum32(mask_words(d, st.s, tmO, runs)), 63);
    if (l == j) {
      v = wO;
      bad = xO != x0j;
    }
    lane_handoff();  // (the next fix overwrites d and aux)
  }
  // inclusive segmented scan over the group (a tile with a message start restarts the sum)
  uint64_t s = v;
  uint32_t f = reset;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int src = l >= o ? l - o : l;
    const uint64_t ps = shfl64(s, src);
    const uint32_t pf = shfl32(f, src);
    if (l >= o) {
      if (!f) s += ps;
      f |= pf;
    }
  }
  const uint64_t agg = readlane64(s, 63);
  const bool aggf = ballot(reset != 0) != 0;
  uint64_t gex = 0;
  if (g == 0) {
    if (l == 0) store_agent(r.gdesc, kDescIncl | agg);
  } else if (aggf) {
    // (the group's total is its words after its last restart: inclusive at once; its tiles up to
    // that restart still need the words before the group)
    if (l == 0) store_agent(r.gdesc + g, kDescIncl | agg);
    gex = lookback<8>(r.gdesc, g, r.err);
  } else {
    if (l == 0) store_agent(r.gdesc + g, kDescAgg | agg);
    gex = lookback<8>(r.gdesc, g, r.err);
    if (l == 0) store_agent(r.gdesc + g, kDescIncl | (gex + agg));
  }
  const int pl = l > 0 ? l - 1 : 0;
  const uint64_t se = shfl64(s, pl);
  const uint32_t fe = shfl32(f, pl);
  const uint64_t ex = l == 0 ? gex : (fe ? se : gex + se);
  if (valid) r.texcl[t] = ex;
  if (ballot(bad != 0) && l == 0) store_agent32(r.gate, 1u);
}

// Status before any record is seen (buffers with no records keep it): flat-packed chunks read
// exactly word_off[m+1]-word_off[m] words; size-only buffers start at 0 words.
__global__ void init_kernel(uint32_t mode, const uint64_t* __restrict__ in_off,
                            const uint64_t* __restrict__ word_off, uint64_t n,
                            int32_t* __restrict__ status, uint64_t* __restrict__ size_out,
                            TileFirstJob tf, uint32_t tf_block) {
  if (run_tile_first(tf, tf_block)) return;
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  const bool empty = in_off[m + 1] == in_off[m];
  if (mode == 2) {
    status[m] = kOK;
    size_out[m] = 0;
  } else {
    const bool zero = word_off[m + 1] == word_off[m];
    status[m] = zero ? (empty ? kOK : kTrailing) : kEOF;
  }
}

}  // namespace

hipError_t launch_unpack_init(uint32_t mode, const uint64_t* in_off, const uint64_t* word_off,
                              uint64_t n, int32_t* status, uint64_t* size_out,
                              const TileFirstJob& tf, hipStream_t stream) {
  const unsigned nb = (unsigned)((n + 255) / 256);
  if (nb + tile_first_blocks(tf) == 0) return hipSuccess;
  hipLaunchKernelGGL(init_kernel, dim3(nb + tile_first_blocks(tf)), dim3(256), 0, stream, mode,
                     in_off, word_off, n, status, size_out, tf, nb);
  return hipGetLastError();
}

uint64_t header_scan_blocks(uint64_t n) {
  const uint64_t blk = 256ull * (uint64_t)hdr_per(n);
  return (n + blk - 1) / blk;
}

hipError_t launch_unpack_header(const uint8_t* packed, uint64_t P, const uint64_t* in_off,
                                uint64_t n, uint64_t limit, uint64_t* word_off,
                                int32_t* hdr_status, int32_t* status, uint64_t* desc,
                                uint32_t* err, const TileFirstJob& tf, hipStream_t stream) {
  const unsigned nb = (unsigned)header_scan_blocks(n);
  if (nb + tile_first_blocks(tf) == 0) return hipSuccess;
  const dim3 g(nb + tile_first_blocks(tf)), blk(256);
  switch (hdr_per(n)) {
    case 1:
      hipLaunchKernelGGL(header_kernel<1>, g, blk, 0, stream, packed, P, in_off, n, limit,
                         word_off, hdr_status, status, desc, err, tf, nb);
      break;
    default:
      hipLaunchKernelGGL(header_kernel<4>, g, blk, 0, stream, packed, P, in_off, n, limit,
                         word_off, hdr_status, status, desc, err, tf, nb);
  }
  return hipGetLastError();
}

hipError_t launch_unpack_resolve(const ResolveArgs& r, hipStream_t stream) {
  const uint64_t ng = resolve_groups(r.ntiles);
  if (ng == 0) return hipSuccess;
  hipLaunchKernelGGL(unpack_resolve_kernel, dim3((unsigned)((ng + 3) / 4)), dim3(256), 0, stream, r);
  return hipGetLastError();
}

hipError_t launch_unpack_stage(int stage, const UnpackArgs& a, hipStream_t stream) {
  if (a.ntiles == 0) return hipSuccess;
  const dim3 grid((unsigned)((a.ntiles + 3) / 4));
  if (stage == kUnpackIndex && a.desc2)
    hipLaunchKernelGGL((unpack_tiles_kernel<true, 1>), grid, dim3(256), 0, stream, a);
  else if (stage == kUnpackExpand && a.desc2)
    hipLaunchKernelGGL((unpack_tiles_kernel<true, 2>), grid, dim3(256), 0, stream, a);
  else if (stage == kUnpackIndex)
    hipLaunchKernelGGL((unpack_tiles_kernel<false, 1>), grid, dim3(256), 0, stream, a);
  else if (stage == kUnpackExpand)
    hipLaunchKernelGGL((unpack_tiles_kernel<false, 2>), grid, dim3(256), 0, stream, a);
  else if (a.desc2)
    hipLaunchKernelGGL((unpack_tiles_kernel<true, 0>), grid, dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL((unpack_tiles_kernel<false, 0>), grid, dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace cpk

#ifdef CPK_DIAG
// diagnostic build only: copies out (and optionally zeroes) the unpack step counters
//  0 tiles  1/2 chain-0 walk trips (wave max / lane sum)  3/4 settle re-walk trips (max / sum)
//  5 settle rounds  6 enter_chain calls  7 lane-0 merge steps  8 merges past the cap
//  9 entries that differed from the optimistic one  10 optimistic entries walked  11 tiles with a start
//  12 flat stream: tiles with a raw-head candidate  13 ... whose chain replaced chain 0
//  14 tiles whose optimistic entry's exit is not their chain-0 exit (no ok bit)
//  16..21 clock cycles (s_memtime) per phase: staging and message window, chain 0, waiting for
//  the predecessor's chain-0 exit, the optimistic entry, the look-back, the expansion
//  22..25 message look-back: windows read, waits for a descriptor not published yet, waits for
//  an INCL (an AGG without the ok bit), polls
//  26/27 flat look-back: waits for an INCL (no INCL within reach, or an entry matching no
//  candidate), waits for a descriptor not published yet
//  28/29 composed flat look-back: windows read before an INCL wait, windows read to resolve
extern "C" int cpk_debug_diag(uint64_t* out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return 10;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cpk::g_diag), 32 * sizeof(uint64_t)) != hipSuccess) return 10;
  if (reset) {
    const uint64_t z[32] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(cpk::g_diag), z, sizeof z) != hipSuccess) return 10;
  }
  return 0;
}

// diagnostic build only: copies out (and zeroes) the timeline of the first n tiles (8 words each)
extern "C" int cpk_debug_timeline(uint64_t* out, int n) {
  if (n > cpk::kTimelineTiles) n = cpk::kTimelineTiles;
  if (hipDeviceSynchronize() != hipSuccess) return 10;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cpk::g_timeline), (size_t)n * 64) != hipSuccess) return 10;
  static uint64_t z[cpk::kTimelineTiles * 8];
  if (hipMemcpyToSymbol(HIP_SYMBOL(cpk::g_timeline), z, sizeof z) != hipSuccess) return 10;
  return 0;
}
#endif
