// cpk_pack.hip -- the pack kernels (gfx950): PackedOutputStream::write (capnproto
// c++/src/capnp/serialize-packed.c++:307-431) once per chunk, for a whole batch of chunks.
//
// Layout.  A workgroup tile is 2048 consecutive words: 4 waves x 64 lanes x 8 CONSECUTIVE words,
// so each lane encodes its own 8-word stretch serially and the cross-lane work is a handful of
// 8-bit mask operations per lane, one wave prefix sum and one workgroup combine.
//
//   classes   per word: tag byte (SWAR), Z all zero, R <= 1 zero byte, F no zero byte, as 8-bit
//             lane masks.  Sync points -- chunk starts (serialize.c++:311-357 + kj/io.c++:109-113
//             make every segment-table and segment write() a chunk), O words (neither Z nor R),
//             the first word of a Z or R stretch -- reset the encoder.
//   coverage  from a lane's entry budget b (words the run open before the lane may still cover,
//             serialize-packed.c++:352-374 zero runs, :376-426 raw runs, both <= 255 words) the
//             covered words and run heads follow from carry-add mask algebra on 8 bits.  A lane
//             with a sync point has an exit budget independent of b; a sync-free lane of one
//             kind (all Z, or all F) maps b -> (b - 8) mod 256, so a sync-free wave of them maps b
//             to itself (512 = 2 * 256).  Other sync-free stretches compose exactly in a scalar
//             pass (rare: a >= 8-word stretch of words with one zero byte and no O word).
//   tiles     one workgroup per tile in blockIdx order: a tile only ever waits for the exit budget
//             of the tile before it (dispatched earlier, so running or done -- whatever else
//             shares the GPU).  The exit budget is published in state[] as soon as it is known
//             (right after the classes when the tile holds a sync point).  A tile's packed bytes
//             go to its own scratch slot; a scan of the tile byte counts and a placement kernel
//             move them to their final offsets (no look-back inside the tile kernel).
//   count     the count byte of a run still open at the tile end depends on words of the next
//             tile.  The tile writes it as if the batch ended there; when the next tile's first
//             word is not a sync point (so the run may go on), the tile leaves that byte out of
//             its stores and the NEXT tile -- which waits for this tile's exit budget anyway --
//             writes it.  No tile ever waits on a later one.
//   emission  each lane ORs its records into the staging slot at their own byte offsets (up to
//             4 dwords each; bytes past a record are zero), empty records into a per-lane trash
//             window; the slot then leaves with 16-byte stores.  A tile whose bytes exceed the
//             slot (> 9 B/word: pathological one-word chunks or alternating raw/other words) is
//             staged in several windows.
#include <stdlib.h>

#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kK = 8;                          // words per lane
constexpr int kWv = 4;                         // waves per workgroup
constexpr int kWW = 64 * kK;                   // words per wave
constexpr int kTW = kWv * kWW;                 // words per workgroup tile
constexpr uint32_t kCap = 9 * kTW;             // staging window (bytes)
constexpr uint32_t kPadF = 16;                 // front pad: records straddling the window start
constexpr int kSlotDw = (kPadF + kCap + 64) / 4;
constexpr int kTrashDw = 64 + 4;               // lane l: dwords l .. l + 3
constexpr uint32_t kArenaTile = kPackArenaTile;  // tiles of at most this many bytes use the arena
constexpr uint64_t kScr = kPackScratchBytes;    // scratch slot per tile (<= 10 B per word)
static_assert(kScr >= 10 * kTW && kScr % 16 == 0, "a tile's bytes fit its scratch slot");

static_assert(kTW == (int)kPackTileWords, "tile size shared with cpk_api.cpp");

__device__ __forceinline__ uint32_t tag_of(uint32_t lo, uint32_t hi) {
  const uint32_t m7 = 0x7f7f7f7fu;
  const uint32_t a = ((lo & m7) + m7) | lo;  // bit 7 of a byte <=> byte non-zero
  const uint32_t b = ((hi & m7) + m7) | hi;
  const uint32_t c = ((a >> 7) & 0x01010101u) | ((b >> 3) & 0x10101010u);
  const uint32_t d = c | (c >> 14);
  return (d | (d >> 7)) & 0xffu;
}

// v_perm selectors placing the non-zero bytes of a word with tag `tag` after its tag byte:
// dword 0 = [tag slot, c0, c1, c2], dword 1 = [c3 .. c6] (c7 only exists for tag 0xff).
__device__ __forceinline__ uint64_t make_sel(uint32_t tag) {
  uint64_t sel = 0x0c0c0c0c0c0c0c0cull;
  int j = 1;
  for (int i = 0; i < 8; i++) {
    if ((tag >> i) & 1) {
      if (j < 8) sel = (sel & ~(0xffull << (8 * j))) | ((uint64_t)i << (8 * j));
      j++;
    }
  }
  return sel;
}

__device__ __forceinline__ int hi_bit(uint32_t m) { return m ? 31 - __clz(m) : -1; }

struct Cov {
  uint32_t cov, zh, fh;  // covered words, zero-run heads, raw-run heads
  uint32_t b_out;        // budget leaving the lane
};

// Coverage of one lane's 8 words for entry budget b.
//   lead    words before the lane's first sync point continue the stretch entering the lane:
//           the first b are covered; in a Z stretch word b is the next head.
//   fill    after a raw-run head (F), the following R words up to the next sync point:
//           ((NS + G) ^ NS) & NS carries each head's bit through the non-sync run behind it.
// A run never closes inside 8 words (255 > 7), so one head per stretch and lane at most.
__device__ __forceinline__ Cov cover8(uint32_t Z, uint32_t F, uint32_t R, uint32_t SY, uint32_t b,
                                      bool last_valid) {
  const uint32_t NS = ~SY & 0xffu;
  const uint32_t LM = NS & (SY - 1u);
  const uint32_t BM = b >= 8u ? 0xffu : ((1u << b) - 1u);
  const uint32_t lead_cov = BM & LM;
  const uint32_t zlead = (BM + 1u) & LM & Z;
  const uint32_t Feff = F & ~lead_cov;
  const uint32_t G = (Feff << 1) & NS;
  const uint32_t fill = ((((NS + G) ^ NS) & NS) | G) & 0xffu;
  Cov c;
  c.fh = Feff & ~fill;
  c.zh = (Z & SY) | zlead;
  c.cov = (R & (fill | lead_cov)) | (Z & ~c.zh);
  c.b_out = 0;
  if (last_valid) {
    const int st = hi_bit(SY);
    const int h = hi_bit(c.zh | c.fh);
    if (h >= 0 && h >= st) c.b_out = 248u + (uint32_t)h;
    else if (SY == 0 && b > 7u) c.b_out = b - 8u;
  }
  return c;
}

// Exit budget of a sync-free lane (lane masks zl, fl) for entry budget b: one kind of word
// (all Z, or b covers the lane) -> (b - 8) mod 256; else the first F word at or after b heads a
// raw run (exit 248 + its position), none -> 0.
__device__ __forceinline__ uint32_t free_lane_exit(uint32_t b, uint32_t zl, uint32_t fl) {
  if (zl == 0xffu || b >= 8u) return (b - 8u) & 0xffu;
  const uint32_t fm = fl >> b;
  return fm ? 248u + b + (uint32_t)__builtin_ctz(fm) : 0u;
}

// Entry budget of every lane given the wave's entry budget bw: lanes with a sync point pass on
// their own exit (ex); sync-free lanes of one kind take 8 words each.  When a sync-free lane
// holds other words (`nonsimple`), a scalar pass composes the exact per-lane functions.
__device__ __forceinline__ uint32_t lane_entries(uint32_t bw, uint64_t hs, uint64_t nonsimple,
                                                 uint32_t ex, uint32_t Z, uint32_t F) {
  const int l = lane_id();
  if (nonsimple == 0) {
    const uint64_t below = hs & mask_lt(l);
    const int j = highest_bit(below);  // -1: no sync lane below
    const uint32_t ej = shfl32(ex, j < 0 ? 0 : j);
    const uint32_t base = j < 0 ? bw : ej;
    const uint32_t d = (uint32_t)(l - 1 - j);  // sync-free lanes in between
    return (base - 8u * d) & 0xffu;
  }
  uint32_t e = 0;
  uint32_t b = bw;
#pragma nounroll
  for (int L = 0; L < 64; L++) {
    if (l == L) e = b;
    if ((hs >> L) & 1) b = readlane32(ex, L);
    else b = free_lane_exit(b, readlane32(Z, L), readlane32(F, L));
  }
  return e;
}

// Exit budget of the wave for entry budget bw (uniform).
__device__ __forceinline__ uint32_t wave_exit(uint32_t bw, uint64_t hs, uint64_t nonsimple,
                                              uint32_t ex, uint32_t Z, uint32_t F) {
  const int j = highest_bit(hs);
  uint32_t b = j < 0 ? bw : readlane32(ex, j);
  const uint64_t after = j < 0 ? ~0ull : ~mask_le(j);
  if ((nonsimple & after) == 0) return (b - 8u * (uint32_t)(63 - j)) & 0xffu;
#pragma nounroll
  for (int L = j + 1; L < 64; L++) b = free_lane_exit(b, readlane32(Z, L), readlane32(F, L));
  return b;
}

// Per-wave summary, exchanged through LDS (double-buffered by tile parity), packed in one
// word: bit 0 the wave holds a sync point (its exit does not depend on its entry), bit 1 no
// lane needs the scalar composition, bits 2-11 its first sync word (wave-relative; kWW: none),
// bits 16-23 its exit when it holds a sync point.
__device__ __forceinline__ uint32_t sum_pack(bool has_sync, bool simple, uint32_t fsw,
                                             uint32_t exit0) {
  return (has_sync ? 1u : 0u) | (simple ? 2u : 0u) | (fsw << 2) | (exit0 << 16);
}
__device__ __forceinline__ bool sum_sync(uint32_t s) { return s & 1u; }
__device__ __forceinline__ bool sum_simple(uint32_t s) { return (s >> 1) & 1u; }
__device__ __forceinline__ uint32_t sum_fsw(uint32_t s) { return (s >> 2) & 0x3ffu; }
__device__ __forceinline__ uint32_t sum_exit(uint32_t s) { return (s >> 16) & 0xffu; }

// Look-back for tile t (one wave): the exclusive byte prefix from the descriptors of its
// predecessors -- a first window of 16 (one 128-byte line: these agent-scope reads go past the L2,
// and the nearest inclusive prefix is usually a few tiles back), then 64 per round trip.
// wait == false: gives up (false) when one before the nearest inclusive prefix has not
// published its byte count yet, or after 272 predecessors (one round trip instead: C3 pack_tile
// 2.18 -> 3.05 ms, fewer tiles resolve in time and more wait).  wait == true re-reads the blocked
// window with every lane; measured and not kept: one lane polling the blocking descriptor (C2 /
// C3 / C4 pack_tile +5 / +6 / +9 %), 128 or 256 tiles per round trip (C3 +7 / +15 %), the 64
// nearest tiles read again beside a blocked window or beside every far one (C2 +5 / +12 %).
__device__ __forceinline__ bool pack_lookback(const uint64_t* desc, uint64_t t, uint64_t* out,
                                              bool wait, uint32_t* err) {
  const int l = lane_id() + (int)opaque_zero();  // (addresses not hoisted out of the caller's loop)
  uint64_t excl = 0;
  int64_t j = (int64_t)t - 1;
  uint32_t spins = 0;
  int width = 16;
  for (int round = 0;;) {
    const int64_t idx = j - l;
    const bool in = l < width;
    const uint64_t d = !in ? 0ull : (idx >= 0 ? load_agent(desc + idx) : kDescIncl);
    const uint64_t f = d & kDescFlags;
    const uint64_t sb = ballot(in && f == kDescIncl), nb = ballot(in && f == 0);
    const int stop_at = sb ? lowest_bit(sb) : 64;
    const int blocked = nb ? lowest_bit(nb) : 64;
    if (blocked < stop_at) {
      if (!wait) return false;
      if (++spins >= kSpinLimit) {
        if (l == 0) raise_error(err, kErrInternal);
        *out = excl;
        return true;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;  // the same window again
    }
    excl += wave_sum64(l <= stop_at && in ? (d & kDescValue) : 0ull);
    if (stop_at < 64) {
      *out = excl;
      return true;
    }
    j -= width;
    width = 64;
    if (!wait && ++round == 5) return false;
  }
}

// The staged tile (tile byte j at stg byte kPadF + j, n bytes) to o0 (any alignment), all
// threads of the workgroup: 16-byte stores in the body, byte stores at both ends and in the one
// 16-byte block holding `hole` (a count byte the next tile writes; ~0: none), which is skipped.
__device__ __forceinline__ void copy_out_final(const uint32_t* stg, uint32_t n, uint8_t* o0,
                                               uint32_t hole, int tid_) {
  const int tid = tid_ + (int)opaque_zero();  // (addresses not hoisted out of the caller's loop)
  const uint8_t* const sb = (const uint8_t*)stg + kPadF;
  const uint64_t A0 = (uint64_t)(uintptr_t)o0;
  const uint64_t A1 = A0 + n;
  const uint64_t al = (A0 + 15) & ~15ull;
  const uint32_t head = (uint32_t)((al < A1 ? al : A1) - A0);
  if ((uint32_t)tid < head && (uint32_t)tid != hole) o0[tid] = sb[tid];
  if (A1 <= al) return;
  const uint32_t body = (uint32_t)((A1 & ~15ull) - A0);
  const uint32_t nblk = (body - head) >> 4;
  const uint32_t sbyte = kPadF + head;
  const uint32_t rr = sbyte & 3u;
  u32x4* const ob = (u32x4*)(o0 + head);
  for (uint32_t i = tid; i < nblk; i += 64 * kWv) {
    const uint32_t b0 = head + 16 * i;
    if (hole - b0 < 16u) {
      for (uint32_t q = 0; q < 16; q++)
        if (b0 + q != hole) o0[b0 + q] = sb[b0 + q];
      continue;
    }
    const uint32_t d = (sbyte >> 2) + 4 * i;
    const uint32_t v0 = stg[d], v1 = stg[d + 1], v2 = stg[d + 2], v3 = stg[d + 3], v4 = stg[d + 4];
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(v1, v0, rr);
    v.y = __builtin_amdgcn_alignbyte(v2, v1, rr);
    v.z = __builtin_amdgcn_alignbyte(v3, v2, rr);
    v.w = __builtin_amdgcn_alignbyte(v4, v3, rr);
    ob[i] = v;
  }
  if (body + (uint32_t)tid < n && body + (uint32_t)tid != hole) o0[body + tid] = sb[body + tid];
}

// ---------------------------------------------------------------------------------------------
// 1. Tile kernel: one workgroup per 2048-word tile, in blockIdx order.  The tile publishes its
//    byte count (desc[T] = AGG | bytes) as soon as it is known, stages its packed bytes in LDS,
//    and then looks back over its predecessors' descriptors without waiting: when they are all
//    there it writes its bytes straight to their final offset (desc[T] = INCL | prefix); else it
//    copies them to a slot of a bounded pool (kPackSlots slots, 16-byte aligned) for the
//    placement launch, and with the pool used up it waits for its offset.  Beside that: its
//    byte count, the position of its provisional count byte (if the next tile may change it)
//    and, for the previous tile, the final value of that byte (written by this tile when it
//    writes its own bytes).  The other wait is for the previous tile's exit budget, and only
//    when this tile's first word goes on with the stretch the previous tile ended in; the
//    previous tile publishes it right after its classes when it holds a sync point.  (A tile
//    only waits on lower ones, dispatched before it.)
#ifdef CPK_DIAG
// diagnostic build only: 0 tiles, 1 offset known in time, 2 slot taken, 3 waited for the offset
__device__ unsigned long long g_pdiag[4];
#define CPK_PDIAG(k, v) atomicAdd(&g_pdiag[k], (unsigned long long)(v))
// per-tile timeline of the first kPTimeline tiles (wall clock, 100 MHz): start, byte count
// published, staged, offset or slot known, end; then the outcome (1 in time, 2 slot, 3 waited)
constexpr int kPTimeline = 1 << 16;
__device__ unsigned long long g_ptimeline[kPTimeline * 8];
#define CPK_PSTAMP(k) (pk[k] = wall_clock64())
#else
#define CPK_PSTAMP(k)
#define CPK_PDIAG(k, v)
#endif


// A tile's global loads (one lane's 8 words, its chunk-start bitmap byte, the word before the
// wave / after the tile, the next tile's start flag, the lane's first requested position).
struct TileLoads {
  uint32_t xlo[kK], xhi[kK];
  uint64_t cb0, xw0, nb0, p00;
};

// All issued before any is waited for (vector loads retire in order; the compiler waits for all
// of them right behind a load whose value it moves to an SGPR or at the join behind a load under
// a branch, so uniform values come through scalar loads and lane-varying guards are clamped
// addresses).
__device__ __forceinline__ void tile_loads(const PackTileArgs& a, uint64_t T, int w, int l,
                                           TileLoads& L) {
  const uint64_t N = a.nwords;
  const uint64_t nbitw = (N + 63) >> 6;
  const uint64_t tbase = T * kTW;
  const uint64_t tend = tbase + kTW < N ? tbase + kTW : N;
  const uint64_t wbase = tbase + (uint64_t)kWW * w;
  const uint64_t w0 = wbase + (uint64_t)kK * l;  // the lane's first word
  // word pairs from clamped indices (no branch: a load under a branch gets its own wait at the
  // join), words past the batch then read as zero (the tile kernel runs for N > 2048 words: one
  // tile goes to the direct kernel)
#pragma unroll
  for (int i = 0; i < kK / 2; i++) {
    const uint64_t j = w0 + 2 * i;
    const u32x4 v = *(const u32x4*)(a.words + (j + 2 <= N ? j : N - 2));
    const bool k0 = j < N, k1 = j + 1 < N, sh = j + 2 > N;  // sh: the pair ending at word N - 1
    L.xlo[2 * i] = k0 ? (sh ? v.z : v.x) : 0u;
    L.xhi[2 * i] = k0 ? (sh ? v.w : v.y) : 0u;
    L.xlo[2 * i + 1] = k1 ? v.z : 0u;
    L.xhi[2 * i + 1] = k1 ? v.w : 0u;
  }
  const uint64_t cbi = (wbase >> 6) + (uint64_t)(l >> 3);
  L.cb0 = a.chunk_bits[cbi < nbitw ? cbi : nbitw - 1];
  // lane 0: the word before the wave; the other lanes: the word after the tile (its class
  // decides whether this tile's open run may go on in the next tile)
  const uint64_t xi = l == 0 ? (wbase > 0 ? wbase - 1 : 0) : (tend < N ? tend : N - 1);
  L.xw0 = a.words[xi < N ? xi : N - 1];
  const uint64_t nbi = T + 1 + (uint64_t)opaque_zero();  // the next tile's start byte
  L.nb0 = a.tile_starts[nbi];
  typedef const __attribute__((address_space(4))) uint64_t cu64;
  const uint64_t pidx = a.pos && !a.frame_mode ? *((cu64*)a.tile_first + T) : 0;  // scalar load
  const uint64_t pi = pidx + l;
  L.p00 = (a.pos ? a.pos : a.words)[a.pos && pi <= a.npos ? pi : 0];
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void
pack_tile_kernel(PackTileArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t stg[kSlotDw];
  __shared__ __attribute__((aligned(16))) uint32_t trash[kWv][kTrashDw];
  __shared__ uint64_t sel_tab[256];
  __shared__ uint32_t s_sum[kWv];    // wave summaries (sum_pack)
  __shared__ uint32_t s_bytes[kWv];  // wave byte counts
  __shared__ uint32_t s_sexit[kWv];  // serial mode: exit of each wave
  __shared__ uint32_t s_hole;        // byte of the tile's provisional count (~0: none)
  __shared__ uint64_t s_dst;         // the tile's output offset when resolved in time (~0: not)
  __shared__ uint32_t s_patch;       // previous tile's count byte | its distance before ours << 8
  __shared__ uint64_t s_piece;       // the tile's arena piece (byte offset; ~0: none)

  const int tid = (int)threadIdx.x;
  const int w = (int)uniform32(threadIdx.x >> 6);
  const uint64_t N = a.nwords;
  const uint64_t nbitw = (N + 63) >> 6;
  sel_tab[tid] = make_sel((uint32_t)tid);
  // chunks of 4 consecutive tiles per XCD: a tile's budget and look-back waits mostly stay on
  // its XCD (C2 / C3 / C5 pack_tile -2.0 / -1.6 / -2.7 %; chunks of 16: +1 / +1.4 / +6 %)
  const uint64_t T = xcd_order<4>(blockIdx.x, gridDim.x);
  const int l = lane_id();
#ifdef CPK_DIAG
  uint64_t pk[5] = {0, 0, 0, 0, 0};
  uint32_t pout = 0;
  CPK_PSTAMP(0);
#endif
  if (a.frame_mode) {
    // a single-tile batch: the framing launch's work first (chunk starts, statuses)
    unsigned long long* const cb = (unsigned long long*)a.chunk_bits;
    if (a.frame_mode == 1) {
      for (uint64_t i = tid; i < a.frame_n; i += 64 * kWv)
        frame_message(a.words, a.frame_off, i, N, cb, a.tile_starts, a.frame_status);
    } else {
      if (tid == 0) mark_chunk(cb, a.tile_starts, 0);  // word 0 always starts a chunk
      for (uint64_t i = tid; i < a.frame_n; i += 64 * kWv) {
        const uint64_t p = a.frame_off[i];
        if (p < N && a.frame_off[i + 1] > p) mark_chunk(cb, a.tile_starts, p);
      }
    }
    __syncthreads();  // (the bitmap's atomics are done at the L2; no wave has read it yet)
  }
  TileLoads cur;
  tile_loads(a, T, w, l, cur);
  for (int i = tid; i < kSlotDw / 4; i += 64 * kWv) ((u32x4*)stg)[i] = (u32x4){0, 0, 0, 0};
  const uint64_t tbase = T * kTW;
  const uint64_t tend = tbase + kTW < N ? tbase + kTW : N;
  const uint64_t wbase = tbase + (uint64_t)kWW * w;
  const int nvw = wbase >= N ? 0 : (int)((N - wbase) < (uint64_t)kWW ? (N - wbase) : kWW);
  uint32_t xlo[kK], xhi[kK];
#pragma unroll
  for (int k = 0; k < kK; k++) {
    xlo[k] = cur.xlo[k];
    xhi[k] = cur.xhi[k];
  }
  const uint64_t cbi = (wbase >> 6) + (uint64_t)(l >> 3);
  const uint64_t xw0 = cur.xw0, nb0 = cur.nb0;
  const uint64_t nbi = T + 1 + (uint64_t)opaque_zero();  // the next tile's start byte
  typedef const __attribute__((address_space(4))) uint64_t cu64;
  const uint64_t pidx = a.pos && !a.frame_mode ? *((cu64*)a.tile_first + T) : 0;  // scalar load
  const uint64_t pi = pidx + l;
  const bool pv = a.pos && pi <= a.npos;
  const uint64_t cbw = cbi < nbitw ? cur.cb0 : 0;
  const uint64_t xw = (wbase > 0 || l != 0) ? xw0 : 0;
  const uint64_t p0 = pv ? cur.p00 : ~0ull;

  // ---- classes -------------------------------------------------------------------------
  uint32_t Zm = 0, Rm = 0, Fm = 0, nzA = 0;
  uint32_t tags[kK / 4] = {0, 0};
#pragma unroll
  for (int k = 0; k < kK; k++) {
    const uint32_t tg = tag_of(xlo[k], xhi[k]);
    const uint32_t nz = __popc(tg);
    tags[k >> 2] |= tg << (8 * (k & 3));
    Zm |= (tg == 0 ? 1u : 0u) << k;
    Rm |= (nz >= 7 ? 1u : 0u) << k;
    Fm |= (tg == 0xffu ? 1u : 0u) << k;
    nzA |= nz << (4 * k);
  }
  const int kv = nvw - kK * l;
  const uint32_t V = kv >= kK ? 0xffu : (kv <= 0 ? 0u : ((1u << kv) - 1u));
  Zm &= V;
  Rm &= V;
  Fm &= V;
  // class of the word before the lane: the previous lane's last word (lane 0: word wbase - 1)
  uint32_t zc = shfl32(Zm >> 7, l > 0 ? l - 1 : 0) & 1u;
  uint32_t rc = shfl32(Rm >> 7, l > 0 ? l - 1 : 0) & 1u;
  const uint32_t xtag = tag_of((uint32_t)xw, (uint32_t)(xw >> 32));
  if (l == 0) {
    zc = (wbase > 0 && xw == 0) ? 1u : 0u;
    rc = (wbase > 0 && __popc(xtag) >= 7) ? 1u : 0u;
  }
  const uint32_t C = (uint32_t)(cbw >> (8 * (l & 7))) & 0xffu;
  const uint32_t O = V & ~Zm & ~Rm;
  const uint32_t SY =
      (C | O | (Zm & ~((Zm << 1) | zc)) | (Rm & ~((Rm << 1) | rc)) | ~V) & 0xffu;
  const bool lv = kv >= kK;

  const uint64_t hs = ballot(SY != 0);
  const bool simple = SY != 0 || Zm == 0xffu || Fm == 0xffu;
  const uint64_t nonsimple = ballot(!simple && kv > 0);
  const Cov c0 = cover8(Zm, Fm, Rm, SY, 0u, lv);  // exits of the lanes with a sync point
  const uint32_t fs = SY ? (uint32_t)__builtin_ctz(SY) : 8u;
  // first sync after the lane, wave-relative
  const uint64_t above = hs & ~mask_le(l);
  const int ja = above ? lowest_bit(above) : 0;
  const uint32_t fsa = shfl32(fs, ja);
  // the tile's exit, with the raw bit (the run open at the tile end is a raw run when the
  // tile's last word is not zero), published by the last wave as soon as it is known: right here
  // when the last wave holds a sync point (its exit is then the tile's, whatever the entry)
  uint32_t t_exit = 0;
  auto publish_state = [&](uint32_t ex) {
    const uint32_t lz = readlane32(Zm >> 7, 63) & 1u;
    t_exit = ex | ((ex != 0 && !lz) ? 0x100u : 0u);
    if (l == 0) store_agent32(a.state + T, 0x80000000u | t_exit);
  };
  {
    const uint32_t exit0 = hs != 0 ? wave_exit(0u, hs, nonsimple, c0.b_out, Zm, Fm) : 0u;
    if (w == kWv - 1 && hs != 0) publish_state(exit0);
    const int L0 = hs ? lowest_bit(hs) : 0;
    const uint32_t fsl = shfl32(fs, L0);
    const uint32_t fsw = hs ? (uint32_t)(kK * L0) + fsl : (uint32_t)kWW;
    if (l == 0) s_sum[w] = sum_pack(hs != 0, nonsimple == 0, fsw, exit0);
  }
  // the word after the tile: a sync point there closes this tile's open run at its end
  bool next_sync = true;
  if (w == kWv - 1) {
    const uint32_t ntag = tag_of((uint32_t)xw0, (uint32_t)(xw0 >> 32));
    const uint32_t nnz = __popc(ntag);
    const bool nC = nb0 != 0;
    const uint32_t lastZ = readlane32(Zm >> 7, 63) & 1u, lastR = readlane32(Rm >> 7, 63) & 1u;
    const bool nZ = ntag == 0, nR = nnz >= 7;
    const bool ns = nC || (!nZ && !nR) || (nZ && !lastZ) || (nR && !lastR);
    next_sync = tend >= N || readlane32(ns ? 1u : 0u, 63) != 0;
  }
  lds_barrier();  // ---- A: wave summaries ---------------------------------------------
  // the chunk-start bits are zero at rest: this tile clears what only it reads (its bitmap words;
  // the bit of its successor's first word, read here and nowhere else)
  if ((l & 7) == 0 && cbi < nbitw && cbw != 0) a.chunk_bits[cbi] = (uint64_t)opaque_zero();
  if (w == kWv - 1 && l == 0 && nb0) a.tile_starts[nbi] = 0;

  uint32_t sm[kWv];
#pragma unroll
  for (int v = 0; v < kWv; v++) sm[v] = uniform32(s_sum[v]);
  bool serial = false;
#pragma unroll
  for (int v = 0; v < kWv; v++) serial |= !sum_sync(sm[v]) && !sum_simple(sm[v]);
  const bool first_sync = sum_fsw(sm[0]) == 0;
  // the tile's entry budget (| 0x100: the run is a raw run), waited for only when the tile's
  // first word goes on with the stretch the previous tile ended in
#ifdef CPK_DIAG
  uint64_t pwait = 0;  // (diagnostic) wall ticks wave 0 waited for the previous tile's exit budget
#endif
  auto tile_entry = [&]() -> uint32_t {
    if (first_sync || T == 0) return 0u;
#ifdef CPK_ABLATE_NOENTRY
    return 0u;  // (ablation only: wrong bytes) no wait for the previous tile's exit budget
#endif
#ifdef CPK_DIAG
    const uint64_t w0c = wall_clock64();
    const uint32_t v = wait_nonzero32(a.state + T - 1, a.err) & 0x1ffu;
    pwait += wall_clock64() - w0c;
    return v;
#else
    return wait_nonzero32(a.state + T - 1, a.err) & 0x1ffu;
#endif
  };
  const bool last_sync = sum_sync(sm[kWv - 1]);  // the exit went out before barrier A
  uint32_t bT = 0, bw = 0;
  bool have_bT = false;
  if (!serial) {
    // the last wave with a sync point fixes the exit; the one-kind sync-free waves behind it map
    // budgets to themselves (512 words = 2 runs of 256)
    int js = -1;
#pragma unroll
    for (int v = 0; v < kWv; v++)
      if (sum_sync(sm[v])) js = v;
    if (js >= 0 && !last_sync && w == kWv - 1) publish_state(sum_exit(sm[js]));
    // this wave's entry: the nearest lower wave with a sync point, else the tile's entry
    int jb = -1;
#pragma unroll
    for (int v = 0; v < kWv; v++)
      if (v < w && sum_sync(sm[v])) jb = v;
    if (jb >= 0) {
      bw = sum_exit(sm[jb]);
    } else {
      bT = tile_entry();
      have_bT = true;
      bw = bT & 0xffu;
    }
    if (js < 0 && w == kWv - 1) publish_state(bw);
  } else {
    // rare: a sync-free wave that needs the scalar composition -- the waves in order
#pragma nounroll
    for (int v = 0; v < kWv; v++) {
      if (w == v) {
        if (v == 0) {
          bT = tile_entry();
          have_bT = true;
          bw = bT & 0xffu;
        } else {
          bw = uniform32(s_sexit[v - 1]);
        }
        const uint32_t ex =
            hs != 0 ? sum_exit(sm[v]) : wave_exit(bw, hs, nonsimple, c0.b_out, Zm, Fm);
        if (l == 0) s_sexit[v] = ex;
        if (v == kWv - 1 && !last_sync) publish_state(ex);
      }
      lds_barrier();
    }
  }
  // wave 0 finishes the previous tile's open run: it needs the entry
  if (w == 0 && !have_bT) bT = tile_entry();

  // ---- coverage, bytes, offsets ----------------------------------------------------------
  const uint32_t ent = lane_entries(bw, hs, nonsimple, c0.b_out, Zm, Fm);
  const Cov cv = cover8(Zm, Fm, Rm, SY, ent, lv);
  const uint32_t heads = V & ~cv.cov;
  const uint32_t rh = cv.zh | cv.fh;
  const uint32_t crf = cv.cov & Rm & ~Fm;
  const uint32_t nzsum = (((nzA & 0x0f0f0f0fu) + ((nzA >> 4) & 0x0f0f0f0fu)) * 0x01010101u) >> 24;
  const uint32_t bytes = nzsum + __popc(heads) + __popc(rh) + __popc(crf);
  const uint32_t incl = wave_incl_sum32(bytes);
  const uint32_t loff = incl - bytes;
  if (l == 63) s_bytes[w] = incl;
  lds_barrier();  // ---- B: wave byte counts -------------------------------------------

  uint32_t woff = 0, agg = 0, s0 = (uint32_t)kTW;
#pragma unroll
  for (int v = 0; v < kWv; v++) {
    const uint32_t bv = uniform32(s_bytes[v]);
    if (v < w) woff += bv;
    agg += bv;
    const uint32_t fv = sum_fsw(sm[v]);
    if (fv < (uint32_t)kWW && (uint32_t)(kWW * v) + fv < s0) s0 = (uint32_t)(kWW * v) + fv;
  }
  // next sync point after this lane's last word, tile-relative (the tile end when none)
  uint32_t nsl = (uint32_t)kTW;
  if (above) {
    nsl = (uint32_t)(kWW * w + kK * ja) + fsa;
  } else {
#pragma unroll
    for (int v = kWv - 1; v >= 0; v--)
      if (v > w && sum_fsw(sm[v]) < (uint32_t)kWW) nsl = (uint32_t)(kWW * v) + sum_fsw(sm[v]);
  }
  if (l == 0) {
    if (w == kWv - 1) {
      a.tile_bytes[T] = agg;
      // The run open at the tile end, when the word after the tile goes on with its stretch:
      // its count byte (written here as if the batch ended at the tile end) is final only
      // once the next tile has seen where the run stops.
      const uint32_t b = t_exit & 0xffu;
      const uint32_t hole = (b != 0 && !next_sync)
                                ? agg - 1u - ((t_exit & 0x100u) ? 8u * (255u - b) : 0u)
                                : 0xffffffffu;
      a.thole[T] = hole;
      s_hole = hole;
    }
    if (w == 0) {
      // the previous tile's open run ends in this tile: its count byte, and how far before this
      // tile's first byte it lies
      const uint32_t b = bT & 0xffu;
      const uint32_t tpv = b != 0 ? 0x100u | (255u - b + (s0 < b ? s0 : b)) : 0u;
      a.tpatch[T] = tpv;
      s_patch = tpv ? (tpv & 0xffu) | ((1u + ((bT & 0x100u) ? 8u * (255u - b) : 0u)) << 8) : 0u;
      // the tile's byte count, for the look-back of the tiles after it (tile 0: its prefix too)
      store_agent(a.desc + T, (T == 0 ? kDescIncl : kDescAgg) | agg);
    }
  }
#ifdef CPK_DIAG
  CPK_PSTAMP(1);
#endif

  // ---- requested positions (message starts) in this wave: bytes before them in the tile ---
  if (a.pos) {
    const uint64_t wend = wbase + kWW < tend ? wbase + kWW : tend;
    uint64_t idx = pidx;
    for (bool first = true;; first = false) {
      const uint64_t i = idx + l;
      const uint64_t p = first ? p0 : (i <= a.npos ? a.pos[i] : ~0ull);
      const bool in_t = p >= tbase && p < tend;
      const bool in_w = p >= wbase && p < wend;
      const uint32_t rel = in_w ? (uint32_t)(p - wbase) : 0u;
      const int L = (int)(rel >> 3);
      const uint32_t k = rel & 7u;
      const uint32_t oL = shfl32(loff, L), hL = shfl32(heads, L), rL = shfl32(rh, L);
      const uint32_t cL = shfl32(crf, L), aL = shfl32(nzA, L);
      const uint32_t mk = (1u << k) - 1u;
      const uint32_t an = aL & ((1u << (4 * k)) - 1u);
      const uint32_t nb = (((an & 0x0f0f0f0fu) + ((an >> 4) & 0x0f0f0f0fu)) * 0x01010101u) >> 24;
      const uint32_t before = nb + __popc(hL & mk) + __popc(rL & mk) + __popc(cL & mk);
      if (in_w) a.pos_out[i] = woff + oL + before;  // tile-relative; placed by pack_place
      const uint64_t inm = ballot(in_t);
      idx += __popcll(inm);
      if (inm != ~0ull) break;
    }
  }

  // ---- emission: records OR-ed into the staging slot at their own byte offsets ------------
  const uint32_t nwin = agg <= kCap ? 1u : (agg + kCap - 1) / kCap;
  uint32_t* const wtr = trash[w] + l;
  for (uint32_t win = 0; win < nwin; win++) {
    const uint32_t wlo = win * kCap;
    const uint32_t whi = wlo + kCap;
    const bool windowed = nwin > 1;
    // the words pass through an opaque move per window, so nothing of the record bodies is
    // hoisted out of this (almost always single-trip) loop: 8 words' worth of records held live
    // at once cost the kernel its occupancy
#pragma unroll
    for (int k = 0; k < kK; k++) asm volatile("" : "+v"(xlo[k]), "+v"(xhi[k]));
    uint32_t ecov = cv.cov, ezh = cv.zh, efh = cv.fh, eSY = SY, eR = Rm, enz = nzA, ensl = nsl;
    uint32_t et0 = tags[0], et1 = tags[1];
    asm volatile("" : "+v"(ecov), "+v"(ezh), "+v"(efh), "+v"(eSY), "+v"(eR), "+v"(enz));
    asm volatile("" : "+v"(ensl), "+v"(et0), "+v"(et1));
    const uint32_t etags[2] = {et0, et1};
    uint32_t o = woff + loff;  // tile byte offset of the lane's next record
    const uint32_t lbase = (uint32_t)(kWW * w + kK * l);
    uint64_t sel_next = sel_tab[etags[0] & 0xffu];
#ifdef CPK_ABLATE_EMIT
    constexpr int kEmitK = CPK_ABLATE_EMIT;  // (ablation only: wrong bytes) words emitted per lane
#else
    constexpr int kEmitK = kK;
#endif
#pragma unroll
    for (int k = 0; k < kEmitK; k++) {
      const uint32_t lo = xlo[k], hi = xhi[k];
      const uint32_t tg = (etags[k >> 2] >> (8 * (k & 3))) & 0xffu;
      const uint64_t sel = sel_next;
      if (k + 1 < kK) sel_next = sel_tab[(etags[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xffu];
      const uint32_t nz = (enz >> (4 * k)) & 15u;
      const bool cvk = (ecov >> k) & 1, zhk = (ezh >> k) & 1, fhk = (efh >> k) & 1;
      const uint32_t aft = eSY & (0xfeu << k);
      const uint32_t ns = aft ? lbase + (uint32_t)__builtin_ctz(aft) : ensl;
      const uint32_t c8 = min(ns - (lbase + (uint32_t)k) - 1u, 255u) << 8;
      uint32_t r0 = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel) | tg | (zhk ? c8 : 0u);
      uint32_t r1 = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
      uint32_t r2 = fhk ? ((hi >> 24) | c8) : 0u;
      uint32_t L = 1u + nz + ((zhk || fhk) ? 1u : 0u);
      if (cvk) {
        r0 = lo;
        r1 = hi;
        r2 = 0;
        L = ((eR >> k) & 1) ? 8u : 0u;
      }
      bool put = L != 0;
      if (windowed) put = put && o < whi && o + L > wlo;
      const uint32_t so = kPadF + o - wlo;  // slot byte (in range whenever put)
      const uint32_t sh = 8u * (so & 3u);
      // an empty record ORs into the lane's trash window (overlapping windows: the 32 lanes of a
      // bank group hit 32 banks)
      uint32_t* const wp = put ? stg + (so >> 2) : wtr;
      const uint64_t q01 = (((uint64_t)r1 << 32) | r0) << sh;
      const uint64_t q12 = (((uint64_t)r2 << 32) | r1) << sh;
      const uint32_t w3 = (uint32_t)(((uint64_t)r2 << sh) >> 32);
      atomicOr(wp, (uint32_t)q01);
      atomicOr(wp + 1, (uint32_t)(q01 >> 32));
      atomicOr(wp + 2, (uint32_t)(q12 >> 32));
      if (ballot(w3 != 0)) atomicOr(wp + 3, w3);
      o += L;
      __builtin_amdgcn_sched_barrier(0);
    }
    lds_barrier();  // ---- C: staged ------------------------------------------------------
#ifdef CPK_DIAG
    if (win == 0) CPK_PSTAMP(2);
#endif
    if (win == 0) {
      // The tile's offset, if the tiles before it have all published their byte counts by now
      // (no waiting): then its bytes go straight to the output.  Otherwise a tile of few bytes
      // (sparse words: at most kArenaTile) goes to a piece of the byte arena -- exactly its size,
      // taken by one atomic add -- for the placement launch, where copying it costs less than
      // holding the CU while it waits; a denser tile (or one finding the arena used up, or one of
      // more bytes than one staging window) waits for its offset: copying it twice costs more
      // than the wait (only ever on lower tiles, which publish their byte counts before anything
      // they could wait for).
      if (w == 0) {
        uint64_t ex = 0;
        bool ok = T == 0, wait = windowed || agg > kArenaTile;
        uint64_t piece = ~0ull;
        while (!ok) {
          ok = pack_lookback(a.desc, T, &ex, wait, a.err);
          if (ok || wait) break;
          const uint64_t need = ((uint64_t)agg + 15u) & ~15ull;
          if (l == 0) piece = atomicAdd((unsigned long long*)a.arena_next, (unsigned long long)need);
          piece = readlane64(piece, 0);
          if (piece + need <= a.arena_cap) break;
          piece = ~0ull;  // (the arena is full: the counter stays past its end)
          wait = true;
        }
        if (l == 0) {
          CPK_PDIAG(0, 1);
          CPK_PDIAG(wait ? 3 : (piece != ~0ull ? 2 : 1), 1);
#ifdef CPK_DIAG
          pout = wait ? 3 : (piece != ~0ull ? 2 : 1);
#endif
        }
        ok = ok && ex + agg <= a.out_capacity;  // (too small an output: placement raises it)
        if (l == 0) {
          if (ok && T != 0) store_agent(a.desc + T, kDescIncl | (ex + agg));
          a.tpiece[T] = piece;  // (~0: written straight out, or not at all)
          s_dst = ok ? ex : ~0ull;
          s_piece = piece;
        }
      }
      lds_barrier();  // ---- D: offset or slot ---------------------------------------------
#ifdef CPK_DIAG
      CPK_PSTAMP(3);
#endif
    }
    const uint64_t ex = uniform64(s_dst);
    if (ex != ~0ull) {
      const uint32_t nw = (whi < agg ? whi : agg) - wlo;
      copy_out_final(stg, nw, a.out + ex + wlo, uniform32(s_hole) - wlo, tid);
      // the previous tile's provisional count byte, now final (its tile left it out)
      const uint32_t pt = uniform32(s_patch);
      if (win == 0 && tid == 0 && pt != 0) a.out[ex - (pt >> 8)] = (uint8_t)pt;
    } else if (!windowed) {
      const uint64_t piece = uniform64(s_piece);
      if (piece != ~0ull) {
        // the tile's bytes to its arena piece: aligned 16-byte copies
        u32x4* const dst = (u32x4*)(a.arena + piece);
        const uint32_t n16 = (agg + 15u) >> 4;
        for (uint32_t i = tid + opaque_zero(); i < n16; i += 64 * kWv)
          dst[i] = ((const u32x4*)stg)[1 + i];
      }
    }
    if (windowed) {
      lds_barrier();
      for (int i = tid; i < kSlotDw / 4; i += 64 * kWv) ((u32x4*)stg)[i] = (u32x4){0, 0, 0, 0};
      lds_barrier();
    }
  }
#ifdef CPK_DIAG
  CPK_PSTAMP(4);
  if (tid == 0 && T < (uint64_t)kPTimeline) {
    for (int k = 0; k < 5; k++) g_ptimeline[8 * T + k] = pk[k];
    g_ptimeline[8 * T + 5] = pout;
    g_ptimeline[8 * T + 6] = agg;
    g_ptimeline[8 * T + 7] = pwait;  // wave 0's wait for the previous tile's exit budget
  }
#endif
  if (a.frame_mode) {
    // (a single-tile batch has no placement launch) the total for the positions at the batch
    // end; a tile the output cannot hold raises the capacity error here
    if (tid == 0 && uniform64(s_dst) == ~0ull) raise_error(a.err, kErrCapacity);
    if (a.pos)
      for (uint64_t i = tid; i <= a.npos; i += 64 * kWv)
        if (a.pos[i] >= N) a.pos_out[i] = agg;
    if (a.total_out && tid == 0) *a.total_out = agg;
    // the call's error word for the host, last (this launch is the whole call; tid 0 raised the
    // only error a single tile can): every wave's stores done, then a system-scope release
    if (a.err_host) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __threadfence_system();
        __hip_atomic_store(a.err_host, load_agent32(a.err), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 2. Placement: one workgroup per group of kPlaceGroup consecutive tiles.  The offsets come from a
//    scan of the tile byte counts (every tile's descriptor holds its count, or its inclusive
//    prefix when the tile kernel resolved it): a group holding such an inclusive prefix knows
//    every offset of the group from it at once (forward and backward from that tile); a group
//    without one looks back over the groups before it (decoupled look-back on group descriptors,
//    zero at rest).  Then the tiles whose bytes wait in the arena are copied to their offsets --
//    one wave per tile, 16-byte stores -- with the count byte of a run the next tile closed, and
//    the requested positions become output offsets.
constexpr int kPlaceGroup = (int)kPackPlaceGroup;  // tiles per workgroup (lane l of wave 0:
                                                   // tile 64g + l)

__global__ __launch_bounds__(256) void pack_place_kernel(PackTileArgs a) {
  __shared__ uint64_t s_off[kPlaceGroup];
  __shared__ uint64_t s_piece[kPlaceGroup];
  __shared__ uint32_t s_n[kPlaceGroup];
  __shared__ uint32_t s_list[kPlaceGroup];  // group-relative indices of the tiles in the arena
  __shared__ uint32_t s_narena;
  __shared__ uint64_t s_pos[2];  // the group's requested positions: [s_pos[0], s_pos[1])
  // the count-byte handoffs around the group's tiles, read with the group's descriptors: thole
  // of tiles T0 - 1 .. T0 + 63 (s_hole[j + 1]: tile T0 + j), tpatch of T0 .. T0 + 64, and the
  // byte count of tile T0 - 1 (a tile's copy then waits on its source bytes alone)
  __shared__ uint32_t s_hole[kPlaceGroup + 1];
  __shared__ uint32_t s_patch[kPlaceGroup + 1];
  __shared__ uint32_t s_nprev;
  const int tid = (int)threadIdx.x;
  const int l = lane_id();
  const int w = (int)uniform32(threadIdx.x >> 6);
  const uint64_t g = blockIdx.x;
  const uint64_t T0 = g * kPlaceGroup;
  if (w == 0) {
    const uint64_t T = T0 + (uint64_t)l;
    const bool in = l < kPlaceGroup && T < a.ntiles;
    const uint64_t n = in ? a.tile_bytes[T] : 0ull;
    const uint64_t dT = in ? load_agent(a.desc + T) : 0ull;
    const uint64_t piece = in ? a.tpiece[T] : ~0ull;
    const uint32_t th = in ? a.thole[T] : 0xffffffffu;
    const uint32_t tp = in ? a.tpatch[T] : 0u;
    const uint64_t T64 = T0 + kPlaceGroup;
    const uint32_t th_m1 = (l == 0 && T0 > 0) ? a.thole[T0 - 1] : 0xffffffffu;
    const uint32_t nb_m1 = (l == 0 && T0 > 0) ? (uint32_t)a.tile_bytes[T0 - 1] : 0u;
    const uint32_t tp_64 = (l == kPlaceGroup - 1 && T64 < a.ntiles) ? a.tpatch[T64] : 0u;
    // the group's positions: from its first tile's first to the next group's first
    const bool pl = a.pos && l < 2;
    const uint64_t pT = T0 + (uint64_t)l * kPlaceGroup;
    const uint64_t pf = pl ? (pT < a.ntiles ? a.tile_first[pT] : a.npos + 1) : 0ull;
    const bool incl = in && (dT & kDescFlags) == kDescIncl;
    const uint64_t inc = wave_incl_sum64(n);  // bytes of the group's tiles up to this one
    const uint64_t gsum = readlane64(inc, kPlaceGroup - 1);
    // the last tile of the group whose inclusive prefix the tile kernel published
    const uint64_t ib = ballot(incl);
    uint64_t base;  // bytes before the group
    if (ib) {
      const int k = highest_bit(ib);
      base = readlane64((dT & kDescValue) - inc, k);
      if (l == 0) store_agent(a.gdesc + g, kDescIncl | (base + gsum));
    } else {
      if (l == 0) store_agent(a.gdesc + g, (g == 0 ? kDescIncl : kDescAgg) | gsum);
      base = 0;
      if (g > 0) {
        pack_lookback(a.gdesc, g, &base, true, a.err);
        if (l == 0) store_agent(a.gdesc + g, kDescIncl | (base + gsum));
      }
    }
    const uint64_t off = base + inc - n;
    const bool arena = in && piece != ~0ull && n != 0 && off + n <= a.out_capacity;
    const uint64_t am = ballot(arena);
    if (in) {
      s_off[l] = off;
      s_n[l] = (uint32_t)n;
      s_piece[l] = piece;
      if (off + n > a.out_capacity) raise_error(a.err, kErrCapacity);
    }
    if (arena) s_list[__popcll(am & ((1ull << l) - 1ull))] = (uint32_t)l;
    if (l == 0) s_narena = (uint32_t)__popcll(am);
    if (pl) s_pos[l] = pf;
    if (l < kPlaceGroup) {
      s_hole[l + 1] = th;
      s_patch[l] = tp;
    }
    if (l == 0) {
      s_hole[0] = th_m1;
      s_nprev = nb_m1;
    }
    if (l == kPlaceGroup - 1) s_patch[kPlaceGroup] = tp_64;
    if (in && T + 1 == a.ntiles && a.total_out) *a.total_out = base + inc;
  }
  __syncthreads();
  // requested positions: tile-relative offsets (pack_tile) + the tile's output offset; a position
  // belongs to the tile holding its word, positions at or past the batch end (the last tile's
  // share) take the total
  if (a.pos) {
    const uint64_t i1 = s_pos[1];
    for (uint64_t i = s_pos[0] + (uint64_t)tid; i < i1; i += 256) {
      // both loads issued before either is waited for (the tile-relative offset does not wait
      // for the position)
      const uint64_t p = a.pos[i];
      const uint64_t rel = a.pos_out[i];
      const uint64_t T = min(p / kPackTileWords, a.ntiles - 1);
      const uint32_t j = (uint32_t)(T - T0);
      if (j >= (uint32_t)kPlaceGroup) continue;  // (unsorted positions: not this group's)
      a.pos_out[i] = (T + 1 == a.ntiles && p >= a.nwords) ? s_off[j] + s_n[j] : rel + s_off[j];
    }
  }
  // the tiles in the arena: one wave per tile
  const uint32_t na = s_narena;
  for (uint32_t q = (uint32_t)w; q < na; q += 4) {
    const uint32_t j = s_list[q];
    const uint64_t T = T0 + j;
    const uint64_t off = s_off[j];
    const uint32_t n = s_n[j];
    {
      // the previous tile's count byte that this tile finishes (the previous tile may have left
      // it out, having written its bytes itself)
      if (T > 0 && l == 0) {
        const uint32_t ph = s_hole[j], pp = s_patch[j];
        const uint32_t nprev = j ? s_n[j - 1] : s_nprev;
        if (ph != 0xffffffffu && pp) a.out[off - nprev + ph] = (uint8_t)pp;
      }
      // count byte patched by the next tile (position, value) -- wave-uniform
      const uint32_t hole = T + 1 < a.ntiles ? s_hole[j + 1] : 0xffffffffu;
      const uint32_t pv = hole != 0xffffffffu ? s_patch[j + 1] : 0u;
      const uint8_t* const src = a.arena + s_piece[j];
      uint8_t* const o0 = a.out + off;
      const uint64_t A0 = (uint64_t)(uintptr_t)o0;
      const uint64_t A1 = A0 + n;
      const uint64_t al = (A0 + 15) & ~15ull;
      const uint32_t head = (uint32_t)((al < A1 ? al : A1) - A0);  // bytes before 16-byte alignment
      auto byte_at = [&](uint32_t q) -> uint8_t {
        const uint8_t v = src[q];
        return (pv && q == hole) ? (uint8_t)pv : v;
      };
      if ((uint32_t)l < head) o0[l] = byte_at(l);
      if (A1 > al) {
        const uint32_t body = (uint32_t)((A1 & ~15ull) - A0);
        const uint32_t nblk = (body - head) >> 4;
        // output block i = source bytes [head + 16i, head + 16i + 16): source dwords from
        // (head >> 2) + 4i, shifted by head & 3 bytes
        const uint32_t rr = head & 3u;
        const uint32_t* const s32 = (const uint32_t*)src;
        u32x4* const ob = (u32x4*)(o0 + head);
        for (uint32_t i = l; i < nblk; i += 64) {
          const uint32_t d = (head >> 2) + 4 * i;
          const uint32_t v0 = s32[d], v1 = s32[d + 1], v2 = s32[d + 2], v3 = s32[d + 3],
                         v4 = s32[d + 4];
          u32x4 v;
          v.x = __builtin_amdgcn_alignbyte(v1, v0, rr);
          v.y = __builtin_amdgcn_alignbyte(v2, v1, rr);
          v.z = __builtin_amdgcn_alignbyte(v3, v2, rr);
          v.w = __builtin_amdgcn_alignbyte(v4, v3, rr);
          const uint32_t b0 = head + 16 * i;
          if (pv && hole >= b0 && hole < b0 + 16) {
            const uint32_t q = hole - b0, sh = 8 * (q & 3), m = ~(0xffu << sh),
                           x = (pv & 0xffu) << sh;
            if (q < 4) v.x = (v.x & m) | x;
            else if (q < 8) v.y = (v.y & m) | x;
            else if (q < 12) v.z = (v.z & m) | x;
            else v.w = (v.w & m) | x;
          }
          ob[i] = v;
        }
        if (body + (uint32_t)l < n) o0[body + l] = byte_at(body + l);
      }
    }
  }
  (void)tid;
}

}  // namespace

hipError_t launch_pack_tiles(const PackTileArgs& a, hipStream_t stream) {
  if (a.ntiles == 0) return hipSuccess;
  if (a.ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  pack_tile_kernel<<<(unsigned)a.ntiles, 256, 0, stream>>>(a);
  return hipGetLastError();
}

hipError_t launch_pack_place(const PackTileArgs& a, hipStream_t stream) {
  if (a.ntiles == 0) return hipSuccess;
  pack_place_kernel<<<(unsigned)pack_place_groups(a.ntiles), 256, 0, stream>>>(a);
  return hipGetLastError();
}

}  // namespace cpk

#ifdef CPK_DIAG
// diagnostic build only: copies out (and zeroes) the pack timeline of the first n tiles
extern "C" int cpk_debug_ptimeline(uint64_t* out, int n) {
  if (n > cpk::kPTimeline) n = cpk::kPTimeline;
  if (hipDeviceSynchronize() != hipSuccess) return 10;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cpk::g_ptimeline), (size_t)n * 64) != hipSuccess) return 10;
  static uint64_t z[cpk::kPTimeline * 8];
  if (hipMemcpyToSymbol(HIP_SYMBOL(cpk::g_ptimeline), z, sizeof z) != hipSuccess) return 10;
  return 0;
}

extern "C" int cpk_debug_pdiag(uint64_t* out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return 10;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cpk::g_pdiag), 4 * sizeof(uint64_t)) != hipSuccess) return 10;
  if (reset) {
    const uint64_t z[4] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(cpk::g_pdiag), z, sizeof z) != hipSuccess) return 10;
  }
  return 0;
}
#endif
