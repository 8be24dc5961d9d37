// cpk_pack3.hip -- lane-serial pack kernel (gfx950).
//
// Same output as pack_tiles_kernel (cpk_pack.hip; functional spec PackedOutputStream::write,
// serialize-packed.c++:307-431, once per chunk) with the work laid out the other way round: a
// tile of 1024 words is 64 lanes x 16 CONSECUTIVE words, so every lane encodes its own stretch
// of the chunk serially and the wave-level work shrinks to a handful of 16-bit mask operations
// per lane and one prefix sum per tile.
//
//   classes   per word: tag byte, Z (all zero), R (<= 1 zero byte), F (no zero byte), as 16-bit
//             lane masks; sync points (chunk starts, O words, family changes) as in cpk_pack.hip
//   coverage  per lane, from its entry budget b (words the run open before the lane may still
//             cover): the same carry-add mask algebra as resolve_step, on 16 words.  A run never
//             closes inside 16 words (255 > 15), so a lane's exit budget depends on b only when
//             the lane has no sync point at all -- and then it is (b - 16) mod 256 for a zero
//             stretch or a stretch of F words (a head every 256 words).  Entry budgets across
//             lanes follow in closed form from the nearest lane with a sync point; other lanes
//             (a word stretch with a non-F word and no sync for 16 words) take a scalar pass.
//   bytes     per lane: sum(nz) + heads + run heads + covered words with one zero byte; one
//             wave prefix sum gives each lane's byte offset in the tile
//   emission  each lane appends its records to the wave's LDS staging area as a byte stream
//             (dword stores; the two dwords a lane may share with its neighbours are OR-ed)
//   tiles     the run budget crosses tiles through state[] (published early when the tile has a
//             sync point), output offsets through the two-level decoupled look-back; the staged
//             bytes are stored with 16-byte stores.
//   waves     persistent; a wave counts its next tile before it does the previous tile's
//             look-back and stores, so the look-back finds its predecessors published (with one
//             wave per tile and no deferral the look-back was half of every wave's lifetime).
//
// Measured against the step-major kernel (cpk_pack.hip) on MI355X: C2 0.209 -> 0.171 ms, C3
// 3.94 -> 2.65 ms, C4 10.5 -> 10.5 ms (PMC: ~1.9k VALU + 0.5k SALU per 1024-word tile, against
// ~4.6k + 3.8k).
#include <stdlib.h>

#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kK = 16;                 // words per lane
constexpr int kT = 64 * kK;            // words per tile
// staging: 16-byte pad, the records of a tile (<= 10 bytes per word: a lone F word chunk), pads;
// then one trash dword per lane for the stores a lane does not need.
constexpr int kStgCap = 10 * kT;
constexpr int kSlotDw = (16 + kStgCap + 48) / 4;  // the staging slot, in dwords
constexpr int kTrashDw = 64 + 4;                   // trash windows behind the slot

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

__device__ __forceinline__ int hi_bit16(uint32_t m) { return m ? 31 - __clz(m) : -1; }

struct Cov {
  uint32_t cov, zh, fh;  // covered words, zero-run heads, raw-run heads
  uint32_t b_out;        // budget leaving the lane
};

// Coverage of one lane's 16 words for entry budget b (resolve_step in cpk_pack.hip, 16 wide).
__device__ __forceinline__ Cov cover16(uint32_t Z, uint32_t F, uint32_t R, uint32_t SY, uint32_t b,
                                       bool last_valid) {
  const uint32_t NS = ~SY & 0xffffu;
  const uint32_t LM = NS & (SY - 1u);                      // lead: words before the first sync
  const uint32_t BM = b >= 16u ? 0xffffu : ((1u << b) - 1u);
  const uint32_t lead_cov = BM & LM;
  const uint32_t zlead = (BM + 1u) & LM & Z;               // zero lead: next head at word b
  const uint32_t Feff = F & ~lead_cov;
  const uint32_t G = (Feff << 1) & NS;
  const uint32_t fill = ((((NS + G) ^ NS) & NS) | G) & 0xffffu;  // after an F head, same segment
  Cov c;
  c.fh = Feff & ~fill;
  c.zh = (Z & SY) | zlead;
  c.cov = (R & (fill | lead_cov)) | (Z & ~c.zh);
  c.b_out = 0;
  if (last_valid) {
    const int st = hi_bit16(SY);
    const int h = hi_bit16(c.zh | c.fh);
    if (h >= 0 && h >= st) c.b_out = 240u + (uint32_t)h;
    else if (SY == 0 && b > 15u) c.b_out = b - 16u;
  }
  return c;
}

// Entry budget of every lane given the tile's entry budget bt: lanes with a sync point pass on
// their own exit (ex); a run of sync-free lanes takes 16 words each, (b - 16) mod 256.  When a
// sync-free lane is a word stretch with a non-F word, its exit is not of that form: a scalar pass
// over the lanes then composes the exact per-lane functions.
__device__ __forceinline__ uint32_t lane_entries(uint32_t bt, uint64_t hs, uint64_t nonsimple,
                                                 uint32_t ex, uint32_t Z, uint32_t F) {
  const int l = lane_id();
  if (nonsimple == 0) {
    const uint64_t below = hs & mask_lt(l);
    const int j = highest_bit(below);  // -1: no sync lane below
    const uint32_t ej = shfl32(ex, j < 0 ? 0 : j);
    const uint32_t base = j < 0 ? bt : ej;
    const uint32_t d = (uint32_t)(l - 1 - j);  // sync-free lanes in between
    return (base - 16u * d) & 0xffu;
  }
  uint32_t e = 0;
  uint32_t b = bt;
  for (int L = 0; L < 64; L++) {
    if (l == L) e = b;
    if ((hs >> L) & 1) {
      b = readlane32(ex, L);
    } else {
      const uint32_t zl = readlane32(Z, L), fl = readlane32(F, L);
      if (zl == 0xffffu || b >= 16u) {
        b = (b - 16u) & 0xffu;
      } else {
        const uint32_t fm = fl >> b;
        b = fm ? 240u + b + (uint32_t)__builtin_ctz(fm) : 0u;
      }
    }
  }
  return e;
}

// Three-level decoupled look-back: tiles, groups of 64 tiles (gdesc), units of 64 groups
// (hdesc).  Every level is published as an aggregate as soon as its tiles have counted, so a
// tile needs at most one round per level (plus rounds over earlier units far behind the
// inclusive front) -- with one tile per wave, thousands of tiles are in flight and the front of
// inclusive prefixes lags far behind the newest tiles.
// Staged bytes [16, 16 + n) of a slot -> out + dst with 16-byte stores; the slot is re-zeroed.
__device__ __forceinline__ void flush_slot(const PackTileArgs& a, uint32_t* stg, uint64_t dst,
                                           uint32_t n) {
  const int l = lane_id();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const uint8_t* const sb = (const uint8_t*)stg;
  if (n) {
    // global pointers (a.out + offset), never through an integer: a pointer rebuilt from an
    // integer is generic, and flat stores count against lgkmcnt, so every LDS wait behind them
    // (the emission that follows) would have to wait for the stores as well
    uint8_t* const o0 = a.out + dst;
    const uint64_t A0 = (uint64_t)(uintptr_t)o0;
    const uint64_t A1 = A0 + n;
    const uint64_t al = (A0 + 15) & ~15ull;
    const uint32_t head = (uint32_t)((al < A1 ? al : A1) - A0);  // bytes before 16-byte alignment
    if ((uint32_t)l < head) o0[l] = sb[16 + l];
    if (A1 > al) {
      const uint32_t body = (uint32_t)((A1 & ~15ull) - A0);  // end of the aligned stores
      const uint32_t nblk = (body - head) >> 4;
      const uint32_t so0 = 16u + head;
      const uint32_t rr = so0 & 3u;
      u32x4* const ob = (u32x4*)(o0 + head);
      for (uint32_t i = l; i < nblk; i += 64) {
        const uint32_t d = (so0 >> 2) + 4 * i;
        const uint32_t v0 = stg[d], v1 = stg[d + 1], v2 = stg[d + 2], v3 = stg[d + 3],
                       v4 = stg[d + 4];
        u32x4 v;
        v.x = __builtin_amdgcn_alignbyte(v1, v0, rr);
        v.y = __builtin_amdgcn_alignbyte(v2, v1, rr);
        v.z = __builtin_amdgcn_alignbyte(v3, v2, rr);
        v.w = __builtin_amdgcn_alignbyte(v4, v3, rr);
        ob[i] = v;
      }
      if (body + (uint32_t)l < n) o0[body + l] = sb[16 + body + l];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const uint32_t nz16 = (16u + n + 4u + 15u) >> 4;
  for (uint32_t i = l; i < nz16; i += 64) ((u32x4*)stg)[i] = (u32x4){0, 0, 0, 0};
}

// A tile once counted and staged: what its look-back, stores and requested positions need.
struct Staged3 {
  uint64_t t, agg, tend, pidx, p0;  // p0: lane l's entry of pos[pidx ..] (loaded early)
  uint32_t loff, heads, rh, crf, nzA, nzB;
  uint32_t patch;  // 0, or 0x80000000 | (word of the open run's head << 16) | its count byte
};

// Requested positions (message starts) inside the tile: excl + lane offset + the lane's bytes
// before the word; the entries at the batch end take the total.
__device__ __forceinline__ void positions3(const PackTileArgs& a, const Staged3& s, uint64_t excl) {
  const int l = lane_id();
  const uint64_t N = a.nwords;
  if (a.pos) {
    const uint64_t tbase = s.t * kT;
    uint64_t idx = s.pidx;
    for (bool first = true;; first = false) {
      const uint64_t i = idx + l;
      const uint64_t p = first ? s.p0 : (i <= a.npos ? a.pos[i] : ~0ull);
      const bool in = p >= tbase && p < s.tend;
      const uint32_t rel = in ? (uint32_t)(p - tbase) : 0u;
      const int L = (int)(rel >> 4);
      const uint32_t k = rel & 15u;
      const uint32_t oL = shfl32(s.loff, L), hL = shfl32(s.heads, L), rL = shfl32(s.rh, L);
      const uint32_t cL = shfl32(s.crf, L);
      const uint32_t aL = shfl32(s.nzA, L), bL = shfl32(s.nzB, L);
      const uint32_t mk = (1u << k) - 1u;
      // nibble sums of nz below word k
      const uint32_t mA = k >= 8 ? 0xffffffffu : ((1u << (4 * k)) - 1u);
      const uint32_t mB = k <= 8 ? 0u : ((1u << (4 * (k - 8))) - 1u);
      auto nib = [](uint32_t x) {
        const uint32_t y = (x & 0x0f0f0f0fu) + ((x >> 4) & 0x0f0f0f0fu);
        return (y * 0x01010101u) >> 24;
      };
      const uint32_t before = nib(aL & mA) + nib(bL & mB) + __popc(hL & mk) + __popc(rL & mk) +
                              __popc(cL & mk);
      if (in) a.pos_out[i] = excl + oL + before;
      const uint64_t inm = ballot(in);
      idx += __popcll(inm);
      if (inm != ~0ull) break;
    }
    if (s.tend == N)
      for (uint64_t i = idx + l; i <= a.npos; i += 64) a.pos_out[i] = excl + s.agg;
  }
  if (s.tend == N && l == 0 && a.total_out) *a.total_out = excl + s.agg;
}

// Look-back, stores and positions of a staged tile.
template <bool STAMPS>
__device__ __forceinline__ void finish3(const PackTileArgs& a, uint32_t* wst, const Staged3& s,
                                        Stamps<STAMPS>& stm) {
#if CPK_P3_NOLB
  const uint64_t excl = 0;  // diagnostic only (output wrong): the look-back's share of the time
#else
  const uint64_t excl = lookback2(a.desc, a.gdesc, s.t, 0, a.err, STAMPS ? stm.acc + 10 : nullptr);
#endif
  stm.mark(9);
  publish_incl(a.desc, a.gdesc, s.t, a.ntiles, excl + s.agg);
  if (s.patch && s.tend < a.nwords) {
    // the run open at the tile end: count = words to the first sync (<= 256 past the tile end)
    const uint32_t lead = wait_nonzero32(a.lead + s.t + 1, a.err) & 0x7fffffffu;
    const uint32_t h = (s.patch >> 16) & 0x7fffu;
    const uint32_t cnt = min((uint32_t)kT + min(lead, 256u) - h - 1u, 255u);
    if (lane_id() == 0) ((uint8_t*)wst)[s.patch & 0xffffu] = (uint8_t)cnt;
    lane_handoff();
  }
  const bool over = excl + s.agg > a.out_capacity;
  if (over && lane_id() == 0) raise_error(a.err, kErrCapacity);
  if (!over) flush_slot(a, wst, excl, (uint32_t)s.agg);
  positions3(a, s, excl);
}

template <bool STAMPS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void pack3_kernel(
    PackTileArgs a) {
  // per wave: the staging slot, then the trash windows (lane l: dwords l .. l + 3)
  __shared__ __attribute__((aligned(16))) uint32_t stg_all[4][kSlotDw + kTrashDw];
  __shared__ uint64_t sel_tab[256];
  const int l = lane_id();
  const int wv = (int)uniform32(threadIdx.x >> 6);
  uint32_t* const wst = stg_all[wv];
  sel_tab[threadIdx.x] = make_sel(threadIdx.x);
  for (int i = l; i < (kSlotDw + kTrashDw) / 4; i += 64) ((u32x4*)wst)[i] = (u32x4){0, 0, 0, 0};
  __syncthreads();
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  const uint64_t N = a.nwords;
  const uint64_t nbitw = (N + 63) >> 6;
  Stamps<STAMPS> stm;
  stm.start(a.stamps);
  uint64_t rt0 = 0;
  if constexpr (STAMPS) rt0 = __builtin_amdgcn_s_memrealtime();
  Staged3 pend;
  bool p_on = false;

  // Tile t is counted first; then the previous tile's look-back (its predecessors have had this
  // wave's loads and counting to publish), stores and positions free the slot, and tile t is
  // staged in it.  One extra turn finishes the last tile.
  for (uint64_t t = (uint64_t)blockIdx.x * 4 + wv;; t += nwaves) {
    if (t >= a.ntiles) {
      if (p_on) finish3(a, wst, pend, stm);
      break;
    }
    stm.restart();
    const uint64_t tbase = t * kT;
    const uint64_t tend = tbase + kT < N ? tbase + kT : N;
    const int nvalid = (int)(tend - tbase);
    const uint64_t w0 = tbase + (uint64_t)kK * l;  // the lane's first word

    // ---- words: lane l takes words 16l .. 16l+15 of the tile (16-byte loads) ----------------
    // Every load of a full tile is unconditional and none is waited for here: vector loads
    // retire in order, and the compiler waits for all of them right behind a load whose value
    // it moves to an SGPR, or at the join behind a load under a branch.  So uniform values come
    // through scalar loads (their own counter) and lane-varying guards become clamped addresses
    // with the value selected afterwards; the partial last tile's loads are waited for inside
    // its own branch.
    uint32_t xlo[kK], xhi[kK];
    if (nvalid == kT) {
      const u32x4* src = (const u32x4*)(a.words + w0);
#pragma unroll
      for (int i = 0; i < kK / 2; i++) {
        const u32x4 v = src[i];
        xlo[2 * i] = v.x;
        xhi[2 * i] = v.y;
        xlo[2 * i + 1] = v.z;
        xhi[2 * i + 1] = v.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kK; k++) {
        const uint64_t x = w0 + k < N ? a.words[w0 + k] : 0;
        xlo[k] = (uint32_t)x;
        xhi[k] = (uint32_t)(x >> 32);
      }
    }
    const uint64_t cbi = (tbase >> 6) + (uint64_t)(l >> 2);
    const uint64_t cb0 = a.chunk_bits[cbi < nbitw ? cbi : nbitw - 1];
    // the word before the tile (lane 0 only; a lane-varying address keeps it in a VGPR)
    const uint64_t pw0 = a.words[l == 0 && tbase > 0 ? tbase - 1 : w0 < N ? w0 : N - 1];
    // requested positions of the tile (message starts): the first 64, needed at the end
    typedef const __attribute__((address_space(4))) uint64_t cu64;
    const uint64_t pidx = a.pos ? *((cu64*)a.tile_first + t) : 0;  // scalar load
    const uint64_t pi = pidx + l;
    const bool pv = a.pos && pi <= a.npos;
    const uint64_t p00 = (a.pos ? a.pos : a.words)[pv ? pi : 0];
    const uint64_t cbw = cbi < nbitw ? cb0 : 0;
    const uint64_t pw = tbase > 0 ? pw0 : 0;
    const uint64_t p0 = pv ? p00 : ~0ull;
    stm.mark(0);
#if CPK_P3_LOADONLY
    {  // diagnostic only (no output): the kernel's loads alone
      uint32_t x = 0;
      for (int k = 0; k < kK; k++) x ^= xlo[k] ^ xhi[k];
      x ^= (uint32_t)cbw ^ (uint32_t)pw ^ (uint32_t)p0;
      if (x == 0x9e3779b9u) a.err[0] = x;
      continue;
    }
#endif

    // ---- classes ----------------------------------------------------------------------------
    uint32_t Zm = 0, Rm = 0, Fm = 0, nzsum = 0, nzA = 0, nzB = 0;
    uint32_t tags[kK / 4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < kK; k++) {
      const uint32_t tg = tag_of(xlo[k], xhi[k]);
      const uint32_t nz = __popc(tg);
      tags[k >> 2] |= tg << (8 * (k & 3));
      Zm |= (tg == 0 ? 1u : 0u) << k;
      Rm |= (nz >= 7 ? 1u : 0u) << k;
      Fm |= (tg == 0xffu ? 1u : 0u) << k;
      nzsum += nz;
      if (k < 8) nzA |= nz << (4 * k);
      else nzB |= nz << (4 * (k - 8));
    }
    const int kv = nvalid - kK * l;
    const uint32_t V = kv >= kK ? 0xffffu : (kv <= 0 ? 0u : ((1u << kv) - 1u));
    Zm &= V;
    Rm &= V;
    Fm &= V;
    // class of the word before the lane: the previous lane's last word (tile: word tbase - 1)
    uint32_t zc = shfl32(Zm >> 15, l > 0 ? l - 1 : 0) & 1u;
    uint32_t rc = shfl32(Rm >> 15, l > 0 ? l - 1 : 0) & 1u;
    if (l == 0) {
      zc = (tbase > 0 && pw == 0) ? 1u : 0u;
      rc = (tbase > 0 && __popc(tag_of((uint32_t)pw, (uint32_t)(pw >> 32))) >= 7) ? 1u : 0u;
    }
    const uint32_t C = (uint32_t)(cbw >> (16 * (l & 3))) & 0xffffu;
    const uint32_t O = V & ~Zm & ~Rm;
    const uint32_t SY =
        (C | O | (Zm & ~((Zm << 1) | zc)) | (Rm & ~((Rm << 1) | rc)) | ~V) & 0xffffu;
    const bool lv = kv >= kK;  // the lane's last word is valid
    stm.mark(1);

    // first sync at / after the next lane's first word (tile-relative)
    const uint64_t hs = ballot(SY != 0);
    const uint32_t fs = SY ? (uint32_t)__builtin_ctz(SY) : 16u;
    const uint64_t above = hs & ~mask_le(l);
    const int ja = above ? lowest_bit(above) : 0;
    const uint32_t fsa = shfl32(fs, ja);
    // a run still open at the tile end: its count byte is written as if the batch ended here and
    // patched at the tile's finish from the next tile's first sync (lead[], published below)
    const uint32_t nsl = above ? (uint32_t)(kK * ja) + fsa : (uint32_t)kT;
    {
      const int L0 = hs ? lowest_bit(hs) : 0;
      const uint32_t lead = hs ? (uint32_t)(kK * L0) + shfl32(fs, L0) : (uint32_t)kT;
      if (l == 0) store_agent32(a.lead + t, 0x80000000u | lead);
    }
    stm.mark(2);

    // ---- entry budgets and coverage ----------------------------------------------------------
    const bool simple = SY != 0 || Zm == 0xffffu || Fm == 0xffffu;
    const uint64_t nonsimple = ballot(!simple && kv > 0);
    const Cov c0 = cover16(Zm, Fm, Rm, SY, 0u, lv);  // exits of lanes with a sync point
    uint32_t bt = 0;
    if (hs != 0) {
      // the tile's exit does not depend on its entry: publish it before waiting for the entry
      const uint32_t e0 = lane_entries(0u, hs, nonsimple, c0.b_out, Zm, Fm);
      const Cov ce = cover16(Zm, Fm, Rm, SY, e0, lv);
      const uint32_t eb = readlane32(ce.b_out, 63);
      if (l == 0) store_agent32(a.state + t, 0x80000000u | eb);
    }
    stm.mark(3);
    if (t > 0 && !(readlane32(SY, 0) & 1u)) bt = wait_nonzero32(a.state + t - 1, a.err) & 0xffu;
    stm.mark(4);
    const uint32_t ent = lane_entries(bt, hs, nonsimple, c0.b_out, Zm, Fm);
    const Cov cv = cover16(Zm, Fm, Rm, SY, ent, lv);
    const uint32_t eb2 = readlane32(cv.b_out, 63);
    if (hs == 0 && l == 0) store_agent32(a.state + t, 0x80000000u | eb2);

    // ---- bytes and offsets -------------------------------------------------------------------
    const uint32_t heads = V & ~cv.cov;
    const uint32_t rh = cv.zh | cv.fh;
    const uint32_t crf = cv.cov & Rm & ~Fm;
    const uint32_t bytes = nzsum + __popc(heads) + __popc(rh) + __popc(crf);
    const uint32_t incl = wave_incl_sum32(bytes);
    const uint32_t loff = incl - bytes;
    const uint64_t agg = readlane32(incl, 63);
    publish_agg(a.desc, a.gdesc, a.gcnt, t, a.ntiles, agg, 0, a.err);
    stm.mark(5);

    // ---- emission: the lane's records as a byte stream at slot byte 16 + (loff - base) -------
    // Offset-indexed emission: every record is OR-ed into the slot at its own byte
    // offset, up to 4 dwords (bytes past a record are zero, so OR-ing a whole window never
    // disturbs a neighbour's bytes, and the slot is zero before a tile is staged) -- no byte carry
    // runs from one record to the next, and the windows' dwords are immediate offsets from one
    // address.  Words past the batch end are zero, not covered and not heads: they OR zeros.
    auto emit2 = [&](uint32_t* stg) {
      uint32_t o = 16u + loff;  // slot byte of the lane's next record
      const uint32_t lbase = (uint32_t)(kK * l);
      uint64_t sel_next = sel_tab[tags[0] & 0xffu];
#pragma unroll
      for (int k = 0; k < kK; k++) {
        const uint32_t lo = xlo[k], hi = xhi[k];
        const uint32_t tg = (tags[k >> 2] >> (8 * (k & 3))) & 0xffu;
        const uint64_t sel = sel_next;
        if (k + 1 < kK) sel_next = sel_tab[(tags[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xffu];
        const uint32_t nz = ((k < 8 ? nzA >> (4 * k) : nzB >> (4 * (k - 8)))) & 15u;
        const bool cvk = (cv.cov >> k) & 1, zhk = (cv.zh >> k) & 1, fhk = (cv.fh >> k) & 1;
        const uint32_t after = SY & (0xfffeu << k);
        const uint32_t ns = after ? lbase + (uint32_t)__builtin_ctz(after) : nsl;
        const uint32_t c8 = min(ns - (lbase + (uint32_t)k) - 1u, 255u) << 8;
        uint32_t r0 = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel) | tg | (zhk ? c8 : 0u);
        uint32_t r1 = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
        uint32_t r2 = fhk ? ((hi >> 24) | c8) : 0u;
        uint32_t L = 1u + nz + ((zhk || fhk) ? 1u : 0u);
        if (cvk) {
          r0 = lo;
          r1 = hi;
          r2 = 0;
          L = ((Rm >> k) & 1) ? 8u : 0u;
        }
        const uint32_t sh = 8u * (o & 3u);
        // an empty record (covered zero word) ORs into the lane's trash window: a zero stretch
        // would otherwise put every lane's atomics on the same slot dwords.  The windows overlap
        // (lane l: dwords l .. l + 3, contents never read), so the 32 lanes of a bank group hit
        // 32 banks; disjoint windows 4 dwords apart made every such OR a 4-way bank conflict.
        uint32_t* const w = L ? stg + (o >> 2) : wst + kSlotDw + l;
        const uint64_t q01 = (((uint64_t)r1 << 32) | r0) << sh;
        const uint64_t q12 = (((uint64_t)r2 << 32) | r1) << sh;
        const uint32_t w3 = (uint32_t)(((uint64_t)r2 << sh) >> 32);
        atomicOr(w, (uint32_t)q01);
        atomicOr(w + 1, (uint32_t)(q01 >> 32));
        atomicOr(w + 2, (uint32_t)(q12 >> 32));
        if (ballot(w3 != 0)) atomicOr(w + 3, w3);
        o += L;
        __builtin_amdgcn_sched_barrier(0);
      }
    };

    // the previous tile: its look-back, stores and positions
    if (p_on) finish3(a, wst, pend, stm);
    stm.mark(6);
    emit2(wst);
    stm.mark(7);
    pend.t = t;
    pend.agg = agg;
    pend.tend = tend;
    pend.pidx = pidx;
    pend.p0 = p0;
    pend.loff = loff;
    pend.heads = heads;
    pend.rh = rh;
    pend.crf = crf;
    pend.nzA = nzA;
    pend.nzB = nzB;
    {
      // The one head whose run may still be open at the tile end (no sync after it in the tile,
      // fewer than 255 words left) got a provisional count (as if the batch ended here): its
      // word and the slot byte of its count go to the finish, which patches the count from the
      // next tile's lead.
      const int hsy = hi_bit16(SY);
      // heads at or after the lane's last sync (a stretch that starts at it has its head there)
      const uint32_t hd = (cv.zh | cv.fh) & (0xffffu << (hsy < 0 ? 0 : hsy)) & 0xffffu;
      const int kk = hi_bit16(hd);
      const uint32_t h = (uint32_t)(kK * l + kk);
      const bool mine = above == 0 && hd != 0 && h + 256u > (uint32_t)kT;
      uint32_t patch = 0;
      if (mine) {
        const uint32_t k = (uint32_t)kk, mk = (1u << k) - 1u;
        const uint32_t mA = k >= 8 ? 0xffffffffu : ((1u << (4 * k)) - 1u);
        const uint32_t mB = k <= 8 ? 0u : ((1u << (4 * (k - 8))) - 1u);
        auto nib = [](uint32_t x) {
          const uint32_t y = (x & 0x0f0f0f0fu) + ((x >> 4) & 0x0f0f0f0fu);
          return (y * 0x01010101u) >> 24;
        };
        const uint32_t before = nib(nzA & mA) + nib(nzB & mB) + __popc(heads & mk) +
                                __popc(rh & mk) + __popc(crf & mk);
        patch = 0x80000000u | (h << 16) | (16u + loff + before + (((cv.zh >> k) & 1) ? 1u : 9u));
      }
      const uint64_t pm = ballot(mine);
      pend.patch = pm ? readlane32(patch, lowest_bit(pm)) : 0u;
    }
    p_on = true;
  }
  stm.mark(8);
  if constexpr (STAMPS) {
    stm.acc[14] = __builtin_amdgcn_s_memrealtime() - rt0;
    stm.acc[15] = 1;
    stm.flush();
  }
}

}  // namespace

bool pack_v3() {
  // the default; A/B knob CPK_PACK3=0 selects the step-major kernels of cpk_pack.hip
  static const bool on = !(getenv("CPK_PACK3") && atoi(getenv("CPK_PACK3")) == 0) &&
                         !(getenv("CPK_PACK_V2") && atoi(getenv("CPK_PACK_V2")) != 0);
  return on;
}

hipError_t launch_pack_tiles3(const PackTileArgs& a, hipStream_t stream) {
  if (a.ntiles == 0) return hipSuccess;
  // persistent: every wave of the grid resident (a tile only waits on lower tiles)
  static const unsigned cap_false = resident_blocks((const void*)pack3_kernel<false>, 256, 0);
  static const unsigned cap_true = resident_blocks((const void*)pack3_kernel<true>, 256, 0);
  const unsigned want = (unsigned)((a.ntiles + 3) / 4);
  // tuning knob: at most CPK_PACK3_BLOCKS workgroups in the grid (fewer waves in flight)
  static const unsigned knob = getenv("CPK_PACK3_BLOCKS") ? (unsigned)atoi(getenv("CPK_PACK3_BLOCKS"))
                                                          : 0u;
  unsigned ct = cap_true, cf = cap_false;
  if (knob) {
    ct = knob < ct ? knob : ct;
    cf = knob < cf ? knob : cf;
  }
  if (a.stamps)
    pack3_kernel<true><<<want < ct ? want : ct, 256, 0, stream>>>(a);
  else
    pack3_kernel<false><<<want < cf ? want : cf, 256, 0, stream>>>(a);
  return hipGetLastError();
}

}  // namespace cpk
