// cpk_pack.hip -- MI355X (gfx950) kernels for Cap'n Proto's packed encoding.
//
// Functional spec: PackedOutputStream::write (capnproto c++/src/capnp/serialize-packed.c++:
// 307-431), applied once per OutputStream::write() piece -- the segment table, then each segment
// (writeMessage serialize.c++:332-357 -> OutputStream::write(pieces) kj/io.c++:109-113).
//
// Data-parallel restatement of the greedy scalar loop.  Every word of a chunk is one of
//   Z  all-zero            F  no zero byte (tag 0xff)
//   R  at most one zero byte (includes F)   O  anything else (>= 2 zero bytes, non-zero)
// A maximal run of same-family words (Z, or R) inside a chunk is a "stretch"; chunk starts,
// O words and family changes are sync points where the scalar loop's state is reset.
//   * In a Z stretch the heads sit at 0, 256, 512, ... from the stretch start; a head emits
//     `00 n` with n = min(255, zeros left in the stretch) (:352-374).
//   * In an R stretch an F word that is a head opens a raw run covering the next <= 255 words of
//     the stretch (:376-426); R words that are not covered are ordinary heads.
//   * Output bytes per word: Z head 2, Z covered 0, F head 10, covered R 8, other heads 1 + nz.
// Inside one 64-word step a run, once opened, never closes (255 > 63), so a step is resolved by
// a handful of 64-bit mask operations on the wave's ballots (scalar unit): raw-run coverage of
// every segment is one carry-propagating add, `((U + G) ^ U) & U` with U = ~sync and G the F
// words shifted by one.  The only state crossing steps is one byte: the budget of the run that
// is open at the step's last word.
//
// Work decomposition: the batch of words is cut into tiles of 64*S words, one wave per tile,
// persistent waves over a static strided tile order (pack_tiles_kernel below).
#include <stdlib.h>

#include <type_traits>

#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// v_writelane: lane `s` (compile-time) of `dst` takes the wave-uniform value `v`.  Inline asm
// (this compiler has no writelane builtin) hides the SGPR read from the hazard recognizer, so
// the value goes through an SALU move first: a writelane reading an SGPR that a VALU (ballot)
// has just written returned stale data.
template <int L>
__device__ __forceinline__ uint32_t setlane(uint32_t dst, uint32_t v) {
  uint32_t tmp;
  asm volatile("s_mov_b32 %1, %2\n\ts_nop 0\n\tv_writelane_b32 %0, %1, %3"
               : "+v"(dst), "=&s"(tmp)
               : "s"((uint32_t)__builtin_amdgcn_readfirstlane((int)v)), "i"(L));
  return dst;
}

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Tag byte of a word (bit i <=> byte i non-zero), SWAR on the two dwords.
__device__ __forceinline__ uint32_t tag_of(uint32_t lo, uint32_t hi) {
  const uint32_t m7 = 0x7f7f7f7fu;
  const uint32_t a = ((lo & m7) + m7) | lo;  // bit 7 of a byte <=> byte non-zero
  const uint32_t b = ((hi & m7) + m7) | hi;
  const uint32_t c = ((a >> 7) & 0x01010101u) | ((b >> 3) & 0x10101010u);  // bits 8k, 8k+4
  const uint32_t d = c | (c >> 14);
  return (d | (d >> 7)) & 0xffu;
}

// Per-lane select by a wave-uniform 64-bit mask held in SGPRs: one v_cndmask.
__device__ __forceinline__ uint32_t msel(uint64_t mask, uint32_t if_set, uint32_t if_clear) {
  uint32_t r;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(mask));
  return r;
}

// Index of the lowest set bit, ~0u for 0 (v_ffbl_b32).
__device__ __forceinline__ uint32_t ffbl32(uint32_t v) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// v_perm selectors placing the non-zero bytes of a word with tag `tag` after a zero byte 0:
// dword 0 = [0, c0, c1, c2], dword 1 = [c3 .. c6] (c7 only exists for tag 0xff).
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

// Head / coverage resolution of one step, entry budget b (words the run open before the step
// may still cover).  All wave-uniform mask arithmetic.
struct StepRes {
  uint64_t covered, runheads;  // covered words; Z heads | F heads
  uint64_t Zheads, Fheads;
  int b_out;                   // budget leaving the step
};

__device__ __forceinline__ StepRes resolve_step(uint64_t Z, uint64_t F, uint64_t R, uint64_t SY,
                                                int b, bool last_valid) {
  const uint64_t LM = ~SY & (SY - 1);                     // lead: words before the first sync
  const uint64_t BM = b >= 64 ? ~0ull : mask_lt(b);       // words the entering run covers
  const uint64_t lead_cov = BM & LM;
  const uint64_t zlead = (BM + 1) & LM & Z;               // Z lead: next head at word b
  const uint64_t Feff = F & ~lead_cov;
  const uint64_t G = (Feff << 1) & ~SY;
  const uint64_t fill = (((~SY + G) ^ ~SY) & ~SY) | G;    // words after an F head, same segment
  const uint64_t Fheads = Feff & ~fill;
  const uint64_t Zheads = (Z & SY) | zlead;
  StepRes r;
  r.covered = (R & (fill | lead_cov)) | (Z & ~Zheads);
  r.runheads = Zheads | Fheads;
  r.Zheads = Zheads;
  r.Fheads = Fheads;
  // budget for the next step: the last run head of the last segment, or the entering run when
  // the whole step is its lead; a last word of class O ends with a sync and a zero budget
  r.b_out = 0;
  if (last_valid) {
    const int st = highest_bit(SY);         // -1: no sync
    const int h = highest_bit(r.runheads);  // -1: no head
    if (h >= 0 && h >= st) r.b_out = 192 + h;
    else if (SY == 0 && b > 63) r.b_out = b - 64;
  }
  return r;
}

// Valid-lane mask of step s of a tile with n valid words.
__device__ __forceinline__ uint64_t valid_mask(int n, int s) {
  const int k = n - 64 * s;
  return k >= 64 ? ~0ull : (k <= 0 ? 0ull : mask_lt(k));
}

template <int S>
struct TileLoad {
  uint64_t x[S];  // word 64*s + lane
  uint64_t nx;    // word tend + lane (look-ahead)
  uint64_t cb;    // lanes < S: chunk-start bits of step `lane`; lane S: those of the next step
  uint64_t pw;    // word before the tile (0 for tile 0)
};

template <int S>
__device__ __forceinline__ void load_tile(const PackTileArgs& a, uint64_t t, TileLoad<S>& L) {
  constexpr int T = 64 * S;
  const int l = lane_id();
  const uint64_t N = a.nwords;
  const uint64_t tbase = t * T;
  const uint64_t tend = tbase + T < N ? tbase + T : N;
#pragma unroll
  for (int s = 0; s < S; s++) {
    const uint64_t g = tbase + 64 * s + l;
    L.x[s] = g < N ? a.words[g] : 0;
  }
  L.nx = tend + l < N ? a.words[tend + l] : 0;
  const uint64_t nbitw = (N + 63) >> 6;
  L.cb = (l <= S && (tbase >> 6) + l < nbitw) ? a.chunk_bits[(tbase >> 6) + l] : 0;
  L.pw = tbase > 0 ? a.words[tbase - 1] : 0;
}

// One wave per tile of 64*S words, persistent waves over a static strided tile order.
//   pass A   classes + sync masks of every step (wave-uniform SGPR masks), packed tags;
//            the tile's exit budget is published at once when it does not depend on the entry
//   entry    the predecessor's exit budget, only when word 0 continues a stretch
//   pass B   per step: resolve heads / coverage (scalar), record lengths, DPP prefix sum,
//            v_perm compaction through a 256-entry selector table, records OR-ed into the
//            wave's LDS staging area at tile-relative byte offsets
//   look-back  two-level decoupled look-back on the tile's byte count
//   flush    staged bytes -> global: 16-byte aligned stores (realigned by v_alignbyte), byte
//            stores for the partial blocks at both ends; the staging area is re-zeroed.
//
// MODE kFused: the single-pass kernel above.  The two-pass form splits it at the look-back:
// MODE kCount (persistent) does pass A and the count pass -- entry budgets still hand over
// between waves, a one-hop wait only where a tile's first word continues a stretch -- and writes
// each tile's entry budget and byte count; a scan turns the counts into output offsets; MODE kEmit
// (one wave per tile, no waits) redoes pass A with the known entry budget, then pass B and the
// flush at the known offset.
constexpr int kFused = 0, kCount = 1, kEmit = 2;

template <int S, bool PF, bool STAMPS, int MODE = kFused>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(S <= 8 ? 6 : 3, 8))) void pack_tiles_kernel(
    PackTileArgs a) {
  static_assert(S >= 2 && S <= 16 && (S % 2) == 0, "S steps per tile");
  constexpr int T = 64 * S;
  // Per-wave staging ring: a tile's records occupy [base, base + 32 + bytes) (16 B pads at both
  // ends), at most 32 + 640 * S bytes; the ring holds the tile being encoded and the previous
  // one, whose look-back and flush are deferred until after this tile's emission pass.  The emit
  // pass flushes each tile at once (one region); the count pass stages nothing.
  constexpr int kMaxRegion = 32 + 640 * S;
  constexpr int kStg = MODE == kCount ? 16
                       : (MODE == kEmit ? ((kMaxRegion + 15) & ~15)
                                        : (((kMaxRegion * 6 / 5) + 15) & ~15));
  __shared__ __attribute__((aligned(16))) uint8_t stg_all[4][kStg];
  __shared__ uint64_t sel_tab[256];

  const int l = lane_id();
  const int wv = (int)uniform32(threadIdx.x >> 6);
  uint8_t* const stg = stg_all[wv];
  sel_tab[threadIdx.x] = make_sel(threadIdx.x);
  for (int i = l; i < kStg / 16; i += 64) ((u32x4*)stg)[i] = (u32x4){0, 0, 0, 0};
  __syncthreads();

  const uint64_t gt_mask = ~mask_le(l);  // lanes above this one
  const uint32_t gt_lo = (uint32_t)gt_mask, gt_hi = (uint32_t)(gt_mask >> 32);
  const uint32_t lp1 = (uint32_t)l + 1u;
  const uint64_t N = a.nwords;
  const uint64_t nbitw = (N + 63) >> 6;
  uint32_t* const state = a.state;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  Stamps<STAMPS> stm;
  stm.start(a.stamps);
  uint64_t t = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  TileLoad<S> cur;
  if (t < a.ntiles) load_tile<S>(a, t, cur);

  // A tile whose look-back and flush are still to be done.
  struct Pending {
    uint64_t t, agg, tend, pidx0, pidx;
    uint32_t base;
    bool on;
  };
  Pending pend;
  pend.on = false;
  auto region = [](uint64_t agg) -> uint32_t { return ((uint32_t)agg + 32u + 15u) & ~15u; };
  // look-back, inclusive publish, flush of the staged bytes, positions
  auto finish = [&](const Pending& p) {
    uint64_t excl = 0;
    if constexpr (MODE == kEmit) {
      excl = uniform64(a.tile_off[p.t]);
    } else if (a.debug_skip & 1) {
      excl = p.t * 4096;  // timing ablation: no look-back (output meaningless)
    } else {
      excl = lookback2(a.desc, a.gdesc, p.t, 0, a.err);
      publish_incl(a.desc, a.gdesc, p.t, a.ntiles, excl + p.agg);
    }
    const uint64_t agg = p.agg;
    uint8_t* const sb = stg + p.base;
    const uint32_t* const sb32 = (const uint32_t*)sb;
    const bool over = excl + agg > a.out_capacity;
    if (over && l == 0) raise_error(a.err, kErrCapacity);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!over && agg) {
      uint8_t* const out = a.out;
      const uint64_t A0 = (uint64_t)(uintptr_t)out + excl;
      const uint64_t A1 = A0 + agg;
      const uint64_t al = (A0 + 15) & ~15ull;
      const uint64_t hl = al < A1 ? al : A1;
      if (A0 + l < hl) *(uint8_t*)(uintptr_t)(A0 + l) = sb[16 + l];
      if (A1 > al) {
        const uint64_t top = A1 & ~15ull;
        const uint32_t nb = (uint32_t)((top - al) >> 4);
        const uint32_t so0 = 16u + (uint32_t)(al - A0);
        const uint32_t rr = so0 & 3u;
        for (uint32_t i = l; i < nb; i += 64) {
          const uint32_t d = (so0 >> 2) + 4 * i;
          const uint32_t v0 = sb32[d], v1 = sb32[d + 1], v2 = sb32[d + 2], v3 = sb32[d + 3],
                         v4 = sb32[d + 4];
          u32x4 v;
          v.x = __builtin_amdgcn_alignbyte(v1, v0, rr);
          v.y = __builtin_amdgcn_alignbyte(v2, v1, rr);
          v.z = __builtin_amdgcn_alignbyte(v3, v2, rr);
          v.w = __builtin_amdgcn_alignbyte(v4, v3, rr);
          *(u32x4*)(uintptr_t)(al + 16ull * i) = v;
        }
        if (top + l < A1) *(uint8_t*)(uintptr_t)(top + l) = sb[16 + (uint32_t)(top - A0) + l];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint32_t nz16 = (uint32_t)((agg + 15) >> 4) + 1;
    for (uint32_t i = l; i < nz16; i += 64) ((u32x4*)(sb + 16))[i] = (u32x4){0, 0, 0, 0};
    // positions: add the tile's global offset (own stores, read back past L1)
    if (a.pos) {
      if constexpr (MODE != kEmit) {  // emit mode wrote absolute positions in pass B
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (uint64_t i = p.pidx0 + l; i < p.pidx; i += 64)
          a.pos_out[i] = load_agent(a.pos_out + i) + excl;
      }
      if (p.tend == N) {
        const uint64_t tot = excl + agg;
        for (uint64_t i = p.pidx + l; i <= a.npos; i += 64) a.pos_out[i] = tot;
      }
    }
    if (p.tend == N && l == 0 && a.total_out) *a.total_out = excl + agg;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  for (; t < a.ntiles; t += nwaves) {
    TileLoad<S> nxt;
    auto tile = [&](auto full_c) {
    constexpr bool FULL = decltype(full_c)::value;
    stm.restart();
    const uint64_t tbase = t * T;
    const uint64_t tend = tbase + T < N ? tbase + T : N;
    const int nvalid = FULL ? T : (int)(tend - tbase);
    const int last = nvalid - 1;
    uint64_t zc0 = 0, rc0 = 0;  // class of the word before the tile
    if (tbase > 0) {
      const uint64_t pw = uniform64(cur.pw);
      zc0 = pw == 0;
      rc0 = __popc(tag_of((uint32_t)pw, (uint32_t)(pw >> 32))) >= 7;
    }

    // ---- pass A --------------------------------------------------------------------------
    // per step: tags and the Z / R / F ballots, parked in VGPR lanes (lane s = step s); the sync
    // masks and state-independent byte counts of all steps are then formed at once in lanes
    uint32_t vSYlo = 0, vSYhi = 0, vFlo = 0, vFhi = 0, vZlo = 0, vZhi = 0, vRlo = 0, vRhi = 0;
    uint32_t vNsa = 0, vBase = 0, vOb = 0;
    uint32_t tagpk[S / 2];
    static_for<0, S>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      const uint64_t x = cur.x[s];
      if (s % 2 == 0) tagpk[s >> 1] = 0;
      const uint64_t Z = ballot(x == 0);  // words past the batch end load as 0: masked below
      vZlo = setlane<s>(vZlo, (uint32_t)Z);
      vZhi = setlane<s>(vZhi, (uint32_t)(Z >> 32));
      if (Z != ~0ull) {  // an all-zero step has tag 0, no R / F word and no O bytes
        const uint32_t tag = tag_of((uint32_t)x, (uint32_t)(x >> 32));
        tagpk[s >> 1] |= tag << (16 * (s & 1));
        asm volatile("" : "+v"(tagpk[s >> 1]));  // keep the packed form (VGPR pressure)
        const uint64_t R = ballot(__popc(tag) >= 7);
        const uint64_t Fs = ballot(tag == 0xff);
        vFlo = setlane<s>(vFlo, (uint32_t)Fs);
        vFhi = setlane<s>(vFhi, (uint32_t)(Fs >> 32));
        vRlo = setlane<s>(vRlo, (uint32_t)R);
        vRhi = setlane<s>(vRhi, (uint32_t)(R >> 32));
        // sum of nz over the O words of the step (their bytes are 1 + nz)
        const uint32_t nz = __popc(tag);
        const uint32_t ob = (x != 0 && nz < 7) ? nz : 0;
        vOb = setlane<s>(vOb, (uint32_t)(__popcll(ballot(ob & 1)) +
                                         2 * __popcll(ballot(ob & 2)) +
                                         4 * __popcll(ballot(ob & 4))));
      }
    });
    bool lastZ, lastR;
    int first_sync = T, sg = -1;
    {
      const int kv = nvalid - 64 * l;
      const uint64_t V = FULL ? ~0ull : (kv >= 64 ? ~0ull : (kv <= 0 ? 0ull : mask_lt(kv)));
      const uint64_t Z = (((uint64_t)vZhi << 32) | vZlo) & V;
      const uint64_t R = (((uint64_t)vRhi << 32) | vRlo) & V;
      const uint64_t F = (((uint64_t)vFhi << 32) | vFlo) & V;
      // class of the word before the step: the previous lane's last word (tile: word tbase-1)
      uint32_t zc = dpp_src<0x111, 0xf>((uint32_t)(Z >> 32)) >> 31;
      uint32_t rc = dpp_src<0x111, 0xf>((uint32_t)(R >> 32)) >> 31;
      if (l == 0) {
        zc = (uint32_t)zc0;
        rc = (uint32_t)rc0;
      }
      const uint64_t C = cur.cb;  // lane s: chunk-start bits of step s
      const uint64_t O = V & ~Z & ~R;
      const uint64_t SY =
          C | O | (Z & ~((Z << 1) | zc)) | (R & ~((R << 1) | rc)) | ~V;
      vSYlo = (uint32_t)SY;
      vSYhi = (uint32_t)(SY >> 32);
      vZlo = (uint32_t)Z;
      vZhi = (uint32_t)(Z >> 32);
      vRlo = (uint32_t)R;
      vRhi = (uint32_t)(R >> 32);
      vFlo = (uint32_t)F;
      vFhi = (uint32_t)(F >> 32);
      // state-independent bytes of the step: 1 + nz per O word, 8 per R word
      vBase = (uint32_t)(__popcll(O) + 8 * __popcll(R)) + vOb;
      const uint64_t m = l < S ? (SY & V) : 0ull;
      const uint64_t bm = ballot(m != 0);
      if (bm) {
        const int fl = lowest_bit(bm), hl = highest_bit(bm);
        first_sync = 64 * fl + lowest_bit(readlane64(m, fl));
        sg = 64 * hl + highest_bit(readlane64(m, hl));
      }
      const int ls = last >> 6;
      lastZ = (readlane64(Z, ls) >> (last & 63)) & 1;
      lastR = (readlane64(R, ls) >> (last & 63)) & 1;
    }
    stm.mark(0);
    // count pass: pass A was the last use of the words, the next tile's can be on their way
    if constexpr (MODE == kCount) {
      if (t + nwaves < a.ntiles) load_tile<S>(a, t + nwaves, cur);
    }

    // ---- look-ahead: distance from tend to the first sync at / after it (<= 256) ------------
    int la = 0;
    if (MODE != kCount && (lastZ || lastR) && tend < N) {
      uint64_t czc = lastZ, crc = lastR;
      la = 256;
      uint64_t xk[4] = {cur.nx, 0, 0, 0}, ck[4] = {readlane64(cur.cb, S), 0, 0, 0};
      for (int k = 0; k < 4; k++) {
        const uint64_t g = tend + 64 * k + l;
        if (k == 1) {
          // words 64 .. 255 past the tile together: one round trip instead of three
#pragma unroll
          for (int j = 1; j < 4; j++) {
            const uint64_t gj = tend + 64 * j + l;
            xk[j] = gj < N ? a.words[gj] : 0;
            ck[j] = ((tend >> 6) + j < nbitw) ? a.chunk_bits[(tend >> 6) + j] : 0;
          }
        }
        const uint64_t xx = xk[k];
        const uint32_t tg = tag_of((uint32_t)xx, (uint32_t)(xx >> 32));
        const uint64_t V = ballot(g < N);
        const uint64_t C = ck[k];
        const uint64_t Z = ballot(xx == 0) & V;
        const uint64_t R = ballot(__popc(tg) >= 7) & V;
        const uint64_t O = V & ~Z & ~R;
        const uint64_t SY = C | O | (Z & ~((Z << 1) | czc)) | (R & ~((R << 1) | crc)) | ~V;
        if (SY) {
          la = 64 * k + lowest_bit(SY);
          break;
        }
        czc = Z >> 63;
        crc = R >> 63;
      }
    }
    // lane s: distance from step s+1's first word to the first sync at / after it
    {
      int v = la;
      static_for<0, S>([&](auto sc) {
        constexpr int s = S - 1 - decltype(sc)::value;
        vNsa = setlane<s>(vNsa, v);
        const int fs = lowest_bit(readlane64(((uint64_t)vSYhi << 32) | vSYlo, s));
        v = fs < 64 ? fs : (v + 64 < 256 ? v + 64 : 256);
      });
    }

    // ---- exit budget, published early when it does not depend on the entry ----------------
    if (first_sync < T) {
      int eb = 0;
      if (lastZ) {
        eb = 255 - ((last - sg) & 255);
      } else if (lastR) {
        int na = sg, qq = -1;
#pragma unroll
        for (int s = 0; s < S; s++) {
          if (64 * s + 63 >= na && 64 * s <= last) {
            uint64_t m = readlane64(((uint64_t)vFhi << 32) | vFlo, s);
            if (na > 64 * s) m &= ~mask_lt(na - 64 * s);
            if (m) {
              qq = 64 * s + lowest_bit(m);
              na = qq + 256;
            }
          }
        }
        eb = (qq >= 0 && last - qq <= 255) ? 255 - (last - qq) : 0;
      }
      if (MODE != kEmit && l == 0) store_agent32(state + t, 0x80000000u | (uint32_t)eb);
    }

    // prefetch the next tile (lands during pass B and the look-back)
    if (PF && t + nwaves < a.ntiles) load_tile<S>(a, t + nwaves, nxt);
    stm.mark(1);

    int b = 0;
    if constexpr (MODE == kEmit) {
      b = (int)uniform32(a.tile_b[t]);
    } else {
      if (first_sync > 0 && t > 0) b = (int)(wait_nonzero32(state + t - 1, a.err) & 0xffu);
    }
    const int b_entry = b;
    stm.mark(2);

    // ---- count pass: heads / coverage of every step, byte offsets --------------------------
    //   bytes(step) = sum over O words of (1 + nz) + 8 |R| + 2 |Z heads + F heads|
    // Lane s resolves step s from the masks parked in its lanes (vector unit, all steps at once);
    // only the entry budgets run step to step on the scalar unit, and a step's exit budget
    // depends on its entry budget only when the step has no sync at all.
    uint32_t vCOVlo, vCOVhi, vZHlo, vZHhi, vFHlo, vFHhi, vSoff;
    uint32_t agg32;
    {
      const uint64_t vZ = ((uint64_t)vZhi << 32) | vZlo;
      const uint64_t vF = ((uint64_t)vFhi << 32) | vFlo;
      const uint64_t vR = ((uint64_t)vRhi << 32) | vRlo;
      const uint64_t vSY = ((uint64_t)vSYhi << 32) | vSYlo;
      const bool lane_step = l < S && 64 * l < nvalid;
      const bool lv = 64 * l + 63 < nvalid;  // the step's last word is valid
      // exit budget of a step with a sync: the same for every entry budget (entry 0 here)
      const StepRes r0 = resolve_step(vZ, vF, vR, vSY, 0, lv);
      const uint32_t info = (vSY != 0 ? 0x80000000u : 0u) | (vZ != 0 ? 0x40000000u : 0u) |
                            (uint32_t)r0.b_out;
      uint32_t vB = 0;
      static_for<0, S>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if (64 * s < nvalid) {
          vB = setlane<s>(vB, (uint32_t)b);
          const uint32_t inf = readlane32(info, s);
          if (inf & 0x80000000u) {
            b = (int)(inf & 0x3ffu);
          } else if (b > 63) {
            b -= 64;  // the entering run covers the whole step
          } else if (inf & 0x40000000u) {
            b += 192;  // zero stretch: a head at word b
          } else {  // word stretch: the first F word at / after b opens a run
            const uint64_t Fm = readlane64(vF, s) & ~mask_lt(b);
            b = Fm ? 192 + lowest_bit(Fm) : 0;
          }
        }
      });
      const StepRes r = resolve_step(vZ, vF, vR, vSY, (int)vB, lv);
      const int kv = nvalid - 64 * l;
      const uint64_t V = kv >= 64 ? ~0ull : (kv <= 0 ? 0ull : mask_lt(kv));
      const uint64_t COV = r.covered | ~V;
      vCOVlo = (uint32_t)COV;
      vCOVhi = (uint32_t)(COV >> 32);
      vZHlo = (uint32_t)r.Zheads;
      vZHhi = (uint32_t)(r.Zheads >> 32);
      vFHlo = (uint32_t)r.Fheads;
      vFHhi = (uint32_t)(r.Fheads >> 32);
      const uint32_t bytes = lane_step ? vBase + 2u * (uint32_t)__popcll(r.runheads) : 0u;
      const uint32_t incl = wave_incl_sum32(bytes);
      vSoff = incl - bytes;
      agg32 = readlane32(incl, S - 1);
    }
    if (MODE != kEmit && first_sync == T && l == 0) store_agent32(state + t, 0x80000000u | (uint32_t)b);
    const uint64_t agg = agg32;
    if constexpr (MODE == kCount) {
      if (l == 0) {
        a.tile_b[t] = (uint32_t)b_entry;
        a.tile_bytes[t] = agg;
      }
      return;
    }
    if (MODE == kFused && !(a.debug_skip & 1))
      publish_agg(a.desc, a.gdesc, a.gcnt, t, a.ntiles, agg, 0, a.err);
    (void)b_entry;
    stm.mark(3);

    // ---- staging region: after the pending tile's, else at 0 (finishing it first if needed) ---
    const uint32_t need = region(agg);
    uint32_t base = 0;
    if (pend.on) {
      const uint32_t pe = pend.base + region(pend.agg);
      if (pe + need <= (uint32_t)kStg) {
        base = pe;
      } else if (need > pend.base) {
        finish(pend);
        pend.on = false;
      }
    }

    // ---- pass B ----------------------------------------------------------------------------
    const uint64_t pidx0 = a.pos ? uniform64(a.tile_first[t]) : 0;
    // emit mode knows the tile's output offset: positions are written absolute
    const uint64_t pos_base = MODE == kEmit ? uniform64(a.tile_off[t]) : 0;
    uint64_t pidx = pidx0;
    uint32_t prel = ~0u;  // next requested position, tile-relative (~0: none in this tile)
    if (a.pos && pidx <= a.npos) {
      const uint64_t pn = uniform64(a.pos[pidx]);
      if (pn - tbase < (uint64_t)T) prel = (uint32_t)(pn - tbase);
    }
#pragma unroll
    for (int s = 0; s < S; s++) {
      if (64 * s < nvalid) {
        const uint64_t x = cur.x[s];
        const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
        const uint32_t tag = (tagpk[s >> 1] >> (16 * (s & 1))) & 0xffu;
        const uint32_t nz = __popc(tag);
        const uint64_t SY = readlane64(((uint64_t)vSYhi << 32) | vSYlo, s);
        const uint64_t COV = readlane64(((uint64_t)vCOVhi << 32) | vCOVlo, s);
        const uint64_t ZH = readlane64(((uint64_t)vZHhi << 32) | vZHlo, s);
        const uint64_t FH = readlane64(((uint64_t)vFHhi << 32) | vFHlo, s);
        const uint32_t soff = readlane32(vSoff, s);
        const uint64_t Zs = ((uint64_t)readlane32(vZhi, s) << 32) | readlane32(vZlo, s);
        if (Zs == ~0ull && !(prel < 64u * s + 64u)) {
          // all-zero step: the records are its Z heads, two bytes each ([00, count]); the tag
          // byte stays zero in the staging area, only a non-zero count is stored
          uint64_t hm = ZH;
          uint32_t k = 0;
          while (hm) {
            const int h = lowest_bit(hm);
            hm &= hm - 1;
            const uint64_t after = SY & ~mask_le(h);
            const uint32_t ns = after ? (uint32_t)lowest_bit(after) : 64u + readlane32(vNsa, s);
            const uint32_t cnt = min(ns - (uint32_t)h - 1u, 255u);
            if (cnt && l == 0) stg[base + 16u + soff + 2 * k + 1] = (uint8_t)cnt;
            k++;
          }
          continue;
        }
        // record length: head 1 + nz (+1 count byte for run heads), covered R 8, covered Z 0
        const uint32_t n1 = nz + 1;
        const uint32_t len = msel(COV, n1 & 8u, n1 + msel(ZH | FH, 1u, 0u));
        const uint32_t inc = wave_incl_sum32(len);
        const uint32_t o = inc - len;
        // run count: stretch words after this one (<= 255); ffbl of 0 is ~0u
        const uint32_t f_lo = ffbl32((uint32_t)SY & gt_lo);
        const uint32_t f_hi = __builtin_elementwise_add_sat(
            ffbl32((uint32_t)(SY >> 32) & gt_hi), 32u);
        const uint32_t ns = min(min(f_lo, f_hi), 64u + readlane32(vNsa, s));
        const uint32_t cnt = min(ns - lp1, 255u);
        // record bytes: [tag, non-zero bytes..., count] for heads, the raw word when covered
        const uint64_t sel = sel_tab[tag];
        const uint32_t c8 = cnt << 8;
        uint32_t w0 = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel) | tag | msel(ZH, c8, 0u);
        uint32_t w1 = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
        const uint32_t w2 = msel(FH, (hi >> 24) | c8, 0u);
        w0 = msel(COV, lo, w0);
        w1 = msel(COV, hi, w1);
        // OR into the staging area at byte 16 + soff + o: four dwords from (at - 1) & ~3, each
        // only where the record has bytes (a lane of a covered zero word has none; empty lanes
        // would all hit the same dword and serialise on it)
        const uint32_t at = base + 16u + soff + o;
        const uint32_t rr = (0u - at) & 3u;
        const uint32_t kk = 4u - rr;     // record start inside the 16-byte window (1..4)
        const uint32_t ee = kk + len;    // record end inside the window
        uint32_t* dp = (uint32_t*)(stg + ((at - 1u) & ~3u));
        if (kk < 4u && len) atomicOr(dp + 0, __builtin_amdgcn_alignbyte(w0, 0u, rr));
        if (ee > 4u) atomicOr(dp + 1, __builtin_amdgcn_alignbyte(w1, w0, rr));
        if (ee > 8u) atomicOr(dp + 2, __builtin_amdgcn_alignbyte(w2, w1, rr));
        if (ee > 12u) atomicOr(dp + 3, __builtin_amdgcn_alignbyte(0u, w2, rr));
        // requested positions inside this step: tile-relative offsets (excl added later)
        if (prel < 64u * s + 64u) {
          const uint64_t g0 = tbase + 64 * s;
          while (true) {
            const uint64_t i = pidx + l;
            const uint64_t p = i <= a.npos ? a.pos[i] : ~0ull;
            const bool in = p < g0 + 64;
            const uint32_t oo = shfl32(o, in ? (int)(p - g0) : 0);
            if (in) a.pos_out[i] = pos_base + soff + oo;
            const uint64_t inm = ballot(in);
            pidx += __popcll(inm);
            const uint64_t pn = pidx <= a.npos ? uniform64(a.pos[pidx]) : ~0ull;
            prel = pn - tbase < (uint64_t)T ? (uint32_t)(pn - tbase) : ~0u;
            if (inm != ~0ull) break;
          }
        }
      }
    }
    stm.mark(4);

    // ---- the next tile's words into the registers pass B no longer needs: issued before the
    //      previous tile's flush stores, so waiting for them never waits for those stores
    if (!PF && t + nwaves < a.ntiles) load_tile<S>(a, t + nwaves, cur);

    // ---- finish the previous tile (its look-back had this tile's passes to resolve) --------
    if (pend.on) finish(pend);
    if constexpr (MODE == kEmit) {  // no look-back to wait for: flush at once
      Pending now;
      now.t = t;
      now.agg = agg;
      now.tend = tend;
      now.pidx0 = pidx0;
      now.pidx = pidx;
      now.base = base;
      now.on = true;
      finish(now);
      return;
    }
    pend.t = t;
    pend.agg = agg;
    pend.tend = tend;
    pend.pidx0 = pidx0;
    pend.pidx = pidx;
    pend.base = base;
    pend.on = true;
    stm.mark(5);
    };
    // one instantiation of the tile body (the partial last tile's masks cost a few VALU per
    // step): a second, full-tile copy doubles the kernel's code for no measurable gain
    tile(std::false_type{});
    if (PF) cur = nxt;
  }  // tile loop
  if (pend.on) finish(pend);
  stm.flush();
}

// Chunk-start bitmap + per-message framing status for a batch of flat messages.
// Message i = words[off[i], off[i+1]): segment table (serializeSegmentTable serialize.c++:
// 311-330) then segments; chunk starts = message start, table end, each segment start.
__global__ void message_bits_kernel(const uint64_t* __restrict__ words,
                                    const uint64_t* __restrict__ off, uint64_t n,
                                    unsigned long long* __restrict__ bits,
                                    int32_t* __restrict__ status, TileFirstJob tf,
                                    uint32_t tf_block) {
  if (run_tile_first(tf, tf_block)) return;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t w0 = off[i], w1 = off[i + 1];
  int32_t st = 0;
  if (w1 <= w0) {
    if (status) status[i] = 11;  // CPK_ERR_EMPTY_MESSAGE
    return;
  }
  atomicOr(bits + (w0 >> 6), 1ull << (w0 & 63));
  const uint64_t nw = w1 - w0;
  const uint32_t* t32 = (const uint32_t*)(words + w0);
  const uint64_t nseg = (uint64_t)t32[0] + 1;
  const uint64_t tw = nseg / 2 + 1;
  bool ok = tw <= nw;
  if (ok) {
    uint64_t total = tw;
    for (uint64_t s = 0; s < nseg && total <= nw; s++) total += t32[s + 1];
    ok = total == nw;
  }
  if (!ok) {
    st = 6;  // CPK_ERR_BAD_FRAMING: packed as one chunk
  } else {
    uint64_t p = w0 + tw;
    if (p < w1) atomicOr(bits + (p >> 6), 1ull << (p & 63));
    for (uint64_t s = 0; s + 1 < nseg; s++) {
      p += t32[s + 1];
      if (p < w1) atomicOr(bits + (p >> 6), 1ull << (p & 63));
    }
  }
  if (status) status[i] = st;
}

__global__ void chunk_bits_kernel(const uint64_t* __restrict__ off, uint64_t n, uint64_t N,
                                  unsigned long long* __restrict__ bits, TileFirstJob tf,
                                  uint32_t tf_block) {
  if (run_tile_first(tf, tf_block)) return;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && N > 0) atomicOr(bits, 1ull);  // word 0 always starts a chunk
  if (i >= n) return;
  const uint64_t p = off[i];
  if (p < N && off[i + 1] > p) atomicOr(bits + (p >> 6), 1ull << (p & 63));
}

// tile_first[t] = first index i in [0, npos] with pos[i] >= t*T (binary search).

}  // namespace

// ---------------------------------------------------------------------------------------------
int pack_steps() {
  static int steps = [] {
    const char* e = getenv("CPK_PACK_STEPS");  // tuning knob: 4, 8 or 16 (default)
    const int v = e ? atoi(e) : kPackSteps;
    return (v == 8 || v == 16 || v == 4) ? v : kPackSteps;
  }();
  return steps;
}

template <int S, bool PF>
hipError_t launch_pack_s(const PackTileArgs& a, hipStream_t stream) {
  // persistent grid: every block resident (the stamp build has its own register footprint)
  static const unsigned cap =
      resident_blocks((const void*)pack_tiles_kernel<S, PF, false>, 256, 0);
  static const unsigned cap_st =
      resident_blocks((const void*)pack_tiles_kernel<S, PF, true>, 256, 0, 128);
  const uint64_t want = (a.ntiles + 3) / 4;
  const unsigned c = a.stamps ? cap_st : cap;
  const unsigned blocks = (unsigned)(want < c ? want : c);
  if (a.stamps)
    hipLaunchKernelGGL((pack_tiles_kernel<S, PF, true>), dim3(blocks), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL((pack_tiles_kernel<S, PF, false>), dim3(blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

// Prefetch of the next tile's words into registers during the current tile: on by default at
// 16 steps per tile, where LDS (the staging ring) and not registers bounds occupancy at 3 waves
// per SIMD; off at 8 steps, where the registers would cost occupancy.  Env CPK_PACK_PF=0/1.
static bool pack_prefetch() {
  static const bool on = [] {
    const char* e = getenv("CPK_PACK_PF");
    return e ? atoi(e) != 0 : pack_steps() == 16;
  }();
  return on;
}

// Two-pass form (default).  stage 0: count pass, persistent grid (its waves hand entry budgets
// over); stage 1: emit pass, one wave per tile.  The caller scans tile_bytes into tile_off in
// between.
template <int S>
hipError_t launch_pack_stage_s(int stage, const PackTileArgs& a, hipStream_t stream) {
  if (stage == 0) {
    static const unsigned cap =
        resident_blocks((const void*)pack_tiles_kernel<S, false, false, kCount>, 256, 0);
    const uint64_t want = (a.ntiles + 3) / 4;
    const unsigned blocks = (unsigned)(want < cap ? want : cap);
    hipLaunchKernelGGL((pack_tiles_kernel<S, false, false, kCount>), dim3(blocks), dim3(256), 0,
                       stream, a);
  } else {
    hipLaunchKernelGGL((pack_tiles_kernel<S, false, false, kEmit>),
                       dim3((unsigned)((a.ntiles + 3) / 4)), dim3(256), 0, stream, a);
  }
  return hipGetLastError();
}

hipError_t launch_pack_stage(int stage, const PackTileArgs& a, hipStream_t stream) {
  if (a.ntiles == 0) return hipSuccess;
  switch (pack_steps()) {
    case 4: return launch_pack_stage_s<4>(stage, a, stream);
    case 8: return launch_pack_stage_s<8>(stage, a, stream);
    default: return launch_pack_stage_s<16>(stage, a, stream);
  }
}

bool pack_fused() {
  static const bool on = [] {
    // A/B knob: CPK_PACK_TWO_PASS=1 selects count + scan + emit (measured slower on C2/C4/C5
    // than the single-pass kernel once the emission's LDS atomics were predicated)
    const char* e = getenv("CPK_PACK_TWO_PASS");
    return !(e && atoi(e) != 0);
  }();
  return on;
}

hipError_t launch_pack_tiles(const PackTileArgs& a, hipStream_t stream) {
  if (a.ntiles == 0) return hipSuccess;
  const bool pf = pack_prefetch();
  switch (pack_steps()) {
    case 4: return pf ? launch_pack_s<4, true>(a, stream) : launch_pack_s<4, false>(a, stream);
    case 8: return pf ? launch_pack_s<8, true>(a, stream) : launch_pack_s<8, false>(a, stream);
    default: return pf ? launch_pack_s<16, true>(a, stream) : launch_pack_s<16, false>(a, stream);
  }
}

hipError_t launch_message_bits(const uint64_t* words, const uint64_t* off, uint64_t n,
                               uint64_t* bits, int32_t* status, const TileFirstJob& tf,
                               hipStream_t stream) {
  const unsigned nb = (unsigned)((n + 255) / 256);
  if (nb + tile_first_blocks(tf) == 0) return hipSuccess;
  hipLaunchKernelGGL(message_bits_kernel, dim3(nb + tile_first_blocks(tf)), dim3(256), 0, stream,
                     words, off, n, (unsigned long long*)bits, status, tf, nb);
  return hipGetLastError();
}

hipError_t launch_chunk_bits(const uint64_t* off, uint64_t n, uint64_t N, uint64_t* bits,
                             const TileFirstJob& tf, hipStream_t stream) {
  const unsigned nb = (n == 0 && N == 0) ? 0u : (unsigned)((n + 256) / 256);
  if (nb + tile_first_blocks(tf) == 0) return hipSuccess;
  hipLaunchKernelGGL(chunk_bits_kernel, dim3(nb + tile_first_blocks(tf)), dim3(256), 0, stream,
                     off, n, N, (unsigned long long*)bits, tf, nb);
  return hipGetLastError();
}


}  // namespace cpk
