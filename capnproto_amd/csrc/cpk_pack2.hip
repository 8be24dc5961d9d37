// cpk_pack2.hip -- two-pass pack for gfx950: PackedOutputStream::write (capnproto c++/src/capnp/
// serialize-packed.c++:307-431) once per chunk, data-parallel, with no in-kernel wait on the
// output offsets.
//
// Word classes and sync points are those of cpk_pack.hip's file comment: Z all-zero, F no zero
// byte (tag 0xff), R at most one zero byte (F included), O the rest; a sync (chunk start, O word,
// first word of a Z or R stretch, a word past the batch end) resets the scalar loop's state.  A
// tile is 64*S words, one wave, S steps of 64 words (lane = word).  The batch is processed in
// groups of tiles ("slices") small enough to stay in the 256 MiB Infinity Cache between the two
// passes, so the words are read from HBM once:
//
//   count_kernel  (persistent)  per tile: tags, the Z / R / F ballots and the sync mask of every
//                 step; the tile's exact packed size; the budget entering every step (how many
//                 words the run open before it may still cover).  The only cross-tile hand-off
//                 is that budget: a tile publishes its exit budget as soon as its pre-pass is
//                 done when it holds a sync (it then does not depend on its entry), and a tile
//                 waits for its predecessor's only when its first word continues a stretch.
//   scan          tile byte counts -> output offsets (one workgroup per slice, carry in).
//   emit_kernel   (one wave per tile, no waits) the records of every step: heads and run
//                 coverage by scalar mask operations on the ballots (resolve_step), record
//                 lengths, a DPP prefix sum, v_perm compaction through a 256-entry selector
//                 table, records OR-ed into an LDS staging area laid out with the output's
//                 16-byte phase, then 16-byte stores.  A run's count comes from the next sync
//                 in the step, or, for a run still open at the step end, is stored when it
//                 closes; a run open at the tile end closes at the next tile's first sync
//                 (recorded by the count pass).  All-zero steps run on the scalar unit alone.
#include <stdlib.h>

#include <type_traits>

#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int L>
__device__ __forceinline__ uint32_t setlane(uint32_t dst, uint32_t v) {
  // v_writelane through an SALU move: a writelane reading an SGPR that a VALU (ballot) has just
  // written returned stale data (the hazard recognizer does not see through inline asm)
  uint32_t tmp;
  asm volatile("s_mov_b32 %1, %2\n\ts_nop 0\n\tv_writelane_b32 %0, %1, %3"
               : "+v"(dst), "=&s"(tmp)
               : "s"((uint32_t)__builtin_amdgcn_readfirstlane((int)v)), "i"(L));
  return dst;
}

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ uint32_t tag_of(uint32_t lo, uint32_t hi) {
  const uint32_t m7 = 0x7f7f7f7fu;
  const uint32_t a = ((lo & m7) + m7) | lo;
  const uint32_t b = ((hi & m7) + m7) | hi;
  const uint32_t c = ((a >> 7) & 0x01010101u) | ((b >> 3) & 0x10101010u);
  const uint32_t d = c | (c >> 14);
  return (d | (d >> 7)) & 0xffu;
}

__device__ __forceinline__ uint32_t msel(uint64_t mask, uint32_t if_set, uint32_t if_clear) {
  uint32_t r;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(mask));
  return r;
}

__device__ __forceinline__ uint32_t ffbl32(uint32_t v) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

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

struct StepRes {
  uint64_t covered, runheads, Zheads, Fheads;
  int b_out;
};

// Heads and coverage of one step with entry budget b (cpk_pack.hip resolve_step): a run open
// before the step covers the words before min(b, first sync); the first F of every R segment
// not so covered opens a run over the rest of its segment (255 > 63: it never closes inside the
// step); a Z stretch has its head at its first word, or at word b when the entering run expires.
__device__ __forceinline__ StepRes resolve_step(uint64_t Z, uint64_t F, uint64_t R, uint64_t SY,
                                                int b, bool last_valid) {
  const uint64_t LM = ~SY & (SY - 1);
  const uint64_t BM = b >= 64 ? ~0ull : mask_lt(b);
  const uint64_t lead_cov = BM & LM;
  const uint64_t zlead = (BM + 1) & LM & Z;
  const uint64_t Feff = F & ~lead_cov;
  const uint64_t G = (Feff << 1) & ~SY;
  const uint64_t fill = (((~SY + G) ^ ~SY) & ~SY) | G;
  const uint64_t Fheads = Feff & ~fill;
  const uint64_t Zheads = (Z & SY) | zlead;
  StepRes r;
  r.covered = (R & (fill | lead_cov)) | (Z & ~Zheads);
  r.runheads = Zheads | Fheads;
  r.Zheads = Zheads;
  r.Fheads = Fheads;
  r.b_out = 0;
  if (last_valid) {
    const int st = highest_bit(SY);
    const int h = highest_bit(r.runheads);
    if (h >= 0 && h >= st) r.b_out = 192 + h;
    else if (SY == 0 && b > 63) r.b_out = b - 64;
  }
  return r;
}

__device__ __forceinline__ uint64_t valid_mask(int n, int s) {
  const int k = n - 64 * s;
  return k >= 64 ? ~0ull : (k <= 0 ? 0ull : mask_lt(k));
}

template <int S>
struct Load2 {
  uint64_t x[S];  // word 64*s + lane
  uint64_t cb;    // lane s < S: chunk-start bits of step s
  uint64_t pw;    // word before the tile (0 for tile 0)
};

template <int S>
__device__ __forceinline__ void load2(const PackTileArgs& a, uint64_t t, Load2<S>& L) {
  constexpr int T = 64 * S;
  const int l = lane_id();
  const uint64_t N = a.nwords;
  const uint64_t tbase = t * T;
#pragma unroll
  for (int s = 0; s < S; s++) {
    const uint64_t g = tbase + 64 * s + l;
    L.x[s] = g < N ? a.words[g] : 0;
  }
  const uint64_t nbitw = (N + 63) >> 6;
  L.cb = (l < S && (tbase >> 6) + l < nbitw) ? a.chunk_bits[(tbase >> 6) + l] : 0;
  L.pw = tbase > 0 ? a.words[tbase - 1] : 0;
}

// Class of the word before the tile (zc: zero, rc: at most one zero byte).
__device__ __forceinline__ void prev_class(uint64_t tbase, uint64_t pw_lane, uint64_t& zc,
                                           uint64_t& rc) {
  zc = rc = 0;
  if (tbase > 0) {
    const uint64_t pw = uniform64(pw_lane);
    zc = pw == 0;
    rc = __popc(tag_of((uint32_t)pw, (uint32_t)(pw >> 32))) >= 7;
  }
}

// Sync mask of a step (chunk starts, O words, stretch starts, lanes past the batch end).
__device__ __forceinline__ uint64_t sync_mask(uint64_t C, uint64_t Z, uint64_t R, uint64_t V,
                                              uint64_t zc, uint64_t rc) {
  const uint64_t O = V & ~Z & ~R;
  return C | O | (Z & ~((Z << 1) | zc)) | (R & ~((R << 1) | rc)) | ~V;
}

// Bytes of the lead (the words before the first sync fs, all continuing one stretch) for entry
// budget b: a Z lead has its head at word b; an R lead is covered up to b, then its first F
// word opens a run over the rest of the lead.  Counted as the lead's part of
//   bytes = sum over non-Z words of (1 + nz) + 2 |Z heads| + |F heads| - |covered F words|.
__device__ __forceinline__ int lead_extra(bool zlead, uint64_t FL, int fs, int b) {
  if (zlead) return b < fs ? 2 : 0;
  if (b >= fs) return -__popcll(FL);
  const uint64_t after = FL & ~mask_lt(b);
  if (!after) return -__popcll(FL & mask_lt(b));
  const int q = lowest_bit(after);
  return 1 - __popcll(FL & mask_lt(b)) - __popcll(FL & ~mask_le(q));
}

// ---------------------------------------------------------------------------------------------
// Count pass.  Writes per tile: tile_bytes[t] (exact packed bytes), tile_b[t] (entry budget in
// bits 0-15, first sync in bits 16-31, capped at 256), step_b[t*S + s] (budget entering step s).
template <int S>
__global__ __launch_bounds__(256) void count_kernel(PackTileArgs a, uint64_t t0, uint64_t t1) {
  constexpr int T = 64 * S;
  const int l = lane_id();
  const int wv = (int)uniform32(threadIdx.x >> 6);
  const uint64_t N = a.nwords;
  uint32_t* const state = a.state;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  uint64_t t = t0 + (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  Load2<S> cur;
  if (t < t1) load2<S>(a, t, cur);
  for (; t < t1; t += nwaves) {
    Load2<S> nxt;
    if (t + nwaves < t1) load2<S>(a, t + nwaves, nxt);
    const uint64_t tbase = t * T;
    const uint64_t tend = tbase + T < N ? tbase + T : N;
    const int nvalid = (int)(tend - tbase);
    const int last = nvalid - 1;
    uint64_t zc, rc;
    prev_class(tbase, cur.pw, zc, rc);

    // ---- pre-pass: per step the sync mask, F mask and exit (parked in lanes), byte terms ----
    uint32_t vSYlo = 0, vSYhi = 0, vFlo = 0, vFhi = 0, vBX = 0;
    uint32_t acc = 0;   // per lane: sum of (1 + nz) over its non-zero words
    int extra0 = 0;     // 2 |Z heads| + |F heads| - |covered F| with every lead at budget 0
    int first_sync = T, last_sync = -1;
    bool lastZ = false, lastR = false;
    static_for<0, S>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      if (64 * s < nvalid) {
        const uint64_t V = valid_mask(nvalid, s);
        const uint64_t x = cur.x[s];
        const uint64_t Z = ballot(x == 0) & V;
        uint64_t R = 0, F = 0;
        if (Z != ~0ull) {
          const uint32_t tag = tag_of((uint32_t)x, (uint32_t)(x >> 32));
          const uint32_t nz = __popc(tag);
          acc += x != 0 ? nz + 1 : 0u;
          R = ballot(nz >= 7) & V;
          F = ballot(tag == 0xff) & V;
        }
        const uint64_t C = readlane64(cur.cb, s) & V;
        const uint64_t SY = sync_mask(C, Z, R, V, zc, rc);
        const bool lz = zc != 0, lr = rc != 0;  // class of the lead (continues the stretch)
        zc = Z >> 63;
        rc = R >> 63;
        const bool lv = 64 * s + 63 <= last;
        const StepRes r0 = resolve_step(Z, F, R, SY, 0, lv);
        extra0 += 2 * __popcll(r0.Zheads) + __popcll(r0.Fheads) - __popcll(r0.covered & F);
        // exit budget when the step holds a sync (entry-independent); else flags: 0x400 no
        // sync, 0x200 Z stretch.  Bits 0x800 / 0x1000: the lead is Z / R.
        uint32_t bx = SY ? (uint32_t)r0.b_out : (0x400u | (Z ? 0x200u : 0u));
        if (!(SY & 1)) bx |= lz ? 0x800u : (lr ? 0x1000u : 0u);
        vSYlo = setlane<s>(vSYlo, (uint32_t)SY);
        vSYhi = setlane<s>(vSYhi, (uint32_t)(SY >> 32));
        vFlo = setlane<s>(vFlo, (uint32_t)F);
        vFhi = setlane<s>(vFhi, (uint32_t)(F >> 32));
        vBX = setlane<s>(vBX, bx);
        const uint64_t SV = SY & V;
        if (SV) {
          if (first_sync == T) first_sync = 64 * s + lowest_bit(SV);
          last_sync = 64 * s + highest_bit(SV);
        }
        if (64 * s <= last && last < 64 * s + 64) {
          lastZ = (Z >> (last & 63)) & 1;
          lastR = (R >> (last & 63)) & 1;
        }
      }
    });
    auto F_of = [&](int s) -> uint64_t {
      return ((uint64_t)readlane32(vFhi, s) << 32) | readlane32(vFlo, s);
    };
    auto SY_of = [&](int s) -> uint64_t {
      return ((uint64_t)readlane32(vSYhi, s) << 32) | readlane32(vSYlo, s);
    };

    // ---- exit budget, published at once when the last stretch starts inside the tile ------
    if (first_sync < T) {
      int eb = 0;
      if (lastZ) {
        eb = 255 - ((last - last_sync) & 255);
      } else if (lastR) {
        int na = last_sync, qq = -1;
        for (int s = last_sync >> 6; s <= (last >> 6); s++) {
          const uint64_t m = F_of(s);
          while (na <= 64 * s + 63) {
            const uint64_t mm = na > 64 * s ? m & ~mask_lt(na - 64 * s) : m;
            if (!mm) break;
            qq = 64 * s + lowest_bit(mm);
            na = qq + 256;
          }
        }
        eb = (qq >= 0 && last - qq <= 255) ? 255 - (last - qq) : 0;
      }
      if (l == 0) store_agent32(state + t, 0x80000000u | (uint32_t)eb);
    }

    // ---- entry budget, then the budget entering every step and the leads' bytes -------------
    int b = 0;
    if (first_sync > 0 && t > 0) b = (int)(wait_nonzero32(state + t - 1, a.err) & 0xffu);
    const int b_entry = b;
    int extra = extra0;
    uint32_t vB = 0;
    static_for<0, S>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      if (64 * s < nvalid) {
        vB = setlane<s>(vB, (uint32_t)b);
        const uint32_t bx = readlane32(vBX, s);
        if (bx & 0x1800u) {  // the step opens with a lead: its bytes depend on the entry
          const uint64_t SY = SY_of(s);
          const int fs = SY ? lowest_bit(SY) : 64;
          const uint64_t FL = fs >= 64 ? F_of(s) : F_of(s) & mask_lt(fs);  // (1 << 64) is 1
          const bool zl = bx & 0x800u;
          extra += lead_extra(zl, FL, fs, b) - lead_extra(zl, FL, fs, 0);
        }
        if (!(bx & 0x400u)) b = (int)(bx & 0x1ffu);
        else if (b > 63) b -= 64;
        else if (bx & 0x200u) b += 192;
        else {
          const uint64_t Fm = F_of(s) & ~mask_lt(b);
          b = Fm ? 192 + lowest_bit(Fm) : 0;
        }
      }
    });
    if (first_sync == T && l == 0) store_agent32(state + t, 0x80000000u | (uint32_t)b);
    const uint32_t bytes = readlane32(wave_incl_sum32(acc), 63) + (uint32_t)extra;
    if (l == 0) {
      a.tile_bytes[t] = bytes;
      // first sync of the tile (the batch end counts), capped at 256: where a run open at the
      // end of the previous tile closes
      const int fsy = first_sync < nvalid ? first_sync : nvalid;
      a.tile_b[t] = (uint32_t)b_entry | ((uint32_t)(fsy < 256 ? fsy : 256) << 16);
    }
    if (l < S) a.step_b[t * S + l] = (uint8_t)vB;
    cur = nxt;
  }
}

// ---------------------------------------------------------------------------------------------
// Scan of one slice's tile byte counts: out[t + 1] = out[t0] + sum of in[t0 .. t], t in
// [t0, t1).  One workgroup of 1024 threads, each a contiguous run of tiles.
__global__ __launch_bounds__(1024) void slice_scan_kernel(const uint64_t* __restrict__ in,
                                                          uint64_t t0, uint64_t t1,
                                                          uint64_t* __restrict__ out) {
  __shared__ uint64_t wsum[16];
  const uint64_t n = t1 - t0;
  const uint64_t per = (n + 1023) / 1024;
  const uint64_t a0 = t0 + threadIdx.x * per;
  const uint64_t a1 = a0 + per < t1 ? a0 + per : t1;
  uint64_t s = 0;
  for (uint64_t i = a0; i < a1; i++) s += in[i];
  const uint64_t inc = wave_incl_sum64(s);
  const int w = threadIdx.x >> 6;
  if (lane_id() == 63) wsum[w] = inc;
  __syncthreads();
  uint64_t before = 0;
  for (int k = 0; k < w; k++) before += wsum[k];
  uint64_t run = (t0 == 0 ? 0 : out[t0]) + before + inc - s;
  if (t0 == 0 && threadIdx.x == 0) out[0] = 0;
  for (uint64_t i = a0; i < a1; i++) {
    run += in[i];
    out[i + 1] = run;
  }
}

// ---------------------------------------------------------------------------------------------
// Emit pass: one wave per tile of the slice [t0, t1), no waits.
template <int S>
struct EmitGeo {
  static constexpr int kStg = ((16 + 640 * S + 32) + 15) & ~15;  // phase pad + worst case + tail
};

template <int S>
__global__ __launch_bounds__(256) void emit_kernel(PackTileArgs a, uint64_t t0, uint64_t t1) {
  constexpr int T = 64 * S;
  constexpr int kStg = EmitGeo<S>::kStg;
  __shared__ __attribute__((aligned(16))) uint8_t stg_all[4][kStg];
  __shared__ uint64_t sel_tab[256];
  const int l = lane_id();
  const int wv = (int)uniform32(threadIdx.x >> 6);
  uint8_t* const stg = stg_all[wv];
  sel_tab[threadIdx.x] = make_sel(threadIdx.x);
  __syncthreads();
  const uint64_t t = t0 + (uint64_t)blockIdx.x * 4 + wv;
  if (t >= t1) return;

  const uint64_t gt_mask = ~mask_le(l);
  const uint32_t gt_lo = (uint32_t)gt_mask, gt_hi = (uint32_t)(gt_mask >> 32);
  const uint32_t lp1 = (uint32_t)l + 1u;
  const uint64_t N = a.nwords;
  const uint64_t nbitw = (N + 63) >> 6;
  const uint64_t tbase = t * T;
  const uint64_t tend = tbase + T < N ? tbase + T : N;
  const int nvalid = (int)(tend - tbase);
  const int last = nvalid - 1;

  Load2<S> cur;
  load2<S>(a, t, cur);
  const uint64_t excl = uniform64(a.tile_off[t]);
  const uint64_t agg = uniform64(a.tile_off[t + 1]) - excl;
  // budget entering step `lane` (count pass)
  const uint32_t vB = l < S ? (uint32_t)a.step_b[t * S + l] : 0u;
  uint64_t zc, rc;
  prev_class(tbase, cur.pw, zc, rc);

  // staging: output byte i of the tile at stg[ph + i], ph = the output's 16-byte phase; only
  // the part the records reach is cleared
  const uint64_t A0 = (uint64_t)(uintptr_t)a.out + excl;
  const uint32_t ph = (uint32_t)(A0 & 15);
  const bool over = excl + agg > a.out_capacity;
  if (over && l == 0) raise_error(a.err, kErrCapacity);
  {
    const uint32_t nclr = (ph + (uint32_t)(agg < (uint64_t)(640 * S) ? agg : 640 * S) + 47) / 16;
    for (uint32_t i = l; i < nclr && i < (uint32_t)(kStg / 16); i += 64)
      ((u32x4*)stg)[i] = (u32x4){0, 0, 0, 0};
    lane_handoff();
  }

  const uint64_t pidx0 = a.pos ? uniform64(a.tile_first[t]) : 0;
  uint64_t pidx = pidx0;
  uint32_t prel = ~0u;
  if (a.pos && pidx <= a.npos) {
    const uint64_t pn = uniform64(a.pos[pidx]);
    if (pn - tbase < (uint64_t)T) prel = (uint32_t)(pn - tbase);
  }
  uint32_t boff = 0;      // tile-relative bytes so far
  bool own = false;       // the run open at the step start has its head in this tile
  uint32_t own_cnt = 0;   // words it has covered so far
  uint32_t own_at = 0;    // staging byte of its count
  static_for<0, S>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    if (64 * s < nvalid) {
      const uint64_t V = valid_mask(nvalid, s);
      const bool lv = 64 * s + 63 <= last;
      const uint64_t x = cur.x[s];
      const uint64_t Z = ballot(x == 0) & V;
      const int b_in = (int)readlane32(vB, s);
      uint64_t R = 0, F = 0;
      uint32_t tag = 0;
      if (Z != ~0ull) {
        tag = tag_of((uint32_t)x, (uint32_t)(x >> 32));
        R = ballot(__popc(tag) >= 7) & V;
        F = ballot(tag == 0xff) & V;
      }
      const uint64_t C = readlane64(cur.cb, s) & V;
      const uint64_t SY = sync_mask(C, Z, R, V, zc, rc);
      zc = Z >> 63;
      rc = R >> 63;
      const int fs = SY ? lowest_bit(SY) : 64;
      const StepRes r = resolve_step(Z, F, R, SY, b_in, lv);
      int open_h = -1;       // head of a run opened in this step and still open at its end
      uint32_t open_at = 0;  // staging byte of that run's count
      const bool open = r.b_out > 0 && r.runheads && highest_bit(r.runheads) >= highest_bit(SY);
      uint32_t step_bytes;
      if (Z == ~0ull && !(prel < 64u * s + 64u)) {
        // all-zero step: the records are the Z heads, two bytes each ([00, count]); the tag
        // byte stays zero in the staging area and only a non-zero count is stored
        uint64_t hm = r.Zheads;
        uint32_t k = 0;
        while (hm) {
          const int h = lowest_bit(hm);
          hm &= hm - 1;
          const uint64_t after = SY & ~mask_le(h);
          if (after) {
            const uint32_t cnt = (uint32_t)(lowest_bit(after) - h - 1);
            if (cnt && l == 0) stg[ph + boff + 2 * k + 1] = (uint8_t)cnt;
          }
          k++;
        }
        step_bytes = 2 * k;
        if (open) {
          open_h = highest_bit(r.runheads);
          open_at = ph + boff + step_bytes - 1u;
        }
      } else {
        const uint32_t nz = __popc(tag);
        const uint64_t COV = r.covered | ~V;
        const uint64_t ZH = r.Zheads, FH = r.Fheads;
        const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
        const uint32_t n1 = nz + 1;
        const uint32_t len = msel(COV, n1 & 8u, n1 + msel(ZH | FH, 1u, 0u));
        const uint32_t inc = wave_incl_sum32(len);
        const uint32_t o = boff + inc - len;
        // run count of a head whose run ends in this step: the words up to the next sync
        const uint32_t f_lo = ffbl32((uint32_t)SY & gt_lo);
        const uint32_t f_hi =
            __builtin_elementwise_add_sat(ffbl32((uint32_t)(SY >> 32) & gt_hi), 32u);
        const uint32_t ns = min(f_lo, f_hi);
        const uint32_t cnt = ns < 64u ? ns - lp1 : 0u;  // a run still open: stored at close
        const uint64_t sel = sel_tab[tag];
        const uint32_t c8 = cnt << 8;
        uint32_t w0 = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel) | tag | msel(ZH, c8, 0u);
        uint32_t w1 = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
        const uint32_t w2 = msel(FH, (hi >> 24) | c8, 0u);
        w0 = msel(COV, lo, w0);
        w1 = msel(COV, hi, w1);
        const uint32_t at = ph + o + 16u;  // +16: keeps (at - 1) non-negative
        const uint32_t rr = (0u - at) & 3u;
        const uint32_t kk = 4u - rr;
        const uint32_t ee = kk + len;
        uint32_t* dp = (uint32_t*)(stg + ((at - 1u) & ~3u) - 16);
        if (kk < 4u && len) atomicOr(dp + 0, __builtin_amdgcn_alignbyte(w0, 0u, rr));
        if (ee > 4u) atomicOr(dp + 1, __builtin_amdgcn_alignbyte(w1, w0, rr));
        if (ee > 8u) atomicOr(dp + 2, __builtin_amdgcn_alignbyte(w2, w1, rr));
        if (ee > 12u) atomicOr(dp + 3, __builtin_amdgcn_alignbyte(0u, w2, rr));
        step_bytes = readlane32(inc, 63);
        // requested positions inside this step (message starts): absolute packed offsets
        if (prel < 64u * s + 64u) {
          const uint64_t g0 = tbase + 64 * s;
          while (true) {
            const uint64_t i = pidx + l;
            const uint64_t p = i <= a.npos ? a.pos[i] : ~0ull;
            const bool in = p < g0 + 64;
            const uint32_t oo = shfl32(o, in ? (int)(p - g0) : 0);
            if (in) a.pos_out[i] = excl + oo;
            const uint64_t inm = ballot(in);
            pidx += __popcll(inm);
            const uint64_t pn = pidx <= a.npos ? uniform64(a.pos[pidx]) : ~0ull;
            prel = pn - tbase < (uint64_t)T ? (uint32_t)(pn - tbase) : ~0u;
            if (inm != ~0ull) break;
          }
        }
        if (open) {
          open_h = highest_bit(r.runheads);
          open_at = ph + readlane32(o, open_h) + (((ZH >> open_h) & 1) ? 1u : 9u);
        }
      }
      // the run entering the step, if its head is in this tile: does it close here?
      if (own) {
        const int cov = b_in < fs ? b_in : fs;
        own_cnt += (uint32_t)cov;
        if (cov < 64 || b_in <= 64) {
          if (l == 0) stg[own_at] = (uint8_t)own_cnt;
          own = false;
        }
      }
      if (open_h >= 0) {
        own = true;
        own_cnt = (uint32_t)(63 - open_h);
        own_at = open_at;
      } else if (r.b_out == 0) {
        own = false;
      }
      boff += step_bytes;
    }
  });
  // a run still open at the tile end closes at the next tile's first sync (within its budget):
  // recorded by the count pass, or -- for the last tile of a slice, whose successor is counted
  // later -- found by looking at the following words
  if (own) {
    const int b_end = 255 - (int)own_cnt;
    int la = 0;
    if (tend < N) {
      if (t + 1 < t1) {
        la = (int)(uniform32(a.tile_b[t + 1]) >> 16);
      } else {
        uint64_t czc = zc, crc = rc;
        la = 256;
        for (int k = 0; k < 4 && la == 256 && 64 * k < b_end; k++) {
          const uint64_t g = tend + 64 * k + l;
          const uint64_t xx = g < N ? a.words[g] : 0;
          const uint64_t ck = ((tend >> 6) + k < nbitw) ? a.chunk_bits[(tend >> 6) + k] : 0;
          const uint32_t tg = tag_of((uint32_t)xx, (uint32_t)(xx >> 32));
          const uint64_t V = ballot(g < N);
          const uint64_t Zk = ballot(xx == 0) & V;
          const uint64_t Rk = ballot(__popc(tg) >= 7) & V;
          const uint64_t SYk = sync_mask(ck, Zk, Rk, V, czc, crc);
          if (SYk) la = 64 * k + lowest_bit(SYk);
          czc = Zk >> 63;
          crc = Rk >> 63;
        }
      }
    }
    own_cnt += (uint32_t)(b_end < la ? b_end : la);
    if (l == 0) stg[own_at] = (uint8_t)own_cnt;
  }
  if (a.pos && tend == N) {
    for (uint64_t i = pidx + l; i <= a.npos; i += 64) a.pos_out[i] = excl + agg;
  }
  if (tend == N && l == 0 && a.total_out) *a.total_out = excl + agg;

  // ---- flush: 16-byte blocks (the staging area has the output's phase), bytes at the ends --
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (!over && agg) {
    const uint64_t A1 = A0 + agg;
    const uint64_t al = (A0 + 15) & ~15ull;  // first whole block
    const uint64_t top = A1 & ~15ull;        // end of the whole blocks
    if (al >= top) {
      for (uint32_t i = l; i < agg; i += 64) *(uint8_t*)(uintptr_t)(A0 + i) = stg[ph + i];
    } else {
      if (A0 + l < al) *(uint8_t*)(uintptr_t)(A0 + l) = stg[ph + l];
      const uint32_t nb = (uint32_t)((top - al) >> 4);
      const uint32_t so0 = ph + (uint32_t)(al - A0);  // multiple of 16
      for (uint32_t i = l; i < nb; i += 64)
        *(u32x4*)(uintptr_t)(al + 16ull * i) = *(const u32x4*)(stg + so0 + 16 * i);
      if (top + l < A1) *(uint8_t*)(uintptr_t)(top + l) = stg[ph + (uint32_t)(top - A0) + l];
    }
  }
}

}  // namespace

int pack2_steps() {
  static const int steps = [] {
    const char* e = getenv("CPK_PACK2_STEPS");  // tuning knob: 8 or 16 (default)
    const int v = e ? atoi(e) : 16;
    return (v == 8 || v == 16) ? v : 16;
  }();
  return steps;
}

bool pack_v2() {
  // A/B knob CPK_PACK_V2=1 (off by default: the count pass is bound by scalar instructions)
  static const bool on = [] {
    const char* e = getenv("CPK_PACK_V2");
    return e && atoi(e) != 0;
  }();
  return on;
}

// Tiles per slice: the slice's words stay in the Infinity Cache between the count and emit
// passes (env CPK_PACK2_SLICE_MB, default 96 MiB of words).
static uint64_t slice_tiles(uint64_t T) {
  static const uint64_t mb = [] {
    const char* e = getenv("CPK_PACK2_SLICE_MB");
    const long v = e ? atol(e) : 96;
    return (uint64_t)(v > 0 ? v : 96);
  }();
  const uint64_t n = (mb << 20) / (T * 8);
  return n ? n : 1;
}

template <int S>
static hipError_t launch_pack2_s(const PackTileArgs& a, hipStream_t stream) {
  constexpr uint64_t T = 64 * S;
  static const unsigned cap = resident_blocks((const void*)count_kernel<S>, 256, 0);
  const uint64_t per = slice_tiles(T);
  for (uint64_t t0 = 0; t0 < a.ntiles; t0 += per) {
    const uint64_t t1 = t0 + per < a.ntiles ? t0 + per : a.ntiles;
    const uint64_t want = (t1 - t0 + 3) / 4;
    const unsigned blocks = (unsigned)(want < cap ? want : cap);
    hipLaunchKernelGGL((count_kernel<S>), dim3(blocks), dim3(256), 0, stream, a, t0, t1);
    hipLaunchKernelGGL(slice_scan_kernel, dim3(1), dim3(1024), 0, stream, a.tile_bytes, t0, t1,
                       a.tile_off);
    hipLaunchKernelGGL((emit_kernel<S>), dim3((unsigned)want), dim3(256), 0, stream, a, t0, t1);
  }
  return hipGetLastError();
}

hipError_t launch_pack_tiles2(const PackTileArgs& a, hipStream_t stream) {
  if (a.ntiles == 0) return hipSuccess;
  if (pack2_steps() == 8) return launch_pack2_s<8>(a, stream);
  return launch_pack2_s<16>(a, stream);
}

}  // namespace cpk
