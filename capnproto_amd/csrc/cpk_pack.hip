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
// Work decomposition: the batch of words is cut into tiles of 64*S words, one wave per tile
// (tile ids from an atomic counter, so every predecessor of a running tile is resident).  The
// wave classifies its words (pass 1), publishes the budget its tile hands to the successor when
// that does not depend on its own entry, takes its entry budget from the predecessor only when
// word 0 continues a stretch, then encodes every step once into a per-wave LDS staging buffer
// (pass 2, tile-relative byte offsets).  The tile's byte count feeds a single-pass decoupled
// look-back; with the global offset known the staged bytes leave as 16-byte aligned stores
// (realigned with v_alignbyte), only the <= 15-byte partial blocks at tile edges as byte stores.
#include <stdlib.h>

#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Lane's bit of a wave-uniform 64-bit mask held in an SGPR pair: one v_cndmask.
__device__ __forceinline__ uint32_t lanebit(uint64_t mask) {
  uint32_t r;
  asm("v_cndmask_b32 %0, 0, 1, %1" : "=v"(r) : "s"(mask));
  return r;
}

// v_perm selector compacting the set-bit bytes of nibble n to the low end (0x0c = zero byte).
__device__ __forceinline__ uint32_t compact_sel(uint32_t n) {
  uint32_t sel = 0x0c0c0c0cu, j = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if ((n >> i) & 1) {
      sel = (sel & ~(0xffu << (8 * j))) | ((uint32_t)i << (8 * j));
      j++;
    }
  }
  return sel;
}

struct Classes {
  uint64_t Z, F, R, SY, V;
};

// Class masks + sync mask of one 64-word step (lane = word).  zc/rc: the word before the step
// is a valid Z / R word of the same chunk-run (chunk starts are part of C).
__device__ __forceinline__ Classes classify_step(uint64_t x, uint32_t tag, bool valid, uint64_t C,
                                                 uint64_t zc, uint64_t rc) {
  const uint32_t nz = __popc(tag);
  Classes k;
  k.Z = ballot(valid && x == 0);
  k.F = ballot(valid && tag == 0xff);
  k.R = ballot(valid && nz >= 7);
  const uint64_t V = ballot(valid);
  k.V = V;
  const uint64_t O = V & ~k.Z & ~k.R;
  const uint64_t prevZ = (k.Z << 1) | zc;
  const uint64_t prevR = (k.R << 1) | rc;
  k.SY = C | O | (k.Z & ~prevZ) | (k.R & ~prevR) | ~V;
  return k;
}

// Head / coverage resolution of one step, entry budget b (words the run open before the step
// may still cover).  All wave-uniform mask arithmetic.
struct StepRes {
  uint64_t covered, runheads;  // covered words; Z heads | F heads
  int b_out;                   // budget leaving the step
};

__device__ __forceinline__ StepRes resolve_step(const Classes& k, int b, bool last_valid) {
  const uint64_t SY = k.SY, U = ~SY;
  const int L0 = lowest_bit(SY);  // 64 if no sync in the step
  const bool leadZ = L0 > 0 && (k.Z & 1);
  const bool leadR = L0 > 0 && (k.R & 1);
  const int cb = b < L0 ? b : L0;  // words of the lead covered by the entering run
  const uint64_t lead_cov = cb >= 64 ? ~0ull : mask_lt(cb);
  const uint64_t zlead = (leadZ && b < L0) ? (1ull << b) : 0;
  const uint64_t Feff = leadR ? (k.F & ~lead_cov) : k.F;
  const uint64_t G = (Feff << 1) & U;
  const uint64_t fill = (((U + G) ^ U) & U) | G;  // words after an F head, same segment
  const uint64_t Rcov = k.R & (fill | (leadR ? lead_cov : 0));
  const uint64_t Fheads = Feff & ~fill;
  const uint64_t Zheads = (k.Z & SY) | zlead;
  StepRes r;
  r.covered = Rcov | (k.Z & ~Zheads);
  r.runheads = Zheads | Fheads;
  r.b_out = 0;
  if (last_valid && (((k.Z | k.R) >> 63) & 1)) {
    const int st63 = highest_bit(SY);
    const int h = highest_bit(r.runheads);
    if (h >= 0 && h >= st63) r.b_out = 255 - (63 - h);
    else if (st63 < 0 && b > 63) r.b_out = b - 64;
  }
  return r;
}

// Words a tile needs, loaded one tile ahead (persistent loop prefetch).
template <int S>
struct TileLoad {
  uint64_t x[S];  // word 64*s + lane
  uint64_t cb;    // chunk-start bits of step `lane` (lanes < S)
  uint64_t pw;    // word before the tile
  uint64_t nx;    // first step of the next tile (look-ahead for run counts)
  uint64_t ncb;   // its chunk-start bits
};

template <int S>
__device__ __forceinline__ void load_tile(const PackTileArgs& a, uint64_t t, TileLoad<S>& L) {
  constexpr int T = 64 * S;
  const int l = lane_id();
  const uint64_t N = a.nwords;
  const uint64_t nbitw = (N + 63) >> 6;
  const uint64_t tbase = t * T;
  const uint64_t tend = tbase + T < N ? tbase + T : N;
#pragma unroll
  for (int s = 0; s < S; s++) {
    const uint64_t g = tbase + 64 * s + l;
    L.x[s] = g < N ? a.words[g] : 0;
  }
  L.cb = (l < S && (tbase >> 6) + l < nbitw) ? a.chunk_bits[(tbase >> 6) + l] : 0;
  L.pw = tbase > 0 ? a.words[tbase - 1] : 0;
  L.nx = tend + l < N ? a.words[tend + l] : 0;
  L.ncb = (tend >> 6) < nbitw ? a.chunk_bits[tend >> 6] : 0;
}

template <int S, bool STAMPS>
__global__ __launch_bounds__(256) void pack_tiles_kernel(PackTileArgs a) {
  static_assert(S >= 1 && S <= 32, "S steps per tile");
  constexpr int T = 64 * S;
  constexpr int kRing = 1024;  // per-wave output ring (one step emits <= 640 bytes)
  __shared__ __attribute__((aligned(16))) uint8_t lds_ring[4][kRing];

  const int l = lane_id();
  const int wv = (int)uniform32(threadIdx.x >> 6);  // wave-uniform (keeps tile math scalar)
  uint8_t* ring = lds_ring[wv];
  *(u32x4*)(ring + 16 * l) = (u32x4){0, 0, 0, 0};
  const uint32_t csel = compact_sel((uint32_t)l & 15);
  const uint64_t gt_mask = ~mask_le(l);  // lanes above this one
  const uint64_t N = a.nwords;
  const uint64_t nbitw = (N + 63) >> 6;
  const uint64_t base_addr = (uint64_t)(uintptr_t)a.out;
  uint32_t* const state = a.state;

  // Persistent waves, static strided tile order (grid <= guaranteed residency, see launch):
  // a tile only waits on lower tiles, which belong to resident waves that reach them first.
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  Stamps<STAMPS> stm;
  uint64_t t = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  TileLoad<S> cur;
  if (t < a.ntiles) load_tile<S>(a, t, cur);
  for (; t < a.ntiles; t += nwaves) {
    stm.start(a.stamps);
    const uint64_t tbase = t * T;
    const uint64_t tend = tbase + T < N ? tbase + T : N;
    const int nvalid = (int)(tend - tbase);
    const int last = nvalid - 1;
    const int nsteps = (nvalid + 63) >> 6;
    uint64_t zc = 0, rc = 0;
    if (tbase > 0) {
      zc = cur.pw == 0;
      rc = __popc(word_tag(cur.pw)) >= 7;
    }

    // ---- pass 1: classes (lane s keeps step s's masks) and O-word bytes ----------------------
    uint64_t myZ = 0, myF = 0, myR = 0, mySY = 0;
    uint32_t myOB = 0;
    int first_sync = T;
    {
      uint64_t czc = zc, crc = rc;
#pragma unroll
      for (int s = 0; s < S; s++) {
        const bool valid = 64 * s + l < nvalid;
        const uint32_t tag = word_tag(cur.x[s]);
        const Classes k = classify_step(cur.x[s], tag, valid, readlane64(cur.cb, s), czc, crc);
        czc = k.Z >> 63;
        crc = k.R >> 63;
        const uint64_t syv = k.SY & k.V;
        if (first_sync == T && syv) first_sync = 64 * s + lowest_bit(syv);
        // bytes of O words (always heads, state independent): 1 + nz <= 7
        const uint32_t nz = __popc(tag);
        const uint32_t ob = (valid && cur.x[s] != 0 && nz < 7) ? 1 + nz : 0;
        const uint32_t OB = (uint32_t)(__popcll(ballot(ob & 1)) + 2 * __popcll(ballot(ob & 2)) +
                                       4 * __popcll(ballot(ob & 4)));
        if (l == s) {
          myZ = k.Z;
          myF = k.F;
          myR = k.R;
          mySY = k.SY;
          myOB = OB;
        }
      }
    }
    stm.mark(0);  // pass 1

    // ---- look-ahead: first sync after the tile (run counts need <= 255 words) -----------------
    int la = 0;
    {
      const bool lastZ = (readlane64(myZ, last >> 6) >> (last & 63)) & 1;
      const bool lastR = (readlane64(myR, last >> 6) >> (last & 63)) & 1;
      if ((lastZ || lastR) && tend < N) {
        uint64_t czc = lastZ, crc = lastR;
        la = 256;
        for (int k = 0; k < 4; k++) {
          const uint64_t g = tend + 64 * k + l;
          const bool valid = g < N;
          uint64_t xx, C;
          if (k == 0) {
            xx = cur.nx;
            C = cur.ncb;
          } else {
            xx = valid ? a.words[g] : 0;
            C = ((tend >> 6) + k < nbitw) ? a.chunk_bits[(tend >> 6) + k] : 0;
          }
          const Classes kk = classify_step(xx, word_tag(xx), valid, C, czc, crc);
          czc = kk.Z >> 63;
          crc = kk.R >> 63;
          if (kk.SY) {
            la = 64 * k + lowest_bit(kk.SY);
            break;
          }
        }
      }
    }
    int myNsa = 0;  // lane s: distance from step s+1 to the first sync at or after it (<= 256)
    {
      int v = la;
      for (int s = S - 1; s >= 0; s--) {
        if (l == s) myNsa = v;
        const int fs = lowest_bit(readlane64(mySY, s));
        v = s >= nsteps ? la : (fs < 64 ? fs : (v + 64 < 256 ? v + 64 : 256));
      }
    }

    // ---- exit budget, published early when it does not depend on our own entry --------------
    auto first_F_from = [&](int xpos) -> int {
      for (int k = xpos >> 6; k < nsteps; k++) {
        uint64_t m = readlane64(myF, k);
        if (k == (xpos >> 6)) m &= ~mask_lt(xpos & 63);
        if (m) return 64 * k + lowest_bit(m);
      }
      return 1 << 20;
    };
    if (first_sync < T) {
      int sg = -1;
      for (int k = last >> 6; k >= 0; k--) {
        uint64_t m = readlane64(mySY, k);
        if (k == (last >> 6)) m &= mask_le(last & 63);
        if (m) {
          sg = 64 * k + highest_bit(m);
          break;
        }
      }
      const bool sZ = (readlane64(myZ, sg >> 6) >> (sg & 63)) & 1;
      const bool sR = (readlane64(myR, sg >> 6) >> (sg & 63)) & 1;
      int eb = 0;
      if (sZ) {
        eb = 255 - ((last - sg) & 255);
      } else if (sR) {
        int qq = -1;
        for (int q = first_F_from(sg); q <= last; q = first_F_from(q + 256)) qq = q;
        eb = (qq >= 0 && last - qq <= 255) ? 255 - (last - qq) : 0;
      }
      if (l == 0) store_agent32(state + t, 0x80000000u | (uint32_t)eb);
    }
    stm.mark(1);  // look-ahead, run-count table, early exit budget
    int b = 0;
    if (first_sync > 0 && t > 0) b = (int)(wait_nonzero32(state + t - 1, a.err) & 0xffu);
    stm.mark(2);  // entry wait

    // ---- count pass (scalar): per-step coverage and byte offsets ------------------------------
    //   bytes(step) = 8 |R| + 2 |Z heads + F heads| + sum over O words of (1 + nz)
    uint64_t myCov = 0;
    uint32_t myOff = 0;
    uint32_t off = 0;
    for (int s = 0; s < nsteps; s++) {
      Classes k;
      k.Z = readlane64(myZ, s);
      k.F = readlane64(myF, s);
      k.R = readlane64(myR, s);
      k.SY = readlane64(mySY, s);
      const StepRes r = resolve_step(k, b, 64 * s + 63 < nvalid);
      const uint32_t bytes = readlane32(myOB, s) + 8 * (uint32_t)__popcll(k.R) +
                             2 * (uint32_t)__popcll(r.runheads);
      if (l == s) {
        myCov = r.covered;
        myOff = off;
      }
      off += bytes;
      b = r.b_out;
    }
    if (first_sync == T && l == 0) store_agent32(state + t, 0x80000000u | (uint32_t)b);
    const uint64_t agg = off;
    stm.mark(3);  // count pass

    // ---- publish, prefetch the next tile, look-back ------------------------------------------
    uint64_t excl = 0;
    if (a.debug_skip & 1) {
      excl = t * 4096;  // timing ablation: no look-back (output meaningless)
    } else {
      publish_agg(a.desc, a.gdesc, a.gcnt, t, a.ntiles, agg, 0, a.err);
    }
    TileLoad<S> nxt;
    if (t + nwaves < a.ntiles) load_tile<S>(a, t + nwaves, nxt);
    if (!(a.debug_skip & 1)) {
      excl = lookback2(a.desc, a.gdesc, t, 0, a.err);
      publish_incl(a.desc, a.gdesc, t, a.ntiles, excl + agg);
    }
    stm.mark(4);  // look-back

    // ---- emission: encode each step through the ring, 16-byte aligned stores ----------------
    const uint64_t A0 = base_addr + excl;
    const uint64_t A1 = A0 + agg;
    const bool over = excl + agg > a.out_capacity;
    if (over && l == 0) raise_error(a.err, kErrCapacity);
    const uint64_t al = (A0 + 15) & ~15ull;
    uint64_t flushed = al;  // next full block to store
    uint64_t hd = A0;       // next head-block byte to store
    uint64_t pidx = a.pos ? uniform64(a.tile_first[t]) : 0;
    uint64_t pnext = (a.pos && pidx <= a.npos) ? uniform64(a.pos[pidx]) : ~0ull;
    for (int s = 0; s < nsteps && !over; s++) {
      const uint64_t Z = readlane64(myZ, s), F = readlane64(myF, s), R = readlane64(myR, s);
      const uint64_t SY = readlane64(mySY, s), COV = readlane64(myCov, s);
      const uint32_t soff = readlane32(myOff, s);
      const int nsa = (int)readlane32((uint32_t)myNsa, s);
      uint64_t xv = 0;
#pragma unroll
      for (int ss = 0; ss < S; ss++)
        if (ss == s) xv = cur.x[ss];
      const uint32_t tag = word_tag(xv);
      const uint32_t isZ = lanebit(Z), isF = lanebit(F), isR = lanebit(R), cov = lanebit(COV);
      const bool valid = 64 * s + l < nvalid;
      // bytes of this word's record
      const uint32_t hlen = isZ ? 2u : (isF ? 10u : 1u + (uint32_t)__popc(tag));
      const uint32_t len = !valid ? 0u : (cov ? (isR ? 8u : 0u) : hlen);
      // run count of Z / F heads: min(255, stretch words left after this one)
      const uint64_t gt = SY & gt_mask;
      const int ns = gt ? lowest_bit(gt) : 64 + nsa;
      const uint32_t cnt = (uint32_t)min(ns - l - 1, 255);
      // string: slo = bytes 0..7, shi = bytes 8..9 (branch-free selects)
      const uint32_t xlo = (uint32_t)xv, xhi = (uint32_t)(xv >> 32);
      const uint32_t tl = tag & 15, th = tag >> 4;
      const uint32_t clo = __builtin_amdgcn_perm(0u, xlo, shfl32(csel, (int)tl));
      const uint32_t chi = __builtin_amdgcn_perm(0u, xhi, shfl32(csel, (int)th));
      const uint64_t comp = (uint64_t)clo | ((uint64_t)chi << (8 * __popc(tl)));
      const uint64_t s_head = (uint64_t)tag | (comp << 8);
      const uint64_t s_f = 0xffull | (xv << 8);
      const uint64_t s_z = (uint64_t)cnt << 8;
      const uint64_t slo = cov ? xv : (isZ ? s_z : (isF ? s_f : s_head));
      const uint32_t shi = (!cov && isF) ? ((xhi >> 24) | (cnt << 8)) : 0u;
      uint32_t total;
      const uint32_t o = wave_excl_sum_small(len, &total);
      const uint64_t A = A0 + soff;
      {
        // OR the string into the ring (zeroed), dword-aligned to its global address
        const uint64_t at = A + o;
        const uint32_t al4 = (uint32_t)at & 3;
        const uint32_t w0 = (uint32_t)slo, w1 = (uint32_t)(slo >> 32), w2 = shi;
        const uint32_t sh = 4 - al4;
        const uint32_t e0 = w0 << (8 * al4);
        const uint32_t e1 = al4 ? __builtin_amdgcn_alignbyte(w1, w0, sh) : w1;
        const uint32_t e2 = al4 ? __builtin_amdgcn_alignbyte(w2, w1, sh) : w2;
        const uint32_t e3 = al4 ? __builtin_amdgcn_alignbyte(0u, w2, sh) : 0u;
        const uint32_t nd = len ? (al4 + len + 3) >> 2 : 0;
        const uint32_t d0 = (uint32_t)(at >> 2);
        uint32_t* rw = (uint32_t*)ring;
        constexpr uint32_t M = kRing / 4 - 1;
        if (nd > 0) atomicOr(rw + ((d0 + 0) & M), e0);
        if (nd > 1) atomicOr(rw + ((d0 + 1) & M), e1);
        if (nd > 2) atomicOr(rw + ((d0 + 2) & M), e2);
        if (nd > 3) atomicOr(rw + ((d0 + 3) & M), e3);
      }
      // requested output offsets (message / chunk starts) inside this step
      const uint64_t g0 = tbase + 64 * s;
      while (pnext < g0 + 64) {
        const uint64_t i = pidx + l;
        const uint64_t p = i <= a.npos ? a.pos[i] : ~0ull;
        const bool in = p < g0 + 64;
        const uint32_t oo = shfl32(o, in ? (int)(p - g0) : 0);
        if (in) a.pos_out[i] = excl + soff + oo;
        const uint64_t inm = ballot(in);
        pidx += __popcll(inm);
        pnext = pidx <= a.npos ? uniform64(a.pos[pidx]) : ~0ull;
        if (inm != ~0ull) break;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const uint64_t Aend = A + total;
      // partial head block (shared with the previous tile's bytes): byte stores
      const uint64_t hlim = Aend < al ? Aend : al;
      if (hd < hlim) {
        const uint64_t p = hd + l;
        if (l < 16 && p < hlim) {
          uint8_t* rb = ring + (p & (kRing - 1));
          *(uint8_t*)(uintptr_t)p = *rb;
          *rb = 0;
        }
        hd = hlim;
      }
      // full 16-byte blocks
      const uint64_t top = Aend & ~15ull;
      if (top > flushed) {
        const uint32_t nb = (uint32_t)((top - flushed) >> 4);
        for (uint32_t i0 = 0; i0 < nb; i0 += 64) {
          const uint32_t i = i0 + l;
          if (i < nb) {
            const uint64_t p = flushed + 16ull * i;
            u32x4* rb = (u32x4*)(ring + (p & (kRing - 1)));
            const u32x4 v = *rb;
            *rb = (u32x4){0, 0, 0, 0};
            *(u32x4*)(uintptr_t)p = v;
          }
        }
        flushed = top;
      }
    }
    if (!over) {
      // partial tail block
      const uint64_t from = flushed > hd ? flushed : hd;
      const uint64_t p = from + l;
      if (l < 16 && p < A1) {
        uint8_t* rb = ring + (p & (kRing - 1));
        *(uint8_t*)(uintptr_t)p = *rb;
        *rb = 0;
      }
    }
    // positions at or past the end of the batch -> total
    if (a.pos && tend == N) {
      const uint64_t tot = excl + agg;
      for (uint64_t i = pidx + l; i <= a.npos; i += 64) a.pos_out[i] = tot;
      if (l == 0 && a.total_out) *a.total_out = tot;
    }
    stm.mark(5);  // emission
    if (STAMPS && l == 0 && a.stamps) atomicAdd(a.stamps + 15, 1ull);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    cur = nxt;
  }  // tile loop
}

// Chunk-start bitmap + per-message framing status for a batch of flat messages.
// Message i = words[off[i], off[i+1]): segment table (serializeSegmentTable serialize.c++:
// 311-330) then segments; chunk starts = message start, table end, each segment start.
__global__ void message_bits_kernel(const uint64_t* __restrict__ words,
                                    const uint64_t* __restrict__ off, uint64_t n,
                                    unsigned long long* __restrict__ bits,
                                    int32_t* __restrict__ status) {
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
                                  unsigned long long* __restrict__ bits) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && N > 0) atomicOr(bits, 1ull);  // word 0 always starts a chunk
  if (i >= n) return;
  const uint64_t p = off[i];
  if (p < N && off[i + 1] > p) atomicOr(bits + (p >> 6), 1ull << (p & 63));
}

// tile_first[t] = first index i in [0, npos] with pos[i] >= t*T (binary search).
__global__ void tile_first_kernel(const uint64_t* __restrict__ pos, uint64_t npos, uint64_t ntiles,
                                  uint64_t T, uint64_t* __restrict__ tile_first) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const uint64_t key = t * T;
  uint64_t lo = 0, hi = npos + 1;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (pos[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  tile_first[t] = lo;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
int pack_steps() {
  static int steps = [] {
    const char* e = getenv("CPK_PACK_STEPS");  // tuning knob: 8 or 16 (default)
    const int v = e ? atoi(e) : kPackSteps;
    return (v == 8 || v == 16 || v == 4) ? v : kPackSteps;
  }();
  return steps;
}

template <int S>
hipError_t launch_pack_s(const PackTileArgs& a, hipStream_t stream) {
  static const unsigned cap = resident_blocks((const void*)pack_tiles_kernel<S, false>, 256, 0);
  const uint64_t want = (a.ntiles + 3) / 4;
  const unsigned blocks = (unsigned)(want < cap ? want : cap);
  if (a.stamps)
    hipLaunchKernelGGL((pack_tiles_kernel<S, true>), dim3(blocks), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL((pack_tiles_kernel<S, false>), dim3(blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_pack_tiles(const PackTileArgs& a, hipStream_t stream) {
  if (a.ntiles == 0) return hipSuccess;
  switch (pack_steps()) {
    case 4: return launch_pack_s<4>(a, stream);
    case 8: return launch_pack_s<8>(a, stream);
    default: return launch_pack_s<16>(a, stream);
  }
}

hipError_t launch_message_bits(const uint64_t* words, const uint64_t* off, uint64_t n,
                               uint64_t* bits, int32_t* status, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(message_bits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     words, off, n, (unsigned long long*)bits, status);
  return hipGetLastError();
}

hipError_t launch_chunk_bits(const uint64_t* off, uint64_t n, uint64_t N, uint64_t* bits,
                             hipStream_t stream) {
  if (n == 0 && N == 0) return hipSuccess;
  hipLaunchKernelGGL(chunk_bits_kernel, dim3((unsigned)((n + 256) / 256)), dim3(256), 0, stream,
                     off, n, N, (unsigned long long*)bits);
  return hipGetLastError();
}

hipError_t launch_tile_first(const uint64_t* pos, uint64_t npos, uint64_t ntiles, uint64_t T,
                             uint64_t* tile_first, hipStream_t stream) {
  if (ntiles == 0) return hipSuccess;
  hipLaunchKernelGGL(tile_first_kernel, dim3((unsigned)((ntiles + 255) / 256)), dim3(256), 0,
                     stream, pos, npos, ntiles, T, tile_first);
  return hipGetLastError();
}

}  // namespace cpk
