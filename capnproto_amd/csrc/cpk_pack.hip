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
//     the stretch (:376-426); R words that are not covered are ordinary heads.  Within any 64-word
//     step each stretch therefore has at most one run head, which lets a wave resolve a step with
//     64-bit ballot masks, carrying one byte of state (the run's remaining budget) between steps.
//   * Output bytes per word: Z head 2, Z covered 0, F head 10, covered R 8, other heads 1 + nz.
//
// Work decomposition: the batch of words is cut into fixed tiles of 64*S words; one wave owns a
// tile (tile ids come from an atomic counter, so every predecessor of a running tile is already
// resident).  A tile resolves itself locally except for the stretch that enters it from its
// predecessor: that needs the predecessor's exit budget (published as early as possible), and
// the byte offset of the tile comes from a single-pass decoupled look-back over tile byte
// counts.  Output bytes are staged in a per-wave LDS ring placed at (address mod 1024) and leave
// as aligned 16-byte stores; only the <= 15-byte partial blocks at tile edges use byte stores.
#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {

namespace {

constexpr int kRing = 1024;  // per-wave LDS output ring (bytes); one step emits <= 640
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct StepMasks {
  uint64_t Z, F, R, SY;  // SY: stretch starts (sync points), incl. invalid lanes
};

// Per-lane resolution of one 64-word step.  `b` = budget entering the step (words the run that
// is open at the previous word may still cover), meaningful when the step's word 0 continues the
// previous stretch.  Returns head/covered for this lane and the budget leaving the step.
struct LaneRes {
  bool head, covered;
};

__device__ __forceinline__ LaneRes resolve_lane(const StepMasks& m, int l, int b, bool valid) {
  const uint64_t bit = 1ull << l;
  const uint64_t syl = m.SY & mask_le(l);
  const int st = highest_bit(syl);
  const int es = st >= 0 ? st : b;  // effective start of this lane's stretch in the step
  LaneRes r{false, false};
  if (!valid) return r;
  if (m.Z & bit) {
    r.head = (l == es);
    r.covered = !r.head;
  } else if (m.R & bit) {
    if (l < es) {
      r.covered = true;
    } else {
      const uint64_t range = mask_lt(l) & ~mask_lt(es);
      r.covered = (m.F & range) != 0;
      r.head = !r.covered;
    }
  } else {
    r.head = true;
  }
  return r;
}

// Budget leaving a step, from the ballot of run heads (Z heads and F heads).
__device__ __forceinline__ int exit_budget(const StepMasks& m, uint64_t runheads, int b,
                                           bool last_is_run_family) {
  if (!last_is_run_family) return 0;
  const int st63 = highest_bit(m.SY);
  const int h = highest_bit(runheads);
  if (h >= 0 && h >= st63) return 255 - (63 - h);
  if (st63 < 0 && b > 63) return b - 64;
  return 0;
}

struct Klass {
  uint64_t Z, F, R, O, V;
};

__device__ __forceinline__ Klass classify(uint64_t x, bool valid) {
  const uint32_t tag = word_tag(x);
  const int nz = __popc(tag);
  Klass k;
  k.Z = ballot(valid && x == 0);
  k.F = ballot(valid && tag == 0xff);
  k.R = ballot(valid && nz >= 7);
  k.O = ballot(valid && x != 0 && nz < 7);
  k.V = ballot(valid);
  return k;
}

// Sync mask of a step given its class masks, chunk-start bits and the carried class of the word
// before the step (zc/rc: previous word was Z / R and valid).
__device__ __forceinline__ uint64_t sync_mask(const Klass& k, uint64_t C, uint64_t zc,
                                              uint64_t rc) {
  const uint64_t prevZ = (k.Z << 1) | zc;
  const uint64_t prevR = (k.R << 1) | rc;
  return C | k.O | (k.Z & ~prevZ) | (k.R & ~prevR) | ~k.V;
}

template <int S>
__global__ __launch_bounds__(256) void pack_tiles_kernel(PackTileArgs a) {
  static_assert(S >= 1 && S <= 64, "S steps per tile");
  constexpr int T = 64 * S;
  __shared__ uint64_t lds_words[4][T];
  __shared__ __attribute__((aligned(16))) uint8_t lds_ring[4][kRing];

  const int l = lane_id();
  const int wv = threadIdx.x >> 6;
  uint64_t* xw = lds_words[wv];
  uint8_t* ring = lds_ring[wv];

  uint32_t t32 = 0;
  if (l == 0) t32 = atomicAdd(a.tile_counter, 1u);
  const uint64_t t = uniform32(t32);
  if (t >= a.ntiles) return;

  const uint64_t N = a.nwords;
  const uint64_t tbase = t * T;
  const uint64_t tend = tbase + T < N ? tbase + T : N;

  // ---- load the tile (coalesced, all loads in flight), then stage into LDS -------------------
  {
    uint64_t v[S];
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t g = tbase + 64 * s + l;
      v[s] = g < N ? a.words[g] : 0;
    }
#pragma unroll
    for (int s = 0; s < S; s++) xw[64 * s + l] = v[s];
  }
  const uint64_t nbitw = (N + 63) >> 6;
  const uint64_t cbw = (l < S && (tbase >> 6) + l < nbitw) ? a.chunk_bits[(tbase >> 6) + l] : 0;

  // Class of the word before the tile (same-chunk test is the chunk bit of word 0).
  uint64_t zc = 0, rc = 0;
  if (tbase > 0) {
    const uint64_t pw = a.words[tbase - 1];
    zc = pw == 0;
    rc = __popc(word_tag(pw)) >= 7;
  }

  // ---- pass 1: per-step class masks; lane s keeps step s's masks -----------------------------
  uint64_t myZ = 0, myF = 0, myR = 0, mySY = 0;
  bool any_sync_valid = false;
  int first_sync = T;  // first sync position among valid words
  {
    uint64_t czc = zc, crc = rc;
    for (int s = 0; s < S; s++) {
      const uint64_t g = tbase + 64 * s + l;
      const bool valid = g < N;
      const uint64_t x = xw[64 * s + l];
      const Klass k = classify(x, valid);
      const uint64_t C = readlane64(cbw, s);
      const uint64_t SY = sync_mask(k, C, czc, crc);
      czc = k.Z >> 63;
      crc = k.R >> 63;
      const uint64_t syv = SY & k.V;
      if (syv && !any_sync_valid) {
        any_sync_valid = true;
        first_sync = 64 * s + lowest_bit(syv);
      }
      if (l == s) {
        myZ = k.Z;
        myF = k.F;
        myR = k.R;
        mySY = SY;
      }
    }
  }
  const int nvalid = (int)(tend - tbase);
  const int last = nvalid - 1;  // tile position of the last valid word
  const bool last_Z = (readlane64(myZ, last >> 6) >> (last & 63)) & 1;
  const bool last_R = (readlane64(myR, last >> 6) >> (last & 63)) & 1;

  // ---- look-ahead: first sync position after the tile (for run counts near the end) ----------
  // la = distance from tend to the first word that ends the trailing stretch (<= 256).
  int la = 0;
  if ((last_Z || last_R) && tend < N) {
    uint64_t czc = last_Z, crc = last_R;
    la = 256;
    for (int k = 0; k < 4; k++) {
      const uint64_t g = tend + 64 * k + l;
      const bool valid = g < N;
      const uint64_t x = valid ? a.words[g] : 0;
      const Klass kk = classify(x, valid);
      const uint64_t C = ((tend >> 6) + k < nbitw) ? a.chunk_bits[(tend >> 6) + k] : 0;
      const uint64_t SY = sync_mask(kk, C, czc, crc);
      czc = kk.Z >> 63;
      crc = kk.R >> 63;
      if (SY) {
        la = 64 * k + lowest_bit(SY);
        break;
      }
    }
  }

  // first sync bit per step (lane s), used for run counts
  const int myFs = lowest_bit(mySY);

  // Distance from the start of step s+1 to the first sync at or after it (capped at 256).
  auto next_sync_after = [&](int s) -> int {
    int d = 0;
    for (int k = s + 1; k < S && d < 256; k++) {
      const int fs = (int)readlane32((uint32_t)myFs, k);
      if (fs < 64) return d + fs;
      d += 64;
    }
    if (s + 1 >= S) return la;
    return d < 256 ? d + la : 256;
  };

  auto masks_of = [&](int s) -> StepMasks {
    StepMasks m;
    m.Z = readlane64(myZ, s);
    m.F = readlane64(myF, s);
    m.R = readlane64(myR, s);
    m.SY = readlane64(mySY, s);
    return m;
  };

  // Byte count of steps [s0, s1) with entry budget b at step s0; lanes with tile position < lo
  // or >= hi are not counted.  Returns the budget leaving step s1-1 in *bout.
  auto count_steps = [&](int s0, int s1, int b, int lo, int hi, int* bout) -> uint64_t {
    uint64_t bytes = 0;
    for (int s = s0; s < s1; s++) {
      const StepMasks m = masks_of(s);
      const int pos = 64 * s + l;
      const bool valid = pos < nvalid;
      const LaneRes r = resolve_lane(m, l, b, valid);
      const uint64_t bit = 1ull << l;
      const uint32_t tag = word_tag(xw[pos]);
      uint32_t len = 0;
      if (r.covered) len = (m.R & bit) ? 8 : 0;
      else if (r.head) len = (m.Z & bit) ? 2 : ((m.F & bit) ? 10 : 1 + __popc(tag));
      if (pos < lo || pos >= hi) len = 0;
      uint32_t tot;
      wave_excl_sum_small(len, &tot);
      bytes += tot;
      const uint64_t runheads = ballot(r.head && ((m.Z | m.F) & bit));
      const int l63 = 64 * s + 63;
      const bool fam = l63 < nvalid && (((m.Z | m.R) >> 63) & 1);
      b = exit_budget(m, runheads, b, fam);
    }
    *bout = b;
    return bytes;
  };

  // ---- exit state (published early when independent of the entry) ---------------------------
  uint32_t* const state = a.state;
  uint64_t bytes_suffix = 0;
  int exit_b = 0;
  if (any_sync_valid) {
    const int s0 = first_sync >> 6;
    bytes_suffix = count_steps(s0, S, 0, first_sync, T, &exit_b);
    if (l == 0) store_agent32(state + t, 0x80000000u | (uint32_t)exit_b);
  }

  // ---- entry budget -------------------------------------------------------------------------
  int b_entry = 0;
  if (first_sync > 0 && t > 0) {
    b_entry = (int)(wait_nonzero32(state + t - 1, a.err) & 0xffu);
  }
  uint64_t bytes_lead = 0;
  if (first_sync > 0) {
    const int s1 = any_sync_valid ? (first_sync >> 6) + 1 : S;
    int bo;
    bytes_lead = count_steps(0, s1, b_entry, 0, first_sync, &bo);
    if (!any_sync_valid) {
      exit_b = bo;
      if (l == 0) store_agent32(state + t, 0x80000000u | (uint32_t)exit_b);
    }
  }
  const uint64_t agg = bytes_lead + bytes_suffix;

  // ---- decoupled look-back for the tile's output offset -------------------------------------
  uint64_t excl = 0;
  if (t == 0) {
    if (l == 0) store_agent(a.desc, kDescIncl | agg);
  } else {
    if (l == 0) store_agent(a.desc + t, kDescAgg | agg);
    excl = lookback(a.desc, t, a.err);
    if (l == 0) store_agent(a.desc + t, kDescIncl | (excl + agg));
  }

  // ---- emission -----------------------------------------------------------------------------
  const uint64_t base_addr = (uint64_t)(uintptr_t)a.out;
  const uint64_t A0 = base_addr + excl;
  const uint64_t A1 = A0 + agg;
  const uint64_t al = (A0 + 15) & ~15ull;
  const bool over = excl + agg > a.out_capacity;
  if (over && l == 0) raise_error(a.err, kErrCapacity);
  uint64_t flushed = al;  // next 16-aligned block to store
  uint64_t hd = A0;       // next head (partial-block) byte to store
  uint64_t A = A0;        // address of the next emitted byte

  // positions whose output offset is requested (message / chunk starts)
  uint64_t pidx = a.pos ? uniform64(a.tile_first[t]) : 0;
  uint64_t pnext = (a.pos && pidx <= a.npos) ? uniform64(a.pos[pidx]) : ~0ull;

  int b = b_entry;
  for (int s = 0; s < S; s++) {
    if (64 * s >= nvalid) break;
    const StepMasks m = masks_of(s);
    const int pos = 64 * s + l;
    const bool valid = pos < nvalid;
    const uint64_t bit = 1ull << l;
    const uint64_t x = xw[pos];
    const uint32_t tag = word_tag(x);
    const LaneRes r = resolve_lane(m, l, b, valid);
    const bool isZ = m.Z & bit, isF = m.F & bit, isR = m.R & bit;
    uint32_t len = 0;
    uint64_t lo = 0;
    uint32_t hi = 0;
    // run count for Z / F heads: min(255, words left in the stretch after this one)
    const int nsa = next_sync_after(s);
    uint32_t cnt = 0;
    if (r.head && (isZ || isF)) {
      const uint64_t gt = m.SY & ~mask_le(l);
      const int ns = gt ? lowest_bit(gt) : 64 + nsa;
      const int c = ns - l - 1;
      cnt = (uint32_t)(c < 255 ? c : 255);
    }
    if (r.covered) {
      if (isR) {
        len = 8;
        lo = x;
      }
    } else if (r.head) {
      if (isZ) {
        len = 2;
        lo = (uint64_t)cnt << 8;
      } else if (isF) {
        len = 10;
        lo = 0xffull | (x << 8);
        hi = (uint32_t)(x >> 56) | (cnt << 8);
      } else {
        len = 1 + __popc(tag);
        lo = (uint64_t)tag | (compact_nonzero(x) << 8);
      }
    }
    uint32_t step_total;
    const uint32_t o = wave_excl_sum_small(len, &step_total);
    if (!over) {
#pragma unroll
      for (int k = 0; k < 10; k++) {
        if ((uint32_t)k < len) {
          const uint8_t byte = k < 8 ? (uint8_t)(lo >> (8 * k)) : (uint8_t)(hi >> (8 * (k - 8)));
          ring[(A + o + k) & (kRing - 1)] = byte;
        }
      }
    }
    // requested output offsets for positions inside this step
    const uint64_t g0 = tbase + 64 * s;
    while (pnext < g0 + 64) {
      const uint64_t i = pidx + l;
      const uint64_t p = i <= a.npos ? a.pos[i] : ~0ull;
      const bool in = p < g0 + 64;
      const uint32_t src = in ? (uint32_t)(p - g0) : 0;
      const uint32_t oo = shfl32(o, (int)src);
      if (in) a.pos_out[i] = (A - base_addr) + oo;
      const uint64_t inm = ballot(in);
      pidx += __popcll(inm);
      pnext = pidx <= a.npos ? uniform64(a.pos[pidx]) : ~0ull;
      if (inm != ~0ull) break;
    }
    b = exit_budget(m, ballot(r.head && ((m.Z | m.F) & bit)), b,
                    (64 * s + 63 < nvalid) && (((m.Z | m.R) >> 63) & 1));
    const uint64_t Aend = A + step_total;
    if (!over) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // partial head block (shared with the previous tile's bytes): byte stores
      const uint64_t hlim = Aend < al ? Aend : al;
      if (hd < hlim) {
        const uint64_t p = hd + l;
        if (l < 16 && p < hlim) *(uint8_t*)(uintptr_t)p = ring[p & (kRing - 1)];
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
            const u32x4 v = *(const u32x4*)(ring + (p & (kRing - 1)));
            *(u32x4*)(uintptr_t)p = v;
          }
        }
        flushed = top;
      }
    }
    A = Aend;
  }
  if (!over) {
    // partial tail block
    const uint64_t from = flushed > hd ? flushed : hd;
    if (from < A1) {
      const uint64_t p = from + l;
      if (l < 16 && p < A1) *(uint8_t*)(uintptr_t)p = ring[p & (kRing - 1)];
    }
  }
  // positions at or past the end of the batch -> total
  if (a.pos && tend == N) {
    const uint64_t total = excl + agg;
    for (uint64_t i = pidx + l; i <= a.npos; i += 64) a.pos_out[i] = total;
    if (l == 0 && a.total_out) *a.total_out = total;
  }
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
hipError_t launch_pack_tiles(const PackTileArgs& a, hipStream_t stream) {
  if (a.ntiles == 0) return hipSuccess;
  const uint64_t waves = a.ntiles;
  const uint64_t blocks = (waves + 3) / 4;
  hipLaunchKernelGGL(pack_tiles_kernel<kPackSteps>, dim3((unsigned)blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
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
