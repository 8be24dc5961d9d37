// cpk_device.h -- wave-level building blocks shared by the pack and unpack kernels (gfx950).
//
// Everything here is written for 64-lane CDNA4 wavefronts: 64-bit ballots, mbcnt prefix counts,
// readlane broadcasts.  Cross-workgroup hand-offs (tile descriptors of the single-pass
// decoupled look-back) follow the "data is the flag" form: one naturally aligned 8-byte word
// written by one agent-scope atomic store and polled by agent-scope atomic loads, so no
// release/acquire fences are needed (MI355X_MICROARCH.md, Valid forms, R2 granule).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cpk_kernels.h"

namespace cpk {

constexpr int kWave = 64;

// Descriptor flags in the top two bits of a 64-bit look-back word.
constexpr uint64_t kDescAgg = 1ull << 62;
constexpr uint64_t kDescIncl = 2ull << 62;
constexpr uint64_t kDescValue = (1ull << 62) - 1;
constexpr uint64_t kDescFlags = 3ull << 62;

// Bound on any spin (iterations of ~100 ns with s_sleep): a protocol bug ends the kernel with an
// error flag instead of hanging the GPU.
constexpr uint32_t kSpinLimit = 1u << 22;

// Error word codes (ctx-level, first writer wins) == include/cpk.h cpk_status.
constexpr uint32_t kErrCapacity = 8;
constexpr uint32_t kErrInternal = 12;

__device__ __forceinline__ int lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ uint32_t readlane32(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  uint32_t lo = readlane32((uint32_t)v, l), hi = readlane32((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t uniform32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  return ((uint64_t)uniform32((uint32_t)(v >> 32)) << 32) | uniform32((uint32_t)v);
}

// Lane shuffle (ds_bpermute); `src` may differ per lane.
__device__ __forceinline__ uint32_t shfl32(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  return ((uint64_t)shfl32((uint32_t)(v >> 32), src) << 32) | shfl32((uint32_t)v, src);
}

// Inclusive wave scans by DPP: row_shr 1/2/4/8 inside each 16-lane row, then row_bcast:15 and
// row_bcast:31 carry row totals upward.  Lanes whose DPP source does not exist read 0 (the
// identity of every scan below: sums and unsigned max).
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_src(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, true);
}
// Lane l receives lane l - 1's v (DPP wave_shr:1, GFX9); lane 0 receives `fill`.
__device__ __forceinline__ uint32_t wave_shr1_32(uint32_t v, uint32_t fill = 0) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x138, 0xf, 0xf, false);
}
template <class Op>
__device__ __forceinline__ uint32_t wave_scan32(uint32_t v, Op op) {
  v = op(v, dpp_src<0x111, 0xf>(v));
  v = op(v, dpp_src<0x112, 0xf>(v));
  v = op(v, dpp_src<0x114, 0xf>(v));
  v = op(v, dpp_src<0x118, 0xf>(v));
  v = op(v, dpp_src<0x142, 0xa>(v));
  v = op(v, dpp_src<0x143, 0xc>(v));
  return v;
}
__device__ __forceinline__ uint32_t wave_incl_sum32(uint32_t v) {
  return wave_scan32(v, [](uint32_t a, uint32_t b) { return a + b; });
}
__device__ __forceinline__ uint32_t wave_incl_max32(uint32_t v) {
  return wave_scan32(v, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
}
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp_src64(uint64_t v) {
  return ((uint64_t)dpp_src<CTRL, ROWS>((uint32_t)(v >> 32)) << 32) |
         dpp_src<CTRL, ROWS>((uint32_t)v);
}
__device__ __forceinline__ uint64_t wave_incl_sum64(uint64_t v) {
  v += dpp_src64<0x111, 0xf>(v);
  v += dpp_src64<0x112, 0xf>(v);
  v += dpp_src64<0x114, 0xf>(v);
  v += dpp_src64<0x118, 0xf>(v);
  v += dpp_src64<0x142, 0xa>(v);
  v += dpp_src64<0x143, 0xc>(v);
  return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
  return readlane64(wave_incl_sum64(v), 63);
}

// Cross-lane hand-off through LDS inside one wave: the wave's LDS instructions execute in
// order, so only the compiler has to be kept from moving memory accesses across this point
// (it reasons per lane and may otherwise reorder a lane's access past another lane's).
__device__ __forceinline__ void lane_handoff() { asm volatile("" ::: "memory"); }

// Marks word p as a chunk start (and, at a pack tile start, the tile's byte: plain byte stores,
// no atomics -- a word shared by 64 tiles, OR-ed and AND-ed by atomics, cost the tile kernel
// half its speed in contention).
__device__ __forceinline__ void mark_chunk(unsigned long long* bits, uint8_t* tstarts,
                                           uint64_t p) {
  atomicOr(bits + (p >> 6), 1ull << (p & 63));
  if (p % kPackTileWords == 0 && p) tstarts[p / kPackTileWords] = 1;  // (tile 0: no predecessor)
}

// Chunk starts of message i = words[off[i], off[i+1]) -- segment table (serializeSegmentTable
// serialize.c++:311-330) then segments; chunk starts = message start, table end, each segment
// start -- and its framing status (cpk_frame.hip's message_bits_kernel; the pack tile kernel
// calls it itself for a single-tile batch).
__device__ __forceinline__ void frame_message(const uint64_t* __restrict__ words,
                                              const uint64_t* __restrict__ off, uint64_t i,
                                              uint64_t N, unsigned long long* __restrict__ bits,
                                              uint8_t* __restrict__ tstarts,
                                              int32_t* __restrict__ status) {
  const uint64_t w0 = off[i], w1 = off[i + 1];
  int32_t st = 0;
  if (w1 <= w0) {
    if (status) status[i] = 11;  // CPK_ERR_EMPTY_MESSAGE
    return;
  }
  if (w1 > N) {
    // a message past the batch's words: no bit outside the words the tiles clear (the bitmap is
    // zero at rest), and nothing read past them
    if (status) status[i] = 6;  // CPK_ERR_BAD_FRAMING
    return;
  }
  const uint64_t nw = w1 - w0;
  const uint32_t* t32 = (const uint32_t*)(words + w0);
  // the table's first word in one load: the segment count and the first segment's size (a
  // one-segment message needs no further load)
  const uint64_t h0 = words[w0];
  const uint64_t nseg = (uint64_t)(uint32_t)h0 + 1;
  const uint64_t tw = nseg / 2 + 1;
  auto seg_size = [&](uint64_t s) -> uint64_t { return s == 0 ? (h0 >> 32) : t32[s + 1]; };
  bool ok = tw <= nw;
  if (ok) {
    uint64_t total = tw;
    for (uint64_t s = 0; s < nseg && total <= nw; s++) total += seg_size(s);
    ok = total == nw;
  }
  // the chunk starts gathered per bitmap word: one atomic per word touched (the message start and
  // its table end usually share one), not one per start
  uint64_t cw = w0 >> 6, cm = 1ull << (w0 & 63);
  auto mark = [&](uint64_t p) {
    if ((p >> 6) != cw) {
      atomicOr(bits + cw, (unsigned long long)cm);
      cw = p >> 6;
      cm = 0;
    }
    cm |= 1ull << (p & 63);
    if (p % kPackTileWords == 0) tstarts[p / kPackTileWords] = 1;
  };
  if (w0 % kPackTileWords == 0 && w0) tstarts[w0 / kPackTileWords] = 1;  // (tile 0: none)
  if (!ok) {
    st = 6;  // CPK_ERR_BAD_FRAMING: packed as one chunk
  } else {
    uint64_t p = w0 + tw;
    if (p < w1) mark(p);
    for (uint64_t s = 0; s + 1 < nseg; s++) {
      p += seg_size(s);
      if (p < w1) mark(p);
    }
  }
  atomicOr(bits + cw, (unsigned long long)cm);
  if (status) status[i] = st;
}

// Workgroup ticket: a launch's tiles in the order their workgroups START (thread 0 takes the next
// ticket from a zeroed counter; the workgroup reads it back from LDS).  A tile that waits only on
// lower tickets then waits only on workgroups that are running or done, whatever else the device
// runs.  The tickets of one launch serialize on one counter (~13 ns each on MI355X: C4's pack
// with a ticket per tile took 20.2 ms instead of 7.6), so only the small resolve launch of the
// split decode uses them; the tile kernels keep blockIdx order, whose forward progress rests on
// the per-XCD in-order dispatch and on the codec never running two of its waiting launches at
// once (cpk_api.cpp DeviceOrder).
__device__ __forceinline__ uint32_t wg_ticket(unsigned int* counter, unsigned int* s_slot) {
  if (threadIdx.x == 0) *s_slot = atomicAdd(counter, 1u);
  __syncthreads();
  return uniform32(*(volatile unsigned int*)s_slot);
}

// Workgroup b's tile-order index when consecutive tiles should share an XCD: workgroups are
// dealt to the 8 XCDs round robin (b % 8 -- for speed only, nothing relies on it), so the j-th
// workgroup of XCD x takes index (j / C) * 8C + x * C + j % C -- chunks of C consecutive indices
// per XCD, a round of 8C over all of them.  (Deadlock-free as the plain order is: a tile waits
// only on lower indices, all within its own round or before it, and a round of 8C workgroups is
// far below the resident ones.)
template <uint64_t C>
__device__ __forceinline__ uint64_t xcd_order(uint64_t b, uint64_t G) {
  constexpr uint64_t R = 8 * C;
  const uint64_t full = (G / R) * R;
  if (b >= full) return b;
  const uint64_t x = b & 7, j = b >> 3;
  return (j / C) * R + x * C + (j % C);
}

// Workgroup barrier ordering LDS only: __syncthreads also releases global memory at workgroup
// scope, which waits for every outstanding vector memory operation -- stores, and loads issued
// ahead for later use.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// A zero the compiler cannot see through: added to a uniform index, it keeps a load in a VGPR
// (a uniform load is otherwise moved to SGPRs with v_readfirstlane right behind it, i.e. waited
// for at once).
__device__ __forceinline__ uint32_t opaque_zero() {
  uint32_t z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}

// Bit masks.
__device__ __forceinline__ uint64_t mask_le(int l) { return (2ull << l) - 1; }   // bits 0..l
__device__ __forceinline__ uint64_t mask_lt(int l) { return (1ull << l) - 1; }   // bits 0..l-1
__device__ __forceinline__ int highest_bit(uint64_t m) { return m ? 63 - __clzll(m) : -1; }
__device__ __forceinline__ int lowest_bit(uint64_t m) { return m ? __ffsll((long long)m) - 1 : 64; }

// Agent-scope relaxed atomics on global memory (sc1 loads/stores; no fences needed because
// every handed-off value is self-contained in the polled word).
__device__ __forceinline__ uint64_t load_agent(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t load_agent32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_agent32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void raise_error(uint32_t* err, uint32_t code) {
  atomicCAS(err, 0u, code);
}

// One lane spins on a 32-bit word until it is non-zero (bounded).  Returns the value, or 0 on
// timeout (after raising kErrInternal).
__device__ __forceinline__ uint32_t wait_nonzero32(const uint32_t* p, uint32_t* err) {
  uint32_t v = 0;
  if (lane_id() == 0) {
    for (uint32_t i = 0; i < kSpinLimit; i++) {
      v = load_agent32(p);
      if (v) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (!v) raise_error(err, kErrInternal);
  }
  return uniform32(v);
}

// Blocks past `first_block` of a prologue kernel compute tile_first (TileFirstJob, cpk_kernels.h):
// tile t's first position index m with pos[m] >= t*T.  With about as many positions as tiles,
// one thread per position index m scatters m to the tiles whose start lies in (pos[m-1], pos[m]]
// (the intervals partition the tiles; the last index also takes the tiles past the last
// position) -- no per-tile binary search, whose 10-20 dependent loads per tile would set the
// time of the launch.  With many tiles per position (large messages: a serial scatter of
// thousands of tiles per thread) one thread per tile searches the few positions instead.
// Further blocks zero tf.zero.  True when this block did either job.
constexpr uint64_t kZeroBlockWords = 4096;  // u64 per zeroing block (256 threads x 16)
__host__ __device__ inline bool tile_first_search(const TileFirstJob& tf) {
  return tf.ntiles > 16 * (tf.npos + 1);
}
__host__ __device__ inline uint64_t tile_first_threads(const TileFirstJob& tf) {
  return !tf.ntiles ? 0 : (tile_first_search(tf) ? tf.ntiles : tf.npos + 1);
}
__device__ __forceinline__ bool run_tile_first(const TileFirstJob& tf, uint32_t first_block,
                                               uint32_t bid) {
  if (bid < first_block) return false;
  const uint32_t tfb = (uint32_t)((tile_first_threads(tf) + 255) / 256);
  if (bid - first_block >= tfb) {
    const uint64_t z0 = (uint64_t)(bid - first_block - tfb) * kZeroBlockWords;
    for (uint64_t i = z0 + threadIdx.x; i < z0 + kZeroBlockWords && i < tf.zero_words; i += 256)
      tf.zero[i] = 0;
    return true;
  }
  if (tile_first_search(tf)) {
    const uint64_t t = (uint64_t)(bid - first_block) * blockDim.x + threadIdx.x;
    if (t >= tf.ntiles) return true;
    // first m in [0, npos] with pos[m] >= t*T (npos + 1: none)
    const uint64_t x = t * tf.T;
    uint64_t lo = 0, n = tf.npos + 1;
    while (n > 0) {
      const uint64_t h = n >> 1;
      if (tf.pos[lo + h] < x) {
        lo += h + 1;
        n -= h + 1;
      } else {
        n = h;
      }
    }
    tf.out[t] = lo;
    if (tf.outpos) tf.outpos[t] = lo <= tf.npos ? tf.pos[lo] : ~0ull;
    return true;
  }
  const uint64_t m = (uint64_t)(bid - first_block) * blockDim.x + threadIdx.x;
  if (m > tf.npos) return true;
  const uint64_t pm = tf.pos[m];
  const uint64_t lo = m == 0 ? 0 : tf.pos[m - 1] / tf.T + 1;  // first tile starting past pos[m-1]
  uint64_t hi = pm / tf.T;                                     // last tile starting at or before pos[m]
  if (hi >= tf.ntiles) hi = tf.ntiles - 1;
  for (uint64_t t = lo; t <= hi && lo <= hi; t++) {
    tf.out[t] = m;
    if (tf.outpos) tf.outpos[t] = pm;
  }
  if (m == tf.npos) {
    // tiles starting past the last position: none of them has a first position
    for (uint64_t t = (pm / tf.T) + 1; t < tf.ntiles; t++) {
      tf.out[t] = tf.npos + 1;
      if (tf.outpos) tf.outpos[t] = ~0ull;
    }
  }
  return true;
}
__device__ __forceinline__ bool run_tile_first(const TileFirstJob& tf, uint32_t first_block) {
  return run_tile_first(tf, first_block, blockIdx.x);
}
inline unsigned tile_first_blocks(const TileFirstJob& tf) {
  return (unsigned)((tile_first_threads(tf) + 255) / 256 +
                    (tf.zero ? (tf.zero_words + kZeroBlockWords - 1) / kZeroBlockWords : 0));
}

// Decoupled look-back (exclusive prefix of tile aggregates) for tile `t` by one wave.
// desc[i] = flags | value; AGG = this tile's own aggregate, INCL = inclusive prefix.
// Segmented variant: when `seg_bit` is non-zero, a descriptor value carrying that bit marks a
// tile whose aggregate restarts the scan (a message start inside it); the look-back stops there
// and the bit is stripped from the sum.
//
// Window: each round reads 64*K predecessors (K per lane, all loads in flight).  The inclusive
// prefix front can only advance one window per round-trip latency, so with thousands of small
// tiles in flight the window width -- not the polling -- bounds throughput (64 tiles per ~1 us
// round on MI355X is far too slow; 512 is not).  While the nearest not-ready predecessor blocks
// progress only a single lane polls it (with s_sleep), so waiting waves do not flood L2.
template <int K = 8>
__device__ __forceinline__ uint64_t lookback(const uint64_t* desc, uint64_t t, uint32_t* err,
                                             uint64_t seg_bit = 0) {
  const int l = lane_id();
  uint64_t excl = 0;
  int64_t j = (int64_t)t - 1;  // nearest predecessor not yet summed
  uint32_t spins = 0;
  while (j >= 0) {
    uint64_t d[K];
#pragma unroll
    for (int i = 0; i < K; i++) {
      const int64_t idx = j - (64 * i + l);
      d[i] = idx >= 0 ? load_agent(desc + idx) : kDescIncl;  // before tile 0: inclusive zero
    }
    // nearest stop (inclusive, or segment restart) in distance order 64*i + lane
    int stop_at = 64 * K;  // distance of the nearest stop (64*K: none in this window)
    int blocked = 64 * K;  // distance of the nearest not-ready descriptor
#pragma unroll
    for (int i = K - 1; i >= 0; i--) {
      const uint64_t f = d[i] & kDescFlags;
      const bool ready = f != 0;
      const bool stop = f == kDescIncl || (seg_bit && ready && (d[i] & seg_bit));
      const uint64_t sb = ballot(stop), nb = ballot(!ready);
      if (sb) stop_at = 64 * i + lowest_bit(sb);
      if (nb) blocked = 64 * i + lowest_bit(nb);
    }
    if (blocked < stop_at) {
      // wait for the nearest blocking predecessor with one lane, then re-read the window
      if (l == 0) {
        const uint64_t* p = desc + (j - blocked);
        while ((load_agent(p) & kDescFlags) == 0 && spins < kSpinLimit) {
          __builtin_amdgcn_s_sleep(1);
          spins++;
        }
      }
      spins = uniform32(spins);
      if (spins >= kSpinLimit) {
        raise_error(err, kErrInternal);
        return excl;
      }
      continue;
    }
    uint64_t contrib = 0;
#pragma unroll
    for (int i = 0; i < K; i++)
      if (64 * i + l <= stop_at) contrib += (d[i] & kDescValue) & ~seg_bit;
    excl += wave_sum64(contrib);
    if (stop_at < 64 * K) break;
    j -= 64 * K;
  }
  return excl;
}

}  // namespace cpk
