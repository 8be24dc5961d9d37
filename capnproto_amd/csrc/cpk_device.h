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

// Number of set bits of `m` at lanes below this lane.
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

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

// Exclusive prefix sum over the wave of small values (0 <= v < 16) via 4 ballots.
__device__ __forceinline__ uint32_t wave_excl_sum_small(uint32_t v, uint32_t* total) {
  uint64_t b0 = ballot(v & 1), b1 = ballot(v & 2), b2 = ballot(v & 4), b3 = ballot(v & 8);
  *total = (uint32_t)(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2) + 8 * __popcll(b3));
  return mbcnt64(b0) + 2 * mbcnt64(b1) + 4 * mbcnt64(b2) + 8 * mbcnt64(b3);
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

// Tag byte of a word: bit i set <=> byte i non-zero (serialize-packed.c++:332-350), by SWAR.
__device__ __forceinline__ uint32_t word_tag(uint64_t x) {
  const uint64_t lo7 = 0x7f7f7f7f7f7f7f7full;
  uint64_t m = (((x & lo7) + lo7) | x) & 0x8080808080808080ull;
  return (uint32_t)(((m >> 7) * 0x0102040810204080ull) >> 56);
}

// Non-zero bytes of x packed to the low end, in byte order.
__device__ __forceinline__ uint64_t compact_nonzero(uint64_t x) {
  uint64_t out = 0;
  uint32_t c = 0;
#pragma unroll
  for (int b = 0; b < 8; b++) {
    uint64_t v = (x >> (8 * b)) & 0xff;
    out |= v << (8 * c);
    c += v != 0;
  }
  return out;
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
  mark_chunk(bits, tstarts, w0);
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
    if (p < w1) mark_chunk(bits, tstarts, p);
    for (uint64_t s = 0; s + 1 < nseg; s++) {
      p += t32[s + 1];
      if (p < w1) mark_chunk(bits, tstarts, p);
    }
  }
  if (status) status[i] = st;
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
__device__ __forceinline__ bool run_tile_first(const TileFirstJob& tf, uint32_t first_block) {
  if (blockIdx.x < first_block) return false;
  const uint32_t tfb = (uint32_t)((tile_first_threads(tf) + 255) / 256);
  if (blockIdx.x - first_block >= tfb) {
    const uint64_t z0 = (uint64_t)(blockIdx.x - first_block - tfb) * kZeroBlockWords;
    for (uint64_t i = z0 + threadIdx.x; i < z0 + kZeroBlockWords && i < tf.zero_words; i += 256)
      tf.zero[i] = 0;
    return true;
  }
  if (tile_first_search(tf)) {
    const uint64_t t = (uint64_t)(blockIdx.x - first_block) * blockDim.x + threadIdx.x;
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
  const uint64_t m = (uint64_t)(blockIdx.x - first_block) * blockDim.x + threadIdx.x;
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

__device__ __forceinline__ uint64_t stamp_now() {
  // no s_waitcnt: a phase ends where the wave gets to, memory still in flight (forcing the wait
  // at every mark serialised the loads the phases are meant to overlap)
  asm volatile("" ::: "memory");
  const uint64_t t = __builtin_amdgcn_s_memtime();
  asm volatile("" ::: "memory");
  return t;
}

// ---------------------------------------------------------------------------------------------
// Two-level decoupled look-back.
//
// Tiles are grouped 64 to a group.  Every tile publishes its aggregate (AGG) in desc[t]; the
// group's last tile combines the group's 64 aggregates in order and publishes the group
// aggregate in gdesc[g] (an arrival ticket instead -- whichever tile counts last -- measured
// slower: the winner's extra round trip made the group aggregates later), and publishes the
// group's inclusive prefix there once it knows its own.  A tile then needs one
// hop over the tiles before it in its group and, unless an inclusive prefix is found there, one
// hop over up to 64 group descriptors (4096 tiles): with thousands of tiles in flight the
// inclusive front no longer has to crawl one window per fabric round trip.
//
// Combination (segmented when seg_bit != 0): a value carrying seg_bit restarts the sum (its
// aggregate counts only from a message start inside the tile / group).
constexpr int kGroup = 64;

__device__ __forceinline__ uint64_t seg_combine(uint64_t before, uint64_t after, uint64_t seg_bit) {
  // value of (before ++ after)
  if (seg_bit && (after & seg_bit)) return after;
  return (before & seg_bit) | ((before & ~seg_bit) + (after & ~seg_bit));
}

// Each lane loads its descriptor and polls it (only lanes whose entry is not ready) until
// ready, sleeping between polls.
__device__ __forceinline__ uint64_t load_ready(const uint64_t* p, bool use, uint32_t* err) {
  if (!use) return kDescIncl;
  uint64_t d = load_agent(p);
  uint32_t spins = 0;
  while ((d & kDescFlags) == 0) {
    if (++spins >= kSpinLimit) {
      raise_error(err, kErrInternal);
      return kDescIncl;
    }
    __builtin_amdgcn_s_sleep(2);
    d = load_agent(p);
  }
  return d;
}

// Sum (segmented) of lanes 0..k of v, in lane order = distance order (lane 0 nearest): i.e.
// value of entries (k, ..., 1, 0) concatenated oldest first.
__device__ __forceinline__ uint64_t reduce_nearest(uint64_t v, int k, uint64_t seg_bit) {
  const int l = lane_id();
  // the nearest stop with seg bit among lanes <= k: everything farther is dropped
  const uint64_t segs = seg_bit ? ballot(l <= k && (v & seg_bit)) : 0;
  const int s = segs ? lowest_bit(segs) : k;  // farthest lane that contributes
  const uint64_t contrib = (l <= s) ? (v & ~seg_bit) : 0;
  const uint64_t sum = wave_sum64(contrib);
  return (segs ? seg_bit : 0) | sum;
}

// Publishes tile t's aggregate; the group's last tile also combines the group's aggregates (it
// waits for its in-group predecessors, all running in the same round of the persistent order)
// and publishes the group aggregate.  gdesc[g] has that single writer (AGG here, then INCL in
// publish_incl), so no ticket atomics or CAS are needed.
__device__ __forceinline__ void publish_agg(uint64_t* desc, uint64_t* gdesc, uint32_t* gcnt,
                                            uint64_t t, uint64_t ntiles, uint64_t agg,
                                            uint64_t seg_bit, uint32_t* err) {
  (void)gcnt;
  const int l = lane_id();
  if (l == 0) store_agent(desc + t, kDescAgg | agg);
  const uint64_t g = t / kGroup;
  const uint64_t g0 = g * kGroup;
  const bool last_of_group = (t + 1) % kGroup == 0 || t + 1 == ntiles;
  if (!last_of_group) return;
  const uint32_t n_in = (uint32_t)(t - g0 + 1);
  // lane i = tile t - i (lane 0: this tile's own aggregate)
  const bool use = l > 0 && (uint32_t)l < n_in;
  const uint64_t d = l == 0 ? (kDescAgg | agg) : load_ready(desc + (t - (uint64_t)(use ? l : 0)),
                                                            use, err);
  const bool stop = use && (d & kDescFlags) == kDescIncl;
  const uint64_t sb = ballot(stop);
  const int k = sb ? lowest_bit(sb) : (int)n_in - 1;
  const uint64_t v = reduce_nearest((l == 0 || use) ? (d & kDescValue) : 0, k, seg_bit);
  if (l == 0) {
    const uint64_t nv = sb ? (kDescIncl | (v & ~seg_bit)) : (kDescAgg | v);
    store_agent(gdesc + g, nv);
  }
}

// Exclusive prefix of tile t (after publish_agg).  Publishes nothing.
__device__ __forceinline__ uint64_t lookback2(const uint64_t* desc, const uint64_t* gdesc,
                                              uint64_t t, uint64_t seg_bit, uint32_t* err,
                                              uint64_t* dbg = nullptr) {
  // dbg (diagnostic builds only): [0] look-backs that went past the group, [1] group windows
  // read, [2] cycles in the in-group hop, [3] cycles in the group hops
  const uint64_t t0 = dbg ? stamp_now() : 0;
  const int l = lane_id();
  const uint64_t g = t / kGroup;
  const int j = (int)(t - g * kGroup);  // predecessors inside the group
  uint64_t excl = 0;                    // value of everything after the stop found so far
  {
    const bool use = l < j;
    const uint64_t d = load_ready(desc + (t - 1 - (uint64_t)(use ? l : 0)), use, err);
    const bool stop = use && (((d & kDescFlags) == kDescIncl) || (seg_bit && (d & seg_bit)));
    const uint64_t sb = ballot(stop);
    const int k = sb ? lowest_bit(sb) : j - 1;
    if (j > 0) excl = reduce_nearest(use ? (d & kDescValue) : 0, k, seg_bit);
    if (dbg) dbg[2] += stamp_now() - t0;
    if (sb || g == 0) return excl & ~seg_bit;
    if (excl & seg_bit) return excl & ~seg_bit;
  }
  const uint64_t t1 = dbg ? stamp_now() : 0;
  if (dbg) dbg[0]++;
  // group-level: groups g-1, g-2, ...
  int64_t G = (int64_t)g - 1;
  while (G >= 0) {
    if (dbg) dbg[1]++;
    const bool use = G - l >= 0;
    if (dbg) {  // diagnostic: group descriptors not yet published at the first read
      const uint64_t d0 = use ? load_agent(gdesc + (G - l)) : kDescIncl;
      dbg[1] += 1000 * (uint64_t)__popcll(ballot((d0 & kDescFlags) == 0));
    }
    const uint64_t d = load_ready(gdesc + (use ? G - l : 0), use, err);
    const bool stop = !use || ((d & kDescFlags) == kDescIncl) || (seg_bit && (d & seg_bit));
    const uint64_t sb = ballot(stop);
    const int k = sb ? lowest_bit(sb) : 63;
    const uint64_t v = reduce_nearest(use ? (d & kDescValue) : 0, k, seg_bit);
    excl = seg_combine(v, excl, seg_bit);
    if (sb) break;
    G -= 64;
  }
  if (dbg) dbg[3] += stamp_now() - t1;
  return excl & ~seg_bit;
}

// After lookback2: publish tile t's inclusive value (and the group's, from its last tile).
__device__ __forceinline__ void publish_incl(uint64_t* desc, uint64_t* gdesc, uint64_t t,
                                             uint64_t ntiles, uint64_t incl) {
  if (lane_id() != 0) return;
  store_agent(desc + t, kDescIncl | incl);
  const uint64_t g = t / kGroup;
  if ((t + 1) % kGroup == 0 || t + 1 == ntiles) store_agent(gdesc + g, kDescIncl | incl);
}

// Diagnostic phase stamps (env CPK_STAMPS=1 selects a separately instantiated kernel; the
// production kernels contain no stamp).  Lane 0 adds per-phase s_memtime deltas into its own
// debug buffer, never into outputs.
template <bool ON>
struct Stamps {
  // deltas accumulate in registers; flush() adds them to the debug buffer once (a global atomic
  // per mark would put its own round trip into every measured phase)
  unsigned long long* buf;
  uint64_t last;
  uint64_t acc[kStampSlots];
  __device__ __forceinline__ void start(unsigned long long* b) {
    if constexpr (ON) {
      buf = b;
      for (int i = 0; i < kStampSlots; i++) acc[i] = 0;
      last = stamp_now();
    }
  }
  __device__ __forceinline__ void restart() {
    if constexpr (ON) last = stamp_now();
  }
  __device__ __forceinline__ void mark(int slot) {
    if constexpr (ON) {
      const uint64_t now = stamp_now();
      acc[slot] += now - last;
      last = now;
    }
  }
  __device__ __forceinline__ void flush() {
    if constexpr (ON) {
      unsigned long long* row = buf + kStampSlots * (blockIdx.x & (kStampRows - 1));
      if (lane_id() == 0 && buf)
        for (int i = 0; i < kStampSlots; i++)
          if (acc[i]) atomicAdd(row + i, (unsigned long long)acc[i]);
    }
  }
};

// Blocks of `threads` threads the whole GPU keeps resident for kernel `fn`: the occupancy API per
// CU, capped by what the kernel's SGPR allocation allows (the API over-reports by one block per
// CU for SGPR-heavy kernels on ROCm 7.2: MI355X_MICROARCH.md, "Occupancy API one block/CU high";
// 800 SGPRs per SIMD, a wave holds ceil(sgprs/16)*16 + 16), minus `margin`, times the CU count.
// Persistent kernels size their grid with it so that every wave of the grid runs concurrently
// (a tile only ever waits on lower tiles).
inline unsigned resident_blocks(const void* fn, int threads, int margin, int sgprs = 112) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, 0) != hipSuccess)
    per_cu = 1;
  const int waves_per_block = (threads + 63) / 64;
  const int sgpr_waves = 800 / (((sgprs + 15) / 16) * 16 + 16);    // per SIMD
  const int sgpr_blocks = sgpr_waves * 4 / waves_per_block;         // 4 SIMDs per CU
  if (per_cu > sgpr_blocks) per_cu = sgpr_blocks;
  per_cu -= margin;
  if (per_cu < 1) per_cu = 1;
  return (unsigned)(per_cu * cus);
}

}  // namespace cpk
