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

// Inclusive wave scans (Hillis-Steele over ds_bpermute / DPP-free; 6 steps).
__device__ __forceinline__ uint32_t wave_incl_sum32(uint32_t v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = shfl32(v, l >= d ? l - d : l);
    if (l >= d) v += o;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_incl_sum64(uint64_t v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t o = shfl64(v, l >= d ? l - d : l);
    if (l >= d) v += o;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_incl_max32(uint32_t v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = shfl32(v, l >= d ? l - d : l);
    if (l >= d) v = v > o ? v : o;
  }
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

// Decoupled look-back (exclusive prefix of tile aggregates) for tile `t` by one wave.
// desc[i] = flags | value; AGG = this tile's own aggregate, INCL = inclusive prefix.
// Segmented variant: when `seg_bit` is non-zero, a descriptor value carrying that bit marks a
// tile whose aggregate restarts the scan (a message start inside it); the look-back stops there
// and the bit is stripped from the sum.
__device__ __forceinline__ uint64_t lookback(const uint64_t* desc, uint64_t t, uint32_t* err,
                                             uint64_t seg_bit = 0) {
  const int l = lane_id();
  uint64_t excl = 0;
  int64_t j = (int64_t)t - 1;
  while (j >= 0) {
    const int64_t idx = j - l;
    uint64_t d = kDescIncl;  // lanes before tile 0 read as an inclusive zero
    if (idx >= 0) {
      uint32_t spins = 0;
      for (;;) {
        d = load_agent(desc + idx);
        if (d & kDescFlags) break;
        if (++spins >= kSpinLimit) {
          raise_error(err, kErrInternal);
          d = kDescIncl;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    const uint64_t val = d & kDescValue;
    const bool stop = (d & kDescFlags) == kDescIncl || (seg_bit && (val & seg_bit));
    const uint64_t stops = ballot(stop);
    const int k = stops ? lowest_bit(stops) : 63;
    const uint64_t contrib = (l <= k) ? (val & ~seg_bit) : 0;
    excl += wave_sum64(contrib);
    if (stops) break;
    j -= 64;
  }
  return excl;
}

}  // namespace cpk
