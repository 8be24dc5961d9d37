// cpk_scan.hip -- single-pass exclusive scan of u64 counts (message sizes -> offsets), one wave
// per 1024-element tile with the shared decoupled look-back (cpk_device.h).
#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {

namespace {

constexpr int kScanSteps = 16;
constexpr uint64_t kScanTile = 64 * kScanSteps;

__global__ __launch_bounds__(256) void scan_kernel(const uint64_t* __restrict__ in, uint64_t n,
                                                   uint64_t* __restrict__ out, uint64_t ntiles,
                                                   uint32_t* counter, uint64_t* desc,
                                                   uint32_t* err) {
  const int l = lane_id();
  uint32_t t32 = 0;
  if (l == 0) t32 = atomicAdd(counter, 1u);
  const uint64_t t = uniform32(t32);
  if (t >= ntiles) return;
  const uint64_t base = t * kScanTile;
  uint64_t v[kScanSteps];
  uint64_t sum = 0;
#pragma unroll
  for (int s = 0; s < kScanSteps; s++) {
    const uint64_t i = base + 64 * s + l;
    v[s] = i < n ? in[i] : 0;
    sum += v[s];
  }
  const uint64_t agg = wave_sum64(sum);
  uint64_t excl = 0;
  if (t == 0) {
    if (l == 0) store_agent(desc, kDescIncl | agg);
  } else {
    if (l == 0) store_agent(desc + t, kDescAgg | agg);
    excl = lookback<8>(desc, t, err);
    if (l == 0) store_agent(desc + t, kDescIncl | (excl + agg));
  }
  uint64_t carry = excl;
#pragma unroll
  for (int s = 0; s < kScanSteps; s++) {
    const uint64_t inc = wave_incl_sum64(v[s]);
    const uint64_t i = base + 64 * s + l;
    if (i < n) out[i] = carry + inc - v[s];
    carry += readlane64(inc, 63);
  }
  if (t == ntiles - 1 && l == 0) out[n] = excl + agg;
}

}  // namespace

uint64_t scan_tiles(uint64_t n) { return (n + kScanTile - 1) / kScanTile; }

hipError_t launch_exclusive_scan(const uint64_t* in, uint64_t n, uint64_t* out, uint32_t* counter,
                                 uint64_t* desc, uint32_t* err, hipStream_t stream) {
  if (n == 0) return hipMemsetAsync(out, 0, sizeof(uint64_t), stream);
  const uint64_t ntiles = scan_tiles(n);
  hipLaunchKernelGGL(scan_kernel, dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0, stream, in, n,
                     out, ntiles, counter, desc, err);
  return hipGetLastError();
}

}  // namespace cpk
