// cpk_gen.hip -- deterministic synthetic message batches, generated on device.
//
// Every word is a pure function of (seed, message index, word index), so each GPU of a sharded
// run builds its own shard in HBM without any transfer, and the host can regenerate any message
// for checking.  The profiles model Cap'n Proto struct data (small ints, u32 pairs, pointers,
// zero padding), pointer-heavy segments with long zero stretches, and text blobs.
#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__host__ __device__ __forceinline__ uint64_t text_word(uint64_t h) {
  uint64_t w = 0;
  for (int b = 0; b < 8; b++) w |= (uint64_t)(0x20 + ((h >> (8 * b)) & 0xff) % 95) << (8 * b);
  return w;
}

__host__ __device__ __forceinline__ uint64_t gen_word(int profile, uint64_t seed, uint64_t msg,
                                                      uint64_t idx) {
  const uint64_t mkey = splitmix64(seed ^ (msg * 0xD1B54A32D192ED03ull));
  if (profile == 3) profile = (int)(mkey % 3);
  const uint64_t h = splitmix64(mkey + idx * 0x9E3779B97F4A7C15ull);
  if (profile == 2) return text_word(h);
  if (profile == 1) {
    const uint64_t blk = idx / 340, p = idx % 340;
    const uint64_t nz = 4 + splitmix64(mkey ^ (blk * 0xA24BAED4963EE407ull)) % 73;
    if (p >= nz) return 0;
    if (h >> 63) return (h & 0xfc) | ((h >> 8) & 0xff) << 32 | ((h >> 16) & 0xffff) << 48;
    return h & 0xffffff;
  }
  const uint32_t r = (uint32_t)((h >> 56) % 100);
  if (r < 45) {
    const int k = 1 + (int)((h >> 48) % 3);
    return h & ((1ull << (8 * k)) - 1);
  }
  if (r < 65) return (h & 0xffff) | (((h >> 16) & 0xffff) << 32);
  if (r < 80) return 0;
  if (r < 90) return (h & 0xff) | ((h >> 8) & 0xff) << 32 | ((h >> 16) & 0xff) << 48;
  return text_word(splitmix64(h));
}

namespace {

// One wave per message: table words, then the segment words (coalesced stores).
__global__ __launch_bounds__(256) void gen_kernel(int profile, uint64_t seed, uint64_t first_msg,
                                                  uint64_t stride, uint64_t nmsgs, uint32_t nseg,
                                                  const uint64_t* __restrict__ off,
                                                  uint64_t* __restrict__ words) {
  const uint64_t m = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int l = lane_id();
  if (m >= nmsgs) return;
  const uint64_t w0 = off[m], w1 = off[m + 1];
  const uint64_t tw = nseg / 2 + 1;
  const uint64_t body = (w1 - w0) - tw;
  const uint64_t seg = body / nseg;  // all segments equal except the last takes the rest
  // table
  for (uint64_t i = l; i < tw; i += 64) {
    uint32_t lo, hi;
    const uint64_t e0 = 2 * i, e1 = 2 * i + 1;  // u32 entries of this table word
    auto entry = [&](uint64_t e) -> uint32_t {
      if (e == 0) return nseg - 1;
      if (e <= nseg) return (uint32_t)(e < nseg ? seg : body - seg * (nseg - 1));
      return 0;
    };
    lo = entry(e0);
    hi = entry(e1);
    words[w0 + i] = ((uint64_t)hi << 32) | lo;
  }
  for (uint64_t i = l; i < body; i += 64)
    words[w0 + tw + i] = gen_word(profile, seed, first_msg + m * stride, i);
}

// Offsets: fixed nseg x seg_words, or (seg_words == 0) one segment of 2^k words, k in [3, 11].
__global__ void gen_sizes_kernel(uint64_t seed, uint64_t first_msg, uint64_t stride, uint64_t nmsgs,
                                 uint32_t nseg,
                                 uint64_t seg_words, uint64_t* __restrict__ sizes) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nmsgs) return;
  const uint64_t tw = nseg / 2 + 1;
  if (seg_words) {
    sizes[m] = tw + (uint64_t)nseg * seg_words;
  } else {
    const uint64_t k = 3 + splitmix64(seed ^ ((first_msg + m * stride) * 0x94D049BB133111EBull)) % 9;
    sizes[m] = tw + (1ull << k);
  }
}

}  // namespace

hipError_t launch_gen(int profile, uint64_t seed, uint64_t first_msg, uint64_t stride,
                      uint64_t nmsgs,
                      uint32_t nseg, const uint64_t* off, uint64_t* words, hipStream_t stream) {
  if (nmsgs == 0) return hipSuccess;
  const uint64_t threads = nmsgs * 64;
  hipLaunchKernelGGL(gen_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream,
                     profile, seed, first_msg, stride, nmsgs, nseg, off, words);
  return hipGetLastError();
}

hipError_t launch_gen_sizes(uint64_t seed, uint64_t first_msg, uint64_t stride, uint64_t nmsgs,
                            uint32_t nseg,
                            uint64_t seg_words, uint64_t* sizes, hipStream_t stream) {
  if (nmsgs == 0) return hipSuccess;
  hipLaunchKernelGGL(gen_sizes_kernel, dim3((unsigned)((nmsgs + 255) / 256)), dim3(256), 0,
                     stream, seed, first_msg, stride, nmsgs, nseg, seg_words, sizes);
  return hipGetLastError();
}

}  // namespace cpk
