// cpk_frame.hip -- writeMessage's chunking for the pack kernel (gfx950): which words start a
// chunk.  serializeSegmentTable (capnproto c++/src/capnp/serialize.c++:311-330) and writeMessage
// (:332-357) hand the segment table and then each segment to PackedOutputStream as separate
// write() pieces (kj/io.c++:109-113), and a run never crosses a piece, so the pack kernel resets
// at every message start, table end and segment start.  flat-packed batches (cpk_pack_chunks)
// give the chunk starts directly.
#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {
namespace {

// Marks word p as a chunk start (and, at a pack tile start, the tile's byte: plain byte stores,
// no atomics -- a word shared by 64 tiles, OR-ed and AND-ed by atomics, cost the tile kernel
// half its speed in contention).
__device__ __forceinline__ void mark(unsigned long long* bits, uint8_t* tstarts, uint64_t p) {
  atomicOr(bits + (p >> 6), 1ull << (p & 63));
  if (p % kPackTileWords == 0 && p) tstarts[p / kPackTileWords] = 1;  // (tile 0: no predecessor)
}

// Chunk-start bitmap + per-message framing status for a batch of flat messages.
// Message i = words[off[i], off[i+1]): segment table (serializeSegmentTable serialize.c++:
// 311-330) then segments; chunk starts = message start, table end, each segment start.
__global__ void message_bits_kernel(const uint64_t* __restrict__ words,
                                    const uint64_t* __restrict__ off, uint64_t n,
                                    unsigned long long* __restrict__ bits,
                                    uint8_t* __restrict__ tstarts,
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
  mark(bits, tstarts, w0);
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
    if (p < w1) mark(bits, tstarts, p);
    for (uint64_t s = 0; s + 1 < nseg; s++) {
      p += t32[s + 1];
      if (p < w1) mark(bits, tstarts, p);
    }
  }
  if (status) status[i] = st;
}

__global__ void chunk_bits_kernel(const uint64_t* __restrict__ off, uint64_t n, uint64_t N,
                                  unsigned long long* __restrict__ bits,
                                  uint8_t* __restrict__ tstarts, TileFirstJob tf,
                                  uint32_t tf_block) {
  if (run_tile_first(tf, tf_block)) return;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && N > 0) mark(bits, tstarts, 0);  // word 0 always starts a chunk
  if (i >= n) return;
  const uint64_t p = off[i];
  if (p < N && off[i + 1] > p) mark(bits, tstarts, p);
}

}  // namespace

hipError_t launch_message_bits(const uint64_t* words, const uint64_t* off, uint64_t n,
                               uint64_t* bits, uint8_t* tstarts, int32_t* status,
                               const TileFirstJob& tf, hipStream_t stream) {
  const unsigned nb = (unsigned)((n + 255) / 256);
  if (nb + tile_first_blocks(tf) == 0) return hipSuccess;
  hipLaunchKernelGGL(message_bits_kernel, dim3(nb + tile_first_blocks(tf)), dim3(256), 0, stream,
                     words, off, n, (unsigned long long*)bits, tstarts,
                     status, tf, nb);
  return hipGetLastError();
}

hipError_t launch_chunk_bits(const uint64_t* off, uint64_t n, uint64_t N, uint64_t* bits,
                             uint8_t* tstarts, const TileFirstJob& tf, hipStream_t stream) {
  const unsigned nb = (n == 0 && N == 0) ? 0u : (unsigned)((n + 256) / 256);
  if (nb + tile_first_blocks(tf) == 0) return hipSuccess;
  hipLaunchKernelGGL(chunk_bits_kernel, dim3(nb + tile_first_blocks(tf)), dim3(256), 0, stream,
                     off, n, N, (unsigned long long*)bits, tstarts, tf, nb);
  return hipGetLastError();
}

}  // namespace cpk
