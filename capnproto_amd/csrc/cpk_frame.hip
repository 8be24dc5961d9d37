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

// Chunk-start bitmap + per-message framing status for a batch of flat messages.
// Message i = words[off[i], off[i+1]): segment table (serializeSegmentTable serialize.c++:
// 311-330) then segments; chunk starts = message start, table end, each segment start.
__global__ void message_bits_kernel(const uint64_t* __restrict__ words,
                                    const uint64_t* __restrict__ off, uint64_t n, uint64_t N,
                                    unsigned long long* __restrict__ bits,
                                    uint8_t* __restrict__ tstarts,
                                    int32_t* __restrict__ status, TileFirstJob tf,
                                    uint32_t tf_block) {
  if (run_tile_first(tf, tf_block)) return;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  frame_message(words, off, i, N, bits, tstarts, status);
}

__global__ void chunk_bits_kernel(const uint64_t* __restrict__ off, uint64_t n, uint64_t N,
                                  unsigned long long* __restrict__ bits,
                                  uint8_t* __restrict__ tstarts, TileFirstJob tf,
                                  uint32_t tf_block) {
  if (run_tile_first(tf, tf_block)) return;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && N > 0) mark_chunk(bits, tstarts, 0);  // word 0 always starts a chunk
  if (i >= n) return;
  const uint64_t p = off[i];
  if (p < N && off[i + 1] > p) mark_chunk(bits, tstarts, p);
}

}  // namespace

hipError_t launch_message_bits(const uint64_t* words, const uint64_t* off, uint64_t n,
                               uint64_t N, uint64_t* bits, uint8_t* tstarts, int32_t* status,
                               const TileFirstJob& tf, hipStream_t stream) {
  const unsigned nb = (unsigned)((n + 255) / 256);
  if (nb + tile_first_blocks(tf) == 0) return hipSuccess;
  hipLaunchKernelGGL(message_bits_kernel, dim3(nb + tile_first_blocks(tf)), dim3(256), 0, stream,
                     words, off, n, N, (unsigned long long*)bits, tstarts,
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
