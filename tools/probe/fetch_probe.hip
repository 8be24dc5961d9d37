// Probe: what rocprofv3's FETCH_SIZE counts for reads of known size and width.  Each kernel reads
// exactly `bytes` bytes of a buffer far larger than the last-level cache, once, coalesced, with
// 1-, 4-, 8- or 16-byte loads per lane; a second set reads 8-byte words at a 64-entry window per
// wave that advances by 2 entries (the shape of the unpack tile kernel's message-window loads on
// C5: neighbouring waves share most lines).  The PMC pass divides FETCH_SIZE (KiB) by the bytes
// each kernel must read, giving the correction per access width.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/fetch_probe tools/probe/fetch_probe.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT -o run -- tools/probe/fetch_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__global__ void read_width(const T* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const T v = p[i];
    if constexpr (sizeof(T) == 16) acc += v.x ^ v.y ^ v.z ^ v.w;
    else acc += (uint32_t)v ^ (uint32_t)((uint64_t)v >> 16);  // (a sum: u8 loads stay)
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;  // never: keeps the loads
}

// wave w reads 8-byte entries [2w, 2w + 64): distinct bytes 16 per wave (+ the last window)
__global__ void read_windows(const uint64_t* __restrict__ p, size_t nwaves, uint32_t* out) {
  const int l = threadIdx.x & 63;
  const size_t stride = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (size_t w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nwaves; w += stride)
    acc += (uint32_t)p[2 * w + l];
  if (acc == 0x12345678u) out[l] = acc;
}

int main() {
  const size_t bytes = 1ull << 30;  // 1 GiB per kernel, 6 buffers (each past the 256 MiB MALL)
  uint8_t* buf[6];
  uint32_t* out;
  for (auto& b : buf) {
    if (hipMalloc(&b, bytes + 4096) != hipSuccess) return 1;
    hipMemset(b, 1, bytes + 4096);
  }
  hipMalloc(&out, 4096);
  const int grid = 256 * 32, block = 256;
  read_width<uint8_t><<<grid, block>>>(buf[0], bytes, out);
  read_width<uint32_t><<<grid, block>>>((const uint32_t*)buf[1], bytes / 4, out);
  read_width<uint64_t><<<grid, block>>>((const uint64_t*)buf[2], bytes / 8, out);
  read_width<u32x4><<<grid, block>>>((const u32x4*)buf[3], bytes / 16, out);
  // windows: nwaves * 16 B distinct = bytes
  const size_t nwaves = bytes / 16;
  read_windows<<<grid, block>>>((const uint64_t*)buf[4], nwaves, out);
  read_width<u32x4><<<grid, block>>>((const u32x4*)buf[5], bytes / 16, out);
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 2;
  printf("fetch_probe: 6 kernels, %zu bytes each (u8, u32, u64, u32x4, windows, u32x4)\n", bytes);
  for (auto& b : buf) hipFree(b);
  hipFree(out);
  return 0;
}
