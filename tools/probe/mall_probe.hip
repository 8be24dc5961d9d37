// Probe: HBM streaming read vs an immediate re-read of the same chunk (Infinity Cache), and a
// copy (read + write).  Informs the chunked count -> emit design.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void read_kernel(const u32x4* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    u32x4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void copy_kernel(const u32x4* __restrict__ p, u32x4* __restrict__ q, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    q[i] = p[i];
}

int main() {
  const size_t total = 1ull << 31;  // 2 GiB source
  u32x4 *src, *dst;
  uint32_t* out;
  hipMalloc(&src, total);
  hipMalloc(&dst, total);
  hipMalloc(&out, 64);
  hipMemset(src, 1, total);
  hipMemset(dst, 0, total);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = 256 * 16, block = 256;
  for (size_t chunk : {16ull << 20, 32ull << 20, 64ull << 20, 128ull << 20, 192ull << 20, 256ull << 20, 512ull << 20}) {
    float t1 = 0, t2 = 0, tc = 0;
    int reps = 0;
    for (size_t off = 0; off + chunk <= total && reps < 8; off += chunk, reps++) {
      const u32x4* p = src + off / 16;
      // flush-ish: read a far region first
      hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(block), 0, 0, src + ((off + total / 2) % total) / 16, (size_t)(256ull << 20) / 16, out);
      hipEventRecord(e0);
      hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(block), 0, 0, p, chunk / 16, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float a; hipEventElapsedTime(&a, e0, e1); t1 += a;
      hipEventRecord(e0);
      hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(block), 0, 0, p, chunk / 16, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&a, e0, e1); t2 += a;
      hipEventRecord(e0);
      hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(block), 0, 0, p, dst + off / 16, chunk / 32);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&a, e0, e1); tc += a;
    }
    printf("chunk %4zu MiB: first read %7.1f GB/s, re-read %7.1f GB/s, copy(half) %7.1f GB/s (r+w)\n",
           chunk >> 20, chunk * reps / (t1 * 1e-3) / 1e9, chunk * reps / (t2 * 1e-3) / 1e9,
           chunk * reps / (tc * 1e-3) / 1e9);
  }
  return 0;
}
