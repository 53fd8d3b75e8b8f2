// Global-atomic throughput on gfx950 for a 2^24-entry colour table
// (count + max key per colour, one 8-B entry) and a 20023-bucket histogram.
//   hipcc --offload-arch=gfx950 -O3 -o atomic_bench tools/atomic_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void gen(uint32_t* px, uint32_t n, uint32_t mask, uint32_t seed) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    uint32_t x = i * 2654435761u ^ seed;
    x ^= x >> 15; x *= 0x2c1b3c6du; x ^= x >> 12; x *= 0x297a2d39u; x ^= x >> 15;
    px[i] = x & mask;
  }
}

__global__ void tab(const uint32_t* px, uint32_t n, uint32_t* T, uint32_t* bcnt, uint32_t* nu) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const uint32_t c = px[i] & 0xFFFFFFu;
    const uint32_t old = atomicAdd(T + 2 * c, 1u);
    atomicMax(T + 2 * c + 1, n - i);
    if (old == 0) {
      const long R = (c >> 16) & 0xFF, G = (c >> 8) & 0xFF, B = c & 0xFF;
      const uint32_t h = (uint32_t)(((R * 33023 + G * 30013 + B * 27011) & 0x7fffffff) % 20023);
      atomicAdd(bcnt + h, 1u);
    }
  }
}

__global__ void tab_only_cnt(const uint32_t* px, uint32_t n, uint32_t* T) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const uint32_t c = px[i] & 0xFFFFFFu;
    atomicAdd(T + 2 * c, 1u);
  }
}

int main() {
  const uint32_t n = 3840 * 2160;
  uint32_t *px, *T, *bcnt, *nu;
  CK(hipMalloc(&px, n * 4));
  CK(hipMalloc(&T, (size_t)8 << 24));
  CK(hipMalloc(&bcnt, 20032 * 4));
  CK(hipMalloc(&nu, 4));
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const uint32_t masks[3] = {0xFFFFFFu, 0x0FFFFFu, 0x00FFFFu};
  for (int m = 0; m < 3; ++m) {
    gen<<<2048, 256>>>(px, n, masks[m], 12345);
    for (int grid = 1024; grid <= 8192; grid *= 2) {
      float best = 1e9, best2 = 1e9, bestm = 1e9;
      for (int r = 0; r < 5; ++r) {
        CK(hipMemset(T, 0, (size_t)8 << 24));
        CK(hipMemset(bcnt, 0, 20032 * 4));
        hipEventRecord(a);
        tab<<<grid, 256>>>(px, n, T, bcnt, nu);
        hipEventRecord(b);
        CK(hipEventSynchronize(b));
        float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
        CK(hipMemset(T, 0, (size_t)8 << 24));
        hipEventRecord(a);
        tab_only_cnt<<<grid, 256>>>(px, n, T);
        hipEventRecord(b);
        CK(hipEventSynchronize(b));
        hipEventElapsedTime(&ms, a, b); if (ms < best2) best2 = ms;
        hipEventRecord(a);
        CK(hipMemsetAsync(T, 0, (size_t)8 << 24));
        hipEventRecord(b);
        CK(hipEventSynchronize(b));
        hipEventElapsedTime(&ms, a, b); if (ms < bestm) bestm = ms;
      }
      printf("mask %06x grid %d: table+hist %.1f us, count only %.1f us, memset 128MB %.1f us\n", masks[m], grid,
             best * 1e3, best2 * 1e3, bestm * 1e3);
    }
  }
  return 0;
}
