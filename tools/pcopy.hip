// tools/pcopy.hip -- bandwidth ceilings for the partition access pattern
// (development tool): plain 16-B copy vs "read 16-B sweeps, write each point
// as a dword into one of two runs per wave" (ballot-ranked, as partsplit).
//   hipcc --offload-arch=gfx950 -O3 -o tools/pcopy tools/pcopy.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void copy16(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// one block per tile of T points; each wave owns 256-point chunks per sweep
// (like partsplit); writes: old run from the wave's region start, new run
// from its end (region = the wave's share of the tile)
__global__ __launch_bounds__(256) void pcopy(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t T) {
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint32_t t0 = blockIdx.x * T;
  const uint4* s4 = reinterpret_cast<const uint4*>(src + t0);
  const uint32_t share = T / 4;                 // this wave's points
  uint32_t oc = t0 + w * share, nc = t0 + (w + 1) * share - 1;   // new run written downward
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, 0x7FFFFFF0, 0x00020000);
  for (uint32_t vs = 0; vs < T; vs += 4096) {
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = s4[(vs >> 2) + j * 256 + threadIdx.x];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t p = e == 0 ? v[j].x : e == 1 ? v[j].y : e == 2 ? v[j].z : v[j].w;
        const bool o = (p ^ (p >> 7)) & 1u;
        const uint64_t bo = __ballot(o);
        const uint32_t ro = __builtin_amdgcn_mbcnt_hi((uint32_t)(bo >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bo, 0u));
        const uint32_t idx = o ? oc + ro : nc - (l - ro);
        __builtin_amdgcn_raw_buffer_store_b32(p, rs, (int)(idx * 4u), 0, 0);
        const uint32_t co = (uint32_t)__popcll(bo);
        oc += co;
        nc -= 64u - co;
      }
    }
  }
}

// pcopy with LDS staging: per wave sweep (1024 points, wave-contiguous
// ranges), points are ranked into LDS (old run first, then new) and written
// back with 16-B stores where a 4-point group lies in one run.
__global__ __launch_bounds__(256) void pcopy_lds(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t T) {
  __shared__ uint32_t stage[4][1024];
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint32_t t0 = blockIdx.x * T;
  const uint32_t share = T / 4;
  const uint32_t r0 = t0 + w * share;
  const uint4* s4 = reinterpret_cast<const uint4*>(src + r0);
  uint32_t oc = r0, nc = r0 + share - 1;   // new run written downward (reversed order)
  uint32_t* st = stage[w];
  for (uint32_t vs = 0; vs < share; vs += 1024) {
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = s4[(vs >> 2) + j * 64 + l];
    uint32_t om = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t p = e == 0 ? v[j].x : e == 1 ? v[j].y : e == 2 ? v[j].z : v[j].w;
        om |= (((p ^ (p >> 7)) & 1u)) << (j * 4 + e);
      }
    // lane prefix of old counts
    const uint32_t co = __builtin_popcount(om);
    uint32_t inc = co;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { const uint32_t u = __shfl_up(inc, o, 64); if (l >= (uint32_t)o) inc += u; }
    const uint32_t tot_old = __shfl(inc, 63, 64);
    uint32_t po = inc - co, pn = tot_old + (l * 16 - (inc - co));
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t p = e == 0 ? v[j].x : e == 1 ? v[j].y : e == 2 ? v[j].z : v[j].w;
        const bool o = (om >> (j * 4 + e)) & 1u;
        st[o ? po : pn] = p;
        po += o; pn += !o;
      }
    __builtin_amdgcn_wave_barrier();
    // write back: LDS [0, tot_old) -> dst[oc ...], [tot_old, 1024) -> dst[nc - ...] (downward)
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t i = (q * 64 + l) * 4;   // 4 consecutive LDS words
      const uint4 x = *reinterpret_cast<const uint4*>(st + i);
      if (i + 4 <= tot_old) {
        __builtin_amdgcn_raw_buffer_store_b128((v4u){x.x, x.y, x.z, x.w}, rs, (int)((oc + i) * 4u), 0, 0);
      } else if (i >= tot_old) {
        // new run grows downward: element k of the new part goes to nc - k
        const uint32_t k = i - tot_old;
        __builtin_amdgcn_raw_buffer_store_b128((v4u){x.w, x.z, x.y, x.x}, rs, (int)((nc - k - 3) * 4u), 0, 0);
      } else {
        const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
        for (int e = 0; e < 4; ++e) {
          const uint32_t ii = i + e;
          const uint32_t idx = ii < tot_old ? oc + ii : nc - (ii - tot_old);
          __builtin_amdgcn_raw_buffer_store_b32(xs[e], rs, (int)(idx * 4u), 0, 0);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    oc += tot_old;
    nc -= 1024 - tot_old;
  }
}

int main(int argc, char** argv) {
  const size_t N = argc > 1 ? strtoull(argv[1], 0, 10) : 66355200;   // 8 x 4K
  uint32_t *a, *b;
  CK(hipMalloc(&a, N * 4)); CK(hipMalloc(&b, N * 4));
  CK(hipMemset(a, 0x5A, N * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto fn) {
    fn(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 20; ++r) fn();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 20;
    printf("%-36s %8.1f us  %7.1f GB/s (read+write)\n", name, us, 8.0 * N / (us * 1e-6) / 1e9);
  };
  for (int g : {1024, 2048, 4096}) {
    char nm[64]; snprintf(nm, 64, "copy16 grid=%d", g);
    run(nm, [&] { copy16<<<g, 256>>>((const uint4*)a, (uint4*)b, N / 4); });
  }
  for (uint32_t T : {8192u, 16384u, 65536u}) {
    char nm[64]; snprintf(nm, 64, "pcopy T=%u", T);
    run(nm, [&] { pcopy<<<(unsigned)(N / T), 256>>>(a, b, T); });
  }
  for (uint32_t T : {8192u, 16384u, 65536u}) {
    char nm[64]; snprintf(nm, 64, "pcopy_lds T=%u", T);
    run(nm, [&] { pcopy_lds<<<(unsigned)(N / T), 256>>>(a, b, T); });
  }
  return 0;
}
