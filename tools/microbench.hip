// tools/microbench.hip -- isolated timings of the hot-path kernels (hipEvents,
// many launches) on one big synthetic node.  Development tool, not shipped.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../clusteringsegmentation-1_amd/csrc/dq_kernels.hip"
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace dq;

__global__ void read_kernel(const uint4* __restrict__ p, size_t n4, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678) out[0] = acc;
}

int main(int argc, char** argv) {
  const size_t N = argc > 1 ? strtoull(argv[1], 0, 10) : 3840 * 2160;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const char* only = argc > 3 ? argv[3] : "";
  uint32_t *d_px, *d_p0, *d_out;
  CK(hipMalloc(&d_px, N * 4 + 64));
  CK(hipMalloc(&d_p0, N * 4 + 64));
  CK(hipMalloc(&d_out, 64));
  std::vector<uint32_t> h(N);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < N; ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = s & 0xFFFFFF; }
  CK(hipMemcpy(d_px, h.data(), N * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto timeit = [&](const char* name, double bytes, auto fn) {
    fn(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) fn();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    double us = ms * 1e3 / reps;
    printf("%-40s %9.2f us  %8.1f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
  };
  if (!strcmp(only, "") || !strcmp(only, "read")) for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64]; snprintf(nm, 64, "read uint4 grid=%d", g);
    timeit(nm, N * 4.0, [&] { read_kernel<<<g, 256>>>((const uint4*)d_px, N / 4, d_out); });
  }
  // one node covering all points, tiles of tl points
  if (!strcmp(only, "") || !strcmp(only, "pass")) for (uint32_t tl : {4096u, 8192u, 16384u, 32768u, 65536u}) {
    const int nt = (int)((N + tl - 1) / tl);
    std::vector<Tile> tiles(nt);
    for (int i = 0; i < nt; ++i) { tiles[i].node = 0; tiles[i].start = i * tl; tiles[i].end = std::min<size_t>(N, (size_t)(i + 1) * tl); tiles[i].old_base = 0; }
    DevNode nd; memset(&nd, 0, sizeof nd);
    nd.src = d_px; nd.dst = d_p0; nd.off = 0; nd.len = N; nd.tile_begin = 0; nd.tile_end = nt;
    nd.s = 1.0 / N; nd.tw = 1.0;
    nd.tm[0] = nd.tm[1] = nd.tm[2] = 127.5;
    Params p; memset(&p, 0, sizeof p);
    double om[3] = {64.3, 127.9, 128.2}, nm[3] = {191.7, 128.1, 127.6};
    p.lhs = 0.5 * (om[0]*om[0] - nm[0]*nm[0] + om[1]*om[1] - nm[1]*nm[1] + om[2]*om[2] - nm[2]*nm[2]);
    p.rr = om[0]-nm[0]; p.rg = om[1]-nm[1]; p.rb = om[2]-nm[2];
    double M = (fabs(p.rr)+fabs(p.rg)+fabs(p.rb))*255 + fabs(p.lhs);
    p.lhsf = p.lhs; p.rrf = p.rr; p.rgf = p.rg; p.rbf = p.rb; p.eps = 8e-7 * M;
    p.thr = 128; p.shift = 16;
    nd.prm = p;
    DevNode* d_nd; Tile* d_t; TilePartial* d_parts;
    CK(hipMalloc(&d_nd, sizeof nd)); CK(hipMalloc(&d_t, nt * sizeof(Tile)));
    CK(hipMalloc(&d_parts, nt * sizeof(TilePartial)));
    CK(hipMemcpy(d_t, tiles.data(), nt * sizeof(Tile), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_nd, &nd, sizeof nd, hipMemcpyHostToDevice));
    RoundArgs ra{d_t, d_nd, d_parts};
    char nm2[80];
    const char* kn[4] = {"init", "split", "kmeans", "klast"};
    for (int kind = 0; kind < 4; ++kind) {
      snprintf(nm2, 80, "pass %-6s tl=%u tiles=%d", kn[kind], tl, nt);
      CK(hipMemcpy(d_nd, &nd, sizeof nd, hipMemcpyHostToDevice));
      timeit(nm2, N * 4.0, [&] { launch_pass(kind, ra, nt, 0); });
    }
    snprintf(nm2, 80, "epilogue kmeans (1 node, %d tiles)", nt);
    timeit(nm2, 0, [&] { launch_epilogue(PASS_KMEANS, ra, 1, 0); });
    snprintf(nm2, 80, "pass+epilogue kmeans tl=%u", tl);
    CK(hipMemcpy(d_nd, &nd, sizeof nd, hipMemcpyHostToDevice));
    timeit(nm2, N * 4.0, [&] { launch_pass(PASS_KMEANS, ra, nt, 0); launch_epilogue(PASS_KMEANS, ra, 1, 0); });
    // partition needs n_new and old_base: run klast + its epilogue once
    CK(hipMemcpy(d_nd, &nd, sizeof nd, hipMemcpyHostToDevice));
    launch_pass(PASS_KLAST, ra, nt, 0); launch_epilogue(PASS_KLAST, ra, 1, 0); CK(hipDeviceSynchronize());
    snprintf(nm2, 80, "partition tl=%u", tl);
    timeit(nm2, N * 8.0, [&] { launch_partition(ra, nt, 0); });
    CK(hipFree(d_nd)); CK(hipFree(d_t)); CK(hipFree(d_parts));
  }
  // memcpy-only baseline for the node reset
  timeit("hipMemcpyAsync node only", 0, [&] { DevNode x; hipMemcpyAsync(d_out, &x, 16, hipMemcpyHostToDevice, 0); });
  // map: random K=256, random K=1024, clustered K=256 palettes; output checked
  // on a sample against the exact (distance, MPS rank) argmin on the host
  if (!strcmp(only, "") || !strcmp(only, "map")) {
    std::vector<uint32_t> outh(N);
    for (int variant = 0; variant < 3; ++variant) {
      const int k = variant == 1 ? 1024 : 256;
      std::vector<uint32_t> pal(k);
      for (int i = 0; i < k; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        pal[i] = variant == 2 ? (0x404040u + (uint32_t)(s & 0x3F3F3F)) : (uint32_t)(s & 0xFFFFFF);
      }
      auto sum = [](uint32_t x) { return ((x >> 16) & 255) + ((x >> 8) & 255) + (x & 255); };
      std::stable_sort(pal.begin(), pal.end(), [&](uint32_t x, uint32_t y) { return sum(x) < sum(y); });
      std::vector<uint16_t> lut(766);
      for (int v = 0; v < 766; ++v) { int best = 0; for (int i = 0; i < k; ++i) if ((int)sum(pal[i]) <= v) best = i; lut[v] = best; }
      uint32_t* d_pal; uint16_t* d_lut; uint32_t* d_rec; uint16_t* d_idx;
      CK(hipMalloc(&d_pal, k * 4)); CK(hipMalloc(&d_lut, 766 * 2)); CK(hipMalloc(&d_rec, kCells * kCellRecWords * 4)); CK(hipMalloc(&d_idx, (size_t)kCells * kCellCap * 2));
      CK(hipMemcpy(d_pal, pal.data(), k * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(d_lut, lut.data(), 766 * 2, hipMemcpyHostToDevice));
      char nm[80];
      snprintf(nm, 80, "build_cells k=%d %s", k, variant == 2 ? "clustered" : "random");
      timeit(nm, 0, [&] { launch_build_cells(d_pal, k, d_rec, d_idx, 0); });
      snprintf(nm, 80, "map k=%d %s", k, variant == 2 ? "clustered" : "random");
      timeit(nm, N * 8.0, [&] { launch_map(d_px, N, d_p0, d_pal, k, d_lut, d_rec, d_idx, 0); });
      CK(hipMemcpy(outh.data(), d_p0, N * 4, hipMemcpyDeviceToHost));
      size_t bad = 0, checked = 0;
      for (size_t i = 0; i < N; i += (i < N - 64 ? 97 : 1)) {
        const uint32_t p = h[i];
        const int s0 = lut[sum(p)];
        uint64_t best = ~0ull; uint32_t ans = 0;
        for (int j = 0; j < k; ++j) {
          const int dr = (int)((p >> 16) & 255) - (int)((pal[j] >> 16) & 255), dg = (int)((p >> 8) & 255) - (int)((pal[j] >> 8) & 255), db = (int)(p & 255) - (int)(pal[j] & 255);
          const uint64_t rank = j > s0 ? 2 * (j - s0) - 1 : 2 * (s0 - j);
          const uint64_t key = ((uint64_t)(dr * dr + dg * dg + db * db) << 32) | rank;
          if (key < best) { best = key; ans = pal[j]; }
        }
        bad += outh[i] != ans; ++checked;
      }
      printf("  map check: %zu / %zu mismatches\n", bad, checked);
      if (variant == 0) for (int bl : {512, 1024, 4096}) {
        snprintf(nm, 80, "map blocks=%d", bl);
        const size_t lds = (size_t)(k + 1) * 8 + 768 * 2;
        timeit(nm, N * 8.0, [&] { map_kernel<false><<<bl, kBlock, lds>>>(d_px, N, d_p0, d_pal, k, d_lut, d_rec, d_idx); });
      }
      CK(hipFree(d_pal)); CK(hipFree(d_lut)); CK(hipFree(d_rec)); CK(hipFree(d_idx));
    }
  }
  return 0;
}
