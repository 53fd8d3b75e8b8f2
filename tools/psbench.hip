// tools/psbench.hip -- partsplit_kernel alone on one synthetic round
// (development tool): one parent node of N points split by a proven cut
// (R >= 128) or by a 2-means plane, its two children (cuts G >= 128 and
// B >= 100) split in the same launch, 64K-point tiles.  Checks the child
// buffer (per-region counts, sums, cut sides) and the children's split sums
// against the host, then times the launch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off [-D...] -o tools/psbench tools/psbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../clusteringsegmentation-1_amd/csrc/dq_kernels.hip"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace dq;

int main(int argc, char** argv) {
  const uint32_t N = argc > 1 ? (uint32_t)strtoul(argv[1], 0, 10) : 66355200u;   // 8 x 4K
  const int planar = argc > 2 ? atoi(argv[2]) : 1;
  const int proven = argc > 3 ? atoi(argv[3]) : 1;
  const uint32_t TL = 65536;
  const uint64_t plane = (N + 255) & ~255u;
  std::vector<uint8_t> h(3 * plane, 0);
  std::vector<uint32_t> hp(N);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (uint32_t i = 0; i < N; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const uint32_t p = (uint32_t)s & 0xFFFFFF;
    hp[i] = p;
    h[i] = p >> 16; h[plane + i] = (p >> 8) & 255; h[2 * plane + i] = p & 255;
  }
  uint8_t *d_src, *d_dst;
  CK(hipMalloc(&d_src, 4 * plane + 64));
  CK(hipMalloc(&d_dst, 4 * plane + 64));
  if (planar) CK(hipMemcpy(d_src, h.data(), 3 * plane, hipMemcpyHostToDevice));
  else CK(hipMemcpy(d_src, hp.data(), 4ull * N, hipMemcpyHostToDevice));
  // the parent's final decision
  Params q;
  memset(&q, 0, sizeof q);
  q.shift = 16; q.thr = 128;
  if (!proven) {   // old iff lhs < rr R + rg G + rb B: a tilted plane
    const double om[3] = {90.0, 120.0, 140.0}, nm[3] = {170.0, 130.0, 110.0};
    q.lhs = 0.5 * (om[0] * om[0] - nm[0] * nm[0] + om[1] * om[1] - nm[1] * nm[1] + om[2] * om[2] - nm[2] * nm[2]);
    q.rr = om[0] - nm[0]; q.rg = om[1] - nm[1]; q.rb = om[2] - nm[2];
    const double M = (fabs(q.rr) + fabs(q.rg) + fabs(q.rb)) * 255.0 + fabs(q.lhs);
    q.lhsf = (float)q.lhs; q.rrf = (float)q.rr; q.rgf = (float)q.rg; q.rbf = (float)q.rb; q.eps = (float)(8e-7 * M);
  }
  auto is_old = [&](uint32_t p) -> bool {
    const uint32_t R = p >> 16, G = (p >> 8) & 255, B = p & 255;
    if (proven) return R < 128;
    double d = q.rr * (double)R; d = d + q.rg * (double)G; d = d + q.rb * (double)B;
    return q.lhs < d;
  };
  const uint32_t nt = (N + TL - 1) / TL;
  std::vector<Tile> tiles(nt);
  uint64_t n_new = 0;
  {
    uint32_t ob = 0, nb = 0;
    for (uint32_t k = 0; k < nt; ++k) {
      Tile& t = tiles[k];
      memset(&t, 0, sizeof t);
      t.node = 0; t.start = k * TL; t.end = std::min<uint32_t>(N, (k + 1) * TL);
      const uint32_t qw = ((t.end - t.start + kSweep - 1) / kSweep) * kWaveSweep;
      for (int w = 0; w < kTileWaves; ++w) {
        const uint32_t ws = std::min(t.start + w * qw, t.end), we = std::min(ws + qw, t.end);
        t.old_base[w] = ob; t.new_base[w] = nb;
        for (uint32_t i = ws; i < we; ++i) (is_old(hp[i]) ? ob : nb)++;
      }
    }
    n_new = nb;
  }
  DevNode par;
  memset(&par, 0, sizeof par);
  par.src = d_src; par.dst = d_dst; par.off = 0; par.len = N; par.tile_begin = 0; par.tile_end = (int)nt;
  par.planar = planar; par.prm = q; par.n_new_local = (uint32_t)n_new; par.proven = proven; par.tile_len = TL;
  const uint32_t n_old = N - (uint32_t)n_new;
  DevNode ch[2];
  memset(ch, 0, sizeof ch);
  const uint32_t nt0 = (n_old + TL - 1) / TL, nt1 = ((uint32_t)n_new + TL - 1) / TL;
  ch[0].off = 0; ch[0].len = n_old; ch[0].tile_len = TL; ch[0].tile_begin = 0; ch[0].tile_end = (int)nt0;
  ch[1].off = n_old; ch[1].len = (uint32_t)n_new; ch[1].tile_len = TL; ch[1].tile_begin = (int)nt0; ch[1].tile_end = (int)(nt0 + nt1);
  const int32_t thr[2] = {128, 100}, shf[2] = {8, 0};
  DevNode *d_par, *d_ch; Tile* d_tiles; PartTile* d_pt; uint32_t* d_wp; TilePartial* d_sp;
  CK(hipMalloc(&d_par, sizeof par)); CK(hipMalloc(&d_ch, sizeof ch));
  CK(hipMalloc(&d_tiles, nt * sizeof(Tile))); CK(hipMalloc(&d_pt, nt * sizeof(PartTile)));
  CK(hipMalloc(&d_wp, (nt0 + nt1 + 1) * kTileWaves * 4)); CK(hipMalloc(&d_sp, 2 * nt * sizeof(TilePartial)));
  CK(hipMemcpy(d_par, &par, sizeof par, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ch, ch, sizeof ch, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_tiles, tiles.data(), nt * sizeof(Tile), hipMemcpyHostToDevice));
  std::vector<PartTile> pts(nt);
  for (uint32_t k = 0; k < nt; ++k) {
    PartTile& p = pts[k];
    memset(&p, 0, sizeof p);
    p.tile = d_tiles + k; p.parent = d_par;
    for (int c = 0; c < 2; ++c) { p.thr[c] = thr[c]; p.shift[c] = shf[c]; p.child[c] = c; }
  }
  CK(hipMemcpy(d_pt, pts.data(), nt * sizeof(PartTile), hipMemcpyHostToDevice));
  CK(hipMemset(d_wp, 0, (nt0 + nt1 + 1) * kTileWaves * 4));
  CK(hipMemset(d_dst, 0, 4 * plane));
  RoundArgs a;
  memset(&a, 0, sizeof a);
  a.nodes = d_ch; a.wparts = d_wp; a.ptiles = d_pt; a.sparts = d_sp; a.plane = plane; a.counts = nullptr;
  launch_partsplit(a, (int)nt, 0);
  CK(hipDeviceSynchronize());
  // checks: each child region holds its half (counts by cut side, channel sums)
  std::vector<uint8_t> o(3 * plane);
  CK(hipMemcpy(o.data(), d_dst, 3 * plane, hipMemcpyDeviceToHost));
  uint64_t want[2][3] = {{0}}, got[2][3] = {{0}}, want_split[2][7] = {{0}};
  for (uint32_t i = 0; i < N; ++i) {
    const uint32_t p = hp[i];
    const int side = is_old(p) ? 0 : 1;
    const uint32_t ch3[3] = {p >> 16, (p >> 8) & 255, p & 255};
    for (int c = 0; c < 3; ++c) want[side][c] += ch3[c];
    const uint32_t v = (p >> shf[side]) & 255;
    if ((int)v >= thr[side]) {
      want_split[side][0]++;
      for (int c = 0; c < 3; ++c) { want_split[side][1 + c] += ch3[c]; want_split[side][4 + c] += ch3[c] * ch3[c]; }
    }
  }
  bool ok = true;
  for (uint32_t i = 0; i < N; ++i) {
    const int side = i < n_old ? 0 : 1;
    const uint32_t p = ((uint32_t)o[i] << 16) | ((uint32_t)o[plane + i] << 8) | o[2 * plane + i];
    if ((is_old(p) ? 0 : 1) != side) { if (ok) printf("point %u on the wrong side\n", i); ok = false; }
    for (int c = 0; c < 3; ++c) got[side][c] += o[c * plane + i];
  }
  for (int sd = 0; sd < 2; ++sd) for (int c = 0; c < 3; ++c) if (got[sd][c] != want[sd][c]) { printf("sum mismatch side %d ch %d\n", sd, c); ok = false; }
  std::vector<TilePartial> sp(2 * nt);
  CK(hipMemcpy(sp.data(), d_sp, 2 * nt * sizeof(TilePartial), hipMemcpyDeviceToHost));
  for (int sd = 0; sd < 2; ++sd)
    for (int f = 0; f < 7; ++f) {
      uint64_t t = 0;
      for (uint32_t k = 0; k < nt; ++k) t += sp[2 * k + sd].f[f];
      if (t != want_split[sd][f]) { printf("split sum mismatch child %d field %d: %llu vs %llu\n", sd, f, (unsigned long long)t, (unsigned long long)want_split[sd][f]); ok = false; }
    }
  printf("check: %s (n=%u, new %llu, planar %d, proven %d)\n", ok ? "ok" : "FAILED", N, (unsigned long long)n_new, planar, proven);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int reps = 20;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch_partsplit(a, (int)nt, 0);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double bytes = (planar ? 3.0 : 4.0) * N + 3.0 * N;
  printf("partsplit %s %s: %.1f us  %.0f GB/s engine model\n", planar ? "planar" : "packed", proven ? "cut" : "plane", us, bytes / (us * 1e-6) / 1e9);
  return ok ? 0 : 1;
}
