// dq_kernels.hip -- gfx950 (CDNA4, wave64) kernels of the DivQuant hot path.
//
// MUST be compiled with -ffp-contract=off: every FP64 expression here mirrors
// an expression of the reference (DivQuant/DivQuantCluster.cpp) operation by
// operation, and a fused multiply-add would change its rounding.
// tests/test_build.py checks the code object for v_fma_f64 in the pass kernels.
//
// Kernels
//   pass_kernel<KIND>     one sweep over the tiles of every node being split:
//                         a per-point decision + exact integer new-side sums
//                         (split pass :438-559, 2-means pass :613-811, root
//                         statistics :49-104).  HBM-bound: 4 B read per point.
//   epilogue_kernel<KIND> per node: sum the node's tile partials and run the
//                         reference's FP64 update (:561-598, :787-871).
//   partition_kernel      writes each node's points into its two children's
//                         segments in index order (replaces the per-split
//                         O(N) member[] gather, :894-1026).
//   build_cells_kernel    map: per 8x8x8 colour cell, the palette entries that
//                         can be nearest to some colour of the cell.
//   map_kernel            map: per pixel argmin over (squared distance, MPS
//                         visit rank) -- identical to map_colors_mps's pruned
//                         walk (DivQuantMapColors.cpp:385-527), see DESIGN.md.
#include <hip/hip_runtime.h>

#include "dq_kernels.h"

namespace dq {

namespace {

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ uint32_t wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ const uint32_t* src_of(const PixelBufs& b, int buf) {
  return buf == BUF_IN ? b.in : (buf == BUF_P0 ? b.p0 : b.p1);
}

// The 2-means decision (:683): a point stays OLD iff
//   lhs < rr*R + rg*G + rb*B    (left to right, every product rounded).
// Ties and NaN (empty new half, :579) go NEW.
__device__ __forceinline__ bool stays_old(uint32_t p, double lhs, double rr,
                                          double rg, double rb) {
  const double R = (double)((p >> 16) & 0xFF);
  const double G = (double)((p >> 8) & 0xFF);
  const double B = (double)(p & 0xFF);
  double d = rr * R;
  d = d + rg * G;
  d = d + rb * B;
  return lhs < d;
}

// (:616-623) decision parameters from the current old/new means.
__device__ __forceinline__ void set_decision(DevNode* n) {
  const double* o = n->om;
  const double* w = n->nm;
  n->lhs = 0.5 * (o[0] * o[0] - w[0] * w[0] + o[1] * o[1] - w[1] * w[1] +
                  o[2] * o[2] - w[2] * w[2]);
  n->rr = o[0] - w[0];
  n->rg = o[1] - w[1];
  n->rb = o[2] - w[2];
}

// (:561-598 / :787-810) means and weights of both halves from the new side's
// exact integer sums.  cnt/sum are exact in double (all < 2^53).
__device__ __forceinline__ void update_means(DevNode* n, uint64_t cnt,
                                             const uint64_t sum[3], double s) {
  const double nw = (double)cnt * s;
  const double ow = n->tw - nw;
  for (int a = 0; a < 3; ++a) {
    double m = (double)sum[a];
    m *= s;
    n->nm[a] = m / nw;
  }
  for (int a = 0; a < 3; ++a)
    n->om[a] = (n->tw * n->tm[a] - nw * n->nm[a]) / ow;
  n->nw = nw;
  n->ow = ow;
  n->n_new = cnt;
}

}  // namespace

// ---------------------------------------------------------------------------
// Statistics pass.  One workgroup per tile; a tile lies inside one node's
// segment, so every point of the workgroup shares the node's parameters
// (scalar loads) and the sums need no per-point binning: lane partials in
// u32 -> wave reduction -> 4 wave totals in LDS -> one u64 partial per tile.
template <int KIND>
__global__ __launch_bounds__(kBlock) void pass_kernel(
    const Tile* __restrict__ tiles, const DevNode* __restrict__ nodes,
    PixelBufs bufs, TilePartial* __restrict__ parts) {
  const Tile t = tiles[blockIdx.x];
  const DevNode* nd = nodes + t.node;
  const uint32_t* __restrict__ src = src_of(bufs, nd->buf);

  int shift = 0;
  double cut = 0.0, lhs = 0.0, rr = 0.0, rg = 0.0, rb = 0.0;
  if (KIND == PASS_SPLIT) {
    shift = 16 - 8 * nd->axis;
    cut = nd->cut;
  }
  if (KIND == PASS_KMEANS || KIND == PASS_KLAST) {
    lhs = nd->lhs;
    rr = nd->rr;
    rg = nd->rg;
    rb = nd->rb;
  }
  constexpr bool kSquares = (KIND == PASS_INIT || KIND == PASS_KLAST);

  uint32_t c = 0, sr = 0, sg = 0, sb = 0, qr = 0, qg = 0, qb = 0;
  const uint32_t end = t.end;
  for (uint32_t base = t.start; base < end; base += kSweep) {
    uint32_t px[kPxPerThread];
    bool ok[kPxPerThread];
#pragma unroll
    for (int j = 0; j < kPxPerThread; ++j) {
      const uint32_t i = base + j * kBlock + threadIdx.x;
      ok[j] = i < end;
      px[j] = src[ok[j] ? i : t.start];
    }
#pragma unroll
    for (int j = 0; j < kPxPerThread; ++j) {
      const uint32_t p = px[j];
      bool take;
      if (KIND == PASS_INIT) {
        take = ok[j];
      } else if (KIND == PASS_SPLIT) {
        take = ok[j] && (cut < (double)((p >> shift) & 0xFF));
      } else {
        take = ok[j] && !stays_old(p, lhs, rr, rg, rb);
      }
      const uint32_t R = (p >> 16) & 0xFF, G = (p >> 8) & 0xFF, B = p & 0xFF;
      c += take ? 1u : 0u;
      sr += take ? R : 0u;
      sg += take ? G : 0u;
      sb += take ? B : 0u;
      if (kSquares) {
        qr += take ? R * R : 0u;
        qg += take ? G * G : 0u;
        qb += take ? B * B : 0u;
      }
    }
  }

  __shared__ uint32_t red[kBlock / 64][8];
  c = wave_sum_u32(c);
  sr = wave_sum_u32(sr);
  sg = wave_sum_u32(sg);
  sb = wave_sum_u32(sb);
  if (kSquares) {
    qr = wave_sum_u32(qr);
    qg = wave_sum_u32(qg);
    qb = wave_sum_u32(qb);
  }
  if (lane_id() == 0) {
    uint32_t* r = red[wave_id()];
    r[0] = c; r[1] = sr; r[2] = sg; r[3] = sb;
    r[4] = qr; r[5] = qg; r[6] = qb; r[7] = 0;
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    uint64_t v = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) v += red[w][threadIdx.x];
    reinterpret_cast<uint64_t*>(parts + blockIdx.x)[threadIdx.x] = v;
  }
}

// ---------------------------------------------------------------------------
// Per-node FP64 epilogue.  One workgroup per node: reduce the node's tile
// partials in u64, then lane 0 applies the reference's update.
template <int KIND>
__global__ __launch_bounds__(kBlock) void epilogue_kernel(
    DevNode* __restrict__ nodes, Tile* __restrict__ tiles,
    const TilePartial* __restrict__ parts, double s) {
  DevNode* nd = nodes + blockIdx.x;
  const int tb = nd->tile_begin, te = nd->tile_end;
  constexpr int kF = (KIND == PASS_INIT || KIND == PASS_KLAST) ? 7 : 4;
  uint64_t acc[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int i = tb + (int)threadIdx.x; i < te; i += kBlock) {
    const uint64_t* p = reinterpret_cast<const uint64_t*>(parts + i);
#pragma unroll
    for (int f = 0; f < kF; ++f) acc[f] += p[f];
  }
  __shared__ uint64_t red[kBlock / 64][8];
  __shared__ uint32_t scan[kBlock];
#pragma unroll
  for (int f = 0; f < kF; ++f) acc[f] = wave_sum_u64(acc[f]);
  if (lane_id() == 0) {
#pragma unroll
    for (int f = 0; f < kF; ++f) red[wave_id()][f] = acc[f];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t tot[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int w = 0; w < kBlock / 64; ++w)
      for (int f = 0; f < kF; ++f) tot[f] += red[w][f];
    const uint64_t cnt = tot[0];
    const uint64_t sum[3] = {tot[1], tot[2], tot[3]};
    if (KIND == PASS_INIT) {
      // DivQuantClusterInitMeanAndVar (:90-104), then the cut (:388-403).
      for (int a = 0; a < 3; ++a) {
        double m = (double)sum[a];
        double v = (double)tot[4 + a];
        m *= s;
        v *= s;
        v -= m * m;
        nd->tm[a] = m;
        nd->tv[a] = v;
      }
      double maxv = nd->tv[0];
      int axis = 0;
      double cut = nd->tm[0];
      if (maxv < nd->tv[1]) { maxv = nd->tv[1]; axis = 1; cut = nd->tm[1]; }
      if (maxv < nd->tv[2]) { axis = 2; cut = nd->tm[2]; }
      nd->axis = axis;
      nd->cut = cut;
    } else if (KIND == PASS_SPLIT || KIND == PASS_KMEANS) {
      update_means(nd, cnt, sum, s);
      set_decision(nd);
    } else {  // PASS_KLAST
      nd->plhs = nd->lhs;
      nd->prr = nd->rr;
      nd->prg = nd->rg;
      nd->prb = nd->rb;
      update_means(nd, cnt, sum, s);
      const double nw = nd->nw, ow = nd->ow, tw = nd->tw;
      for (int a = 0; a < 3; ++a) {          // (:836-838)
        double q = (double)tot[4 + a];
        q *= s;
        nd->nv[a] = q / nw - nd->nm[a] * nd->nm[a];
      }
      for (int a = 0; a < 3; ++a) {          // (:845-855)
        const double dn = nd->nm[a] - nd->tm[a];
        const double dox = nd->om[a] - nd->tm[a];
        nd->ov[a] = ((tw * nd->tv[a] - nw * (nd->nv[a] + dn * dn)) / ow) - dox * dox;
      }
      nd->tse_old = ow * (nd->ov[0] + nd->ov[1] + nd->ov[2]);   // (:870-871)
      nd->tse_new = nw * (nd->nv[0] + nd->nv[1] + nd->nv[2]);
    }
  }
  if (KIND == PASS_KLAST) {
    // Rank of each tile's first OLD point among the node's old points: an
    // exclusive scan of the tiles' old counts, chunked per lane.
    const int T = te - tb;
    const int chunk = (T + kBlock - 1) / kBlock;
    const int c0 = tb + (int)threadIdx.x * chunk;
    const int c1 = min(te, c0 + chunk);
    uint32_t local = 0;
    for (int i = c0; i < c1; ++i)
      local += (tiles[i].end - tiles[i].start) - (uint32_t)parts[i].cnt;
    scan[threadIdx.x] = local;
    __syncthreads();
    for (int o = 1; o < kBlock; o <<= 1) {
      const uint32_t v = threadIdx.x >= (uint32_t)o ? scan[threadIdx.x - o] : 0u;
      __syncthreads();
      scan[threadIdx.x] += v;
      __syncthreads();
    }
    uint32_t run = scan[threadIdx.x] - local;
    for (int i = c0; i < c1; ++i) {
      tiles[i].old_base = run;
      run += (tiles[i].end - tiles[i].start) - (uint32_t)parts[i].cnt;
    }
  }
}

// ---------------------------------------------------------------------------
// Partition sweep: recompute the last 2-means decision (identical inputs ->
// identical result) and write OLD points to [off, off+n_old) and NEW points to
// [off+n_old, off+len) of the child buffer, both in index order.
__global__ __launch_bounds__(kBlock) void partition_kernel(
    const Tile* __restrict__ tiles, const DevNode* __restrict__ nodes,
    PixelBufs bufs) {
  const Tile t = tiles[blockIdx.x];
  const DevNode* nd = nodes + t.node;
  const uint32_t* __restrict__ src = src_of(bufs, nd->buf);
  uint32_t* __restrict__ dst = nd->buf == BUF_P0 ? bufs.p1 : bufs.p0;
  const double lhs = nd->plhs, rr = nd->prr, rg = nd->prg, rb = nd->prb;
  const uint32_t n_old = nd->len - (uint32_t)nd->n_new;
  uint32_t old_cur = nd->off + t.old_base;
  uint32_t new_cur = nd->off + n_old + ((t.start - nd->off) - t.old_base);

  __shared__ uint32_t cnt[2][kPxPerThread * (kBlock / 64)];
  __shared__ uint32_t tot[2];
  const uint32_t w = wave_id(), l = lane_id();
  for (uint32_t base = t.start; base < t.end; base += kSweep) {
    uint32_t px[kPxPerThread];
    uint32_t slot[kPxPerThread];   // bit 31: old, bit 30: new; low bits: rank in wave
#pragma unroll
    for (int j = 0; j < kPxPerThread; ++j) {
      const uint32_t i = base + j * kBlock + threadIdx.x;
      const bool ok = i < t.end;
      px[j] = src[ok ? i : t.start];
      const bool old = ok && stays_old(px[j], lhs, rr, rg, rb);
      const bool nw = ok && !old;
      const uint64_t mo = __ballot(old), mn = __ballot(nw);
      slot[j] = old ? (0x80000000u | mbcnt64(mo)) : (nw ? (0x40000000u | mbcnt64(mn)) : 0u);
      if (l == 0) {
        cnt[0][j * (kBlock / 64) + w] = (uint32_t)__popcll(mo);
        cnt[1][j * (kBlock / 64) + w] = (uint32_t)__popcll(mn);
      }
    }
    __syncthreads();
    if (w < 2) {   // wave 0 scans the old counts, wave 1 the new counts (64 entries)
      const uint32_t v = cnt[w][l];
      uint32_t inc = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, 64);
        if (l >= (uint32_t)o) inc += u;
      }
      cnt[w][l] = inc - v;
      if (l == 63) tot[w] = inc;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPxPerThread; ++j) {
      const uint32_t sl = slot[j];
      const uint32_t r = sl & 0x3FFFFFFFu;
      if (sl & 0x80000000u) dst[old_cur + cnt[0][j * (kBlock / 64) + w] + r] = px[j];
      else if (sl & 0x40000000u) dst[new_cur + cnt[1][j * (kBlock / 64) + w] + r] = px[j];
    }
    old_cur += tot[0];
    new_cur += tot[1];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Map, step 1: per colour cell (8x8x8 values), the palette entries whose
// minimum distance to the cell does not exceed the smallest maximum distance
// of any entry to the cell.  Every exact argmin for a colour of the cell is
// among them (ties included: <=).  One wave per cell.
__global__ __launch_bounds__(kBlock) void build_cells_kernel(
    const uint32_t* __restrict__ pal, int k, uint16_t* __restrict__ cell_cnt,
    uint16_t* __restrict__ cell_idx) {
  extern __shared__ uint32_t spal[];
  for (int i = threadIdx.x; i < k; i += kBlock) spal[i] = pal[i];
  __syncthreads();
  const int cell = blockIdx.x * (kBlock / 64) + (int)wave_id();
  if (cell >= kCells) return;
  const int lane = (int)lane_id();
  const int cw = 1 << (8 - kCellBits);
  int lo[3], hi[3];
  lo[0] = (cell >> (2 * kCellBits)) * cw;
  lo[1] = ((cell >> kCellBits) & ((1 << kCellBits) - 1)) * cw;
  lo[2] = (cell & ((1 << kCellBits) - 1)) * cw;
  for (int a = 0; a < 3; ++a) hi[a] = lo[a] + cw - 1;

  uint32_t bound = 0xFFFFFFFFu;
  for (int e = lane; e < k; e += 64) {
    const uint32_t q = spal[e];
    const int v[3] = {(int)((q >> 16) & 0xFF), (int)((q >> 8) & 0xFF), (int)(q & 0xFF)};
    uint32_t d = 0;
    for (int a = 0; a < 3; ++a) {
      const int x = max(v[a] - lo[a], hi[a] - v[a]);
      d += (uint32_t)(x * x);
    }
    bound = min(bound, d);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) bound = min(bound, (uint32_t)__shfl_xor(bound, o, 64));

  uint32_t count = 0;
  for (int b = 0; b < k; b += 64) {
    const int e = b + lane;
    bool cand = false;
    if (e < k) {
      const uint32_t q = spal[e];
      const int v[3] = {(int)((q >> 16) & 0xFF), (int)((q >> 8) & 0xFF), (int)(q & 0xFF)};
      uint32_t d = 0;
      for (int a = 0; a < 3; ++a) {
        const int x = v[a] < lo[a] ? lo[a] - v[a] : (v[a] > hi[a] ? v[a] - hi[a] : 0);
        d += (uint32_t)(x * x);
      }
      cand = d <= bound;
    }
    const uint64_t m = __ballot(cand);
    if (cand) {
      const uint32_t pos = count + mbcnt64(m);
      if (pos < (uint32_t)kCellCap) cell_idx[(size_t)cell * kCellCap + pos] = (uint16_t)e;
    }
    count += (uint32_t)__popcll(m);
  }
  if (lane == 0) cell_cnt[cell] = count > (uint32_t)kCellCap ? kCellOverflow : (uint16_t)count;
}

// Map, step 2.  Key = (squared distance, MPS visit rank) where the walk
// starts at s = lut_init[R+G+B] and visits s, s+1, s-1, s+2, s-2, ...:
// rank(j) = 2(j-s)-1 for j > s, 2(s-j) otherwise.  The minimum key's entry is
// exactly what map_colors_mps returns (strict '<' keeps the first visited;
// the floor(d^2/3) pruning never drops a strictly closer entry).
template <bool kWide>
__global__ __launch_bounds__(kBlock) void map_kernel(
    const uint32_t* __restrict__ in, uint32_t n, uint32_t* __restrict__ out,
    const uint32_t* __restrict__ pal, int k, const uint16_t* __restrict__ lut,
    const uint16_t* __restrict__ cell_cnt, const uint16_t* __restrict__ cell_idx) {
  extern __shared__ uint32_t smem[];
  uint32_t* spal = smem;
  uint16_t* slut = reinterpret_cast<uint16_t*>(smem + k);
  for (int i = threadIdx.x; i < k; i += kBlock) spal[i] = pal[i];
  for (int i = threadIdx.x; i < 766; i += kBlock) slut[i] = lut[i];
  __syncthreads();
  using Key = typename std::conditional<kWide, uint64_t, uint32_t>::type;
  constexpr int kRankBits = kWide ? 32 : 11;
  const uint32_t stride = gridDim.x * kBlock;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const uint32_t p = in[i];
    const int R = (p >> 16) & 0xFF, G = (p >> 8) & 0xFF, B = p & 0xFF;
    const int s0 = slut[R + G + B];
    const uint32_t cell = ((uint32_t)(R >> (8 - kCellBits)) << (2 * kCellBits)) |
                          ((uint32_t)(G >> (8 - kCellBits)) << kCellBits) |
                          (uint32_t)(B >> (8 - kCellBits));
    const uint32_t cc = cell_cnt[cell];
    Key best = (Key)~(Key)0;
    auto eval = [&](int j) {
      const uint32_t q = spal[j];
      const int dr = R - (int)((q >> 16) & 0xFF);
      const int dg = G - (int)((q >> 8) & 0xFF);
      const int db = B - (int)(q & 0xFF);
      const uint32_t d = (uint32_t)(dr * dr + dg * dg + db * db);
      const int tt = j - s0;
      const uint32_t rank = tt > 0 ? (uint32_t)(2 * tt - 1) : (uint32_t)(-2 * tt);
      const Key key = ((Key)d << kRankBits) | (Key)rank;
      best = key < best ? key : best;
    };
    if (cc == kCellOverflow) {
      for (int j = 0; j < k; ++j) eval(j);
    } else {
      const uint16_t* lst = cell_idx + (size_t)cell * kCellCap;
      for (uint32_t m = 0; m < cc; ++m) eval(lst[m]);
    }
    const uint32_t rank = (uint32_t)(best & (((Key)1 << kRankBits) - 1));
    const int j = (rank & 1) ? s0 + (int)((rank + 1) >> 1) : s0 - (int)(rank >> 1);
    out[i] = spal[j];
  }
}

// ---------------------------------------------------------------------------
// Launchers.
void launch_pass(int kind, const Tile* tiles, int ntiles, const DevNode* nodes,
                 PixelBufs bufs, TilePartial* parts, hipStream_t stream) {
  if (ntiles <= 0) return;
  const dim3 g(ntiles), b(kBlock);
  switch (kind) {
    case PASS_INIT: pass_kernel<PASS_INIT><<<g, b, 0, stream>>>(tiles, nodes, bufs, parts); break;
    case PASS_SPLIT: pass_kernel<PASS_SPLIT><<<g, b, 0, stream>>>(tiles, nodes, bufs, parts); break;
    case PASS_KMEANS: pass_kernel<PASS_KMEANS><<<g, b, 0, stream>>>(tiles, nodes, bufs, parts); break;
    default: pass_kernel<PASS_KLAST><<<g, b, 0, stream>>>(tiles, nodes, bufs, parts); break;
  }
}

void launch_epilogue(int kind, DevNode* nodes, int nnodes, Tile* tiles,
                     const TilePartial* parts, double s, hipStream_t stream) {
  if (nnodes <= 0) return;
  const dim3 g(nnodes), b(kBlock);
  switch (kind) {
    case PASS_INIT: epilogue_kernel<PASS_INIT><<<g, b, 0, stream>>>(nodes, tiles, parts, s); break;
    case PASS_SPLIT: epilogue_kernel<PASS_SPLIT><<<g, b, 0, stream>>>(nodes, tiles, parts, s); break;
    case PASS_KMEANS: epilogue_kernel<PASS_KMEANS><<<g, b, 0, stream>>>(nodes, tiles, parts, s); break;
    default: epilogue_kernel<PASS_KLAST><<<g, b, 0, stream>>>(nodes, tiles, parts, s); break;
  }
}

void launch_partition(const Tile* tiles, int ntiles, const DevNode* nodes,
                      PixelBufs bufs, hipStream_t stream) {
  if (ntiles <= 0) return;
  partition_kernel<<<dim3(ntiles), dim3(kBlock), 0, stream>>>(tiles, nodes, bufs);
}

void launch_build_cells(const uint32_t* pal_sorted, int k, uint16_t* cell_cnt,
                        uint16_t* cell_idx, hipStream_t stream) {
  const int blocks = kCells / (kBlock / 64);
  build_cells_kernel<<<dim3(blocks), dim3(kBlock), (size_t)k * 4, stream>>>(
      pal_sorted, k, cell_cnt, cell_idx);
}

void launch_map(const uint32_t* in, uint32_t n, uint32_t* out,
                const uint32_t* pal_sorted, int k, const uint16_t* lut_init,
                const uint16_t* cell_cnt, const uint16_t* cell_idx,
                hipStream_t stream) {
  if (n == 0) return;
  const size_t lds = (size_t)k * 4 + 768 * 2;
  uint32_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  if (k <= 1024)
    map_kernel<false><<<dim3(blocks), dim3(kBlock), lds, stream>>>(
        in, n, out, pal_sorted, k, lut_init, cell_cnt, cell_idx);
  else
    map_kernel<true><<<dim3(blocks), dim3(kBlock), lds, stream>>>(
        in, n, out, pal_sorted, k, lut_init, cell_cnt, cell_idx);
}

}  // namespace dq
