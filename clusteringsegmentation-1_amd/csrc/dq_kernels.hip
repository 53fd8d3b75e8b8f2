// dq_kernels.hip -- gfx950 (CDNA4, wave64) kernels of the DivQuant hot path.
//
// MUST be compiled with -ffp-contract=off: every FP64 expression here mirrors
// an expression of the reference (DivQuant/DivQuantCluster.cpp) operation by
// operation, and a fused multiply-add would change its rounding.
// tests/test_build.py checks the code object for v_fma_f64 outside divisions.
//
// Kernels
//   pass_kernel<KIND>     one sweep over the tiles of every node being split
//                         (all frames of the batch): per-point decision +
//                         exact integer new-side sums (split pass :438-559,
//                         2-means pass :613-811, root statistics :49-104),
//                         one plain 32-B partial per tile.  HBM/MALL-bound:
//                         4 B read per point.
//   epilogue_kernel<KIND> per node: sum its tile partials in u64 and run the
//                         reference's FP64 update (:561-598, :787-871),
//                         publishing the next pass's decision in DevNode.
//   partition_kernel      writes each node's points into its two children's
//                         segments (replaces the per-split O(N) member[]
//                         gather, :894-1026).  Reads 4 B, writes 4 B per point.
//   build_cells_kernel    map: per 8x8x8 colour cell, the palette entries that
//                         can be nearest to some colour of the cell.
//   map_kernel            map: per pixel argmin over (squared distance, MPS
//                         visit rank) -- identical to map_colors_mps's pruned
//                         walk (DivQuantMapColors.cpp:385-527), see DESIGN.md.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "dq_kernels.h"

namespace dq {

namespace {

// Global-address-space views: pointers read from DevNode are generic, and
// generic (flat_*) loads make the compiler wait vmcnt(0)+lgkmcnt(0) around
// them; these casts give global_load/store with an SGPR base.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) uint32_t g_cu32;
typedef const __attribute__((address_space(1))) u32x4 g_cu4;
typedef __attribute__((address_space(1))) uint32_t g_u32;
__device__ __forceinline__ g_cu4* as_g4(const uint32_t* p) { return (g_cu4*)p; }
__device__ __forceinline__ g_cu32* as_g(const uint32_t* p) { return (g_cu32*)p; }
__device__ __forceinline__ g_u32* as_gw(uint32_t* p) { return (g_u32*)p; }

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

// (:561-598 / :787-810) means and weights of both halves from the new side's
// exact integer sums.  cnt/sums are exact in double (all < 2^53).
__device__ __forceinline__ void means_from_sums(const uint64_t t[F_NUM], double s, double tw,
                                                const double tm[3], double om[3], double nm[3],
                                                double* nw_out, double* ow_out) {
  const double nw = (double)t[F_CNT] * s;
  const double ow = tw - nw;
  for (int c = 0; c < 3; ++c) {
    double m = (double)t[F_SR + c];
    m *= s;
    nm[c] = m / nw;
  }
  for (int c = 0; c < 3; ++c) om[c] = (tw * tm[c] - nw * nm[c]) / ow;
  *nw_out = nw;
  *ow_out = ow;
}

// (:616-623) + the FP32 filter bound.  The filter evaluates
//   df = rr*R + rg*G + rb*B - lhs   in f32 (3 fma).
// With M = (|rr|+|rg|+|rb|)*255 + |lhs|, its error is below 7*2^-24*M (four
// f32 conversions, three f32 roundings) and the FP64 sum's error is below
// 4*2^-53*M, so whenever |df| > eps = 8e-7*M the sign of df equals the sign
// of the FP64 expression's (lhs < sum) outcome.  Non-finite or tiny M
// (NaN/inf means of an empty half) disables the filter: eps = +inf.
__device__ __forceinline__ void decision_from_means(const double om[3], const double nm[3],
                                                    Params* p) {
  p->lhs = 0.5 * (om[0] * om[0] - nm[0] * nm[0] + om[1] * om[1] - nm[1] * nm[1] +
                  om[2] * om[2] - nm[2] * nm[2]);
  p->rr = om[0] - nm[0];
  p->rg = om[1] - nm[1];
  p->rb = om[2] - nm[2];
  const double M = (fabs(p->rr) + fabs(p->rg) + fabs(p->rb)) * 255.0 + fabs(p->lhs);
  p->lhsf = (float)p->lhs;
  p->rrf = (float)p->rr;
  p->rgf = (float)p->rg;
  p->rbf = (float)p->rb;
  p->eps = (M > 1e-30 && M < 1e30) ? (float)(8e-7 * M) : __builtin_inff();
}

// Split pass threshold: cut_pos < v  <=>  v >= thr for integer v in [0,255].
__device__ __forceinline__ int32_t split_threshold(double cut) {
  if (!(cut == cut)) return 256;     // NaN: nothing moves
  if (cut < 0.0) return 0;
  if (cut >= 255.0) return 256;
  return (int32_t)floor(cut) + 1;
}

// The 2-means decision (:683): a point stays OLD iff lhs < rr*R + rg*G + rb*B
// (left to right, every product rounded).  Ties and NaN go NEW.
__device__ __forceinline__ bool stays_old_exact(uint32_t p, const Params& q) {
  const double R = (double)((p >> 16) & 0xFF);
  const double G = (double)((p >> 8) & 0xFF);
  const double B = (double)(p & 0xFF);
  double d = q.rr * R;
  d = d + q.rg * G;
  d = d + q.rb * B;
  return q.lhs < d;
}

__device__ __forceinline__ bool stays_old(uint32_t p, const Params& q) {
  const float R = (float)((p >> 16) & 0xFF);
  const float G = (float)((p >> 8) & 0xFF);
  const float B = (float)(p & 0xFF);
  const float df = __builtin_fmaf(q.rrf, R, __builtin_fmaf(q.rgf, G, __builtin_fmaf(q.rbf, B, -q.lhsf)));
  const bool sure = __builtin_fabsf(df) > q.eps;
  bool old = df > 0.0f;
  if (!__all(sure)) {   // wave-uniform: only waves holding a near-boundary point pay FP64
    const bool ex = stays_old_exact(p, q);
    old = sure ? old : ex;
  }
  return old;
}

__device__ __forceinline__ uint32_t vec_elem(const u32x4& v, int e) { return v[e]; }

// This lane's kVecPerThread uint4 of the sweep starting at vs (16-B aligned).
// FULL: the whole sweep lies inside the tile.  Otherwise vectors starting at
// or past `end` are not loaded; a vector straddling `end` is loaded whole --
// every working buffer keeps >= 3 readable words of slack past each frame.
template <bool FULL>
__device__ __forceinline__ void load_sweep(g_cu4* src4, uint32_t vs, uint32_t end,
                                           u32x4 v[kVecPerThread]) {
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) {
    const uint32_t i = vs + 4u * (j * kBlock + threadIdx.x);
    if (FULL || i < end) v[j] = src4[i >> 2];
    else v[j] = (u32x4){0u, 0u, 0u, 0u};
  }
}

// Decision for one point of a pass (KIND) -- true: the point goes NEW.
template <int KIND>
__device__ __forceinline__ bool goes_new(uint32_t p, const Params& q) {
  if (KIND == PASS_INIT) return true;
  if (KIND == PASS_SPLIT) return (int32_t)((p >> q.shift) & 0xFF) >= q.thr;
  return !stays_old(p, q);
}

// Lane partial sums.  rb = R<<16 | B sums, gc = cnt<<16 | G sums: each half
// stays < 2^16 because a tile gives a lane at most 256 points.
struct LaneSums {
  uint32_t rb = 0, gc = 0, qr = 0, qg = 0, qb = 0;
};

template <int KIND, bool FULL>
__device__ __forceinline__ void sweep_sums(const u32x4 v[kVecPerThread], uint32_t vs,
                                           uint32_t start, uint32_t end, const Params& q,
                                           LaneSums& s) {
  constexpr bool kSquares = (KIND == PASS_INIT || KIND == PASS_KLAST);
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) {
    const uint32_t i0 = vs + 4u * (j * kBlock + threadIdx.x);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t p = vec_elem(v[j], e);
      bool take = goes_new<KIND>(p, q);
      if (!FULL) take = take && (i0 + e >= start) && (i0 + e < end);
      s.rb += take ? (p & 0x00FF00FFu) : 0u;
      s.gc += take ? (((p >> 8) & 0xFFu) | 0x10000u) : 0u;
      if (kSquares) {
        const uint32_t R = (p >> 16) & 0xFF, G = (p >> 8) & 0xFF, B = p & 0xFF;
        s.qr += take ? R * R : 0u;
        s.qg += take ? G * G : 0u;
        s.qb += take ? B * B : 0u;
      }
    }
  }
}

// The FP64 update after pass KIND from the node's total sums t[] (exact
// integers).  Publishes the next pass's Params, or after PASS_KLAST the
// split's results, in DevNode.
template <int KIND>
__device__ void node_update(DevNode* w, const uint64_t t[F_NUM]) {
  const double s = w->s, tw = w->tw;
  if (KIND == PASS_INIT) {
    // DivQuantClusterInitMeanAndVar (:90-104), then the cut (:388-403).
    double tm[3], tv[3];
    for (int c = 0; c < 3; ++c) {
      double m = (double)t[F_SR + c];
      double q = (double)t[F_QR + c];
      m *= s;
      q *= s;
      q -= m * m;
      tm[c] = m;
      tv[c] = q;
      w->tm[c] = m;
      w->tv[c] = q;
    }
    double maxv = tv[0], cut = tm[0];
    int axis = 0;
    if (maxv < tv[1]) { maxv = tv[1]; axis = 1; cut = tm[1]; }
    if (maxv < tv[2]) { axis = 2; cut = tm[2]; }
    w->prm.thr = split_threshold(cut);
    w->prm.shift = 16 - 8 * axis;
    return;
  }
  double tm[3];
  for (int c = 0; c < 3; ++c) tm[c] = w->tm[c];
  double om[3], nm[3], nw, ow;
  means_from_sums(t, s, tw, tm, om, nm, &nw, &ow);
  if (KIND == PASS_SPLIT || KIND == PASS_KMEANS) {
    Params p = w->prm;
    decision_from_means(om, nm, &p);
    w->prm = p;
    return;
  }
  // PASS_KLAST: the split's results (:787-871).  prm keeps the last decision
  // (the partition replays it).
  double nv[3], ov[3];
  for (int c = 0; c < 3; ++c) {                  // (:836-838)
    double q = (double)t[F_QR + c];
    q *= s;
    nv[c] = q / nw - nm[c] * nm[c];
  }
  for (int c = 0; c < 3; ++c) {                  // (:845-855)
    const double dn = nm[c] - tm[c];
    const double dox = om[c] - tm[c];
    ov[c] = ((tw * w->tv[c] - nw * (nv[c] + dn * dn)) / ow) - dox * dox;
  }
  for (int c = 0; c < 3; ++c) {
    w->om[c] = om[c];
    w->nm[c] = nm[c];
    w->nv[c] = nv[c];
    w->ov[c] = ov[c];
  }
  w->nw = nw;
  w->ow = ow;
  w->tse_old = ow * (ov[0] + ov[1] + ov[2]);   // (:870-871)
  w->tse_new = nw * (nv[0] + nv[1] + nv[2]);
  w->n_new = t[F_CNT];
}

}  // namespace

// ---------------------------------------------------------------------------
// Statistics pass.  One workgroup per tile; a tile lies inside one node's
// segment, so every point of the workgroup shares the node's parameters and
// the sums need no per-point binning: packed lane partials -> wave sums ->
// LDS -> one 32-B partial per tile.
template <int KIND>
__global__ __launch_bounds__(kBlock) void pass_kernel(RoundArgs a) {
  const Tile t = a.tiles[blockIdx.x];
  const DevNode& nd = a.nodes[t.node];
  g_cu4* src4 = as_g4(nd.src);
  const Params q = nd.prm;
  constexpr bool kSquares = (KIND == PASS_INIT || KIND == PASS_KLAST);
  constexpr int kNF = kSquares ? 7 : 4;

  __shared__ uint32_t red[kBlock / 64][8];
  LaneSums s;
  u32x4 v[kVecPerThread];
  for (uint32_t vs = t.start & ~3u; vs < t.end; vs += kSweep) {
    if (vs >= t.start && vs + kSweep <= t.end) {   // wave-uniform
      load_sweep<true>(src4, vs, t.end, v);
      sweep_sums<KIND, true>(v, vs, t.start, t.end, q, s);
    } else {
      load_sweep<false>(src4, vs, t.end, v);
      sweep_sums<KIND, false>(v, vs, t.start, t.end, q, s);
    }
  }

  uint32_t f[8] = {s.gc >> 16, s.rb >> 16, s.gc & 0xFFFF, s.rb & 0xFFFF, s.qr, s.qg, s.qb, 0};
#pragma unroll
  for (int k = 0; k < kNF; ++k) f[k] = wave_sum_u32(f[k]);
  if (lane_id() == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[wave_id()][k] = k < kNF ? f[k] : 0u;
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    uint32_t x = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) x += red[w][threadIdx.x];
    as_gw(a.parts[blockIdx.x].f)[threadIdx.x] = x;
  }
}

// ---------------------------------------------------------------------------
// Epilogue: one workgroup per node.
template <int KIND>
__global__ __launch_bounds__(kBlock) void epilogue_kernel(RoundArgs a) {
  DevNode* w = a.nodes + blockIdx.x;
  const int tb = w->tile_begin, te = w->tile_end;
  constexpr bool kSquares = (KIND == PASS_INIT || KIND == PASS_KLAST);
  constexpr int kNF = kSquares ? 7 : 4;
  const g_cu4* parts4 = (const g_cu4*)a.parts;

  uint64_t acc[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int base = tb; base < te; base += 4 * kBlock) {
    u32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {   // issue every load of the chunk first
      const int i = base + u * kBlock + (int)threadIdx.x;
      if (i < te) {
        x[u] = parts4[2 * i];
        if (kSquares) y[u] = parts4[2 * i + 1];
      } else {
        x[u] = (u32x4){0u, 0u, 0u, 0u};
        y[u] = (u32x4){0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc[0] += x[u][0];
      acc[1] += x[u][1];
      acc[2] += x[u][2];
      acc[3] += x[u][3];
      if (kSquares) {
        acc[4] += y[u][0];
        acc[5] += y[u][1];
        acc[6] += y[u][2];
      }
    }
  }
  __shared__ uint64_t red[kBlock / 64][8];
#pragma unroll
  for (int k = 0; k < kNF; ++k) acc[k] = wave_sum_u64(acc[k]);
  if (lane_id() == 0) {
#pragma unroll
    for (int k = 0; k < kNF; ++k) red[wave_id()][k] = acc[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t tot[F_NUM] = {0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < kNF; ++k)
      for (int v = 0; v < kBlock / 64; ++v) tot[k] += red[v][k];
    node_update<KIND>(w, tot);
  }
  if (KIND == PASS_KLAST) {
    // Each tile's first OLD point's rank among the node's old points: an
    // exclusive scan of the tiles' old counts, chunked per lane.
    __shared__ uint32_t scan[kBlock];
    const int T = te - tb;
    const int chunk = (T + kBlock - 1) / kBlock;
    const int c0 = tb + (int)threadIdx.x * chunk;
    const int c1 = min(te, c0 + chunk);
    uint32_t local = 0;
    for (int i = c0; i < c1; ++i)
      local += (a.tiles[i].end - a.tiles[i].start) - a.parts[i].f[F_CNT];
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
      a.tiles[i].old_base = run;
      run += (a.tiles[i].end - a.tiles[i].start) - a.parts[i].f[F_CNT];
    }
  }
}

// ---------------------------------------------------------------------------
// Partition: replay the last 2-means decision (DevNode.prm, bit-identical
// inputs -> bit-identical outcome) and write OLD points to [off, off+n_old)
// and NEW points to [off+n_old, off+len) of the child buffer.  Within a sweep
// points are ranked in (slot, wave, lane) order and tiles follow each other,
// so each half is a fixed permutation of the parent's points.
__global__ __launch_bounds__(kBlock) void partition_kernel(RoundArgs a) {
  const Tile t = a.tiles[blockIdx.x];
  const DevNode& nd = a.nodes[t.node];
  g_cu4* src4 = as_g4(nd.src);
  g_u32* dst = as_gw(nd.dst);
  const Params q = nd.prm;

  __shared__ uint32_t cnt[2][kVecPerThread * 4 * (kBlock / 64)];
  __shared__ uint32_t tot[2];

  const uint32_t n_old = nd.len - (uint32_t)nd.n_new;
  uint32_t old_cur = nd.off + t.old_base;
  uint32_t new_cur = nd.off + n_old + ((t.start - nd.off) - t.old_base);

  const uint32_t w = wave_id(), l = lane_id();
  constexpr int kSlots = kVecPerThread * 4;
  u32x4 v[kVecPerThread];
  for (uint32_t vs = t.start & ~3u; vs < t.end; vs += kSweep) {
    const bool full = vs >= t.start && vs + kSweep <= t.end;
    if (full) load_sweep<true>(src4, vs, t.end, v);
    else load_sweep<false>(src4, vs, t.end, v);
    uint32_t slot[kSlots];   // bit 31: old, bit 30: new; low bits: rank in wave
#pragma unroll
    for (int j = 0; j < kVecPerThread; ++j) {
      const uint32_t i0 = vs + 4u * (j * kBlock + threadIdx.x);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t p = vec_elem(v[j], e);
        const uint32_t i = i0 + e;
        const bool valid = full || ((i >= t.start) & (i < t.end));
        const bool old = valid && stays_old(p, q);
        const bool nw = valid && !old;
        const uint64_t mo = __ballot(old), mn = __ballot(nw);
        const int sidx = j * 4 + e;
        slot[sidx] = old ? (0x80000000u | mbcnt64(mo)) : (nw ? (0x40000000u | mbcnt64(mn)) : 0u);
        if (l == 0) {
          cnt[0][sidx * (kBlock / 64) + w] = (uint32_t)__popcll(mo);
          cnt[1][sidx * (kBlock / 64) + w] = (uint32_t)__popcll(mn);
        }
      }
    }
    __syncthreads();
    // Exclusive scan over the 64 (slot, wave) counts: wave 0 old, wave 1 new.
    if (w < 2) {
      const uint32_t val = cnt[w][l];
      uint32_t inc = val;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, 64);
        if (l >= (uint32_t)o) inc += u;
      }
      cnt[w][l] = inc - val;
      if (l == 63) tot[w] = inc;
    }
    __syncthreads();
#pragma unroll
    for (int sidx = 0; sidx < kSlots; ++sidx) {
      const uint32_t sl = slot[sidx];
      const uint32_t r = sl & 0x3FFFFFFFu;
      const uint32_t p = vec_elem(v[sidx >> 2], sidx & 3);
      if (sl & 0x80000000u) dst[old_cur + cnt[0][sidx * (kBlock / 64) + w] + r] = p;
      else if (sl & 0x40000000u) dst[new_cur + cnt[1][sidx * (kBlock / 64) + w] + r] = p;
    }
    old_cur += tot[0];
    new_cur += tot[1];
    __syncthreads();
  }
}

// Map, step 1: per colour cell (8x8x8 values), the palette entries whose
// minimum distance to the cell does not exceed the smallest maximum distance
// of any entry to the cell.  Every exact argmin for a colour of the cell is
// among them (ties included: <=).  One LANE per cell: the palette is read from
// LDS by broadcast (every lane the same entry, no bank conflicts).
// Record (16 B): x[15:0] count c; x[31:16], y, z, w: the first kCellInline
// candidates' sorted indices (u16), unused slots = k (a sentinel entry that is
// farther than any real one); c > kCellInline: all c indices in
// cell_idx[cell*kCellCap ...]; c == kCellBrute: scan the whole palette.
__global__ __launch_bounds__(kBlock) void build_cells_kernel(
    const uint32_t* __restrict__ pal, int k, uint32_t* __restrict__ cell_rec,
    uint16_t* __restrict__ cell_idx) {
  extern __shared__ uint32_t spal[];
  for (int i = threadIdx.x; i < k; i += kBlock) spal[i] = pal[i];
  __syncthreads();
  const uint32_t cell = blockIdx.x * kBlock + threadIdx.x;
  if (cell >= (uint32_t)kCells) return;
  const int cw = 1 << (8 - kCellBits);
  const int lo0 = (int)(cell >> (2 * kCellBits)) * cw;
  const int lo1 = (int)((cell >> kCellBits) & ((1 << kCellBits) - 1)) * cw;
  const int lo2 = (int)(cell & ((1 << kCellBits) - 1)) * cw;
  const int hi0 = lo0 + cw - 1, hi1 = lo1 + cw - 1, hi2 = lo2 + cw - 1;
  auto far2 = [](int v, int lo, int hi) { const int x = max(v - lo, hi - v); return x * x; };
  auto near2 = [](int v, int lo, int hi) {
    const int x = v < lo ? lo - v : (v > hi ? v - hi : 0);
    return x * x;
  };
  int bound = 0x7FFFFFFF;
  for (int e = 0; e < k; ++e) {
    const uint32_t q = spal[e];
    const int d = far2((q >> 16) & 0xFF, lo0, hi0) + far2((q >> 8) & 0xFF, lo1, hi1) +
                  far2(q & 0xFF, lo2, hi2);
    bound = min(bound, d);
  }
  uint32_t count = 0;
  uint32_t inl[kCellInline];
#pragma unroll
  for (int m = 0; m < kCellInline; ++m) inl[m] = (uint32_t)k;
  uint16_t* lst = cell_idx + (size_t)cell * kCellCap;
  for (int e = 0; e < k; ++e) {
    const uint32_t q = spal[e];
    const int d = near2((q >> 16) & 0xFF, lo0, hi0) + near2((q >> 8) & 0xFF, lo1, hi1) +
                  near2(q & 0xFF, lo2, hi2);
    if (d <= bound) {
      if (count < (uint32_t)kCellCap) lst[count] = (uint16_t)e;
#pragma unroll
      for (int m = 0; m < kCellInline; ++m)
        if (count == (uint32_t)m) inl[m] = (uint32_t)e;
      ++count;
    }
  }
  uint4 r;
  const uint32_t c = count > (uint32_t)kCellCap ? kCellBrute : count;
  r.x = c | (inl[0] << 16);
  r.y = inl[1] | (inl[2] << 16);
  r.z = inl[3] | (inl[4] << 16);
  r.w = inl[5] | (inl[6] << 16);
  reinterpret_cast<uint4*>(cell_rec)[cell] = r;
}

// Map, step 2.  The answer is the entry minimising (squared distance, MPS
// visit rank) where the walk starts at s = lut_init[R+G+B] and visits s,
// s+1, s-1, s+2, s-2, ...: rank(j) = 2(j-s)-1 for j > s, 2(s-j) otherwise.
// That entry is exactly what map_colors_mps returns (strict '<' keeps the
// first visited; the floor(d^2/3) pruning never drops a strictly closer
// entry).  Fast path: d = |p|^2 + |c|^2 - 2 p.c (v_dot4_u32_u8) over the
// cell's inline candidates, palette entries (colour, |c|^2 | j<<18) in LDS;
// the rank is only needed when the minimum distance is shared or the cell
// overflows, which takes a wave-uniform slow path.
__global__ __launch_bounds__(kBlock) void map_kernel(
    const uint32_t* __restrict__ in, uint32_t n, uint32_t* __restrict__ out,
    const uint32_t* __restrict__ pal, int k, const uint16_t* __restrict__ lut,
    const uint32_t* __restrict__ cell_rec, const uint16_t* __restrict__ cell_idx) {
  extern __shared__ uint32_t smem[];
  uint2* spal = reinterpret_cast<uint2*>(smem);              // k+1 entries
  uint16_t* slut = reinterpret_cast<uint16_t*>(smem + 2 * (k + 1));
  for (int i = threadIdx.x; i <= k; i += kBlock) {
    const uint32_t q = i < k ? pal[i] : 0u;
    const uint32_t c2 = i < k ? __builtin_amdgcn_udot4(q, q, 0u, false) : 0x3FFFFu;
    spal[i] = make_uint2(q, c2 | ((uint32_t)i << 18));
  }
  for (int i = threadIdx.x; i < 766; i += kBlock) slut[i] = lut[i];
  __syncthreads();
  g_cu4* rec4 = (g_cu4*)cell_rec;

  auto map_one = [&](uint32_t p) -> uint32_t {
    p &= 0xFFFFFF;
    const uint32_t R = (p >> 16) & 0xFF, G = (p >> 8) & 0xFF, B = p & 0xFF;
    const uint32_t cell = ((R >> (8 - kCellBits)) << (2 * kCellBits)) |
                          ((G >> (8 - kCellBits)) << kCellBits) | (B >> (8 - kCellBits));
    const uint32_t pp = __builtin_amdgcn_udot4(p, p, 0u, false);
    const u32x4 r = rec4[cell];
    const uint32_t idx[kCellInline] = {r[0] >> 16, r[1] & 0xFFFF, r[1] >> 16, r[2] & 0xFFFF,
                                       r[2] >> 16, r[3] & 0xFFFF, r[3] >> 16};
    uint32_t best = 0xFFFFFFFFu, bc = 0;
    bool tie = false;
#pragma unroll
    for (int m = 0; m < kCellInline; ++m) {
      const uint2 e = spal[idx[m]];
      const uint32_t d = (e.y & 0x3FFFFu) + pp - 2u * __builtin_amdgcn_udot4(p, e.x, 0u, false);
      const bool lt = d < best;
      tie = lt ? false : (tie || d == best);
      best = lt ? d : best;
      bc = lt ? e.x : bc;
    }
    const uint32_t cnt = r[0] & 0xFFFF;
    const bool slow = tie || cnt > (uint32_t)kCellInline;
    if (__any(slow)) {
      if (slow) {
        // exact key (d << 32) | rank over every candidate (the list has them all)
        const int s0 = slut[R + G + B];
        uint64_t bkey = ~0ull;
        auto ev = [&](int j) {
          const uint2 e = spal[j];
          const uint32_t d = (e.y & 0x3FFFFu) + pp - 2u * __builtin_amdgcn_udot4(p, e.x, 0u, false);
          const int tt = j - s0;
          const uint32_t rank = tt > 0 ? (uint32_t)(2 * tt - 1) : (uint32_t)(-2 * tt);
          const uint64_t key = ((uint64_t)d << 32) | rank;
          if (key < bkey) { bkey = key; bc = e.x; }
        };
        if (cnt == kCellBrute) {
          for (int j = 0; j < k; ++j) ev(j);
        } else {
          const uint16_t* lst = cell_idx + (size_t)cell * kCellCap;
          for (uint32_t m = 0; m < cnt; ++m) ev(lst[m]);
        }
      }
    }
    return bc;
  };

  const uint32_t nvec = n / 4;
  g_cu4* in4 = (g_cu4*)in;
  const uint32_t stride = gridDim.x * kBlock;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < nvec; i += stride) {
    const u32x4 p = in4[i];
    uint4 o;
    o.x = map_one(p[0]);
    o.y = map_one(p[1]);
    o.z = map_one(p[2]);
    o.w = map_one(p[3]);
    reinterpret_cast<uint4*>(out)[i] = o;
  }
  const uint32_t tail = nvec * 4 + blockIdx.x * kBlock + threadIdx.x;
  if (blockIdx.x == 0 && tail < n) out[tail] = map_one(in[tail]);
}

// ---------------------------------------------------------------------------
// Launchers.
void launch_pass(int kind, const RoundArgs& a, int ntiles, hipStream_t stream) {
  if (ntiles <= 0) return;
  const dim3 g(ntiles), b(kBlock);
  switch (kind) {
    case PASS_INIT: pass_kernel<PASS_INIT><<<g, b, 0, stream>>>(a); break;
    case PASS_SPLIT: pass_kernel<PASS_SPLIT><<<g, b, 0, stream>>>(a); break;
    case PASS_KMEANS: pass_kernel<PASS_KMEANS><<<g, b, 0, stream>>>(a); break;
    default: pass_kernel<PASS_KLAST><<<g, b, 0, stream>>>(a); break;
  }
}

void launch_epilogue(int kind, const RoundArgs& a, int nnodes, hipStream_t stream) {
  if (nnodes <= 0) return;
  const dim3 g(nnodes), b(kBlock);
  switch (kind) {
    case PASS_INIT: epilogue_kernel<PASS_INIT><<<g, b, 0, stream>>>(a); break;
    case PASS_SPLIT: epilogue_kernel<PASS_SPLIT><<<g, b, 0, stream>>>(a); break;
    case PASS_KMEANS: epilogue_kernel<PASS_KMEANS><<<g, b, 0, stream>>>(a); break;
    default: epilogue_kernel<PASS_KLAST><<<g, b, 0, stream>>>(a); break;
  }
}

void launch_partition(const RoundArgs& a, int ntiles, hipStream_t stream) {
  if (ntiles <= 0) return;
  partition_kernel<<<dim3(ntiles), dim3(kBlock), 0, stream>>>(a);
}

void launch_build_cells(const uint32_t* pal_sorted, int k, uint32_t* cell_rec,
                        uint16_t* cell_idx, hipStream_t stream) {
  const int blocks = kCells / kBlock;
  build_cells_kernel<<<dim3(blocks), dim3(kBlock), (size_t)k * 4, stream>>>(
      pal_sorted, k, cell_rec, cell_idx);
}

void launch_map(const uint32_t* in, uint32_t n, uint32_t* out,
                const uint32_t* pal_sorted, int k, const uint16_t* lut_init,
                const uint32_t* cell_rec, const uint16_t* cell_idx,
                hipStream_t stream) {
  if (n == 0) return;
  const size_t lds = (size_t)(k + 1) * 8 + 768 * 2;
  uint32_t blocks = (n / 4 + kBlock - 1) / kBlock;
  if (blocks > 2048) blocks = 2048;
  if (blocks == 0) blocks = 1;
  map_kernel<<<dim3(blocks), dim3(kBlock), lds, stream>>>(in, n, out, pal_sorted, k, lut_init,
                                                         cell_rec, cell_idx);
}

}  // namespace dq
