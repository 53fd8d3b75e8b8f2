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
//                         publishing the next pass's decision in DevNode;
//                         a node whose split is final writes its results
//                         straight to host memory; 2-means launches publish
//                         a per-launch status word the host polls.
//   partsplit_kernel      writes the points of nodes split in an earlier round
//                         into their two children's segments (replaces the
//                         per-split O(N) member[] gather, :894-1026) and
//                         accumulates the children's split-pass statistics on
//                         the way.  Reads 4 B, writes 4 B per point.
//   build_cells_kernel    map: per 8x8x8 colour cell, the palette entries that
//                         can be nearest to some colour of the cell.
//   map_kernel            map: per pixel argmin over (squared distance, MPS
//                         visit rank) -- identical to map_colors_mps's pruned
//                         walk (DivQuantMapColors.cpp:385-527), see DESIGN.md.
//   block_hist_kernel     genHistogramsForBlocks' per-block mode over a mapped
//                         frame (ClusteringSegmentation.cpp:420-563): one lane
//                         per dim x dim block, unordered_map tie-break order
//                         from stl_order.h.  Reads 4 B per pixel.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "dq_kernels.h"
#include "stl_order.h"

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
// (readfirstlane: provably wave-uniform, so values derived from it stay scalar)
__device__ __forceinline__ uint32_t wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

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

// Test-only stalls (RoundArgs::debug, kDebugUneven / kDebugPlanStall): about
// `us` microseconds of s_sleep by the calling wave.
__device__ __forceinline__ void debug_sleep_us(int us) {
  for (int i = 0; i < us; ++i) __builtin_amdgcn_s_sleep(40);   // (64 x 40 cycles ~ 1 us)
}
// 1 in 8 workgroups, by a hash of the workgroup index
__device__ __forceinline__ bool debug_unlucky(uint32_t b) { return ((b * 2654435761u) >> 29) == 0u; }

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


// Wave w of a workgroup owns the contiguous range [ws, we) of its tile
// [start, end): four ranges of q = ceil(len / 4096) * 1024 points (the last
// ones cut at `end`, possibly empty).  Every kernel sweeping tiles, and the
// partition's per-(tile, wave) cursors, use this ownership.  A wave sweeps
// its range in sweeps of kWaveSweep points from ws & ~3; lane l holds the
// uint4 at vs + 4 * (j * 64 + l), j < kVecPerThread.
__device__ __forceinline__ void wave_range(uint32_t start, uint32_t end, uint32_t w,
                                           uint32_t& ws, uint32_t& we) {
  const uint32_t q = ((end - start + kSweep - 1) / kSweep) * kWaveSweep;
  ws = min(start + w * q, end);
  we = min(ws + q, end);
}

// ---------------------------------------------------------------------------
// Point sweeps.  The caller's frames hold packed 0x00RRGGBB words (4 B per
// point).  The working buffers P0 / P1 hold every frame shard as three byte
// planes R, G, B, RoundArgs::plane bytes apart (3 B per point): a partition
// writes 3 B per point instead of 4, and every later pass reads 3.  A wave
// sweeps kWaveSweep points at a time (16-point aligned); each lane keeps 16
// of them byte-transposed (Sweep): word j of a channel holds the lane's slots
// 4j .. 4j+3, slot s in byte s & 3 -- the form v_dot4_u32_u8 sums directly.
// Where slot s of lane l lies (slot_pos):
//   packed source (16-B loads of 4 words at vs + 4 (64 j + l)):  vs + 256 j + 4 l + e
//   planar source (one 16-B load per plane at vs + 16 l):        vs + 16 l + s
struct RawSweep {
  u32x4 v[kVecPerThread];   // packed: 4 vectors of 4 words; planar: R, G, B (v[3] unused)
};
struct Sweep {
  uint32_t r[kVecPerThread], g[kVecPerThread], b[kVecPerThread];
};

template <bool PLANAR>
__device__ __forceinline__ uint32_t slot_pos(uint32_t vs, int s) {
  return PLANAR ? vs + 16u * lane_id() + (uint32_t)s
                : vs + 256u * (uint32_t)(s >> 2) + 4u * lane_id() + (uint32_t)(s & 3);
}

// bit s: slot s lies in [start, end)
template <bool PLANAR>
__device__ __forceinline__ uint32_t valid_mask(uint32_t vs, uint32_t start, uint32_t end) {
  uint32_t m = 0;
#pragma unroll
  for (int s = 0; s < kVecPerThread * 4; ++s)
    m |= (uint32_t)((slot_pos<PLANAR>(vs, s) - start) < (end - start)) << s;
  return m;
}

// This lane's loads of the sweep at vs.  FULL: the whole sweep lies inside
// the range.  Otherwise vectors starting at or past `end` are not loaded; a
// vector straddling `end` is loaded whole (every buffer keeps >= 16 readable
// bytes of slack past each frame shard).  `src`: the shard's element 0 (a
// packed frame) or its R plane (planar; G, B at + plane, + 2 plane).
//   BGR24 source (PLANAR's slot layout; a lane's 16 points are 48 contiguous
//   bytes B G R B G R .. at 3 (vs + 16 l): three 16-B loads, 16-B aligned
//   because vs is a multiple of 16 and the frame is 16-B aligned)
template <bool PLANAR, bool FULL, bool NT = false, bool BGR = false>
__device__ __forceinline__ void fetch_sweep(const uint8_t* src, uint64_t plane, uint32_t vs, uint32_t end,
                                            RawSweep& x) {
  if (BGR) {
    const uint32_t i = vs + 16u * lane_id();
    g_cu4* p = (g_cu4*)(src + 3ull * i);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      if (FULL || i < end) x.v[c] = NT ? __builtin_nontemporal_load(p + c) : p[c];
      else x.v[c] = (u32x4){0u, 0u, 0u, 0u};
    }
  } else if (PLANAR) {
    const uint32_t i = vs + 16u * lane_id();
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      g_cu4* p = (g_cu4*)(src + (uint64_t)c * plane + i);
      if (FULL || i < end) x.v[c] = NT ? __builtin_nontemporal_load(p) : *p;
      else x.v[c] = (u32x4){0u, 0u, 0u, 0u};
    }
  } else {
    g_cu4* s4 = (g_cu4*)src;
#pragma unroll
    for (int j = 0; j < kVecPerThread; ++j) {
      const uint32_t i = vs + 4u * (j * 64 + lane_id());
      if (FULL || i < end) x.v[j] = NT ? __builtin_nontemporal_load(s4 + (i >> 2)) : s4[i >> 2];
      else x.v[j] = (u32x4){0u, 0u, 0u, 0u};
    }
  }
}

// Raw loads -> channel words (packed: 5 v_perm_b32 per 4 points; BGR24: 6,
// from the three words w0 = B0 G0 R0 B1, w1 = G1 R1 B2 G2, w2 = R2 B3 G3 R3
// holding slots 4j .. 4j+3).
template <bool PLANAR, bool BGR = false>
__device__ __forceinline__ void unpack_sweep(const RawSweep& x, Sweep& w) {
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) {
    if (BGR) {
      const uint32_t w0 = x.v[(3 * j) >> 2][(3 * j) & 3];
      const uint32_t w1 = x.v[(3 * j + 1) >> 2][(3 * j + 1) & 3];
      const uint32_t w2 = x.v[(3 * j + 2) >> 2][(3 * j + 2) & 3];
      w.b[j] = __builtin_amdgcn_perm(w2, __builtin_amdgcn_perm(w1, w0, 0x0C060300u), 0x05020100u);
      w.g[j] = __builtin_amdgcn_perm(w2, __builtin_amdgcn_perm(w1, w0, 0x0C070401u), 0x06020100u);
      w.r[j] = __builtin_amdgcn_perm(w2, __builtin_amdgcn_perm(w1, w0, 0x0C0C0502u), 0x07040100u);
    } else if (PLANAR) {
      w.r[j] = x.v[0][j];
      w.g[j] = x.v[1][j];
      w.b[j] = x.v[2][j];
    } else {
      const u32x4 m = x.v[j];
      const uint32_t u01 = __builtin_amdgcn_perm(m[1], m[0], 0x05010400u);  // B0 B1 G0 G1
      const uint32_t u23 = __builtin_amdgcn_perm(m[3], m[2], 0x05010400u);  // B2 B3 G2 G3
      w.b[j] = __builtin_amdgcn_perm(u23, u01, 0x05040100u);                // B0 B1 B2 B3
      w.g[j] = __builtin_amdgcn_perm(u23, u01, 0x07060302u);                // G0 G1 G2 G3
      w.r[j] = __builtin_amdgcn_perm(m[1], m[0], 0x0C0C0602u) |             // R0 R1 0 0
               __builtin_amdgcn_perm(m[3], m[2], 0x06020C0Cu);              // 0 0 R2 R3
    }
  }
}

__device__ __forceinline__ uint32_t chan_byte(uint32_t w, int s) { return (w >> (8 * (s & 3))) & 0xFFu; }

// Slots whose byte on the cut axis (shift 16: R, 8: G, 0: B) is >= thr: the
// split pass's NEW side (cut_pos < v_axis, :438-559).  thr in [0, 256].
__device__ __forceinline__ uint32_t cut_new_mask(const Sweep& w, uint32_t shift, int32_t thr) {
  // the axis words by two v_perm_b32 with uniform selectors (a select of the
  // channel arrays becomes an indexed access through scratch memory)
  const uint32_t s1 = shift == 8u ? 0x07060504u : 0x03020100u, s2 = shift == 0u ? 0x07060504u : 0x03020100u;
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) {
    const uint32_t x = __builtin_amdgcn_perm(w.b[j], __builtin_amdgcn_perm(w.g[j], w.r[j], s1), s2);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      m |= ((uint32_t)(thr - 1 - (int32_t)chan_byte(x, e)) >> 31) << (4 * j + e);
  }
  return m;
}

// The 2-means decision (:683) for every slot: bit s of the result = slot s
// stays OLD.  FP32 filter in 32-bit integer arithmetic (no 64-bit compare
// masks): with a finite eps, df is finite, sign(df) > 0 <=> -bits(df) has
// bit 31 set (a -0 result has |df| <= eps and takes the exact path), and
// |df| <= eps <=> bits(|df|) - bits(eps) - 1 has bit 31 set.  Valid slots the
// filter cannot decide (every slot, when the node's filter is off) take the
// exact FP64 expression; that branch is wave-uniform.
__device__ __forceinline__ bool stays_old_exact3(uint32_t r, uint32_t g, uint32_t b, const Params& q) {
  const double R = (double)r, G = (double)g, B = (double)b;
  double d = q.rr * R;
  d = d + q.rg * G;
  d = d + q.rb * B;
  return q.lhs < d;
}

__device__ __forceinline__ uint32_t old_mask(const Sweep& w, uint32_t validm, const Params& q, bool exact_all) {
  const uint32_t epsb = __float_as_uint(q.eps);
  uint32_t om = 0;
  // 4 slots (one channel word) at a time, each group's FP64 fallback before
  // the next group: live ranges stay at one group's
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) {
    uint32_t o4 = 0, u4 = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float R = (float)chan_byte(w.r[j], e), G = (float)chan_byte(w.g[j], e), B = (float)chan_byte(w.b[j], e);
      const float df = __builtin_fmaf(q.rrf, R, __builtin_fmaf(q.rgf, G, __builtin_fmaf(q.rbf, B, -q.lhsf)));
      const uint32_t db = __float_as_uint(df);
      o4 |= ((0u - db) >> 31) << e;
      u4 |= (((db & 0x7FFFFFFFu) - epsb - 1u) >> 31) << e;
    }
    if (exact_all) u4 = 0xFu;
    u4 &= (validm >> (4 * j)) & 0xFu;
    if (__any(u4 != 0)) {   // wave-uniform
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (__any((u4 >> e) & 1u)) {
          const bool ex = stays_old_exact3(chan_byte(w.r[j], e), chan_byte(w.g[j], e), chan_byte(w.b[j], e), q);
          if ((u4 >> e) & 1u) o4 = (o4 & ~(1u << e)) | ((ex ? 1u : 0u) << e);
        }
      }
    }
    om |= o4 << (4 * j);
    __builtin_amdgcn_sched_barrier(0);
  }
  return om & validm;
}

// Lane partial sums: count, sums and sums of squares of the three channels
// over the slots of a mask (a lane sees at most 256 points of a tile: all
// exact in u32).  Per 4 slots the mask becomes 0/1 byte weights (4 bits *
// 0x204081 puts bit i at bit 8i), then v_dot4_u32_u8 of each channel word
// with the weights gives its sum, and of the masked word with itself its
// sum of squares.
struct SplitSums {
  uint32_t cnt = 0, sr = 0, sg = 0, sb = 0, qr = 0, qg = 0, qb = 0;
};
struct LaneSums : SplitSums {
  uint32_t vcnt = 0;   // points of the lane inside the tile (partition cursors)
};

template <bool ALL = false>
__device__ __forceinline__ void add_sums(const Sweep& w, uint32_t m, SplitSums& s) {
  s.cnt += ALL ? (uint32_t)(kVecPerThread * 4) : (uint32_t)__builtin_popcount(m);
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) {
    const uint32_t wt = ALL ? 0x01010101u : ((((m >> (4 * j)) & 0xFu) * 0x204081u) & 0x01010101u);
    const uint32_t mk = wt * 0xFFu;
    s.sr = __builtin_amdgcn_udot4(w.r[j], wt, s.sr, false);
    s.sg = __builtin_amdgcn_udot4(w.g[j], wt, s.sg, false);
    s.sb = __builtin_amdgcn_udot4(w.b[j], wt, s.sb, false);
    s.qr = __builtin_amdgcn_udot4(w.r[j] & mk, w.r[j], s.qr, false);
    s.qg = __builtin_amdgcn_udot4(w.g[j] & mk, w.g[j], s.qg, false);
    s.qb = __builtin_amdgcn_udot4(w.b[j] & mk, w.b[j], s.qb, false);
  }
}

// One sweep of a statistics pass: the NEW side's sums (PASS_INIT: every point).
template <int KIND, bool PLANAR, bool FULL>
__device__ __forceinline__ void sweep_sums(const Sweep& w, uint32_t vs, uint32_t start, uint32_t end,
                                           const Params& q, bool exact_all, LaneSums& s) {
  const uint32_t vm = FULL ? 0xFFFFu : valid_mask<PLANAR>(vs, start, end);
  s.vcnt += FULL ? (uint32_t)(kVecPerThread * 4) : (uint32_t)__builtin_popcount(vm);
  if (KIND == PASS_INIT) {
    if (FULL) add_sums<true>(w, vm, s);
    else add_sums(w, vm, s);
  } else if (KIND == PASS_SPLIT) {
    add_sums(w, vm & cut_new_mask(w, (uint32_t)q.shift, q.thr), s);
  } else {
    add_sums(w, vm & ~old_mask(w, vm, q, exact_all), s);
  }
}

// A wave's sweeps over [ws, we) of a pass (pass_kernel, kpass_kernel), the
// next sweep's loads issued before this sweep's arithmetic.
template <int KIND, bool PLANAR, bool BGR = false>
__device__ __forceinline__ void wave_pass(const uint8_t* src, uint64_t plane, uint32_t ws, uint32_t we,
                                          const Params& q, LaneSums& s) {
  const bool exact_all = !(q.eps < __builtin_inff());   // FP32 filter off for this node
  uint32_t vs = ws & ~15u;
  bool full = vs >= ws && vs + kWaveSweep <= we;
  RawSweep x;
  if (vs < we) {
    if (full) fetch_sweep<PLANAR, true, false, BGR>(src, plane, vs, we, x);
    else fetch_sweep<PLANAR, false, false, BGR>(src, plane, vs, we, x);
  }
  while (vs < we) {
    Sweep w;
    unpack_sweep<PLANAR, BGR>(x, w);
    const uint32_t nvs = vs + kWaveSweep;
    const bool nfull = nvs + kWaveSweep <= we;
    if (nvs < we) {
      if (nfull) fetch_sweep<PLANAR, true, false, BGR>(src, plane, nvs, we, x);
      else fetch_sweep<PLANAR, false, false, BGR>(src, plane, nvs, we, x);
    }
    if (full) sweep_sums<KIND, PLANAR, true>(w, vs, ws, we, q, exact_all, s);
    else sweep_sums<KIND, PLANAR, false>(w, vs, ws, we, q, exact_all, s);
    vs = nvs;
    full = nfull;
  }
}

// The split's results from the final partition's sums (:787-871).
__device__ void node_results(NodeResult* r, const DevNode* w, const uint64_t t[F_NUM],
                             const double om[3], const double nm[3], double nw, double ow) {
  const double s = w->s, tw = w->tw;
  double nv[3], ov[3];
  for (int c = 0; c < 3; ++c) {                  // (:836-838)
    double q = (double)t[F_QR + c];
    q *= s;
    nv[c] = q / nw - nm[c] * nm[c];
  }
  for (int c = 0; c < 3; ++c) {                  // (:845-855)
    const double dn = nm[c] - w->tm[c];
    const double dox = om[c] - w->tm[c];
    ov[c] = ((tw * w->tv[c] - nw * (nv[c] + dn * dn)) / ow) - dox * dox;
  }
  for (int c = 0; c < 3; ++c) {
    r->om[c] = om[c];
    r->nm[c] = nm[c];
    r->nv[c] = nv[c];
    r->ov[c] = ov[c];
  }
  r->nw = nw;
  r->ow = ow;
  r->tse_old = ow * (ov[0] + ov[1] + ov[2]);   // (:870-871)
  r->tse_new = nw * (nv[0] + nv[1] + nv[2]);
  r->n_new = t[F_CNT];
}

// Is the first 2-means iteration after the split a fixed point, for every
// point the node can hold?  p is that iteration's decision (old iff lhs <
// rr*R + rg*G + rb*B, :683), the split sent v_axis >= thr new (:438-559).
// On the node's box (w->box_lo/hi) the decision is checked at the corners of
// both halves of the cut: every point with v_axis >= thr must go new (max of
// the linear form <= lhs - margin) and every other point must stay old (min
// >= lhs + margin).  The margin 1e-12*M dwarfs the FP64 evaluation's error
// (< 4*2^-53*M, decision_from_means), so each point's exact outcome equals
// the cut's.  Then the iteration's halves -- hence its exact integer sums --
// are the split's, the next decision is p again, and the results are what
// the first 2-means epilogue would publish as a fixed point.
__device__ bool cut_is_fixed_point(const DevNode* w, const Params& p) {
  const double M = (fabs(p.rr) + fabs(p.rg) + fabs(p.rb)) * 255.0 + fabs(p.lhs);
  if (!(M > 1e-30 && M < 1e30)) return false;
  const double mg = 1e-12 * M;
  const double c[3] = {p.rr, p.rg, p.rb};
  const int axis = (16 - p.shift) >> 3;
  for (int side = 0; side < 2; ++side) {   // 0: the cut's old half, 1: its new half
    int lo[3], hi[3];
    for (int k = 0; k < 3; ++k) { lo[k] = w->box_lo[k]; hi[k] = w->box_hi[k]; }
    if (side) lo[axis] = max(lo[axis], p.thr);
    else hi[axis] = min(hi[axis], p.thr - 1);
    if (lo[axis] > hi[axis]) continue;   // the box holds no point of this half
    double ext = 0.0;
    for (int k = 0; k < 3; ++k) {
      const double a = c[k] * (double)lo[k], b = c[k] * (double)hi[k];
      ext += side ? fmax(a, b) : fmin(a, b);
    }
    if (side ? !(ext <= p.lhs - mg) : !(ext >= p.lhs + mg)) return false;
  }
  return true;
}

// The FP64 update after pass KIND from the node's total sums t[] (exact
// integers).  Publishes the next pass's Params, or -- when the results are
// final (PASS_KLAST, or a PASS_KMEANS at a fixed point: prm then already
// holds the decision that produced them) -- the split's results into *r and
// returns true.
template <int KIND>
__device__ bool node_update(DevNode* w, NodeResult* r, const uint64_t t[F_NUM], bool fixed_point) {
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
    return false;
  }
  double tm[3];
  for (int c = 0; c < 3; ++c) tm[c] = w->tm[c];
  double om[3], nm[3], nw, ow;
  bool final = KIND == PASS_KLAST;
  if (KIND == PASS_KMEANS) {
    w->iter += 1;
    final = fixed_point && t[F_CNT] == w->prev[0] && t[F_SR] == w->prev[1] &&
            t[F_SG] == w->prev[2] && t[F_SB] == w->prev[3];
  }
  means_from_sums(t, s, tw, tm, om, nm, &nw, &ow);
  if (final) {
    node_results(r, w, t, om, nm, nw, ow);
    w->done_it = KIND == PASS_KMEANS ? w->iter : -1;
    r->proven = 0;
    return true;
  }
  for (int c = 0; c < 4; ++c) w->prev[c] = t[F_CNT + c];
  Params p = w->prm;
  decision_from_means(om, nm, &p);
  w->prm = p;
  if (KIND == PASS_SPLIT && fixed_point && t[F_CNT] != 0 && ow > 0.0 && cut_is_fixed_point(w, p)) {
    // exactly the first 2-means epilogue's fixed-point branch on sums t
    w->iter = 1;
    node_results(r, w, t, om, nm, nw, ow);
    w->done_it = 1;
    w->proven = 1;
    r->proven = 1;
    return true;
  }
  return false;
}

}  // namespace

// ---------------------------------------------------------------------------
// Statistics pass.  One workgroup per tile; a tile lies inside one node's
// segment, so every point of the workgroup shares the node's parameters and
// the sums need no per-point binning: packed lane partials -> wave sums ->
// LDS -> one 32-B partial per tile.
// Waves per SIMD the pass kernels are compiled for (VGPR budget 512 / n).
constexpr int kPassWaves = 4;
template <int KIND>
__global__ __launch_bounds__(kBlock, kPassWaves) void pass_kernel(RoundArgs a) {
  const Tile t = a.tiles[blockIdx.x];
  const DevNode& nd = a.nodes[t.node];
  if ((KIND == PASS_KMEANS || KIND == PASS_KLAST) && nd.done_it != 0) return;   // final
  const Params q = nd.prm;
  constexpr int kNF = F_NUM;

  __shared__ uint32_t red[kBlock / 64][8];
  LaneSums s;
  uint32_t ws, we;
  wave_range(t.start, t.end, wave_id(), ws, we);
  if (nd.planar == SRC_PLANAR) wave_pass<KIND, true>(nd.src, a.plane, ws, we, q, s);
  else if (nd.planar == SRC_BGR24) wave_pass<KIND, true, true>(nd.src, a.plane, ws, we, q, s);
  else wave_pass<KIND, false>(nd.src, a.plane, ws, we, q, s);

  uint32_t f[8] = {s.cnt, s.sr, s.sg, s.sb, s.qr, s.qg, s.qb, 0};
#pragma unroll
  for (int k = 0; k < kNF; ++k) f[k] = wave_sum_u32(f[k]);
  if (KIND != PASS_INIT) {
    // this wave's (old, new) counts: the partition cursors if this pass is final
    const uint32_t vsum = wave_sum_u32(s.vcnt);
    if (lane_id() == 0) a.wparts[blockIdx.x * kTileWaves + wave_id()] = (vsum - f[F_CNT]) | (f[F_CNT] << 16);
  }
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
// This lane's share of the sums of one node record's pass: its tile partials
// in u64 (PASS_SPLIT of a record whose parent was partitioned this round: its
// half of the parent's fused partition+split partials instead).
template <int KIND, int W = kBlock>
__device__ __forceinline__ void sum_record(const RoundArgs& a, const DevNode* w, uint64_t acc[7],
                                           int tid = (int)threadIdx.x) {
  if (KIND == PASS_SPLIT && w->split_pb >= 0) {
    // the fused pass's partials of this half: TilePartial 2 * i + side
    const g_cu4* sp4 = (const g_cu4*)a.sparts;
    const int side = w->split_side;
    for (int i = w->split_pb + tid; i < w->split_pe; i += W) {
      const u32x4 x = sp4[4 * i + 2 * side], y = sp4[4 * i + 2 * side + 1];
      acc[0] += x[0];
      acc[1] += x[1];
      acc[2] += x[2];
      acc[3] += x[3];
      acc[4] += y[0];
      acc[5] += y[1];
      acc[6] += y[2];
    }
    return;
  }
  const int tb = w->tile_begin, te = w->tile_end;
  const g_cu4* parts4 = (const g_cu4*)a.parts;
  constexpr bool kSquares = true;   // (the split pass's: results of a proven split)
  for (int base = tb; base < te; base += 4 * W) {
    u32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {   // issue every load of the chunk first
      const int i = base + u * W + tid;
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
}

// Workgroup sum of the lanes' acc[] into tot[] (valid in thread 0).
__device__ __forceinline__ void block_sum7(uint64_t acc[7], uint64_t (*red)[8], uint64_t tot[7]) {
#pragma unroll
  for (int k = 0; k < F_NUM; ++k) acc[k] = wave_sum_u64(acc[k]);
  if (lane_id() == 0) {
#pragma unroll
    for (int k = 0; k < F_NUM; ++k) red[wave_id()][k] = acc[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 0; k < F_NUM; ++k) {
      tot[k] = 0;
      for (int v = 0; v < kBlock / 64; ++v) tot[k] += red[v][k];
    }
  }
}

// Sharded rounds: one workgroup per LOGICAL node sums the pass over all its
// shard records into a.tot (8 u64; the host then allreduces a.tot across
// processes with RCCL -- integer sums, so exact in any order).
template <int KIND>
__global__ __launch_bounds__(kBlock) void nodesum_kernel(RoundArgs a) {
  constexpr bool kMeans = KIND == PASS_KMEANS || KIND == PASS_KLAST;
  if (a.counts && a.counts[2] != 0) return;   // planned round aborted by its plan
  __shared__ uint64_t red[kBlock / 64][8];
  const DevNode* w0 = a.nodes + (size_t)blockIdx.x * a.nshard;
  uint64_t acc[7] = {0, 0, 0, 0, 0, 0, 0};
  if (!(kMeans && w0->done_it != 0))   // (all records of a node agree on done_it)
    for (int sh = 0; sh < a.nshard; ++sh) sum_record<KIND>(a, w0 + sh, acc);
  uint64_t tot[7];
  block_sum7(acc, red, tot);   // (valid in thread 0)
  if (threadIdx.x == 0) {
    uint64_t* g = a.tot + (size_t)blockIdx.x * 8;
    for (int k = 0; k < F_NUM; ++k) g[k] = tot[k];
    g[7] = 0;
  }
}

// ---------------------------------------------------------------------------
// Finalisation steps of a node record, one wave (epilogue_kernel and the
// fused 2-means pass, kpass_kernel).
//
// Partition cursors: for every (tile, wave) of the record, the OLD and NEW
// points before its share -- an exclusive shuffle scan of the final pass's
// per-wave counts, chunked per lane over the tiles [tb, te).  COHERENT: the
// counts were written by other workgroups of the running kernel
// (agent-scope loads).
template <bool COHERENT = false>
__device__ __forceinline__ void record_cursors(Tile* tiles, const uint32_t* wp, int tb, int te,
                                               uint32_t lane) {
  const int T = te - tb;
  const int chunk = (T + 63) / 64;
  const int c0 = tb + (int)lane * chunk;
  const int c1 = min(te, c0 + chunk);
  auto ld = [&](int i) -> uint32_t {
    if (COHERENT) return __hip_atomic_load(wp + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return wp[i];
  };
  uint64_t local = 0;   // old | new << 32
  for (int i = c0; i < c1; ++i)
    for (int ww = 0; ww < kTileWaves; ++ww) {
      const uint32_t x = ld(i * kTileWaves + ww);
      local += (uint64_t)(x & 0xFFFFu) | ((uint64_t)(x >> 16) << 32);
    }
  uint64_t inc = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += u;
  }
  const uint64_t run0 = inc - local;
  uint32_t ro = (uint32_t)run0, rn = (uint32_t)(run0 >> 32);
  for (int i = c0; i < c1; ++i)
    for (int ww = 0; ww < kTileWaves; ++ww) {
      const uint32_t x = ld(i * kTileWaves + ww);
      tiles[i].old_base[ww] = ro;
      tiles[i].new_base[ww] = rn;
      ro += x & 0xFFFFu;
      rn += x >> 16;
    }
}

// record_cursors over a whole workgroup of W lanes (the split / sharded
// epilogue: a record of an early round has ~1000 tiles).  Every lane of the
// workgroup must call it; s_tot: W / 64 words of LDS.
template <int W>
__device__ __forceinline__ void block_cursors(Tile* tiles, const uint32_t* wp, int tb, int te,
                                              uint64_t* s_tot, int wbase = 0) {
  const int T = te - tb;
  const int chunk = (T + W - 1) / W;
  const int c0 = tb + (int)threadIdx.x * chunk;
  const int c1 = min(te, c0 + chunk);
  const uint32_t lane = lane_id(), wv = wave_id();
  uint64_t local = 0;   // old | new << 32
  for (int i = c0; i < c1; ++i) {
    const u32x4 x = *(const u32x4*)(wp + (size_t)(i - wbase) * kTileWaves);
#pragma unroll
    for (int ww = 0; ww < kTileWaves; ++ww) local += (uint64_t)(x[ww] & 0xFFFFu) | ((uint64_t)(x[ww] >> 16) << 32);
  }
  uint64_t inc = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += u;
  }
  if (lane == 63) s_tot[wv] = inc;
  __syncthreads();
  uint64_t base = 0;
  for (uint32_t w = 0; w < wv; ++w) base += s_tot[w];
  const uint64_t run0 = base + inc - local;
  uint32_t ro = (uint32_t)run0, rn = (uint32_t)(run0 >> 32);
  for (int i = c0; i < c1; ++i) {
    const u32x4 x = *(const u32x4*)(wp + (size_t)(i - wbase) * kTileWaves);
    u32x4 ob, nb;
#pragma unroll
    for (int ww = 0; ww < kTileWaves; ++ww) {
      ob[ww] = ro;
      nb[ww] = rn;
      ro += x[ww] & 0xFFFFu;
      rn += x[ww] >> 16;
    }
    *(u32x4*)tiles[i].old_base = ob;
    *(u32x4*)tiles[i].new_base = nb;
  }
}

// Final results go straight to host-coherent memory: relaxed system-scope
// 8-B stores, one per lane (no L2 write-back); the device copy (ddst, may be
// null) is what the next round's plan reads.  The last word (len_local,
// tag = round seq) is stored only after the others completed (vmcnt(0)), so
// a host that sees the tag sees the record; the caller drains the tag store
// before arriving.
// sum (may be null): the record's RecSummary, from its final record w.
__device__ __forceinline__ void store_result(NodeResult* dst, NodeResult* ddst, NodeResult& r,
                                             uint32_t lane, uint32_t len_local, uint64_t seq,
                                             RecSummary* sum, const DevNode* w) {
  constexpr int kWords = (int)(sizeof(NodeResult) / 8);
  static_assert(kWords <= 64, "one wave stores the result");
  if (lane == 0) {
    r.len_local = len_local;
    r.tag = (uint32_t)seq;
  }
  if (sum && lane == 1) {
    typedef __attribute__((address_space(1))) u32x4 g_u4;
    g_u4* s4 = (g_u4*)sum;
    s4[0] = (u32x4){w->off, w->len, r.n_new_local, (uint32_t)(w->tile_end - w->tile_begin)};
    s4[1] = (u32x4){(uint32_t)w->tile_begin, 1u, 0u, 0u};
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint64_t v = lane < (uint32_t)kWords ? reinterpret_cast<const uint64_t*>(&r)[lane] : 0ull;
  // (all words in one store instruction: the host reads a round's results
  // only after its status word, which the last arriver publishes after every
  // record's vmcnt(0) -- the tag check stays as a consistency check; the
  // ordered form waited one extra host-memory round trip per record)
  if (lane < (uint32_t)kWords) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(dst) + lane, v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    if (ddst) reinterpret_cast<uint64_t*>(ddst)[lane] = v;
  }
}

// One record's arrival on a launch's counters (lane 0): 64-bit words (low =
// arrived, high = still active) on the record's shard; the shard's last
// arriver forwards to `top`, whose last arriver publishes the status word
// (seq << 32) | (active << 1) | 1 to host memory.
__device__ __forceinline__ void arrive(LaunchCtr* c, uint32_t rec, uint32_t nn, bool active,
                                       uint64_t* hstat, uint64_t seq) {
  const uint32_t sh = rec % kArrShards;
  const uint32_t nsh = min(nn, (uint32_t)kArrShards);
  const uint32_t in_shard = (nn - sh + kArrShards - 1) / kArrShards;
  const uint64_t mine = 1ull | ((uint64_t)active << 32);
  const uint64_t old = __hip_atomic_fetch_add(&c->shard[sh].word, mine, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
  if ((uint32_t)old == in_shard - 1) {
    const uint64_t fwd = 1ull | (((old >> 32) + (mine >> 32)) << 32);
    const uint64_t t = __hip_atomic_fetch_add(&c->top.word, fwd, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)t == nsh - 1) {
      const uint64_t act = (t >> 32) + (fwd >> 32);
      __hip_atomic_store(hstat, (seq << 32) | (act << 1) | 1ull, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---------------------------------------------------------------------------
// Epilogue: ONE WORKGROUP per node record of the round.
//   * the node's sums (MODE, TotMode): its own partials (TOT_OWN), those of
//     every shard record of the logical node (TOT_NODE), or the node's
//     totals from nodesum + allreduce (TOT_ALLREDUCE); its own partials
//     always give the record's local new-half size.  Summed by all kEpiBlock
//     lanes (a record of an early round has ~1000 tile partials), then
//     reduced in LDS;
//   * wave 0, lane 0 runs the FP64 update (node_update) -- every record of a
//     logical node runs it on the same totals, so all agree bit for bit;
//   * a record whose split became final: the partition's per-(tile, wave)
//     write cursors (a shuffle scan over the lanes' tile chunks), and the
//     results written straight to host memory (NodeResult) and to the
//     device copy the next round's plan reads;
//   * 2-means and split launches: every record arrives on the launch's
//     (sharded) counter; the last to arrive publishes (round seq, records
//     still active) to the host, which stops launching iterations once no
//     node is active (after the split: nodes proven final by
//     cut_is_fixed_point need no 2-means pass at all).
constexpr int kEpiBlock = 256;
// The record and (up to kEpiStageTiles tiles) its per-(tile, wave) counts
// are staged in LDS at the start, beside the partial sums: the FP64 update
// and the cursor scan then read LDS, not one dependent global round trip
// after another; the updated record is written back once.
constexpr int kEpiStageTiles = 1024;
template <int KIND, int MODE>
__global__ __launch_bounds__(kEpiBlock) void epilogue_kernel(RoundArgs a) {
  constexpr bool kMeans = KIND == PASS_KMEANS || KIND == PASS_KLAST;
  if (a.counts && a.counts[2] != 0) return;   // planned round aborted by its plan
  DevNode* gw = a.nodes + blockIdx.x;
  const uint32_t lane = lane_id();
  __shared__ __attribute__((aligned(16))) DevNode sw;
  __shared__ __attribute__((aligned(16))) uint32_t s_wp[kEpiStageTiles * kTileWaves];
  static_assert(sizeof(DevNode) % 16 == 0, "the record is staged in 16-B words");
  constexpr int kW16 = (int)(sizeof(DevNode) / 16);
  typedef __attribute__((address_space(1))) u32x4 g_u4;
  if (threadIdx.x < (uint32_t)kW16) reinterpret_cast<u32x4*>(&sw)[threadIdx.x] = ((const g_cu4*)gw)[threadIdx.x];
  __syncthreads();
  DevNode* w = &sw;
  const bool skip = kMeans && w->done_it != 0;   // final in an earlier launch
  const int tb = w->tile_begin, te = w->tile_end;
  const bool stage_wp = (kMeans || KIND == PASS_SPLIT) && !skip && te - tb <= kEpiStageTiles;
  if (stage_wp) {
    const g_cu4* wp4 = (const g_cu4*)(a.wparts + (size_t)tb * kTileWaves);
    for (int i = (int)threadIdx.x; i < te - tb; i += kEpiBlock) reinterpret_cast<u32x4*>(s_wp)[i] = wp4[i];
  }
  __shared__ NodeResult sres;
  __shared__ uint64_t red[kEpiBlock / 64][8];
  uint64_t tot[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t own_new = 0;   // the record's own new-side count (its partition share)
  if (!skip) {
    uint64_t acc[7] = {0, 0, 0, 0, 0, 0, 0};
    sum_record<KIND, kEpiBlock>(a, w, acc, (int)threadIdx.x);
    own_new = acc[F_CNT];
    if (MODE == TOT_NODE) {   // every shard record of the logical node
      const int r0 = (int)(blockIdx.x / a.nshard) * a.nshard;
      for (int r = r0; r < r0 + a.nshard; ++r)
        if (r != (int)blockIdx.x) sum_record<KIND, kEpiBlock>(a, a.nodes + r, acc, (int)threadIdx.x);
    }
    own_new = wave_sum_u64(own_new);
#pragma unroll
    for (int k = 0; k < F_NUM; ++k) acc[k] = wave_sum_u64(acc[k]);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < F_NUM; ++k) red[wave_id()][k] = acc[k];
      red[wave_id()][7] = own_new;
    }
    __syncthreads();
    own_new = 0;
#pragma unroll
    for (int k = 0; k < F_NUM; ++k)
      for (int v = 0; v < kEpiBlock / 64; ++v) tot[k] += red[v][k];   // (every lane)
    for (int v = 0; v < kEpiBlock / 64; ++v) own_new += red[v][7];
  }
  // lane 0 of wave 0: the FP64 update; the workgroup: the partition cursors
  // of a record whose split became final; wave 0: results + arrival
  __shared__ int s_fin;
  __shared__ uint64_t s_tot[kEpiBlock / 64];
  if (threadIdx.x == 0) {
    int fin = 0;
    if (!skip) {
      const uint32_t local_new = (uint32_t)own_new;
      if (MODE == TOT_ALLREDUCE) {
        const uint64_t* g = a.tot + (size_t)(blockIdx.x / a.nshard) * 8;
        for (int k = 0; k < F_NUM; ++k) tot[k] = g[k];
      }
      fin = node_update<KIND>(w, &sres, tot, a.fixed_point != 0) ? 1 : 0;
      if (fin) {
        for (int c = 0; c < 3; ++c) { sres.tm[c] = w->tm[c]; sres.tv[c] = w->tv[c]; }
        w->n_new_local = local_new;
        sres.n_new_local = local_new;
        sres.done_it = w->done_it;
      }
    }
    s_fin = fin;
  }
  __syncthreads();
  if (!skip && threadIdx.x < (uint32_t)kW16)   // the updated record back (read by later launches)
    ((g_u4*)gw)[threadIdx.x] = reinterpret_cast<const u32x4*>(&sw)[threadIdx.x];
  const bool final_results = s_fin != 0;
  if ((kMeans || KIND == PASS_SPLIT) && final_results) {
    if (stage_wp) block_cursors<kEpiBlock>(a.tiles, s_wp, tb, te, s_tot, tb);
    else block_cursors<kEpiBlock>(a.tiles, a.wparts, tb, te, s_tot);
  }
  if (wave_id() != 0) return;
  if (kMeans || KIND == PASS_SPLIT) {   // (split: proven fixed points, status slot max_iters)
    if ((a.debug & kDebugUneven) && debug_unlucky(blockIdx.x)) debug_sleep_us(10);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (final_results)
      store_result(a.hres + blockIdx.x, a.dres ? a.dres + blockIdx.x : nullptr, sres, lane, w->len, a.seq,
                   a.rsum ? a.rsum + blockIdx.x : nullptr, w);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      arrive(a.ctr + a.it, blockIdx.x, (uint32_t)a.nn, !skip && !final_results, a.hstat + a.it, a.seq);
  }
}

// ---------------------------------------------------------------------------
// 2-means pass with its epilogue fused: pass_kernel's sweep, then the LOGICAL
// node's last workgroup to finish (over the tiles of all its shard records)
// runs the node's epilogue in one wave: the node's totals, then lane s the
// FP64 update of shard record s (every record on the same totals, so all
// agree bit for bit), each record's partition cursors, results and arrival --
// exactly epilogue_kernel<KIND, TOT_OWN / TOT_NODE> for the records.  With
// TOT_ALLREDUCE the wave only writes the node's totals of this process to
// a.tot; the allreduce and epilogue_kernel<KIND, TOT_ALLREDUCE> follow.
// Partials and per-wave counts: see the hand-off comment in kpass_kernel.
// it_arr: the launch counter / status slot the records arrive on; final_only:
// arrive only once final (kpersist_kernel: every record arrives once, on the
// counter of iteration max_iters - 1).
template <int KIND>
__device__ __forceinline__ void kmeans_epilogue_wave(const RoundArgs& a, int node, NodeResult* sres, int it_arr,
                                                     bool final_only) {
  const int S = a.nshard, r0 = node * S;
  const uint32_t lane = lane_id();
  const uint32_t* pp = reinterpret_cast<const uint32_t*>(a.parts);
  uint64_t tot[F_NUM] = {0, 0, 0, 0, 0, 0, 0};
  uint32_t my_new = 0;   // lane s: shard record s's own new-side count
  for (int sh = 0; sh < S; ++sh) {
    const DevNode* w = a.nodes + r0 + sh;
    const int tb = w->tile_begin, te = w->tile_end;
    uint64_t acc[F_NUM] = {0, 0, 0, 0, 0, 0, 0};
    for (int i = tb + (int)lane; i < te; i += 64)
#pragma unroll
      for (int k = 0; k < F_NUM; ++k)
        acc[k] += __hip_atomic_load(pp + (size_t)i * 8 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int k = 0; k < F_NUM; ++k) {
      const uint64_t v = wave_sum_u64(acc[k]);
      tot[k] += v;
      if (k == F_CNT && lane == (uint32_t)sh) my_new = (uint32_t)v;
    }
  }
  if (a.tot_mode == TOT_ALLREDUCE) {   // this process's node totals, for the allreduce
    if (lane < (uint32_t)F_NUM + 1) {
      uint64_t v = 0;
#pragma unroll
      for (int k = 0; k < F_NUM; ++k) v = lane == (uint32_t)k ? tot[k] : v;
      a.tot[(size_t)node * 8 + lane] = v;
    }
    return;
  }
  int fin = 0;
  if (lane < (uint32_t)S) {
    DevNode* w = a.nodes + r0 + lane;
    NodeResult* r = sres + lane;
    fin = node_update<KIND>(w, r, tot, a.fixed_point != 0) ? 1 : 0;
    if (fin) {
      for (int c = 0; c < 3; ++c) { r->tm[c] = w->tm[c]; r->tv[c] = w->tv[c]; }
      w->n_new_local = my_new;
      r->n_new_local = my_new;
      r->done_it = w->done_it;
    }
  }
  const bool final_results = __shfl(fin, 0, 64) != 0;   // (every record of the node agrees)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (final_results) {
    for (int sh = 0; sh < S; ++sh) {
      const DevNode* w = a.nodes + r0 + sh;
      record_cursors<true>(a.tiles, a.wparts, w->tile_begin, w->tile_end, lane);
      store_result(a.hres + r0 + sh, a.dres ? a.dres + r0 + sh : nullptr, sres[sh], lane, w->len, a.seq,
                   a.rsum ? a.rsum + r0 + sh : nullptr, w);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane < (uint32_t)S && (final_results || !final_only))
    arrive(a.ctr + it_arr, (uint32_t)(r0 + lane), (uint32_t)a.nn, !final_results, a.hstat + it_arr, a.seq);
}

template <int KIND>
__global__ __launch_bounds__(kBlock, kPassWaves) void kpass_kernel(RoundArgs a) {
  const Tile t = a.tiles[blockIdx.x];
  const int rec = t.node;
  const int S = a.nshard;
  const int node = S == 1 ? rec : rec / S;
  const DevNode& nd = a.nodes[rec];
  if (nd.done_it != 0) {   // final in an earlier launch: its first tile arrives for it
    if (a.tot_mode != TOT_ALLREDUCE && (int)blockIdx.x == nd.tile_begin && threadIdx.x == 0)
      arrive(a.ctr + a.it, (uint32_t)rec, (uint32_t)a.nn, false, a.hstat + a.it, a.seq);
    return;   // (TOT_ALLREDUCE: the epilogue kernel arrives for every record)
  }
  const Params q = nd.prm;
  __shared__ uint32_t red[kBlock / 64][8];
  __shared__ int slast;
  __shared__ NodeResult sres[kMaxShard];
  LaneSums s;
  uint32_t ws, we;
  wave_range(t.start, t.end, wave_id(), ws, we);
  if (nd.planar == SRC_PLANAR) wave_pass<KIND, true>(nd.src, a.plane, ws, we, q, s);
  else if (nd.planar == SRC_BGR24) wave_pass<KIND, true, true>(nd.src, a.plane, ws, we, q, s);
  else wave_pass<KIND, false>(nd.src, a.plane, ws, we, q, s);
  uint32_t f[8] = {s.cnt, s.sr, s.sg, s.sb, s.qr, s.qg, s.qb, 0};
#pragma unroll
  for (int k = 0; k < F_NUM; ++k) f[k] = wave_sum_u32(f[k]);
  const uint32_t vsum = wave_sum_u32(s.vcnt);
  if (a.debug & kDebugPrewarm) {   // (tests) the node's hand-off lines into this CU's caches
    const uint32_t* pp = reinterpret_cast<const uint32_t*>(a.parts);
    const int tb0 = a.nodes[node * S].tile_begin, te0 = a.nodes[node * S + S - 1].tile_end;
    uint32_t x = 0;
    for (int i = tb0 + (int)lane_id(); i < te0; i += 64) {
      for (int k = 0; k < 8; ++k) x += pp[(size_t)i * 8 + k];
      for (int k = 0; k < 8; ++k) x += __hip_atomic_load(pp + (size_t)i * 8 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int ww = 0; ww < kTileWaves; ++ww) x += a.wparts[(size_t)i * kTileWaves + ww];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(x) : "memory");
  }
  if ((a.debug & kDebugUneven) && debug_unlucky(blockIdx.x)) debug_sleep_us(10);
  if (lane_id() == 0) {
    __hip_atomic_store(a.wparts + blockIdx.x * kTileWaves + wave_id(),
                       (vsum - f[F_CNT]) | (f[F_CNT] << 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int k = 0; k < 8; ++k) red[wave_id()][k] = k < F_NUM ? f[k] : 0u;
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    uint32_t x = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) x += red[w][threadIdx.x];
    __hip_atomic_store(a.parts[blockIdx.x].f + threadIdx.x, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // Hand-off to the node's last arriver (the gfx950 agent-
  // scope protocol of MI355X_MICROARCH.md "inter-workgroup visibility"):
  //   producer (every workgroup): the partial and the per-wave counts are
  //     write-through (sc1) stores; EVERY wave drains them (asm vmcnt(0):
  //     __syncthreads() alone emits no wait) before the workgroup's one
  //     arrival (lane 0, behind the barrier), an agent-scope RELEASE add:
  //     the ordering is then the language's, not only the ISA's (its
  //     buffer_wbl2 costs ~0.6 us per launch, +4 %, measured round 4);
  //   consumer (the workgroup whose add returns count - 1): an agent-scope
  //     ACQUIRE (buffer_inv sc1) before any load of the handed-off lines, so
  //     no copy this CU's L1 or its XCD's L2 holds from before the stores
  //     is read (kDebugPrewarm plants exactly such copies; tests/
  //     test_gpu_handoff.py).  Only the acquiring wave reads.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int ntiles = S == 1 ? nd.tile_end - nd.tile_begin
                              : a.nodes[node * S + S - 1].tile_end - a.nodes[node * S].tile_begin;
    const bool last = __hip_atomic_fetch_add(a.rdone + (size_t)a.it * a.nn + node, 1u, __ATOMIC_RELEASE,
                                             __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)ntiles - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    slast = last;
  }
  __syncthreads();
  if (slast && wave_id() == 0) kmeans_epilogue_wave<KIND>(a, node, sres, a.it, false);
}

// ---------------------------------------------------------------------------
// Every 2-means iteration of a round in ONE launch over the round's tiles
// (one workgroup per tile, as kpass_kernel).  Each workgroup
// keeps its own LDS copy of its record and loops over the iterations: it
// sweeps its tile with the copy's decision, stores its partial (write-
// through; partials alternate between two buffers by iteration parity) and
// its per-wave counts, drains them and makes one agent-scope RELEASE add on
// rdone[it][record]; then it waits until the word counts every tile of the
// record (the add that returns ntiles - 1 needs no wait), acquires, sums the
// record's partials itself and runs node_update on its copy -- the same
// function on the same exact integer sums in every workgroup, so every copy
// takes the same decision, fixed point and result as kpass's single
// epilogue.  No second hand-off per iteration: each workgroup computes what
// a last arriver would have published.  When the record is final, the
// workgroup of its first tile writes the record back, the partition cursors
// (this iteration's per-wave counts), the results and the record's one
// arrival on the counter of iteration max_iters - 1 (kloop_kernel's status
// contract); the others exit.  A workgroup reads the partials of iteration
// it after the record's workgroups all stored them, and it overwrites its
// own buffer of that parity only at it + 2, after every workgroup arrived at
// it + 1 -- which each does after its reads of iteration it.
// Waits only on the record's own workgroups, which all arrive before they
// wait: no cycle.  Eligible rounds (Engine::persist_ok) have at most as many
// active records' tiles as the GPU holds resident workgroups, so a record's
// workgroups are co-resident even if none of its round exits; every wait is
// bounded (a record's workgroups give up after ~2^26 polls and leave its
// status unset: the host's wait then reports the stream drained without it).
constexpr uint32_t kPersistSpin = 1u << 26;

// A Params copy in LDS read into SGPRs (wave-uniform: every lane holds the
// same bytes).
__device__ __forceinline__ Params uniform_params(const Params& p) {
  Params q;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&p);
  uint32_t* d = reinterpret_cast<uint32_t*>(&q);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(Params) / 4); ++i) d[i] = (uint32_t)__builtin_amdgcn_readfirstlane(s[i]);
  return q;
}

__global__ __launch_bounds__(kBlock, kPassWaves) void kpersist_kernel(RoundArgs a, int32_t max_iters) {
  typedef __attribute__((address_space(1))) u32x4 g_u4;
  const Tile t = a.tiles[blockIdx.x];
  const int rec = t.node;   // (one shard per record: S == 1, TOT_OWN)
  DevNode* gw = a.nodes + rec;
  const uint32_t lane = lane_id();
  __shared__ __attribute__((aligned(16))) DevNode sw;   // this workgroup's copy of the record
  __shared__ NodeResult sres;
  __shared__ uint32_t red[kBlock / 64][8];
  __shared__ int sgo, sfin;
  static_assert(sizeof(DevNode) % 16 == 0, "the record is staged in 16-B words");
  constexpr int kW16 = (int)(sizeof(DevNode) / 16);
  if (threadIdx.x < (uint32_t)kW16) reinterpret_cast<u32x4*>(&sw)[threadIdx.x] = ((const g_cu4*)gw)[threadIdx.x];
  __syncthreads();
  const int tb = sw.tile_begin, te = sw.tile_end;
  const int ntiles = te - tb;
  const bool lead = (int)blockIdx.x == tb;   // the record's first tile: its final stores
  if (sw.done_it != 0) {   // final at its split: its first tile arrives for it
    if (lead && threadIdx.x == 0)
      arrive(a.ctr + (max_iters - 1), (uint32_t)rec, (uint32_t)a.nn, false, a.hstat + (max_iters - 1), a.seq);
    return;
  }
  const uintptr_t srcw = (uintptr_t)sw.src;   // (each half through uint32_t: readfirstlane returns int)
  const uint8_t* src = (const uint8_t*)(((uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(srcw >> 32)) << 32) |
                                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)srcw));
  for (int it = 0; it < max_iters; ++it) {
    const bool klast = it == max_iters - 1;
    TilePartial* parts = (it & 1) ? a.parts2 : a.parts;
    const Params q = uniform_params(sw.prm);   // (this iteration's decision)
    LaneSums s;
    uint32_t ws, we;
    wave_range(t.start, t.end, wave_id(), ws, we);
    wave_pass<PASS_KMEANS, true>(src, a.plane, ws, we, q, s);
    uint32_t f[8] = {s.cnt, s.sr, s.sg, s.sb, s.qr, s.qg, s.qb, 0};
#pragma unroll
    for (int k = 0; k < F_NUM; ++k) f[k] = wave_sum_u32(f[k]);
    const uint32_t vsum = wave_sum_u32(s.vcnt);
    if (lane == 0) {
      __hip_atomic_store(a.wparts + blockIdx.x * kTileWaves + wave_id(),
                         (vsum - f[F_CNT]) | (f[F_CNT] << 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int k = 0; k < 8; ++k) red[wave_id()][k] = k < F_NUM ? f[k] : 0u;
    }
    __syncthreads();
    if (threadIdx.x < 8) {
      uint32_t x = 0;
#pragma unroll
      for (int w = 0; w < kBlock / 64; ++w) x += red[w][threadIdx.x];
      __hip_atomic_store(parts[blockIdx.x].f + threadIdx.x, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if ((a.debug & kDebugUneven) && debug_unlucky(blockIdx.x + 131u * (uint32_t)it)) debug_sleep_us(10);
    if ((a.debug & kDebugPrewarm) && wave_id() == 0) {   // (tests) the record's partials into this CU's caches
      const uint32_t* pp = reinterpret_cast<const uint32_t*>(parts);
      uint32_t x = 0;
      for (int i = tb + (int)lane; i < te; i += 64)
        for (int k = 0; k < 8; ++k) x += pp[(size_t)i * 8 + k];
      asm volatile("s_waitcnt vmcnt(0)" ::"v"(x) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (kpass_kernel's hand-off)
    __syncthreads();
    uint32_t* word = a.rdone + (size_t)it * a.nn + rec;
    if (threadIdx.x == 0) {
      int go = 1;
      if (__hip_atomic_fetch_add(word, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) != (uint32_t)ntiles - 1u) {
        for (uint32_t spin = 0;
             __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (uint32_t)ntiles; ++spin) {
          if (spin == kPersistSpin) {   // (never in a correct run: the record's status stays unset)
            go = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      sgo = go;
    }
    __syncthreads();
    if (!sgo) return;
    // every workgroup: the record's totals, the FP64 update on its copy
    if (wave_id() == 0) {
      const uint32_t* pp = reinterpret_cast<const uint32_t*>(parts);
      uint64_t tot[F_NUM] = {0, 0, 0, 0, 0, 0, 0};
      for (int i = tb + (int)lane; i < te; i += 64)
#pragma unroll
        for (int k = 0; k < F_NUM; ++k)
          tot[k] += __hip_atomic_load(pp + (size_t)i * 8 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int k = 0; k < F_NUM; ++k) tot[k] = wave_sum_u64(tot[k]);
      if (lane == 0) {
        const bool fin = klast ? node_update<PASS_KLAST>(&sw, &sres, tot, a.fixed_point != 0)
                               : node_update<PASS_KMEANS>(&sw, &sres, tot, a.fixed_point != 0);
        if (fin) {
          for (int c = 0; c < 3; ++c) { sres.tm[c] = sw.tm[c]; sres.tv[c] = sw.tv[c]; }
          sw.n_new_local = (uint32_t)tot[F_CNT];
          sres.n_new_local = (uint32_t)tot[F_CNT];
          sres.done_it = sw.done_it;
        }
        sfin = fin ? 1 : 0;
      }
    }
    __syncthreads();
    if (sfin) {   // (uniform; PASS_KLAST finalises every record)
      if (lead && wave_id() == 0) {   // the record, its cursors, results and arrival
        if (lane < (uint32_t)kW16) ((g_u4*)gw)[lane] = reinterpret_cast<const u32x4*>(&sw)[lane];
        record_cursors<true>(a.tiles, a.wparts, tb, te, lane);
        store_result(a.hres + rec, a.dres ? a.dres + rec : nullptr, sres, lane, sw.len, a.seq,
                     a.rsum ? a.rsum + rec : nullptr, &sw);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0)
          arrive(a.ctr + (max_iters - 1), (uint32_t)rec, (uint32_t)a.nn, false, a.hstat + (max_iters - 1), a.seq);
      }
      return;
    }
  }
}

// ---------------------------------------------------------------------------
// Fused partition + split pass over the tiles of parents split in an earlier
// round (replaces the reference's per-split O(N) member[] gather, :894-1026,
// and the children's split pass, :438-559).  Replays the parent's final
// 2-means decision (bit-identical inputs -> bit-identical outcome), writes
// OLD points to [off, off+n_old) and NEW points to [off+n_old, off+len) of
// the child buffer, and accumulates each child's split-pass statistics
// (cut_pos < v_axis -> the child's new side) from the same registers.
//
// Every wave works alone: its share of the tile (the same points the final
// 2-means pass gave it) starts at the cursors the finalising epilogue scanned
// from that pass's per-wave counts (Tile::old_base / new_base).  Per sweep:
// decisions into lane bit masks (FP64 only on a wave-uniform branch for
// near-plane points), then per slot one ballot-ranked store of the wave's
// points into the old or the new run (each store instruction covers at most
// two contiguous runs of the child buffer), with the next sweep's loads in
// flight.  No LDS and no barrier until the final reduction of the sums.
// Two 32-B partials per tile: the old child's (count, sums, sums of squares),
// then the new child's; the children's per-(tile, wave) split counts go to
// wparts (chunk_run).
// A child's split-pass (old, new) counts per (tile, wave) of the CHILD's
// tiling, from the run of the child buffer one partsplit wave writes (its
// positions only grow, sweep after sweep).  A "chunk" is one wave range of a
// child tile (wave_range): at least kWaveSweep points, except the segment's
// last non-empty one, which ends where the segment does -- so the <= 1024
// points a sweep writes to a child cross at most one chunk end.  The wave
// keeps the chunk it is in (wave-uniform), counts its points as old in
// `acc` (old | new << 16) and the new ones per lane in `lnew`, and adds acc
// with one atomic when it leaves the chunk.
struct ChunkAcc {
  bool on;                // the child is split this round
  uint32_t off, len, tl;  // its segment and tile length
  uint32_t* w0;           // its first tile's wave words in wparts
  uint32_t k, t0, tend, q;// current child tile, its range, its wave range size
  uint32_t w, end;        // current wave range and its end
  uint32_t acc;
  uint32_t lnew;          // per LANE: new points of the chunk not yet in acc
};

__device__ __forceinline__ void chunk_tile(ChunkAcc& c) {
  c.t0 = c.off + c.k * c.tl;
  c.tend = min(c.t0 + c.tl, c.off + c.len);
  c.q = ((c.tend - c.t0 + kSweep - 1) / kSweep) * kWaveSweep;
}

// A child's segment and tiling (its record's off, len, tile_len and
// tile_begin): what the partition's per-(tile, wave) counts need of it.
struct ChildInfo {
  uint32_t off, len, tl, tb;
  int32_t on;               // the child is split this round
};

__device__ __forceinline__ ChildInfo child_info(const DevNode* nodes, int rec) {
  const DevNode* ch = nodes + (rec >= 0 ? rec : 0);
  ChildInfo c;
  c.on = rec >= 0;
  c.off = ch->off;
  c.len = ch->len;
  c.tl = ch->tile_len;
  c.tb = (uint32_t)ch->tile_begin;
  return c;
}

// (plain values: a `const RoundArgs&` parameter made the kernel argument
// addressable and cost partsplit ~80 VGPRs).  Enters the chunk holding p,
// the wave's first position in the child.
__device__ __forceinline__ void chunk_init(ChunkAcc& c, const ChildInfo& ci, uint32_t* wparts, uint32_t p) {
  c.on = ci.on != 0;
  c.off = ci.off;
  c.len = ci.len;
  c.tl = ci.tl;
  c.w0 = wparts + (size_t)ci.tb * kTileWaves;
  c.acc = c.lnew = 0;
  c.k = c.w = 0;
  if (c.on && p < c.off + c.len) {
    c.k = (p - c.off) / c.tl;
    chunk_tile(c);
    c.w = (p - c.t0) / c.q;
    c.end = min(c.t0 + (c.w + 1u) * c.q, c.tend);
  } else {
    c.end = 0xFFFFFFFFu;   // writes nothing to this child
  }
}

// Leave the chunk: fold the lanes' new counts into acc, add acc, step to
// the next chunk (next wave range, or the next tile's first).
__device__ __forceinline__ void chunk_next(ChunkAcc& c) {
  const uint32_t nn = wave_sum_u32(c.lnew);
  const uint32_t v = c.acc + (nn << 16) - nn;
  if (v != 0 && lane_id() == 0) atomicAdd(c.w0 + c.k * kTileWaves + c.w, v);
  c.acc = 0;
  c.lnew = 0;
  if (c.end == c.tend) {
    c.k += 1;
    chunk_tile(c);
    c.w = 0;
  } else {
    c.w += 1;
  }
  c.end = min(c.t0 + (c.w + 1u) * c.q, c.tend);
}

__device__ __forceinline__ void chunk_finish(ChunkAcc& c) {
  if (!c.on) return;
  const uint32_t nn = wave_sum_u32(c.lnew);
  const uint32_t v = c.acc + (nn << 16) - nn;
  if (v != 0 && lane_id() == 0) atomicAdd(c.w0 + c.k * kTileWaves + c.w, v);
}

// Occupancy of partsplit: 4 waves per SIMD (LDS staging 25 KB per
// workgroup, <= 128 VGPRs).
// partsplit works on byte masks: word j of a SweepMask holds 0x01 in byte e
// iff slot 4j + e is in the set -- the 0/1 byte weights v_dot4 sums with,
// and what the SWAR cut comparison produces (partsplit was VALU-bound with
// per-slot bit masks: ~69 VALU per point, the cuts alone 19).
struct SweepMask {
  uint32_t m[kVecPerThread];
};

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}

// Bytes of x that are >= thr, as 0x01 bytes; k = (256 - thr) * 0x00010001,
// thr in [0, 256].  Bytes 0, 2 and 1, 3 spread into 16-bit lanes; b + 256 -
// thr < 512 sets bit 8 iff b >= thr.
__device__ __forceinline__ uint32_t ge_bytes(uint32_t x, uint32_t k) {
  const uint32_t lo = pk_add_u16(__builtin_amdgcn_perm(0u, x, 0x0C020C00u), k);   // b0, b2
  const uint32_t hi = pk_add_u16(__builtin_amdgcn_perm(0u, x, 0x0C030C01u), k);   // b1, b3
  return __builtin_amdgcn_perm(hi, lo, 0x07030501u) & 0x01010101u;
}

// Word j of the cut axis' channel (shift 16: R, 8: G, 0: B) by two v_perm_b32
// with uniform selectors (a select between the channel arrays is compiled as
// an indexed access through scratch memory).
__device__ __forceinline__ uint32_t axis_word(const Sweep& w, int j, uint32_t shift) {
  const uint32_t s1 = shift == 8u ? 0x07060504u : 0x03020100u;   // R or G
  const uint32_t s2 = shift == 0u ? 0x07060504u : 0x03020100u;   // that or B
  return __builtin_amdgcn_perm(w.b[j], __builtin_amdgcn_perm(w.g[j], w.r[j], s1), s2);
}

// Slots whose byte on the cut axis is >= thr: the split pass's NEW side.
__device__ __forceinline__ SweepMask cut_new_bytes(const Sweep& w, uint32_t shift, int32_t thr) {
  const uint32_t k = (uint32_t)(256 - thr) * 0x00010001u;
  SweepMask m;
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) m.m[j] = ge_bytes(axis_word(w, j, shift), k);
  return m;
}

__device__ __forceinline__ SweepMask bits_to_bytes(uint32_t b16) {
  SweepMask m;
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) m.m[j] = ((((b16 >> (4 * j)) & 0xFu) * 0x204081u) & 0x01010101u);
  return m;
}

__device__ __forceinline__ bool slot_in(const SweepMask& m, int s) {
  return ((m.m[s >> 2] >> (8 * (s & 3))) & 0xFFu) != 0u;
}

__device__ __forceinline__ uint32_t mask_count(const SweepMask& m) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) c += (uint32_t)__builtin_popcount(m.m[j]);
  return c;
}

// Count (cnt: mask_count(m)), sums and sums of squares over the slots of a
// byte mask.
__device__ __forceinline__ void add_sums_bytes(const Sweep& w, const SweepMask& m, uint32_t cnt, SplitSums& s) {
  s.cnt += cnt;
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) {
    // 0x01 -> 0xFF per byte as a shift and a subtract: left alone the
    // compiler folds them into a quarter-rate v_mul_lo_u32 (x 0xFF)
    const uint32_t wt = m.m[j];
    uint32_t sh = wt << 8;
    asm("" : "+v"(sh));
    const uint32_t mk = sh - wt;
    s.sr = __builtin_amdgcn_udot4(w.r[j], wt, s.sr, false);
    s.sg = __builtin_amdgcn_udot4(w.g[j], wt, s.sg, false);
    s.sb = __builtin_amdgcn_udot4(w.b[j], wt, s.sb, false);
    s.qr = __builtin_amdgcn_udot4(w.r[j] & mk, w.r[j], s.qr, false);
    s.qg = __builtin_amdgcn_udot4(w.g[j] & mk, w.g[j], s.qg, false);
    s.qb = __builtin_amdgcn_udot4(w.b[j] & mk, w.b[j], s.qb, false);
  }
}

// ---------------------------------------------------------------------------
// LDS-staged stores: a wave writes each sweep's points as bytes into its own
// LDS staging -- per plane, one region per run (old / new) whose byte i is
// the child position cb + i, cb the 16-B aligned start of the run's first
// unwritten chunk -- then stores every completed 16-B chunk with one
// buffer_store_dwordx4 per plane and moves the partial last chunk to the
// front.  Versus one byte store per point and plane this cuts the vector-
// memory instructions of a sweep from 48 to ~3-6 (the address unit bounded
// the byte-store form: TA busy 81 %).  A chunk holding the run's first
// position (shared with the neighbouring wave's run) and the run's last
// partial chunk are written byte by byte.
constexpr uint32_t kStageRun = 1056;                // bytes per (wave, plane, run): 15 + 1024 + slack
constexpr uint32_t kStagePlane = 2 * kStageRun;     // old region, new region
constexpr uint32_t kStageWave = 3 * kStagePlane;

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct PlaneRsrc {
  __amdgpu_buffer_rsrc_t r, g, b;
};

// A buffer offset past every range (< 2^31 bytes + 64): the buffer range
// check drops the store / returns 0 for the load, so a lane opts out of an
// access without a branch.
constexpr uint32_t kOOB = 0xF0000000u;

// This lane's loads of the sweep at vs through buffer resources over the
// parent's segment (planar: the R, G, B planes; packed: the frame words in
// r), branch-free: vectors starting at or past `end` read kOOB (zeros).  A
// planar vector straddling `end` is loaded whole (16 B of slack per shard).
template <bool PLANAR, bool BGR = false>
__device__ __forceinline__ void fetch_sweep_rs(const PlaneRsrc& s, uint32_t vs, uint32_t end, RawSweep& x) {
  if (BGR) {   // 48 bytes at 3 i through the frame's resource (s.r)
    const uint32_t i = vs + 16u * lane_id();
    const int o = (int)(i < end ? 3u * i : kOOB);
#pragma unroll
    for (int c = 0; c < 3; ++c)
      x.v[c] = __builtin_amdgcn_raw_buffer_load_b128(s.r, o + 16 * c, 0, 0);
  } else if (PLANAR) {
    const uint32_t i = vs + 16u * lane_id();
    const int o = (int)(i < end ? i : kOOB);
    x.v[0] = __builtin_amdgcn_raw_buffer_load_b128(s.r, o, 0, 0);
    x.v[1] = __builtin_amdgcn_raw_buffer_load_b128(s.g, o, 0, 0);
    x.v[2] = __builtin_amdgcn_raw_buffer_load_b128(s.b, o, 0, 0);
  } else {
#pragma unroll
    for (int j = 0; j < kVecPerThread; ++j) {
      const uint32_t i = vs + 4u * (j * 64 + lane_id());
      x.v[j] = __builtin_amdgcn_raw_buffer_load_b128(s.r, (int)(i < end ? 4u * i : kOOB), 0,
                                                     0);
    }
  }
}

// A wave's two runs (wave-uniform): child position of staging byte 0, the
// next staging byte (the new run's region starts at kStageRun), the wave's
// first position.  The run's next child position is cb + p (- kStageRun).
struct Stage {
  uint32_t cbo, cbn, po, pn, loo, lon;
};

// This wave's points of one sweep into the staging, slot by slot, ranked by
// ballot (a full sweep: a lane's rank among the new points is its lane id
// minus its rank among the old ones).  Each run's positions are in slot-major
// order: slot s's points follow slot s-1's, by lane (run_below relies on it).
template <bool STORE = true>
__device__ __forceinline__ void stage_sweep(const Sweep& w, const SweepMask& om, const SweepMask& nm, bool full,
                                            uint8_t* st, Stage& g, uint32_t l) {
  constexpr int kSlots = kVecPerThread * 4;
  auto put = [&](int s, uint32_t lp) {
    const int j = s >> 2, sh = 8 * (s & 3);
    if (STORE) {   // (STORE false: the run positions only, for the children's counts)
      st[lp] = (uint8_t)(w.r[j] >> sh);
      st[kStagePlane + lp] = (uint8_t)(w.g[j] >> sh);
      st[2 * kStagePlane + lp] = (uint8_t)(w.b[j] >> sh);
    }
  };
  if (full) {   // (wave-uniform)
    const uint32_t po0 = g.po;
    uint32_t t = g.pn + l;
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      const bool o = slot_in(om, s);
      const uint64_t bo = __ballot(o);
      if (STORE) {
        const uint32_t ro = mbcnt64(bo);
        put(s, o ? g.po + ro : t - ro);
      }
      const uint32_t co = (uint32_t)__popcll(bo);
      g.po += co;
      t += 64u - co;
    }
    g.pn += (uint32_t)kWaveSweep - (g.po - po0);   // every slot valid: old + new = 1024
  } else {
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      const bool o = slot_in(om, s), n = slot_in(nm, s);
      const uint64_t bo = __ballot(o), bn = __ballot(n);
      if (STORE && (o || n)) put(s, o ? g.po + mbcnt64(bo) : g.pn + mbcnt64(bn));
      g.po += (uint32_t)__popcll(bo);
      g.pn += (uint32_t)__popcll(bn);
    }
  }
}

// Slots of a byte mask as lane bits (bit s = slot s): bytes 0x00 / 0x01 of
// word j -> bits 4j..4j+3 (the multiply moves byte e's bit to bit 24 + e,
// no carries).
__device__ __forceinline__ uint32_t bytes_to_bits(const SweepMask& m) {
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) b |= ((m.m[j] * 0x01020408u) >> 24) << (4 * j);
  return b;
}

// This lane's points of xb (a subset of its run members mb, bit s = slot s)
// among the first `rel` positions of the sweep's run (slot-major, lanes by
// rank within a slot: stage_sweep's order).  Only on sweeps whose run
// crosses a chunk end: the slot holding position rel - 1 is found by a scan
// of the slots' ballot counts (a uniform loop); below it every member
// counts, in it those of rank below the rest.  (Was a compare per slot and
// lane on every such sweep.)
__device__ __forceinline__ uint32_t run_below(uint32_t mb, uint32_t xb, uint32_t rel) {
  uint32_t cum = 0, ss = 0;
  uint64_t bs;
#pragma unroll 1
  for (;; ++ss) {   // (wave-uniform; rel < the run's count, so a slot holds position rel - 1)
    bs = __ballot((mb >> ss) & 1u);
    const uint32_t c = (uint32_t)__popcll(bs);
    if (rel <= cum + c || ss == kVecPerThread * 4 - 1) break;
    cum += c;
  }
  const uint32_t low = (uint32_t)__builtin_popcount(xb & ((1u << ss) - 1u));
  const bool in = ((xb >> ss) & 1u) != 0u && mbcnt64(bs) < rel - cum;
  return low + (in ? 1u : 0u);
}

// Book one sweep's points [p0, p1) of this child's run: mb = the lane's run
// members, xm = those on the child's split-new side, cnt = mask_count(xm).
__device__ __forceinline__ void chunk_sweep(ChunkAcc& c, uint32_t p0, uint32_t p1, const SweepMask& mb,
                                            const SweepMask& xm, uint32_t cnt) {
  if (!c.on) return;
  if (p1 <= c.end) {
    c.acc += p1 - p0;
    c.lnew += cnt;
    return;
  }
  const uint32_t before = c.end - p0;
  const uint32_t pre = run_below(bytes_to_bits(mb), bytes_to_bits(xm), before);
  c.acc += before;
  c.lnew += pre;
  chunk_next(c);
  c.acc = (p1 - p0) - before;
  c.lnew = cnt - pre;
}


// Lanes 0-15 / 16-31 write the staged bytes i of the old / new run's first
// chunk whose child positions lie in [max(cb, lo), hi).
__device__ __forceinline__ void stage_bytes(const uint8_t* st, const PlaneRsrc& d, const Stage& g,
                                            uint32_t hi_o, uint32_t hi_n, uint32_t l) {
  const uint32_t run = (l >> 4) & 1u, i = l & 15u;
  const uint32_t pos = (run ? g.cbn : g.cbo) + i;
  const uint32_t lo = run ? g.lon : g.loo, hi = run ? hi_n : hi_o;
  const uint32_t lp = run * kStageRun + i;   // (lanes 32-63 read a staged byte, store nothing)
  const uint32_t o = (l < 32u && pos >= lo && pos < hi) ? pos : kOOB;
  __builtin_amdgcn_raw_buffer_store_b8(st[lp], d.r, (int)o, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(st[kStagePlane + lp], d.g, (int)o, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(st[2 * kStagePlane + lp], d.b, (int)o, 0, 0);
}

// Chunk q of a flush (q < nfo: the old run's, else the new run's), stored by
// every lane: a lane with no chunk, or whose chunk starts below its run's
// first position (stage_bytes writes that one), stores at kOOB (dropped by
// the buffer range check).  No branch around the stores: the compiler's
// vmcnt bookkeeping then sees a fixed count of vector-memory operations per
// sweep and waits for the prefetched loads only (a data-dependent store
// count made every wait a vmcnt(0) that drained the sweep's stores too).
__device__ __forceinline__ void flush_chunk(const uint8_t* st, const PlaneRsrc& d, const Stage& g,
                                            uint32_t q, uint32_t nfo, uint32_t nf) {
  const bool run = q >= nfo;
  const uint32_t k16 = 16u * (run ? q - nfo : q);
  const uint32_t pos = (run ? g.cbn : g.cbo) + k16;
  const bool ok = q < nf && pos >= (run ? g.lon : g.loo);
  const uint32_t lp = ok ? (run ? kStageRun : 0u) + k16 : 0u;
  const uint32_t o = (ok) ? pos : kOOB;
  const u32x4 vr = *reinterpret_cast<const u32x4*>(st + lp);
  const u32x4 vg = *reinterpret_cast<const u32x4*>(st + kStagePlane + lp);
  const u32x4 vb = *reinterpret_cast<const u32x4*>(st + 2 * kStagePlane + lp);
  __builtin_amdgcn_raw_buffer_store_b128(vr, d.r, (int)o, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(vg, d.g, (int)o, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(vb, d.b, (int)o, 0, 0);
}

// After a sweep: the completed chunks of both runs (at most 65: <= 15 + 15
// staged bytes before the sweep + its 1024), then the partial chunks moved to
// the front of their regions.
__device__ __forceinline__ void stage_flush(uint8_t* st, const PlaneRsrc& d, Stage& g, uint32_t l) {
  wave_lds_sync();
  const uint32_t nfo = g.po >> 4, nfn = (g.pn - kStageRun) >> 4;
  const uint32_t nf = nfo + nfn;
  flush_chunk(st, d, g, l, nfo, nf);
  // (the rare second chunk row and the first chunks' bytes below are stored
  // unconditionally -- at kOOB when there is nothing to store -- so every
  // sweep issues the same count of vector-memory operations and the next
  // sweep's wait for its loads need not drain these stores)
  flush_chunk(st, d, g, 64u + l, nfo, nf);
  // a completed first chunk that starts below the wave's first position
  const uint32_t ho = (nfo > 0u && g.cbo < g.loo) ? g.cbo + 16u : 0u;
  const uint32_t hn = (nfn > 0u && g.cbn < g.lon) ? g.cbn + 16u : 0u;
  stage_bytes(st, d, g, ho, hn, l);
  if (nfo | nfn) {   // the partial chunks to the front
    const uint32_t run = (l >> 4) & 1u, i = l & 15u;
    const uint32_t nf = run ? nfn : nfo;
    const uint32_t src = (run ? kStageRun : 0u) + 16u * nf + i;
    const bool mv = l < 32u && nf > 0u;
    uint8_t cr = 0, cg = 0, cb = 0;
    wave_lds_sync();
    if (mv) {
      cr = st[src];
      cg = st[kStagePlane + src];
      cb = st[2 * kStagePlane + src];
    }
    wave_lds_sync();
    if (mv) {
      const uint32_t dst = (run ? kStageRun : 0u) + i;
      st[dst] = cr;
      st[kStagePlane + dst] = cg;
      st[2 * kStagePlane + dst] = cb;
    }
    g.cbo += 16u * nfo;
    g.po -= 16u * nfo;
    g.cbn += 16u * nfn;
    g.pn -= 16u * nfn;
  }
  wave_lds_sync();
}

typedef uint8_t StageMem;

// The kernel's loop for one source format of the parent.
// (records and tiles through global-address-space views: generic pointers
// read from a PartTile made these flat loads)
typedef const __attribute__((address_space(1))) DevNode g_cnode;
typedef const __attribute__((address_space(1))) Tile g_ctile;
template <bool PLANAR, bool BGR, int MODE>
__device__ __forceinline__ void partsplit_run(const PartTile& pt, g_cnode& nd, g_ctile* tp,
                                              const ChildInfo& ci0, const ChildInfo& ci1, uint32_t* wparts,
                                              uint64_t plane, StageMem* st, SplitSums& so, SplitSums& sn) {
  const uint32_t w = wave_id(), l = lane_id();
  uint32_t start, end;   // this wave's range of the parent tile (wave-uniform)
  wave_range(__builtin_amdgcn_readfirstlane(tp->start), __builtin_amdgcn_readfirstlane(tp->end), w, start, end);
  // the child's planes of the frame shard: every index < off + len < 2^30
  const int nrec = (int)(nd.off + nd.len);
  PlaneRsrc d;
  d.r = __builtin_amdgcn_make_buffer_rsrc(nd.dst, (short)0, nrec, 0x00020000);
  d.g = __builtin_amdgcn_make_buffer_rsrc(nd.dst + plane, (short)0, nrec, 0x00020000);
  d.b = __builtin_amdgcn_make_buffer_rsrc(nd.dst + 2 * plane, (short)0, nrec, 0x00020000);
  Params q;   // (field by field: an address-space-qualified struct has no copy for the host pass)
  q.lhs = nd.prm.lhs;
  q.rr = nd.prm.rr;
  q.rg = nd.prm.rg;
  q.rb = nd.prm.rb;
  q.lhsf = nd.prm.lhsf;
  q.rrf = nd.prm.rrf;
  q.rgf = nd.prm.rgf;
  q.rbf = nd.prm.rbf;
  q.eps = nd.prm.eps;
  q.thr = nd.prm.thr;
  q.shift = nd.prm.shift;
  q.pad = 0;
  const uint32_t n_old = nd.len - nd.n_new_local;
  const uint32_t oc0 = nd.off + tp->old_base[w];
  const uint32_t nc0 = nd.off + n_old + tp->new_base[w];
  const bool exact_all = !(q.eps < __builtin_inff());   // FP32 filter off for this node
  const bool cut = nd.proven != 0;
  const uint32_t sh0 = (uint32_t)pt.shift[0], sh1 = (uint32_t)pt.shift[1];
  const int32_t thr0 = pt.thr[0], thr1 = pt.thr[1];
  constexpr bool kStore = MODE != PS_STATS, kSums = MODE == PS_FULL || MODE == PS_STATS;
  // the children's per-(tile, wave) counts (their partition cursors): PS_FULL
  // only.  A PS_STATS round is a frame's last planned one; the few of its
  // records a later host round partitions get theirs then (launch_fix_cursors)
  // -- the walk cost PS_STATS a third of its time.
  constexpr bool kCounts = MODE == PS_FULL;
  ChunkAcc cx, cy;
  ChildInfo off{0u, 0u, 1u, 0u, 0};
  chunk_init(cx, kCounts ? ci0 : off, wparts, oc0);
  chunk_init(cy, kCounts ? ci1 : off, wparts, nc0);
  Stage g;
  constexpr uint32_t kPnOff = kStageRun;
  g.cbo = oc0 & ~15u;
  g.po = oc0 & 15u;
  g.loo = oc0;
  g.cbn = nc0 & ~15u;
  g.pn = kPnOff + (nc0 & 15u);
  g.lon = nc0;

  // the parent's segment (hoisted: a pointer read from the record inside the
  // loop was re-loaded every sweep behind a vmcnt(0))
  PlaneRsrc s;
  {
    const uint8_t* src = nd.src;
    const uint32_t ext = nd.off + nd.len;
    if (BGR) {
      // a 16-B load is dropped whole when any byte of it is out of range: the
      // range covers a straddling vector's 48 bytes (a frame whose size is not
      // a multiple of 16 points is an aligned copy with >= 48 B of slack; a
      // caller's frame that is one has no vector past its end)
      s.r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)(3u * ext + 48u), 0x00020000);
      s.g = s.b = s.r;
    } else if (PLANAR) {
      const int nb = (int)(ext + 16u);   // (16 B of slack after every shard)
      s.r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nb, 0x00020000);
      s.g = __builtin_amdgcn_make_buffer_rsrc((void*)(src + plane), (short)0, nb, 0x00020000);
      s.b = __builtin_amdgcn_make_buffer_rsrc((void*)(src + 2 * plane), (short)0, nb, 0x00020000);
    } else {
      s.r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)(4u * ext), 0x00020000);
      s.g = s.b = s.r;
    }
  }
  RawSweep xn;
  uint32_t vs = start & ~15u;
  bool full = vs >= start && vs + kWaveSweep <= end;
  fetch_sweep_rs<PLANAR, BGR>(s, vs, end, xn);
  // the vector-memory operations a sweep issues after its loads, here as
  // no-ops (kOOB): the loop's top then waits for the previous loads only,
  // entered from here or from the previous sweep alike
  if (kStore) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){0u, 0u, 0u, 0u}, d.r, (int)kOOB, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){0u, 0u, 0u, 0u}, d.g, (int)kOOB, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){0u, 0u, 0u, 0u}, d.b, (int)kOOB, 0, 0);
    }
  }
  while (vs < end) {
    // this sweep's points: a copy of the loads issued one sweep ago, made
    // HERE (the asm makes x a value of its own): left to the compiler, the
    // loop-carried copy sat at the end of the sweep and waited there for the
    // loads the sweep had just issued, exposing the memory latency per sweep
    // (2 sweeps of loads in flight measured no faster, tools/psbench)
    RawSweep x = xn;
    asm volatile("" : "+v"(x.v[0]), "+v"(x.v[1]), "+v"(x.v[2]), "+v"(x.v[3]));
    const uint32_t nvs = vs + kWaveSweep;
    const bool nfull = nvs + kWaveSweep <= end;
    // the next sweep's loads in flight during this one (past the end: kOOB,
    // no memory access -- a fixed load count per sweep)
    fetch_sweep_rs<PLANAR, BGR>(s, nvs, end, xn);
    Sweep sw;
    unpack_sweep<PLANAR, BGR>(x, sw);
    // the parent's final decision: its cut when proven, else its last 2-means plane
    SweepMask om, nm;
    if (full) {
      if (cut) {
        nm = cut_new_bytes(sw, (uint32_t)q.shift, q.thr);
#pragma unroll
        for (int j = 0; j < kVecPerThread; ++j) om.m[j] = nm.m[j] ^ 0x01010101u;
      } else {
        om = bits_to_bytes(old_mask(sw, 0xFFFFu, q, exact_all));
#pragma unroll
        for (int j = 0; j < kVecPerThread; ++j) nm.m[j] = om.m[j] ^ 0x01010101u;
      }
    } else {
      const uint32_t validm = valid_mask<PLANAR>(vs, start, end);
      const uint32_t ob = cut ? validm & ~cut_new_mask(sw, (uint32_t)q.shift, q.thr)
                              : old_mask(sw, validm, q, exact_all);
      om = bits_to_bytes(ob);
      nm = bits_to_bytes(validm & ~ob);
    }
    // the children's split pass on the same registers (cut_pos < v_axis <=>
    // v_axis >= thr): each child's new-side slots, counted and summed
    SweepMask xm = cut_new_bytes(sw, sh0, thr0), ym = cut_new_bytes(sw, sh1, thr1);
#pragma unroll
    for (int j = 0; j < kVecPerThread; ++j) {
      xm.m[j] &= om.m[j];   // new for the old child
      ym.m[j] &= nm.m[j];   // new for the new child
    }
    const uint32_t xc = mask_count(xm), yc = mask_count(ym);
    if (kSums) {
      add_sums_bytes(sw, xm, xc, so);
      add_sums_bytes(sw, ym, yc, sn);
    }
    // this wave's points into the runs (PS_STATS: the run positions only --
    // the children's per-(tile, wave) counts are the partition cursors a
    // later round may need -- no stores)
    if (kStore || kCounts) {
      const uint32_t oc = g.cbo + g.po, nc = g.cbn + g.pn - kPnOff;
      stage_sweep<kStore>(sw, om, nm, full, st, g, l);
      chunk_sweep(cx, oc, g.cbo + g.po, om, xm, xc);
      chunk_sweep(cy, nc, g.cbn + g.pn - kPnOff, nm, ym, yc);
    }
    if (kStore) stage_flush(st, d, g, l);
    vs = nvs;
    full = nfull;
  }
  if (kStore) stage_bytes(st, d, g, g.cbo + g.po, g.cbn + g.pn - kStageRun, l);   // the runs' last partial chunks
  if (kCounts) {
    chunk_finish(cx);
    chunk_finish(cy);
  }
}

// One part tile's partition + children's split pass (pt: the parent's tile,
// record and children; ci0 / ci1: the children's segments and tiling).
// FMT: the source format of every parent of the launch (FMT_ANY: read from
// each record -- every path compiled into one kernel, whose register
// allocation is then the largest path's).
// The children's split totals of a parent whose part tiles this launch
// partitions, by the parent's last workgroup to finish (RoundArgs::sdone;
// TOT_ALLREDUCE with one shard: exactly nodesum_kernel<PASS_SPLIT>'s sums,
// without its launch).  Hand-off as kpass_kernel's: the partials (sparts,
// write-through stores) drained by every wave before the workgroup's one
// agent-scope release add; the last arriver acquires before it reads them.
// KOFF: the byte offset of the launch's RoundArgs in its kernarg segment --
// the arguments and the part tile are loaded again here, through a laundered
// pointer: kept live across the partition, they spilled its registers.
template <size_t KOFF>
__device__ __forceinline__ void split_totals_last(uint64_t (*red64)[8]) {
  typedef __attribute__((address_space(4))) const char* k_cp;
  k_cp kp = (k_cp)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(kp));
  RoundArgs a;
  __builtin_memcpy(&a, (const char*)kp + KOFF, sizeof(RoundArgs));
  if (!a.sdone) return;
  __shared__ int s_last;
  PartTile pt;
  {
    typedef const __attribute__((address_space(1))) u32x4 g_cu4_;
    static_assert(sizeof(PartTile) % 16 == 0, "16-B words");
    const g_cu4_* src = (const g_cu4_*)(a.ptiles + blockIdx.x);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(PartTile) / 16); ++i) reinterpret_cast<u32x4*>(&pt)[i] = src[i];
  }
  const int32_t key = pt.child[0] >= 0 ? pt.child[0] : pt.child[1];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const g_cnode& P = *(g_cnode*)pt.parent;
    const uint32_t nt = (uint32_t)(P.tile_end - P.tile_begin);   // the parent's part tiles
    const bool last = __hip_atomic_fetch_add(a.sdone + key, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) ==
                      nt - 1u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  for (int c = 0; c < 2; ++c) {
    const int32_t ch = pt.child[c];
    if (ch < 0) continue;   // (uniform: a child this round does not split)
    // (sum_record<PASS_SPLIT>'s fused-partials branch, through global pointers)
    const g_cnode& w = *(g_cnode*)(a.nodes + ch);
    const int side = w.split_side, pb = w.split_pb, pe = w.split_pe;
    const g_cu4* sp4 = (const g_cu4*)a.sparts;
    uint64_t acc[7] = {0, 0, 0, 0, 0, 0, 0}, tot[7];
    for (int i = pb + (int)threadIdx.x; i < pe; i += kBlock) {
      const u32x4 x = sp4[4 * i + 2 * side], y = sp4[4 * i + 2 * side + 1];
      acc[0] += x[0];
      acc[1] += x[1];
      acc[2] += x[2];
      acc[3] += x[3];
      acc[4] += y[0];
      acc[5] += y[1];
      acc[6] += y[2];
    }
    block_sum7(acc, red64, tot);   // (valid in thread 0)
    if (threadIdx.x == 0) {
      typedef __attribute__((address_space(1))) uint64_t g_u64;
      g_u64* g = (g_u64*)(a.tot + (size_t)ch * 8);   // (one shard: record = logical node)
      for (int k = 0; k < F_NUM; ++k) g[k] = tot[k];
      g[7] = 0;
    }
    __syncthreads();   // (red64 reused)
  }
}

template <int MODE, int FMT, size_t KOFF>
__device__ __forceinline__ void partsplit_tile(const RoundArgs& a, const PartTile& pt, const ChildInfo& ci0,
                                               const ChildInfo& ci1, uint8_t* stage, uint32_t (*red)[16]) {
  g_cnode& nd = *(g_cnode*)pt.parent;
  g_ctile* tp = (g_ctile*)pt.tile;
  SplitSums so, sn;
  StageMem* st = stage ? stage + wave_id() * kStageWave : nullptr;
  if (FMT == FMT_PLANAR || (FMT == FMT_ANY && nd.planar == SRC_PLANAR))
    partsplit_run<true, false, MODE>(pt, nd, tp, ci0, ci1, a.wparts, a.plane, st, so, sn);
  else if (FMT == FMT_BGR || (FMT == FMT_ANY && nd.planar == SRC_BGR24))
    partsplit_run<true, true, MODE>(pt, nd, tp, ci0, ci1, a.wparts, a.plane, st, so, sn);
  else partsplit_run<false, false, MODE>(pt, nd, tp, ci0, ci1, a.wparts, a.plane, st, so, sn);
  if (MODE == PS_WRITE || MODE == PS_LATE) return;   // (no sums: the round's sparts stay)

  if ((a.debug & kDebugUneven) && debug_unlucky(blockIdx.x)) debug_sleep_us(10);
  const uint32_t w = wave_id(), l = lane_id();
  uint32_t f[16] = {so.cnt, so.sr, so.sg, so.sb, so.qr, so.qg, so.qb, 0u,
                    sn.cnt, sn.sr, sn.sg, sn.sb, sn.qr, sn.qg, sn.qb, 0u};
#pragma unroll
  for (int k = 0; k < 16; ++k) f[k] = (k & 7) == 7 ? 0u : wave_sum_u32(f[k]);
  if (l == 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) red[w][k] = f[k];
  }
  __syncthreads();
  if (threadIdx.x < 16) {
    uint32_t x = 0;
#pragma unroll
    for (int ww = 0; ww < kTileWaves; ++ww) x += red[ww][threadIdx.x];
    // (2 TilePartials: 16 words)
    __hip_atomic_store(a.sparts[2 * blockIdx.x].f + threadIdx.x, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (MODE == PS_FULL || MODE == PS_STATS) {
    __shared__ uint64_t red64[kBlock / 64][8];
    split_totals_last<KOFF>(red64);
  }
}

template <int MODE, int FMT>
__device__ __forceinline__ void partsplit_body(const RoundArgs& a, uint8_t* stage, uint32_t (*red)[16]) {
  const PartTile pt = a.ptiles[blockIdx.x];
  if (MODE == PS_LATE) {   // only parents with a child still active after its split epilogue
    const bool a0 = pt.child[0] >= 0 && a.nodes[pt.child[0]].done_it == 0;
    const bool a1 = pt.child[1] >= 0 && a.nodes[pt.child[1]].done_it == 0;
    if (!a0 && !a1) return;
  }
  const ChildInfo ci0 = child_info(a.nodes, pt.child[0]), ci1 = child_info(a.nodes, pt.child[1]);
  partsplit_tile<MODE, FMT, 0>(a, pt, ci0, ci1, stage, red);
}

// One kernel per (mode, parent format): each gets the registers its own path
// needs, and PS_STATS (no stores) no LDS staging at all.
template <int MODE, int FMT>
__global__ __launch_bounds__(kBlock, 4) void partsplit_kernel(RoundArgs a) {
  if (a.counts && blockIdx.x >= a.counts[1]) return;   // planned round: grid is an upper bound
  __shared__ uint32_t red[kTileWaves][16];
  if constexpr (MODE == PS_STATS) {
    partsplit_body<MODE, FMT>(a, nullptr, red);
  } else {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kTileWaves * kStageWave];
    partsplit_body<MODE, FMT>(a, stage, red);
  }
}

// ---------------------------------------------------------------------------
// All 2-means iterations of a round in ONE launch, one workgroup per record
// (kloop_kernel).  Late rounds split nodes of ~10^4-10^5
// points, and their 2-means loop (:613-811) is a chain of up to max_iters
// dependent passes: as kpass launches each costs a kernel boundary, a sweep
// over 8+ tiles and the last arriver's hand-off (~11 us at C3, ~13 at C2),
// almost none of it moving bytes.  Here the record's points are loaded ONCE
// into the workgroup's registers (kLoopRegChunks 16-point chunks per lane;
// a longer record streams the rest from memory every iteration) and every
// iteration is a sweep over registers, a workgroup reduction and the
// reference's FP64 update (node_update, the same function as kpass's
// epilogue, on the same exact integer sums), with no other workgroup
// involved.  After the final iteration the record's per-(tile, wave) counts
// under its final decision give the partition cursors (block_cursors), the
// results go to the host as from kpass, and every record arrives once on
// the launch counter of iteration max_iters - 1 (the status word the host
// waits for).  One shard per record (S == 1, TOT_OWN), planar segments.
constexpr int kLoopBlock = 1024;
constexpr int kLoopRegChunks = 4;          // 4 x 16 points per sweeping lane in registers: 61440 points
constexpr int kLoopMaxBuckets = 4096;      // (tile, wave) buckets: 1024 tiles per record

// Valid slots of the 16-point chunk at absolute index c16 for the segment [lo, hi).
__device__ __forceinline__ uint32_t chunk_valid(uint32_t c16, uint32_t lo, uint32_t hi) {
  const int a = (int)lo - (int)c16, b = (int)hi - (int)c16;
  uint32_t m = b >= 16 ? 0xFFFFu : (b <= 0 ? 0u : (1u << b) - 1u);
  if (a > 0) m &= a >= 16 ? 0u : ~((1u << a) - 1u);
  return m;
}

__device__ __forceinline__ Sweep chunk_sweep_of(const u32x4& r, const u32x4& g, const u32x4& b) {
  Sweep w;
#pragma unroll
  for (int j = 0; j < kVecPerThread; ++j) {
    w.r[j] = r[j];
    w.g[j] = g[j];
    w.b[j] = b[j];
  }
  return w;
}

// (tile, wave) bucket of absolute point p of a record: tile k = [off + k tl,
// ...), its waves per wave_range.
__device__ __forceinline__ uint32_t loop_bucket(uint32_t p, uint32_t off, uint32_t len, uint32_t tl) {
  const uint32_t k = (p - off) / tl;
  const uint32_t ts = off + k * tl, te = min(off + len, ts + tl);
  const uint32_t q = ((te - ts + kSweep - 1) / kSweep) * kWaveSweep;
  return 4u * k + (p - ts) / q;
}

// Waves 0 .. kLoopDataWaves-1 hold the points and sweep them; the last wave
// runs the FP64 update between the two barriers of every iteration.  (Two
// loops, one per role: the sweepers' registers are not live across the
// update, whose FP64 temporaries would otherwise spill them.)
constexpr int kLoopDataWaves = kLoopBlock / 64 - 1;
constexpr uint32_t kLoopDataLanes = 64u * kLoopDataWaves;
__global__ __launch_bounds__(kLoopBlock) void kloop_kernel(RoundArgs a, int32_t max_iters) {
  if (a.counts && a.counts[2] != 0) return;   // planned round aborted by its plan
  typedef __attribute__((address_space(1))) u32x4 g_u4;
  const uint32_t rec = blockIdx.x;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  DevNode* gw = a.nodes + rec;
  __shared__ __attribute__((aligned(16))) DevNode sw;
  __shared__ NodeResult sres;
  __shared__ uint32_t s_red[kLoopDataWaves][8];
  __shared__ uint64_t s_tot[kLoopBlock / 64];
  __shared__ __attribute__((aligned(16))) uint32_t s_b[kLoopMaxBuckets];
  __shared__ int s_fin;
  constexpr int kW16 = (int)(sizeof(DevNode) / 16);
  if (tid < (uint32_t)kW16) reinterpret_cast<u32x4*>(&sw)[tid] = ((const g_cu4*)gw)[tid];
  for (uint32_t i = tid; i < (uint32_t)kLoopMaxBuckets; i += kLoopBlock) s_b[i] = 0u;
  __syncthreads();
  const int tb = sw.tile_begin, te = sw.tile_end;
  // (the host's eligibility rules, checked again: a record outside them is
  // left untouched and arrives active, which the host reports)
  const bool bad = sw.done_it == 0 && (sw.planar != SRC_PLANAR || sw.len > kLoopMaxLen || tb < 0 ||
                                       te - tb > (int)kLoopMaxTiles || te <= tb || sw.tile_len == 0);
  const bool skip = sw.done_it != 0 || bad;   // final at its split (or in an earlier launch)
  if (!skip) {
    if (wv < (uint32_t)kLoopDataWaves) {
      // (wave-uniform values read from LDS: readfirstlane keeps them, and the
      // buffer resources built from them, in scalar registers)
      const uint32_t off = __builtin_amdgcn_readfirstlane(sw.off);
      const uint32_t len = __builtin_amdgcn_readfirstlane(sw.len), end = off + len;
      const uint32_t base = off & ~15u;
      const uint32_t nch = (end - base + 15u) >> 4;   // 16-point chunks of the segment
      const uint64_t srcu = reinterpret_cast<uint64_t>(sw.src);
      // (readfirstlane returns int: each half goes through uint32_t, or the
      // low half's bit 31 would sign-extend over the high half)
      const uint8_t* src = reinterpret_cast<const uint8_t*>(
          ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(srcu >> 32)) << 32) |
          (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)srcu));
      PlaneRsrc s;
      {
        const int nb = (int)(end + 16u);   // (16 B of slack after every shard)
        s.r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nb, 0x00020000);
        s.g = __builtin_amdgcn_make_buffer_rsrc((void*)(src + a.plane), (short)0, nb, 0x00020000);
        s.b = __builtin_amdgcn_make_buffer_rsrc((void*)(src + 2 * a.plane), (short)0, nb, 0x00020000);
      }
      auto load = [&](uint32_t c, u32x4& r, u32x4& g, u32x4& b) {
        const int o = (int)(c < nch ? base + 16u * c : kOOB);
        r = __builtin_amdgcn_raw_buffer_load_b128(s.r, o, 0, 0);
        g = __builtin_amdgcn_raw_buffer_load_b128(s.g, o, 0, 0);
        b = __builtin_amdgcn_raw_buffer_load_b128(s.b, o, 0, 0);
      };
      u32x4 rr[kLoopRegChunks], gg[kLoopRegChunks], bb[kLoopRegChunks];
#pragma unroll
      for (int k = 0; k < kLoopRegChunks; ++k) load(tid + k * kLoopDataLanes, rr[k], gg[k], bb[k]);
      const uint32_t tail0 = kLoopRegChunks * kLoopDataLanes;   // first streamed chunk row
      auto valid = [&](uint32_t c) { return c < nch ? chunk_valid(base + 16u * c, off, end) : 0u; };
      for (;;) {
        const Params q = sw.prm;
        const bool exact_all = !(q.eps < __builtin_inff());
        SplitSums ls;
        // (the points are loop-invariant: without this the compiler hoists
        // their per-slot conversions out of the loop and spills)
#pragma unroll
        for (int k = 0; k < kLoopRegChunks; ++k) asm volatile("" : "+v"(rr[k]), "+v"(gg[k]), "+v"(bb[k]));
#pragma unroll
        for (int k = 0; k < kLoopRegChunks; ++k) {
          if (wv * 64u + k * kLoopDataLanes >= nch) break;   // (wave-uniform: the wave's chunks are past the segment)
          const uint32_t vm = valid(tid + k * kLoopDataLanes);
          const Sweep w = chunk_sweep_of(rr[k], gg[k], bb[k]);
          add_sums(w, vm & ~old_mask(w, vm, q, exact_all), ls);
        }
        for (uint32_t c = tail0 + tid; c - tid < nch; c += kLoopDataLanes) {   // (wave-uniform trip count)
          u32x4 r, g, b;
          load(c, r, g, b);
          const uint32_t vm = valid(c);
          const Sweep w = chunk_sweep_of(r, g, b);
          add_sums(w, vm & ~old_mask(w, vm, q, exact_all), ls);
        }
        // (a wave holds at most 64 chunk rows = 65536 points of a record of
        // at most kLoopMaxLen points: its u32 sums of squares are exact)
        uint32_t f[F_NUM] = {ls.cnt, ls.sr, ls.sg, ls.sb, ls.qr, ls.qg, ls.qb};
#pragma unroll
        for (int k = 0; k < F_NUM; ++k) f[k] = wave_sum_u32(f[k]);
        if (lane == 0) {
#pragma unroll
          for (int k = 0; k < F_NUM; ++k) s_red[wv][k] = f[k];
        }
        __syncthreads();   // (A) partial sums in
        __syncthreads();   // (B) the update out
        if (s_fin) break;
      }
      // per-(tile, wave) old | new << 16 counts under the final decision (the
      // one that produced the final halves: node_update leaves prm unchanged
      // when it finalises)
      const Params q = sw.prm;
      const bool exact_all = !(q.eps < __builtin_inff());
      const uint32_t tl = __builtin_amdgcn_readfirstlane(sw.tile_len);
      // (the register chunks' masks first, so their points are dead before
      // the bucket arithmetic)
      auto count = [&](uint32_t c, uint32_t om, uint32_t vm) {
        const uint32_t nm = vm & ~om;
        if (vm == 0u) return;
        const uint32_t p0 = base + 16u * c + (uint32_t)__builtin_ctz(vm);
        const uint32_t p1 = base + 16u * c + 31u - (uint32_t)__builtin_clz(vm);
        const uint32_t b0 = loop_bucket(p0, off, len, tl);
        if (b0 == loop_bucket(p1, off, len, tl)) {
          atomicAdd(&s_b[b0], (uint32_t)__builtin_popcount(om) | ((uint32_t)__builtin_popcount(nm) << 16));
        } else {
          for (int e = 0; e < 16; ++e)
            if ((vm >> e) & 1u)
              atomicAdd(&s_b[loop_bucket(base + 16u * c + (uint32_t)e, off, len, tl)],
                        ((om >> e) & 1u) ? 1u : 0x10000u);
        }
      };
      uint32_t omk[kLoopRegChunks];
#pragma unroll
      for (int k = 0; k < kLoopRegChunks; ++k) asm volatile("" : "+v"(rr[k]), "+v"(gg[k]), "+v"(bb[k]));
#pragma unroll
      for (int k = 0; k < kLoopRegChunks; ++k) {
        omk[k] = 0u;
        if (wv * 64u + k * kLoopDataLanes >= nch) continue;   // (wave-uniform)
        const uint32_t vm = valid(tid + k * kLoopDataLanes);
        omk[k] = old_mask(chunk_sweep_of(rr[k], gg[k], bb[k]), vm, q, exact_all) | (vm << 16);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int k = 0; k < kLoopRegChunks; ++k) count(tid + k * kLoopDataLanes, omk[k] & 0xFFFFu, omk[k] >> 16);
      for (uint32_t c = tail0 + tid; c - tid < nch; c += kLoopDataLanes) {
        u32x4 r, g, b;
        load(c, r, g, b);
        const uint32_t vm = valid(c);
        count(c, old_mask(chunk_sweep_of(r, g, b), vm, q, exact_all), vm);
      }
    } else {
      // the update wave: iteration it's totals -> node_update (lane 0)
      for (int it = sw.iter;; ++it) {
        __syncthreads();   // (A)
        if (lane == 0) {
          uint64_t t[F_NUM];
#pragma unroll
          for (int k = 0; k < F_NUM; ++k) {
            t[k] = 0;
            for (int v = 0; v < kLoopDataWaves; ++v) t[k] += s_red[v][k];
          }
          const bool fin = it == max_iters - 1 ? node_update<PASS_KLAST>(&sw, &sres, t, a.fixed_point != 0)
                                               : node_update<PASS_KMEANS>(&sw, &sres, t, a.fixed_point != 0);
          if (fin) {
            for (int c = 0; c < 3; ++c) { sres.tm[c] = sw.tm[c]; sres.tv[c] = sw.tv[c]; }
            sw.n_new_local = (uint32_t)t[F_CNT];
            sres.n_new_local = (uint32_t)t[F_CNT];
            sres.done_it = sw.done_it;
          }
          s_fin = fin ? 1 : 0;
        }
        __syncthreads();   // (B)
        if (s_fin) break;
      }
    }
    __syncthreads();   // counts in
    block_cursors<kLoopBlock>(a.tiles, s_b, tb, te, s_tot, tb);
    if (tid < (uint32_t)kW16)   // the final record back (later launches read it)
      ((g_u4*)gw)[tid] = reinterpret_cast<const u32x4*>(&sw)[tid];
  }
  // every wave's cursor / record stores complete before the results and the
  // arrival (the host and later launches read them after the status word /
  // the kernel boundary)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (wv != 0) return;
  if ((a.debug & kDebugUneven) && debug_unlucky(blockIdx.x)) debug_sleep_us(10);
  if (!skip)
    store_result(a.hres + rec, a.dres ? a.dres + rec : nullptr, sres, lane, sw.len, a.seq,
                 a.rsum ? a.rsum + rec : nullptr, &sw);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0)
    arrive(a.ctr + (max_iters - 1), rec, (uint32_t)a.nn, bad, a.hstat + (max_iters - 1), a.seq);
}

// ---------------------------------------------------------------------------
// Device-planned rounds (PlanArgs, dq_kernels.h).  The tables a host-built
// round gets from Engine::run_round -- records, tiles, part tiles, cleared
// counters -- built on the device from the previous round's records and
// results, so the round can be enqueued before those results exist.  The
// layout rules are Engine::tile_len and the record fill of run_round,
// restated; the host mirrors them (Engine::mirror_planned) and checks the
// counts.
// Exact a / b for a < 2^22, b >= 1: a float reciprocal (error < 0.75 on the
// quotient) and one correction each way.  (A generic 32-bit division is ~4x
// the code; the sharded plan inlines 30+ of them and outgrew the I-cache.)
__device__ __forceinline__ uint32_t small_udiv(uint32_t a, uint32_t b) {
  uint32_t q = (uint32_t)((float)a * __builtin_amdgcn_rcpf((float)b));
  int32_t r = (int32_t)(a - q * b);
  if (r < 0) { q -= 1u; r += (int32_t)b; }
  if ((uint32_t)r >= b) q += 1u;
  return q;
}

// Tile length of a record of `len` points, in whole 4096-point sweeps:
// Engine::tile_len_of (roundup_4096(ceil(len / nt)) clamped to [4096, tl])
// restated on L = ceil(len / 4096) < 2^20 sweeps -- nested ceilings:
// ceil(ceil(len / nt) / 4096) = ceil(L / nt).  tl is a whole number of sweeps
// (round_tile_len, tile_max_), nt <= 65536 (apply_tune).
static_assert(kSweep == 4096, "plan_tile_sweeps shifts by 12");
__device__ __forceinline__ uint32_t plan_tile_sweeps(uint32_t len, uint32_t tl, int32_t nt) {
  const uint32_t L = (len >> 12) + ((len & (kSweep - 1)) != 0 ? 1u : 0u);
  const uint32_t m = small_udiv(L + (uint32_t)nt - 1u, (uint32_t)nt);
  return max(1u, min(tl / kSweep, m));
}

__device__ __forceinline__ uint32_t plan_tile_len(uint32_t len, uint32_t tl, int32_t nt) {
  return plan_tile_sweeps(len, tl, nt) * kSweep;
}

// ceil(len / tile length) = ceil(L / m) (nested ceilings again)
__device__ __forceinline__ uint32_t plan_ntiles(uint32_t len, uint32_t tl, int32_t nt) {
  if (len == 0) return 1;   // an empty record still gets one (empty) tile
  const uint32_t L = (len >> 12) + ((len & (kSweep - 1)) != 0 ? 1u : 0u);
  const uint32_t m = plan_tile_sweeps(len, tl, nt);
  return small_udiv(L + m - 1u, m);
}

// The split threshold / shift of a child (the cut of :388-403 from its mean
// and variance), as plan_child and Engine::run_round.
__device__ __forceinline__ void plan_cut(const NodeResult& r, int side, int32_t* thr, int32_t* shift) {
  const double* mean = side ? r.nm : r.om;
  const double* var = side ? r.nv : r.ov;
  double maxv = var[0], cut = mean[0];
  int axis = 0;
  if (maxv < var[1]) { maxv = var[1]; axis = 1; cut = mean[1]; }
  if (maxv < var[2]) { axis = 2; cut = mean[2]; }
  *thr = split_threshold(cut);
  *shift = 16 - 8 * axis;
}

// One child record: the parent's old (side 0) or new (side 1) half
// (run_round's fill for a node fused into its parent's partition).
// (Fields are stored one by one: a DevNode built in registers and copied as
// a whole went through scratch memory.)
__device__ void plan_child(const PlanArgs& a, const DevNode& P, const NodeResult& r, int side,
                           int32_t rec, uint32_t off, uint32_t len, int32_t tb, int32_t pb, int32_t pe) {
  // everything read first (the stores below may not be reordered with loads
  // of possibly aliasing memory); channels as scalars, not an indexed array
  const uint8_t* pd = P.dst;
  const double ps = P.s;
  const double tw = side ? r.nw : r.ow;
  const double* mp = side ? r.nm : r.om;
  const double* vp = side ? r.nv : r.ov;
  const double m0 = mp[0], m1 = mp[1], m2 = mp[2];
  const double v0 = vp[0], v1 = vp[1], v2 = vp[2];
  const int32_t pthr = P.prm.thr, pax = (16 - P.prm.shift) >> 3;
  int32_t lo[3] = {P.box_lo[0], P.box_lo[1], P.box_lo[2]};
  int32_t hi[3] = {P.box_hi[0], P.box_hi[1], P.box_hi[2]};
  const bool proven = r.proven != 0;

  DevNode* d = a.cn + rec;
  d->src = pd;
  const bool in_p0 = pd >= a.p0 && pd < a.p0 + a.cap_bytes;
  d->dst = const_cast<uint8_t*>(in_p0 ? a.p1 + (pd - a.p0) : a.p0 + (pd - a.p1));
  d->off = off;
  d->len = len;
  d->tile_begin = tb;
  const uint32_t tln = plan_tile_len(len, a.tl, a.node_tiles);
  d->tile_end = tb + (int32_t)plan_ntiles(len, a.tl, a.node_tiles);
  d->split_pb = pb;
  d->split_pe = pe;
  d->split_side = side;
  d->planar = SRC_PLANAR;
  d->s = ps;
  d->tw = tw;
  d->tm[0] = m0;
  d->tm[1] = m1;
  d->tm[2] = m2;
  d->tv[0] = v0;
  d->tv[1] = v1;
  d->tv[2] = v2;
  // the cut of :388-403 (plan_cut)
  double maxv = v0, cut = m0;
  int axis = 0;
  if (maxv < v1) { maxv = v1; axis = 1; cut = m1; }
  if (maxv < v2) { axis = 2; cut = m2; }
  d->prm.lhs = d->prm.rr = d->prm.rg = d->prm.rb = 0.0;
  d->prm.lhsf = d->prm.rrf = d->prm.rgf = d->prm.rbf = d->prm.eps = 0.0f;
  d->prm.thr = split_threshold(cut);
  d->prm.shift = 16 - 8 * axis;
  d->prm.pad = 0;
  for (int c = 0; c < 4; ++c) d->prev[c] = 0;
  d->n_new_local = 0;
  d->iter = 0;
  d->done_it = 0;
  d->tile_len = tln;
  d->proven = 0;
  d->pad2[0] = d->pad2[1] = d->pad2[2] = 0;
  // the box: the parent's, clipped at the parent's cut when its halves are the cut's
  for (int c = 0; c < 3; ++c) {
    if (proven && c == pax) {
      if (side) lo[c] = max(lo[c], pthr);
      else hi[c] = min(hi[c], pthr - 1);
    }
    d->box_lo[c] = lo[c];
    d->box_hi[c] = hi[c];
  }
}

// Plan + partition in one launch (one shard per node): the
// planned round's part tile j is partitioned by workgroup j right after
// plan_kernel's bookkeeping, restated per workgroup -- every workgroup scans
// all parents (abort check, the tile counts' exclusive bases), finds the
// parent of part tile j, and the workgroup of a parent's FIRST part tile
// writes the parent's two child records and their tiles (read by the next
// launches only).  The partition itself reads nothing this launch writes:
// its part tile and the children's segments and tilings are computed here
// (ChildInfo), so no workgroup waits for another.  Saves plan_kernel's
// launch and its dependent round trips (~8-10 us per round at C3).  The
// round's counters, per-(tile, wave) counts and arrival words must be zero
// on entry: the invariant's owner is Engine::run, which zeroes every byte of
// the arena a run used with one launch behind that run's last kernel (and a
// new chunk is zeroed when allocated); kDebugArenaCheck verifies it at the
// next run's entry.
template <int MODE, int FMT>
__device__ __forceinline__ void plansplit_body(const PlanArgs& pa, const RoundArgs& a, uint8_t* stage,
                                               uint32_t (*red)[16]) {
  __shared__ uint32_t s_w[kBlock / 64][2];
  __shared__ uint32_t s_abort;
  __shared__ int32_t s_par;
  __shared__ uint32_t s_cb, s_pb;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  const int32_t np = pa.np;
  const uint32_t j = blockIdx.x;
  auto parent = [&](int32_t i) -> int32_t { return pa.plist ? pa.plist[i] : i; };
  auto ntl = [&](uint32_t len) { return plan_ntiles(len, pa.tl, pa.node_tiles); };
  if (tid == 0) {
    s_abort = 0;
    s_par = -1;
  }
  __syncthreads();
  constexpr int kPer = 4;
  uint32_t run_t = 0, run_p = 0;
  bool bad = false;
  for (int32_t c0 = 0; c0 < np; c0 += kBlock * kPer) {
    const int32_t i0 = c0 + (int32_t)tid * kPer;
    uint32_t t[kPer], q[kPer];
    uint32_t lt = 0, lp = 0;
#pragma unroll
    for (int e = 0; e < kPer; ++e) {
      t[e] = q[e] = 0;
      if (i0 + e < np) {
        const RecSummary& P = pa.psum[parent(i0 + e)];
        bad |= P.final == 0;
        const uint32_t nn = P.n_new_local;
        t[e] = ntl(P.len - nn) + ntl(nn);
        q[e] = P.ntiles;
      }
      lt += t[e];
      lp += q[e];
    }
    uint32_t it = lt, ip = lp;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(it, o, 64), v = __shfl_up(ip, o, 64);
      if (lane >= (uint32_t)o) { it += u; ip += v; }
    }
    if (lane == 63) { s_w[wv][0] = it; s_w[wv][1] = ip; }
    __syncthreads();
    uint32_t bt = run_t + it - lt, bp = run_p + ip - lp;
    for (uint32_t w = 0; w < wv; ++w) { bt += s_w[w][0]; bp += s_w[w][1]; }
#pragma unroll
    for (int e = 0; e < kPer; ++e) {
      if (i0 + e < np && j >= bp && j < bp + q[e]) {   // (one lane of the grid's chunk owns part tile j)
        s_par = i0 + e;
        s_cb = bt;
        s_pb = bp;
      }
      bt += t[e];
      bp += q[e];
    }
    for (int w = 0; w < kBlock / 64; ++w) { run_t += s_w[w][0]; run_p += s_w[w][1]; }
    __syncthreads();   // (s_w reuse)
  }
  if (__any(bad) && lane == 0) s_abort = 1;
  const bool cancelled = pa.cancel && pa.cancel[2] == 0;
  __syncthreads();
  const bool overflow = run_t > pa.tiles_cap || run_p > pa.ptiles_cap;
  if (j == 0 && tid == 0) {
    if (pa.debug & kDebugPlanStall) debug_sleep_us(20);
    const uint32_t ab = cancelled ? 3u : (s_abort ? 1u : (overflow ? 2u : 0u));
    const uint32_t c[3] = {ab ? 0u : run_t, ab ? 0u : run_p, ab};
    for (int k = 0; k < 3; ++k) {
      pa.counts[k] = c[k];
      __hip_atomic_store(pa.hcounts + k, c[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (cancelled || s_abort || overflow || j >= run_p) return;   // (uniform)
  // (workgroup-uniform values read from LDS: readfirstlane puts them, and
  // every address and load derived from them, in SGPRs -- as VGPRs they
  // pushed partsplit_tile's body over 128 VGPRs and into scratch)
  const int32_t i = __builtin_amdgcn_readfirstlane(s_par);
  const uint32_t cb = __builtin_amdgcn_readfirstlane(s_cb), pb = __builtin_amdgcn_readfirstlane(s_pb);
  const int32_t ai = __builtin_amdgcn_readfirstlane(parent(i));
  const DevNode* Pp = pa.pn + ai;
  const NodeResult* rp = pa.pres + ai;
  const uint32_t nn = Pp->n_new_local, lo = Pp->len - nn, off = Pp->off;
  const uint32_t nto = ntl(lo), ntn = ntl(nn);
  const int32_t pe = (int32_t)pb + (Pp->tile_end - Pp->tile_begin);
  if (j == pb) {   // the parent's first part tile: its children's records and tiles
    if (tid == 0) plan_child(pa, *Pp, *rp, 0, 2 * i, off, lo, (int32_t)cb, (int32_t)pb, pe);
    if (tid == 64) plan_child(pa, *Pp, *rp, 1, 2 * i + 1, off + lo, nn, (int32_t)(cb + nto), (int32_t)pb, pe);
    const uint32_t tlo = plan_tile_len(lo, pa.tl, pa.node_tiles), tln = plan_tile_len(nn, pa.tl, pa.node_tiles);
    for (uint32_t k = tid; k < nto + ntn; k += kBlock) {
      const int side = k < nto ? 0 : 1;
      const uint32_t kk = side ? k - nto : k;
      const uint32_t coff = side ? off + lo : off, clen = side ? nn : lo, ctl = side ? tln : tlo;
      Tile* tt = pa.ct + cb + k;
      tt->node = 2 * i + side;
      tt->start = coff + kk * ctl;
      tt->end = coff + min(clen, (kk + 1) * ctl);
      tt->pad = 0;
      for (int w = 0; w < kTileWaves; ++w) { tt->old_base[w] = 0; tt->new_base[w] = 0; }
    }
  }
  PartTile pt;
  pt.tile = pa.ptiles + Pp->tile_begin + (j - pb);
  pt.parent = Pp;
  plan_cut(*rp, 0, &pt.thr[0], &pt.shift[0]);
  plan_cut(*rp, 1, &pt.thr[1], &pt.shift[1]);
  for (int s = 0; s < 2; ++s) {   // (FP64 compares run on the VALU: back to SGPRs)
    pt.thr[s] = __builtin_amdgcn_readfirstlane(pt.thr[s]);
    pt.shift[s] = __builtin_amdgcn_readfirstlane(pt.shift[s]);
  }
  pt.child[0] = 2 * i;
  pt.child[1] = 2 * i + 1;
  if (tid == 0) pa.cpt[j] = pt;   // (for the round's PS_LATE partition)
  ChildInfo ci0, ci1;
  ci0.on = ci1.on = 1;
  ci0.off = off;
  ci0.len = lo;
  ci0.tl = plan_tile_len(lo, pa.tl, pa.node_tiles);
  ci0.tb = cb;
  ci1.off = off + lo;
  ci1.len = nn;
  ci1.tl = plan_tile_len(nn, pa.tl, pa.node_tiles);
  ci1.tb = cb + nto;
  for (ChildInfo* c : {&ci0, &ci1}) {   // (the tile lengths: VALU divisions)
    c->tl = __builtin_amdgcn_readfirstlane(c->tl);
    c->tb = __builtin_amdgcn_readfirstlane(c->tb);
  }
  static_assert(sizeof(PlanArgs) % alignof(RoundArgs) == 0, "kernarg layout: (PlanArgs, RoundArgs) packed");
  partsplit_tile<MODE, FMT, sizeof(PlanArgs)>(a, pt, ci0, ci1, stage, red);
}

template <int MODE, int FMT>
__global__ __launch_bounds__(kBlock, 4) void plansplit_kernel(PlanArgs pa, RoundArgs a) {
  __shared__ uint32_t red[kTileWaves][16];
  if constexpr (MODE == PS_STATS) {
    plansplit_body<MODE, FMT>(pa, a, nullptr, red);
  } else {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kTileWaves * kStageWave];
    plansplit_body<MODE, FMT>(pa, a, stage, red);
  }
}


// grid: nb_rec + nb_tile workgroups.  Every workgroup checks that all listed
// parents are final (else the round aborts) and scans all parents' tile
// counts into LDS (children's tiles, part tiles: exclusive bases).  Then
// workgroup b < nb_rec writes the child records of (parent, shard) pairs
// [b * kPlanBlock, ...) (one lane each); the others write one child tile and
// one part tile per lane (output slot -> parent by binary search, then the
// shard record by a walk over the parent's S records), so a parent with
// ~1000 tiles is spread over the grid.
// Shards (a.nshard = S): logical parent i has records pi*S + s; its children
// are logical nodes 2i (old half) and 2i+1 (new half) with records
// (2i+side)*S + s, tiles in record order (old half's shards, then the new
// half's), part tiles in the parent's record order -- Engine::enqueue_host_
// round's layout.  SH (S > 1): each node's S records are read as kMaxShard
// clamped loads issued together (then masked by shard < S), not a walk of
// dependent loads: with 8 shards the walks made the plan ~35 us per round.
constexpr int kPlanBlock = 256;
#ifndef DQ_PLAN_SHARD_WGS
#define DQ_PLAN_SHARD_WGS 64
#endif
constexpr int kPlanShardTileWgs = DQ_PLAN_SHARD_WGS;   // tile workgroups of a sharded plan
template <bool SH>
__global__ __launch_bounds__(kPlanBlock) void plan_kernel(PlanArgs a, uint32_t nb_rec) {
  __shared__ uint32_t s_cb[kPlanMaxParents + 1];   // children's tiles before parent i
  __shared__ uint32_t s_pb[kPlanMaxParents + 1];   // part tiles before parent i
  __shared__ uint32_t s_abort;
  __shared__ uint32_t s_w[kPlanBlock / 64][2];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  const int32_t np = a.np, S = a.nshard;
  auto parent = [&](int32_t i) -> int32_t { return a.plist ? a.plist[i] : i; };   // logical, in prev
  auto ntl = [&](uint32_t len) { return plan_ntiles(len, a.tl, a.node_tiles); };
  if (tid == 0) s_abort = 0;
  __syncthreads();   // (the round's [LaunchCtr | wparts | rdone | summaries] are zero on entry: plansplit_body)
  // (1) every parent final? exclusive scans of the tile counts, chunk by
  //     chunk; a lane takes kPlanPer consecutive parents of a chunk (all their
  //     loads in flight together)
  constexpr int kPlanPer = SH ? 2 : 4;
  constexpr int SM = SH ? kMaxShard : 1;   // shard records read per node
  auto shard = [&](int x) -> int { return SH ? min(x, S - 1) : 0; };
  uint32_t run_t = 0, run_p = 0;
  bool bad = false;
  for (int32_t c0 = 0; c0 < np; c0 += kPlanBlock * kPlanPer) {
    const int32_t i0 = c0 + (int32_t)tid * kPlanPer;
    uint32_t t[kPlanPer], q[kPlanPer];
    uint32_t lt = 0, lp = 0;
#pragma unroll
    for (int e = 0; e < kPlanPer; ++e) {
      t[e] = q[e] = 0;
      if (i0 + e < np) {
        const RecSummary* P0 = a.psum + (size_t)parent(i0 + e) * S;
        bad |= P0->final == 0;   // (every shard record of a node agrees)
#pragma unroll
        for (int sh = 0; sh < SM; ++sh) {
          const RecSummary& P = P0[shard(sh)];
          const uint32_t nn = P.n_new_local;
          const bool on = !SH || sh < S;
          t[e] += on ? ntl(P.len - nn) + ntl(nn) : 0u;
          q[e] += on ? P.ntiles : 0u;
        }
      }
      lt += t[e];
      lp += q[e];
    }
    uint32_t it = lt, ip = lp;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(it, o, 64), v = __shfl_up(ip, o, 64);
      if (lane >= (uint32_t)o) { it += u; ip += v; }
    }
    if (lane == 63) { s_w[wv][0] = it; s_w[wv][1] = ip; }
    __syncthreads();
    uint32_t bt = run_t + it - lt, bp = run_p + ip - lp;
    for (uint32_t w = 0; w < wv; ++w) { bt += s_w[w][0]; bp += s_w[w][1]; }
#pragma unroll
    for (int e = 0; e < kPlanPer; ++e) {
      if (i0 + e < np) {
        s_cb[i0 + e] = bt;
        s_pb[i0 + e] = bp;
      }
      bt += t[e];
      bp += q[e];
    }
    for (int w = 0; w < kPlanBlock / 64; ++w) { run_t += s_w[w][0]; run_p += s_w[w][1]; }
    __syncthreads();   // (s_w reuse)
  }
  if (__any(bad) && lane == 0) s_abort = 1;
  // a re-plan whose first plan ran (did not abort) is not needed
  const bool cancelled = a.cancel && a.cancel[2] == 0;
  if (tid == 0) { s_cb[np] = run_t; s_pb[np] = run_p; }
  __syncthreads();
  const bool overflow = run_t > a.tiles_cap || run_p > a.ptiles_cap;
  if (blockIdx.x == 0 && tid == 0) {
    if (a.debug & kDebugPlanStall) debug_sleep_us(20);
    const uint32_t ab = cancelled ? 3u : (s_abort ? 1u : (overflow ? 2u : 0u));
    const uint32_t c[3] = {ab ? 0u : run_t, ab ? 0u : run_p, ab};
    for (int k = 0; k < 3; ++k) {
      a.counts[k] = c[k];
      __hip_atomic_store(a.hcounts + k, c[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (cancelled || s_abort || overflow) return;
  if (blockIdx.x < nb_rec) {
    // (2a) records: (parent i, shard sh) -> records (2i)*S + sh (old half),
    //      (2i+1)*S + sh (new half)
    const int32_t u = (int32_t)(blockIdx.x * kPlanBlock + tid);
    if (u >= np * S) return;
    const int32_t i = u / S, sh = u - i * S;
    const int32_t ai = parent(i) * S;
    uint32_t told = 0, tnew_all = 0, tnew = 0, pbo = 0;   // tiles / part tiles before this shard's
#pragma unroll
    for (int x = 0; x < SM; ++x) {
      const RecSummary& Q = a.psum[ai + shard(x)];
      const bool on = !SH || x < S;
      const uint32_t nn = Q.n_new_local;
      const uint32_t to = ntl(Q.len - nn), tn = ntl(nn), pq = Q.ntiles;
      if (on && x < sh) {
        told += to;
        tnew += tn;
        pbo += pq;
      }
      tnew_all += on ? to : 0u;
    }
    const DevNode& P = a.pn[ai + sh];
    const NodeResult& r = a.pres[ai + sh];
    const uint32_t nn = P.n_new_local, lo = P.len - nn;
    const int32_t pb = (int32_t)(s_pb[i] + pbo), pe = pb + (P.tile_end - P.tile_begin);
    plan_child(a, P, r, 0, (2 * i) * S + sh, P.off, lo, (int32_t)(s_cb[i] + told), pb, pe);
    plan_child(a, P, r, 1, (2 * i + 1) * S + sh, P.off + lo, nn, (int32_t)(s_cb[i] + tnew_all + tnew), pb, pe);
    return;
  }
  // (2b) child tiles and part tiles, one of each per lane per step, grid-
  //      stride over the tile workgroups of the launch (S > 1 launches only
  //      a few: every workgroup's scan of the parents' S records above costs
  //      more than the tiles it then writes)
  auto find = [&](const uint32_t* base, uint32_t x) -> int32_t {   // last i with base[i] <= x
    int32_t lo = 0, hi = np - 1;
    while (lo < hi) {
      const int32_t mid = (lo + hi + 1) >> 1;
      if (base[mid] <= x) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  const uint32_t nbt = gridDim.x - nb_rec;
  for (uint32_t j = (blockIdx.x - nb_rec) * kPlanBlock + tid; j < max(run_t, run_p); j += nbt * kPlanBlock) {
  if (j < run_t) {
    const int32_t i = find(s_cb, j);
    const int32_t ai = parent(i) * S;
    uint32_t k = j - s_cb[i];
    // the child record holding slot k: old half's shards, then the new half's
    uint32_t qlo[SM], qnn[SM], qoff[SM];
#pragma unroll
    for (int x = 0; x < SM; ++x) {
      const RecSummary& Q = a.psum[ai + shard(x)];
      qnn[x] = Q.n_new_local;
      qlo[x] = Q.len - qnn[x];
      qoff[x] = Q.off;
    }
    int side = 0, sh = 0;
    uint32_t off = 0, len = 0;
    bool found = false;
#pragma unroll
    for (int v = 0; v < 2 * SM; ++v) {
      const int nw = v >= SM ? 1 : 0, x = nw ? v - SM : v;
      if (found || (SH && x >= S)) continue;
      const uint32_t l = nw ? qnn[x] : qlo[x], nt = ntl(l);
      if (k < nt) {
        found = true;
        side = nw;
        sh = x;
        off = nw ? qoff[x] + qlo[x] : qoff[x];
        len = l;
      } else {
        k -= nt;
      }
    }
    const uint32_t tln = plan_tile_len(len, a.tl, a.node_tiles);
    Tile* tt = a.ct + j;
    tt->node = (2 * i + side) * S + sh;
    tt->start = off + k * tln;
    tt->end = off + min(len, (k + 1) * tln);
    tt->pad = 0;
    for (int w = 0; w < kTileWaves; ++w) { tt->old_base[w] = 0; tt->new_base[w] = 0; }
  }
  if (j < run_p) {
    const int32_t i = find(s_pb, j);
    const int32_t ai = parent(i) * S;
    uint32_t k = j - s_pb[i];
    uint32_t qnt[SM];
#pragma unroll
    for (int x = 0; x < SM; ++x) qnt[x] = a.psum[ai + shard(x)].ntiles;
    int sh = 0;
    bool stop = false;
#pragma unroll
    for (int x = 0; x < SM - 1; ++x) {
      if (stop || x >= S - 1) continue;
      if (k < qnt[x]) stop = true;
      else { k -= qnt[x]; sh = x + 1; }
    }
    const NodeResult& r = a.pres[ai + sh];
    PartTile* pt = a.cpt + j;
    pt->tile = a.ptiles + a.psum[ai + sh].tile_begin + k;
    pt->parent = a.pn + ai + sh;
    int32_t thr0, sh0, thr1, sh1;
    plan_cut(r, 0, &thr0, &sh0);
    plan_cut(r, 1, &thr1, &sh1);
    pt->thr[0] = thr0;
    pt->thr[1] = thr1;
    pt->shift[0] = sh0;
    pt->shift[1] = sh1;
    pt->child[0] = (2 * i) * S + sh;
    pt->child[1] = (2 * i + 1) * S + sh;
  }
  }
}

// Host-built round tables: host-coherent staging -> the round's device block.
__global__ __launch_bounds__(256) void upload_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                     uint32_t n16) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n16; i += gridDim.x * 256u) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void zero_kernel(u32x4* __restrict__ dst, uint32_t n16) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n16; i += gridDim.x * 256u) dst[i] = (u32x4){0u, 0u, 0u, 0u};
}

// The in-process loopback collective's reduction (tests): dst[i] = sum over
// the ranks' buffers of src[r][i] (u64, exact).
__global__ __launch_bounds__(256) void sum_u64_kernel(SumSrcs s, int nsrc, uint64_t* __restrict__ dst,
                                                      uint32_t count) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < count; i += gridDim.x * 256u) {
    uint64_t v = 0;
    for (int r = 0; r < nsrc; ++r) v += s.p[r][i];
    dst[i] = v;
  }
}

// Map, step 1: per colour cell (8x8x8 values), the palette entries that can
// be the nearest entry of some colour of the cell.  Two exact filters:
//   (a) min distance of e to the cell <= the smallest max distance of any
//       entry to the cell (else some entry is closer for every colour);
//   (b) dominance: e is dropped when ONE other candidate f (one of the 4
//       with the smallest max distance) is strictly closer than e for every
//       colour x of the cell, i.e. 2 (e - f).x < |e|^2 - |f|^2 at the cell
//       corner maximising (e - f).x (strict: an entry that can tie is kept
//       -- ties are broken by the MPS rank in the map).
// Every exact argmin for a colour of the cell survives both, so the map's
// answer is unchanged.  grid = (kCells / kBlock, tasks): the task's palette
// is staged in LDS once per workgroup.
// Outputs per cell (surviving candidates in palette order):
//   16-B record: x[15:0] count c; x[31:16], y, z, w: the first kCellInline
//     indices (u16), unused slots = k (a sentinel farther than any entry);
//     c > kCellInline: all c indices in cell_idx[cell*kCellCap ...];
//     c == kCellBrute: scan the whole palette;
//   compact 32-bit record (K <= 1024): 1..3 candidates inline (10-bit
//     indices, unused slots repeat the first), else (count << 16 | cell)
//     with bits 31:30 = 0 (count 63: whole palette).
// One LANE per cell (grid.x = kCells / kBlock): every lane of a wave reads
// the same palette entry at the same time (LDS broadcast); each lane keeps
// its loose candidate list in a transposed LDS array.
template <int BR, int BG, int BB>
__global__ __launch_bounds__(BR * BG * BB) void build_cells_kernel(const MapTask* __restrict__ tasks) {
  constexpr int kThreads = BR * BG * BB;
  constexpr int kWaves = kThreads / 64;
  const MapTask tk = tasks[blockIdx.y];
  const int k = tk.k;
  extern __shared__ uint32_t spal_c[];   // k colours, then k region-list entries (u16)
  uint16_t* slist = reinterpret_cast<uint16_t*>(spal_c + k);
  __shared__ uint32_t scand[kCellCap * kThreads];   // [i][thread]
  __shared__ int sred[kWaves];
  __shared__ uint32_t swoff[kWaves + 1];
  for (int i = threadIdx.x; i < k; i += kThreads) spal_c[i] = as_g(tk.pal)[i];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  auto far2 = [](int v, int lo, int hi) { const int x = max(v - lo, hi - v); return x * x; };
  auto near2 = [](int v, int lo, int hi) {
    const int x = max(max(lo - v, v - hi), 0);
    return x * x;
  };
  // This workgroup's cells: a BR x BG x BB block of the 32^3 grid (R x G x B),
  // so that one region list serves all of them.  For a cell C inside the
  // region R, C's candidates {e : near2(e,C) <= min_f far2(f,C)} are
  // candidates of R (near2(e,R) <= near2(e,C), far2(f,C) <= far2(f,R)), and
  // C's minimiser of far2 is one too: scanning R's list (palette order)
  // gives exactly the bound and the candidates of a scan over the palette.
  constexpr int kSide = 1 << kCellBits;
  static_assert(kSide % BR == 0 && kSide % BG == 0 && kSide % BB == 0 && kThreads % 64 == 0,
                "whole blocks of cells, whole waves");
  constexpr uint32_t nbb = kSide / BB, nbg = kSide / BG;
  const uint32_t bb = blockIdx.x % nbb, bg = (blockIdx.x / nbb) % nbg, br = blockIdx.x / (nbb * nbg);
  const uint32_t c0 = br * BR + tid / (BG * BB), c1 = bg * BG + (tid / BB) % BG, c2 = bb * BB + tid % BB;
  const uint32_t cell = (c0 << (2 * kCellBits)) | (c1 << kCellBits) | c2;
  const int cw = 1 << (8 - kCellBits);
  const int rlo0 = (int)br * BR * cw, rlo1 = (int)bg * BG * cw, rlo2 = (int)bb * BB * cw;
  const int rhi0 = rlo0 + BR * cw - 1, rhi1 = rlo1 + BG * cw - 1, rhi2 = rlo2 + BB * cw - 1;
  __syncthreads();
  // region bound: min over entries of the max distance to the region
  int rb = 0x7FFFFFFF;
  for (int e = (int)tid; e < k; e += kThreads) {
    const uint32_t q = spal_c[e];
    rb = min(rb, far2((q >> 16) & 0xFF, rlo0, rhi0) + far2((q >> 8) & 0xFF, rlo1, rhi1) +
                     far2(q & 0xFF, rlo2, rhi2));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) rb = min(rb, __shfl_xor(rb, o, 64));
  if (lane == 0) sred[wv] = rb;
  __syncthreads();
  rb = sred[0];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) rb = min(rb, sred[w]);
  // region list in palette order: chunks of one entry per thread, ballot-ranked
  uint32_t nlist = 0;
  for (int base = 0; base < k; base += kThreads) {
    const int e = base + (int)tid;
    bool in = false;
    if (e < k) {
      const uint32_t q = spal_c[e];
      in = near2((q >> 16) & 0xFF, rlo0, rhi0) + near2((q >> 8) & 0xFF, rlo1, rhi1) +
               near2(q & 0xFF, rlo2, rhi2) <= rb;
    }
    const uint64_t m = __ballot(in);
    if (lane == 0) swoff[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = nlist;
    for (uint32_t w = 0; w < wv; ++w) off += swoff[w];
    if (in) slist[off + mbcnt64(m)] = (uint16_t)e;
    for (int w = 0; w < kWaves; ++w) nlist += swoff[w];
    __syncthreads();
  }
  const int lo0 = (int)c0 * cw, lo1 = (int)c1 * cw, lo2 = (int)c2 * cw;
  const int hi0 = lo0 + cw - 1, hi1 = lo1 + cw - 1, hi2 = lo2 + cw - 1;
  int bound = 0x7FFFFFFF;
#pragma unroll 4
  for (uint32_t i = 0; i < nlist; ++i) {
    const uint32_t q = spal_c[slist[i]];
    bound = min(bound, far2((q >> 16) & 0xFF, lo0, hi0) + far2((q >> 8) & 0xFF, lo1, hi1) +
                           far2(q & 0xFF, lo2, hi2));
  }
  // (a) loose candidates, palette order
  uint32_t count = 0;
#pragma unroll 4
  for (uint32_t i = 0; i < nlist; ++i) {
    const uint32_t e = slist[i];
    const uint32_t q = spal_c[e];
    const bool cand = near2((q >> 16) & 0xFF, lo0, hi0) + near2((q >> 8) & 0xFF, lo1, hi1) +
                          near2(q & 0xFF, lo2, hi2) <= bound;
    if (cand && count < (uint32_t)kCellCap) scand[count * kThreads + tid] = e;
    count += cand ? 1u : 0u;
  }
  // (b) dominance by the 4 candidates with the smallest max distance (as
  //     tight as all pairs on the measured palettes, O(4c) instead of c^2),
  //     compacted in place (order kept)
  const bool brute = count > (uint32_t)kCellCap;
  uint32_t fcount = brute ? 0u : count;
  if (!brute && count > 1) {
    constexpr int kRefs = 4;
    int rf[kRefs] = {0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF};
    uint32_t rq[kRefs] = {0u, 0u, 0u, 0u};
    for (uint32_t i = 0; i < count; ++i) {   // the 4 smallest (far2, colour)
      const uint32_t q = spal_c[scand[i * kThreads + tid]];
      int f = far2((q >> 16) & 0xFF, lo0, hi0) + far2((q >> 8) & 0xFF, lo1, hi1) + far2(q & 0xFF, lo2, hi2);
      uint32_t c = q;
#pragma unroll
      for (int r = 0; r < kRefs; ++r) {
        if (f < rf[r]) {
          const int tf = rf[r];
          const uint32_t tq = rq[r];
          rf[r] = f;
          rq[r] = c;
          f = tf;
          c = tq;
        }
      }
    }
    const int nref = (int)min(count, (uint32_t)kRefs);
    uint32_t kept = 0;
    for (uint32_t i = 0; i < count; ++i) {
      const uint32_t ei = scand[i * kThreads + tid];
      const uint32_t qe = spal_c[ei];
      const int e0 = (qe >> 16) & 0xFF, e1 = (qe >> 8) & 0xFF, e2 = qe & 0xFF;
      const int ee = e0 * e0 + e1 * e1 + e2 * e2;
      bool keep = true;
#pragma unroll
      for (int r = 0; r < kRefs; ++r) {
        if (r >= nref) break;
        const uint32_t qf = rq[r];
        const int f0 = (qf >> 16) & 0xFF, f1 = (qf >> 8) & 0xFF, f2 = qf & 0xFF;
        const int d0 = e0 - f0, d1 = e1 - f1, d2 = e2 - f2;
        const int dx = d0 * (d0 > 0 ? hi0 : lo0) + d1 * (d1 > 0 ? hi1 : lo1) + d2 * (d2 > 0 ? hi2 : lo2);
        // (f == e: dx = 0 = rhs, never strict)
        keep = keep && !(2 * dx < ee - (f0 * f0 + f1 * f1 + f2 * f2));
      }
      if (keep) scand[(kept++) * kThreads + tid] = ei;
    }
    fcount = kept;
  }
  uint16_t* lst = tk.cell_idx + (size_t)cell * kCellCap;
  for (uint32_t i = 0; i < fcount; ++i) lst[i] = (uint16_t)scand[i * kThreads + tid];
  const uint32_t c = brute ? kCellBrute : fcount;
  uint32_t slot[kCellInline];
#pragma unroll
  for (int i = 0; i < kCellInline; ++i) slot[i] = (uint32_t)i < fcount ? scand[i * kThreads + tid] : (uint32_t)k;
  uint4 r;
  r.x = c | (slot[0] << 16);
  r.y = slot[1] | (slot[2] << 16);
  r.z = slot[3] | (slot[4] << 16);
  r.w = slot[5] | (slot[6] << 16);
  reinterpret_cast<uint4*>(tk.cell_rec)[cell] = r;
  // compact record (K <= 1024): bit 31 -- one candidate, its colour in bits
  // 0-23 (every filter is an exact elimination, so it is every colour's
  // answer); bits 31:30 = 01 -- 2 or 3 candidates, 10-bit indices (unused
  // slots repeat the first); 00 -- count << 16 | cell (count 63: whole palette)
  uint32_t c32;
  if (fcount == 1) {
    c32 = 0x80000000u | spal_c[slot[0]];
  } else if (fcount >= 2 && fcount <= 3) {
    const uint32_t j0 = slot[0], j1 = slot[1];
    const uint32_t j2 = fcount > 2 ? slot[2] : j0;
    c32 = 0x40000000u | j0 | (j1 << 10) | (j2 << 20);
  } else {
    c32 = ((brute ? 63u : fcount) << 16) | cell;
  }
  if (tk.cell_c32) tk.cell_c32[cell] = c32;
}

// Map, step 2.  The answer is the entry minimising (squared distance, MPS
// visit rank) where the walk starts at s = lut_init[R+G+B] and visits s,
// s+1, s-1, s+2, s-2, ...: rank(j) = 2(j-s)-1 for j > s, 2(s-j) otherwise.
// That entry is exactly what map_colors_mps returns (strict '<' keeps the
// first visited; the floor(d^2/3) pruning never drops a strictly closer
// entry).  One 32-bit key per candidate carries both, exactly:
//   d'  = (|c|^2 + 2^19) - 2 p.c  = d - |p|^2 + 2^19, in (0, 2^20)  (v_dot4)
//   sad = |4j - (4s+1)| = 2 rank(j) + 1 < 2^12           (v_sad_u16; K<=1024 here)
//   key = d' << 12 | sad;  the minimum key's j = the answer.
// j is recovered from sad (4j = 4s+1 +- sad).  Inline candidates are
// branch-free; only cells with more than kCellInline candidates take a
// wave-uniform slow path over their list.
// Batched: workgroup b serves the task whose [block_begin, +blocks) holds b
// and maps that task's groups of kMapPx pixels [lb*gpb, (lb+1)*gpb).
constexpr int kMapPx = 8;   // pixels per lane per iteration (two 16-B loads)

template <bool kWide>
__device__ __forceinline__ uint32_t entry_from_sad(uint32_t S, uint32_t sad) {
  const uint32_t x = S + sad;
  return (x & 3u) == 0 ? (x >> 2) : ((S - sad) >> 2);
}

template <bool kWide>
__global__ __launch_bounds__(kBlock) void map_kernel(const MapTask* __restrict__ tasks, int ntasks) {
  int ti = 0;
  while (ti + 1 < ntasks && tasks[ti + 1].block_begin <= blockIdx.x) ++ti;
  const MapTask tk = tasks[ti];
  const uint32_t* __restrict__ in = tk.in;
  uint32_t* __restrict__ out = tk.out;
  const uint32_t n = tk.n;
  const int k = tk.k;
  const uint16_t* __restrict__ cell_idx = tk.cell_idx;
  extern __shared__ uint32_t smem[];
  uint2* spal = reinterpret_cast<uint2*>(smem);              // k+1: colour, |c|^2 + 2^19
  uint16_t* slut = reinterpret_cast<uint16_t*>(smem + 2 * (k + 1));
  g_cu32* gpal = as_g(tk.pal);
  typedef const __attribute__((address_space(1))) uint16_t g_cu16;
  g_cu16* glut = (g_cu16*)tk.lut;
  g_cu16* gidx = (g_cu16*)cell_idx;
  for (int i = threadIdx.x; i <= k; i += kBlock) {
    const uint32_t q = i < k ? gpal[i] : 0u;
    // the sentinel (index k, unused inline slots) has d' = 2^20 - 1: it never wins
    const uint32_t c2 = i < k ? __builtin_amdgcn_udot4(q, q, 0u, false) + (1u << 19) : 0xFFFFFu;
    spal[i] = make_uint2(q, c2);
  }
  for (int i = threadIdx.x; i < 766; i += kBlock) slut[i] = glut[i];
  __syncthreads();
  g_cu4* rec4 = (g_cu4*)tk.cell_rec;
  g_cu4* in4 = (g_cu4*)in;
  typedef __attribute__((address_space(1))) u32x4 g_u4;

  // exact (d, rank) key of palette entry j for pixel p (S = 4 s + 1)
  auto full_key = [&](uint32_t p, uint32_t S, uint32_t j) -> uint64_t {
    const uint2 en = spal[j];
    const uint32_t d = (uint32_t)((int32_t)en.y - 2 * (int32_t)__builtin_amdgcn_udot4(p, en.x, 0u, false));
    const uint32_t sad = __builtin_amdgcn_sad_u16(4u * j, S, 0u);
    return kWide ? (((uint64_t)d << 32) | sad) : (uint64_t)((d << 12) | sad);
  };

  const uint32_t ngrp = n / kMapPx;
  const uint32_t lb = blockIdx.x - tk.block_begin;
  const uint32_t g0 = lb * tk.grp_per_block;
  const uint32_t g1 = min(ngrp, g0 + tk.grp_per_block);
  for (uint32_t gb = g0; gb < g1; gb += kBlock) {
    const uint32_t g = gb + threadIdx.x;
    const bool have = g < g1;
    uint32_t px[kMapPx];
    {
      const u32x4 a = have ? in4[2 * g] : (u32x4){0u, 0u, 0u, 0u};
      const u32x4 b = have ? in4[2 * g + 1] : (u32x4){0u, 0u, 0u, 0u};
      for (int e = 0; e < 4; ++e) { px[e] = a[e] & 0xFFFFFFu; px[4 + e] = b[e] & 0xFFFFFFu; }
    }
    uint32_t cell[kMapPx];
    u32x4 r[kMapPx];
#pragma unroll
    for (int e = 0; e < kMapPx; ++e) {   // issue every gather before using any
      const uint32_t p = px[e];
      cell[e] = ((p >> (24 - kCellBits)) << (2 * kCellBits)) |
                (((p >> (16 - kCellBits)) & ((1u << kCellBits) - 1)) << kCellBits) |
                ((p >> (8 - kCellBits)) & ((1u << kCellBits) - 1));
      r[e] = rec4[cell[e]];
    }
    uint32_t res[kMapPx];
    bool over[kMapPx];
    uint32_t Ss[kMapPx];
#pragma unroll
    for (int e = 0; e < kMapPx; ++e) {
      const uint32_t p = px[e];
      const uint32_t S = 4u * slut[((p >> 16) & 0xFF) + ((p >> 8) & 0xFF) + (p & 0xFF)] + 1u;
      Ss[e] = S;
      const uint32_t idx[kCellInline] = {r[e][0] >> 16, r[e][1] & 0xFFFF, r[e][1] >> 16,
                                         r[e][2] & 0xFFFF, r[e][2] >> 16, r[e][3] & 0xFFFF,
                                         r[e][3] >> 16};
      uint64_t best = ~0ull;
#pragma unroll
      for (int m = 0; m < kCellInline; ++m) {
        const uint64_t key = full_key(p, S, idx[m]);
        best = key < best ? key : best;
      }
      const uint32_t sad = (uint32_t)(kWide ? (best & 0xFFFFFFFFull) : (best & 0xFFFu));
      res[e] = spal[entry_from_sad<kWide>(S, sad)].x;
      over[e] = (r[e][0] & 0xFFFF) > (uint32_t)kCellInline;
    }
    bool any_over = false;
#pragma unroll
    for (int e = 0; e < kMapPx; ++e) any_over |= over[e];
    if (__any(any_over)) {
#pragma unroll
      for (int e = 0; e < kMapPx; ++e) {
        if (!over[e]) continue;
        const uint32_t p = px[e], S = Ss[e];
        const uint32_t cnt = r[e][0] & 0xFFFF;
        uint64_t best = ~0ull;
        if (cnt == kCellBrute) {
          for (int j = 0; j < k; ++j) { const uint64_t key = full_key(p, S, (uint32_t)j); best = key < best ? key : best; }
        } else {
          g_cu16* lst = gidx + (size_t)cell[e] * kCellCap;
          for (uint32_t m = 0; m < cnt; ++m) { const uint64_t key = full_key(p, S, lst[m]); best = key < best ? key : best; }
        }
        const uint32_t sad = (uint32_t)(kWide ? (best & 0xFFFFFFFFull) : (best & 0xFFFu));
        res[e] = spal[entry_from_sad<kWide>(S, sad)].x;
      }
    }
    if (have) {
      ((g_u4*)as_gw(out))[2 * g] = (u32x4){res[0], res[1], res[2], res[3]};
      ((g_u4*)as_gw(out))[2 * g + 1] = (u32x4){res[4], res[5], res[6], res[7]};
    }
  }
  // tail (n % kMapPx points): the task's first workgroup, one point per lane, whole palette
  const uint32_t t = ngrp * kMapPx + threadIdx.x;
  if (lb == 0 && t < n) {
    const uint32_t p = as_g(in)[t] & 0xFFFFFFu;
    const uint32_t S = 4u * slut[((p >> 16) & 0xFF) + ((p >> 8) & 0xFF) + (p & 0xFF)] + 1u;
    uint64_t best = ~0ull;
    for (int j = 0; j < k; ++j) { const uint64_t key = full_key(p, S, (uint32_t)j); best = key < best ? key : best; }
    const uint32_t sad = (uint32_t)(kWide ? (best & 0xFFFFFFFFull) : (best & 0xFFFu));
    as_gw(out)[t] = spal[entry_from_sad<kWide>(S, sad)].x;
  }
}

// Map with the compact cell table in LDS (K <= 1024): one workgroup of
// kMapLdsBlock threads per CU stages its task's 32768 compact records
// (128 KB), the sorted palette and the start LUT, then maps its share of the
// task's pixels, 8 per lane per iteration.
//   * A cell with ONE candidate (64 % of the cells for a 256-colour palette of
//     uniform frames) holds its answer colour in the record: such a pixel
//     needs no other LDS read (the candidate reads below are exec-masked, so
//     their lanes cost no LDS cycles; the LDS bank conflicts of the random
//     palette reads were ~2.5x the map's active LDS time).
//   * 2-3 inline candidates are evaluated branch-free.
//   * Pixels of cells with more candidates are queued in LDS (per wave, in
//     slot order) and resolved cooperatively: lane i takes queue entry i and
//     scans that cell's list; the results return through the queue.  Queue
//     overflow (more than 64 such pixels in one wave-iteration) falls back to
//     a per-lane loop.
// Same keys and the same answer as map_kernel.
constexpr int kMapQ = 64;
#ifndef DQ_MAP_PF
#define DQ_MAP_PF 2
#endif
constexpr uint32_t kMapPf = DQ_MAP_PF;   // iterations of pixels in flight ahead (1 or 2)
#ifndef DQ_MAP_LC
#define DQ_MAP_LC 1
#endif
constexpr bool kMapLc = DQ_MAP_LC;       // packed pixels: lane-contiguous 16-B chunks
// 12 BGR24 bytes (3 words, little-endian) -> 4 packed 0x00RRGGBB words.
__device__ __forceinline__ u32x4 bgr12_to_px4(uint32_t w0, uint32_t w1, uint32_t w2) {
  u32x4 o;
  o.x = w0 & 0x00FFFFFFu;
  o.y = __builtin_amdgcn_perm(w1, w0, 0x0C050403u);   // b3 b4 b5 0
  o.z = __builtin_amdgcn_perm(w2, w1, 0x0C040302u);   // b6 b7 b8 0
  o.w = w2 >> 8;                                       // b9 b10 b11 0
  return o;
}

template <bool BGR>
__global__ __launch_bounds__(kMapLdsBlock) void map_lds_kernel(const MapTask* __restrict__ tasks,
                                                              int ntasks) {
  int ti = 0;
  while (ti + 1 < ntasks && tasks[ti + 1].block_begin <= blockIdx.x) ++ti;
  const MapTask tk = tasks[ti];
  const uint32_t n = tk.n;
  const int k = tk.k;
  extern __shared__ uint32_t smem[];
  uint32_t* stab = smem;                                      // kCells compact records
  uint32_t* squeue = smem + kCells;                           // per wave: kMapQ pixels / results
  uint2* spal = reinterpret_cast<uint2*>(squeue + (kMapLdsBlock / 64) * kMapQ);   // k+1
  uint16_t* slut = reinterpret_cast<uint16_t*>(reinterpret_cast<uint32_t*>(spal) + 2 * (k + 1));
  typedef const __attribute__((address_space(1))) uint16_t g_cu16;
  {
    g_cu4* t4 = (g_cu4*)tk.cell_c32;
    u32x4* s4 = reinterpret_cast<u32x4*>(stab);
#pragma unroll 4
    for (int i = threadIdx.x; i < kCells / 4; i += kMapLdsBlock) s4[i] = t4[i];
    g_cu32* gpal = as_g(tk.pal);
    for (int i = threadIdx.x; i <= k; i += kMapLdsBlock) {
      const uint32_t q = i < k ? gpal[i] : 0u;
      const uint32_t c2 = i < k ? __builtin_amdgcn_udot4(q, q, 0u, false) + (1u << 19) : 0xFFFFFu;
      spal[i] = make_uint2(q, c2 << 12);   // c2 < 2^20: the key's distance field, pre-shifted
    }
    g_cu16* glut = (g_cu16*)tk.lut;
    for (int i = threadIdx.x; i < 766; i += kMapLdsBlock) slut[i] = (uint16_t)(4u * glut[i] + 1u);   // S = 4s + 1
  }
  __syncthreads();
  const uint32_t lane = lane_id();
  uint32_t* wq = squeue + wave_id() * kMapQ;
  g_cu4* gidx4 = (g_cu4*)tk.cell_idx;
  g_cu16* gidx = (g_cu16*)tk.cell_idx;
  g_cu4* in4 = (g_cu4*)tk.in;
  // a BGR24 frame (tk.bgr): group g is the 24 bytes at 24 g, three 8-B loads
  typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
  typedef const __attribute__((address_space(1))) u32x2v g_cu2;
  g_cu2* in2 = (g_cu2*)tk.in;
  constexpr bool bgr = BGR;   // (every task of a launch has the same pixel format)
  const uint32_t ngrp = n / kMapPx;
  const uint32_t lb = blockIdx.x - tk.block_begin;
  const uint32_t g0 = lb * tk.grp_per_block;
  const uint32_t g1 = min(ngrp, g0 + tk.grp_per_block);
  // packed pixels: the lane's two 16-B chunks of its wave's 2 KB, lane-
  // contiguous per load instruction (chunks lane and 64 + lane of the wave's
  // 128) when kMapLc, else the lane's own 32 B (chunks 2 lane, 2 lane + 1)
  auto chunk = [&](uint32_t gi, uint32_t h) -> uint32_t {
    return kMapLc ? 2u * (gi - lane) + 64u * h + lane : 2u * gi + h;
  };
  auto load_group = [&](uint32_t gi, u32x4& a, u32x4& b) {   // (nothing past the task's groups)
    if (bgr) {
      if (gi < g1) {
        const u32x2v x0 = in2[3 * gi], x1 = in2[3 * gi + 1], x2 = in2[3 * gi + 2];
        a = (u32x4){x0.x, x0.y, x1.x, x1.y};
        b = (u32x4){x2.x, x2.y, 0u, 0u};
      }
    } else {
      const uint32_t c0 = chunk(gi, 0), c1 = chunk(gi, 1);
      if (c0 < 2u * g1) a = in4[c0];
      if (c1 < 2u * g1) b = in4[c1];
    }
  };
  // the output through a buffer resource: a lane past the task's groups
  // stores at kOOB (dropped), so every iteration issues the same count of
  // vector-memory operations after its loads (see the loop's top)
  const __amdgpu_buffer_rsrc_t orsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)tk.out, (short)0, (int)(4ull * n), 0x00020000);   // (n <= 2^28: Engine::map_many)

  // (c2 - 2 dot) << 12 | sad, as (c2 << 12) - (dot << 13) + sad: the low 12
  // bits of the first two terms are zero and sad < 4096, so the OR is an add
  // and folds into v_sad_u16's accumulator (same 32-bit key as map_kernel)
  // (c2 << 12) - (dot << 13) as one v_mad_i32_i24 (dot < 2^18).  The factor
  // is -8192 at run time but not a compile-time constant (k < 2^30), or the
  // compiler turns the multiply back into a shift and a subtract.
  const int32_t m8192 = -(int32_t)(8192u | ((uint32_t)k >> 30));
  auto key = [&](uint32_t p, uint32_t S, uint32_t j) -> uint32_t {
    const uint2 en = spal[j];
    const uint32_t hi = en.y + (uint32_t)__mul24((int)__builtin_amdgcn_udot4(p, en.x, 0u, false), m8192);
    return __builtin_amdgcn_sad_u16(4u * j, S, hi);
  };
  auto answer = [&](uint32_t S, uint32_t best) -> uint32_t {
    return spal[entry_from_sad<false>(S, best & 0xFFFu)].x;
  };
  // the record of p's cell (the top byte of p is ignored everywhere): byte
  // offset 4 * cell = (R'' << 10) + (G'' << 5) + B'' with X'' = (X >> 3) << 2,
  // the bytes of m = (p >> 1) & 0x7C7C7C
  static_assert(kCellBits == 5, "cell record offset assumes 5 bits per channel");
  auto cell_rec = [&](uint32_t p) -> uint32_t {
    const uint32_t m = (p >> 1) & 0x7C7C7Cu;
    const uint32_t off = ((m >> 16) << 10) + __builtin_amdgcn_udot4(m, 0x00002001u, 0u, false);
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(stab) + off);
  };
  auto start_of = [&](uint32_t p) -> uint32_t {   // R + G + B in one dot4
    return slut[__builtin_amdgcn_udot4(p, 0x00010101u, 0u, false)];
  };
  // the exact answer for a pixel of a cell with 2 or more candidates
  auto resolve = [&](uint32_t p, uint32_t r) -> uint32_t {
    const uint32_t S = start_of(p);
    if (r & 0x40000000u) {   // 2-3 inline candidates (unused slots repeat the first)
      const uint32_t j0 = r & 0x3FFu, j1 = (r >> 10) & 0x3FFu, j2 = (r >> 20) & 0x3FFu;
      const uint32_t q0 = spal[j0].x, q1 = spal[j1].x, q2 = spal[j2].x;
      const uint32_t k0 = key(p, S, j0), k1 = key(p, S, j1), k2 = key(p, S, j2);
      // keys of distinct entries differ (the tie field is |4j - S|, S odd):
      // the answer is the winning candidate's own entry
      const uint32_t best = min(k0, min(k1, k2));
      return best == k0 ? q0 : (best == k1 ? q1 : q2);
    }
    const uint32_t cnt = (r >> 16) & 0x3Fu;
    uint32_t best = 0xFFFFFFFFu;
    if (cnt == 63u) {
      for (int j = 0; j < k; ++j) best = min(best, key(p, S, (uint32_t)j));
    } else {
      const uint32_t row = (r & 0xFFFFu) * (kCellCap / 8);   // 8 u16 per 16 B
      const u32x4 f8 = gidx4[row];
      const uint32_t l8[8] = {f8[0] & 0xFFFFu, f8[0] >> 16, f8[1] & 0xFFFFu, f8[1] >> 16,
                              f8[2] & 0xFFFFu, f8[2] >> 16, f8[3] & 0xFFFFu, f8[3] >> 16};
#pragma unroll
      for (uint32_t m = 0; m < 8; ++m)
        if (m < cnt) best = min(best, key(p, S, l8[m]));
      for (uint32_t m = 8; m < cnt; ++m) best = min(best, key(p, S, gidx[(r & 0xFFFFu) * kCellCap + m]));
    }
    return answer(S, best);
  };

  // the pixels of the next kMapPf iterations are in flight while one
  // iteration's are mapped: kMapPf register buffers, used in turn (the
  // iteration reloads the buffer it consumed)
  auto noop_stores = [&]() {   // an iteration's two stores, as no-ops (kOOB)
    __builtin_amdgcn_raw_buffer_store_b128((u32x4){0u, 0u, 0u, 0u}, orsrc, (int)kOOB, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128((u32x4){0u, 0u, 0u, 0u}, orsrc, (int)kOOB, 0, 0);
  };
  auto iter = [&](uint32_t gb, u32x4& ca, u32x4& cb) {
    const uint32_t g = gb + threadIdx.x;
    // (the lane's pixels 0-3 / 4-7: chunk(g, 0) / chunk(g, 1))
    const bool have_a = bgr ? g < g1 : chunk(g, 0) < 2u * g1;
    const bool have_b = bgr ? g < g1 : chunk(g, 1) < 2u * g1;
    uint32_t px[kMapPx];
    {
      // a copy of the loads issued kMapPf iterations ago, made HERE (the asm
      // makes it a value of its own): left to the compiler, the loop-carried
      // copy sat at the end of the iteration and waited there for the loads
      // the iteration had just issued
      u32x4 a = ca, b = cb;
      asm volatile("" : "+v"(a), "+v"(b));
      load_group(g + kMapPf * kMapLdsBlock, ca, cb);
      if (bgr) {
        const u32x4 lo = bgr12_to_px4(a[0], a[1], a[2]), hi = bgr12_to_px4(a[3], b[0], b[1]);
#pragma unroll
        for (int e = 0; e < 4; ++e) { px[e] = lo[e]; px[4 + e] = hi[e]; }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) { px[e] = a[e]; px[4 + e] = b[e]; }
      }
    }
    uint32_t res[kMapPx], rec[kMapPx];
#pragma unroll
    for (int e = 0; e < kMapPx; ++e) rec[e] = cell_rec(px[e]);
#pragma unroll
    for (int e = 0; e < kMapPx; ++e) {
      // branch-free (every pixel's reads in flight together); a pixel whose
      // cell is not 2-3 inline candidates reads entry 0 and LUT entry 0 --
      // one broadcast address, no bank conflicts -- and keeps its answer
      const uint32_t r0 = rec[e];
      const bool inl = (r0 >> 30) == 1u;
      const uint32_t r = inl ? r0 : 0u, p = inl ? px[e] : 0u;
      const uint32_t S = start_of(p);
      const uint32_t j0 = r & 0x3FFu, j1 = (r >> 10) & 0x3FFu, j2 = (r >> 20) & 0x3FFu;
      const uint32_t q0 = spal[j0].x, q1 = spal[j1].x, q2 = spal[j2].x;
      const uint32_t k0 = key(p, S, j0), k1 = key(p, S, j1), k2 = key(p, S, j2);
      // keys of distinct entries differ (the tie field is |4j - S|, S odd):
      // the answer is the winning candidate's own entry
      const uint32_t best = min(k0, min(k1, k2));
      const uint32_t qi = best == k0 ? q0 : (best == k1 ? q1 : q2);
      res[e] = inl ? qi : (r0 & 0xFFFFFFu);   // (one candidate: its colour)
    }
    // cells with more candidates: queue (lane order: an exclusive scan of the
    // lanes' counts), resolve cooperatively, read back
    uint32_t ovm = 0;
#pragma unroll
    for (int e = 0; e < kMapPx; ++e) ovm |= (uint32_t)((rec[e] >> 30) == 0) << e;
    ovm &= (have_a ? 0x0Fu : 0u) | (have_b ? 0xF0u : 0u);
    const uint32_t cnt = (uint32_t)__builtin_popcount(ovm);
    uint32_t inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += u;
    }
    const uint32_t qn = __shfl(inc, 63, 64);
    if (qn > 0) {   // wave-uniform
      const uint32_t pos0 = inc - cnt;   // this lane's first queue position
      {
        uint32_t pos = pos0;
#pragma unroll
        for (int e = 0; e < kMapPx; ++e) {
          const bool ov = (ovm >> e) & 1u;
          if (ov && pos < (uint32_t)kMapQ) wq[pos] = px[e];
          pos += ov ? 1u : 0u;
        }
      }
      wave_lds_sync();
      if (lane < min(qn, (uint32_t)kMapQ)) {
        const uint32_t p = wq[lane];
        wq[lane] = resolve(p, cell_rec(p));
      }
      wave_lds_sync();
      uint32_t pos = pos0;
#pragma unroll
      for (int e = 0; e < kMapPx; ++e) {
        const bool ov = (ovm >> e) & 1u;
        if (ov) res[e] = pos < (uint32_t)kMapQ ? wq[pos] : resolve(px[e], rec[e]);   // (queue full: in lane)
        pos += ov ? 1u : 0u;
      }
      wave_lds_sync();
    }
    {
      // (nontemporal, aux bit 1: streamed past the caches -- the next call's
      // root pass found its frame in L2 / MALL instead of the map's output)
      const int oa = (int)(have_a ? 16u * (bgr ? 2u * g : chunk(g, 0)) : kOOB);
      const int ob = (int)(have_b ? 16u * (bgr ? 2u * g + 1u : chunk(g, 1)) : kOOB);
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){res[0], res[1], res[2], res[3]}, orsrc, oa, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){res[4], res[5], res[6], res[7]}, orsrc, ob, 0, 2);
    }
  };
  // (the prologue issues what an iteration issues after its loads, so the
  // loop's top waits for the same count of operations on entry and after
  // an iteration: its own buffer's loads only)
  u32x4 na = (u32x4){0u, 0u, 0u, 0u}, nb = na, ma = na, mb = na;
  load_group(g0 + threadIdx.x, na, nb);
  noop_stores();
  if (kMapPf == 2) {
    load_group(g0 + kMapLdsBlock + threadIdx.x, ma, mb);
    noop_stores();
  }
  for (uint32_t gb = g0; gb < g1; gb += kMapPf * kMapLdsBlock) {
    iter(gb, na, nb);
    if (kMapPf == 1 || gb + kMapLdsBlock >= g1) continue;   // (uniform)
    iter(gb + kMapLdsBlock, ma, mb);
  }
  // tail (n % kMapPx points): the task's first workgroup, whole palette
  const uint32_t t = ngrp * kMapPx + threadIdx.x;
  if (lb == 0 && t < n) {
    typedef const __attribute__((address_space(1))) uint8_t g_cu8;
    g_cu8* b8 = (g_cu8*)tk.in;
    const uint32_t p = bgr ? ((uint32_t)b8[3 * t + 2] << 16) | ((uint32_t)b8[3 * t + 1] << 8) | b8[3 * t]
                           : as_g(tk.in)[t] & 0xFFFFFFu;
    const uint32_t S = start_of(p);
    uint32_t best = 0xFFFFFFFFu;
    for (int j = 0; j < k; ++j) best = min(best, key(p, S, (uint32_t)j));
    as_gw(tk.out)[t] = answer(S, best);
  }
}

// The cursor scan of one record's tiles from their per-(tile, wave) counts
// (launch_fix_cursors).
__global__ __launch_bounds__(kEpiBlock) void cursor_scan_kernel(Tile* tiles, const uint32_t* wp, int ntiles) {
  __shared__ uint64_t s_tot[kEpiBlock / 64];
  block_cursors<kEpiBlock>(tiles, wp, 0, ntiles, s_tot);
}

// ---------------------------------------------------------------------------
// Launchers.
void launch_fix_cursors(const RoundArgs& a, int ntiles, hipStream_t stream) {
  if (ntiles <= 0) return;
  pass_kernel<PASS_SPLIT><<<dim3(ntiles), dim3(kBlock), 0, stream>>>(a);
  cursor_scan_kernel<<<dim3(1), dim3(kEpiBlock), 0, stream>>>(a.tiles, a.wparts, ntiles);
}

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

void launch_kpass(int kind, const RoundArgs& a, int ntiles, hipStream_t stream) {
  if (ntiles <= 0) return;
  const dim3 g(ntiles), b(kBlock);
  if (kind == PASS_KLAST) kpass_kernel<PASS_KLAST><<<g, b, 0, stream>>>(a);
  else kpass_kernel<PASS_KMEANS><<<g, b, 0, stream>>>(a);
}

void launch_kpersist(const RoundArgs& a, int ntiles, int max_iters, hipStream_t stream) {
  if (ntiles <= 0) return;
  kpersist_kernel<<<dim3(ntiles), dim3(kBlock), 0, stream>>>(a, max_iters);
}

void launch_epilogue(int kind, const RoundArgs& a, int nnodes, hipStream_t stream) {
  if (nnodes <= 0) return;
  const dim3 g(nnodes), b(kEpiBlock);
#define DQ_EPI(MODE)                                                                \
  switch (kind) {                                                                   \
    case PASS_INIT: epilogue_kernel<PASS_INIT, MODE><<<g, b, 0, stream>>>(a); break;   \
    case PASS_SPLIT: epilogue_kernel<PASS_SPLIT, MODE><<<g, b, 0, stream>>>(a); break; \
    case PASS_KMEANS: epilogue_kernel<PASS_KMEANS, MODE><<<g, b, 0, stream>>>(a); break; \
    default: epilogue_kernel<PASS_KLAST, MODE><<<g, b, 0, stream>>>(a); break;          \
  }
  if (a.tot_mode == TOT_ALLREDUCE) DQ_EPI(TOT_ALLREDUCE)
  else if (a.tot_mode == TOT_NODE) DQ_EPI(TOT_NODE)
  else DQ_EPI(TOT_OWN)
#undef DQ_EPI
}

void launch_nodesum(int kind, const RoundArgs& a, int nlogical, hipStream_t stream) {
  if (nlogical <= 0) return;
  const dim3 g(nlogical), b(kBlock);
  switch (kind) {
    case PASS_INIT: nodesum_kernel<PASS_INIT><<<g, b, 0, stream>>>(a); break;
    case PASS_SPLIT: nodesum_kernel<PASS_SPLIT><<<g, b, 0, stream>>>(a); break;
    case PASS_KMEANS: nodesum_kernel<PASS_KMEANS><<<g, b, 0, stream>>>(a); break;
    default: nodesum_kernel<PASS_KLAST><<<g, b, 0, stream>>>(a); break;
  }
}

template <int MODE>
static void partsplit_fmt(const RoundArgs& a, int nptiles, int fmt, hipStream_t stream) {
  const dim3 g(nptiles), b(kBlock);
  switch (fmt) {
    case FMT_PLANAR: partsplit_kernel<MODE, FMT_PLANAR><<<g, b, 0, stream>>>(a); break;
    case FMT_BGR: partsplit_kernel<MODE, FMT_BGR><<<g, b, 0, stream>>>(a); break;
    case FMT_PACKED: partsplit_kernel<MODE, FMT_PACKED><<<g, b, 0, stream>>>(a); break;
    default: partsplit_kernel<MODE, FMT_ANY><<<g, b, 0, stream>>>(a); break;
  }
}

void launch_partsplit(const RoundArgs& a, int nptiles, int fmt, hipStream_t stream) {
  if (nptiles <= 0) return;
  switch (a.ps_mode) {
    case PS_STATS: partsplit_fmt<PS_STATS>(a, nptiles, fmt, stream); break;
    case PS_LATE: partsplit_fmt<PS_LATE>(a, nptiles, fmt, stream); break;
    case PS_WRITE: partsplit_fmt<PS_WRITE>(a, nptiles, fmt, stream); break;
    default: partsplit_fmt<PS_FULL>(a, nptiles, fmt, stream); break;
  }
}

void launch_kloop(const RoundArgs& a, int nrec, int max_iters, hipStream_t stream) {
  if (nrec <= 0) return;
  kloop_kernel<<<dim3(nrec), dim3(kLoopBlock), 0, stream>>>(a, max_iters);
}

template <int MODE>
static void plansplit_fmt(const PlanArgs& pa, const RoundArgs& a, int grid, int fmt, hipStream_t stream) {
  const dim3 g(grid), b(kBlock);
  switch (fmt) {
    case FMT_PLANAR: plansplit_kernel<MODE, FMT_PLANAR><<<g, b, 0, stream>>>(pa, a); break;
    case FMT_BGR: plansplit_kernel<MODE, FMT_BGR><<<g, b, 0, stream>>>(pa, a); break;
    case FMT_PACKED: plansplit_kernel<MODE, FMT_PACKED><<<g, b, 0, stream>>>(pa, a); break;
    default: plansplit_kernel<MODE, FMT_ANY><<<g, b, 0, stream>>>(pa, a); break;
  }
}

void launch_plansplit(const PlanArgs& pa, const RoundArgs& a, int grid, int fmt, hipStream_t stream) {
  if (grid <= 0) return;
  if (a.ps_mode == PS_STATS) plansplit_fmt<PS_STATS>(pa, a, grid, fmt, stream);
  else plansplit_fmt<PS_FULL>(pa, a, grid, fmt, stream);
}

void launch_plan(const PlanArgs& a, hipStream_t stream) {
  const uint32_t nb_rec = (uint32_t)max(1, (a.np * a.nshard + kPlanBlock - 1) / kPlanBlock);
  uint32_t nb_tile = (max(a.tiles_cap, a.ptiles_cap) + kPlanBlock - 1) / kPlanBlock;
  if (a.nshard > 1) {   // (grid-stride tile workgroups: see plan_kernel (2b))
    nb_tile = min(nb_tile, (uint32_t)kPlanShardTileWgs);
    plan_kernel<true><<<dim3(nb_rec + nb_tile), dim3(kPlanBlock), 0, stream>>>(a, nb_rec);
  } else {
    plan_kernel<false><<<dim3(nb_rec + nb_tile), dim3(kPlanBlock), 0, stream>>>(a, nb_rec);
  }
}

void launch_zero(void* dst, size_t bytes, hipStream_t stream) {
  const uint32_t n16 = (uint32_t)(bytes / 16);
  if (n16 == 0) return;
  const uint32_t nb = min(1024u, (n16 + 255u) / 256u);
  zero_kernel<<<dim3(nb), dim3(256), 0, stream>>>((u32x4*)dst, n16);
}

void launch_sum_u64(const SumSrcs& s, int nsrc, uint64_t* dst, size_t count, hipStream_t stream) {
  if (count == 0) return;
  const uint32_t nb = (uint32_t)std::min<size_t>(256, (count + 255) / 256);
  sum_u64_kernel<<<dim3(nb), dim3(256), 0, stream>>>(s, nsrc, dst, (uint32_t)count);
}

void launch_upload(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  const uint32_t n16 = (uint32_t)((bytes + 15) / 16);
  if (n16 == 0) return;
  const uint32_t nb = min(256u, (n16 + 255u) / 256u);
  upload_kernel<<<dim3(nb), dim3(256), 0, stream>>>((u32x4*)dst, (const u32x4*)src, n16);
}

void launch_build_cells(const MapTask* tasks, int ntasks, int kmax, hipStream_t stream) {
  if (ntasks <= 0) return;
  static bool attr = false;
  if (!attr) {   // palettes up to 16384 entries: up to 96 KB of dynamic LDS beside 32 KB static
    (void)hipFuncSetAttribute((const void*)build_cells_kernel<4, 8, 8>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024);
    (void)hipFuncSetAttribute((const void*)build_cells_kernel<4, 4, 4>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024);
    attr = true;
  }
  const size_t lds = (size_t)kmax * 6 + 16;
  // A few palettes (one frame per call): 4 x 4 x 4 cells per one-wave
  // workgroup -- 512 workgroups per palette instead of 128 on 256 CUs, and a
  // cubic region (32^3 colours) keeps each region's list short.  Batches
  // keep 256-thread workgroups (the palette staged once per 256 cells).
  if (ntasks * (kCells / 256) < 2 * 256)
    build_cells_kernel<4, 4, 4><<<dim3(kCells / 64, ntasks), dim3(64), lds, stream>>>(tasks);
  else
    build_cells_kernel<4, 8, 8><<<dim3(kCells / 256, ntasks), dim3(256), lds, stream>>>(tasks);
}

uint32_t map_groups_per_block(uint32_t n) {
  // ~8 groups of kMapPx pixels per lane per workgroup: 16K pixels
  (void)n;
  return 8u * kBlock;
}

void launch_map_lds(const MapTask* tasks, int ntasks, int kmax, uint32_t nblocks, bool bgr,
                    hipStream_t stream) {
  if (ntasks <= 0 || nblocks == 0) return;
  const size_t lds = (size_t)kCells * 4 + (size_t)(kMapLdsBlock / 64) * kMapQ * 4 +
                     (size_t)(kmax + 1) * 8 + 768 * 2;
  static bool attr = false;
  if (!attr) {   // more than 64 KB of dynamic LDS
    (void)hipFuncSetAttribute((const void*)map_lds_kernel<false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)map_lds_kernel<true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  if (bgr) map_lds_kernel<true><<<dim3(nblocks), dim3(kMapLdsBlock), lds, stream>>>(tasks, ntasks);
  else map_lds_kernel<false><<<dim3(nblocks), dim3(kMapLdsBlock), lds, stream>>>(tasks, ntasks);
}

void launch_map(const MapTask* tasks, int ntasks, int kmax, uint32_t nblocks, hipStream_t stream) {
  if (ntasks <= 0 || nblocks == 0) return;
  const size_t lds = (size_t)(kmax + 1) * 8 + 768 * 2;
  if (kmax <= 1024)   // 12-bit rank field in the 32-bit key
    map_kernel<false><<<dim3(nblocks), dim3(kBlock), lds, stream>>>(tasks, ntasks);
  else
    map_kernel<true><<<dim3(nblocks), dim3(kBlock), lds, stream>>>(tasks, ntasks);
}

// ---------------------------------------------------------------------------
// Block histograms (genHistogramsForBlocks, ClusteringSegmentation.cpp:420-563)
// One lane per block: the block's pixels in row-major order (clipped at the
// frame edge) are slots; a slot is a map key when it is the first occurrence
// of its colour, its insertion index = number of keys before it.  The mode is
// the key with the largest count that comes first in the histogram's
// iteration order (stl_rank_slots).  Lanes of a wave own horizontally
// adjacent blocks, so each block row is one contiguous 16-B-per-lane load.
// Two kernels: the light one settles blocks whose largest count is unique (or
// that hold one colour) and queues the rest; the ranking kernel (O(N^2)
// compares, ~5x the registers) runs over the queue only.
template <int DIM>
__device__ __forceinline__ void block_slots(const BlockHistArgs& a, uint32_t bx, uint32_t by,
                                            uint32_t* px, int* ins, uint32_t* cnt, int& d) {
  constexpr int N = DIM * DIM;
  const uint32_t x0 = bx * DIM, y0 = by * DIM;
  const uint32_t nx = min((uint32_t)DIM, a.width - x0), ny = min((uint32_t)DIM, a.height - y0);
  g_cu32* q = (g_cu32*)a.quant;
  bool valid[N];
  if (DIM == 4 && nx == 4 && ny == 4 && (a.width & 3) == 0) {
#pragma unroll
    for (int r = 0; r < DIM; ++r) {
      const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)(q + (size_t)(y0 + r) * a.width + x0);
      px[r * DIM + 0] = v.x; px[r * DIM + 1] = v.y; px[r * DIM + 2] = v.z; px[r * DIM + 3] = v.w;
#pragma unroll
      for (int c = 0; c < DIM; ++c) valid[r * DIM + c] = true;
    }
  } else {
#pragma unroll
    for (int r = 0; r < DIM; ++r)
#pragma unroll
      for (int c = 0; c < DIM; ++c) {
        const bool ok = (uint32_t)r < ny && (uint32_t)c < nx;
        valid[r * DIM + c] = ok;
        px[r * DIM + c] = ok ? q[(size_t)(y0 + r) * a.width + x0 + c] : 0u;
      }
  }
  // keys: first occurrences in slot order; counts over all valid slots
  d = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    bool first = valid[i];
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const bool same = valid[j] && px[j] == px[i];
      if (j < i && same) first = false;
      c += same ? 1u : 0u;
    }
    ins[i] = first ? d : -1;
    d += first ? 1 : 0;
    cnt[i] = c;
  }
}

template <int DIM>
__global__ __launch_bounds__(256) void block_hist_kernel(BlockHistArgs a) {
  constexpr int N = DIM * DIM;
  const uint32_t b = blockIdx.x * 256u + threadIdx.x;   // nblocks < 2^32 (host check)
  const bool live = b < a.block_w * a.block_h;
  bool queue = false;
  if (live) {
    const uint32_t by = b / a.block_w, bx = b - by * a.block_w;
    const uint32_t x0 = bx * DIM, y0 = by * DIM;
    const uint32_t nx = min((uint32_t)DIM, a.width - x0), ny = min((uint32_t)DIM, a.height - y0);
    g_cu32* q = (g_cu32*)a.quant;
    uint32_t px[N];
    uint32_t vm = 0;   // valid slots
    if (DIM == 4 && nx == 4 && ny == 4 && (a.width & 3) == 0) {
#pragma unroll
      for (int r = 0; r < DIM; ++r) {
        const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)(q + (size_t)(y0 + r) * a.width + x0);
        px[r * DIM + 0] = v.x; px[r * DIM + 1] = v.y; px[r * DIM + 2] = v.z; px[r * DIM + 3] = v.w;
      }
      vm = (1u << N) - 1u;
    } else {
#pragma unroll
      for (int r = 0; r < DIM; ++r)
#pragma unroll
        for (int c = 0; c < DIM; ++c) {
          const bool ok = (uint32_t)r < ny && (uint32_t)c < nx;
          vm |= (ok ? 1u : 0u) << (r * DIM + c);
          px[r * DIM + c] = ok ? q[(size_t)(y0 + r) * a.width + x0 + c] : 0u;
        }
    }
    // one iteration per distinct colour, in first-occurrence order
    uint32_t rem = vm, best = 0, best_c = 0, nbest = 0, d = 0;
    while (rem) {
      const int s0 = __builtin_ctz(rem);
      uint32_t k = px[0];
#pragma unroll
      for (int i = 1; i < N; ++i) k = s0 == i ? px[i] : k;
      uint32_t m = 0;
#pragma unroll
      for (int i = 0; i < N; ++i) m |= (px[i] == k ? 1u : 0u) << i;
      m &= rem;
      const uint32_t c = (uint32_t)__popc(m);
      rem &= ~m;
      ++d;
      if (c > best_c) {
        best = k;
        best_c = c;
        nbest = 1;
      } else if (c == best_c) {
        ++nbest;
      }
    }
    queue = d > 1 && (nbest > 1 || a.keys);   // needs the iteration order
    if (!queue) {
      // one colour (the reference's all-same shortcut, :509-520) or a unique maximum
      a.mode[b] = best;
      if (a.ndistinct) a.ndistinct[b] = d;
      if (a.keys) {   // d == 1 here
        a.keys[(uint64_t)b * N] = best;
        a.counts[(uint64_t)b * N] = best_c;
      }
    }
  }
  // one atomic per wave on one of kBhQueues counters (a single counter
  // serialises ~8K same-address atomics per 4K frame: ~50 us, dq_kernels.h)
  const uint64_t m = __ballot(queue);
  if (m == 0) return;
  const uint32_t lane = __lane_id(), qi = blockIdx.x % kBhQueues;
  uint32_t base = 0;
  if (lane == (uint32_t)__builtin_ctzll(m))
    base = atomicAdd(a.work_n + qi * kBhQueueStride, (uint32_t)__popcll(m));
  base = __shfl(base, __builtin_ctzll(m));
  if (queue) a.work[qi * a.queue_cap + base + __popcll(m & ((1ull << lane) - 1))] = b;
}

template <int DIM>
__global__ __launch_bounds__(256) void block_rank_kernel(BlockHistArgs a) {
  constexpr int N = DIM * DIM;
  const uint32_t w = blockIdx.x * 256u + threadIdx.x, qi = blockIdx.y;
  if (w >= a.work_n[qi * kBhQueueStride]) return;
  const uint32_t b = a.work[qi * a.queue_cap + w];
  const uint32_t by = b / a.block_w, bx = b - by * a.block_w;
  uint32_t px[N], cnt[N];
  int ins[N], d, rank[N];
  block_slots<DIM>(a, bx, by, px, ins, cnt, d);
  stl_rank_slots<N>(px, ins, d, rank);
  uint32_t best = px[0], best_c = 0;
  int best_r = N;
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (ins[i] >= 0 && (cnt[i] > best_c || (cnt[i] == best_c && rank[i] < best_r))) {
      best = px[i];
      best_c = cnt[i];
      best_r = rank[i];
    }
  a.mode[b] = best;
  if (a.ndistinct) a.ndistinct[b] = (uint32_t)d;
  if (a.keys) {
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (ins[i] >= 0) {
        a.keys[(uint64_t)b * N + rank[i]] = px[i];
        a.counts[(uint64_t)b * N + rank[i]] = cnt[i];
      }
  }
}

template <int DIM>
static void launch_block_hist_dim(const BlockHistArgs& a, dim3 grid, hipStream_t stream) {
  block_hist_kernel<DIM><<<grid, dim3(256), 0, stream>>>(a);
  block_rank_kernel<DIM><<<dim3((a.queue_cap + 255) / 256, kBhQueues), dim3(256), 0, stream>>>(a);
}

size_t block_hist_scratch_words(uint32_t block_w, uint32_t block_h) {
  const uint64_t nwg = ((uint64_t)block_w * block_h + 255) / 256;
  return (size_t)kBhQueues * kBhQueueStride + (size_t)kBhQueues * ((nwg + kBhQueues - 1) / kBhQueues) * 256;
}

int launch_block_hist(const BlockHistArgs& a0, int dim, hipStream_t stream) {
  const uint64_t nb = (uint64_t)a0.block_w * a0.block_h;
  if (nb == 0) return 0;
  BlockHistArgs a = a0;   // a.work_n: kBhQueues counters, then the queues
  const uint64_t nwg = (nb + 255) / 256;
  a.queue_cap = (uint32_t)(((nwg + kBhQueues - 1) / kBhQueues) * 256);
  a.work = a.work_n + kBhQueues * kBhQueueStride;
  if (hipMemsetAsync(a.work_n, 0, (size_t)kBhQueues * kBhQueueStride * 4, stream) != hipSuccess)
    return -2;
  const dim3 grid((uint32_t)nwg);
  switch (dim) {
    case 1: launch_block_hist_dim<1>(a, grid, stream); break;
    case 2: launch_block_hist_dim<2>(a, grid, stream); break;
    case 3: launch_block_hist_dim<3>(a, grid, stream); break;
    case 4: launch_block_hist_dim<4>(a, grid, stream); break;
    default: return -1;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// BGR24 ingestion and output.  The app builds the u32
// frame on the CPU, pixel by pixel, from an OpenCV CV_8UC3 Mat
// (Vec3BToUID, superpixels/OpenCVUtil.h:19-27, loops at
// ClusteringSegmentation.cpp:381-395 and the region gather :1795-1800), and
// writes mapped colours back with PixelToVec3b (OpenCVUtil.h:53-59,
// ClusteringSegmentation.cpp:1812-1817).  Memory bytes of a BGR pixel are
// B, G, R; the packed word 0x00RRGGBB has the same three bytes in the same
// little-endian order plus a zero, so packing is a byte shuffle.
// Fast path (row stride, width and base 4-B aligned, output 16-B aligned):
// one lane per 4 pixels of a row, 12 B read as three dwords, 16 B written.
// HBM-bound: 7 B per pixel.  Rows are blockIdx.y (+ gridDim.y strides).
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
// Frame reads and packed writes are nontemporal (streaming: pack 12.8 ->
// 10.9 us per 4K frame); unpack's BGR stores are plain.
constexpr uint32_t kBgrRowCap = 65535u;   // grid rows; a workgroup strides over the rest (a cap
                                          // of 270 or 540 rows measured slower)


__device__ __forceinline__ void px4_to_bgr12(u32x4 p, uint32_t& w0, uint32_t& w1, uint32_t& w2) {
  w0 = __builtin_amdgcn_perm(p.y, p.x, 0x04020100u);   // B0 G0 R0 B1
  w1 = __builtin_amdgcn_perm(p.z, p.y, 0x05040201u);   // G1 R1 B2 G2
  w2 = __builtin_amdgcn_perm(p.w, p.z, 0x06050402u);   // R2 B3 G3 R3
}

template <bool FAST>
__global__ __launch_bounds__(256) void bgr24_pack_kernel(const uint8_t* __restrict__ bgr,
                                                         uint32_t width, uint32_t height,
                                                         uint32_t stride, uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;   // pixel quad (FAST) or pixel
  for (uint32_t y = blockIdx.y; y < height; y += gridDim.y) {
    const uint8_t* row = bgr + (size_t)y * stride;
    if (FAST) {
      if (4u * i >= width) return;
      const __attribute__((address_space(1))) uint32_t* r =
          (const __attribute__((address_space(1))) uint32_t*)(row + 12u * i);
      const u32x3 w = {__builtin_nontemporal_load(r), __builtin_nontemporal_load(r + 1),
                       __builtin_nontemporal_load(r + 2)};
      __builtin_nontemporal_store(bgr12_to_px4(w.x, w.y, w.z),
                                  (__attribute__((address_space(1))) u32x4*)(out + (size_t)y * width + 4u * i));
    } else {
      if (i >= width) return;
      const uint8_t* q = row + 3u * i;
      out[(size_t)y * width + i] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16);
    }
  }
}

template <bool FAST>
__global__ __launch_bounds__(256) void bgr24_unpack_kernel(const uint32_t* __restrict__ in,
                                                           uint32_t width, uint32_t height,
                                                           uint32_t stride, uint8_t* __restrict__ bgr) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  for (uint32_t y = blockIdx.y; y < height; y += gridDim.y) {
    uint8_t* row = bgr + (size_t)y * stride;
    if (FAST) {
      if (4u * i >= width) return;
      const u32x4 p = __builtin_nontemporal_load(
          (const __attribute__((address_space(1))) u32x4*)(in + (size_t)y * width + 4u * i));
      uint32_t w0, w1, w2;
      px4_to_bgr12(p, w0, w1, w2);
      const u32x3 w = {w0, w1, w2};
      *(__attribute__((address_space(1))) u32x3*)(row + 12u * i) = w;
    } else {
      if (i >= width) return;
      const uint32_t p = in[(size_t)y * width + i];
      uint8_t* q = row + 3u * i;
      q[0] = (uint8_t)p;
      q[1] = (uint8_t)(p >> 8);
      q[2] = (uint8_t)(p >> 16);
    }
  }
}

// Region gather: out[i] = Vec3BToUID(img.at<Vec3b>(c.y, c.x)) for the i-th
// Coord {uint16 x, uint16 y} (superpixels/Coord.h:30-33: one 32-bit word,
// x in the low half).
__global__ __launch_bounds__(256) void bgr24_gather_kernel(const uint8_t* __restrict__ bgr,
                                                           uint32_t stride,
                                                           const uint32_t* __restrict__ coords,
                                                           uint32_t n, uint32_t* __restrict__ out) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    const uint32_t c = coords[i];
    const uint8_t* q = bgr + (size_t)(c >> 16) * stride + 3u * (c & 0xFFFFu);
    out[i] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16);
  }
}

static bool bgr24_fast(const void* bgr, uint32_t width, uint32_t stride, const void* px) {
  return (width & 3u) == 0 && (stride & 3u) == 0 && ((uintptr_t)bgr & 3u) == 0 &&
         ((uintptr_t)px & 15u) == 0;
}

static dim3 bgr24_grid(uint32_t width, uint32_t height, bool fast) {
  const uint32_t per_row = fast ? width / 4u : width;
  return dim3((per_row + 255u) / 256u, height < kBgrRowCap ? height : kBgrRowCap);
}

void launch_bgr24_pack(const uint8_t* bgr, uint32_t width, uint32_t height, uint32_t stride,
                       uint32_t* out, hipStream_t stream) {
  const bool fast = bgr24_fast(bgr, width, stride, out);
  const dim3 g = bgr24_grid(width, height, fast);
  if (fast) bgr24_pack_kernel<true><<<g, dim3(256), 0, stream>>>(bgr, width, height, stride, out);
  else bgr24_pack_kernel<false><<<g, dim3(256), 0, stream>>>(bgr, width, height, stride, out);
}

void launch_bgr24_unpack(const uint32_t* in, uint32_t width, uint32_t height, uint32_t stride,
                         uint8_t* bgr, hipStream_t stream) {
  const bool fast = bgr24_fast(bgr, width, stride, in);
  const dim3 g = bgr24_grid(width, height, fast);
  if (fast) bgr24_unpack_kernel<true><<<g, dim3(256), 0, stream>>>(in, width, height, stride, bgr);
  else bgr24_unpack_kernel<false><<<g, dim3(256), 0, stream>>>(in, width, height, stride, bgr);
}

void launch_bgr24_gather(const uint8_t* bgr, uint32_t stride, const uint32_t* coords, uint32_t n,
                         uint32_t* out, hipStream_t stream) {
  uint32_t nwg = (n + 255u) / 256u;
  if (nwg > 65536u) nwg = 65536u;
  bgr24_gather_kernel<<<dim3(nwg), dim3(256), 0, stream>>>(bgr, stride, coords, n, out);
}

}  // namespace dq
