// dq_weighted.hip -- the weighted path of quant_recurse (allPixelsUnique = 0,
// every live app call site, ClusteringSegmentation.cpp:1803) on gfx950.
//
// quant_varpart_fast (DivQuantCluster.cpp:1133-1138) dedups the pixels with
// calc_color_table (DivQuantMapColors.cpp:82-203) and clusters the unique
// colours with weights count / N (DivQuantCluster<false,MT,true>).  Every
// weighted statistic is a SEQUENTIAL FP64 fold over a cluster's points in
// point order (:73-85, :496-517, :719-770), and the reference's weighted and
// uniform-weight outputs differ on duplicate-heavy inputs (tests/golden/
// weighted2.json: 55 of 352 cases), so this path reproduces the folds
// exactly:
//   * the colour table: radix sort of (colour, pixel index), run heads ->
//     unique colours with counts and first occurrences, a second sort by
//     (hash bucket, first occurrence descending) -- the order the reference's
//     prepended hash chains emit, weights norm * count (:184-195);
//   * wsplit_kernel: ONE workgroup per node of a round runs the node's whole
//     split -- (root) the init folds, the split pass, the local 2-means
//     iterations to a fixed point or max_iters, the FP64 epilogue, and the
//     stable partition of its points into its children's segments.  Per
//     chunk of 256 points all lanes evaluate the decisions and the products
//     (w * R, ...); lane 0 then adds them in point order (products of points
//     not taken are +0.0, which leaves a non-negative sum bit-identical).
//     The fold is sequential by definition; the nodes of a round run in
//     parallel.
// MUST be compiled with -ffp-contract=off (the Makefile does).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "dq_weighted.h"

namespace dq {

namespace {

// --- colour table ----------------------------------------------------------
__global__ void ct_keys_kernel(const uint32_t* __restrict__ px, uint32_t n, uint32_t* __restrict__ key,
                               uint32_t* __restrict__ idx) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    key[i] = px[i] & 0xFFFFFFu;
    idx[i] = i;
  }
}

__global__ void ct_heads_kernel(const uint32_t* __restrict__ skey, uint32_t n, uint32_t* __restrict__ flag) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
    flag[i] = (i == 0 || skey[i] != skey[i - 1]) ? 1u : 0u;
}

// Run heads -> unique colour u: its colour, first occurrence (the sort is
// stable, so the run's first index) and the run start; the ordering key
// (hash << 32) | ~first sorts by bucket ascending, first occurrence descending.
__global__ void ct_scatter_kernel(const uint32_t* __restrict__ skey, const uint32_t* __restrict__ sidx,
                                  const uint32_t* __restrict__ flag, const uint32_t* __restrict__ pos,
                                  uint32_t n, uint32_t* __restrict__ ucol, uint32_t* __restrict__ head,
                                  uint64_t* __restrict__ okey, uint32_t* __restrict__ oval) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    if (!flag[i]) continue;
    const uint32_t u = pos[i], c = skey[i];
    const long R = (c >> 16) & 0xFF, G = (c >> 8) & 0xFF, B = c & 0xFF;
    const uint64_t h = (uint64_t)(((R * 33023 + G * 30013 + B * 27011) & 0x7fffffff) % 20023);   // HASH, :56-62
    ucol[u] = c;
    head[u] = i;
    okey[u] = (h << 32) | (uint64_t)(0xFFFFFFFFu - sidx[i]);
    oval[u] = u;
  }
}

__global__ void ct_final_kernel(const uint32_t* __restrict__ sval, const uint32_t* __restrict__ ucol_tmp,
                                const uint32_t* __restrict__ head, uint32_t nu, uint32_t n, double norm,
                                uint32_t* __restrict__ ucol, double* __restrict__ uw) {
  for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < nu; j += gridDim.x * 256u) {
    const uint32_t u = sval[j];
    const uint32_t count = (u + 1 < nu ? head[u + 1] : n) - head[u];
    ucol[j] = ucol_tmp[u];
    uw[j] = norm * (int)count;   // weights[index] = norm_factor * bucket->value (:195)
  }
}

// --- node splits ------------------------------------------------------------
constexpr int kWBlock = 256;
enum WMode : int { W_INIT = 0, W_SPLIT, W_KM, W_KMSQ, W_SQ };

struct WDecision {
  int32_t axis;
  double cut;                 // split: new iff cut < v_axis (:473)
  double lhs, rr, rg, rb;     // 2-means: old iff lhs < rr*R + rg*G + rb*B (:683)
};

// One pass over the node's points in point order.  Chains (lane 0, in
// order): INIT: sum w*R, w*G, w*B, w*(R*R), w*(G*G), w*(B*B) over all points;
// SPLIT / KM: w*R, w*G, w*B, w over the new side; KMSQ: those + w*(R*R)...;
// SQ: w*(R*R), w*(G*G), w*(B*B) over the new side.  cnt: points taken.
template <int MODE>
__device__ void wpass(const WNode& nd, const uint32_t* __restrict__ ucol, const double* __restrict__ uw,
                      const WDecision& d, double (*s_prod)[kWBlock], uint32_t* s_cnt, double acc[7],
                      uint32_t* cnt) {
  constexpr int NC = MODE == W_INIT ? 6 : (MODE == W_KMSQ ? 7 : (MODE == W_SQ ? 3 : 4));
  const uint32_t tid = threadIdx.x;
  for (uint32_t base = 0; base < nd.len; base += kWBlock) {
    const uint32_t i = base + tid;
    double p[7] = {0, 0, 0, 0, 0, 0, 0};
    bool take = false;
    if (i < nd.len) {
      const uint32_t id = nd.src[nd.off + i];
      const uint32_t c = ucol[id];
      const double w = uw[id];
      const uint32_t R = (c >> 16) & 0xFF, G = (c >> 8) & 0xFF, B = c & 0xFF;
      const double red = (double)R, green = (double)G, blue = (double)B;
      if (MODE == W_INIT) take = true;
      else if (MODE == W_SPLIT) take = d.cut < (d.axis == 0 ? red : (d.axis == 1 ? green : blue));
      else take = !(d.lhs < ((d.rr * red) + (d.rg * green) + (d.rb * blue)));
      if (take) {
        if (MODE == W_INIT) {
          p[0] = w * red; p[1] = w * green; p[2] = w * blue;
          p[3] = w * (double)(R * R); p[4] = w * (double)(G * G); p[5] = w * (double)(B * B);
        } else if (MODE == W_SQ) {
          p[0] = w * (double)(R * R); p[1] = w * (double)(G * G); p[2] = w * (double)(B * B);
        } else {
          p[0] = w * red; p[1] = w * green; p[2] = w * blue; p[3] = w;
          if (MODE == W_KMSQ) {
            p[4] = w * (double)(R * R); p[5] = w * (double)(G * G); p[6] = w * (double)(B * B);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) s_prod[k][tid] = p[k];
    const uint64_t m = __ballot(take);
    if ((tid & 63) == 0) s_cnt[tid >> 6] = (uint32_t)__popcll(m);
    __syncthreads();
    if (tid == 0) {
      const uint32_t nj = min((uint32_t)kWBlock, nd.len - base);
      for (uint32_t j = 0; j < nj; ++j) {
#pragma unroll
        for (int k = 0; k < NC; ++k) acc[k] += s_prod[k][j];
      }
      *cnt += s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    }
    __syncthreads();
  }
}

__device__ void w_decision_from_means(const double om[3], const double nm[3], WDecision* d) {
  d->lhs = 0.5 * (om[0] * om[0] - nm[0] * nm[0] + om[1] * om[1] - nm[1] * nm[1] + om[2] * om[2] -
                  nm[2] * nm[2]);                                        // :616-619
  d->rr = om[0] - nm[0];
  d->rg = om[1] - nm[1];
  d->rb = om[2] - nm[2];
}

}  // namespace

__global__ __launch_bounds__(kWBlock) void wsplit_kernel(WArgs a) {
  const WNode nd = a.nodes[blockIdx.x];
  __shared__ double s_prod[7][kWBlock];
  __shared__ uint32_t s_cnt[kWBlock / 64];
  __shared__ WDecision s_dec;
  __shared__ uint32_t s_flag;
  __shared__ uint32_t s_wc[kWBlock / 64][2];
  const uint32_t tid = threadIdx.x;
  // lane 0's state
  double tm[3], tv[3], om[3], nm[3], nw = 0.0, ow = 0.0, nsq[3] = {0, 0, 0};
  double prev[4] = {0, 0, 0, 0};
  uint32_t n_new = 0;
  const double tw = nd.tw;
  int done_it = -1;
  // (root) DivQuantClusterInitMeanAndVar, weighted (:49-104)
  if (nd.root) {
    double acc[7] = {0, 0, 0, 0, 0, 0, 0};
    uint32_t cnt = 0;
    wpass<W_INIT>(nd, a.ucol, a.uw, s_dec, s_prod, s_cnt, acc, &cnt);
    if (tid == 0)
      for (int c = 0; c < 3; ++c) {
        tm[c] = acc[c];
        tv[c] = acc[3 + c];
        tv[c] -= tm[c] * tm[c];   // var -= SQR(mean) (:99-101)
      }
  } else if (tid == 0) {
    for (int c = 0; c < 3; ++c) { tm[c] = nd.tm[c]; tv[c] = nd.tv[c]; }
  }
  // cut axis / position (:388-403)
  if (tid == 0) {
    double maxv = tv[0], cut = tm[0];
    int axis = 0;
    if (maxv < tv[1]) { maxv = tv[1]; axis = 1; cut = tm[1]; }
    if (maxv < tv[2]) { axis = 2; cut = tm[2]; }
    s_dec.axis = axis;
    s_dec.cut = cut;
  }
  __syncthreads();
  {   // split pass (:438-559), then :561-598
    double acc[7] = {0, 0, 0, 0, 0, 0, 0};
    uint32_t cnt = 0;
    const WDecision d = s_dec;
    wpass<W_SPLIT>(nd, a.ucol, a.uw, d, s_prod, s_cnt, acc, &cnt);
    if (tid == 0) {
      nw = acc[3];
      ow = tw - nw;
      for (int c = 0; c < 3; ++c) {
        nm[c] = acc[c];
        nm[c] /= nw;
      }
      for (int c = 0; c < 3; ++c) om[c] = (tw * tm[c] - nw * nm[c]) / ow;
      prev[0] = acc[0]; prev[1] = acc[1]; prev[2] = acc[2]; prev[3] = acc[3];
      w_decision_from_means(om, nm, &s_dec);
    }
    __syncthreads();
  }
  // local 2-means (:613-811), to a fixed point or max_iters
  for (int it = 0; it < a.max_iters; ++it) {
    const bool last = it == a.max_iters - 1;
    const WDecision d = s_dec;
    double acc[7] = {0, 0, 0, 0, 0, 0, 0};
    uint32_t cnt = 0;
    if (last) wpass<W_KMSQ>(nd, a.ucol, a.uw, d, s_prod, s_cnt, acc, &cnt);
    else wpass<W_KM>(nd, a.ucol, a.uw, d, s_prod, s_cnt, acc, &cnt);
    if (tid == 0) {
      // the state (sums, weight) equal to the previous pass's: every later
      // iteration recomputes the same means and decision (a fixed point)
      const bool fixed = a.fixed_point && !last &&
                         __double_as_longlong(acc[0]) == __double_as_longlong(prev[0]) &&
                         __double_as_longlong(acc[1]) == __double_as_longlong(prev[1]) &&
                         __double_as_longlong(acc[2]) == __double_as_longlong(prev[2]) &&
                         __double_as_longlong(acc[3]) == __double_as_longlong(prev[3]);
      nw = acc[3];
      n_new = cnt;
      for (int c = 0; c < 3; ++c) {
        nm[c] = acc[c];
        nm[c] /= nw;                                             // :800-802
      }
      ow = tw - nw;                                              // :805
      for (int c = 0; c < 3; ++c) om[c] = (tw * tm[c] - nw * nm[c]) / ow;   // :808-810
      for (int c = 0; c < 3; ++c) nsq[c] = acc[4 + c];
      for (int c = 0; c < 4; ++c) prev[c] = acc[c];
      s_flag = last ? 1u : (fixed ? 2u : 0u);
      if (!last && !fixed) w_decision_from_means(om, nm, &s_dec);   // next pass's decision
      if (last || fixed) done_it = it + 1;
    }
    __syncthreads();
    const uint32_t fl = s_flag;
    __syncthreads();
    if (fl == 2u) {   // fixed point: the sums of squares of this membership (decision d)
      double sq[7] = {0, 0, 0, 0, 0, 0, 0};
      uint32_t c2 = 0;
      wpass<W_SQ>(nd, a.ucol, a.uw, d, s_prod, s_cnt, sq, &c2);
      if (tid == 0)
        for (int c = 0; c < 3; ++c) nsq[c] = sq[c];
    }
    if (fl != 0u) break;
  }
  // results (:820-871)
  if (tid == 0) {
    NodeResult r;
    double nv[3], ov[3];
    for (int c = 0; c < 3; ++c) nv[c] = nsq[c] / nw - nm[c] * nm[c];   // :836-838
    for (int c = 0; c < 3; ++c) {
      const double dn = nm[c] - tm[c];
      const double dox = om[c] - tm[c];
      ov[c] = ((tw * tv[c] - nw * (nv[c] + dn * dn)) / ow) - dox * dox;   // :845-855
    }
    for (int c = 0; c < 3; ++c) {
      r.om[c] = om[c]; r.nm[c] = nm[c]; r.nv[c] = nv[c]; r.ov[c] = ov[c];
      r.tm[c] = tm[c]; r.tv[c] = tv[c];
    }
    r.nw = nw;
    r.ow = ow;
    r.tse_old = ow * (ov[0] + ov[1] + ov[2]);   // :870-871
    r.tse_new = nw * (nv[0] + nv[1] + nv[2]);
    r.n_new = n_new;
    r.n_new_local = n_new;
    r.done_it = done_it;
    r.proven = 0;
    r.pad = 0;
    r.len_local = nd.len;
    r.tag = 0;
    a.res[blockIdx.x] = r;
  }
  // stable partition of the points by the final decision: old half first
  // (point order kept in both halves: the reference's gather visits
  // member[] in index order, :894-1026)
  __syncthreads();
  const WDecision d = s_dec;
  __shared__ uint32_t s_nnew;
  if (tid == 0) s_nnew = n_new;
  __syncthreads();
  const uint32_t n_old = nd.len - s_nnew;
  uint32_t run_o = 0, run_n = 0;
  const uint32_t lane = tid & 63, wv = tid >> 6;
  for (uint32_t base = 0; base < nd.len; base += kWBlock) {
    const uint32_t i = base + tid;
    const bool valid = i < nd.len;
    uint32_t id = 0;
    bool nw_side = false;
    if (valid) {
      id = nd.src[nd.off + i];
      const uint32_t c = a.ucol[id];
      const double red = (double)((c >> 16) & 0xFF), green = (double)((c >> 8) & 0xFF), blue = (double)(c & 0xFF);
      nw_side = !(d.lhs < ((d.rr * red) + (d.rg * green) + (d.rb * blue)));
    }
    const uint64_t mo = __ballot(valid && !nw_side), mn = __ballot(valid && nw_side);
    if (lane == 0) {
      s_wc[wv][0] = (uint32_t)__popcll(mo);
      s_wc[wv][1] = (uint32_t)__popcll(mn);
    }
    __syncthreads();
    uint32_t bo = run_o, bn = run_n;
    for (uint32_t w = 0; w < wv; ++w) { bo += s_wc[w][0]; bn += s_wc[w][1]; }
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    if (valid) {
      if (nw_side) nd.dst[nd.off + n_old + bn + (uint32_t)__popcll(mn & below)] = id;
      else nd.dst[nd.off + bo + (uint32_t)__popcll(mo & below)] = id;
    }
    for (uint32_t w = 0; w < kWBlock / 64; ++w) { run_o += s_wc[w][0]; run_n += s_wc[w][1]; }
    __syncthreads();
  }
}

// --- launchers ----------------------------------------------------------------
static inline uint32_t grid_for(uint32_t n) {
  const uint32_t g = (n + 255u) / 256u;
  return g == 0 ? 1u : (g > 65535u ? 65535u : g);
}

size_t color_table_scratch_bytes(uint32_t n) {
  size_t sort1 = 0, sort2 = 0, scan = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort1, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 24);
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort2, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 48);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
  const size_t tmp = std::max(sort1, std::max(sort2, scan));
  // key, idx, skey, sidx, flag, pos, ucol_tmp, head, oval, sval (u32) + okey, sokey (u64)
  return ((tmp + 255) & ~(size_t)255) + (size_t)n * (10 * 4 + 2 * 8) + 16 * 256;
}

int launch_color_table(const uint32_t* px, uint32_t n, double norm, void* scratch, size_t scratch_bytes,
                       uint32_t* ucol, double* uw, uint32_t* h_nu, hipStream_t stream) {
  size_t sort1 = 0, sort2 = 0, scan = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort1, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 24);
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort2, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 48);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
  size_t tmp = std::max(sort1, std::max(sort2, scan));
  tmp = (tmp + 255) & ~(size_t)255;
  if (scratch_bytes < color_table_scratch_bytes(n)) return -1;
  char* p = static_cast<char*>(scratch);
  void* temp = p;
  p += tmp;
  auto take32 = [&]() { uint32_t* q = reinterpret_cast<uint32_t*>(p); p += ((size_t)n * 4 + 255) & ~(size_t)255; return q; };
  auto take64 = [&]() { uint64_t* q = reinterpret_cast<uint64_t*>(p); p += ((size_t)n * 8 + 255) & ~(size_t)255; return q; };
  uint32_t *key = take32(), *idx = take32(), *skey = take32(), *sidx = take32(), *flag = take32(), *pos = take32();
  uint32_t *ucol_tmp = take32(), *head = take32(), *oval = take32(), *sval = take32();
  uint64_t *okey = take64(), *sokey = take64();
  const dim3 g(grid_for(n)), b(256);
  ct_keys_kernel<<<g, b, 0, stream>>>(px, n, key, idx);
  size_t t1 = sort1;
  if (hipcub::DeviceRadixSort::SortPairs(temp, t1, key, skey, idx, sidx, (int)n, 0, 24, stream) != hipSuccess)
    return -2;
  ct_heads_kernel<<<g, b, 0, stream>>>(skey, n, flag);
  size_t t3 = scan;
  if (hipcub::DeviceScan::ExclusiveSum(temp, t3, flag, pos, (int)n, stream) != hipSuccess) return -2;
  // U = pos[n-1] + flag[n-1]
  uint32_t last[2];
  if (hipMemcpyAsync(&last[0], pos + n - 1, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipMemcpyAsync(&last[1], flag + n - 1, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return -2;
  const uint32_t nu = last[0] + last[1];
  ct_scatter_kernel<<<g, b, 0, stream>>>(skey, sidx, flag, pos, n, ucol_tmp, head, okey, oval);
  size_t t2 = sort2;
  if (hipcub::DeviceRadixSort::SortPairs(temp, t2, okey, sokey, oval, sval, (int)nu, 0, 48, stream) != hipSuccess)
    return -2;
  ct_final_kernel<<<dim3(grid_for(nu)), b, 0, stream>>>(sval, ucol_tmp, head, nu, n, norm, ucol, uw);
  *h_nu = nu;
  return 0;
}

__global__ void iota_kernel(uint32_t* __restrict__ dst, uint32_t n) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) dst[i] = i;
}

// One output point per lane, grid-stride: the row / column split of t is one
// 32-bit division per point (nr * nc < 2^32); an HBM gather (4 B read at the
// decimated index, 4 B written), not worth an LDS stage.
__global__ __launch_bounds__(256) void cut_gather_kernel(const uint32_t* in,
                                                         uint32_t* out, uint32_t nr,
                                                         uint32_t nc, uint32_t dec, uint32_t stride,
                                                         uint32_t sr, uint32_t sg, uint32_t sb) {
  const uint32_t n = nr * nc;
  for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < n; t += gridDim.x * 256u) {
    const uint32_t a = t / nc, b = t - a * nc;
    const uint64_t i = (uint64_t)b * dec + (uint64_t)a * dec * stride;
    const uint32_t p = __builtin_nontemporal_load(in + i);
    out[t] = ((((p >> 16) & 0xFFu) >> sr) << 16) | ((((p >> 8) & 0xFFu) >> sg) << 8) | ((p & 0xFFu) >> sb);
  }
}

void launch_cut_gather(const uint32_t* in, uint32_t* out, uint32_t nr, uint32_t nc, uint32_t dec,
                       uint32_t stride, uint32_t sr, uint32_t sg, uint32_t sb, hipStream_t stream) {
  if ((uint64_t)nr * nc == 0) return;
  cut_gather_kernel<<<dim3(grid_for(nr * nc)), dim3(256), 0, stream>>>(in, out, nr, nc, dec, stride, sr, sg, sb);
}

void launch_iota(uint32_t* dst, uint32_t n, hipStream_t stream) {
  if (n == 0) return;
  iota_kernel<<<dim3(grid_for(n)), dim3(256), 0, stream>>>(dst, n);
}

void launch_wsplit(const WArgs& a, int nnodes, hipStream_t stream) {
  if (nnodes <= 0) return;
  wsplit_kernel<<<dim3(nnodes), dim3(kWBlock), 0, stream>>>(a);
}

}  // namespace dq
