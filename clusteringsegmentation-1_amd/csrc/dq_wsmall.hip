// dq_wsmall.hip -- the weighted quant_recurse of a small input (a superpixel
// region) in ONE workgroup, one launch (dq_weighted.h, launch_wsmall).
//
// ClusteringSegmentation.cpp:1779-1803 calls quant_recurse(N_region, .., K=4,
// allPixelsUnique=0) once per region, 10^3-10^5 pixels each.  The multi-kernel
// weighted path (dq_weighted.hip) spends ~1 ms per call there in launches and
// host round trips (tools/weighted_regions.py), while the reference needs
// 30-1000 us on one core.  Here one 1024-thread workgroup does the whole call:
//   A. calc_color_table (DivQuantMapColors.cpp:82-203): an LDS hash set of the
//      colours with counts and first occurrences, then a counting sort by hash
//      bucket and, inside a bucket, first occurrence descending -- the order
//      the reference's prepended chains emit -- into (colour | count << 32)
//      records, weights norm * count (:195);
//   B. DivQuantCluster<false,*,true> (DivQuantCluster.cpp:133-1097) split by
//      split in the reference's own order: the init folds, the split pass, the
//      2-means passes to the exact fixed point or max_iters, the FP64 epilogue,
//      a stable partition of the node's records (point order kept: the
//      reference gathers by ascending index), and STEP 4's greedy choice.
//      Every statistic is a SEQUENTIAL FP64 fold in point order, as the
//      reference's: 15 waves compute a chunk's summands into LDS while lanes
//      0-6 of wave 0 -- one per fold -- add the previous chunk's, one
//      v_add_f64 per summand in point order (exact integer runs of 64
//      summands, dq_weighted.hip's "exact parallel fold", measured slower at
//      these sizes: their scans and checks cost about 25 adds per run);
//   C. the final centres (:1029-1096), the first-occurrence dedup
//      (quant_util.cpp:93-118) and, for at most kWsMapMax deduped colours,
//      map_colors_mps: the palette sorted by R+G+B -- for <= 16 entries
//      libstdc++'s std::sort is its insertion sort, which is stable -- the
//      rounded-midpoint lut_init (:331-383), and per pixel the argmin over
//      (squared distance, MPS visit rank), the walk's answer.
// MUST be compiled with -ffp-contract=off (the Makefile does): every FP64
// expression mirrors the reference's operation by operation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>

#include "dq_weighted.h"

namespace dq {

namespace {

constexpr int kWsThreads = 1024;
constexpr int kWsWaves = kWsThreads / 64;
constexpr uint32_t kWsTable = 8192;               // hash slots: <= kWsMaxU + 1024 in flight, always a free one
constexpr uint32_t kWsBuckets = 20023;            // HASH_SIZE (DivQuantMapColors.cpp:56-62)
constexpr uint32_t kWsHistWords = (kWsBuckets + 1) / 2;   // two 16-bit bucket counts per word
constexpr uint32_t kWsBucketsPer = 20;            // buckets per thread in the scan (even: whole words)
constexpr size_t kWsBuf = (size_t)kWsMaxU * 8;    // one record buffer
constexpr size_t kWsOffB = kWsBuf;                // LDS [48K, 96K): bucket-sorted entries, then records B
constexpr size_t kWsOffA = 2 * kWsBuf;            // LDS [96K, 144K): dense entries, then records A
constexpr size_t kWsLds = 3 * kWsBuf;
static_assert(3 * (size_t)kWsTable * 4 <= kWsOffA, "the hash table lies below buffer A");
static_assert((size_t)kWsHistWords * 4 <= kWsOffB, "the bucket counts lie below buffer B");
static_assert(kWsBucketsPer * kWsThreads >= kWsBuckets && kWsBucketsPer % 2 == 0, "bucket scan ownership");
static_assert(kWsMaxN < (1u << 17), "first occurrences in 17 bits");
static_assert(kWsMaxU <= 65535, "16-bit bucket bases");

enum : int32_t { WS_INIT = 0, WS_SPLIT = 1, WS_KM = 2 };
constexpr uint32_t kWsSeqChunk = 368;   // points per summand chunk of a fold pass

// the reference's per-cluster-index arrays (weight[], size[], mean[], var[],
// tse[], zero-initialised, :287-314) plus where the cluster's points lie
struct WsClu {
  uint32_t off, len;
  int32_t buf;                // 0: records A, 1: records B
  int32_t lo[3], hi[3];       // a box holding every point (the split proof)
  int32_t pad;
  double w, tse;
  double mean[3], var[3];
  int64_t size;
};

// the split in progress (thread 0 writes, every thread reads after a barrier)
struct WsCtl {
  int32_t old_index, kind, axis, fkind;   // pass kind; the final membership's kind
  int32_t done, proven, it, status;
  uint32_t off, len, n_new, cnt;
  int32_t src, over;
  uint32_t nu, ndense;
  double tw, cut, lhs, rr, rg, rb;
  double tm[3], tv[3], nm[3], om[3], nsq[3], prev[4];
  double nw, ow;
  double acc[8];
  uint32_t passes;
  uint64_t t_pass, t_part, nkind;   // profile: ticks in passes / partitions, passes by kind
};

__device__ __forceinline__ int ws_binade(double v) {   // exponent of a positive normal double
  return (int)((__double_as_longlong(v) >> 52) & 0x7FF) - 1023;
}

// the pass's membership: init -- every point; split -- cut < v_axis (:473);
// 2-means -- the new side, !(lhs < rr*R + rg*G + rb*B) (:683)
__device__ __forceinline__ bool ws_take(int kind, int axis, double cut, double lhs, double rr, double rg,
                                        double rb, uint32_t R, uint32_t G, uint32_t B) {
  if (kind == WS_INIT) return true;
  const double red = (double)R, green = (double)G, blue = (double)B;
  if (kind == WS_SPLIT) return cut < (axis == 0 ? red : (axis == 1 ? green : blue));
  return !(lhs < ((rr * red) + (rg * green) + (rb * blue)));
}

// the reference's summands (:73-85, :496-517, :719-770)
__device__ __forceinline__ double ws_prod(int ch, uint32_t R, uint32_t G, uint32_t B, double w) {
  switch (ch) {
    case 0: return w * (double)R;
    case 1: return w * (double)G;
    case 2: return w * (double)B;
    case 3: return w;
    case 4: return w * (double)(R * R);
    case 5: return w * (double)(G * G);
    default: return w * (double)(B * B);
  }
}

// Inclusive scan of a 64-bit integer over the wave by DPP (row_shr 1, 2, 4,
// 8 inside each row of 16 lanes, then row_bcast 15 and 31 across rows): six
// steps of VALU moves instead of the shuffles' LDS-crossbar round trips --
// a fold's running sum waits on every such step.
template <int CTRL, int ROWS>
__device__ __forceinline__ int64_t ws_dpp(int64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROWS, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)((uint64_t)v >> 32), CTRL, ROWS, 0xF, true);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ int64_t ws_wave_scan_i64(int64_t v) {
  v += ws_dpp<0x111, 0xF>(v);   // row_shr:1
  v += ws_dpp<0x112, 0xF>(v);   // row_shr:2
  v += ws_dpp<0x114, 0xF>(v);   // row_shr:4
  v += ws_dpp<0x118, 0xF>(v);   // row_shr:8
  v += ws_dpp<0x142, 0xA>(v);   // row_bcast:15 -> rows 1, 3
  v += ws_dpp<0x143, 0xC>(v);   // row_bcast:31 -> rows 2, 3
  return v;
}
__device__ __forceinline__ int64_t ws_readlane_i64(int64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t ws_wave_sum_i64(int64_t v) { return ws_readlane_i64(ws_wave_scan_i64(v), 63); }

__device__ __forceinline__ int32_t ws_threshold(double cut) {   // cut < v <=> v >= thr
  if (!(cut == cut)) return 256;
  if (cut < 0.0) return 0;
  if (cut >= 255.0) return 256;
  return (int32_t)floor(cut) + 1;
}

// dq_weighted.hip w_cut_is_fixed_point: the first 2-means decision keeps
// every point of the node's box on its side of the cut, so the first 2-means
// pass folds exactly the split's summands (a fixed point at once).
__device__ bool ws_cut_is_fixed_point(const WsCtl& w, const int32_t blo[3], const int32_t bhi[3]) {
  const double M = (fabs(w.rr) + fabs(w.rg) + fabs(w.rb)) * 255.0 + fabs(w.lhs);
  if (!(M > 1e-30 && M < 1e30)) return false;
  const double mg = 1e-12 * M;
  const double c[3] = {w.rr, w.rg, w.rb};
  const int thr = ws_threshold(w.cut);
  for (int side = 0; side < 2; ++side) {
    int lo[3], hi[3];
    for (int k = 0; k < 3; ++k) { lo[k] = blo[k]; hi[k] = bhi[k]; }
    if (side) lo[w.axis] = max(lo[w.axis], thr);
    else hi[w.axis] = min(hi[w.axis], thr - 1);
    if (lo[w.axis] > hi[w.axis]) continue;
    double ext = 0.0;
    for (int k = 0; k < 3; ++k) {
      const double x = c[k] * (double)lo[k], y = c[k] * (double)hi[k];
      ext += side ? fmax(x, y) : fmin(x, y);
    }
    if (side ? !(ext <= w.lhs - mg) : !(ext >= w.lhs + mg)) return false;
  }
  return true;
}

__device__ __forceinline__ void ws_decision(WsCtl& w) {   // :616-623
  w.lhs = 0.5 * (w.om[0] * w.om[0] - w.nm[0] * w.nm[0] + w.om[1] * w.om[1] - w.nm[1] * w.nm[1] +
                 w.om[2] * w.om[2] - w.nm[2] * w.nm[2]);
  w.rr = w.om[0] - w.nm[0];
  w.rg = w.om[1] - w.nm[1];
  w.rb = w.om[2] - w.nm[2];
}

// map_colors_mps (DivQuantMapColors.cpp:385-527) of px[i] for i = first,
// first + step, .. < n: the argmin over the sorted palette of (squared
// distance, visit rank of the walk from lut_init[R+G+B]) -- the walk's
// answer; rank = 2(j - s) - 1 above the start s, 2(s - j) at or
// below it; m <= kWsMapMax (the key's rank field is 6 bits).
constexpr uint32_t kWsMapInline = 16384;   // pixels mapped by wsmall_kernel itself
__device__ void ws_map(const uint32_t* px, uint32_t* out, uint32_t n, uint32_t first, uint32_t step,
                       const uint32_t* pal, const uint16_t* lut, int m) {
  constexpr int kLoads = 4;   // pixels per thread in flight
  for (uint32_t i0 = first; i0 < n; i0 += kLoads * step) {
    uint32_t ps[kLoads];
#pragma unroll
    for (int u = 0; u < kLoads; ++u) {
      const uint32_t i = i0 + (uint32_t)u * step;
      ps[u] = i < n ? px[i] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kLoads; ++u) {
      const uint32_t i = i0 + (uint32_t)u * step;
      if (i >= n) break;
      const uint32_t p = ps[u];
      const int R = (int)((p >> 16) & 0xFF), G = (int)((p >> 8) & 0xFF), B = (int)(p & 0xFF);
      const int s = lut[R + G + B];
      uint32_t best = 0xFFFFFFFFu, bj = 0;
      for (int j = 0; j < m; ++j) {
        const uint32_t q = pal[j];
        const int dr = R - (int)((q >> 16) & 0xFF), dg = G - (int)((q >> 8) & 0xFF), db = B - (int)(q & 0xFF);
        const uint32_t rank = j > s ? 2u * (uint32_t)(j - s) - 1u : 2u * (uint32_t)(s - j);
        const uint32_t key = (uint32_t)(dr * dr + dg * dg + db * db) * 64u + rank;
        if (key < best) {
          best = key;
          bj = (uint32_t)j;
        }
      }
      out[i] = pal[bj];
    }
  }
}

__device__ __forceinline__ void ws_store_status(WSmallResult* r, uint32_t v) {
  __threadfence_system();
  __hip_atomic_store(&r->status, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The whole call of one input (one workgroup); the single-call kernel and
// the batch kernel (one workgroup per region) below.
__device__ __forceinline__ void wsmall_body(const WSmallArgs& a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ WsClu clu[kWsMaxK];
  __shared__ WsCtl ctl;
  __shared__ uint32_t s_wo[kWsWaves], s_wn[kWsWaves];
  __shared__ double s_acc[8];
  __shared__ uint32_t s_pal[kWsMapMax], s_ct[kWsMaxK];
  __shared__ uint16_t s_lut[766];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t n = a.n;
  const int K = a.k;
  WSmallResult* res = a.res;

  if (tid == 0) {
    res->prof[0] = wall_clock64();
    if (a.maptab) a.maptab->go = 0;
  }
  // ---- A. calc_color_table -------------------------------------------------
  uint32_t* hkey = reinterpret_cast<uint32_t*>(lds);   // colour + 1 (0: free)
  uint32_t* hcnt = hkey + kWsTable;
  uint32_t* hfirst = hcnt + kWsTable;
  for (uint32_t s = tid; s < kWsTable; s += kWsThreads) {
    hkey[s] = 0;
    hcnt[s] = 0;
    hfirst[s] = 0xFFFFFFFFu;
  }
  if (tid == 0) {
    ctl.nu = 0;
    ctl.over = 0;
    ctl.ndense = 0;
  }
  __syncthreads();
  // Equal colours of neighbouring pixels (a region's flat areas) would queue
  // on one LDS address: a wave's run of equal colours goes in once, from its
  // first lane (the smallest index), with the run's length as its count.
  constexpr int kWsLoads = 8;   // pixels per thread in flight
  for (uint32_t i0 = tid; i0 < n; i0 += kWsLoads * kWsThreads) {
    uint32_t cs[kWsLoads];
#pragma unroll
    for (int u = 0; u < kWsLoads; ++u) {
      const uint32_t i = i0 + (uint32_t)u * kWsThreads;
      cs[u] = i < n ? a.px[i] & 0xFFFFFFu : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int u = 0; u < kWsLoads; ++u) {
      const uint32_t i = i0 + (uint32_t)u * kWsThreads, c = cs[u];
      // the lane below's colour (DPP row_shr:1; a row's first lane gets none: a head)
      const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFFu, (int)c, 0x111, 0xF, 0xF, false);
      const bool valid = i < n;
      const bool head = valid && ((lane & 15) == 0 || up != c);
      const uint64_t hm = __ballot(head), vm = __ballot(valid);
      if (vm == 0) break;
      // (bail out once more colours than the buffers hold have come in: every
      // thread then inserts at most the one key it is probing for, so the
      // table keeps free slots and every probe ends)
      if (*(volatile int32_t*)&ctl.over) break;
      if (head) {
        const uint64_t above = hm & (lane == 63 ? 0ull : (~0ull << (lane + 1)));
        const uint32_t nxt = above ? (uint32_t)__builtin_ctzll(above) : (uint32_t)__popcll(vm);
        uint32_t h = (c * 0x9E3779B1u) >> 19;
        for (;;) {
          const uint32_t k0 = hkey[h];
          if (k0 == c + 1u) break;
          if (k0 == 0u) {
            const uint32_t prev = atomicCAS(&hkey[h], 0u, c + 1u);
            if (prev == 0u) {
              if (atomicAdd(&ctl.nu, 1u) + 1u > kWsMaxU) ctl.over = 1;
              break;
            }
            if (prev == c + 1u) break;
          }
          h = (h + 1u) & (kWsTable - 1u);
        }
        atomicAdd(&hcnt[h], nxt - lane);
        atomicMin(&hfirst[h], i);
      }
    }
  }
  __syncthreads();
  if (tid == 0) res->prof[1] = wall_clock64();
  const uint32_t nu = ctl.nu;
  if (ctl.over || nu > kWsMaxU) {   // (uniform) the multi-kernel path takes it
    if (tid == 0) {
      res->nu = nu;
      ws_store_status(res, 2u);
    }
    return;
  }
  // dense entries (bucket << 17 | first) << 32 | count, in slot order
  uint64_t* dense = reinterpret_cast<uint64_t*>(lds + kWsOffA);
  for (uint32_t s = tid; s < kWsTable; s += kWsThreads) {
    const uint32_t kk = hkey[s];
    if (kk) {
      const uint32_t c = kk - 1u;
      const long R = (c >> 16) & 0xFF, G = (c >> 8) & 0xFF, B = c & 0xFF;
      const uint32_t b = (uint32_t)(((R * 33023 + G * 30013 + B * 27011) & 0x7fffffff) % 20023);   // HASH
      const uint32_t p = atomicAdd(&ctl.ndense, 1u);
      dense[p] = ((uint64_t)((b << 17) | hfirst[s]) << 32) | hcnt[s];
    }
  }
  __syncthreads();
  // counting sort by bucket: 16-bit counts, two per word
  uint32_t* hist = reinterpret_cast<uint32_t*>(lds);
  uint16_t* h16 = reinterpret_cast<uint16_t*>(lds);
  for (uint32_t w = tid; w < kWsHistWords; w += kWsThreads) hist[w] = 0;
  __syncthreads();
  for (uint32_t u = tid; u < nu; u += kWsThreads) {
    const uint32_t b = (uint32_t)(dense[u] >> 49);
    atomicAdd(&hist[b >> 1], 1u << (16 * (b & 1u)));
  }
  __syncthreads();
  {
    const uint32_t b0 = tid * kWsBucketsPer;
    uint32_t tot = 0;
    for (uint32_t b = b0; b < b0 + kWsBucketsPer && b < kWsBuckets; ++b) tot += h16[b];
    uint32_t inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += v;
    }
    if (lane == 63) s_wo[wv] = inc;
    __syncthreads();
    uint32_t run = inc - tot;
    for (uint32_t w = 0; w < wv; ++w) run += s_wo[w];
    for (uint32_t b = b0; b < b0 + kWsBucketsPer && b < kWsBuckets; ++b) {
      const uint32_t c = h16[b];
      h16[b] = (uint16_t)run;
      run += c;
    }
  }
  __syncthreads();
  uint64_t* sorted = reinterpret_cast<uint64_t*>(lds + kWsOffB);
  for (uint32_t u = tid; u < nu; u += kWsThreads) {
    const uint64_t e = dense[u];
    const uint32_t b = (uint32_t)(e >> 49), sh = 16 * (b & 1u);
    const uint32_t old = atomicAdd(&hist[b >> 1], 1u << sh);
    sorted[(old >> sh) & 0xFFFFu] = e;
  }
  __syncthreads();
  // inside a bucket: first occurrence descending (the chains are prepended,
  // :154-158); h16[b] is now the end of bucket b, h16[b - 1] its start
  uint64_t* recA = reinterpret_cast<uint64_t*>(lds + kWsOffA);
  uint64_t* recB = reinterpret_cast<uint64_t*>(lds + kWsOffB);
  for (uint32_t i = tid; i < nu; i += kWsThreads) {
    const uint64_t e = sorted[i];
    const uint32_t b = (uint32_t)(e >> 49), f = (uint32_t)(e >> 32) & 0x1FFFFu;
    const uint32_t st = b ? h16[b - 1] : 0u, en = h16[b];
    uint32_t rank = 0;
    for (uint32_t j = st; j < en; ++j) rank += ((uint32_t)(sorted[j] >> 32) & 0x1FFFFu) > f ? 1u : 0u;
    const uint32_t col = a.px[f] & 0xFFFFFFu;
    recA[st + rank] = (uint64_t)col | ((e & 0xFFFFFFFFull) << 32);
  }
  // (the writes land in dense's region: dense was last read before the barrier above)

  // ---- B. DivQuantCluster<false,*,true>, split by split -----------------------
  if (tid < (uint32_t)kWsMaxK) {
    WsClu& q = clu[tid];
    q.off = q.len = 0;
    q.buf = 0;
    for (int c = 0; c < 3; ++c) {
      q.lo[c] = 0;
      q.hi[c] = 255;
      q.mean[c] = q.var[c] = 0.0;
    }
    q.w = q.tse = 0.0;
    q.size = 0;
    if (tid == 0) {
      q.len = nu;
      q.w = 1.0;   // :329
      q.size = nu;
    }
  }
  if (tid == 0) {
    ctl.old_index = 0;
    ctl.passes = 0;
    ctl.status = 1;
    ctl.t_pass = ctl.t_part = ctl.nkind = 0;
  }
  __syncthreads();
  if (tid == 0) res->prof[2] = wall_clock64();
  const double norm = a.norm;
  // One pass's seven folds (every thread; the sums land in ctl.acc, the
  // taken points in ctl.cnt).  Waves 1-15 compute the summands of a chunk of
  // kWsSeqChunk points into LDS -- once per pass, not once per fold -- while
  // lanes 0-6 of wave 0, one per fold, add the previous chunk's in point
  // order: the reference's own adds, one dependent v_add_f64 per point and
  // fold (measured faster at these sizes than 64-summand exact runs, whose
  // per-run scan and checks cost about as much as 25 single adds).
  double* xs = reinterpret_cast<double*>(lds);   // [2][kWsSeqChunk + 16][8] (LDS [0, 48K): free in B)
  static_assert(2 * (kWsSeqChunk + 16) * 8 * sizeof(double) <= kWsOffB, "the summand chunks lie below buffer B");
  auto pass = [&](int kind) {
    const uint64_t t0 = wall_clock64();
    const uint64_t* recs = ctl.src ? recB : recA;
    const uint32_t off = ctl.off, len = ctl.len;
    const int axis = ctl.axis;
    const double cut = ctl.cut, lhs = ctl.lhs, rr = ctl.rr, rg = ctl.rg, rb = ctl.rb;
    const uint32_t nch = (len + kWsSeqChunk - 1) / kWsSeqChunk;
    double s = 0.0;
    uint32_t wc = 0;
    for (uint32_t c = 0; c <= nch; ++c) {
      if (wv != 0 && c < nch) {   // the summands of chunk c
        double* xb = xs + (size_t)(c & 1) * (kWsSeqChunk + 16) * 8;
        const uint32_t c0 = c * kWsSeqChunk, cl = min(kWsSeqChunk, len - c0);
        for (uint32_t p = tid - 64; p < cl; p += kWsThreads - 64) {
          const uint64_t r = recs[off + c0 + p];
          const uint32_t col = (uint32_t)r;
          const uint32_t R = (col >> 16) & 0xFF, G = (col >> 8) & 0xFF, B = col & 0xFF;
          const bool take = ws_take(kind, axis, cut, lhs, rr, rg, rb, R, G, B);
          const double w = norm * (int)(uint32_t)(r >> 32);   // weights[] (:195)
          double* xp = xb + (size_t)p * 8;
#pragma unroll
          for (int ch = 0; ch < 7; ++ch) xp[ch] = take ? ws_prod(ch, R, G, B, w) : 0.0;
          wc += take ? 1u : 0u;
        }
      }
      if (wv == 0 && c > 0 && lane < 7) {   // fold `lane` over chunk c - 1, in order
        // (the next 8 summands' LDS reads are issued before these 8 are
        // added; reads past the chunk land in its padding or the next
        // buffer and are never added)
        const double* xb = xs + (size_t)((c - 1) & 1) * (kWsSeqChunk + 16) * 8 + lane;
        const uint32_t cl = min(kWsSeqChunk, len - (c - 1) * kWsSeqChunk);
        // two register sets in turn (a copy between them made the compiler
        // wait for every read before the next were issued)
        constexpr uint32_t U = 8;
        double va[U], vb[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) va[u] = xb[(size_t)u * 8];
        uint32_t t = 0;
        // (sched_barrier: the scheduler merged the two read groups and then
        // waited for the first right after issuing both)
        for (; t + 2 * U <= cl; t += 2 * U) {
#pragma unroll
          for (uint32_t u = 0; u < U; ++u) vb[u] = xb[(size_t)(t + U + u) * 8];
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (uint32_t u = 0; u < U; ++u) s += va[u];
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (uint32_t u = 0; u < U; ++u) va[u] = xb[(size_t)(t + 2 * U + u) * 8];
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (uint32_t u = 0; u < U; ++u) s += vb[u];
          __builtin_amdgcn_sched_barrier(0);
        }
        // the last < 16 (va holds t .. t + 7)
        if (t + U <= cl) {
#pragma unroll
          for (uint32_t u = 0; u < U; ++u) vb[u] = xb[(size_t)(t + U + u) * 8];
#pragma unroll
          for (uint32_t u = 0; u < U; ++u) s += va[u];
          t += U;
#pragma unroll
          for (uint32_t u = 0; u < U; ++u)
            if (t + u < cl) s += vb[u];
        } else {
#pragma unroll
          for (uint32_t u = 0; u < U; ++u)
            if (t + u < cl) s += va[u];
        }
      }
      __syncthreads();
    }
    const uint32_t ws = (uint32_t)ws_wave_sum_i64((int64_t)wc);   // the taken points
    if (lane == 0) s_wo[wv] = ws;
    if (wv == 0 && lane < 7) s_acc[lane] = s;
    __syncthreads();
    if (tid == 0) {
      for (int c = 0; c < 7; ++c) ctl.acc[c] = s_acc[c];
      uint32_t cnt = 0;
      for (int w = 0; w < kWsWaves; ++w) cnt += s_wo[w];
      ctl.cnt = cnt;
      ctl.passes++;
      ctl.t_pass += wall_clock64() - t0;
      ctl.nkind += 1ull << (16 * kind);
    }
  };
  for (int new_index = 1; new_index < K; ++new_index) {
    if (tid == 0) {
      const WsClu& C = clu[ctl.old_index];
      ctl.src = C.buf;
      ctl.off = C.off;
      ctl.len = C.len;
      ctl.tw = C.w;   // total_weight = weight[old_index] (:353)
      ctl.kind = WS_INIT;
      for (int c = 0; c < 3; ++c) { ctl.tm[c] = C.mean[c]; ctl.tv[c] = C.var[c]; }
    }
    __syncthreads();
    if (new_index == 1) {   // DivQuantClusterInitMeanAndVar, weighted (:73-85, :99-101)
      pass(WS_INIT);
      if (tid == 0)
        for (int c = 0; c < 3; ++c) {
          ctl.tm[c] = ctl.acc[c];
          ctl.tv[c] = ctl.acc[4 + c];
          ctl.tv[c] -= ctl.tm[c] * ctl.tm[c];
        }
    }
    if (tid == 0) {   // the cut (:388-403)
      double maxv = ctl.tv[0], cut = ctl.tm[0];
      int axis = 0;
      if (maxv < ctl.tv[1]) { maxv = ctl.tv[1]; axis = 1; cut = ctl.tm[1]; }
      if (maxv < ctl.tv[2]) { axis = 2; cut = ctl.tm[2]; }
      ctl.axis = axis;
      ctl.cut = cut;
      ctl.kind = WS_SPLIT;
    }
    __syncthreads();
    pass(WS_SPLIT);   // (:438-559) then its epilogue (:561-598, weighted: no data_weight scaling)
    if (tid == 0) {
      WsCtl& w = ctl;
      w.nw = w.acc[3];
      w.ow = w.tw - w.nw;
      for (int c = 0; c < 3; ++c) {
        w.nm[c] = w.acc[c];
        w.nm[c] /= w.nw;
      }
      for (int c = 0; c < 3; ++c) w.om[c] = (w.tw * w.tm[c] - w.nw * w.nm[c]) / w.ow;
      for (int c = 0; c < 4; ++c) w.prev[c] = w.acc[c];
      ws_decision(w);
      w.n_new = w.cnt;
      w.it = 0;
      w.done = 0;
      w.proven = 0;
      w.fkind = WS_SPLIT;
      const WsClu& C = clu[w.old_index];
      if (a.fixed_point && w.cnt != 0 && w.ow > 0.0 && ws_cut_is_fixed_point(w, C.lo, C.hi)) {
        for (int c = 0; c < 3; ++c) w.nsq[c] = w.acc[4 + c];
        w.proven = 1;
        w.done = 1;
      } else {
        w.kind = WS_KM;
      }
    }
    __syncthreads();
    while (!ctl.done) {   // the local 2-means (:613-811)
      pass(WS_KM);
      if (tid == 0) {
        WsCtl& w = ctl;
        const bool last = w.it == a.max_iters - 1;
        const bool fixed = a.fixed_point && !last &&
                           __double_as_longlong(w.acc[0]) == __double_as_longlong(w.prev[0]) &&
                           __double_as_longlong(w.acc[1]) == __double_as_longlong(w.prev[1]) &&
                           __double_as_longlong(w.acc[2]) == __double_as_longlong(w.prev[2]) &&
                           __double_as_longlong(w.acc[3]) == __double_as_longlong(w.prev[3]);
        w.nw = w.acc[3];
        w.n_new = w.cnt;
        for (int c = 0; c < 3; ++c) {
          w.nm[c] = w.acc[c];
          w.nm[c] /= w.nw;                                                  // :800-802
        }
        w.ow = w.tw - w.nw;                                                  // :805
        for (int c = 0; c < 3; ++c) w.om[c] = (w.tw * w.tm[c] - w.nw * w.nm[c]) / w.ow;   // :808-810
        for (int c = 0; c < 3; ++c) w.nsq[c] = w.acc[4 + c];
        for (int c = 0; c < 4; ++c) w.prev[c] = w.acc[c];
        w.fkind = WS_KM;
        if (last || fixed) w.done = 1;   // (the decision that made these sums stays: the final membership)
        else {
          ws_decision(w);
          w.it++;
        }
      }
      __syncthreads();
    }
    const int oi = ctl.old_index;
    const bool final_split = new_index == K - 1;
    if (!final_split) {   // the stable partition (:894-1026): old half first, point order kept
      const uint64_t tp0 = wall_clock64();
      const uint64_t* src = ctl.src ? recB : recA;
      uint64_t* dst = ctl.src ? recA : recB;
      const uint32_t off = ctl.off, end = ctl.off + ctl.len, n_old = ctl.len - ctl.n_new;
      const int kind = ctl.fkind, axis = ctl.axis;
      const double cut = ctl.cut, lhs = ctl.lhs, rr = ctl.rr, rg = ctl.rg, rb = ctl.rb;
      uint32_t run_o = 0, run_n = 0;
      for (uint32_t base = off; base < end; base += kWsThreads) {
        const uint32_t j = base + tid;
        uint64_t r = 0;
        bool valid = j < end, take = false;
        if (valid) {
          r = src[j];
          const uint32_t col = (uint32_t)r;
          take = ws_take(kind, axis, cut, lhs, rr, rg, rb, (col >> 16) & 0xFF, (col >> 8) & 0xFF, col & 0xFF);
        }
        const uint64_t bo = __ballot(valid && !take), bn = __ballot(take);
        if (lane == 0) {
          s_wo[wv] = (uint32_t)__popcll(bo);
          s_wn[wv] = (uint32_t)__popcll(bn);
        }
        __syncthreads();
        uint32_t po = run_o, pn = run_n;
        for (uint32_t w = 0; w < (uint32_t)kWsWaves; ++w) {
          if (w < wv) { po += s_wo[w]; pn += s_wn[w]; }
          run_o += s_wo[w];
          run_n += s_wn[w];
        }
        const uint32_t lo = __builtin_amdgcn_mbcnt_hi((uint32_t)(bo >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bo, 0u));
        const uint32_t ln = __builtin_amdgcn_mbcnt_hi((uint32_t)(bn >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bn, 0u));
        if (valid) {
          if (take) dst[off + n_old + pn + ln] = r;
          else dst[off + po + lo] = r;
        }
        __syncthreads();
      }
      if (tid == 0) {
        if (run_n != ctl.n_new) ctl.status = 3;   // (the fold's count and the partition's must agree)
        ctl.t_part += wall_clock64() - tp0;
      }
    }
    if (tid == 0) {   // the split's results (:820-871) and STEP 4 (:873-892)
      WsCtl& w = ctl;
      WsClu& C = clu[oi];
      WsClu& D = clu[new_index];
      const int64_t parent_size = C.size;
      int64_t* t = res->trace + 4 * (new_index - 1);
      t[0] = new_index;
      t[1] = oi;
      t[2] = parent_size;
      t[3] = w.n_new;
      C.size = parent_size - (int64_t)w.n_new;
      D.size = w.n_new;
      for (int c = 0; c < 3; ++c) { C.mean[c] = w.om[c]; D.mean[c] = w.nm[c]; }
      const int other = w.src ^ 1;
      C.buf = D.buf = other;
      C.off = w.off;
      C.len = w.len - w.n_new;
      D.off = w.off + C.len;
      D.len = w.n_new;
      if (!final_split) {
        double nv[3], ov[3];
        for (int c = 0; c < 3; ++c) nv[c] = w.nsq[c] / w.nw - w.nm[c] * w.nm[c];   // :836-838
        for (int c = 0; c < 3; ++c) {
          const double dn = w.nm[c] - w.tm[c];
          const double dox = w.om[c] - w.tm[c];
          ov[c] = ((w.tw * w.tv[c] - w.nw * (nv[c] + dn * dn)) / w.ow) - dox * dox;   // :845-855
        }
        for (int c = 0; c < 3; ++c) { C.var[c] = ov[c]; D.var[c] = nv[c]; }
        C.w = w.ow;   // :859-863
        D.w = w.nw;
        C.tse = w.ow * (ov[0] + ov[1] + ov[2]);   // :870-871
        D.tse = w.nw * (nv[0] + nv[1] + nv[2]);
        for (int c = 0; c < 3; ++c) { D.lo[c] = C.lo[c]; D.hi[c] = C.hi[c]; }
        if (w.proven) {   // the halves are the cut's: v_axis < thr | >= thr
          const int thr = ws_threshold(w.cut);
          C.hi[w.axis] = min(C.hi[w.axis], thr - 1);
          D.lo[w.axis] = max(D.lo[w.axis], thr);
        }
        double best = DBL_MIN;
        for (int ic = 0; ic <= new_index; ++ic)
          if (best < clu[ic].tse) {
            best = clu[ic].tse;
            w.old_index = ic;
          }
      }
    }
    __syncthreads();
  }

  // ---- C. final centres, dedup, map ---------------------------------------------
  if (tid == 0) {
    res->prof[3] = wall_clock64();
    res->prof[5] = ctl.t_pass;
    res->prof[6] = ctl.t_part;
    res->prof[7] = ctl.nkind;
    uint32_t out = 0, empty = 0;
    for (int ic = 0; ic < K; ++ic) {
      const WsClu& q = clu[ic];
      for (int c = 0; c < 3; ++c) res->means[3 * ic + c] = q.mean[c];
      res->sizes[ic] = q.size;
      if (q.size > 0) {   // round (:1030, :1050-1054)
        const uint32_t R = (uint32_t)(uint8_t)(q.mean[0] + 0.5);
        const uint32_t G = (uint32_t)(uint8_t)(q.mean[1] + 0.5);
        const uint32_t B = (uint32_t)(uint8_t)(q.mean[2] + 0.5);
        const uint32_t col = (R << 16) | (G << 8) | B;
        res->ct[out] = col;
        s_ct[out++] = col;
      } else {
        ++empty;
      }
    }
    uint32_t m = 0;   // first-occurrence dedup (quant_util.cpp:93-118)
    for (uint32_t i = 0; i < out; ++i) {
      bool seen = false;
      for (uint32_t j = 0; j < m; ++j) seen = seen || s_ct[j] == s_ct[i];
      if (!seen) s_ct[m++] = s_ct[i];
    }
    res->nu = nu;
    res->k_raw = out;
    res->num_empty = empty;
    res->m = m;
    res->passes = ctl.passes;
    // (a batch has no grid map behind it: a larger region's map is the host's)
    const bool map = a.out != nullptr && m <= (uint32_t)kWsMapMax && ctl.status == 1 &&
                     (n <= kWsMapInline || a.maptab != nullptr);
    res->mapped = map ? 1u : 0u;
    ctl.done = map ? 1 : 0;
    if (map) {
      // sort_color (:227-238): std::sort by R+G+B; for <= 16 entries libstdc++
      // runs __insertion_sort alone (stable)
      int wt[kWsMapMax];
      for (uint32_t i = 0; i < m; ++i) {
        const uint32_t q = s_ct[i];
        int wq = (int)((q >> 16) & 0xFF) + (int)((q >> 8) & 0xFF) + (int)(q & 0xFF);
        uint32_t j = i;
        while (j > 0 && wq < wt[j - 1]) {
          wt[j] = wt[j - 1];
          s_pal[j] = s_pal[j - 1];
          --j;
        }
        wt[j] = wq;
        s_pal[j] = q;
      }
      // lut_init (:331-383), in the reference's order of writes
      const int k = (int)m;
      const int low = k >= 2 ? (int)(0.5 * (wt[0] + wt[1]) + 0.5) : 1;
      for (int v = 0; v < low; ++v) s_lut[v] = 0;
      const int high = k >= 2 ? (int)(0.5 * (wt[k - 2] + wt[k - 1]) + 0.5) : 1;
      for (int v = high; v < 766; ++v) s_lut[v] = (uint16_t)(k - 1);
      for (int i = 1; i < k - 1; ++i) {
        const int lo = (int)(0.5 * (wt[i - 1] + wt[i]) + 0.5);
        const int hi = (int)(0.5 * (wt[i] + wt[i + 1]) + 0.5);
        for (int v = lo; v < hi; ++v) s_lut[v] = (uint16_t)i;
      }
    }
  }
  __syncthreads();
  if (ctl.done) {   // map_colors_mps: here, or by wsmap_kernel's grid for larger inputs
    const int m = (int)res->m;
    if (n <= kWsMapInline) {
      ws_map(a.px, a.out, n, tid, kWsThreads, s_pal, s_lut, m);
    } else {
      for (uint32_t i = tid; i < 766; i += kWsThreads) a.maptab->lut[i] = s_lut[i];
      if (tid < (uint32_t)m) a.maptab->pal[tid] = s_pal[tid];
      if (tid == 0) a.maptab->m = (uint32_t)m;
      __syncthreads();
      if (tid == 0) a.maptab->go = 1;   // (the next launch reads it: stream order)
    }
  }
  __syncthreads();
  if (tid == 0) {
    res->prof[4] = wall_clock64();
    ws_store_status(res, (uint32_t)ctl.status);
  }
}

__global__ __launch_bounds__(kWsThreads) void wsmall_kernel(WSmallArgs a) { wsmall_body(a); }

// Many inputs (the app's superpixel regions) in one launch: workgroup b runs
// region b's whole call (as[b]; maptab null).
__global__ __launch_bounds__(kWsThreads) void wsmall_batch_kernel(const WSmallArgs* __restrict__ as) {
  const WSmallArgs a = as[blockIdx.x];
  wsmall_body(a);
}

// The map of a larger small-path input (n > kWsMapInline) over a grid, from
// the palette and lut_init wsmall_kernel left in `t` (go = 0: it did not map:
// nothing to do).
__global__ __launch_bounds__(256) void wsmap_kernel(const uint32_t* __restrict__ px, uint32_t* __restrict__ out,
                                                    uint32_t n, const WsMapTab* __restrict__ t) {
  __shared__ uint32_t s_pal[kWsMapMax];
  __shared__ uint16_t s_lut[766];
  if (t->go == 0) return;
  const int m = (int)t->m;
  for (uint32_t i = threadIdx.x; i < 766; i += 256) s_lut[i] = t->lut[i];
  if (threadIdx.x < (uint32_t)m) s_pal[threadIdx.x] = t->pal[threadIdx.x];
  __syncthreads();
  ws_map(px, out, n, blockIdx.x * 256u + threadIdx.x, gridDim.x * 256u, s_pal, s_lut, m);
}

}  // namespace

hipError_t launch_wsmall(const WSmallArgs& a, hipStream_t stream) {
  static hipError_t attr = hipErrorNotReady;
  if (attr != hipSuccess) {   // more than 64 KB of dynamic LDS (its static LDS on top: at most 160 KB in all)
    attr = hipFuncSetAttribute((const void*)wsmall_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kWsLds);
    if (attr != hipSuccess) return attr;
  }
  wsmall_kernel<<<dim3(1), dim3(kWsThreads), kWsLds, stream>>>(a);
  if (a.out && a.n > kWsMapInline) {   // (exits at once unless wsmall_kernel left it a palette)
    const uint32_t grid = std::min<uint32_t>(1024u, (a.n + 256u * 8u - 1u) / (256u * 8u));
    wsmap_kernel<<<dim3(grid), dim3(256), 0, stream>>>(a.px, a.out, a.n, a.maptab);
  }
  return hipGetLastError();
}

hipError_t launch_wsmall_batch(const WSmallArgs* d_args, int nregions, hipStream_t stream) {
  if (nregions <= 0) return hipSuccess;
  static hipError_t attr = hipErrorNotReady;
  if (attr != hipSuccess) {
    attr = hipFuncSetAttribute((const void*)wsmall_batch_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)kWsLds);
    if (attr != hipSuccess) return attr;
  }
  wsmall_batch_kernel<<<dim3(nregions), dim3(kWsThreads), kWsLds, stream>>>(d_args);
  return hipGetLastError();
}

}  // namespace dq
