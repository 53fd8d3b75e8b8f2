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
//   * the colour table: runs of equal pixels partitioned by hash-bucket
//     group, one LDS hash table per group, each colour ranked inside its
//     bucket by first occurrence descending -- the order the reference's
//     prepended hash chains emit, weights norm * count (:184-195);
//   * the node splits of a round, pass by pass over tiles of every node:
//     the init folds (root), the split pass, the local 2-means passes to a
//     fixed point or max_iters, each an EXACT PARALLEL FOLD (below), the
//     reference's FP64 epilogue, then a stable partition of each node's
//     points into its children's segments (point order kept).
//
// Exact parallel fold.  s_{i+1} = fl(s_i + x_i), s_0 = 0, x_i >= 0.  While
// s_i and the exact s_i + x_i lie in one binade [2^e, 2^(e+1)), the sum is
// rounded to the grid u = 2^(e-52) and s_{i+1} = s_i + u * RNE(x_i / u)
// unless x_i / u is exactly halfway (a tie, decided by s_i's parity).  So a
// run of summands inside one binade adds u * (an exact integer sum) -- in any
// order, on any number of workgroups.  The binade each summand sees is
// bounded from an estimate of the prefix (the tiles' sums scanned in any
// order): |s_i - prefix_i| <= i * 2^-53 * s_i and the estimate's own error
// is as small, so a summand whose interval [P(1-2^-20), (P+x)(1+2^-20)]
// lies in one binade is a run member; the others (binade crossings, ties,
// the first summand) are "specials" the chain adds in hardware, in order.
// The chain (one wave per node) applies each tile's runs and specials in
// sequence order, checks every run against the running sum's binade, and
// folds a tile summand by summand whenever its description does not apply.
// The result is the sequential fold's double, bit for bit.
// MUST be compiled with -ffp-contract=off (the Makefile does).
#include <hip/hip_runtime.h>
#include <algorithm>

#include "dq_weighted.h"

namespace dq {

namespace {

// --- colour table ----------------------------------------------------------
// calc_color_table (DivQuantMapColors.cpp:82-203) without a sort.  Its output
// order is the hash chains': bucket HASH(c) = ((R*33023 + G*30013 + B*27011)
// & 0x7fffffff) % 20023 ascending (:56-62, :186-201), and inside a bucket the
// first occurrence DESCENDING (each new colour is prepended to its chain,
// :132-158).  So colours never need a global order, only a bucket and a rank
// inside it:
//   1. ct_runs<COUNT>: per block of kCtChunk consecutive pixels, the runs of
//      equal colour (a lane's 16 consecutive pixels; a run ends at the next
//      different pixel in the wave's 1024 or at a 256-pixel boundary), each a
//      record (first index, length, colour), counted per bucket GROUP
//      (kCtGB consecutive buckets) in LDS -> hist[block][group];
//   2. ct_colscan + ct_gscan: the records' exclusive offsets, group-major;
//   3. ct_runs<SCATTER>: the same runs scattered to their group's range;
//   4. ct_group: one workgroup per group -- an LDS hash table of the group's
//      colours (count = sum of lengths, first = min of firsts; a group holds
//      at most kCtGB * 844 colours: no bucket has more than 844 of the 2^24),
//      then per bucket each colour's rank by first occurrence descending (in
//      sub-buckets: 16 bins of the first occurrence), and
//      the colours as records colour | count << 32 in calc_color_table's
//      order, at the group's offset;
//   5. ct_gscan + ct_compact: the groups' outputs packed into rec.
// LDS atomics only (a device-wide table of global atomics measured ~27 G
// atomic ops/s on this part, profiles/r06_ct/atomic_bench.txt: slower than
// the sorts it would replace).
constexpr uint32_t kCtBuckets = 20023;
constexpr uint32_t kCtGB = 4;                                       // buckets per group
constexpr uint32_t kCtGroups = (kCtBuckets + kCtGB - 1) / kCtGB;    // 5006
constexpr uint32_t kCtMaxPerGroup = kCtGB * 844;                    // colours of one group, at most
constexpr uint32_t kCtSlots = 4096;                                 // LDS hash slots (> kCtMaxPerGroup)
constexpr int kCtSlotShift = 20;                                    // 32 - log2(kCtSlots)
constexpr int kCtThreads = 1024;                                    // ct_runs: 16 waves x 1024 pixels a step
constexpr int kCtGroupThreads = 1024;
constexpr uint32_t kCtEmpty = 0xFFFFFFFFu;
constexpr uint32_t kCtSub = 16;                                     // first-occurrence bins per bucket
constexpr uint32_t kCtList = kCtMaxPerGroup + 4 * kCtGB * kCtSub;   // the firsts by sub-bucket, each padded to 4
constexpr size_t kCtGroupLds = (size_t)kCtSlots * 12 + (size_t)kCtList * 6 + 64;
static_assert(kCtSlots > kCtMaxPerGroup, "the group table never fills");

__device__ __forceinline__ uint32_t ct_bucket(uint32_t c) {   // HASH (:56-62): the sum is < 2^31
  const uint32_t R = (c >> 16) & 0xFFu, G = (c >> 8) & 0xFFu, B = c & 0xFFu;
  return (R * 33023u + G * 30013u + B * 27011u) % kCtBuckets;
}

// The runs of one wave's 1024 pixels [wb, wb + 1024) of px[0..n): lane l
// holds pixels wb + 16 l + k.  f(c, first, len) for every run head, len <= 256.
template <typename F>
__device__ __forceinline__ void ct_wave_runs(const uint32_t* __restrict__ px, uint32_t n, uint32_t wb, F&& f) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t p0 = wb + 16u * lane;
  uint32_t c[16];
  if (p0 + 16u <= n && ((uintptr_t)px & 15u) == 0) {
    const uint4* v = reinterpret_cast<const uint4*>(px + p0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 x = v[j];
      c[4 * j] = x.x & 0xFFFFFFu;
      c[4 * j + 1] = x.y & 0xFFFFFFu;
      c[4 * j + 2] = x.z & 0xFFFFFFu;
      c[4 * j + 3] = x.w & 0xFFFFFFu;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) c[k] = p0 + (uint32_t)k < n ? (px[p0 + k] & 0xFFFFFFu) : kCtEmpty;
  }
  const uint32_t prev = __shfl_up(c[15], 1, 64);
  // brk bit k: a run starts at k, or k is past the input
  uint32_t brk = (lane & 15u) == 0u || prev != c[0] ? 1u : 0u;
#pragma unroll
  for (int k = 1; k < 16; ++k) brk |= (c[k] != c[k - 1] ? 1u : 0u) << k;
  // lane slots inside the input
  const uint32_t valid = p0 + 16u <= n ? 0xFFFFu : (n > p0 ? (1u << (n - p0)) - 1u : 0u);
  brk |= 0xFFFFu & ~valid;
  // the first break of the later lanes (suffix minimum; 1024: none)
  const uint32_t mine = brk ? 16u * lane + (uint32_t)__builtin_ctz(brk) : 1024u;
  uint32_t nx = __shfl_down(mine, 1, 64);
  if (lane == 63u) nx = 1024u;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_down(nx, d, 64);
    if (lane + (uint32_t)d < 64u) nx = min(nx, u);
  }
  uint32_t heads = brk & valid;   // runs start inside the input only
  while (heads) {
    const int k = __builtin_ctz(heads);
    heads &= heads - 1u;
    const uint32_t later = brk >> (k + 1);
    const uint32_t end = later ? 16u * lane + (uint32_t)k + 1u + (uint32_t)__builtin_ctz(later) : nx;
    uint32_t ck = c[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) ck = k == j ? c[j] : ck;
    f(ck, p0 + (uint32_t)k, end - (16u * lane + (uint32_t)k));
  }
}

// Steps 1 and 3.  COUNT: hist[block][group] = the block's runs per group.
// SCATTER: each run to part[gstart[group] + off[block][group] + its rank in
// the block] as (first << 32) | (len - 1) << 24 | colour.
template <bool COUNT>
__global__ __launch_bounds__(kCtThreads) void ct_runs(const uint32_t* __restrict__ px, uint32_t n, uint32_t chunk,
                                                      uint32_t* __restrict__ hist, const uint32_t* __restrict__ gstart,
                                                      uint64_t* __restrict__ part) {
  __shared__ uint32_t s_h[kCtGroups];
  uint32_t* row = hist + (size_t)blockIdx.x * kCtGroups;
  for (uint32_t g = threadIdx.x; g < kCtGroups; g += kCtThreads) s_h[g] = COUNT ? 0u : gstart[g] + row[g];
  __syncthreads();
  const uint32_t b0 = blockIdx.x * chunk, b1 = min(n, b0 + chunk);
  for (uint32_t wb = b0 + (threadIdx.x >> 6) * 1024u; wb < b1; wb += (kCtThreads / 64) * 1024u)
    ct_wave_runs(px, b1, wb, [&](uint32_t c, uint32_t first, uint32_t len) {
      const uint32_t g = ct_bucket(c) / kCtGB;
      if (COUNT) {
        atomicAdd(&s_h[g], 1u);
      } else {
        const uint32_t pos = atomicAdd(&s_h[g], 1u);
        part[pos] = ((uint64_t)first << 32) | ((uint64_t)(len - 1u) << 24) | c;
      }
    });
  if (COUNT) {
    __syncthreads();
    for (uint32_t g = threadIdx.x; g < kCtGroups; g += kCtThreads) row[g] = s_h[g];
  }
}

// Step 2a: per group, the exclusive prefix over blocks of hist[b][g] (in
// place) and the group's total.  64 groups per workgroup (coalesced rows),
// 16 block ranges per group.
__global__ __launch_bounds__(1024) void ct_colscan(uint32_t* __restrict__ hist, uint32_t nblk,
                                                   uint32_t* __restrict__ gtot) {
  __shared__ uint32_t s_p[16][64];
  const uint32_t gl = threadIdx.x & 63u, part = threadIdx.x >> 6;
  const uint32_t g = blockIdx.x * 64u + gl;
  const uint32_t per = (nblk + 15u) / 16u, bb = part * per, be = min(nblk, bb + per);
  uint32_t s = 0;
  if (g < kCtGroups)
    for (uint32_t b = bb; b < be; ++b) s += hist[(size_t)b * kCtGroups + g];
  s_p[part][gl] = s;
  __syncthreads();
  uint32_t run = 0, tot = 0;
  for (uint32_t q = 0; q < 16u; ++q) {
    if (q < part) run += s_p[q][gl];
    tot += s_p[q][gl];
  }
  if (g < kCtGroups) {
    for (uint32_t b = bb; b < be; ++b) {
      uint32_t* h = hist + (size_t)b * kCtGroups + g;
      const uint32_t v = *h;
      *h = run;
      run += v;
    }
    if (part == 0) gtot[g] = tot;
  }
}

// Step 2b / 5a: out[0..m] = exclusive prefix of in[0..m), out[m] = total (one
// workgroup; m = kCtGroups).
__global__ __launch_bounds__(1024) void ct_gscan(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t m) {
  __shared__ uint32_t s_w[16];
  const uint32_t per = (m + 1023u) / 1024u, i0 = threadIdx.x * per, i1 = min(m, i0 + per);
  uint32_t s = 0;
  for (uint32_t i = i0; i < i1; ++i) s += in[i];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += u;
  }
  if (lane == 63u) s_w[wv] = inc;
  __syncthreads();
  uint32_t base = 0;
  for (uint32_t w = 0; w < wv; ++w) base += s_w[w];
  uint32_t run = base + inc - s;
  for (uint32_t i = i0; i < i1; ++i) {
    const uint32_t v = in[i];
    out[i] = run;
    run += v;
  }
  if (threadIdx.x == 1023u) out[m] = base + inc;
}

// Step 4: one workgroup per group.  Reads the group's runs part[gstart[g] ..
// gstart[g + 1]) and writes its colours in calc_color_table's order to the
// same range's front (every read is done before the first write), ucnt[g]
// their number.
__global__ __launch_bounds__(kCtGroupThreads) void ct_group(uint64_t* __restrict__ part,
                                                            const uint32_t* __restrict__ gstart,
                                                            uint32_t* __restrict__ ucnt, uint32_t binshift) {
  extern __shared__ __attribute__((aligned(16))) uint8_t ct_lds[];
  uint32_t* key = reinterpret_cast<uint32_t*>(ct_lds);
  uint32_t* cnt = key + kCtSlots;
  uint32_t* fst = cnt + kCtSlots;
  uint32_t* lf = fst + kCtSlots;                          // [kCtList] firsts, by bucket (16-B aligned runs)
  uint16_t* ls = reinterpret_cast<uint16_t*>(lf + kCtList); // [kCtList] their slots
  __shared__ uint32_t s_bc[64], s_bs[65], s_b4[65], s_cur[64];
  const uint32_t g = blockIdx.x, t = threadIdx.x;
  const uint32_t r0 = gstart[g], r1 = gstart[g + 1];
  // the first kCtPre runs per thread loaded before the table is cleared (the
  // loads' latency under the clear)
  constexpr int kCtPre = 2;   // (pre[0], pre[1] below)
  uint64_t pre[kCtPre];
#pragma unroll
  for (int q = 0; q < kCtPre; ++q) {
    const uint32_t i = r0 + t + (uint32_t)q * kCtGroupThreads;
    pre[q] = i < r1 ? part[i] : 0ull;
  }
  for (uint32_t s = t; s < kCtSlots; s += kCtGroupThreads) {
    key[s] = kCtEmpty;
    cnt[s] = 0u;
    fst[s] = 0xFFFFFFFFu;
  }
  if (t < 64u) s_bc[t] = s_cur[t] = 0u;
  __syncthreads();
  for (uint32_t i = r0 + t, q = 0; i < r1; i += kCtGroupThreads, ++q) {
    const uint64_t r = q == 0 ? pre[0] : (q == 1 ? pre[1] : part[i]);
    const uint32_t c = (uint32_t)r & 0xFFFFFFu, len = (((uint32_t)r >> 24) & 0xFFu) + 1u, first = (uint32_t)(r >> 32);
    uint32_t s = (c * 2654435761u) >> kCtSlotShift;
    for (;;) {
      const uint32_t k = atomicCAS(&key[s], kCtEmpty, c);
      if (k == kCtEmpty || k == c) break;
      s = (s + 1u) & (kCtSlots - 1u);
    }
    atomicAdd(&cnt[s], len);
    atomicMin(&fst[s], first);
  }
  __syncthreads();
  // sub-buckets: (bucket ascending, first-occurrence bin descending), the
  // bins monotone in the first occurrence (its top 4 bits below n), so
  // ranking by first occurrence inside a sub-bucket is ranking inside the
  // bucket at 1/16 of the comparisons
  const uint32_t bb = g * kCtGB;
  auto sub = [&](uint32_t s) { return (ct_bucket(key[s]) - bb) * kCtSub + (kCtSub - 1u) - (fst[s] >> binshift); };
  for (uint32_t s = t; s < kCtSlots; s += kCtGroupThreads)
    if (key[s] != kCtEmpty) atomicAdd(&s_bc[sub(s)], 1u);
  __syncthreads();
  if (t < 64u) {   // s_bs: the sub-buckets' output offsets; s_b4: their lists' (padded to 4)
    static_assert(kCtGB * kCtSub == 64, "one wave scans the sub-buckets");
    const uint32_t c = s_bc[t], c4 = (c + 3u) & ~3u;
    uint32_t inc = c, inc4 = c4;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64), u4 = __shfl_up(inc4, o, 64);
      if (t >= (uint32_t)o) {
        inc += u;
        inc4 += u4;
      }
    }
    s_bs[t] = inc - c;
    s_b4[t] = inc4 - c4;
    if (t == 63u) {
      s_bs[64] = inc;
      s_b4[64] = inc4;
    }
  }
  __syncthreads();
  for (uint32_t x = t; x < s_b4[64]; x += kCtGroupThreads) {   // (pads: first 0 is never > f)
    lf[x] = 0u;
    ls[x] = 0xFFFFu;
  }
  __syncthreads();
  for (uint32_t s = t; s < kCtSlots; s += kCtGroupThreads)
    if (key[s] != kCtEmpty) {
      const uint32_t j = sub(s);
      const uint32_t x = s_b4[j] + atomicAdd(&s_cur[j], 1u);
      lf[x] = fst[s];
      ls[x] = (uint16_t)s;
    }
  __syncthreads();
  // rank inside the sub-bucket: colours first seen later come first
  // (:132-158); 4 firsts a read
  const uint32_t tot4 = s_b4[64];
  const uint4* l4 = reinterpret_cast<const uint4*>(lf);
  for (uint32_t x = t; x < tot4; x += kCtGroupThreads) {
    const uint32_t s = ls[x];
    if (s == 0xFFFFu) continue;   // a pad
    const uint32_t j = sub(s), f = lf[x];
    uint32_t rank = 0;
#pragma unroll 2
    for (uint32_t y = s_b4[j] / 4u; y < s_b4[j + 1] / 4u; ++y) {
      const uint4 v = l4[y];
      rank += (v.x > f ? 1u : 0u) + (v.y > f ? 1u : 0u) + (v.z > f ? 1u : 0u) + (v.w > f ? 1u : 0u);
    }
    part[r0 + s_bs[j] + rank] = (uint64_t)key[s] | ((uint64_t)cnt[s] << 32);
  }
  const uint32_t tot = s_bs[64];
  if (t == 0) ucnt[g] = tot;
}

// Step 5b: group g's colours to rec[uoff[g] ..).
__global__ __launch_bounds__(256) void ct_compact(const uint64_t* __restrict__ part, const uint32_t* __restrict__ gstart,
                                                  const uint32_t* __restrict__ uoff, uint64_t* __restrict__ rec) {
  const uint32_t g = blockIdx.x, o = uoff[g], m = uoff[g + 1] - o;
  const uint64_t* src = part + gstart[g];
  for (uint32_t i = threadIdx.x; i < m; i += 256u) rec[o + i] = src[i];
}


// --- weighted node splits: exact parallel folds --------------------------------
constexpr int kWThreads = 256;
constexpr int kWPer = (int)kWTile / kWThreads;   // consecutive points per lane
constexpr int32_t kWNone = -100001;             // quick form: no summand changes the sum
constexpr double kWMargin = 0x1p-20;            // relative bound on |s_i - prefix estimate|

__device__ __forceinline__ bool w_take(int pass, const WState& st, uint32_t R, uint32_t G, uint32_t B) {
  if (pass == WP_INIT) return true;
  const double red = (double)R, green = (double)G, blue = (double)B;
  if (pass == WP_SPLIT) return st.cut < (st.axis == 0 ? red : (st.axis == 1 ? green : blue));   // :473
  return !(st.lhs < ((st.rr * red) + (st.rg * green) + (st.rb * blue)));                         // :683
}

// The reference's summands (:73-85, :496-517, :719-770): w*R (R converted),
// w*(R*R) (the product in uint32), the weight itself.
__device__ __forceinline__ double w_prod(int ch, uint32_t R, uint32_t G, uint32_t B, double w) {
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

// weights[index] = norm_factor * bucket->value (:195), from a point's record
__device__ __forceinline__ double w_weight(const WArgs& a, uint64_t rec) { return a.norm * (int)(uint32_t)(rec >> 32); }

struct WPts {
  uint32_t R[kWPer], G[kWPer], B[kWPer];
  double w[kWPer];
  uint32_t take;   // bit k: point k of this lane is a summand of the pass
};

__device__ __forceinline__ void w_load(const WArgs& a, const WState& st, const WTile& t, int pass, WPts& q) {
  q.take = 0;
  const uint32_t p0 = t.start + (uint32_t)kWPer * threadIdx.x;
#pragma unroll
  for (int k = 0; k < kWPer; ++k) {
    const uint32_t p = p0 + (uint32_t)k;
    q.R[k] = q.G[k] = q.B[k] = 0;
    q.w[k] = 0.0;
    if (p < t.end) {
      const uint64_t r = st.src[p];
      const uint32_t c = (uint32_t)r;
      q.w[k] = w_weight(a, r);
      q.R[k] = (c >> 16) & 0xFF;
      q.G[k] = (c >> 8) & 0xFF;
      q.B[k] = c & 0xFF;
      if (w_take(pass, st, q.R[k], q.G[k], q.B[k])) q.take |= 1u << k;
    }
  }
}

// The same points, lane-interleaved (point k of a lane is the tile's
// k * kWThreads + lane): coalesced, for folds whose order does not matter
// (the tile sums, the one-binade tiles' integer sums).
__device__ __forceinline__ void w_load_co(const WArgs& a, const WState& st, const WTile& t, int pass, WPts& q) {
  q.take = 0;
#pragma unroll
  for (int k = 0; k < kWPer; ++k) {
    const uint32_t p = t.start + (uint32_t)(k * kWThreads) + threadIdx.x;
    q.R[k] = q.G[k] = q.B[k] = 0;
    q.w[k] = 0.0;
    if (p < t.end) {
      const uint64_t r = st.src[p];
      const uint32_t c = (uint32_t)r;
      q.w[k] = w_weight(a, r);
      q.R[k] = (c >> 16) & 0xFF;
      q.G[k] = (c >> 8) & 0xFF;
      q.B[k] = c & 0xFF;
      if (w_take(pass, st, q.R[k], q.G[k], q.B[k])) q.take |= 1u << k;
    }
  }
}

__device__ __forceinline__ double w_x(const WPts& q, int k, int ch) {
  return ((q.take >> k) & 1u) ? w_prod(ch, q.R[k], q.G[k], q.B[k], q.w[k]) : 0.0;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Pass step 1: per tile, its summands' sums in any order (an estimate of the
// fold, for the prefix) and the summand count.
__global__ __launch_bounds__(kWThreads) void wk_tilesum(WArgs a, int pass) {
  const WTile t = a.tiles[blockIdx.x];
  const WState& st = a.nodes[t.node];
  if (st.done) return;
  WPts q;
  w_load_co(a, st, t, pass, q);
  __shared__ double red[kWThreads / 64][8];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int ch = 0; ch < kWCh; ++ch) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < kWPer; ++k) v += w_x(q, k, ch);
    v = wave_sum_f64(v);
    if (lane == 0) red[wv][ch] = v;
  }
  const uint32_t c = (uint32_t)__popc(q.take);
  uint32_t cs = c;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) cs += __shfl_xor(cs, o, 64);
  if (lane == 0) red[wv][7] = (double)cs;
  __syncthreads();
  if (threadIdx.x < 8) {
    double v = 0.0;
    for (int w = 0; w < kWThreads / 64; ++w) v += red[w][threadIdx.x];
    a.tsum[(size_t)blockIdx.x * 8 + threadIdx.x] = v;
  }
}

// Pass step 2: per node (one wave), the exclusive prefix of its tiles' sums.
// (one wave per fold: the folds' prefixes are independent)
__global__ __launch_bounds__(64 * kWCh) void wk_prefix(WArgs a) {
  const WState& st = a.nodes[blockIdx.x];
  if (st.done) return;
  const int lane = (int)(threadIdx.x & 63);
  {
    const int ch = (int)(threadIdx.x >> 6);
    double run = 0.0;
    for (int b = st.tile_begin; b < st.tile_end; b += 64) {
      const int i = b + lane;
      const double v = i < st.tile_end ? a.tsum[(size_t)i * 8 + ch] : 0.0;
      double inc = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
      }
      const double up = __shfl_up(inc, 1, 64);   // (every lane: a shuffle's source lane must be active)
      const double ex = lane == 0 ? 0.0 : up;
      if (i < st.tile_end) a.tpre[(size_t)i * 8 + ch] = run + ex;
      run += __shfl(inc, 63, 64);
    }
  }
}

// ilogb of a positive normal double (its binade's exponent)
__device__ __forceinline__ int w_binade(double v) {
  return (int)((__double_as_longlong(v) >> 52) & 0x7FF) - 1023;
}

// Pass step 3a: one workgroup per tile, the folds whose tile lies in one
// binade.  With the tile's prefix estimate P0 and its sum estimate Tt, every
// summand's interval lies inside [P0 (1 - 2^-20), (P0 + Tt) (1 + 2^-20)] (the
// prefixes grow from P0, the summands are >= 0, and the estimates' errors are
// far inside the margin), so when that interval is in one binade e every
// nonzero summand of the fold is a run member of e: the description is one
// segment (e, sum of RNE(x / 2^(e-52))) -- no scans, no slots, and the order
// of the summands does not matter (an integer sum).  Nearly every tile past a
// node's first few is one-binade in all seven folds: the tile is loaded ONCE,
// coalesced, for all of them (the round-5 form loaded it once per fold, seven
// workgroups per tile).  A tie anywhere in a fold's tile (x / u exactly
// halfway) and the folds that are not one-binade go to wk_classify (gen).
__global__ __launch_bounds__(kWThreads) void wk_classify_fast(WArgs a, int pass) {
  const uint32_t ti = blockIdx.x;
  const WTile t = a.tiles[ti];
  const WState& st = a.nodes[t.node];
  if (st.done) return;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int kW = kWThreads / 64;
  __shared__ long long s_fm[kW][kWCh];
  __shared__ uint32_t s_tie[kW];
  uint32_t fast = 0;   // (block-uniform: tile values)
  int el[kWCh];
#pragma unroll
  for (int ch = 0; ch < kWCh; ++ch) {
    const double P0 = a.tpre[(size_t)ti * 8 + ch], Tt = a.tsum[(size_t)ti * 8 + ch];
    const double lo = P0 * (1.0 - kWMargin), hi = (P0 + Tt) * (1.0 + kWMargin);
    el[ch] = lo > 0.0 ? w_binade(lo) : 0;
    if (lo > 0.0 && el[ch] == w_binade(hi)) fast |= 1u << ch;
  }
  uint32_t tie = 0;
  if (fast) {
    WPts qc;
    w_load_co(a, st, t, pass, qc);
#pragma unroll
    for (int ch = 0; ch < kWCh; ++ch) {
      if (!((fast >> ch) & 1u)) continue;
      long long mm = 0;
      bool tch = false;
#pragma unroll
      for (int k = 0; k < kWPer; ++k) {
        const double tt = ldexp(w_x(qc, k, ch), 52 - el[ch]);   // exact (x < 2^(el+1)); 0 for a non-summand
        const double fl = floor(tt), fr = tt - fl;
        tch |= fr == 0.5;
        mm += (long long)fl + (fr > 0.5 ? 1 : 0);
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mm += __shfl_xor(mm, o, 64);
      if (lane == 0) s_fm[wv][ch] = mm;
      if (__ballot(tch)) tie |= 1u << ch;
    }
  }
  if (lane == 0) s_tie[wv] = tie;
  __syncthreads();
  uint32_t ties = 0;
#pragma unroll
  for (int w = 0; w < kW; ++w) ties |= s_tie[w];
  const uint32_t done = fast & ~ties;
  if (threadIdx.x < (uint32_t)kWCh && ((done >> threadIdx.x) & 1u)) {
    const int ch = (int)threadIdx.x;
    long long M = 0;
    for (int w = 0; w < kW; ++w) M += s_fm[w][ch];
    WFold& f = a.fold[(size_t)ti * kWCh + ch];
    WQuick& qk = a.quick[(size_t)ti * kWCh + ch];
    if (M == 0) {
      f.nseg = 0;
      qk.e = kWNone;
      qk.m = 0;
    } else {
      WSegment g;
      g.e = el[ch];
      g.pad = 0;
      g.v = (int64_t)M;
      f.seg[0] = g;
      f.nseg = 1;
      qk.e = el[ch];
      qk.m = (int64_t)M;
    }
  }
  if (threadIdx.x == 0) {
    a.gen[ti] = ~done & ((1u << kWCh) - 1u);
    a.quick[(size_t)ti * kWCh].cnt = (uint32_t)a.tsum[(size_t)ti * 8 + 7];
  }
}

// Pass step 3b: per tile and fold (the folds wk_classify_fast left), each summand's class (zero, run member of
// binade e with integer m = RNE(x / 2^(e-52)), or special) from the prefix
// estimate, then the tile's description: its segments in sequence order --
// every special, and every maximal stretch of run members with m != 0 and
// one key (specials before them, binade).  A segment's slot is the number of
// segments that start before it: block scans of the lanes' specials and
// segment starts (a lane's first member starts one when its key differs from
// the last member of the nearest earlier lane that has one).  The slots are
// sequence order by construction, whatever the keys do along the tile.
constexpr int kWKeyBias = 1100;   // binade e of a double in [-1074, 1023] -> e + bias in [26, 2123]
// One workgroup per (tile, fold): the seven folds' descriptions of a tile
// are independent, and were classified one after another (each with its
// barriers) by one workgroup.  Workgroups are dealt round-robin over the 8
// XCDs (b and b + 8 share one; speed only, nothing relies on it), so a
// tile's seven workgroups take seven consecutive slots of ONE residue class
// b % 8: they run together on one XCD and read the tile through its L2
// instead of fetching it into seven.
__global__ __launch_bounds__(kWThreads) void wk_classify(WArgs a, int pass) {
  const uint32_t slot = blockIdx.x >> 3;
  const uint32_t ti = (slot / (uint32_t)kWCh) * 8u + (blockIdx.x & 7u);
  const int ch = (int)(slot % (uint32_t)kWCh);
  if (ti >= (uint32_t)a.ntiles) return;
  const WTile t = a.tiles[ti];
  const WState& st = a.nodes[t.node];
  if (st.done) return;
  if (!((a.gen[ti] >> ch) & 1u)) return;   // described by wk_classify_fast
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int kW = kWThreads / 64;
  __shared__ double s_wt[kW];
  __shared__ int s_sp[kW];                 // specials per wave
  __shared__ int s_wk[kW][3];              // per wave: first / last member key (-1: none), starts
  __shared__ unsigned long long s_m[kWSeg];
  __shared__ int s_e[kWSeg];
  WPts q;
  w_load(a, st, t, pass, q);
  {
    double x[kWPer];
    double T = 0.0;
#pragma unroll
    for (int k = 0; k < kWPer; ++k) {
      x[k] = w_x(q, k, ch);
      T += x[k];
    }
    // block exclusive scan of the lanes' totals (an estimate: any rounding)
    double inc = T;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double u = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += u;
    }
    if (lane == 63) s_wt[wv] = inc;
    for (int b = (int)threadIdx.x; b < kWSeg; b += kWThreads) s_m[b] = 0ull;
    __syncthreads();
    double P = a.tpre[(size_t)ti * 8 + ch];
    for (uint32_t w = 0; w < wv; ++w) P += s_wt[w];
    const double up = __shfl_up(inc, 1, 64);   // (every lane: a shuffle's source lane must be active)
    P += lane == 0 ? 0.0 : up;
    // classes: e[k] (run member, m != 0), kWNone (zero or m = 0) or special
    int e[kWPer];
    int64_t m[kWPer];
    uint32_t spm = 0;   // bit k: special
#pragma unroll
    for (int k = 0; k < kWPer; ++k) {
      e[k] = kWNone;
      m[k] = 0;
      if (x[k] != 0.0) {
        const double lo = P * (1.0 - kWMargin), hi = (P + x[k]) * (1.0 + kWMargin);
        bool special = !(lo > 0.0);
        int el = 0;
        if (!special) {
          el = w_binade(lo);
          special = el != w_binade(hi);
        }
        if (!special) {
          const double tt = ldexp(x[k], 52 - el);   // exact (x < 2^(el+1))
          const double fl = floor(tt), fr = tt - fl;
          special = fr == 0.5;                      // a tie: the parity of s decides
          m[k] = (int64_t)fl + (fr > 0.5 ? 1 : 0);
          if (!special && m[k] != 0) e[k] = el;     // (m = 0: adds nothing)
        }
        if (special) spm |= 1u << k;
      }
      P += x[k];
    }
    // specials before each lane (block exclusive scan)
    const int nsl = __popc(spm);
    int si = nsl;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(si, o, 64);
      if (lane >= (uint32_t)o) si += u;
    }
    if (lane == 63) s_sp[wv] = si;
    // the lane's member keys: first, last, starts after its first member
    int spb = si - nsl;   // (wave-local until the block offset is added)
    __syncthreads();
    int nsp = 0;
    for (int w = 0; w < kW; ++w) {
      if (w < (int)wv) spb += s_sp[w];
      nsp += s_sp[w];
    }
    int kfirst = -1, klast = -1, inner = 0;
    {
      int sp = spb;
#pragma unroll
      for (int k = 0; k < kWPer; ++k) {
        if ((spm >> k) & 1u) {
          ++sp;
        } else if (e[k] != kWNone) {
          const int key = (sp << 12) | (e[k] + kWKeyBias);
          if (kfirst < 0) kfirst = key;
          else if (key != klast) ++inner;
          klast = key;
        }
      }
    }
    // the nearest earlier lane of the wave with members: its last key
    const uint64_t hm = __ballot(kfirst >= 0);
    const uint64_t before = hm & ((1ull << lane) - 1ull);
    const int jp = before ? 63 - __builtin_clzll(before) : 0;
    const int kprev_w = __shfl(klast, jp, 64);
    const bool first_known = before != 0;   // else: from the earlier waves
    int starts = inner + ((kfirst >= 0 && first_known && kfirst != kprev_w) ? 1 : 0);
    // wave aggregates: first member key (of the wave's first lane with
    // members), last member key, starts except that first lane's first one
    int ws = starts;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) ws += __shfl_xor(ws, o, 64);
    const int jf = hm ? __builtin_ctzll(hm) : 0, jl = hm ? 63 - __builtin_clzll(hm) : 0;
    const int wfirst = __shfl(kfirst, jf, 64), wlast = __shfl(klast, jl, 64);
    if (lane == 0) {
      s_wk[wv][0] = hm ? wfirst : -1;
      s_wk[wv][1] = hm ? wlast : -1;
      s_wk[wv][2] = ws;
    }
    __syncthreads();
    // starts before this wave, and the last member key before it
    int sbefore = 0, kprev = -1, ntot = 0, kp = -1;
    for (int w = 0; w < kW; ++w) {
      const int f = s_wk[w][0], l = s_wk[w][1];
      const int add = s_wk[w][2] + ((f >= 0 && f != kp) ? 1 : 0);
      if (w < (int)wv) sbefore += add;
      if (w == (int)wv) kprev = kp;
      ntot += add;
      if (l >= 0) kp = l;
    }
    if (kfirst >= 0 && !first_known && kfirst != kprev) starts += 1;
    int sx = starts;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(sx, o, 64);
      if (lane >= (uint32_t)o) sx += u;
    }
    // place: a run member's slot = (segment starts up to it) - 1 + specials
    // before it; a special's = segment starts before it + its special index
    const int nseg = ntot + nsp;
    {
      int r = sbefore + sx - starts;
      int sp = spb;
      int key = first_known ? kprev_w : kprev;
      int cur = -1;                 // slot of the lane's open accumulation
      unsigned long long acc = 0ull;
#pragma unroll
      for (int k = 0; k < kWPer; ++k) {
        if ((spm >> k) & 1u) {
          const int slot = r + sp;
          if (slot < kWSeg) {
            s_e[slot] = kWSpecial;
            s_m[slot] = (unsigned long long)__double_as_longlong(x[k]);
          }
          ++sp;
        } else if (e[k] != kWNone) {
          const int kk = (sp << 12) | (e[k] + kWKeyBias);
          if (kk != key) {
            ++r;
            key = kk;
          }
          const int slot = r - 1 + sp;
          if (slot != cur) {
            if (cur >= 0 && cur < kWSeg) atomicAdd(&s_m[cur], acc);
            cur = slot;
            acc = 0ull;
            if (slot < kWSeg) s_e[slot] = e[k];   // (every writer of a slot stores the same e)
          }
          acc += (unsigned long long)m[k];
        }
      }
      if (cur >= 0 && cur < kWSeg) atomicAdd(&s_m[cur], acc);
    }
    __syncthreads();
    WFold& f = a.fold[(size_t)ti * kWCh + ch];
    const int ns = nseg > kWSeg ? -1 : nseg;
    if (ns > 0) {
      for (int i = (int)threadIdx.x; i < ns; i += kWThreads) {
        WSegment g;
        g.e = s_e[i];
        g.pad = 0;
        g.v = (int64_t)s_m[i];
        f.seg[i] = g;
      }
    }
    if (threadIdx.x == 0) {
      f.nseg = ns;
      WQuick& qk = a.quick[(size_t)ti * kWCh + ch];
      if (ns == 0) {
        qk.e = kWNone;
        qk.m = 0;
      } else if (ns == 1 && nsp == 0) {
        qk.e = s_e[0];
        qk.m = (int64_t)s_m[0];
      } else {
        qk.e = kWComplex;
        qk.m = 0;
      }
    }
  }
}

// s += u_e * M for a run of binade e; false if s is not in binade e or the
// run would leave it (the description does not apply: fold the summands).
__device__ __forceinline__ bool w_apply_run(double& s, int e, int64_t M) {
  if (!(s > 0.0) || w_binade(s) != e) return false;
  const int64_t si = (int64_t)ldexp(s, 52 - e) + M;   // (s / u exact: s is on the grid)
  if (si > (1ll << 53)) return false;
  s = ldexp((double)si, e - 52);                      // exact (si <= 2^53)
  return true;
}

// Every lane of the wave holds the same s (uniform); the tile's summands of
// fold ch added one at a time, in order (64 per load).
__device__ void w_fold_tile_seq(const WArgs& a, const WState& st, const WTile& t, int pass, int ch, double& s) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t b = t.start; b < t.end; b += 64) {
    const uint32_t p = b + lane;
    double x = 0.0;
    if (p < t.end) {
      const uint64_t r = st.src[p];
      const uint32_t c = (uint32_t)r;
      const uint32_t R = (c >> 16) & 0xFF, G = (c >> 8) & 0xFF, B = c & 0xFF;
      if (w_take(pass, st, R, G, B)) x = w_prod(ch, R, G, B, w_weight(a, r));
    }
    const uint32_t n = min(64u, t.end - b);
    for (uint32_t j = 0; j < n; ++j) s += __shfl(x, (int)j, 64);
  }
}

// A tile's description applied to s (fold ch); sequential when it does not apply.
__device__ void w_apply_tile(const WArgs& a, const WState& st, int ti, int pass, int ch, double& s) {
  const WFold& f = a.fold[(size_t)ti * kWCh + ch];
  bool ok = f.nseg >= 0;
  double v = s;
  for (int i = 0; ok && i < f.nseg; ++i) {
    const WSegment g = f.seg[i];
    if (g.e == kWSpecial) v += __longlong_as_double(g.v);
    else ok = w_apply_run(v, g.e, g.v);
  }
  if (ok) {
    s = v;
    return;
  }
  const WTile t = a.tiles[ti];
  if ((threadIdx.x & 63) == 0) atomicAdd((uint32_t*)&a.nodes[t.node].seq_tiles, 1u);
  w_fold_tile_seq(a, st, t, pass, ch, s);
}

__device__ void w_cut(WState& w, const double tm[3], const double tv[3]) {   // :388-403
  double maxv = tv[0], cut = tm[0];
  int axis = 0;
  if (maxv < tv[1]) { maxv = tv[1]; axis = 1; cut = tm[1]; }
  if (maxv < tv[2]) { axis = 2; cut = tm[2]; }
  w.axis = axis;
  w.cut = cut;
}

__device__ int32_t w_threshold(double cut) {   // cut < v <=> v >= thr (integer v in [0, 255])
  if (!(cut == cut)) return 256;
  if (cut < 0.0) return 0;
  if (cut >= 255.0) return 256;
  return (int32_t)floor(cut) + 1;
}

// The first 2-means decision after the split keeps every point of the node's
// box on its side of the cut (dq_kernels.hip cut_is_fixed_point, the same
// corner test and margin): the first 2-means pass then folds exactly the
// split's summands and is a fixed point.
__device__ bool w_cut_is_fixed_point(const WState& w) {
  const double M = (fabs(w.rr) + fabs(w.rg) + fabs(w.rb)) * 255.0 + fabs(w.lhs);
  if (!(M > 1e-30 && M < 1e30)) return false;
  const double mg = 1e-12 * M;
  const double c[3] = {w.rr, w.rg, w.rb};
  const int thr = w_threshold(w.cut);
  for (int side = 0; side < 2; ++side) {
    int lo[3], hi[3];
    for (int k = 0; k < 3; ++k) { lo[k] = w.box_lo[k]; hi[k] = w.box_hi[k]; }
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

__device__ void w_decision(WState& w) {   // :616-623
  w.lhs = 0.5 * (w.om[0] * w.om[0] - w.nm[0] * w.nm[0] + w.om[1] * w.om[1] - w.nm[1] * w.nm[1] +
                 w.om[2] * w.om[2] - w.nm[2] * w.nm[2]);
  w.rr = w.om[0] - w.nm[0];
  w.rg = w.om[1] - w.nm[1];
  w.rb = w.om[2] - w.nm[2];
}

// Pass step 4: per node (one wave), the folds in sequence order -- tiles in
// chunks of 64 (one per lane): consecutive run tiles of one binade applied as
// one integer sum, the others one by one -- then the reference's FP64
// epilogue of the pass (lane-uniform; lane 0 stores).
// One wave per fold (kWCh waves per node): the seven folds are independent
// chains over the same tiles, walked side by side; wave 0 then runs the
// pass's epilogue on the seven sums.
constexpr int kWChainThreads = 64 * kWCh;
__global__ __launch_bounds__(kWChainThreads) void wk_chain(WArgs a, int pass) {
  WState& st = a.nodes[blockIdx.x];
  if (st.done) return;
  const uint32_t lane = threadIdx.x & 63;
  const int ch = (int)(threadIdx.x >> 6);   // this wave's fold
  __shared__ double s_acc[kWCh];
  __shared__ uint32_t s_cnt;
  double s = 0.0;
  uint32_t cnt = 0;
  for (int b = st.tile_begin; b < st.tile_end; b += 64) {
    const int ti = b + (int)lane;
    const bool have = ti < st.tile_end;
    const int nt = min(64, st.tile_end - b);
    if (ch == 0) {
      uint32_t c = have ? a.quick[(size_t)ti * kWCh].cnt : 0u;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
      cnt += c;
    }
    WQuick qk;
    qk.e = kWNone;
    qk.m = 0;
    if (have) qk = a.quick[(size_t)ti * kWCh + ch];
    {
      // walk: [pos, next complex) by binade groups, then the complex tile
      const uint64_t cm = __ballot(have && qk.e == kWComplex);
      int pos = 0;
      while (pos < nt) {
        const uint64_t rest = cm & (pos >= 64 ? 0ull : (~0ull << pos));
        const int nc = rest ? (int)__builtin_ctzll(rest) : nt;
        // quick tiles [pos, nc): groups of equal binade, ascending -- sequence
        // order when the binades never decrease along the tiles (they do not
        // when every summand is classified right); otherwise tile by tile
        const bool run = have && (int)lane >= pos && (int)lane < nc && qk.e != kWNone && qk.e != kWComplex;
        uint64_t live = __ballot(run);
        int pmax = run ? qk.e : -0x7FFFFFFF;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int u = __shfl_up(pmax, o, 64);
          if (lane >= (uint32_t)o) pmax = max(pmax, u);
        }
        const int up = __shfl_up(pmax, 1, 64);     // (every lane: a shuffle's source lane must be active)
        const int before = lane == 0 ? -0x7FFFFFFF : up;
        if (__ballot(run && qk.e < before)) {
          for (int j = pos; j < nc; ++j) {
            const int ej = __shfl(qk.e, j, 64);
            const int64_t mj = __shfl(qk.m, j, 64);
            if (ej != kWNone && !w_apply_run(s, ej, mj)) w_apply_tile(a, st, b + j, pass, ch, s);
          }
          live = 0;
        }
        while (live) {
          int emin = ((live >> lane) & 1ull) ? qk.e : 0x7FFFFFFF;
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1) emin = min(emin, __shfl_xor(emin, o, 64));
          const bool mine = ((live >> lane) & 1ull) && qk.e == emin;
          const uint64_t grp = __ballot(mine);
          int64_t M = mine ? qk.m : 0;
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1) M += __shfl_xor(M, o, 64);
          if (!w_apply_run(s, emin, M)) {   // tile by tile (each one's own check)
            for (uint64_t g = grp; g; g &= g - 1) {
              const int j = (int)__builtin_ctzll(g);
              const int64_t mj = __shfl(qk.m, j, 64);
              if (!w_apply_run(s, emin, mj)) w_apply_tile(a, st, b + j, pass, ch, s);
            }
          }
          live &= ~grp;
        }
        if (nc < nt) w_apply_tile(a, st, b + nc, pass, ch, s);
        pos = nc + 1;
      }
    }
  }
  if (lane == 0) {
    s_acc[ch] = s;
    if (ch == 0) s_cnt = cnt;
  }
  __syncthreads();
  if (ch != 0) return;
  double acc[kWCh];
  for (int c = 0; c < kWCh; ++c) acc[c] = s_acc[c];
  cnt = s_cnt;
  // the pass's epilogue (every lane computes the same values; lane 0 stores)
  WState w = st;
  if (pass == WP_INIT) {   // DivQuantClusterInitMeanAndVar (:90-104), weighted
    double tm[3], tv[3];
    for (int c2 = 0; c2 < 3; ++c2) {
      tm[c2] = acc[c2];
      tv[c2] = acc[4 + c2];
      tv[c2] -= tm[c2] * tm[c2];
      w.tm[c2] = tm[c2];
      w.tv[c2] = tv[c2];
    }
    w_cut(w, tm, tv);
  } else if (pass == WP_SPLIT) {   // :561-598 (weighted: no data_weight scaling)
    w.nw = acc[3];
    w.ow = w.tw - w.nw;
    for (int c2 = 0; c2 < 3; ++c2) {
      w.nm[c2] = acc[c2];
      w.nm[c2] /= w.nw;
    }
    for (int c2 = 0; c2 < 3; ++c2) w.om[c2] = (w.tw * w.tm[c2] - w.nw * w.nm[c2]) / w.ow;
    for (int c2 = 0; c2 < 4; ++c2) w.prev[c2] = acc[c2];
    w_decision(w);
    w.n_new = cnt;
    w.iter = 0;
    if (a.fixed_point && cnt != 0 && w.ow > 0.0 && w_cut_is_fixed_point(w)) {
      // the first 2-means pass would fold the split's summands again: the
      // fixed point, with the split's squares (same membership, same order)
      for (int c2 = 0; c2 < 3; ++c2) w.nsq[c2] = acc[4 + c2];
      w.iter = 1;
      w.done_it = 1;
      w.proven = 1;
      w.done = 1;
    }
  } else {   // 2-means pass a.it (:613-811)
    const bool last = a.it == a.max_iters - 1;
    const bool fixed = a.fixed_point && !last &&
                       __double_as_longlong(acc[0]) == __double_as_longlong(w.prev[0]) &&
                       __double_as_longlong(acc[1]) == __double_as_longlong(w.prev[1]) &&
                       __double_as_longlong(acc[2]) == __double_as_longlong(w.prev[2]) &&
                       __double_as_longlong(acc[3]) == __double_as_longlong(w.prev[3]);
    w.nw = acc[3];
    w.n_new = cnt;
    for (int c2 = 0; c2 < 3; ++c2) {
      w.nm[c2] = acc[c2];
      w.nm[c2] /= w.nw;                                                  // :800-802
    }
    w.ow = w.tw - w.nw;                                                  // :805
    for (int c2 = 0; c2 < 3; ++c2) w.om[c2] = (w.tw * w.tm[c2] - w.nw * w.nm[c2]) / w.ow;   // :808-810
    for (int c2 = 0; c2 < 3; ++c2) w.nsq[c2] = acc[4 + c2];
    for (int c2 = 0; c2 < 4; ++c2) w.prev[c2] = acc[c2];
    w.iter = a.it + 1;
    if (last || fixed) {
      w.done_it = a.it + 1;
      w.done = 1;
    } else {
      w_decision(w);   // the next pass's decision
    }
  }
  if (lane == 0) {
    st = w;
    if (!w.done && pass != WP_INIT)   // (host-coherent: a flag, every writer stores 1)
      __hip_atomic_store(a.active, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Round end, step 1: per node (one wave), the tiles' old / new bases -- a
// tile's new-side count under the final membership is its count of taken
// summands in the node's last pass (tsum[.][7]: the pass whose decision
// produced the final sums; a final node's tiles are skipped by later passes)
// -- and the node's results (:820-871) into res.
__global__ __launch_bounds__(64) void wk_part_scan(WArgs a) {
  const WState& st = a.nodes[blockIdx.x];
  const int lane = (int)threadIdx.x;
  uint32_t run_o = 0, run_n = 0;
  for (int b = st.tile_begin; b < st.tile_end; b += 64) {
    const int i = b + lane;
    uint32_t nw = 0, ol = 0;
    if (i < st.tile_end) {
      const WTile t = a.tiles[i];
      nw = (uint32_t)a.tsum[(size_t)i * 8 + 7];
      ol = (t.end - t.start) - nw;
    }
    uint32_t io = ol, in = nw;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(io, o, 64), v = __shfl_up(in, o, 64);
      if (lane >= o) { io += u; in += v; }
    }
    if (i < st.tile_end) {
      a.pbase[(size_t)i * 2] = run_o + io - ol;
      a.pbase[(size_t)i * 2 + 1] = run_n + in - nw;
    }
    run_o += __shfl(io, 63, 64);
    run_n += __shfl(in, 63, 64);
  }
  if (lane == 0) {
    NodeResult r;
    double nv[3], ov[3];
    for (int c = 0; c < 3; ++c) nv[c] = st.nsq[c] / st.nw - st.nm[c] * st.nm[c];   // :836-838
    for (int c = 0; c < 3; ++c) {
      const double dn = st.nm[c] - st.tm[c];
      const double dox = st.om[c] - st.tm[c];
      ov[c] = ((st.tw * st.tv[c] - st.nw * (nv[c] + dn * dn)) / st.ow) - dox * dox;   // :845-855
    }
    for (int c = 0; c < 3; ++c) {
      r.om[c] = st.om[c]; r.nm[c] = st.nm[c]; r.nv[c] = nv[c]; r.ov[c] = ov[c];
      r.tm[c] = st.tm[c]; r.tv[c] = st.tv[c];
    }
    r.nw = st.nw;
    r.ow = st.ow;
    r.tse_old = st.ow * (ov[0] + ov[1] + ov[2]);   // :870-871
    r.tse_new = st.nw * (nv[0] + nv[1] + nv[2]);
    r.n_new = st.n_new;
    r.n_new_local = run_n;
    r.done_it = st.done_it;
    r.proven = st.proven;
    r.pad = (int32_t)st.seq_tiles;
    r.len_local = st.len;
    r.tag = 0;
    a.res[blockIdx.x] = r;
  }
}

// Step 2: per tile, the stable partition of its records by the final
// decision (old half first; point order kept in both halves, as the
// reference's gather by ascending index, :894-1026): each record to its rank
// in the tile's old / new run in LDS, then both runs out in coalesced 8-B
// stores.
__global__ __launch_bounds__(kWThreads) void wk_part_scatter(WArgs a) {
  const WTile t = a.tiles[blockIdx.x];
  const WState& st = a.nodes[t.node];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t p0 = t.start + (uint32_t)kWPer * threadIdx.x;
  const uint32_t nv = p0 < t.end ? min((uint32_t)kWPer, t.end - p0) : 0u;
  // The tile's records in through LDS: coalesced global loads (lane-
  // interleaved), then each lane reads its kWPer consecutive records (one
  // pad slot per kWPer records: conflict-free 8-B reads).  Loaded once (the
  // decision needs only the colour: no weights) and kept for the staging.
  __shared__ uint64_t s_rec[kWTile + kWTile / kWPer];
#pragma unroll
  for (int k = 0; k < kWPer; ++k) {
    const uint32_t p = (uint32_t)(k * kWThreads) + threadIdx.x;
    if (t.start + p < t.end) s_rec[p + p / (uint32_t)kWPer] = st.src[t.start + p];
  }
  __syncthreads();
  uint64_t rv[kWPer];
  uint32_t take = 0;
#pragma unroll
  for (int k = 0; k < kWPer; ++k) {
    rv[k] = 0;
    if ((uint32_t)k < nv) {
      rv[k] = s_rec[threadIdx.x * (uint32_t)(kWPer + 1) + (uint32_t)k];
      const uint32_t c = (uint32_t)rv[k];
      if (w_take(WP_KM, st, (c >> 16) & 0xFF, (c >> 8) & 0xFF, c & 0xFF)) take |= 1u << k;
    }
  }
  const uint32_t nn = (uint32_t)__popc(take), no = nv - nn;
  uint32_t io = no, in = nn;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(io, o, 64), v = __shfl_up(in, o, 64);
    if (lane >= (uint32_t)o) { io += u; in += v; }
  }
  __shared__ uint32_t s_w[kWThreads / 64][2];
  if (lane == 63) { s_w[wv][0] = io; s_w[wv][1] = in; }
  __syncthreads();   // (also: every lane's records are out of s_rec)
  uint32_t to = io - no, tn = in - nn, tno = 0;   // this lane's ranks in the tile's runs; the old run's size
  for (uint32_t w = 0; w < kWThreads / 64; ++w) {
    if (w < wv) { to += s_w[w][0]; tn += s_w[w][1]; }
    tno += s_w[w][0];
  }
#pragma unroll
  for (int k = 0; k < kWPer; ++k) {
    if ((uint32_t)k < nv) {
      if ((take >> k) & 1u) s_rec[tno + tn++] = rv[k];
      else s_rec[to++] = rv[k];
    }
  }
  __syncthreads();
  const uint32_t tlen = t.end - t.start;
  const uint32_t n_old = st.len - st.n_new;
  uint64_t* const dold = st.dst + st.off + a.pbase[(size_t)blockIdx.x * 2];
  uint64_t* const dnew = st.dst + st.off + n_old + a.pbase[(size_t)blockIdx.x * 2 + 1];
  for (uint32_t i = threadIdx.x; i < tlen; i += kWThreads) {
    if (i < tno) dold[i] = s_rec[i];
    else dnew[i - tno] = s_rec[i];
  }
}
}  // namespace

// --- launchers ----------------------------------------------------------------
static inline uint32_t grid_for(uint32_t n) {
  const uint32_t g = (n + 255u) / 256u;
  return g == 0 ? 1u : (g > 65535u ? 65535u : g);
}

// The colour table's scratch: the runs (at most one per pixel), hist / off
// [blocks][groups], the groups' totals, offsets and colour counts.
static uint32_t ct_chunk(uint32_t n) {   // pixels per ct_runs block: at most kCtMaxBlocks blocks
  constexpr uint32_t kCtMaxBlocks = 256, kStep = (kCtThreads / 64) * 1024u;
  const uint64_t per = ((uint64_t)n + kCtMaxBlocks - 1) / kCtMaxBlocks;
  return (uint32_t)std::max<uint64_t>(kStep, (per + kStep - 1) / kStep * kStep);
}

size_t color_table_scratch_bytes(uint32_t n) {
  const uint32_t nblk = (uint32_t)(((uint64_t)n + ct_chunk(n) - 1) / ct_chunk(n));
  return (((size_t)n * 8 + 255) & ~(size_t)255) + (((size_t)nblk * kCtGroups * 4 + 255) & ~(size_t)255) +
         4 * ((((size_t)kCtGroups + 1) * 4 + 255) & ~(size_t)255);
}

int launch_color_table(const uint32_t* px, uint32_t n, void* scratch, size_t scratch_bytes, uint64_t* rec,
                       uint32_t* h_nu, hipStream_t stream) {
  if (n == 0) {
    *h_nu = 0;
    return 0;
  }
  if (scratch_bytes < color_table_scratch_bytes(n)) return -1;
  if (hipFuncSetAttribute((const void*)ct_group, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCtGroupLds) !=
      hipSuccess)
    return -2;
  const uint32_t chunk = ct_chunk(n), nblk = (uint32_t)(((uint64_t)n + chunk - 1) / chunk);
  char* p = static_cast<char*>(scratch);
  auto take = [&](size_t bytes) { char* q = p; p += (bytes + 255) & ~(size_t)255; return q; };
  uint64_t* part = reinterpret_cast<uint64_t*>(take((size_t)n * 8));
  uint32_t* hist = reinterpret_cast<uint32_t*>(take((size_t)nblk * kCtGroups * 4));
  uint32_t* gtot = reinterpret_cast<uint32_t*>(take(((size_t)kCtGroups + 1) * 4));
  uint32_t* gstart = reinterpret_cast<uint32_t*>(take(((size_t)kCtGroups + 1) * 4));
  uint32_t* ucnt = reinterpret_cast<uint32_t*>(take(((size_t)kCtGroups + 1) * 4));
  uint32_t* uoff = reinterpret_cast<uint32_t*>(take(((size_t)kCtGroups + 1) * 4));
  ct_runs<true><<<dim3(nblk), dim3(kCtThreads), 0, stream>>>(px, n, chunk, hist, nullptr, nullptr);
  ct_colscan<<<dim3((kCtGroups + 63) / 64), dim3(1024), 0, stream>>>(hist, nblk, gtot);
  ct_gscan<<<dim3(1), dim3(1024), 0, stream>>>(gtot, gstart, kCtGroups);
  ct_runs<false><<<dim3(nblk), dim3(kCtThreads), 0, stream>>>(px, n, chunk, hist, gstart, part);
  uint32_t nb = 1;   // bits of n - 1: first >> (nb - 4) is a 4-bit bin, monotone in first
  while (nb < 32 && ((n - 1u) >> nb) != 0) ++nb;
  const uint32_t binshift = nb > 4 ? nb - 4 : 0;
  ct_group<<<dim3(kCtGroups), dim3(kCtGroupThreads), kCtGroupLds, stream>>>(part, gstart, ucnt, binshift);
  ct_gscan<<<dim3(1), dim3(1024), 0, stream>>>(ucnt, uoff, kCtGroups);
  ct_compact<<<dim3(kCtGroups), dim3(256), 0, stream>>>(part, gstart, uoff, rec);
  if (hipGetLastError() != hipSuccess) return -2;
  if (hipMemcpyAsync(h_nu, uoff + kCtGroups, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return -2;
  return 0;
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



void launch_wpass(int pass, const WArgs& a, hipStream_t stream) {
  if (a.ntiles <= 0 || a.nn <= 0) return;
  wk_tilesum<<<dim3(a.ntiles), dim3(kWThreads), 0, stream>>>(a, pass);
  wk_prefix<<<dim3(a.nn), dim3(64 * kWCh), 0, stream>>>(a);
  wk_classify_fast<<<dim3(a.ntiles), dim3(kWThreads), 0, stream>>>(a, pass);
  wk_classify<<<dim3(((a.ntiles + 7) / 8) * 8 * kWCh), dim3(kWThreads), 0, stream>>>(a, pass);
  wk_chain<<<dim3(a.nn), dim3(kWChainThreads), 0, stream>>>(a, pass);
}

void launch_wfinish(const WArgs& a, hipStream_t stream) {
  if (a.ntiles <= 0 || a.nn <= 0) return;
  wk_part_scan<<<dim3(a.nn), dim3(64), 0, stream>>>(a);
  wk_part_scatter<<<dim3(a.ntiles), dim3(kWThreads), 0, stream>>>(a);
}

}  // namespace dq
