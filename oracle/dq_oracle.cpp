// =============================================================================
// oracle/dq_oracle.cpp -- CPU restatement of the DivQuant hot path.
//
// TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py may load this library, and only as the checker
// (or the timed CPU baseline) -- never as the thing measured or shipped.  The
// product library (clusteringsegmentation-1_amd/csrc) must not link it.
//
// What it restates (all citations relative to /root/reference):
//   * quant_recurse                    DivQuant/quant_util.cpp:20-158
//   * quant_varpart_fast, UW dispatch  DivQuant/DivQuantCluster.cpp:1099-1179
//   * DivQuantClusterInitMeanAndVar    DivQuant/DivQuantCluster.cpp:36-123
//   * DivQuantCluster<true,MT,true>    DivQuant/DivQuantCluster.cpp:133-1097
//   * map_colors_mps                   DivQuant/DivQuantMapColors.cpp:243-539
//
// How it is restated (deliberately NOT the reference's code shape):
//   - every cluster keeps its own vector of packed pixels instead of the
//     reference's member[] array + O(N) gather per split (:894-1026).  Uniform
//     weight sums are exact integers, so visiting order is irrelevant;
//   - sums are uint64 integers converted to double once; the reference's
//     0xFFFF-point uint32 chunks folded into doubles (:438-559, :639-777) are
//     exact too (every partial < 2^53), so the doubles are identical;
//   - the FP64 epilogue is spelled out operation by operation with the same
//     evaluation order as the reference (no contraction: built -ffp-contract=off).
//
// Parity pin: tests/test_oracle_golden.py checks this file against the 7
// Test/DivQuantTest.m known-answer tests and against outputs of the unmodified
// reference compiled by oracle/Makefile (fixtures in tests/golden/).
// =============================================================================
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

struct Sums {            // exact integer statistics of a point set
  uint64_t n = 0;
  uint64_t s[3] = {0, 0, 0};   // sum R, G, B
  uint64_t q[3] = {0, 0, 0};   // sum R^2, G^2, B^2
};

inline void unpack(uint32_t p, uint32_t c[3]) {
  c[0] = (p >> 16) & 0xFF;  // R
  c[1] = (p >> 8) & 0xFF;   // G
  c[2] = p & 0xFF;          // B
}

struct Cluster {
  std::vector<uint32_t> px;  // packed 0x00RRGGBB points of this cluster
  double weight = 0.0;
  double mean[3] = {0, 0, 0};
  double var[3] = {0, 0, 0};
  double tse = 0.0;
  int64_t size = 0;
};

}  // namespace

extern "C" {

// One greedy DivQuant run, uniform-weight path (allPixelsUnique=1, num_bits=8,
// dec_factor=1).  Writes <=K colours to ct and the number to *k_inout, exactly
// like DivQuantCluster's tail (DivQuantCluster.cpp:1029-1094).
//   means_out  : optional [K*3] final double centroids per cluster index
//                (NaN-free only where sizes_out>0) -- the north star's 1e-5 check.
//   sizes_out  : optional [K] cluster sizes per index.
//   trace_out  : optional [(K-1)*4] per split: new_index, old_index, |C|, |new|.
int dqo_cluster(uint32_t num_points, const uint32_t* data, uint32_t* k_inout,
                uint32_t* ct, int max_iters, double* means_out,
                int64_t* sizes_out, int64_t* trace_out) {
  if (num_points == 0 || *k_inout == 0 || max_iters < 1) return -1;
  const int K = (int)*k_inout;
  // get_double_scale: 1/(ceil(1/1)*ceil(N/1)) (DivQuantMapColors.cpp:205-220)
  const double s = 1.0 / (std::ceil(1 / 1.0) * std::ceil(num_points / 1.0));

  std::vector<Cluster> cl(K);
  cl[0].px.assign(data, data + num_points);
  for (auto& p : cl[0].px) p &= 0xFFFFFF;
  cl[0].weight = 1.0;                       // :329, literal 1.0 (not N*s)
  cl[0].size = num_points;
  int old_index = 0;

  for (int new_index = 1; new_index < K; ++new_index) {
    Cluster& C = cl[old_index];
    const double tw = C.weight;
    double tm[3], tv[3];
    if (new_index == 1) {                   // :355-358 -> InitMeanAndVar :49-104
      Sums r;
      for (uint32_t p : C.px) {
        uint32_t c[3];
        unpack(p, c);
        for (int a = 0; a < 3; ++a) { r.s[a] += c[a]; r.q[a] += c[a] * c[a]; }
      }
      for (int a = 0; a < 3; ++a) {
        double m = (double)r.s[a];
        double v = (double)r.q[a];
        m *= s;
        v *= s;
        v -= m * m;
        tm[a] = m;
        tv[a] = v;
      }
    } else {                                // :365-374
      for (int a = 0; a < 3; ++a) { tm[a] = C.mean[a]; tv[a] = C.var[a]; }
    }

    // STEPS 1&2 (:388-403): max-variance axis, strict '<' keeps lower axis.
    int axis = 0;
    double maxv = tv[0], cut = tm[0];
    if (maxv < tv[1]) { maxv = tv[1]; axis = 1; cut = tm[1]; }
    if (maxv < tv[2]) { axis = 2; cut = tm[2]; }

    // STEP 3 split pass (:438-559): new side iff cut_pos < v_axis.
    Sums ns;
    for (uint32_t p : C.px) {
      uint32_t c[3];
      unpack(p, c);
      if (cut < (double)c[axis]) {
        ns.n++;
        for (int a = 0; a < 3; ++a) ns.s[a] += c[a];
      }
    }
    double nm[3], om[3], nw, ow;
    nw = (double)ns.n * s;                               // :566
    ow = tw - nw;                                        // :576
    for (int a = 0; a < 3; ++a) nm[a] = ((double)ns.s[a] * s) / nw;   // :562,579
    for (int a = 0; a < 3; ++a) om[a] = (tw * tm[a] - nw * nm[a]) / ow;  // :596

    // Local 2-means (:613-811).
    std::vector<uint32_t> keep, moved;
    double nvq[3] = {0, 0, 0};
    int64_t new_size = 0;
    for (int it = 0; it < max_iters; ++it) {
      const bool last = (it == max_iters - 1);
      double lhs = 0.5 * (om[0] * om[0] - nm[0] * nm[0] + om[1] * om[1] -
                          nm[1] * nm[1] + om[2] * om[2] - nm[2] * nm[2]);  // :616
      double rr = om[0] - nm[0], rg = om[1] - nm[1], rb = om[2] - nm[2];
      Sums k;
      if (last) { keep.clear(); moved.clear(); }
      for (uint32_t p : C.px) {
        uint32_t c[3];
        unpack(p, c);
        double red = c[0], green = c[1], blue = c[2];
        if (lhs < ((rr * red) + (rg * green) + (rb * blue))) {   // :683 -> old
          if (last) keep.push_back(p);
        } else {                                                 // new (ties, NaN)
          k.n++;
          for (int a = 0; a < 3; ++a) k.s[a] += c[a];
          if (last) {
            for (int a = 0; a < 3; ++a) k.q[a] += c[a] * c[a];
            moved.push_back(p);
          }
        }
      }
      new_size = (int64_t)k.n;
      double nsum[3], nsq[3];
      for (int a = 0; a < 3; ++a) {
        nsum[a] = (double)k.s[a] * s;                   // :788-790
        nsq[a] = (double)k.q[a] * s;                    // :794-796
      }
      nw = (double)new_size * s;                        // :792
      for (int a = 0; a < 3; ++a) nm[a] = nsum[a] / nw; // :800-802
      ow = tw - nw;                                     // :805
      for (int a = 0; a < 3; ++a) om[a] = (tw * tm[a] - nw * nm[a]) / ow;  // :808
      for (int a = 0; a < 3; ++a) nvq[a] = nsq[a];
    }

    Cluster& D = cl[new_index];
    const int64_t parent_size = C.size;
    if (trace_out) {
      int64_t* t = trace_out + 4 * (new_index - 1);
      t[0] = new_index; t[1] = old_index; t[2] = parent_size; t[3] = new_size;
    }
    C.size = parent_size - new_size;                    // :820-821
    D.size = new_size;
    for (int a = 0; a < 3; ++a) { C.mean[a] = om[a]; D.mean[a] = nm[a]; }
    C.px.swap(keep);
    D.px.swap(moved);
    std::vector<uint32_t>().swap(keep);
    std::vector<uint32_t>().swap(moved);

    if (new_index == K - 1) break;                      // :823-832

    double nv[3], ov[3];
    for (int a = 0; a < 3; ++a) nv[a] = nvq[a] / nw - nm[a] * nm[a];   // :836-838
    for (int a = 0; a < 3; ++a) {                                       // :845-855
      double dn = nm[a] - tm[a];
      double dox = om[a] - tm[a];
      ov[a] = ((tw * tv[a] - nw * (nv[a] + dn * dn)) / ow) - dox * dox;
    }
    for (int a = 0; a < 3; ++a) { C.var[a] = ov[a]; D.var[a] = nv[a]; }
    C.weight = ow;                                      // :862-863
    D.weight = nw;
    C.tse = ow * (ov[0] + ov[1] + ov[2]);               // :870-871
    D.tse = nw * (nv[0] + nv[1] + nv[2]);

    // STEP 4 (:876-887): first index with max TSE above DBL_MIN; if none,
    // old_index is left unchanged (the old half is split again).
    double best = DBL_MIN;
    for (int ic = 0; ic <= new_index; ++ic) {
      if (best < cl[ic].tse) { best = cl[ic].tse; old_index = ic; }
    }
  }

  // Final centres (:1029-1094): round, pack, drop empty clusters.
  int out = 0;
  for (int ic = 0; ic < K; ++ic) {
    if (means_out) {
      for (int a = 0; a < 3; ++a) means_out[3 * ic + a] = cl[ic].mean[a];
    }
    if (sizes_out) sizes_out[ic] = cl[ic].size;
    if (cl[ic].size > 0) {
      uint32_t R = (uint8_t)(cl[ic].mean[0] + 0.5);
      uint32_t G = (uint8_t)(cl[ic].mean[1] + 0.5);
      uint32_t B = (uint8_t)(cl[ic].mean[2] + 0.5);
      ct[out++] = (R << 16) | (G << 8) | B;
    }
  }
  *k_inout = (uint32_t)out;
  return K - out;   // number of empty clusters
}

// map_colors_mps restated (DivQuantMapColors.cpp:243-539): palette sorted by
// R+G+B with std::sort (same comparator => same unstable order on the same
// libstdc++, :227-238), start entry from a rounded-midpoint LUT (:331-383),
// alternating up/down walk pruned by floor(d^2/3) (:285-311, :385-521).
struct PalEntry { int r, g, b, w; };

void dqo_map(const uint32_t* in, uint32_t n, uint32_t* out,
             const uint32_t* ct, int k) {
  std::vector<PalEntry> pal(k);
  for (int i = 0; i < k; ++i) {
    uint32_t c[3];
    unpack(ct[i], c);
    pal[i] = {(int)c[0], (int)c[1], (int)c[2], (int)(c[0] + c[1] + c[2])};
  }
  std::sort(pal.begin(), pal.end(),
            [](const PalEntry& a, const PalEntry& b) { return a.w < b.w; });
  int ssd_buf[2 * 765 + 1];
  int* ssd = ssd_buf + 765;
  ssd[0] = 0;
  for (int d = 1; d <= 765; ++d) ssd[d] = ssd[-d] = (int)((d * d) / 3.0);
  int start[766];
  auto mid = [&](int i) { return (int)(0.5 * (pal[i].w + pal[i + 1].w) + 0.5); };
  int lo = k >= 2 ? mid(0) : 1;
  for (int v = 0; v < lo; ++v) start[v] = 0;
  int hi = k >= 2 ? mid(k - 2) : 1;
  for (int v = hi; v < 766; ++v) start[v] = k - 1;
  for (int i = 1; i < k - 1; ++i)
    for (int v = mid(i - 1); v < mid(i); ++v) start[v] = i;

  for (uint32_t ip = 0; ip < n; ++ip) {
    uint32_t c[3];
    unpack(in[ip], c);
    const int r = c[0], g = c[1], b = c[2], sum = r + g + b;
    int best = start[sum];
    auto d2 = [&](int i) {
      int dr = r - pal[i].r, dg = g - pal[i].g, db = b - pal[i].b;
      return dr * dr + dg * dg + db * db;
    };
    int bestd = d2(best);
    int up = best, dn = best;
    bool go_up = true, go_dn = true;
    while (go_up || go_dn) {
      if (go_up) {
        ++up;
        if (up > k - 1 || ssd[sum - pal[up].w] >= bestd) go_up = false;
        else { int d = d2(up); if (d < bestd) { bestd = d; best = up; } }
      }
      if (go_dn) {
        --dn;
        if (dn < 0 || ssd[sum - pal[dn].w] >= bestd) go_dn = false;
        else { int d = d2(dn); if (d < bestd) { bestd = d; best = dn; } }
      }
    }
    out[ip] = ((uint32_t)pal[best].r << 16) | ((uint32_t)pal[best].g << 8) |
              (uint32_t)pal[best].b;
  }
}

// The identity the GPU map kernel relies on, evaluated by brute force: with the
// same sorted palette and start LUT as dqo_map, the answer is the entry that
// minimises (squared distance, MPS visit rank), rank(j) = 2(j-s)-1 for j > s
// and 2(s-j) otherwise (s = start[R+G+B]).  Test infrastructure only.
void dqo_map_argmin(const uint32_t* in, uint32_t n, uint32_t* out,
                    const uint32_t* ct, int k) {
  std::vector<PalEntry> pal(k);
  for (int i = 0; i < k; ++i) {
    uint32_t c[3];
    unpack(ct[i], c);
    pal[i] = {(int)c[0], (int)c[1], (int)c[2], (int)(c[0] + c[1] + c[2])};
  }
  std::sort(pal.begin(), pal.end(),
            [](const PalEntry& a, const PalEntry& b) { return a.w < b.w; });
  int start[766];
  auto mid = [&](int i) { return (int)(0.5 * (pal[i].w + pal[i + 1].w) + 0.5); };
  int lo = k >= 2 ? mid(0) : 1;
  for (int v = 0; v < lo; ++v) start[v] = 0;
  int hi = k >= 2 ? mid(k - 2) : 1;
  for (int v = hi; v < 766; ++v) start[v] = k - 1;
  for (int i = 1; i < k - 1; ++i)
    for (int v = mid(i - 1); v < mid(i); ++v) start[v] = i;
  for (uint32_t ip = 0; ip < n; ++ip) {
    uint32_t c[3];
    unpack(in[ip], c);
    const int s0 = start[c[0] + c[1] + c[2]];
    uint64_t best = ~0ull;
    int bj = 0;
    for (int j = 0; j < k; ++j) {
      const int dr = (int)c[0] - pal[j].r, dg = (int)c[1] - pal[j].g, db = (int)c[2] - pal[j].b;
      const uint64_t d = (uint64_t)(dr * dr + dg * dg + db * db);
      const int t = j - s0;
      const uint64_t rank = t > 0 ? (uint64_t)(2 * t - 1) : (uint64_t)(-2 * t);
      const uint64_t key = (d << 32) | rank;
      if (key < best) { best = key; bj = j; }
    }
    out[ip] = ((uint32_t)pal[bj].r << 16) | ((uint32_t)pal[bj].g << 8) | (uint32_t)pal[bj].b;
  }
}

// quant_recurse restated (quant_util.cpp:20-158), UW path only, no stdout
// timer lines: cluster -> first-seen colortable dedup (:93-118) -> map (:139).
int dqo_quant_recurse(uint32_t n, const uint32_t* in, uint32_t* out,
                      uint32_t* k_inout, uint32_t* ct) {
  int empty = dqo_cluster(n, in, k_inout, ct, 10, nullptr, nullptr, nullptr);
  if (empty < 0) return empty;
  std::unordered_set<uint32_t> seen;
  uint32_t m = 0;
  for (uint32_t i = 0; i < *k_inout; ++i)
    if (seen.insert(ct[i]).second) ct[m++] = ct[i];
  *k_inout = m;
  dqo_map(in, n, out, ct, (int)m);
  return empty;
}

// ---------------------------------------------------------------------------
// Weighted path (allPixelsUnique=0): quant_varpart_fast's calc_color_table
// dedup + DivQuantCluster<false,MT,true> (DivQuantCluster.cpp:1133-1138,
// :1163-1166).  Every weighted statistic is a sequential FP64 fold over the
// cluster's points in point order, so the restatement keeps each cluster's
// (colour, weight) points in order (the reference gathers them by ascending
// point index, :894-1026) and folds exactly as the reference does.

// calc_color_table restated (DivQuantMapColors.cpp:82-203): unique colours of
// in[0..n) with weights norm*count, ordered by hash bucket ((R*33023 +
// G*30013 + B*27011) & 0x7fffffff) % 20023 ascending and, inside a bucket,
// by first occurrence DESCENDING (chains are prepended, :154-158).  Returns the
// number of colours.  (numRows = 1, dec_factor = 1: the quant_recurse call.)
static int color_table_norm(uint32_t n, const uint32_t* in, uint32_t* colours, double* weights,
                            double norm);

int dqo_color_table(uint32_t n, const uint32_t* in, uint32_t* colours, double* weights) {
  const double norm = 1.0 / (std::ceil(1 / 1.0) * std::ceil(n / 1.0));   // :184
  return color_table_norm(n, in, colours, weights, norm);
}

static int color_table_norm(uint32_t n, const uint32_t* in, uint32_t* colours, double* weights,
                            double norm) {
  struct E { uint32_t c, first, count, hash; };
  std::unordered_map<uint32_t, uint32_t> at;
  std::vector<E> es;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t c = in[i] & 0xFFFFFF;
    auto it = at.find(c);
    if (it != at.end()) { es[it->second].count++; continue; }
    const long R = (c >> 16) & 0xFF, G = (c >> 8) & 0xFF, B = c & 0xFF;
    at.emplace(c, (uint32_t)es.size());
    es.push_back({c, i, 1u, (uint32_t)(((R * 33023 + G * 30013 + B * 27011) & 0x7fffffff) % 20023)});
  }
  std::vector<uint32_t> ord(es.size());
  for (size_t i = 0; i < ord.size(); ++i) ord[i] = (uint32_t)i;
  std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
    return es[a].hash != es[b].hash ? es[a].hash < es[b].hash : es[a].first > es[b].first;
  });
  for (size_t i = 0; i < ord.size(); ++i) {
    colours[i] = es[ord[i]].c;
    weights[i] = norm * es[ord[i]].count;                                  // :195
  }
  return (int)es.size();
}

// DivQuantCluster<false,*,true> restated over (colour, weight) points.
// Outputs as dqo_cluster; sizes and the trace count points (unique colours).
// num_bits < 8 (cut_bits input): final centres shifted left by 8 - num_bits
// (DivQuantCluster.cpp:1030, :1050-1052).
static int cluster_weighted_bits(uint32_t num_points, const uint32_t* data, const double* wts,
                                 uint32_t* k_inout, uint32_t* ct, int max_iters, double* means_out,
                                 int64_t* sizes_out, int64_t* trace_out, int num_bits);

int dqo_cluster_weighted(uint32_t num_points, const uint32_t* data, const double* wts,
                         uint32_t* k_inout, uint32_t* ct, int max_iters, double* means_out,
                         int64_t* sizes_out, int64_t* trace_out) {
  return cluster_weighted_bits(num_points, data, wts, k_inout, ct, max_iters, means_out, sizes_out,
                               trace_out, 8);
}

static int cluster_weighted_bits(uint32_t num_points, const uint32_t* data, const double* wts,
                                 uint32_t* k_inout, uint32_t* ct, int max_iters, double* means_out,
                                 int64_t* sizes_out, int64_t* trace_out, int num_bits) {
  if (num_points == 0 || *k_inout == 0 || max_iters < 1) return -1;
  const int K = (int)*k_inout;
  struct P { uint32_t c; double w; };
  struct WC {
    std::vector<P> px;
    double weight = 0.0, mean[3] = {0, 0, 0}, var[3] = {0, 0, 0}, tse = 0.0;
    int64_t size = 0;
  };
  std::vector<WC> cl(K);
  cl[0].px.resize(num_points);
  for (uint32_t i = 0; i < num_points; ++i) cl[0].px[i] = {data[i] & 0xFFFFFF, wts[i]};
  cl[0].weight = 1.0;                                   // :329
  cl[0].size = num_points;
  int old_index = 0;
  for (int new_index = 1; new_index < K; ++new_index) {
    WC& C = cl[old_index];
    const double tw = C.weight;
    double tm[3], tv[3];
    if (new_index == 1) {                               // InitMeanAndVar, weighted (:73-85, :99-101)
      double m[3] = {0, 0, 0}, v[3] = {0, 0, 0};
      for (const P& p : C.px) {
        uint32_t c[3];
        unpack(p.c, c);
        for (int a = 0; a < 3; ++a) {
          m[a] += p.w * c[a];
          v[a] += p.w * (c[a] * c[a]);
        }
      }
      for (int a = 0; a < 3; ++a) {
        v[a] -= m[a] * m[a];
        tm[a] = m[a];
        tv[a] = v[a];
      }
    } else {
      for (int a = 0; a < 3; ++a) { tm[a] = C.mean[a]; tv[a] = C.var[a]; }
    }
    int axis = 0;                                       // :388-403
    double maxv = tv[0], cut = tm[0];
    if (maxv < tv[1]) { maxv = tv[1]; axis = 1; cut = tm[1]; }
    if (maxv < tv[2]) { axis = 2; cut = tm[2]; }
    // split pass (:438-559), weighted folds in point order
    double nm[3] = {0, 0, 0}, nw = 0.0, om[3], ow;
    for (const P& p : C.px) {
      uint32_t c[3];
      unpack(p.c, c);
      if (cut < (double)c[axis]) {
        for (int a = 0; a < 3; ++a) nm[a] += p.w * c[a];
        nw += p.w;
      }
    }
    ow = tw - nw;                                       // :576
    for (int a = 0; a < 3; ++a) nm[a] /= nw;            // :579-581
    for (int a = 0; a < 3; ++a) om[a] = (tw * tm[a] - nw * nm[a]) / ow;   // :596-598
    std::vector<P> keep, moved;
    double nvq[3] = {0, 0, 0};
    int64_t new_size = 0;
    for (int it = 0; it < max_iters; ++it) {            // :613-811
      const bool last = it == max_iters - 1;
      const double lhs = 0.5 * (om[0] * om[0] - nm[0] * nm[0] + om[1] * om[1] - nm[1] * nm[1] +
                                om[2] * om[2] - nm[2] * nm[2]);
      const double rr = om[0] - nm[0], rg = om[1] - nm[1], rb = om[2] - nm[2];
      double sm[3] = {0, 0, 0}, sq[3] = {0, 0, 0};
      nw = 0.0;
      new_size = 0;
      if (last) { keep.clear(); moved.clear(); }
      for (const P& p : C.px) {
        uint32_t c[3];
        unpack(p.c, c);
        const double red = c[0], green = c[1], blue = c[2];
        if (lhs < ((rr * red) + (rg * green) + (rb * blue))) {
          if (last) keep.push_back(p);
        } else {
          sm[0] += p.w * red;
          sm[1] += p.w * green;
          sm[2] += p.w * blue;
          if (last) {
            for (int a = 0; a < 3; ++a) sq[a] += p.w * (c[a] * c[a]);
            moved.push_back(p);
          }
          nw += p.w;
          new_size++;
        }
      }
      for (int a = 0; a < 3; ++a) nm[a] = sm[a] / nw;   // :800-802
      ow = tw - nw;                                     // :805
      for (int a = 0; a < 3; ++a) om[a] = (tw * tm[a] - nw * nm[a]) / ow;
      for (int a = 0; a < 3; ++a) nvq[a] = sq[a];
    }
    WC& D = cl[new_index];
    const int64_t parent_size = C.size;
    if (trace_out) {
      int64_t* t = trace_out + 4 * (new_index - 1);
      t[0] = new_index; t[1] = old_index; t[2] = parent_size; t[3] = new_size;
    }
    C.size = parent_size - new_size;
    D.size = new_size;
    for (int a = 0; a < 3; ++a) { C.mean[a] = om[a]; D.mean[a] = nm[a]; }
    C.px.swap(keep);
    D.px.swap(moved);
    if (new_index == K - 1) break;
    double nv[3], ov[3];
    for (int a = 0; a < 3; ++a) nv[a] = nvq[a] / nw - nm[a] * nm[a];   // :836-838
    for (int a = 0; a < 3; ++a) {
      const double dn = nm[a] - tm[a], dox = om[a] - tm[a];
      ov[a] = ((tw * tv[a] - nw * (nv[a] + dn * dn)) / ow) - dox * dox;
    }
    for (int a = 0; a < 3; ++a) { C.var[a] = ov[a]; D.var[a] = nv[a]; }
    C.weight = ow;
    D.weight = nw;
    C.tse = ow * (ov[0] + ov[1] + ov[2]);
    D.tse = nw * (nv[0] + nv[1] + nv[2]);
    double best = DBL_MIN;
    for (int ic = 0; ic <= new_index; ++ic)
      if (best < cl[ic].tse) { best = cl[ic].tse; old_index = ic; }
  }
  int out = 0;
  for (int ic = 0; ic < K; ++ic) {
    if (means_out)
      for (int a = 0; a < 3; ++a) means_out[3 * ic + a] = cl[ic].mean[a];
    if (sizes_out) sizes_out[ic] = cl[ic].size;
    if (cl[ic].size > 0) {
      const uint32_t sh = (uint32_t)(8 - num_bits);
      const uint32_t R = (uint32_t)(uint8_t)(cl[ic].mean[0] + 0.5) << sh;
      const uint32_t G = (uint32_t)(uint8_t)(cl[ic].mean[1] + 0.5) << sh;
      const uint32_t B = (uint32_t)(uint8_t)(cl[ic].mean[2] + 0.5) << sh;
      ct[out++] = (R << 16) | (G << 8) | B;
    }
  }
  *k_inout = (uint32_t)out;
  return K - out;
}

// cut_bits restated (DivQuantUni.cpp:28-100): each channel shifted right by
// 8 - num_bits (the whole-word form at :63-77 gives the same words).
void dqo_cut_bits(const uint32_t* in, uint32_t n, uint32_t* out, int nbr, int nbg, int nbb) {
  const uint32_t sr = 8 - nbr, sg = 8 - nbg, sb = 8 - nbb;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t p = in[i];
    out[i] = ((((p >> 16) & 0xFF) >> sr) << 16) | ((((p >> 8) & 0xFF) >> sg) << 8) | ((p & 0xFF) >> sb);
  }
}

// calc_color_table with decimation (DivQuantMapColors.cpp:82-203): the points
// visited are in[ic + ir*numRows] for ir = 0, dec, .. < numRows (outer) and ic
// = 0, dec, .. < numCols (inner) -- the reference's numRows stride (:124) kept
// -- and norm = 1 / (ceil(numRows/dec) * ceil(numCols/dec)) (:184).  Returns
// the number of colours, or -1 if an index reaches n (the reference reads past
// its buffer there).
int dqo_color_table_dec(uint32_t n, const uint32_t* in, uint32_t rows, uint32_t cols, int dec,
                        uint32_t* colours, double* weights) {
  if (dec <= 0) return -1;
  std::vector<uint32_t> seq;
  for (uint64_t ir = 0; ir < rows; ir += (uint64_t)dec)
    for (uint64_t ic = 0; ic < cols; ic += (uint64_t)dec) {
      const uint64_t i = ic + ir * rows;
      if (i >= n) return -1;
      seq.push_back(in[i]);
    }
  const double norm = 1.0 / (std::ceil(rows / (double)dec) * std::ceil(cols / (double)dec));
  return color_table_norm((uint32_t)seq.size(), seq.data(), colours, weights, norm);
}

// quant_varpart_fast restated (DivQuantCluster.cpp:1099-1179) for every
// (num_bits, dec_factor, allPixelsUnique): the uniform-weight path when
// allPixelsUnique && num_bits == 8 && dec == 1, else cut_bits (num_bits < 8,
// or the uniform flag with decimation) + calc_color_table(dec) + the
// weighted clustering with final centres shifted by 8 - num_bits.
// Returns the number of empty clusters, or < 0.
int dqo_quant_varpart(uint32_t n, const uint32_t* in, uint32_t rows, uint32_t cols, uint32_t* k_inout,
                      uint32_t* ct, int num_bits, int dec, int max_iters, int uniq, double* means_out,
                      int64_t* sizes_out, int64_t* trace_out) {
  if (num_bits < 1 || num_bits > 8) return -2;
  if (uniq && num_bits == 8 && dec == 1)
    return dqo_cluster(n, in, k_inout, ct, max_iters, means_out, sizes_out, trace_out);
  std::vector<uint32_t> cut(in, in + n);
  if (!(!uniq && num_bits == 8)) dqo_cut_bits(in, n, cut.data(), num_bits, num_bits, num_bits);
  std::vector<uint32_t> colours(n);
  std::vector<double> w(n);
  const int u = dqo_color_table_dec(n, cut.data(), rows, cols, dec, colours.data(), w.data());
  if (u <= 0) return -3;
  return cluster_weighted_bits((uint32_t)u, colours.data(), w.data(), k_inout, ct, max_iters, means_out,
                               sizes_out, trace_out, num_bits);
}

// quant_recurse(..., allPixelsUnique = 0): table, weighted clustering, dedup, map.
int dqo_quant_recurse_weighted(uint32_t n, const uint32_t* in, uint32_t* out, uint32_t* k_inout,
                               uint32_t* ct) {
  std::vector<uint32_t> colours(n);
  std::vector<double> w(n);
  const int u = dqo_color_table(n, in, colours.data(), w.data());
  int empty = dqo_cluster_weighted((uint32_t)u, colours.data(), w.data(), k_inout, ct, 10, nullptr,
                                   nullptr, nullptr);
  if (empty < 0) return empty;
  std::unordered_set<uint32_t> seen;
  uint32_t m = 0;
  for (uint32_t i = 0; i < *k_inout; ++i)
    if (seen.insert(ct[i]).second) ct[m++] = ct[i];
  *k_inout = m;
  dqo_map(in, n, out, ct, (int)m);
  return empty;
}

// getSubdividedColors restated (superpixels/OpenCVUtil.cpp:853-897): the 5^3
// cube {0,63,127,191,255}, R outermost, B innermost, alpha 0xFF.
void dqo_subdivided_colors(uint32_t* out125) {
  static const uint32_t v[5] = {0, 63, 127, 191, 255};
  int i = 0;
  for (int r = 0; r < 5; ++r)
    for (int g = 0; g < 5; ++g)
      for (int b = 0; b < 5; ++b)
        out125[i++] = 0xFF000000u | (v[r] << 16) | (v[g] << 8) | v[b];
}

// genHistogramsForBlocks' block loop restated (ClusteringSegmentation.cpp:
// 420-563) over an already mapped frame `quant` (W*H, 0x00RRGGBB): per block
// of dim x dim pixels (clipped at the right/bottom edge, row-major inside the
// block) a std::unordered_map<uint32_t,uint32_t> histogram, filled in pixel
// order, then the FIRST entry in the map's iteration order with the largest
// count wins (strict '>' from maxCount 0).  The same container type is used on
// purpose: the tie-break is its (libstdc++) iteration order.  keys/counts
// (optional, [nblocks*dim*dim]) receive the table in iteration order,
// ndistinct (optional) its size.
void dqo_block_hist(const uint32_t* quant, uint32_t width, uint32_t height,
                    uint32_t block_w, uint32_t block_h, uint32_t dim, uint32_t* mode,
                    uint32_t* ndistinct, uint32_t* keys, uint32_t* counts) {
  const uint32_t cap = dim * dim;
  for (uint32_t by = 0; by < block_h; ++by)
    for (uint32_t bx = 0; bx < block_w; ++bx) {
      const uint64_t b = (uint64_t)by * block_w + bx;
      std::vector<uint32_t> px;
      for (uint32_t y = by * dim; y < by * dim + dim; ++y)
        for (uint32_t x = bx * dim; x < bx * dim + dim; ++x)
          if (x < width && y < height) px.push_back(quant[(size_t)y * width + x]);
      std::unordered_map<uint32_t, uint32_t> table;
      bool same = true;
      for (uint32_t p : px) same = same && p == px[0];
      if (same) {
        table[px[0]] = (uint32_t)px.size();  // the reference's all-same shortcut (:509-520)
      } else {
        for (uint32_t p : px) table[p] += 1;
      }
      uint32_t best = 0, best_n = 0, i = 0;
      for (const auto& kv : table) {
        if (kv.second > best_n) {
          best_n = kv.second;
          best = kv.first;
        }
        if (keys) keys[b * cap + i] = kv.first;
        if (counts) counts[b * cap + i] = kv.second;
        ++i;
      }
      if (same) best = px[0];
      mode[b] = best;
      if (ndistinct) ndistinct[b] = i;
    }
}

// ---- BGR24 <-> packed frames ----------------------------
// Vec3BToUID (superpixels/OpenCVUtil.h:19-27) over a CV_8UC3 frame, row by
// row as the loop at ClusteringSegmentation.cpp:381-395 visits it.
void dqo_pack_bgr24(const uint8_t* bgr, uint32_t width, uint32_t height, uint32_t stride,
                    uint32_t* out) {
  for (uint32_t y = 0; y < height; ++y)
    for (uint32_t x = 0; x < width; ++x) {
      const uint8_t* v = bgr + (size_t)y * stride + 3u * x;   // v[0]=B v[1]=G v[2]=R
      out[(size_t)y * width + x] = ((uint32_t)v[2] << 16) | ((uint32_t)v[1] << 8) | (uint32_t)v[0];
    }
}

// PixelToVec3b (OpenCVUtil.h:53-59): B = bits 0-7, G = 8-15, R = 16-23.
void dqo_unpack_bgr24(const uint32_t* in, uint32_t width, uint32_t height, uint32_t stride,
                      uint8_t* bgr) {
  for (uint32_t y = 0; y < height; ++y)
    for (uint32_t x = 0; x < width; ++x) {
      const uint32_t p = in[(size_t)y * width + x];
      uint8_t* v = bgr + (size_t)y * stride + 3u * x;
      v[0] = (uint8_t)(p & 0xFF);
      v[1] = (uint8_t)((p >> 8) & 0xFF);
      v[2] = (uint8_t)((p >> 16) & 0xFF);
    }
}

// Region gather (ClusteringSegmentation.cpp:1795-1800): Coord {uint16 x, y}
// (superpixels/Coord.h:30-33) as one word x | y << 16.
void dqo_gather_bgr24(const uint8_t* bgr, uint32_t stride, const uint32_t* coords, uint32_t n,
                      uint32_t* out) {
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t cx = coords[i] & 0xFFFFu, cy = coords[i] >> 16;
    const uint8_t* v = bgr + (size_t)cy * stride + 3u * cx;
    out[i] = ((uint32_t)v[2] << 16) | ((uint32_t)v[1] << 8) | (uint32_t)v[0];
  }
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Fixture helpers shared by tests/ and bench.py (test infrastructure too).
// SURVEY 8c generator: xorshift64 (s^=s<<13; s^=s>>7; s^=s<<17), one draw per
// pixel in row-major order, pixel = draw & 0xFFFFFF.
extern "C" void dqo_xorshift_fill(uint32_t* out, uint64_t n, uint64_t seed) {
  uint64_t s = seed;
  for (uint64_t i = 0; i < n; ++i) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    out[i] = (uint32_t)(s & 0xFFFFFF);
  }
}

// SURVEY 8c hash: word-wise FNV-1a-64 over uint32 words.
extern "C" uint64_t dqo_fnv1a64(const uint32_t* w, uint64_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint64_t i = 0; i < n; ++i) {
    h ^= w[i];
    h *= 0x100000001b3ull;
  }
  return h;
}
