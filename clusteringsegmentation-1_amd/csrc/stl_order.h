// =============================================================================
// stl_order.h -- iteration order of a std::unordered_map<uint32_t, V>.
//
// genHistogramsForBlocks (ClusteringSegmentation.cpp:476-551) picks a block's
// colour as the FIRST entry, in the histogram's iteration order, whose count is
// the largest.  Ties are common (a 4x4 block split 8/8), so that order is part
// of the result.  The histogram is a std::unordered_map<uint32_t,uint32_t>
// filled by `table[p] += 1` in pixel order; on the reference's toolchain here
// (g++ 11 / libstdc++) this is:
//   * std::hash<uint32_t> is the identity, bucket = key % bucket_count;
//   * bucket counts 1 -> 13 (1st insert) -> 29 (14th) -> 59 (30th) -> 127 (60th)
//     -> 257 (128th) (max load factor 1; measured, tests/native/);
//   * a key whose bucket is empty is linked at the FRONT of the node list, a
//     key whose bucket is occupied right BEFORE that bucket's first node;
//   * a rehash re-links the nodes in list order by the same two rules.
// Hence for an insertion sequence S and bucket count B the list is: buckets
// ordered by their first appearance in S, latest first; inside a bucket, keys
// ordered by position in S, latest first.  A rehash restarts S as (current
// list order) ++ (later keys).  stl_rank() evaluates that closed form with
// O(d^2) compares and no data-dependent indexing (registers only when N is a
// compile-time size and the loops unroll).
//
// Pinned against the real container by tests/test_block_hist.py
// (tests/native/stl_order_check.cpp, random key sequences, d = 1..300).
// =============================================================================
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define DQ_HD __host__ __device__
#else
#define DQ_HD
#endif

namespace dq {

// Bucket count of level L (L rehashes done) for the libstdc++ prime policy
// (growth factor 2, next prime above); level L holds up to that many keys.
template <int L>
struct StlLevel {
  static constexpr uint32_t nb = L == 0 ? 13u : L == 1 ? 29u : L == 2 ? 59u : L == 3 ? 127u : 257u;
};
constexpr int kStlMaxLevels = 5;  // up to 257 distinct keys

// One level: rank the keys inserted so far (ins < min(d, nb)) by the closed
// form with bucket count nb; returns true when every key is in (done).
template <int N, int L>
DQ_HD inline bool stl_level(const uint32_t* keys, const int* ins, int d, int* seq, int* rank) {
  constexpr uint32_t nb = StlLevel<L>::nb;
  const int lim = d < (int)nb ? d : (int)nb;
  uint32_t bk[N];
  bool mem[N];
  int gf[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    bk[i] = keys[i] % nb;   // constant divisor: multiply-shift
    mem[i] = ins[i] >= 0 && ins[i] < lim;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    int g = seq[i];
#pragma unroll
    for (int j = 0; j < N; ++j)
      g = (mem[j] && bk[j] == bk[i] && seq[j] < g) ? seq[j] : g;
    gf[i] = g;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    int r = 0;
#pragma unroll
    for (int j = 0; j < N; ++j)
      r += (mem[j] && (gf[j] > gf[i] || (gf[j] == gf[i] && seq[j] > seq[i]))) ? 1 : 0;
    rank[i] = r;
  }
  if (lim == d) return true;
  // rehash: the list so far, then the keys not inserted yet (seq = ins there)
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (mem[i]) seq[i] = rank[i];
  return false;
}

// Slot form: slot i holds keys[i]; ins[i] is its insertion index (0..d-1) if
// the slot is a map key, -1 otherwise (d <= N <= 257).  rank[i] (for key
// slots) = its position in the map's iteration order after all d inserts.
// Only the levels N keys can reach are emitted.
template <int N>
DQ_HD inline void stl_rank_slots(const uint32_t* keys, const int* ins, int d, int* rank) {
  static_assert(N <= 257, "more keys than the level table covers");
  int seq[N];
#pragma unroll
  for (int i = 0; i < N; ++i) seq[i] = ins[i];
  if (stl_level<N, 0>(keys, ins, d, seq, rank)) return;
  if constexpr (N > 13) { if (stl_level<N, 1>(keys, ins, d, seq, rank)) return; }
  if constexpr (N > 29) { if (stl_level<N, 2>(keys, ins, d, seq, rank)) return; }
  if constexpr (N > 59) { if (stl_level<N, 3>(keys, ins, d, seq, rank)) return; }
  if constexpr (N > 127) { stl_level<N, 4>(keys, ins, d, seq, rank); }
}

// Compact form: keys[0..d) distinct, in first-insertion order (d <= N).
template <int N>
DQ_HD inline void stl_rank(const uint32_t* keys, int d, int* rank) {
  uint32_t k[N];
  int ins[N];
  for (int i = 0; i < N; ++i) {
    k[i] = i < d ? keys[i] : 0u;
    ins[i] = i < d ? i : -1;
  }
  stl_rank_slots<N>(k, ins, d, rank);
}

}  // namespace dq
