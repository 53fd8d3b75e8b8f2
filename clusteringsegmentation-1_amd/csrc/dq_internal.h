// dq_internal.h -- structures shared by the host engine (dq_engine.cpp) and the
// gfx950 kernels (dq_kernels.hip).  Not part of the public ABI (see include/).
//
// Vocabulary follows the reference (DivQuant/DivQuantCluster.cpp):
//   cluster / node  -- a set of points that DivQuantCluster splits in two:
//                      the "old" half keeps the parent's cluster index, the
//                      "new" half gets new_index (:346, :410, :595);
//   pass            -- one sweep over the points of every node being split:
//                      the split pass (:438-559) or one local 2-means
//                      iteration (:613-811);
//   segment         -- the contiguous range [off, off+len) of a working pixel
//                      buffer that holds one node's points;
//   tile            -- the part of a segment one workgroup sweeps in a pass;
//   frame           -- one quant_recurse input; a round may mix frames.
#pragma once
#include <stdint.h>

namespace dq {

// Pass kinds (kernel template parameter).
enum PassKind : int32_t {
  PASS_INIT = 0,     // root only: count, sums and sums of squares (:49-104)
  PASS_SPLIT = 1,    // cut_pos < v_axis -> new (:438-559)
  PASS_KMEANS = 2,   // lhs < rr*R + rg*G + rb*B -> old (:683), new-side sums
  PASS_KLAST = 3,    // last 2-means iteration: also sums of squares (:726-748)
};

// Per-tile partial statistics of the new side (all points in PASS_INIT):
// count, sums and sums of squares in every pass; plain 32-B stores, exact in
// u32 because a tile has at most 65536 points (65536 * 255^2 < 2^32).  The
// node's epilogue sums them in u64.
enum PartField : int32_t { F_CNT = 0, F_SR, F_SG, F_SB, F_QR, F_QG, F_QB, F_NUM };
struct alignas(32) TilePartial {
  uint32_t f[8];
};

// Decision parameters of one pass for one node (:616-623, :683).
struct alignas(16) Params {
  double lhs, rr, rg, rb;          // exact FP64 decision
  float lhsf, rrf, rgf, rbf, eps;  // FP32 pre-filter (dq_kernels.hip, stays_old)
  int32_t thr, shift;              // split pass: new iff ((p >> shift) & 0xFF) >= thr
  int32_t pad;
};

// Per-node state for one round.
struct alignas(16) DevNode {
  // --- set by the host when the round starts
  const uint32_t* src;      // element 0 of the frame in the buffer holding the node
  uint32_t* dst;            // element 0 of the frame in the child buffer
  uint32_t off, len;        // segment, relative to src / dst
  int32_t tile_begin;       // this node's tiles are [tile_begin, tile_end)
  int32_t tile_end;
  double s;                 // data_weight of the frame (get_double_scale)
  double tw;                // total_weight = weight[old_index]  (:353)
  double tm[3], tv[3];      // total_mean / total_var (root: written by PASS_INIT)
  // --- parameters of the next pass (host for the split pass of non-roots,
  //     otherwise written by the node's epilogue)
  Params prm;
  // --- results of the node's split (written by the PASS_KLAST epilogue, or
  //     by the PASS_KMEANS epilogue that finds the 2-means at a fixed point;
  //     prm then still holds the last 2-means decision)
  double om[3], nm[3];      // old_mean / new_mean after the last pass
  double nv[3], ov[3];      // new_var / old_var (:836-855)
  double nw, ow;            // new_weight / old_weight
  double tse_old, tse_new;  // (:870-871)
  uint64_t n_new;           // new_size (:820-821)
  // --- fixed-point detection.  The 2-means state after a pass is the new
  //     side's exact integer (count, sums): when a pass reproduces the
  //     previous pass's, every later iteration is bit-identical (same sums ->
  //     same means -> same decision), so the results are final and the
  //     remaining passes skip the node.
  uint64_t prev[4];         // count, sum R, G, B of the previous pass
  int32_t iter;             // 2-means iterations completed (epilogue count)
  int32_t done_it;          // 0: active; else 1 + the iteration found at the fixed point
};

// One workgroup's share of a pass.
struct alignas(16) Tile {
  int32_t node;             // index into the round's DevNode array
  uint32_t start, end;      // pixel range relative to the node's src
  uint32_t old_base;        // partition: old points in the node's earlier tiles
};

}  // namespace dq
