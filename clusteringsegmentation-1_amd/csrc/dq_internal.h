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
//   tile            -- the part of a segment one workgroup sweeps in a pass.
#pragma once
#include <stdint.h>

namespace dq {

// Pixel buffers a segment can live in.  The root lives in the caller's input;
// children of a node in buffer b are written to the "other" working buffer.
enum BufId : int32_t { BUF_IN = 0, BUF_P0 = 1, BUF_P1 = 2 };
inline int child_buf(int b) { return b == BUF_P0 ? BUF_P1 : BUF_P0; }

// Pass kinds (kernel template parameter).
enum PassKind : int32_t {
  PASS_INIT = 0,     // root only: count, sums and sums of squares (:49-104)
  PASS_SPLIT = 1,    // cut_pos < v_axis -> new (:438-559)
  PASS_KMEANS = 2,   // lhs < rr*R + rg*G + rb*B -> old (:683), new-side sums
  PASS_KLAST = 3,    // last 2-means iteration: also sums of squares (:726-748)
};

// Per-node state for one round.  All FP64 fields follow the reference's
// variable of the same role; the device epilogue updates them between passes.
struct alignas(16) DevNode {
  // --- set by the host when the round starts
  uint32_t off, len;        // segment of this node's points
  int32_t buf;              // BufId the points live in
  int32_t tile_begin;       // this node's tiles are [tile_begin, tile_end)
  int32_t tile_end;
  int32_t axis;             // split pass: cut axis (0=R,1=G,2=B) (:388-403)
  double cut;               // split pass: cut position
  double tw;                // total_weight = weight[old_index]  (:353)
  double tm[3], tv[3];      // total_mean / total_var           (:357-374)
  // --- current 2-means decision parameters (written by the epilogues)
  double lhs, rr, rg, rb;   // (:616-623)
  double om[3], nm[3];      // old_mean / new_mean
  // --- decision of the LAST 2-means pass (kept for the partition sweep)
  double plhs, prr, prg, prb;
  // --- results of the node's split (read back by the host)
  uint64_t n_new;           // new_size (:820-821)
  double nw, ow;            // new_weight / old_weight
  double nv[3], ov[3];      // new_var / old_var (:836-855)
  double tse_old, tse_new;  // (:870-871)
};

// One workgroup's share of a pass.
struct alignas(16) Tile {
  int32_t node;             // index into the round's DevNode array
  uint32_t start, end;      // absolute pixel range in the node's buffer
  uint32_t old_base;        // partition: rank of this tile's first old point
};

// Per-tile partial statistics of the new side (or of all points in PASS_INIT).
struct alignas(16) TilePartial {
  uint64_t cnt;
  uint64_t s[3];            // sum R, G, B
  uint64_t q[3];            // sum R^2, G^2, B^2 (PASS_INIT / PASS_KLAST)
  uint64_t pad;
};

}  // namespace dq
