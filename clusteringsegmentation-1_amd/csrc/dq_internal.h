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
//   frame           -- one quant_recurse input; a round may mix frames;
//   shard           -- (row-tile mode) the rows of a frame one GPU holds; every
//                      count/sum below is then LOCAL to the shard unless it is
//                      called global (the allreduced value).
#pragma once
#include <stdint.h>

namespace dq {

// Row-range shards a frame may be split into inside ONE process (virtual
// shards on one GPU: the exact arithmetic of multi-GPU row sharding).
constexpr int kMaxShard = 8;

// Pass kinds (kernel template parameter).
enum PassKind : int32_t {
  PASS_INIT = 0,     // root only: count, sums and sums of squares (:49-104)
  PASS_SPLIT = 1,    // cut_pos < v_axis -> new (:438-559)
  PASS_KMEANS = 2,   // lhs < rr*R + rg*G + rb*B -> old (:683), new-side sums
  PASS_KLAST = 3,    // last 2-means iteration: also sums of squares (:726-748)
};

// Per-tile partial statistics of the new side (all points in PASS_INIT):
// count, sums and sums of squares; plain 32-B stores, exact in u32 because a
// tile has at most 65536 points (65536 * 255^2 < 2^32).  The node's epilogue
// sums them in u64.
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

// Per-node state.  One record per node per round it is split in; the records
// of earlier rounds stay valid for the whole run (a later round partitions a
// node through its record and tiles, see PartTile).
// DevNode::planar: how a node's points are stored at src.
enum SrcFormat : int32_t {
  SRC_PACKED = 0,   // the caller's u32 0x00RRGGBB frame (4 B per point)
  SRC_PLANAR = 1,   // byte planes R, G, B of P0 / P1 (3 B per point)
  SRC_BGR24 = 2,    // the caller's BGR24 frame (OpenCV CV_8UC3 rows, 3 B per point)
};

struct alignas(16) DevNode {
  // --- set by the host when the round starts
  const uint8_t* src;       // the frame (shard) in the buffer holding the node: element 0 of
                            //   the caller's packed u32 frame, or byte 0 of its R plane in
                            //   P0 / P1 (planar: G, B at + RoundArgs::plane, + 2 plane)
  uint8_t* dst;             // byte 0 of the frame (shard)'s R plane in the child buffer
  uint32_t off, len;        // local segment, relative to src / dst
  int32_t tile_begin;       // this node's tiles are [tile_begin, tile_end) of the round
  int32_t tile_end;
  int32_t split_pb, split_pe;   // fused split: the parent's PartTiles [pb, pe) of the round
  int32_t split_side;           //   0: this node is the parent's old half, 1: the new half
                                //   (split_pb < 0: the node has its own split pass)
  int32_t planar;               // source format of src (SrcFormat): the caller's packed
                                //   frame, the byte planes of P0 / P1, or a BGR24 frame
  double s;                 // data_weight of the frame (get_double_scale)
  double tw;                // total_weight = weight[old_index]  (:353)
  double tm[3], tv[3];      // total_mean / total_var (root: written by PASS_INIT)
  // --- parameters of the next pass (host for the split pass of non-roots,
  //     otherwise written by the node's epilogue); after the split is final
  //     prm holds the 2-means decision that produced the final halves.
  Params prm;
  // --- fixed-point detection.  The 2-means state after a pass is the new
  //     side's exact integer (count, sums): when a pass reproduces the
  //     previous pass's, every later iteration is bit-identical (same sums ->
  //     same means -> same decision), so the results are final and the
  //     remaining passes skip the node.
  uint64_t prev[4];         // count, sum R, G, B of the previous pass (global)
  uint32_t n_new_local;     // final new-half size in this shard (partition)
  int32_t iter;             // 2-means iterations completed (epilogue count)
  int32_t done_it;          // 0: active; else 1 + the iteration found at the fixed point
  uint32_t tile_len;        // this record's tiles: [off + k*tile_len, ...) (last one shorter)
  int32_t proven;           // set by the split epilogue: the final halves are the cut's
                            //   (a later partition replays the cut, prm.thr / prm.shift)
  int32_t pad2[3];
  // --- a box holding every point of the node (channel c: R, G, B), from the
  //     host: the root's is the cube, a child's is its parent's, clipped at
  //     the parent's cut when the parent's halves are proven to be the cut's
  //     (split epilogue, cut_is_fixed_point)
  int32_t box_lo[3], box_hi[3];
};

// The split's results, written by the finalising epilogue straight into
// host-coherent pinned memory (the host reads them without a copy).
struct alignas(16) NodeResult {
  double om[3], nm[3];      // old_mean / new_mean after the last pass
  double nv[3], ov[3];      // new_var / old_var (:836-855)
  double tm[3], tv[3];      // the node's own mean / var (root: from PASS_INIT)
  double nw, ow;            // new_weight / old_weight
  double tse_old, tse_new;  // (:870-871)
  uint64_t n_new;           // new_size (:820-821), global
  uint32_t n_new_local;     // new half in this shard
  int32_t done_it;          // see DevNode
  int32_t proven;           // 1: final at the split epilogue -- the halves are the cut's
  int32_t pad;
  uint32_t len_local;       // the record's points (the host checks its mirror of the layout)
  uint32_t tag;             // round sequence number, stored LAST (after the other words
                            //   completed): the host reads a record only once it matches
};

// One workgroup's share of a pass.  Inside a tile, wave w of the workgroup
// owns a contiguous range of it (dq_kernels.hip, wave_range: the same in
// every kernel), so the final pass's per-wave counts let each wave of the
// partition write its points with no block-level synchronisation.
constexpr int kTileWaves = 4;
struct alignas(16) Tile {
  int32_t node;             // index into the round's DevNode array
  uint32_t start, end;      // pixel range relative to the node's src
  uint32_t pad;
  // partition cursors of each wave (set by the finalising epilogue):
  uint32_t old_base[kTileWaves];   // OLD points of the node before this wave's share
  uint32_t new_base[kTileWaves];   // NEW points of the node before this wave's share
};

// One workgroup's share of a fused partition + split pass: a tile of a
// parent node split in an EARLIER round.  Its points are written to the two
// children's segments (replaying the parent's final decision) and each
// child's split-pass statistics (:438-559) are accumulated on the way.
// Besides the children's split sums (count, sums, sums of squares of each
// child's new side: 2 x TilePartial per PartTile) it adds each child's
// per-(tile, wave) counts of its split-pass halves into Tile-wave words of
// RoundArgs::wparts (old | new << 16, zeroed for the round): the partition
// cursors of a child whose split turns out final at its split epilogue.
struct alignas(32) PartTile {
  const Tile* tile;         // the parent's tile (cursors final)
  const DevNode* parent;    // the parent's record
  int32_t thr[2];           // children's split thresholds (256: child not split this round)
  int32_t shift[2];
  int32_t child[2];         // the children's records in this round (-1: not split in it)
};

// Per-launch completion counters of the round's 2-means epilogues (device
// memory, zeroed with the round's tables).  Each word: low 32 bits =
// arrivals, high 32 = records not final.  Workgroup b arrives on shard
// b % kArrShards (one atomic per workgroup on one address serialises at
// ~13 ns: 1024 workgroups cost ~13 us); a shard's last arriver forwards the
// shard's active count to `top`, whose last arriver publishes the status.
constexpr int kArrShards = 16;
struct alignas(64) ArrWord {
  uint64_t word;
  uint64_t pad[7];
};
struct alignas(64) LaunchCtr {
  ArrWord shard[kArrShards];
  ArrWord top;
};

// The last-arriving epilogue workgroup of 2-means iteration `it` publishes
// the status word (round sequence << 32) | (active nodes << 1) | 1 to host
// memory (RoundArgs::hstat[it]).

}  // namespace dq
