// dq_kernels.h -- host-callable launchers for the gfx950 kernels in
// dq_kernels.hip.  Every launcher only enqueues work on `stream`; none of
// them allocates, copies or synchronises (so a caller may capture them in a
// hipGraph).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dq_internal.h"

namespace dq {

constexpr int kBlock = 64 * kTileWaves;          // 4 wave64 per workgroup
constexpr int kVecPerThread = 4;                // uint4 loads per lane per sweep
constexpr int kSweep = kBlock * kVecPerThread * 4;   // 4096 points: tile lengths are multiples
constexpr int kWaveSweep = 64 * kVecPerThread * 4;   // 1024 points: one wave's sweep
constexpr uint32_t kMaxTilePx = 16 * kSweep;    // keeps packed 16-bit lane sums exact

// Map (nearest palette entry) cell grid: 32 cells of 8 values per channel.
constexpr int kCellBits = 5;
constexpr int kCells = 1 << (3 * kCellBits);
constexpr int kCellInline = 7;                  // candidates stored in the record
constexpr int kCellRecWords = 4;                // 16-B record per cell
constexpr int kCellCap = 32;                    // candidates in the overflow list
constexpr uint32_t kCellBrute = 0xFFFF;         // count marker: scan the whole palette

// The source format of every parent of a partition launch (launch_partsplit,
// launch_plansplit), or FMT_ANY (mixed: each record's own, in a kernel
// compiled for all of them).
enum SrcFmt : int { FMT_PLANAR = 0, FMT_BGR = 1, FMT_PACKED = 2, FMT_ANY = 3 };

// What a plan reads of each record of the round it is planned from, written
// by whichever kernel finalises the record (store_result), 32 B contiguous
// per record: the plan's scan over every parent's (shard) records reads these
// instead of fields spread over 272-B DevNodes (with 8 shard records per
// parent the scattered loads were most of a sharded plan's time).  Zero
// (final = 0) until the record is final: the round arena is zero on entry.
struct alignas(16) RecSummary {
  uint32_t off, len, n_new_local, ntiles;   // local segment, final new half, the record's tiles
  int32_t tile_begin;
  uint32_t final;                           // 1 once the record's split is final
  uint32_t pad[2];
};

// Tables of one round (device pointers unless noted).
struct RoundArgs {
  Tile* tiles;              // the round's tiles (kept: a later round partitions through them)
  DevNode* nodes;           // the round's node records (kept, as tiles)
  TilePartial* parts;       // one per tile, rewritten by every pass
  TilePartial* parts2;      // one per tile: kpersist_kernel's odd iterations (its
                            //   workgroups read a whole record's partials while others
                            //   already write the next iteration's)
  uint32_t* wparts;         // per (tile, wave): old | new << 16 of the last pass (the
                            //   split pass's: own split pass, or added up by partsplit)
  const PartTile* ptiles;   // fused partition + split work of this round
  TilePartial* sparts;      // two per PartTile (old child, new child)
  NodeResult* hres;         // host-coherent pinned: final results per node
  LaunchCtr* ctr;           // per 2-means iteration, then one for the split epilogue
  uint64_t* hstat;          // host-coherent pinned: status word per 2-means iteration,
                            //   then the split epilogue's (index max_iters)
  uint64_t seq;             // round sequence number (tags the status words)
  int32_t fixed_point;      // epilogues finalise nodes at a 2-means fixed point
  int32_t it;               // 2-means iteration of an epilogue launch (split: max_iters)
  int32_t nn;               // node records in the round (logical nodes x shards)
  // sharded rounds (a frame split into row ranges, one record per shard):
  uint64_t* tot;            // per logical node: 8 u64 totals (nodesum, then allreduce)
  int32_t nshard;           // records per logical node (record r = node * nshard + shard)
  int32_t debug;            // kDebug* flags (tests only: forced interleavings, 0 in production)
  uint32_t* rdone;          // per (2-means iteration, record): kpass workgroups finished
  NodeResult* dres;         // device copy of the final results (read by the next round's plan)
  const uint32_t* counts;   // planned rounds: [tiles, part tiles, aborted] written by
                            //   plan_kernel (grids are upper bounds); nullptr: host-built
  uint64_t plane;           // bytes between the R, G and B planes of P0 / P1
  int32_t tot_mode;         // where a record's pass totals come from (TotMode)
  int32_t ps_mode;          // what partsplit_kernel does (PsMode)
  RecSummary* rsum;         // per record, written with its final results (the next plan's scan)
  uint32_t* sdone;          // TOT_ALLREDUCE, one shard: per parent (at its first listed
                            //   child's record index), its partition workgroups finished --
                            //   the last writes the children's split totals to tot (no
                            //   nodesum_kernel); nullptr otherwise
};

// partsplit_kernel's work (RoundArgs::ps_mode):
//   PS_FULL  -- the parents' points into the children's segments, the
//               children's split-pass sums and per-(tile, wave) counts;
//   PS_STATS -- the children's split-pass sums only, nothing written (a
//               frame's last round: its nodes' children are leaves, and a
//               node's own points are needed only for its 2-means passes);
//   PS_LATE  -- after PS_STATS and the split epilogue: the points of every
//               parent with a child still active (not proven at its split),
//               for the children's 2-means passes; nothing else;
//   PS_WRITE -- the points of the listed parents only (a later round needs
//               the segments of nodes a PS_STATS round left unwritten).
enum PsMode : int32_t { PS_FULL = 0, PS_STATS = 1, PS_LATE = 2, PS_WRITE = 3 };

// How the FP64 update of a pass gets the node's totals (RoundArgs::tot_mode):
// the record's own tile partials (one shard, no communicator); the partials
// of every shard record of the logical node (virtual row shards in this
// process); or RoundArgs::tot, the logical node's totals of this process
// allreduced across processes (RCCL) before the epilogue.
enum TotMode : int32_t { TOT_OWN = 0, TOT_NODE = 1, TOT_ALLREDUCE = 2 };

// A round planned on the device (plan_kernel): the children of every listed
// record of the previous round are this round's nodes, record 2i = the old
// half of parent plist[i], 2i+1 = its new half ("device-planned
// rounds").  The host enqueues the round before the previous round's results
// exist; the plan aborts the round (counts[2] = 1, every kernel of it exits)
// when a listed parent is not final after its split epilogue.
struct PlanArgs {
  const DevNode* pn;        // previous round: records
  const RecSummary* psum;   //                 their summaries (the scans)
  const NodeResult* pres;   //                 results (device copy)
  const Tile* ptiles;       //                 tiles (the part tiles point into them)
  const int32_t* plist;     // parent (logical) nodes to split (host-coherent pinned memory)
  int32_t np;
  int32_t node_tiles;       // tiles per record at least (Engine::tile_len)
  uint32_t tl;              // tile length of the round (Engine::tile_len)
  uint32_t tiles_cap, ptiles_cap;
  DevNode* cn;              // this round: 2 np records
  Tile* ct;
  PartTile* cpt;
  uint32_t* counts;         // device: tiles, part tiles, aborted (1: a listed parent not
                            //   final, 2: overflow, 3: cancelled -- see `cancel`)
  uint32_t* hcounts;        // host-coherent mirror of counts
  const uint32_t* cancel;   // a re-plan (Engine::finish_round): the counts of the first
                            //   plan of the same round; it cancels itself if that one ran
  const uint8_t* p0;        // the two working buffers (a child's dst is the
  const uint8_t* p1;        //   other one of its src)
  uint64_t cap_bytes;       // bytes per working buffer
  int32_t debug;            // kDebug* flags
  int32_t nshard;           // records per logical node (record = node * nshard + shard)
};
constexpr int kPlanMaxParents = 6144;   // parents per planned round (LDS scans)

// Test-only interleaving knobs (dq_hip_set_debug): each forces a timing or
// cache state the production path must tolerate, with identical outputs.
//   kDebugPrewarm:   every 2-means workgroup loads its record's tile partials
//                    and per-wave counts (into its L1 and its XCD's L2)
//                    before storing its own, so a last arriver that skipped
//                    the agent-scope acquire would read stale lines;
//   kDebugUneven:    1 in 8 workgroups of every 2-means pass and partition
//                    stalls ~10 us before publishing (uneven arrival order);
//   kDebugHostDelay: the host sleeps 200 us between a round's status word and
//                    reading its results, and before enqueueing a round (the
//                    GPU runs ahead into the other parity slot);
//   kDebugPlanStall: the plan kernel's first workgroup stalls ~20 us before
//                    publishing the plan's counts.
//   kDebugArenaCheck: every run first checks on the host that the round
//                    arena is all zero (the planned rounds' invariant) and
//                    aborts naming the first non-zero byte.
//   kDebugFreshArena: every run first releases the round arena, so its
//                    rounds allocate (and clear) new chunks while the other
//                    lanes' runs are in flight -- the order in which a
//                    null-stream clear once raced the round's kernels.
constexpr int32_t kDebugPrewarm = 1, kDebugUneven = 2, kDebugHostDelay = 4, kDebugPlanStall = 8,
                  kDebugArenaCheck = 16, kDebugFreshArena = 32;
// plan_kernel: the planned round's tables.  Like plansplit below, it relies on
// the round block's [LaunchCtr | wparts | rdone | summaries] being zero on
// entry (the round arena's invariant, Engine::run).
void launch_plan(const PlanArgs& a, hipStream_t stream);
// plan_kernel's work and the planned round's partition (PS_FULL / PS_STATS)
// in one launch of `grid` (= the part tiles' upper bound) workgroups; one
// shard per node only.  The round block's [LaunchCtr | wparts | rdone |
// summaries] must already be zero.
void launch_plansplit(const PlanArgs& pa, const RoundArgs& a, int grid, int fmt, hipStream_t stream);
// Host-built round tables: copy `bytes` from host-coherent pinned staging
// (device view) into the round's device block on the round's stream (no
// copy-engine hop between the host and the round's first kernel).
void launch_upload(void* dst, const void* src_dev_view, size_t bytes, hipStream_t stream);
// Zero `bytes` (a multiple of 16, 16-B aligned) on the stream (hipMemsetAsync
// cost ~20 us of host time at the end of a call).
void launch_zero(void* dst, size_t bytes, hipStream_t stream);
// dst[i] = sum of src.p[r][i] over r < nsrc (u64; the test-only loopback
// collective of Engine, dq_engine.cpp).  dst must not alias a source.
struct SumSrcs { const uint64_t* p[kMaxShard]; };
void launch_sum_u64(const SumSrcs& src, int nsrc, uint64_t* dst, size_t count, hipStream_t stream);

// One statistics pass over tiles [0, ntiles) of the round (one workgroup per tile).
void launch_pass(int kind, const RoundArgs& a, int ntiles, hipStream_t stream);
// A 2-means pass with its epilogue fused (kpass_kernel): the logical node's
// last workgroup runs the FP64 update of every shard record of the node; with
// TOT_ALLREDUCE it only writes the node's totals to a.tot (the allreduce and
// launch_epilogue follow).
void launch_kpass(int kind, const RoundArgs& a, int ntiles, hipStream_t stream);
// The FP64 update after a pass, one workgroup per node record: the node's
// totals per a.tot_mode, the record's own partials for its local counts;
// publishes the next pass's decision (or the split's results).
void launch_epilogue(int kind, const RoundArgs& a, int nnodes, hipStream_t stream);
// The partition cursors of ONE record finalised at a PS_STATS round's split
// (that partition counts no children): its split decision's per-(tile, wave)
// counts over its points (pass_kernel<PASS_SPLIT> on a.tiles[0 .. ntiles),
// into a.wparts), then the cursor scan into its tiles.  a.nodes: its round's
// records (Tile::node indexes them).
void launch_fix_cursors(const RoundArgs& a, int ntiles, hipStream_t stream);
// TOT_ALLREDUCE rounds: per logical node, the sums of the pass over all its
// shard records' tiles into a.tot (to be allreduced across processes).
void launch_nodesum(int kind, const RoundArgs& a, int nlogical, hipStream_t stream);
// All 2-means iterations of the round in one launch, one workgroup per
// record (kloop_kernel): records of one shard (S == 1, TOT_OWN) with planar
// segments of at most kLoopMaxLen points and at most kLoopMaxTiles tiles.
// Every record arrives on the counter of iteration max_iters - 1.
constexpr uint32_t kLoopMaxTiles = 1024;
// A data wave of kloop_kernel sweeps 64 of every 960 16-point chunks: with
// at most 64 chunk rows (61440 chunks, less the 16-B alignment slack of the
// segment's first chunk) it sums at most 65536 points, and 65536 * 255^2 <
// 2^32 keeps its u32 sums of squares exact.
constexpr uint32_t kLoopMaxLen = 61440u * 16u - 32u;
void launch_kloop(const RoundArgs& a, int nrec, int max_iters, hipStream_t stream);
// All 2-means iterations of the round in one launch over its ntiles tiles,
// one workgroup per tile, the records' workgroups meeting per iteration on
// rdone (kpersist_kernel): one shard per record (TOT_OWN), planar records,
// ntiles at most the resident workgroups of the device (Engine::persist_ok).
// Every record arrives on the counter of iteration max_iters - 1.
void launch_kpersist(const RoundArgs& a, int ntiles, int max_iters, hipStream_t stream);
// Fused partition + split pass over the round's PartTiles: writes each
// parent's points into its two children's segments (old half first, then new
// half) of the child buffer, using the parent's final 2-means decision, and
// accumulates the children's split-pass statistics.
void launch_partsplit(const RoundArgs& a, int nptiles, int fmt, hipStream_t stream);

// One map_colors_mps job of a batched map launch (device-resident table).
struct alignas(16) MapTask {
  const uint32_t* in;       // n pixels (16-B aligned)
  uint32_t* out;            // n mapped colours (16-B aligned)
  const uint32_t* pal;      // k colours sorted by R+G+B (reference comparator)
  const uint16_t* lut;      // 766 start entries (lut_init)
  uint32_t* cell_rec;       // kCells x 16 B candidate records
  uint16_t* cell_idx;       // kCells x kCellCap overflow lists
  uint32_t* cell_c32;       // kCells compact records (K <= 1024, LDS-resident in the map)
  uint32_t n;
  int32_t k;
  uint32_t block_begin;     // first map workgroup of this task
  uint32_t grp_per_block;   // groups of kMapPx pixels per workgroup
  int32_t bgr;              // in is a BGR24 frame (3 B per pixel, 8-B aligned; map_lds_kernel only)
};

// Map: candidate records per colour cell for every task (one launch), then
// the per-pixel argmin over (squared distance, MPS visit rank) for every
// task (one launch of nblocks workgroups; task t owns workgroups
// [block_begin, block_begin + ceil(n / kMapPx / grp_per_block))).
void launch_build_cells(const MapTask* tasks, int ntasks, int kmax, hipStream_t stream);
uint32_t map_groups_per_block(uint32_t n);
void launch_map(const MapTask* tasks, int ntasks, int kmax, uint32_t nblocks, hipStream_t stream);
// K <= 1024: the same map with the compact cell table staged in LDS (one
// 1024-thread workgroup per CU); map_lds_blocks gives each task's share of
// the grid (block_begin / grp_per_block set by the caller from it).
constexpr int kMapLdsBlock = 1024;
// bgr: every task's input is a BGR24 frame (MapTask::bgr), else every task's is packed.
void launch_map_lds(const MapTask* tasks, int ntasks, int kmax, uint32_t nblocks, bool bgr,
                    hipStream_t stream);

// Block histograms of a mapped frame (genHistogramsForBlocks' block loop,
// ClusteringSegmentation.cpp:420-563).  Blocks of dim x dim pixels, dim 1..4 (the app: 4);
// keys/counts (optional, nblocks * dim^2) get each block's histogram in the
// reference's iteration order.  Requires block_w*dim < width+dim and
// block_h*dim < height+dim (every block holds a pixel).
struct BlockHistArgs {
  const uint32_t* quant;
  uint32_t width, height, block_w, block_h;
  uint32_t* mode;
  uint32_t* ndistinct;
  uint32_t* keys;
  uint32_t* counts;
  uint32_t* work_n;   // block_hist_scratch_words() of device scratch (tie queues)
  uint32_t* work;     // set by launch_block_hist
  uint32_t queue_cap; // set by launch_block_hist
};
// Tie queues: one per (workgroup % kBhQueues), counters 128 B apart.  Measured
// per 4K frame (light + rank kernel, us): 1 queue 61+21 (same-address
// atomics), 8: 15+21, 16: 10+22, 32: 9+93, 64: 10+157 (the ranking kernel
// degrades with many sparse queues; not understood yet).
constexpr uint32_t kBhQueues = 16, kBhQueueStride = 32;
size_t block_hist_scratch_words(uint32_t block_w, uint32_t block_h);
int launch_block_hist(const BlockHistArgs& a, int dim, hipStream_t stream);

// BGR24 (OpenCV CV_8UC3, `stride` bytes per row) <-> packed 0x00RRGGBB
// frames: Vec3BToUID / PixelToVec3b (superpixels/OpenCVUtil.h:19-27, 53-59)
// over a whole frame, and the Coord-list gather of ClusteringSegmentation.cpp:1795-1800.
void launch_bgr24_pack(const uint8_t* bgr, uint32_t width, uint32_t height, uint32_t stride,
                       uint32_t* out, hipStream_t stream);
void launch_bgr24_unpack(const uint32_t* in, uint32_t width, uint32_t height, uint32_t stride,
                         uint8_t* bgr, hipStream_t stream);
void launch_bgr24_gather(const uint8_t* bgr, uint32_t stride, const uint32_t* coords, uint32_t n,
                         uint32_t* out, hipStream_t stream);

}  // namespace dq
