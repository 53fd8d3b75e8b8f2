// dq_weighted.h -- launchers of the weighted path (allPixelsUnique = 0),
// dq_weighted.hip.  Not part of the public ABI (see include/).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dq_internal.h"

namespace dq {

// calc_color_table (DivQuantMapColors.cpp:82-203) on the device: the unique
// colours of px[0..n) in the reference's output order (hash bucket ascending,
// first occurrence descending inside a bucket) as point records colour |
// count << 32 into rec (n entries of room; the weight of a point is norm *
// count, :195); *h_nu = the number of colours.  Waits for the stream once
// (the colour count).  Returns 0, or < 0 (-1: scratch too small).
size_t color_table_scratch_bytes(uint32_t n);
int launch_color_table(const uint32_t* px, uint32_t n, void* scratch, size_t scratch_bytes, uint64_t* rec,
                       uint32_t* h_nu, hipStream_t stream);

// ---------------------------------------------------------------------------
// DivQuantCluster<false,*,true> (DivQuantCluster.cpp:133-1097) over a round of
// nodes.  Every weighted statistic is a SEQUENTIAL FP64 fold s += x_i over a
// node's points in point order (:73-85, :496-517, :719-770).  The passes
// reproduce each fold exactly with the whole GPU (dq_weighted.hip, "exact
// parallel fold"): tiles of kWTile points classify every summand by the
// binade its running sum is certain to lie in, reduce RNE(x / ulp) as exact
// integers per binade run, and a per-node chain applies runs and the rare
// uncertain summands ("specials": binade crossings, ties) in order.
constexpr uint32_t kWTile = 4096;   // points per tile (256 lanes x 16 consecutive points)
constexpr int kWCh = 7;              // folds per pass: w*R, w*G, w*B, w, w*R^2, w*G^2, w*B^2
enum WPass : int32_t { WP_INIT = 0, WP_SPLIT = 1, WP_KM = 2 };

// One node of a weighted round: its record and the state carried across the
// round's passes (written by the chain kernel).
struct alignas(16) WState {
  const uint64_t* src;        // point records (colour | count << 32) at src[off .. off+len), point order
  uint64_t* dst;              // the children's records: old half at dst[off ..), then the new half
  uint32_t off, len;
  int32_t tile_begin, tile_end;
  int32_t root;               // 1: the init folds first (DivQuantClusterInitMeanAndVar, :36-123)
  int32_t done;               // 0: active; 1: the split is final
  double tw;                  // weight[old_index] (root: 1.0, :329)
  double tm[3], tv[3];        // node mean / var (root: from the init folds)
  int32_t box_lo[3], box_hi[3];   // a box holding every point (R, G, B)
  int32_t axis, iter;         // cut axis (:388-403); 2-means passes completed
  double cut;                 // split: new iff cut < v_axis (:473)
  double lhs, rr, rg, rb;     // 2-means: old iff lhs < rr*R + rg*G + rb*B (:683)
  double prev[4];             // the last pass's sums and weight (fixed-point test)
  double nw, ow, nm[3], om[3], nsq[3];
  uint32_t n_new;             // new-side points of the final membership
  int32_t done_it;            // 2-means iterations at finalisation
  int32_t proven;             // final at the split: the cut is the 2-means fixed point
  uint32_t seq_tiles;         // tiles whose folds ran one summand at a time (diagnostic)
};

struct alignas(16) WTile {
  int32_t node;               // index into the round's WState array
  uint32_t start, end;        // positions in the node's id buffer (absolute)
  uint32_t pad;
};

// A tile's contribution to one fold, as the chain applies it: its summands
// in tile order as at most kWSeg segments -- a run of binade e adding the
// exact integer sum M of RNE(x / 2^(e-52)), or one special summand x added
// in hardware.  nseg < 0: more segments than that (a node's first tile has
// 20-40: its sum crosses a binade every few summands from s = 0; on a 4K
// noise frame 7 of the deep levels' first tiles had more than 64): the
// chain folds the tile's summands one at a time (~20 us per tile and fold).
constexpr int kWSeg = 128;
constexpr int32_t kWSpecial = -100002;   // segment kind: a special summand (v = its bits)
struct alignas(16) WSegment {
  int32_t e;                  // binade of a run, or kWSpecial
  int32_t pad;
  int64_t v;                  // run: M; special: the summand's bits
};
struct alignas(16) WFold {
  int32_t nseg, pad[3];
  WSegment seg[kWSeg];
};
// The chain's quick form of a tile's fold: one run (e, M) and nothing else,
// or kWComplex (read the WFold).
constexpr int32_t kWComplex = -100000;
struct alignas(16) WQuick {
  int32_t e;
  uint32_t cnt;               // (channel 0's record: the tile's taken points)
  int64_t m;
};

struct WArgs {
  WState* nodes;
  const WTile* tiles;
  double norm;                // calc_color_table's norm_factor (a point's weight: norm * count)
  double* tsum;               // [tile][8] the tile's sums (any order: an estimate)
  double* tpre;               // [tile][8] exclusive node prefix of tsum
  WFold* fold;                // [tile][kWCh]
  WQuick* quick;              // [tile][kWCh]
  uint32_t* pbase;            // [tile][2] partition bases (old, new) inside the node
  uint32_t* active;           // host-coherent flag: 1 when a node is not final after the split pass
  uint32_t* gen;              // [tile] folds whose description needs the general classify (bit ch)
  NodeResult* res;            // [node] (host-coherent)
  int32_t nn, ntiles, max_iters, fixed_point, it, pad;
};
void launch_wpass(int pass, const WArgs& a, hipStream_t stream);   // one statistics pass + epilogues
void launch_wfinish(const WArgs& a, hipStream_t stream);           // partition + results

// cut_bits + calc_color_table's decimated walk (DivQuantUni.cpp:28-100,
// DivQuantMapColors.cpp:120-125): out[t] for t = a*nc + b (a < nr, b < nc) is
// in[b*dec + a*dec*stride] with each channel shifted right by sr / sg / sb --
// the reference's loop order and its numRows stride.  The caller checks that
// every index lies inside the input.
void launch_cut_gather(const uint32_t* in, uint32_t* out, uint32_t nr, uint32_t nc, uint32_t dec,
                       uint32_t stride, uint32_t sr, uint32_t sg, uint32_t sb, hipStream_t stream);

// ---------------------------------------------------------------------------
// The whole weighted quant_recurse of a SMALL input in one workgroup
// (dq_wsmall.hip): the app calls quant_recurse(N_region, .., K=4,
// allPixelsUnique=0) once per superpixel region (ClusteringSegmentation.cpp:
// 1779-1803), 10^3-10^5 pixels each, where the multi-kernel path above pays
// ~1 ms of launches and host round trips per call against the reference's
// 30-1000 us on one core.  One launch: calc_color_table in LDS (hash table,
// counting sort by bucket, first occurrence descending inside a bucket),
// then DivQuantCluster<false,*,true> split by split in the reference's own
// order (:346-892, the greedy choice on the device), every fold sequential in
// point order as the reference's (one wave per fold; 64 summands added as one
// exact integer run when they provably stay in one binade), the stable
// partitions in LDS, the final centres and the first-occurrence dedup
// (quant_util.cpp:93-118), and -- for at most kWsMapMax deduped colours,
// where std::sort is libstdc++'s insertion sort (stable) -- the palette sort,
// lut_init and map_colors_mps (DivQuantMapColors.cpp:227-527) too.
constexpr uint32_t kWsMaxN = 131071;   // pixels (first occurrences fit 17 bits)
constexpr uint32_t kWsMaxU = 6144;     // unique colours (LDS: two 48-KB record buffers)
constexpr int kWsMaxK = 64;            // clusters
constexpr int kWsMapMax = 16;          // deduped colours mapped in the kernel
struct WSmallResult {                  // host-coherent pinned memory
  uint32_t status;                     // 1: done; 2: more than kWsMaxU colours (nothing else valid)
  uint32_t nu, k_raw, num_empty;       // colours; ct entries before the dedup; empty clusters
  uint32_t mapped, m, passes, pad;     // out written; deduped colours; fold passes run
  uint32_t ct[kWsMaxK];                // final centres, empty clusters dropped (:1029-1096)
  double means[kWsMaxK * 3];           // mean[] per cluster index (diagnostics)
  int64_t sizes[kWsMaxK];
  int64_t trace[(kWsMaxK - 1) * 4];    // new_index old_index |C| |new| per split
  // phase profile (wall_clock64 ticks, 100 MHz): [0] start, [1] hash set
  // built, [2] table sorted, [3] clustering done, [4] map done; [5] ticks in
  // fold passes, [6] in partitions; [7] passes by kind: init | split << 16 | 2-means << 32
  uint64_t prof[8];
};
struct WsMapTab {                      // device: the palette for the grid map of a larger input
  uint32_t go, m;                      // go: wsmall_kernel left a palette (0: nothing to map)
  uint32_t pal[kWsMapMax];             // sorted by R+G+B (sort_color)
  uint16_t lut[766];                   // lut_init
};
struct WSmallArgs {
  const uint32_t* px;                  // n pixels (device)
  uint32_t* out;                       // mapped colours, or nullptr (cluster only)
  WSmallResult* res;                   // device view of the host-coherent result
  WsMapTab* maptab;                    // device scratch (the map of inputs above 16384 pixels)
  double norm;                         // calc_color_table's norm_factor (:184)
  uint32_t n;
  int32_t k, max_iters, fixed_point;
};
hipError_t launch_wsmall(const WSmallArgs& a, hipStream_t stream);   // (the launch's error, if any)
// Many inputs in one launch, one workgroup each (d_args: nregions argument
// records in device-visible memory, maptab null: a region whose map needs
// the grid kernel is left unmapped, res->mapped = 0).
hipError_t launch_wsmall_batch(const WSmallArgs* d_args, int nregions, hipStream_t stream);

}  // namespace dq
