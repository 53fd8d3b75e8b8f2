// dq_kernels.h -- host-callable launchers for the gfx950 kernels in
// dq_kernels.hip.  Every launcher only enqueues work on `stream`; none of
// them allocates, copies or synchronises (so a caller may capture them in a
// hipGraph).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dq_internal.h"

namespace dq {

constexpr int kBlock = 256;                 // 4 wave64 per workgroup
constexpr int kPxPerThread = 16;            // points per lane per sweep step
constexpr int kSweep = kBlock * kPxPerThread;   // 4096 points per step
constexpr uint32_t kMaxTilePx = 16 * kSweep;    // keeps per-wave u32 sums exact

// Map (nearest palette entry) cell grid: 32 cells of 8 values per channel.
constexpr int kCellBits = 5;
constexpr int kCells = 1 << (3 * kCellBits);
constexpr int kCellCap = 32;                // candidates stored per cell
constexpr uint16_t kCellOverflow = 0xFFFF;  // count marker: scan whole palette

struct PixelBufs {
  const uint32_t* in;
  uint32_t* p0;
  uint32_t* p1;
};

// One statistics pass over every tile of the round.
void launch_pass(int kind, const Tile* tiles, int ntiles, const DevNode* nodes,
                 PixelBufs bufs, TilePartial* parts, hipStream_t stream);

// FP64 epilogue of a pass, one workgroup per node (reduces that node's tiles).
void launch_epilogue(int kind, DevNode* nodes, int nnodes, Tile* tiles,
                     const TilePartial* parts, double s, hipStream_t stream);

// Writes every node's points into its two children's segments (old half
// first, then new half), in index order, in the other working buffer.
void launch_partition(const Tile* tiles, int ntiles, const DevNode* nodes,
                      PixelBufs bufs, hipStream_t stream);

// Map: candidate lists per colour cell, then the per-pixel argmin over
// (squared distance, MPS visit rank).
void launch_build_cells(const uint32_t* pal_sorted, int k, uint16_t* cell_cnt,
                        uint16_t* cell_idx, hipStream_t stream);
void launch_map(const uint32_t* in, uint32_t n, uint32_t* out,
                const uint32_t* pal_sorted, int k, const uint16_t* lut_init,
                const uint16_t* cell_cnt, const uint16_t* cell_idx,
                hipStream_t stream);

}  // namespace dq
