// dq_weighted.h -- launchers of the weighted path (allPixelsUnique = 0),
// dq_weighted.hip.  Not part of the public ABI (see include/).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dq_internal.h"

namespace dq {

// calc_color_table (DivQuantMapColors.cpp:82-203) on the device: the unique
// colours of px[0..n) in the reference's output order (hash bucket ascending,
// first occurrence descending inside a bucket) into ucol, weights norm*count
// into uw (n entries of room each); *h_nu = the number of colours.  Waits for
// the stream once (the colour count).  Returns 0, or < 0 (-1: scratch too small).
size_t color_table_scratch_bytes(uint32_t n);
int launch_color_table(const uint32_t* px, uint32_t n, double norm, void* scratch, size_t scratch_bytes,
                       uint32_t* ucol, double* uw, uint32_t* h_nu, hipStream_t stream);

// One node of a weighted round: its points are ids into (ucol, uw) at
// src[off .. off+len) in point order; the split writes the old half to
// dst[off ..), then the new half (both in point order).
struct alignas(16) WNode {
  const uint32_t* src;
  uint32_t* dst;
  uint32_t off, len;
  double tw;                  // weight[old_index] (root: 1.0, :329)
  double tm[3], tv[3];        // mean / var of the node (root: from its init folds)
  int32_t root, pad;
};
struct WArgs {
  const WNode* nodes;
  const uint32_t* ucol;
  const double* uw;
  NodeResult* res;            // device, one per node
  int32_t max_iters;
  int32_t fixed_point;
};
// cut_bits + calc_color_table's decimated walk (DivQuantUni.cpp:28-100,
// DivQuantMapColors.cpp:120-125): out[t] for t = a*nc + b (a < nr, b < nc) is
// in[b*dec + a*dec*stride] with each channel shifted right by sr / sg / sb --
// the reference's loop order and its numRows stride.  The caller checks that
// every index lies inside the input.
void launch_cut_gather(const uint32_t* in, uint32_t* out, uint32_t nr, uint32_t nc, uint32_t dec,
                       uint32_t stride, uint32_t sr, uint32_t sg, uint32_t sb, hipStream_t stream);
// dst[i] = i (the root's point ids)
void launch_iota(uint32_t* dst, uint32_t n, hipStream_t stream);
// DivQuantCluster<false,*,true>'s split of every node (one workgroup each).
void launch_wsplit(const WArgs& a, int nnodes, hipStream_t stream);

}  // namespace dq
