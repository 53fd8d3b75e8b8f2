/*
 * quant_util.h -- drop-in declaration of the reference's C-linkage entry
 * point (DivQuant/quant_util.h:6-14), served by libdivquant_hip.so.
 * Can be included from C or C++.
 */
#ifndef quant_util_h
#define quant_util_h

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Replaces DivQuant/quant_util.cpp:20-158: cluster numPixels 0x00RRGGBB
 * pixels into <= *numClustersPtr colours (max_iters=10, num_bits=8,
 * dec_factor=1), dedup the colortable by first occurrence, and write every
 * pixel's nearest palette colour to outColorTableOffsetPtr (it receives
 * COLOURS, quant_util.cpp:139).  in and out must not alias.  Prints the
 * reference's two timing lines unless DQ_HIP_QUIET is set. */
void quant_recurse ( uint32_t numPixels, const uint32_t *inPixelsPtr, uint32_t *outColorTableOffsetPtr, uint32_t *numClustersPtr, uint32_t *outColortablePtr, int allPixelsUnique );

#ifdef __cplusplus
}
#endif

#endif /* quant_util_h */
