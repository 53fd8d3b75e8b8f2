/*
 * DivQuantHeader.h -- drop-in declarations of the reference DivQuant API,
 * served by libdivquant_hip.so (MI355X / gfx950).
 *
 * Same types, macros and prototypes (C++ linkage) as the reference header
 * DivQuant/DivQuantHeader.h:31-96, so callers such as
 * ClusteringSegmentation/ClusteringSegmentation.cpp compile and link against
 * this library unchanged.  Each prototype names the reference definition it
 * replaces.  Like the reference header, <stdint.h> is expected from the
 * includer; it is included here as well for convenience.
 */
#ifndef DivQuantHeader_h
#define DivQuantHeader_h

#include <ctype.h>
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <vector>

#define MAX_RGB     ( 255 )     /* DivQuantHeader.h:31 */
#define MAX_RGB_SQR ( 65025 )   /* DivQuantHeader.h:32 */
#define MAX_COLORS  ( 256 )     /* DivQuantHeader.h:33 */

typedef unsigned char uchar;    /* :35-38 */
typedef unsigned short ushort;
typedef unsigned int uint;
typedef unsigned long ulong;

/* :40-44 */
typedef struct
{
  int red, green, blue;
  int weight;
} Pixel_Int;

/* :46-50 */
typedef struct
{
  double red, green, blue;
  double weight;
} Pixel_Double;

/* DivQuantMisc.cpp:18-22 -- CPU clock() timer start. */
clock_t start_timer ( void );
/* DivQuantMisc.cpp:24-28 -- seconds since start_timer(). */
double stop_timer ( const clock_t );

/* DivQuantMapColors.cpp:43-51 -- abort with "Insufficient memory !" if x != 0. */
void check_mem ( const int );

/* DivQuantMapColors.cpp:205-220 -- uniform point weight 1/numPixels. */
double
get_double_scale(const uint32_t *inPixels,
                 const uint32_t numPixels);

/* DivQuantMisc.cpp:30-34 -- elapsed milliseconds between two clock() values. */
long timediff(clock_t t1, clock_t t2);

/* DivQuantMapColors.cpp:243-539 -- nearest palette colour per pixel
 * (MPS search semantics).  GPU: sorted palette + LUT on the host, per-pixel
 * argmin on the MI355X.  outColortablePtr is read only. */
void map_colors_mps ( const uint32_t *inPixelsPtr, uint32_t numPixels, uint32_t *outPixelsPtr, uint32_t *outColortablePtr, int colormapSize );

/* DivQuantMapColors.cpp:82-203 -- unique colours + normalised counts
 * (hash-bucket order).  Host utility; returns new[]-allocated weights. */
double *
calc_color_table ( const uint32_t *inPixels,
                  const uint32_t numPixels,
                  uint32_t *outPixels,
                  const uint32_t numRows,
                  const uint32_t numCols,
                  const int dec_factor,
                  int *num_colors );

/* DivQuantUni.cpp:28-100 -- uniform bit truncation (host utility). */
void
cut_bits ( const uint32_t *inPixels,
          const uint32_t numPixels,
          uint32_t *outPixels,
          const uchar num_bits_red,
          const uchar num_bits_green,
          const uchar num_bits_blue );

/* DivQuantCluster.cpp:1099-1179 -- divisive clustering into <= *numClustersPtr
 * colours, on the GPU for every (num_bits, dec_factor, allPixelsUnique):
 * the uniform-weight rounds for allPixelsUnique && num_bits == 8 &&
 * dec_factor == 1 (the combination quant_recurse uses), else cut_bits + the
 * decimated calc_color_table walk + the weighted rounds (:1130-1146).  A walk
 * that would read past the input (numRows > numCols: the reference reads out
 * of bounds there) aborts with a message. */
void
quant_varpart_fast (
                    const uint32_t numPixels,
                    const uint32_t *inPixels,
                    uint32_t *tmpPixels,
                    const uint32_t numRows,
                    const uint32_t numCols,
                    uint32_t *numClustersPtr,
                    uint32_t *colortablePtr,
                    const int num_bits,
                    const int dec_factor,
                    const int max_iters,
                    const int allPixelsUnique);

/* DivQuantMisc.cpp:36-46 -- 1 if 0 < num_bits <= 8 else 0 (prints an error). */
int validate_num_bits ( const uchar );

#endif /* DivQuantHeader_h */
