/*
 * dq_hip.h -- the thin C ABI of libdivquant_hip.so (MI355X / gfx950).
 *
 * Plain pointers and sizes only (no torch, no HIP types in the signatures;
 * `stream` is a hipStream_t passed as void*; NULL = the library's stream,
 * which first waits for the work already queued on the default stream, so
 * inputs written there -- a framework's host-to-device copy -- are seen).
 * The reference-signature wrappers (include/DivQuantHeader.h,
 * include/quant_util.h) are implemented on top of these entry points; an FFI
 * (ctypes, cgo, JNI...) can bind them directly -- see INTEGRATION.md.
 *
 * Errors: HIP/runtime failures abort the process with a message on stderr,
 * like the reference's abort() paths (DivQuantCluster.cpp:1021-1026,
 * DivQuantMapColors.cpp:43-51).  Invalid arguments return a negative code.
 */
#ifndef DQ_HIP_H
#define DQ_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DQ_HIP_ABI_VERSION 1

int dq_hip_abi_version(void);
/* Number of visible HIP devices (0 when none). */
int dq_hip_device_count(void);

/* ---- host-pointer entry points (SURVEY 8b build-side shim) ---------------
 * dq_hip_quant: quant_recurse semantics (quant_util.cpp:20-158) without the
 * stdout timer lines.  uniq: allPixelsUnique (1: uniform weights; 0: the
 * weighted path -- calc_color_table dedup + ordered FP64 folds, exactly the
 * reference's).  ngpus <= 1: current device; ngpus > 1 (uniform
 * weights): the pixels split into ngpus ranges over devices 0..ngpus-1 of
 * this process (clamped to the visible devices), every pass's node totals
 * allreduced over an in-process RCCL communicator set (ncclCommInitAll,
 * xGMI), each device mapping its own range.
 * Returns the number of empty clusters (>= 0) or < 0 on bad arguments. */
int dq_hip_quant(const uint32_t *in, uint32_t n, uint32_t *out, uint32_t *k,
                 uint32_t *ct, int uniq, int ngpus);
/* map_colors_mps semantics (DivQuantMapColors.cpp:243-539). */
int dq_hip_map(const uint32_t *in, uint32_t n, uint32_t *out,
               const uint32_t *ct, int k);

/* genHistogramsForBlocks (ClusteringSegmentation.cpp:365-576) without the
 * OpenCV Mats: map the W x H frame `in` (0x00RRGGBB, Vec3BToUID packing,
 * OpenCVUtil.h:19-27) onto `palette` (npal colours; the app passes
 * getSubdividedColors, see dq_subdivided_colors) with map_colors_mps, then per
 * block of dim x dim pixels (block_w x block_h blocks, row-major) the most
 * frequent mapped colour, ties broken by the reference's unordered_map
 * iteration order.  mode: block_w*block_h words = HistogramForBlock::
 * regionQuantPixel (and the BGR of blockMat).  Optional (NULL to skip):
 * quant (W*H mapped frame), ndistinct (per block table size), keys/counts
 * (block_w*block_h*dim*dim words: each block's pixelToCountTable in iteration
 * order).  dim 1..4 (the app uses 4, ClusteringSegmentationMain.cpp:138);
 * every block must hold a pixel.  Returns 0 or < 0. */
int dq_hip_block_hist(const uint32_t *in, uint32_t width, uint32_t height,
                      const uint32_t *palette, int npal, uint32_t dim,
                      uint32_t block_w, uint32_t block_h, uint32_t *quant,
                      uint32_t *mode, uint32_t *ndistinct, uint32_t *keys,
                      uint32_t *counts);
/* getSubdividedColors (superpixels/OpenCVUtil.cpp:853-897): 125 colours. */
void dq_subdivided_colors(uint32_t *out125);
/* Synthetic benchmark frames: xorshift64 s^=s<<13; s^=s>>7;
 * s^=s<<17, one draw per pixel, pixel = draw & 0xFFFFFF; frame f of a batch
 * uses seed 0x9E3779B97F4A7C15 + f.  Host memory, no GPU needed. */
void dq_synth_xorshift(uint32_t *out, uint64_t n, uint64_t seed);
/* Word-wise FNV-1a-64 of n uint32 words (the golden fixtures' output hash). */
uint64_t dq_fnv1a64(const uint32_t *w, uint64_t n);

/* ---- device-pointer entry points (inputs already resident in HBM) --------
 * d_in/d_out: device pointers on `device`; k/ct: host.  Synchronous with
 * respect to the host on return (ct and *k are final). */
int dq_hip_quant_dev(int device, const uint32_t *d_in, uint32_t n,
                     uint32_t *d_out, uint32_t *k, uint32_t *ct,
                     int max_iters, void *stream);
/* A batch of frames in one call: every pass of every split round is one
 * kernel launch over the points of all frames.  d_in/d_out/n: nframes
 * entries; ct: nframes*k host words (frame i at ct + i*k); k_out[i] = its
 * colour count.  Returns the total number of empty clusters or < 0. */
int dq_hip_quant_batch_dev(int device, int nframes, const uint32_t *const *d_in,
                           const uint32_t *n, uint32_t *const *d_out, uint32_t k,
                           uint32_t *ct, uint32_t *k_out, int max_iters,
                           void *stream);
/* dq_hip_block_hist on device pointers (in, quant, mode, ndistinct, keys,
 * counts; quant is required: the mapped frame); palette is host memory.
 * Asynchronous on `stream`; with stream NULL the legacy default stream is
 * ordered after the work (as for every asynchronous entry below). */
int dq_hip_block_hist_dev(int device, const uint32_t *d_in, uint32_t width,
                          uint32_t height, const uint32_t *palette, int npal,
                          uint32_t dim, uint32_t block_w, uint32_t block_h,
                          uint32_t *d_quant, uint32_t *d_mode,
                          uint32_t *d_ndistinct, uint32_t *d_keys,
                          uint32_t *d_counts, void *stream);
/* BGR24 ingestion / output, device pointers, asynchronous
 * on `stream` (NULL: the library's stream of `device`).  d_bgr: an OpenCV
 * CV_8UC3 frame, `stride` bytes per row (>= 3*width; 3*width when
 * continuous).  Fast path when width, stride and d_bgr are 4-B aligned and
 * the u32 frame is 16-B aligned; any other layout is handled per pixel.
 * Return 0 or -1 on bad arguments.
 *   pack:   d_out[y*width+x] = Vec3BToUID(img(y,x))   (superpixels/OpenCVUtil.h:19-27;
 *           the loop at ClusteringSegmentation.cpp:381-395)
 *   unpack: img(y,x) = PixelToVec3b(d_in[y*width+x])  (OpenCVUtil.h:53-59;
 *           ClusteringSegmentation.cpp:1812-1817); bits 24-31 are dropped
 *   gather: d_out[i] = Vec3BToUID(img(c.y, c.x)) for the i-th Coord, passed
 *           as its 32-bit layout (x | y << 16, superpixels/Coord.h:30-33);
 *           ClusteringSegmentation.cpp:1795-1800.  Coords are not range-checked. */
int dq_hip_pack_bgr24_dev(int device, const uint8_t *d_bgr, uint32_t width,
                          uint32_t height, uint32_t stride, uint32_t *d_out,
                          void *stream);
int dq_hip_unpack_bgr24_dev(int device, const uint32_t *d_in, uint32_t width,
                            uint32_t height, uint32_t stride, uint8_t *d_bgr,
                            void *stream);
int dq_hip_gather_bgr24_dev(int device, const uint8_t *d_bgr, uint32_t stride,
                            const uint32_t *d_coords, uint32_t n, uint32_t *d_out,
                            void *stream);
/* Row-tile sharding.  Frame i's rows are d_in[i] (n[i] points,
 * width[i] per row; width NULL or 0: shard boundaries on 4-point multiples).
 * Inside this process the rows are split into nshard (1..8) row ranges that
 * are processed as separate shards on `device` (the exact arithmetic of
 * multi-GPU sharding); across processes, n_global[i] (NULL or 0: n[i]) is the
 * whole frame's size and every pass's integer node totals are allreduced
 * over the communicator of dq_hip_comm_init (RCCL over xGMI).  Every
 * process gets the same colortables; d_out[i] receives this process's rows
 * mapped (d_out NULL: clustering only).  Returns empty clusters, -1 on bad
 * arguments, -2 if n_global > n without a communicator. */
int dq_hip_quant_rows_dev(int device, int nframes, const uint32_t *const *d_in,
                          const uint32_t *n, const uint32_t *width,
                          const uint64_t *n_global, int nshard,
                          uint32_t *const *d_out, uint32_t k, uint32_t *ct,
                          uint32_t *k_out, int max_iters, void *stream);
/* RCCL communicator of the engine on `device` (one process per GPU): rank 0
 * creates the 128-byte id, the launcher broadcasts it (e.g. with
 * torch.distributed), every rank calls dq_hip_comm_init.  Return 0 / < 0. */
int dq_hip_comm_unique_id(void *id128);
int dq_hip_comm_init(int device, int nranks, int rank, const void *id128);
int dq_hip_comm_destroy(int device);
/* Ranks of the engine's communicator on `device` (1: none). */
int dq_hip_comm_size(int device);
/* Clustering only (quant_varpart_fast, DivQuantCluster.cpp:1099-1179):
 * writes the non-empty cluster colours (cluster-index order, NOT deduped). */
int dq_hip_cluster_dev(int device, const uint32_t *d_in, uint32_t n,
                       uint32_t *k, uint32_t *ct, int max_iters, void *stream);
/* The weighted path (allPixelsUnique = 0) on device pixels: calc_color_table
 * on the GPU (DivQuantMapColors.cpp:82-203), DivQuantCluster<false,*,true>
 * with the reference's ordered FP64 folds, then (d_out != NULL) the colortable
 * dedup and map_colors_mps into d_out; d_out NULL: quant_varpart_fast's table
 * (cluster-index order, not deduped).  Synchronous on return. */
int dq_hip_quant_weighted_dev(int device, const uint32_t *d_in, uint32_t n,
                              uint32_t *d_out, uint32_t *k, uint32_t *ct,
                              int max_iters, void *stream);
/* Many weighted calls at once -- the app's per-superpixel-region
 * quant_recurse(N_region, .., K, allPixelsUnique=0)
 * (ClusteringSegmentation.cpp:1779-1803): region i reads d_ins[i][0..ns[i]),
 * writes its mapped colours to d_outs[i] (d_outs may be NULL: cluster + dedup
 * only), its deduped colortable to cts + i*ct_stride (ks[i] <= ct_stride
 * entries of room) and its size to k_outs[i].  Regions of at most 131071
 * pixels, 6144 colours and K <= 64 run in ONE launch, one workgroup each;
 * the others one by one.  Every result equals the region's own call.
 * Returns the total of empty clusters, or < 0 (bad arguments). */
int dq_hip_quant_weighted_regions_dev(int device, int nregions, const uint32_t *const *d_ins,
                                      const uint32_t *ns, uint32_t *const *d_outs, const uint32_t *ks,
                                      uint32_t *cts, uint32_t ct_stride, uint32_t *k_outs,
                                      int max_iters, void *stream);
/* quant_varpart_fast semantics (DivQuantCluster.cpp:1099-1179) on device
 * pixels for every (num_bits, dec_factor, allPixelsUnique): uniform weights
 * when uniq && num_bits == 8 && dec_factor == 1, else cut_bits to num_bits
 * (DivQuantUni.cpp:28-100; skipped when !uniq && num_bits == 8), the
 * decimated calc_color_table walk over a rows x cols frame with the
 * reference's numRows stride (DivQuantMapColors.cpp:120-125) and the weighted
 * clustering, centres shifted back by 8 - num_bits (:1050-1052).  ct gets
 * the table in cluster-index order (not deduped, not mapped).  Returns the
 * number of empty clusters, -1 on bad arguments, -2 when the walk would read
 * past n (the reference reads out of bounds there).  Synchronous on return. */
int dq_hip_varpart_dev(int device, const uint32_t *d_in, uint32_t n, uint32_t rows,
                       uint32_t cols, uint32_t *k, uint32_t *ct, int num_bits,
                       int dec_factor, int max_iters, int uniq, void *stream);
/* cut_bits (DivQuantUni.cpp:28-100) on device pixels: each channel shifted
 * right by 8 - its bit count (1..8); d_out may equal d_in.  Stream-ordered. */
int dq_hip_cut_bits_dev(int device, const uint32_t *d_in, uint32_t n, uint32_t *d_out,
                        int num_bits_red, int num_bits_green, int num_bits_blue,
                        void *stream);
int dq_hip_map_dev(int device, const uint32_t *d_in, uint32_t n,
                   uint32_t *d_out, const uint32_t *ct, int k, void *stream);

/* ---- BGR24 frames (OpenCV CV_8UC3: B, G, R bytes, `stride` bytes per row)
 * quant_recurse of device BGR24 frames without the packed conversion
 * (SURVEY 8f.3): with uniq = 1 and continuous rows (stride == 3*width) the
 * root's passes, its partition and the map read the 3-B pixels directly
 * (a frame whose pointer is not 16-B aligned or whose pixel count is not a
 * multiple of 16 is first copied to aligned scratch); padded rows or uniq = 0
 * (the weighted path's colour table) pack the frame on the GPU first.  d_out
 * gets packed 0x00RRGGBB colours (the reference's output format).  The batch
 * form runs every frame of a call over the engine lanes like
 * dq_hip_quant_batch_dev (ct: nframes * k, k_out: nframes).  Returns the
 * number of empty clusters or < 0. */
int dq_hip_quant_bgr24_batch_dev(int device, int nframes, const uint8_t *const *d_bgr,
                                 uint32_t width, uint32_t height, uint32_t stride,
                                 uint32_t *const *d_out, uint32_t k, uint32_t *ct,
                                 uint32_t *k_out, int uniq, int max_iters, void *stream);
int dq_hip_quant_bgr24_dev(int device, const uint8_t *d_bgr, uint32_t width, uint32_t height,
                           uint32_t stride, uint32_t *d_out, uint32_t *k, uint32_t *ct,
                           int uniq, int max_iters, void *stream);
/* map_colors_mps of a device BGR24 frame (read directly when K <= 1024 and
 * the rows are continuous) into packed colours. */
int dq_hip_map_bgr24_dev(int device, const uint8_t *d_bgr, uint32_t width, uint32_t height,
                         uint32_t stride, uint32_t *d_out, const uint32_t *ct, int k,
                         void *stream);

/* ---- diagnostics of the last clustering on `device` ----------------------
 * means: k*3 doubles (the reference's mean[ic] per cluster index, the north
 * star's "float centroids"); sizes: k cluster sizes; trace: (k-1)*4 of
 * new_index, old_index, |C|, |new| per split.  Return 0 or < 0. */
int dq_hip_last_centroids(int device, double *means, int64_t *sizes, int k);
int dq_hip_last_trace(int device, int64_t *trace, int k);
int dq_hip_last_rounds(int device);
/* Points read by all statistics passes of the last clustering. */
uint64_t dq_hip_last_points_swept(int device);
/* Points the last run would have swept without fixed-point finalisation
 * (every split: split pass + max_iters 2-means passes, as the reference). */
uint64_t dq_hip_last_points_full(int device);
/* Weighted path: tiles of the last run whose folds ran one summand at a time
 * (the exact parallel fold's fallback). */
uint64_t dq_hip_last_seq_tiles(int device);
/* Records of the last run finalised at a frame's last planned round (whose
 * partition counts no partition cursors) that a later round partitioned:
 * their cursors counted then. */
uint64_t dq_hip_last_cursor_fixes(int device);
/* Fixed-point finalisation (default on; DQ_HIP_TUNE=full_iters=1 turns the
 * default off).  A split whose 2-means pass reproduces the previous pass's exact
 * integer sums is final: the remaining iterations of the reference's loop
 * (DivQuantCluster.cpp:613) would recompute the same means and decision.
 * Outputs are identical either way; only the swept points differ. */
void dq_hip_set_fixed_point(int device, int on);
/* Device-planned rounds (default on; DQ_HIP_TUNE=plan=0 turns the default off):
 * while a frame may still need splits, the next round's tables are built on
 * the GPU from the current round's results and the round is enqueued before
 * the host has seen them.  Outputs are identical either way;
 * speculation may expand nodes the greedy replay never uses.
 * dq_hip_last_planned_rounds: how many rounds of the last run were planned. */
void dq_hip_set_planned_rounds(int device, int on);
int dq_hip_last_planned_rounds(int device);
/* One-launch 2-means loops: a round whose records all hold at
 * most max_points points (default 49152; DQ_HIP_TUNE=kloop_max=N) and that has at
 * most one record per CU runs all its 2-means iterations in one
 * kloop_kernel launch, one workgroup per record.  0 turns it off.  Outputs
 * are identical either way.  dq_hip_last_loop_rounds: how many rounds of the
 * last run did so. */
void dq_hip_set_loop_max(int device, uint32_t max_points);
int dq_hip_last_loop_rounds(int device);
/* One-launch 2-means loops over a round's tiles (default on,
 * DQ_HIP_TUNE=persist=0 turns the default off): a round kloop does not take,
 * of one shard per record, planar records and at most 4 tiles per CU (or,
 * once its split status is known, at most 4 tiles per CU of records still
 * active), runs all its 2-means iterations in one kpersist_kernel launch, a
 * record's workgroups meeting per iteration.  Outputs are identical either way.
 * dq_hip_last_persist_rounds: how many rounds of the last run did so. */
void dq_hip_set_persist(int device, int on);
int dq_hip_last_persist_rounds(int device);
/* The weighted path (allPixelsUnique = 0) of a small input -- at most 131071
 * pixels, 6144 colours, 64 clusters, no cut_bits / decimation: a superpixel
 * region of the app, ClusteringSegmentation.cpp:1779-1803 -- in ONE launch of
 * one workgroup (DESIGN.md 5d'; default on, DQ_HIP_TUNE=wsmall=0 turns the
 * default off): colour table, the splits in the reference's order with its
 * sequential folds, dedup and, for at most 16 deduped colours, the map.
 * Outputs are identical either way. */
void dq_hip_set_wsmall(int device, int on);
/* Phase profile of the last weighted call if it took the one-launch path
 * (0 values otherwise): wall_clock64 ticks (100 MHz) at its start, hash set,
 * sorted colour table, clustering, map; ticks in fold passes and partitions;
 * passes by kind (init | split << 16 | 2-means << 32).  Returns the count. */
int dq_hip_last_wsmall_profile(int device, uint64_t* out, int nout);

/* Engine lanes a batch of frames is split over (each: own stream, own host
 * thread; DQ_HIP_LANES; default 4 when GPU_MAX_HW_QUEUES >= 6 at the first
 * batch call, else 3 -- HIP reads GPU_MAX_HW_QUEUES once, when it
 * initialises, so set it before any HIP call of the process).  lanes = 0
 * restores the default. */
void dq_hip_set_lanes(int lanes);
int dq_hip_get_lanes(void);

/* ---- per-kernel timing (HIP events on the launch stream) -----------------
 * kinds: 0 init pass, 1 split pass, 2 2-means pass, 3 last 2-means pass,
 * 4 epilogue, 5 partition, 6 map cells, 7 map, 8 plan.  bytes = the engine
 * work model's bytes (4 B per point read from the caller's
 * packed frame, 3 B per point read or written in the planar working
 * buffers, 8 B per mapped pixel); units = points (pixels) processed. */
void dq_hip_set_timing(int device, int on);
void dq_hip_reset_stats(int device);
int dq_hip_get_stat(int device, int kind, uint64_t *launches, double *ms,
                    double *bytes);
int dq_hip_get_stat_units(int device, int kind, double *units);
const char *dq_hip_stat_name(int kind);

/* ---- build identity and test-only knobs ----------------------------------
 * dq_hip_build_id: FNV-1a-64 of the sources the library was built from
 * (tools/source_id.py; a test compares it with the tree beside the .so).
 * dq_hip_set_debug: interleaving knobs for the hand-off tests (flags of
 * dq_kernels.h kDebug*: 1 prewarm the 2-means hand-off lines, 2 uneven
 * workgroup stalls, 4 host delays between status and results, 8 plan-kernel
 * stall, 16 abort unless the round arena is all zero when a run starts, 32
 * release the round arena at every run's start: new chunks); every
 * lane of `device`; 0 (the default) in production.  Outputs are identical
 * under every flag. */
uint64_t dq_hip_build_id(void);
void dq_hip_set_debug(int device, int flags);
/* Test-only: the row-tile sharding of nranks (1..8) processes, run by
 * nranks engines of THIS process on `device`, each with its own stream and
 * host thread, joined by an in-process loopback collective instead of RCCL
 * (the TOT_ALLREDUCE path with every rank's local counts != the global
 * totals).  Rank r holds rows [r*height/nranks, (r+1)*height/nranks) of every
 * frame (width x height, d_in / d_out whole frames), maps them into the same
 * rows of d_out and writes its colortables to ct + (r*nframes + i)*k, its
 * counts to k_out[r*nframes + i].  coll_log (nranks x log_cap, may be NULL)
 * gets the element count of each collective rank r enqueued, log_len[r] how
 * many it enqueued.  Synchronous; returns rank 0's empty clusters or -1. */
int dq_hip_loopback_rows_dev(int device, int nranks, int nframes, const uint32_t *const *d_in,
                             uint32_t width, uint32_t height, uint32_t *const *d_out,
                             uint32_t k, uint32_t *ct, uint32_t *k_out, int max_iters,
                             uint64_t *coll_log, int log_cap, int *log_len);

#ifdef __cplusplus
}
#endif

#endif /* DQ_HIP_H */
