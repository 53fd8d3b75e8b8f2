"""clusteringsegmentation-1_amd -- MI355X-native DivQuant hot path.

Python mirror of the reference's DivQuant interface (DivQuant/quant_util.h,
DivQuant/DivQuantHeader.h) over the C ABI of ``libdivquant_hip.so``
(include/dq_hip.h).  The compute runs in hand-written gfx950 kernels; there is
no CPU fallback: without the built library or without a HIP device every
compute call raises.

The directory name is not a Python identifier, so load it with
``load_package()`` (tests/, bench.py and __graft_entry__.py do).

Reference-named entry points (same argument meaning, host numpy arrays):
    quant_recurse(pixels, num_clusters, all_pixels_unique=1) -> (out, colortable)
    map_colors_mps(pixels, colortable)                       -> out
    quant_varpart_fast(pixels, num_clusters, max_iters=10)   -> colortable
Device-resident entry points (torch tensors / raw device pointers on HBM):
    quant_device, quant_batch_device, cluster_device, map_device
Row-tile sharding (one frame over shards / GPUs, RCCL allreduce per pass):
    quant_rows_device, comm_init_torch (comm_unique_id, comm_init, comm_destroy);
    loopback_rows_device (tests: N ranks in one process, loopback collective)
Full-frame block histograms (genHistogramsForBlocks):
    get_subdivided_colors, gen_histograms_for_blocks, block_hist_device
BGR24 (OpenCV CV_8UC3) ingestion / output on the GPU (Vec3BToUID / PixelToVec3b):
    pack_bgr24_device, unpack_bgr24_device, gather_bgr24_device
"""
import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# DQ_HIP_LIB: another build of the same library (kernel variants in experiments)
LIB_PATH = os.environ.get("DQ_HIP_LIB") or os.path.join(PKG_DIR, "libdivquant_hip.so")

STAT_KINDS = ["pass_init", "pass_split", "pass_kmeans", "pass_klast",
              "epilogue", "partition", "map_cells", "map", "plan", "kloop"]

_lib = None


class DivQuantError(RuntimeError):
    pass


def lib():
    """The ctypes handle of libdivquant_hip.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP/HSA runtime per process: when PyTorch is present, import it first
    # so the library binds (by soname) to the libamdhip64 torch already mapped
    # instead of mapping /opt/rocm's copy beside it -- two runtimes in one
    # process cannot both open the GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise DivQuantError("libdivquant_hip.so is not built (run __graft_entry__.build() "
                            "or make -C clusteringsegmentation-1_amd)")
    L = ctypes.CDLL(LIB_PATH)
    u32p, vp = ctypes.POINTER(ctypes.c_uint32), ctypes.c_void_p
    c = ctypes
    sigs = {
        "dq_hip_abi_version": ([], c.c_int),
        "dq_hip_device_count": ([], c.c_int),
        "dq_hip_quant": ([vp, c.c_uint32, vp, u32p, vp, c.c_int, c.c_int], c.c_int),
        "dq_hip_map": ([vp, c.c_uint32, vp, vp, c.c_int], c.c_int),
        "dq_hip_quant_dev": ([c.c_int, vp, c.c_uint32, vp, u32p, vp, c.c_int, vp], c.c_int),
        "dq_hip_quant_batch_dev": ([c.c_int, c.c_int, vp, vp, vp, c.c_uint32, vp, vp, c.c_int, vp],
                                   c.c_int),
        "dq_hip_quant_rows_dev": ([c.c_int, c.c_int, vp, vp, vp, vp, c.c_int, vp, c.c_uint32, vp, vp,
                                   c.c_int, vp], c.c_int),
        "dq_hip_comm_unique_id": ([vp], c.c_int),
        "dq_hip_comm_init": ([c.c_int, c.c_int, c.c_int, vp], c.c_int),
        "dq_hip_comm_destroy": ([c.c_int], c.c_int),
        "dq_hip_comm_size": ([c.c_int], c.c_int),
        "dq_hip_cluster_dev": ([c.c_int, vp, c.c_uint32, u32p, vp, c.c_int, vp], c.c_int),
        "dq_hip_map_dev": ([c.c_int, vp, c.c_uint32, vp, vp, c.c_int, vp], c.c_int),
        "dq_hip_quant_weighted_dev": ([c.c_int, vp, c.c_uint32, vp, u32p, vp, c.c_int, vp], c.c_int),
        "dq_hip_quant_weighted_regions_dev": ([c.c_int, c.c_int, vp, vp, vp, vp, vp, c.c_uint32, vp, c.c_int, vp],
                                              c.c_int),
        "dq_hip_last_centroids": ([c.c_int, vp, vp, c.c_int], c.c_int),
        "dq_hip_last_trace": ([c.c_int, vp, c.c_int], c.c_int),
        "dq_hip_last_rounds": ([c.c_int], c.c_int),
        "dq_hip_last_points_swept": ([c.c_int], c.c_uint64),
        "dq_hip_last_points_full": ([c.c_int], c.c_uint64),
        "dq_hip_last_seq_tiles": ([c.c_int], c.c_uint64),
        "dq_hip_last_cursor_fixes": ([c.c_int], c.c_uint64),
        "dq_hip_set_fixed_point": ([c.c_int, c.c_int], None),
        "dq_hip_set_planned_rounds": ([c.c_int, c.c_int], None),
        "dq_hip_last_planned_rounds": ([c.c_int], c.c_int),
        "dq_hip_set_loop_max": ([c.c_int, c.c_uint32], None),
        "dq_hip_last_loop_rounds": ([c.c_int], c.c_int),
        "dq_hip_set_persist": ([c.c_int, c.c_int], None),
        "dq_hip_set_wsmall": ([c.c_int, c.c_int], None),
        "dq_hip_last_wsmall_profile": ([c.c_int, c.c_void_p, c.c_int], c.c_int),
        "dq_hip_last_persist_rounds": ([c.c_int], c.c_int),
        "dq_hip_set_timing": ([c.c_int, c.c_int], None),
        "dq_hip_reset_stats": ([c.c_int], None),
        "dq_hip_get_stat": ([c.c_int, c.c_int, c.POINTER(c.c_uint64), c.POINTER(c.c_double),
                             c.POINTER(c.c_double)], c.c_int),
        "dq_hip_stat_name": ([c.c_int], c.c_char_p),
        "dq_hip_set_lanes": ([c.c_int], None),
        "dq_hip_get_lanes": ([], c.c_int),
        "dq_hip_block_hist": ([vp, c.c_uint32, c.c_uint32, vp, c.c_int, c.c_uint32, c.c_uint32,
                               c.c_uint32, vp, vp, vp, vp, vp], c.c_int),
        "dq_hip_block_hist_dev": ([c.c_int, vp, c.c_uint32, c.c_uint32, vp, c.c_int, c.c_uint32,
                                   c.c_uint32, c.c_uint32, vp, vp, vp, vp, vp, vp], c.c_int),
        "dq_subdivided_colors": ([vp], None),
        "dq_synth_xorshift": ([vp, c.c_uint64, c.c_uint64], None),
        "dq_fnv1a64": ([vp, c.c_uint64], c.c_uint64),
        "dq_hip_pack_bgr24_dev": ([c.c_int, vp, c.c_uint32, c.c_uint32, c.c_uint32, vp, vp], c.c_int),
        "dq_hip_unpack_bgr24_dev": ([c.c_int, vp, c.c_uint32, c.c_uint32, c.c_uint32, vp, vp],
                                    c.c_int),
        "dq_hip_gather_bgr24_dev": ([c.c_int, vp, c.c_uint32, vp, c.c_uint32, vp, vp], c.c_int),
        "dq_hip_varpart_dev": ([c.c_int, vp, c.c_uint32, c.c_uint32, c.c_uint32, u32p, vp, c.c_int, c.c_int,
                                c.c_int, c.c_int, vp], c.c_int),
        "dq_hip_cut_bits_dev": ([c.c_int, vp, c.c_uint32, vp, c.c_int, c.c_int, c.c_int, vp], c.c_int),
        "dq_hip_quant_bgr24_batch_dev": ([c.c_int, c.c_int, vp, c.c_uint32, c.c_uint32, c.c_uint32, vp,
                                          c.c_uint32, vp, vp, c.c_int, c.c_int, vp], c.c_int),
        "dq_hip_quant_bgr24_dev": ([c.c_int, vp, c.c_uint32, c.c_uint32, c.c_uint32, vp, u32p, vp, c.c_int,
                                    c.c_int, vp], c.c_int),
        "dq_hip_map_bgr24_dev": ([c.c_int, vp, c.c_uint32, c.c_uint32, c.c_uint32, vp, vp, c.c_int, vp],
                                 c.c_int),
        "quant_recurse": ([c.c_uint32, vp, vp, u32p, vp, c.c_int], None),
        "dq_hip_build_id": ([], c.c_uint64),
        "dq_hip_set_debug": ([c.c_int, c.c_int], None),
        "dq_hip_loopback_rows_dev": ([c.c_int, c.c_int, c.c_int, vp, c.c_uint32, c.c_uint32, vp, c.c_uint32,
                                      vp, vp, c.c_int, vp, c.c_int, vp], c.c_int),
    }
    ab = "DQ_HIP_LIB" in os.environ   # (A/B runs against an older build: its newer entry points absent)
    for name, (args, res) in sigs.items():
        if ab and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def _require_gpu():
    if lib().dq_hip_device_count() < 1:
        raise DivQuantError("no HIP device visible: the DivQuant hot path runs only on the GPU")


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


# ---------------------------------------------------------------------------
# Reference-named host entry points.
def quant_recurse(pixels, num_clusters, all_pixels_unique=1):
    """quant_recurse (DivQuant/quant_util.cpp:20-158): returns (out, colortable)."""
    _require_gpu()
    px = _u32(pixels).reshape(-1)
    if px.size == 0 or num_clusters <= 0:
        raise DivQuantError("numPixels and numClusters must be > 0")
    out = np.zeros(px.size, np.uint32)
    ct = np.zeros(num_clusters, np.uint32)
    k = ctypes.c_uint32(num_clusters)
    lib().quant_recurse(px.size, _ptr(px), _ptr(out), ctypes.byref(k), _ptr(ct), int(all_pixels_unique))
    return out, ct[:k.value].copy()


def quant_host(pixels, num_clusters, all_pixels_unique=1, ngpus=1):
    """dq_hip_quant (quant_recurse without the timer lines) on host pixels;
    ngpus > 1 shards the frame over this process's devices (RCCL in-process)."""
    _require_gpu()
    px = _u32(pixels).reshape(-1)
    out = np.zeros(px.size, np.uint32)
    ct = np.zeros(num_clusters, np.uint32)
    k = ctypes.c_uint32(num_clusters)
    if lib().dq_hip_quant(_ptr(px), px.size, _ptr(out), ctypes.byref(k), _ptr(ct), int(all_pixels_unique),
                          int(ngpus)) < 0:
        raise DivQuantError("dq_hip_quant: bad arguments")
    return out, ct[:k.value].copy()


def map_colors_mps(pixels, colortable):
    """map_colors_mps (DivQuant/DivQuantMapColors.cpp:243-539)."""
    _require_gpu()
    px = _u32(pixels).reshape(-1)
    ct = _u32(colortable).reshape(-1)
    if ct.size == 0:
        raise DivQuantError("colormapSize must be > 0")
    out = np.zeros(px.size, np.uint32)
    if lib().dq_hip_map(_ptr(px), px.size, _ptr(out), _ptr(ct), ct.size) < 0:
        raise DivQuantError("dq_hip_map failed")
    return out


def quant_varpart_fast(pixels, num_clusters, max_iters=10, device=0, all_pixels_unique=1, num_bits=8,
                       dec_factor=1, num_rows=1, num_cols=None):
    """quant_varpart_fast (DivQuantCluster.cpp:1099-1179): the non-empty
    cluster colours in cluster-index order (not deduplicated); uniform-weight
    path, or the weighted one for all_pixels_unique=0; num_bits < 8 /
    dec_factor > 1 take cut_bits and the decimated colour table over a
    num_rows x num_cols frame (:1139-1146)."""
    import torch
    _require_gpu()
    px = torch.from_numpy(_u32(pixels).reshape(-1).view(np.int32)).to(f"cuda:{device}")
    if num_bits != 8 or dec_factor != 1 or num_rows != 1 or (num_cols not in (None, px.numel())):
        ct = np.zeros(num_clusters, np.uint32)
        k = ctypes.c_uint32(num_clusters)
        rc = lib().dq_hip_varpart_dev(device, _dptr(px), px.numel(), num_rows,
                                      px.numel() if num_cols is None else num_cols, ctypes.byref(k), _ptr(ct),
                                      num_bits, dec_factor, max_iters, all_pixels_unique, None)
        if rc < 0:
            raise DivQuantError("dq_hip_varpart_dev: bad arguments (%d)" % rc)
        return ct[:k.value].copy()
    if all_pixels_unique:
        ct, _ = cluster_device(px, num_clusters, max_iters=max_iters, device=device)
        return ct
    ct = np.zeros(num_clusters, np.uint32)
    k = ctypes.c_uint32(num_clusters)
    if lib().dq_hip_quant_weighted_dev(device, _dptr(px), px.numel(), None, ctypes.byref(k), _ptr(ct),
                                       max_iters, None) < 0:
        raise DivQuantError("dq_hip_quant_weighted_dev: bad arguments")
    return ct[:k.value].copy()


# ---------------------------------------------------------------------------
# Device-resident entry points.  `t_in` / `t_out` are torch tensors (int32 or
# uint32 storage, contiguous, on cuda:device) or raw integer device pointers.
def _dptr(t):
    return ctypes.c_void_p(t if isinstance(t, int) else t.data_ptr())


def _nelem(t, n):
    return n if n is not None else t.numel()


def _stream_ptr(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)


def quant_device(t_in, t_out, num_clusters, max_iters=10, device=0, n=None, stream=None,
                 all_pixels_unique=1):
    """Cluster + dedup + map of device-resident pixels; returns (colortable, empty).
    all_pixels_unique=0: the weighted path (calc_color_table + ordered folds)."""
    n = _nelem(t_in, n)
    ct = np.zeros(num_clusters, np.uint32)
    k = ctypes.c_uint32(num_clusters)
    fn = lib().dq_hip_quant_dev if all_pixels_unique else lib().dq_hip_quant_weighted_dev
    r = fn(device, _dptr(t_in), n, _dptr(t_out), ctypes.byref(k), _ptr(ct), max_iters, _stream_ptr(stream))
    if r < 0:
        raise DivQuantError("dq_hip_quant_dev: bad arguments")
    return ct[:k.value].copy(), r


class WeightedRegions:
    """A set of device-resident regions for dq_hip_quant_weighted_regions_dev
    with its argument arrays built once (for repeated calls on the same
    buffers: the per-call marshalling of thousands of pointers is Python's
    cost, not the library's)."""

    def __init__(self, t_ins, t_outs, num_clusters):
        nr = len(t_ins)
        self.nr = nr
        self.ks = np.array(num_clusters if hasattr(num_clusters, "__len__") else [num_clusters] * nr, np.uint32)
        self.stride = int(self.ks.max()) if nr else 1
        self.ins = (ctypes.c_void_p * max(nr, 1))(*[_dptr(t).value for t in t_ins])
        self.outs = (ctypes.c_void_p * max(nr, 1))(*[_dptr(t).value for t in t_outs]) if t_outs is not None else None
        self.ns = np.array([t.numel() for t in t_ins], np.uint32)
        self.ct = np.zeros((max(nr, 1), self.stride), np.uint32)
        self.kout = np.zeros(max(nr, 1), np.uint32)
        self._refs = (t_ins, t_outs)   # (keep the buffers alive)

    def run(self, max_iters=10, device=0, stream=None):
        """One call over every region; returns the total of empty clusters
        (colortables: self.colortable(i))."""
        r = lib().dq_hip_quant_weighted_regions_dev(
            device, self.nr, ctypes.cast(self.ins, ctypes.c_void_p), _ptr(self.ns),
            ctypes.cast(self.outs, ctypes.c_void_p) if self.outs is not None else None,
            _ptr(self.ks), _ptr(self.ct), self.stride, _ptr(self.kout), max_iters, _stream_ptr(stream))
        if r < 0:
            raise DivQuantError("dq_hip_quant_weighted_regions_dev: bad arguments")
        return r

    def colortable(self, i):
        return self.ct[i, :self.kout[i]].copy()


def quant_weighted_regions_device(t_ins, t_outs, num_clusters, max_iters=10, device=0, stream=None):
    """The app's per-superpixel-region calls quant_recurse(N_region, .., K,
    allPixelsUnique=0) (ClusteringSegmentation.cpp:1779-1803) for many
    device-resident regions in one call (one launch for every region of at
    most 131071 pixels / 6144 colours / K <= 64).  num_clusters: one K or a
    list.  t_outs may be None (cluster + dedup only).  Returns ([colortable
    per region], total_empty)."""
    w = WeightedRegions(t_ins, t_outs, num_clusters)
    r = w.run(max_iters, device, stream)
    return [w.colortable(i) for i in range(w.nr)], r


def quant_batch_device(t_ins, t_outs, num_clusters, max_iters=10, device=0, stream=None):
    """quant_recurse over a batch of device-resident frames in one call (every
    pass of every split round is one launch over all frames).
    Returns ([colortable per frame], total_empty)."""
    nf = len(t_ins)
    ins = (ctypes.c_void_p * nf)(*[_dptr(t).value for t in t_ins])
    outs = (ctypes.c_void_p * nf)(*[_dptr(t).value for t in t_outs])
    ns = np.array([t.numel() for t in t_ins], np.uint32)
    ct = np.zeros((nf, num_clusters), np.uint32)
    kout = np.zeros(nf, np.uint32)
    r = lib().dq_hip_quant_batch_dev(device, nf, ctypes.cast(ins, ctypes.c_void_p),
                                     _ptr(ns), ctypes.cast(outs, ctypes.c_void_p), num_clusters,
                                     _ptr(ct), _ptr(kout), max_iters, _stream_ptr(stream))
    if r < 0:
        raise DivQuantError("dq_hip_quant_batch_dev: bad arguments")
    return [ct[i, :kout[i]].copy() for i in range(nf)], r


def quant_bgr24_batch_device(t_bgrs, width, height, t_outs, num_clusters, stride=None, max_iters=10,
                             device=0, stream=None, all_pixels_unique=1):
    """quant_recurse of device BGR24 frames (OpenCV CV_8UC3 rows), read
    directly by the root's passes, partition and map; outputs
    packed colours.  Returns ([colortable per frame], total_empty)."""
    nf = len(t_bgrs)
    stride = 3 * width if stride is None else stride
    ins = (ctypes.c_void_p * nf)(*[_dptr(t).value for t in t_bgrs])
    outs = (ctypes.c_void_p * nf)(*[_dptr(t).value for t in t_outs])
    ct = np.zeros((nf, num_clusters), np.uint32)
    kout = np.zeros(nf, np.uint32)
    r = lib().dq_hip_quant_bgr24_batch_dev(device, nf, ctypes.cast(ins, ctypes.c_void_p), width, height, stride,
                                           ctypes.cast(outs, ctypes.c_void_p), num_clusters, _ptr(ct), _ptr(kout),
                                           all_pixels_unique, max_iters, _stream_ptr(stream))
    if r < 0:
        raise DivQuantError("dq_hip_quant_bgr24_batch_dev: bad arguments")
    return [ct[i, :kout[i]].copy() for i in range(nf)], r


def quant_bgr24_device(t_bgr, width, height, t_out, num_clusters, stride=None, max_iters=10, device=0,
                       stream=None, all_pixels_unique=1):
    """quant_recurse of one device BGR24 frame; returns (colortable, empty)."""
    cts, r = quant_bgr24_batch_device([t_bgr], width, height, [t_out], num_clusters, stride, max_iters, device,
                                      stream, all_pixels_unique)
    return cts[0], r


def map_bgr24_device(t_bgr, width, height, t_out, colortable, stride=None, device=0, stream=None):
    """map_colors_mps of a device BGR24 frame into packed colours."""
    stride = 3 * width if stride is None else stride
    ct = _u32(colortable)
    if lib().dq_hip_map_bgr24_dev(device, _dptr(t_bgr), width, height, stride, _dptr(t_out), _ptr(ct), len(ct),
                                  _stream_ptr(stream)) < 0:
        raise DivQuantError("dq_hip_map_bgr24_dev: bad arguments")


def quant_rows_device(t_ins, t_outs, num_clusters, widths=None, n_globals=None, nshard=1,
                      max_iters=10, device=0, stream=None):
    """Row-tile sharded quant_recurse: t_ins[i] holds THIS
    process's rows of frame i.  nshard > 1 splits them into row ranges
    processed as separate shards on this GPU; n_globals[i] > numel means the
    other rows live in other processes, joined by the RCCL communicator of
    comm_init (every pass's integer node totals are allreduced).  Returns
    ([colortable per frame], total_empty) -- identical on every process."""
    nf = len(t_ins)
    ins = (ctypes.c_void_p * nf)(*[_dptr(t).value for t in t_ins])
    outs = None
    if t_outs is not None:
        outs = (ctypes.c_void_p * nf)(*[_dptr(t).value for t in t_outs])
    ns = np.array([t.numel() for t in t_ins], np.uint32)
    ws = np.array(widths if widths is not None else [0] * nf, np.uint32)
    ng = np.array(n_globals if n_globals is not None else [0] * nf, np.uint64)
    ct = np.zeros((nf, num_clusters), np.uint32)
    kout = np.zeros(nf, np.uint32)
    r = lib().dq_hip_quant_rows_dev(device, nf, ctypes.cast(ins, ctypes.c_void_p), _ptr(ns),
                                    _ptr(ws), _ptr(ng), nshard,
                                    ctypes.cast(outs, ctypes.c_void_p) if outs is not None else None,
                                    num_clusters, _ptr(ct), _ptr(kout), max_iters,
                                    _stream_ptr(stream))
    if r == -2:
        raise DivQuantError("dq_hip_quant_rows_dev: n_global > n needs comm_init first")
    if r < 0:
        raise DivQuantError("dq_hip_quant_rows_dev: bad arguments")
    return [ct[i, :kout[i]].copy() for i in range(nf)], r


def loopback_rows_device(t_ins, t_outs, width, height, num_clusters, nranks, max_iters=10, device=0,
                         log_cap=8192):
    """Test-only: row-tile sharding of `nranks` processes, run as nranks
    engines of this process on `device` (own stream and host thread each)
    joined by the in-process loopback collective instead of RCCL -- the
    TOT_ALLREDUCE path with every rank's local counts != the global totals.
    t_ins / t_outs: whole width x height frames; rank r maps its rows
    [r*H/N, (r+1)*H/N) into t_outs.  Returns (cts, logs, empty): cts[r][i] =
    rank r's colortable of frame i, logs[r] = the element counts of the
    collectives rank r enqueued, in order."""
    nf = len(t_ins)
    ins = (ctypes.c_void_p * nf)(*[_dptr(t).value for t in t_ins])
    outs = (ctypes.c_void_p * nf)(*[_dptr(t).value for t in t_outs])
    ct = np.zeros((nranks, nf, num_clusters), np.uint32)
    kout = np.zeros((nranks, nf), np.uint32)
    log = np.zeros((nranks, log_cap), np.uint64)
    nlog = np.zeros(nranks, np.int32)
    r = lib().dq_hip_loopback_rows_dev(device, nranks, nf, ctypes.cast(ins, ctypes.c_void_p), width, height,
                                       ctypes.cast(outs, ctypes.c_void_p), num_clusters, _ptr(ct), _ptr(kout),
                                       max_iters, _ptr(log), log_cap, _ptr(nlog))
    if r < 0:
        raise DivQuantError("dq_hip_loopback_rows_dev: bad arguments")
    if nlog.max() > log_cap:
        raise DivQuantError("collective log longer than log_cap")
    cts = [[ct[q, i, :kout[q, i]].copy() for i in range(nf)] for q in range(nranks)]
    logs = [log[q, :nlog[q]].tolist() for q in range(nranks)]
    return cts, logs, r


def comm_unique_id():
    """128-byte RCCL id (rank 0 creates it; broadcast it to the other ranks)."""
    buf = ctypes.create_string_buffer(128)
    if lib().dq_hip_comm_unique_id(buf) != 0:
        raise DivQuantError("dq_hip_comm_unique_id failed")
    return buf.raw


def comm_init(nranks, rank, uid, device=0):
    """Join the engine on `device` to an RCCL communicator (one process per GPU)."""
    buf = ctypes.create_string_buffer(bytes(uid), 128)
    if lib().dq_hip_comm_init(device, nranks, rank, buf) != 0:
        raise DivQuantError("dq_hip_comm_init: bad arguments")


def comm_destroy(device=0):
    lib().dq_hip_comm_destroy(device)


def comm_size(device=0):
    """Ranks of the engine's RCCL communicator on `device` (1: none)."""
    return lib().dq_hip_comm_size(device)


def comm_init_torch(device=0, group=None):
    """comm_init over an initialised torch.distributed process group: rank 0's
    id is broadcast with the group (any backend), then every rank joins."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    obj = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    comm_init(world, rank, obj[0], device=device)


def cluster_device(t_in, num_clusters, max_iters=10, device=0, n=None, stream=None):
    """DivQuantCluster on device-resident pixels; returns (colortable, empty)."""
    n = _nelem(t_in, n)
    ct = np.zeros(num_clusters, np.uint32)
    k = ctypes.c_uint32(num_clusters)
    r = lib().dq_hip_cluster_dev(device, _dptr(t_in), n, ctypes.byref(k), _ptr(ct), max_iters,
                                 _stream_ptr(stream))
    if r < 0:
        raise DivQuantError("dq_hip_cluster_dev: bad arguments")
    return ct[:k.value].copy(), r


def map_device(t_in, t_out, colortable, device=0, n=None, stream=None):
    n = _nelem(t_in, n)
    ct = _u32(colortable).reshape(-1)
    if lib().dq_hip_map_dev(device, _dptr(t_in), n, _dptr(t_out), _ptr(ct), ct.size,
                            _stream_ptr(stream)) < 0:
        raise DivQuantError("dq_hip_map_dev: bad arguments")


# ---------------------------------------------------------------------------
# BGR24 frames.  `t_bgr`: uint8 device tensor (or pointer)
# holding a CV_8UC3 frame, `stride` bytes per row (default 3 * width).
def pack_bgr24_device(t_bgr, width, height, t_out, stride=None, device=0, stream=None):
    """t_out[y*width+x] = Vec3BToUID(img(y, x)) (OpenCVUtil.h:19-27), asynchronous."""
    stride = 3 * width if stride is None else stride
    if lib().dq_hip_pack_bgr24_dev(device, _dptr(t_bgr), width, height, stride, _dptr(t_out),
                                   _stream_ptr(stream)) < 0:
        raise DivQuantError("dq_hip_pack_bgr24_dev: bad arguments")


def unpack_bgr24_device(t_in, width, height, t_bgr, stride=None, device=0, stream=None):
    """img(y, x) = PixelToVec3b(t_in[y*width+x]) (OpenCVUtil.h:53-59), asynchronous."""
    stride = 3 * width if stride is None else stride
    if lib().dq_hip_unpack_bgr24_dev(device, _dptr(t_in), width, height, stride, _dptr(t_bgr),
                                     _stream_ptr(stream)) < 0:
        raise DivQuantError("dq_hip_unpack_bgr24_dev: bad arguments")


def gather_bgr24_device(t_bgr, stride, t_coords, n, t_out, device=0, stream=None):
    """t_out[i] = Vec3BToUID(img(c.y, c.x)) for Coord words c = x | y << 16
    (Coord.h:30-33; ClusteringSegmentation.cpp:1795-1800), asynchronous."""
    if lib().dq_hip_gather_bgr24_dev(device, _dptr(t_bgr), stride, _dptr(t_coords), n,
                                     _dptr(t_out), _stream_ptr(stream)) < 0:
        raise DivQuantError("dq_hip_gather_bgr24_dev: bad arguments")


# ---------------------------------------------------------------------------
# Synthetic benchmark frames and the fixtures' output checksum (host code).
SYNTH_SEED = 0x9E3779B97F4A7C15


def synth_frame(n, frame=0, seed=SYNTH_SEED):
    """Frame `frame` of the benchmark batch: n xorshift64 draws
    & 0xFFFFFF from seed + frame."""
    out = np.empty(n, np.uint32)
    lib().dq_synth_xorshift(_ptr(out), n, (seed + frame) & 0xFFFFFFFFFFFFFFFF)
    return out


def fnv1a64(a):
    """Word-wise FNV-1a-64 of a uint32 array (the golden fixtures' out_fnv)."""
    a = _u32(a).reshape(-1)
    return int(lib().dq_fnv1a64(_ptr(a), a.size))


# ---------------------------------------------------------------------------
# Full-frame fixed-palette map + per-block mode.
def get_subdivided_colors():
    """getSubdividedColors (superpixels/OpenCVUtil.cpp:853-897): the 125
    colours 0xFFRRGGBB of the {0,63,127,191,255}^3 cube (no GPU needed)."""
    out = np.zeros(125, np.uint32)
    lib().dq_subdivided_colors(_ptr(out))
    return out


def block_grid(width, height, superpixel_dim=4):
    """(blockWidth, blockHeight) as clusteringCombine computes them
    (ClusteringSegmentationMain.cpp:138-149): ceil(W/dim), ceil(H/dim)."""
    return -(-width // superpixel_dim), -(-height // superpixel_dim)


def gen_histograms_for_blocks(frame, superpixel_dim=4, palette=None, tables=False):
    """genHistogramsForBlocks (ClusteringSegmentation.cpp:365-576) on a frame of
    0x00RRGGBB words shaped (H, W) (the Vec3BToUID packing of the BGR Mat).

    Returns (block_bgr, region_quant_pixel, quant[, (ndistinct, keys, counts)]):
    block_bgr (bh, bw, 3) uint8 is the returned blockMat (B, G, R bytes);
    region_quant_pixel (bh, bw) uint32 is each block's HistogramForBlock::
    regionQuantPixel; quant (H, W) the map_colors_mps output.  With tables=True
    also each block's pixelToCountTable in iteration order: ndistinct (bh, bw)
    and keys/counts (bh, bw, dim*dim), zero past ndistinct."""
    _require_gpu()
    fr = _u32(frame)
    if fr.ndim != 2 or fr.size == 0:
        raise DivQuantError("frame must be a non-empty (H, W) array")
    h, w = fr.shape
    bw, bh = block_grid(w, h, superpixel_dim)
    pal = get_subdivided_colors() if palette is None else _u32(palette).reshape(-1)
    quant = np.zeros((h, w), np.uint32)
    mode = np.zeros((bh, bw), np.uint32)
    cap = superpixel_dim * superpixel_dim
    nd = np.zeros((bh, bw), np.uint32) if tables else None
    keys = np.zeros((bh, bw, cap), np.uint32) if tables else None
    counts = np.zeros((bh, bw, cap), np.uint32) if tables else None
    none = ctypes.c_void_p(0)
    rc = lib().dq_hip_block_hist(_ptr(fr), w, h, _ptr(pal), pal.size, superpixel_dim, bw, bh,
                                 _ptr(quant), _ptr(mode), _ptr(nd) if tables else none,
                                 _ptr(keys) if tables else none, _ptr(counts) if tables else none)
    if rc < 0:
        raise DivQuantError("dq_hip_block_hist: bad arguments")
    bgr = np.stack([mode & 0xFF, (mode >> 8) & 0xFF, (mode >> 16) & 0xFF], axis=-1).astype(np.uint8)
    if tables:
        return bgr, mode, quant, (nd, keys, counts)
    return bgr, mode, quant


def block_hist_device(t_in, width, height, t_quant, t_mode, palette=None, superpixel_dim=4,
                      t_ndistinct=None, t_keys=None, t_counts=None, device=0, stream=None):
    """dq_hip_block_hist_dev on torch tensors / device pointers (asynchronous)."""
    pal = get_subdivided_colors() if palette is None else _u32(palette).reshape(-1)
    bw, bh = block_grid(width, height, superpixel_dim)
    opt = lambda t: _dptr(t) if t is not None else ctypes.c_void_p(0)  # noqa: E731
    if lib().dq_hip_block_hist_dev(device, _dptr(t_in), width, height, _ptr(pal), pal.size,
                                   superpixel_dim, bw, bh, _dptr(t_quant), _dptr(t_mode),
                                   opt(t_ndistinct), opt(t_keys), opt(t_counts),
                                   _stream_ptr(stream)) < 0:
        raise DivQuantError("dq_hip_block_hist_dev: bad arguments")


def last_centroids(k, device=0):
    """(means[k,3] float64, sizes[k] int64) of the last clustering on `device`."""
    means = np.zeros((k, 3), np.float64)
    sizes = np.zeros(k, np.int64)
    if lib().dq_hip_last_centroids(device, _ptr(means), _ptr(sizes), k) < 0:
        raise DivQuantError("k does not match the last clustering")
    return means, sizes


def last_trace(k, device=0):
    tr = np.zeros((max(k - 1, 0), 4), np.int64)
    if lib().dq_hip_last_trace(device, _ptr(tr) if tr.size else None, k) < 0:
        raise DivQuantError("k does not match the last clustering")
    return tr


def last_rounds(device=0):
    return lib().dq_hip_last_rounds(device)


def last_points_swept(device=0):
    return int(lib().dq_hip_last_points_swept(device))


def last_points_full(device=0):
    """Points the last run would have swept with all max_iters iterations."""
    return int(lib().dq_hip_last_points_full(device))


def last_seq_tiles(device=0):
    """Weighted path: tiles of the last run folded one summand at a time."""
    return int(lib().dq_hip_last_seq_tiles(device))


def last_cursor_fixes(device=0):
    """Records of the last run partitioned after a frame's last planned round
    (PS_STATS: no cursors counted there) whose cursors were counted then."""
    return int(lib().dq_hip_last_cursor_fixes(device))


def set_fixed_point(on, device=0):
    """Fixed-point finalisation of 2-means splits (identical outputs)."""
    lib().dq_hip_set_fixed_point(device, 1 if on else 0)


def set_planned_rounds(on, device=0):
    """Device-planned (speculative) rounds (identical outputs)."""
    lib().dq_hip_set_planned_rounds(device, 1 if on else 0)


def last_planned_rounds(device=0):
    return lib().dq_hip_last_planned_rounds(device)


def set_loop_max(max_points, device=0):
    """kloop_kernel eligibility: records of at most max_points points (0: off)."""
    lib().dq_hip_set_loop_max(device, int(max_points))


def last_loop_rounds(device=0):
    return lib().dq_hip_last_loop_rounds(device)


def set_persist(on, device=0):
    """kpersist_kernel rounds on / off (every lane of the device)."""
    lib().dq_hip_set_persist(device, 1 if on else 0)


def set_wsmall(on, device=0):
    """The one-launch weighted path for small inputs on / off (every lane)."""
    lib().dq_hip_set_wsmall(device, 1 if on else 0)


def last_wsmall_profile(device=0):
    """The last weighted call's one-launch phase profile in microseconds
    (hash set, colour table, clustering, map, of which fold passes and
    partitions) and its passes by kind; {} if it did not take that path."""
    buf = np.zeros(8, np.uint64)
    if lib().dq_hip_last_wsmall_profile(device, buf.ctypes.data_as(ctypes.c_void_p), 8) < 8:
        return {}
    t = [float(v) / 100.0 for v in buf[:7]]   # 100 MHz ticks -> us
    k = int(buf[7])
    return {"hash_us": t[1] - t[0], "table_us": t[2] - t[1], "cluster_us": t[3] - t[2], "map_us": t[4] - t[3],
            "passes_us": t[5], "partitions_us": t[6],
            "passes": {"init": k & 0xFFFF, "split": (k >> 16) & 0xFFFF, "kmeans": (k >> 32) & 0xFFFF}}


def last_persist_rounds(device=0):
    return lib().dq_hip_last_persist_rounds(device)


def set_lanes(lanes):
    """Engine lanes a batch is split over (0: default, DQ_HIP_LANES, else 4 with
    GPU_MAX_HW_QUEUES >= 6, else 3)."""
    lib().dq_hip_set_lanes(int(lanes))


def get_lanes():
    return lib().dq_hip_get_lanes()


def build_id():
    """FNV-1a-64 of the sources the loaded library was built from (tools/source_id.py)."""
    return int(lib().dq_hip_build_id())


def set_debug(flags, device=0):
    """Test-only interleaving knobs (dq_hip.h dq_hip_set_debug; 0 in production):
    1 prewarm the 2-means hand-off lines, 2 uneven workgroup stalls, 4 host
    delays between a round's status and its results, 8 plan-kernel stall,
    16 check that the round arena is all zero when a run starts, 32 release the
    round arena at every run's start (its rounds allocate new chunks)."""
    lib().dq_hip_set_debug(device, int(flags))


def set_timing(on, device=0):
    lib().dq_hip_set_timing(device, 1 if on else 0)


def reset_stats(device=0):
    lib().dq_hip_reset_stats(device)


def get_stats(device=0):
    """{kind: (launches, total_ms, engine-model bytes, points)} from HIP events on the launch stream."""
    res = {}
    for i, name in enumerate(STAT_KINDS):
        l, ms, b, u = ctypes.c_uint64(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        lib().dq_hip_get_stat(device, i, ctypes.byref(l), ctypes.byref(ms), ctypes.byref(b))
        lib().dq_hip_get_stat_units(device, i, ctypes.byref(u))
        res[name] = (int(l.value), float(ms.value), float(b.value), float(u.value))
    return res
