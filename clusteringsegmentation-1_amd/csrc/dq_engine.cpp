// dq_engine.cpp -- host side of the DivQuant hot path (see dq_engine.h).
#include "dq_engine.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <unordered_set>

namespace dq {

void die(const char* what, const char* file, int line, const char* detail) {
  std::fprintf(stderr, "divquant-hip: fatal: %s (%s:%d): %s\n", what, file, line,
               detail ? detail : "");
  std::fflush(stderr);
  std::abort();
}

namespace {

constexpr int BUF_IN = 0, BUF_P0 = 1, BUF_P1 = 2;
inline int child_buf(int b) { return b == BUF_P0 ? BUF_P1 : BUF_P0; }
inline size_t align4(size_t x) { return (x + 3) & ~(size_t)3; }

// Split-pass threshold (:473): cut_pos < v <=> v >= thr for integer v.
int32_t split_threshold(double cut) {
  if (!(cut == cut)) return 256;
  if (cut < 0.0) return 0;
  if (cut >= 255.0) return 256;
  return (int32_t)std::floor(cut) + 1;
}

}  // namespace

Engine::Engine(int device) : device_(device) {
  const char* full = getenv("DQ_HIP_FULL_ITERS");
  fixed_point_ = !(full && full[0] == '1');
  DQ_HIP(hipSetDevice(device_));
  DQ_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  DQ_HIP(hipMalloc((void**)&d_pal_, 16384 * sizeof(uint32_t)));
  DQ_HIP(hipMalloc((void**)&d_lut_, 768 * sizeof(uint16_t)));
  DQ_HIP(hipMalloc((void**)&d_cell_rec_, (size_t)kCells * kCellRecWords * sizeof(uint32_t)));
  DQ_HIP(hipMalloc((void**)&d_cell_idx_, (size_t)kCells * kCellCap * sizeof(uint16_t)));
  DQ_HIP(hipHostMalloc((void**)&h_pal_, 16384 * sizeof(uint32_t), hipHostMallocDefault));
  DQ_HIP(hipHostMalloc((void**)&h_lut_, 768 * sizeof(uint16_t), hipHostMallocDefault));
}

Engine::~Engine() {
  // Process-lifetime object; the runtime may already be torn down at exit,
  // so release nothing here (the driver reclaims device memory).
}

// ---------------------------------------------------------------------------
// timing
hipEvent_t Engine::take_event() {
  if (!event_pool_.empty()) {
    hipEvent_t e = event_pool_.back();
    event_pool_.pop_back();
    return e;
  }
  hipEvent_t e;
  DQ_HIP(hipEventCreate(&e));
  return e;
}

void Engine::timed_begin(hipStream_t stream) {
  if (!timing_) return;
  PendingEvent pe{take_event(), nullptr, -1, 0.0};
  DQ_HIP(hipEventRecord(pe.a, stream));
  pending_.push_back(pe);
}

void Engine::timed_end(int kind, double bytes, hipStream_t stream) {
  if (!timing_) return;
  PendingEvent& pe = pending_.back();
  pe.b = take_event();
  pe.kind = kind;
  pe.bytes = bytes;
  DQ_HIP(hipEventRecord(pe.b, stream));
}

void Engine::collect_timing() {
  for (auto& pe : pending_) {
    float ms = 0.f;
    DQ_HIP(hipEventSynchronize(pe.b));
    DQ_HIP(hipEventElapsedTime(&ms, pe.a, pe.b));
    KernelStat& st = stats[pe.kind];
    st.launches++;
    st.ms += ms;
    st.bytes += pe.bytes;
    event_pool_.push_back(pe.a);
    event_pool_.push_back(pe.b);
  }
  pending_.clear();
}

void Engine::reset_stats() {
  for (auto& s : stats) s = KernelStat();
}

// ---------------------------------------------------------------------------
// buffers
void Engine::ensure_pixels(size_t total) {
  if (total > cap_px_ || !d_p0_) {
    if (d_p0_) DQ_HIP(hipFree(d_p0_));
    if (d_p1_) DQ_HIP(hipFree(d_p1_));
    DQ_HIP(hipMalloc((void**)&d_p0_, total * sizeof(uint32_t)));
    DQ_HIP(hipMalloc((void**)&d_p1_, total * sizeof(uint32_t)));
    cap_px_ = total;
  }
}

void Engine::stage_in(const uint32_t* h_in, uint32_t n, hipStream_t stream) {
  const size_t want = align4((size_t)n) + 4;
  if (want > cap_stage_ || !d_stage_in_) {
    if (d_stage_in_) DQ_HIP(hipFree(d_stage_in_));
    if (d_stage_out_) DQ_HIP(hipFree(d_stage_out_));
    DQ_HIP(hipMalloc((void**)&d_stage_in_, want * sizeof(uint32_t)));
    DQ_HIP(hipMalloc((void**)&d_stage_out_, want * sizeof(uint32_t)));
    cap_stage_ = want;
  }
  DQ_HIP(hipMemcpyAsync(d_stage_in_, h_in, (size_t)n * sizeof(uint32_t),
                        hipMemcpyHostToDevice, stream));
}

void Engine::ensure_round(size_t nnodes, size_t ntiles) {
  if (nnodes > cap_nodes_ || !d_nodes_) {
    size_t c = std::max<size_t>(nnodes, 256);
    if (d_nodes_) DQ_HIP(hipFree(d_nodes_));
    if (h_nodes_) DQ_HIP(hipHostFree(h_nodes_));
    DQ_HIP(hipMalloc((void**)&d_nodes_, c * sizeof(DevNode)));
    DQ_HIP(hipHostMalloc((void**)&h_nodes_, c * sizeof(DevNode), hipHostMallocDefault));
    cap_nodes_ = c;
  }
  if (ntiles > cap_tiles_ || !d_tiles_) {
    size_t c = std::max<size_t>(ntiles, 4096);
    if (d_tiles_) DQ_HIP(hipFree(d_tiles_));
    if (d_parts_) DQ_HIP(hipFree(d_parts_));
    if (h_tiles_) DQ_HIP(hipHostFree(h_tiles_));
    DQ_HIP(hipMalloc((void**)&d_tiles_, c * sizeof(Tile)));
    DQ_HIP(hipMalloc((void**)&d_parts_, c * sizeof(TilePartial)));
    DQ_HIP(hipHostMalloc((void**)&h_tiles_, c * sizeof(Tile), hipHostMallocDefault));
    cap_tiles_ = c;
  }
}

const uint32_t* Engine::buf_ptr(int buf, const FrameState& f) const {
  if (buf == BUF_IN) return f.in;
  return (buf == BUF_P0 ? d_p0_ : d_p1_) + f.base;
}

// ---------------------------------------------------------------------------
// One round: split every node in `active` (one launch per pass for all).
void Engine::run_round(const std::vector<int>& active, bool root_round, int max_iters,
                       hipStream_t stream) {
  const int nn = (int)active.size();
  uint64_t total = 0;
  for (int id : active) total += nodes_[id].len;
  // Tile length: whole 4096-point sweeps, ~1024 tiles for big rounds (4 per
  // CU: measured best for one 4K frame and for 8-frame batches, microbench).
  uint64_t tl = (total + 1023) / 1024;
  tl = ((tl + kSweep - 1) / kSweep) * kSweep;
  tl = std::max<uint64_t>(kSweep, std::min<uint64_t>(tl, kMaxTilePx));
  size_t ntiles = 0;
  for (int id : active)   // empty nodes get one empty tile (their epilogue still runs)
    ntiles += std::max<size_t>(1, (nodes_[id].len + tl - 1) / tl);
  ensure_round(nn, ntiles);

  int t = 0;
  for (int a = 0; a < nn; ++a) {
    const Node& n = nodes_[active[a]];
    const FrameState& fs = frames_[n.frame];
    DevNode& d = h_nodes_[a];
    std::memset(&d, 0, sizeof(d));
    d.src = buf_ptr(n.buf, fs);
    d.dst = (child_buf(n.buf) == BUF_P0 ? d_p0_ : d_p1_) + fs.base;
    d.off = n.off;
    d.len = n.len;
    d.s = fs.s;
    d.tw = n.w;
    for (int c = 0; c < 3; ++c) { d.tm[c] = n.mean[c]; d.tv[c] = n.var[c]; }
    if (!root_round) {
      // Cut axis/position (:388-403): comparisons and copies only.  (The
      // root's come from its PASS_INIT epilogue on the device.)
      double maxv = n.var[0], cut = n.mean[0];
      int axis = 0;
      if (maxv < n.var[1]) { maxv = n.var[1]; axis = 1; cut = n.mean[1]; }
      if (maxv < n.var[2]) { axis = 2; cut = n.mean[2]; }
      d.prm.thr = split_threshold(cut);
      d.prm.shift = 16 - 8 * axis;
    }
    d.tile_begin = t;
    for (uint64_t o = 0; o == 0 || o < n.len; o += tl) {
      Tile& tt = h_tiles_[t++];
      tt.node = a;
      tt.start = n.off + (uint32_t)o;
      tt.end = n.off + (uint32_t)std::min<uint64_t>(n.len, o + tl);
      tt.old_base = 0;
    }
    d.tile_end = t;
  }
  DQ_HIP(hipMemcpyAsync(d_nodes_, h_nodes_, nn * sizeof(DevNode), hipMemcpyHostToDevice, stream));
  DQ_HIP(hipMemcpyAsync(d_tiles_, h_tiles_, ntiles * sizeof(Tile), hipMemcpyHostToDevice, stream));

  RoundArgs ra;
  ra.tiles = d_tiles_;
  ra.nodes = d_nodes_;
  ra.parts = d_parts_;
  ra.fixed_point = fixed_point_ ? 1 : 0;
  const double bytes = 4.0 * (double)total;
  const int nt = (int)ntiles;
  // 2-means passes (iteration index) whose timing entry gets its swept bytes
  // once the nodes' done_it are known
  std::vector<std::pair<size_t, int>> km_events;
  auto pass = [&](int kind, int st, int it) {
    timed_begin(stream);
    launch_pass(kind, ra, nt, stream);
    timed_end(st, bytes, stream);
    if (timing_ && it >= 0) km_events.push_back({pending_.size() - 1, it});
    timed_begin(stream);
    launch_epilogue(kind, ra, nn, stream);
    timed_end(ST_EPILOGUE, 0.0, stream);
  };
  if (root_round) pass(PASS_INIT, ST_INIT, -1);
  pass(PASS_SPLIT, ST_SPLIT, -1);
  for (int it = 0; it < max_iters; ++it) {
    const bool last = (it == max_iters - 1);
    pass(last ? PASS_KLAST : PASS_KMEANS, last ? ST_KLAST : ST_KMEANS, it);
  }
  timed_begin(stream);
  launch_partition(ra, nt, stream);
  timed_end(ST_PARTITION, 2.0 * bytes, stream);

  DQ_HIP(hipMemcpyAsync(h_nodes_, d_nodes_, nn * sizeof(DevNode), hipMemcpyDeviceToHost, stream));
  DQ_HIP(hipStreamSynchronize(stream));
  // points actually swept: iteration `it` reads a node iff it is not final
  // before it (done_it == 0, or it < done_it)
  auto swept_in = [&](int it) {
    uint64_t px = 0;
    for (int a = 0; a < nn; ++a) {
      const DevNode& d = h_nodes_[a];
      if (d.done_it == 0 || it < d.done_it) px += d.len;
    }
    return px;
  };
  last_points_full += total * (uint64_t)((root_round ? 2 : 1) + max_iters);
  last_points_swept += total * (uint64_t)(root_round ? 2 : 1);
  for (int it = 0; it < max_iters; ++it) last_points_swept += swept_in(it);
  for (auto& e : km_events) pending_[e.first].bytes = 4.0 * (double)swept_in(e.second);
  collect_timing();

  for (int a = 0; a < nn; ++a) {
    const int id = active[a];
    const DevNode& d = h_nodes_[a];
    if (root_round) {
      for (int c = 0; c < 3; ++c) { nodes_[id].mean[c] = d.tm[c]; nodes_[id].var[c] = d.tv[c]; }
    }
    const Node& p = nodes_[id];
    const uint32_t n_new = (uint32_t)d.n_new;
    const uint32_t n_old = p.len - n_new;
    Node co, cn;
    co.frame = cn.frame = p.frame;
    co.w = d.ow;
    cn.w = d.nw;
    for (int c = 0; c < 3; ++c) {
      co.mean[c] = d.om[c];
      cn.mean[c] = d.nm[c];
      co.var[c] = d.ov[c];
      cn.var[c] = d.nv[c];
    }
    co.tse = d.tse_old;
    cn.tse = d.tse_new;
    co.off = p.off;
    co.len = n_old;
    cn.off = p.off + n_old;
    cn.len = n_new;
    co.buf = cn.buf = child_buf(p.buf);
    const int io = (int)nodes_.size();
    nodes_.push_back(co);
    nodes_.push_back(cn);
    Node& pp = nodes_[id];
    pp.child_old = io;
    pp.child_new = io + 1;
    pp.expanded = true;
  }
}

// ---------------------------------------------------------------------------
// Replay the reference's greedy order (:346-892) as far as the expanded tree
// allows; f.need = the unexpanded node it stopped at (-1 when all K-1 splits
// are known).
void Engine::replay(FrameState& f) {
  const int k = f.job->k;
  f.need = -1;
  while (f.new_index < k) {
    const int x = f.leaf[f.old_index];
    if (!nodes_[x].expanded) { f.need = x; return; }
    const int co = nodes_[x].child_old, cn = nodes_[x].child_new;
    f.trace.push_back(f.new_index);
    f.trace.push_back(f.old_index);
    f.trace.push_back(nodes_[x].len);
    f.trace.push_back(nodes_[cn].len);
    f.leaf[f.old_index] = co;
    f.leaf[f.new_index] = cn;
    if (f.new_index == k - 1) { ++f.new_index; return; }     // :823-832
    // STEP 4 (:876-887): max TSE above DBL_MIN, lowest index among equals;
    // if none qualifies old_index stays (the old half is split again).
    if (nodes_[co].tse > DBL_MIN) f.heap.push({{nodes_[co].tse, -f.old_index}, co});
    if (nodes_[cn].tse > DBL_MIN) f.heap.push({{nodes_[cn].tse, -f.new_index}, cn});
    while (!f.heap.empty() && f.leaf[-f.heap.top().first.second] != f.heap.top().second)
      f.heap.pop();
    if (!f.heap.empty()) f.old_index = -f.heap.top().first.second;
    ++f.new_index;
  }
}

// Next round's nodes of a frame: the node the replay waits for plus every
// unexpanded leaf among the top r = (splits left) of the greedy order -- a
// leaf outside the current top r can never be picked in the remaining splits.
void Engine::next_active(FrameState& f, std::vector<int>* active) {
  if (f.need < 0) return;
  const int r = f.job->k - f.new_index;
  active->push_back(f.need);
  auto h = f.heap;
  int taken = 0;
  while (!h.empty() && taken < r) {
    const auto top = h.top();
    h.pop();
    const int idx = -top.first.second, node = top.second;
    if (f.leaf[idx] != node) continue;
    ++taken;
    if (!nodes_[node].expanded && node != f.need) active->push_back(node);
  }
}

// Final centres (:1029-1094): round, pack, drop empty clusters.
void Engine::finish_frame(FrameState& f, bool last) {
  FrameJob& job = *f.job;
  const int k = job.k;
  int out = 0, empty = 0;
  if (last) {
    last_means.assign((size_t)k * 3, 0.0);
    last_sizes.assign(k, 0);
    last_trace = f.trace;
  }
  if (k == 1) {
    // No split happens: mean[0] keeps its zero initialisation (:309).
    job.ct[out++] = 0;
    if (last) last_sizes[0] = job.n;
  } else {
    for (int ic = 0; ic < k; ++ic) {
      const Node& nd = nodes_[f.leaf[ic]];
      if (last) {
        for (int c = 0; c < 3; ++c) last_means[3 * ic + c] = nd.mean[c];
        last_sizes[ic] = nd.len;
      }
      if (nd.len > 0) {
        const uint32_t R = (uint8_t)(nd.mean[0] + 0.5);
        const uint32_t G = (uint8_t)(nd.mean[1] + 0.5);
        const uint32_t B = (uint8_t)(nd.mean[2] + 0.5);
        job.ct[out++] = (R << 16) | (G << 8) | B;
      } else {
        ++empty;
      }
    }
  }
  job.k_out = out;
  job.num_empty = empty;
}

void Engine::run(FrameJob* jobs, int nframes, int max_iters, bool dedup_map,
                 hipStream_t stream) {
  DQ_CHECK(nframes > 0, "empty batch");
  DQ_CHECK(max_iters >= 1, "max_iters < 1 is not supported (the reference never writes member[] then)");
  DQ_HIP(hipSetDevice(device_));
  if (!stream) stream = stream_;

  frames_.assign(nframes, FrameState());
  nodes_.clear();
  last_rounds = 0;
  last_points_swept = 0;
  last_points_full = 0;
  size_t total = 0, align_need = 0;
  for (int i = 0; i < nframes; ++i) {
    FrameJob& j = jobs[i];
    DQ_CHECK(j.n > 0, "num_points must be > 0 (DivQuantCluster.cpp:211)");
    DQ_CHECK(j.k > 0, "num_colors must be > 0 (DivQuantCluster.cpp:229)");
    DQ_CHECK(j.d_in && j.ct, "null buffer");
    frames_[i].job = &j;
    frames_[i].base = (uint32_t)total;
    total += align4(j.n) + 4;
    if (((uintptr_t)j.d_in & 15) != 0 || (j.n & 3) != 0) align_need += align4(j.n) + 4;
  }
  DQ_CHECK(total < (1ull << 32), "batch larger than 2^32 points");
  ensure_pixels(total);
  if (align_need > cap_align_) {
    if (d_align_) DQ_HIP(hipFree(d_align_));
    DQ_HIP(hipMalloc((void**)&d_align_, align_need * sizeof(uint32_t)));
    cap_align_ = align_need;
  }
  size_t aoff = 0;
  std::vector<int> active;
  for (int i = 0; i < nframes; ++i) {
    FrameState& f = frames_[i];
    FrameJob& j = *f.job;
    // get_double_scale (DivQuantMapColors.cpp:205-220)
    f.s = 1.0 / (std::ceil(1 / 1.0) * std::ceil(j.n / 1.0));
    f.in = j.d_in;
    if (((uintptr_t)j.d_in & 15) != 0 || (j.n & 3) != 0) {   // 16-B loads may read up to align4(n)
      DQ_HIP(hipMemcpyAsync(d_align_ + aoff, j.d_in, (size_t)j.n * 4, hipMemcpyDeviceToDevice, stream));
      f.in = d_align_ + aoff;
      aoff += align4(j.n) + 4;
    }
    Node root;
    root.frame = i;
    root.w = 1.0;          // :329
    root.len = j.n;
    root.buf = BUF_IN;
    f.leaf.assign(j.k, -1);
    f.leaf[0] = (int)nodes_.size();
    nodes_.push_back(root);
    if (j.k > 1) active.push_back(f.leaf[0]);
  }

  bool root_round = true;
  while (!active.empty()) {
    run_round(active, root_round, max_iters, stream);
    root_round = false;
    last_rounds++;
    active.clear();
    for (auto& f : frames_) {
      if (f.job->k <= 1 || (f.need < 0 && f.new_index >= f.job->k)) continue;
      replay(f);
      next_active(f, &active);
    }
  }

  for (int i = 0; i < nframes; ++i) finish_frame(frames_[i], i == nframes - 1);

  if (dedup_map) {
    for (auto& f : frames_) {
      FrameJob& j = *f.job;
      // First-occurrence colortable dedup (quant_util.cpp:93-118).
      std::unordered_set<uint32_t> seen;
      int m = 0;
      for (int i = 0; i < j.k_out; ++i)
        if (seen.insert(j.ct[i]).second) j.ct[m++] = j.ct[i];
      j.k_out = m;
      if (j.d_out) map(f.in, j.n, j.d_out, j.ct, m, stream);
    }
  }
}

// ---------------------------------------------------------------------------
void Engine::map(const uint32_t* d_in, uint32_t n, uint32_t* d_out,
                 const uint32_t* ct, int k, hipStream_t stream) {
  DQ_CHECK(k > 0, "colormapSize must be > 0 (DivQuantMapColors.cpp:264)");
  DQ_CHECK(k <= 16384, "colormapSize > 16384 is not supported by the LDS palette");
  DQ_HIP(hipSetDevice(device_));
  if (!stream) stream = stream_;
  if (((uintptr_t)d_in & 15) != 0 || ((uintptr_t)d_out & 15) != 0) {
    // the map kernel uses 16-B loads/stores: go through aligned staging
    const size_t want = align4(n) + 4;
    if (2 * want > cap_map_align_) {
      if (d_map_align_) DQ_HIP(hipFree(d_map_align_));
      DQ_HIP(hipMalloc((void**)&d_map_align_, want * 2 * sizeof(uint32_t)));
      cap_map_align_ = want * 2;
    }
    uint32_t* ain = d_map_align_;
    uint32_t* aout = d_map_align_ + want;
    DQ_HIP(hipMemcpyAsync(ain, d_in, (size_t)n * 4, hipMemcpyDeviceToDevice, stream));
    map(ain, n, aout, ct, k, stream);
    DQ_HIP(hipMemcpyAsync(d_out, aout, (size_t)n * 4, hipMemcpyDeviceToDevice, stream));
    DQ_HIP(hipStreamSynchronize(stream));
    return;
  }
  // Palette sorted by R+G+B with std::sort and the reference comparator
  // (:227-238, :314-323) -- same algorithm, same input => same tie order.
  struct Ent { int red, green, blue, weight; };
  std::vector<Ent> pal(k);
  for (int i = 0; i < k; ++i) {
    const uint32_t p = ct[i];
    pal[i].blue = p & 0xFF;
    pal[i].green = (p >> 8) & 0xFF;
    pal[i].red = (p >> 16) & 0xFF;
    pal[i].weight = pal[i].red + pal[i].green + pal[i].blue;
  }
  std::sort(pal.begin(), pal.end(),
            [](const Ent& a, const Ent& b) { return a.weight < b.weight; });
  // Start-entry LUT from rounded midpoints (:331-383).
  int lut[766];
  const int low = k >= 2 ? (int)(0.5 * (pal[0].weight + pal[1].weight) + 0.5) : 1;
  for (int v = 0; v < low; ++v) lut[v] = 0;
  const int high = k >= 2 ? (int)(0.5 * (pal[k - 2].weight + pal[k - 1].weight) + 0.5) : 1;
  for (int v = high; v < 766; ++v) lut[v] = k - 1;
  for (int i = 1; i < k - 1; ++i) {
    const int lo = (int)(0.5 * (pal[i - 1].weight + pal[i].weight) + 0.5);
    const int hi = (int)(0.5 * (pal[i].weight + pal[i + 1].weight) + 0.5);
    for (int v = lo; v < hi; ++v) lut[v] = i;
  }
  // The pinned staging below is reused by the next call: wait for the
  // previous map's copies first.
  DQ_HIP(hipStreamSynchronize(stream));
  for (int i = 0; i < k; ++i)
    h_pal_[i] = ((uint32_t)pal[i].red << 16) | ((uint32_t)pal[i].green << 8) | (uint32_t)pal[i].blue;
  for (int v = 0; v < 766; ++v) h_lut_[v] = (uint16_t)lut[v];
  DQ_HIP(hipMemcpyAsync(d_pal_, h_pal_, k * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
  DQ_HIP(hipMemcpyAsync(d_lut_, h_lut_, 766 * sizeof(uint16_t), hipMemcpyHostToDevice, stream));
  timed_begin(stream);
  launch_build_cells(d_pal_, k, d_cell_rec_, d_cell_idx_, stream);
  timed_end(ST_CELLS, 0.0, stream);
  timed_begin(stream);
  launch_map(d_in, n, d_out, d_pal_, k, d_lut_, d_cell_rec_, d_cell_idx_, stream);
  timed_end(ST_MAP, 8.0 * (double)n, stream);
  DQ_HIP(hipStreamSynchronize(stream));
  collect_timing();
}

Engine& engine_for(int device) {
  static std::mutex mu;
  static std::map<int, Engine*> engines;
  std::lock_guard<std::mutex> g(mu);
  auto it = engines.find(device);
  if (it != engines.end()) return *it->second;
  Engine* e = new Engine(device);
  engines[device] = e;
  return *e;
}

}  // namespace dq
