// dq_engine.cpp -- host side of the DivQuant hot path (see dq_engine.h).
#include "dq_engine.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <queue>

namespace dq {

void die(const char* what, const char* file, int line, const char* detail) {
  std::fprintf(stderr, "divquant-hip: fatal: %s (%s:%d): %s\n", what, file, line,
               detail ? detail : "");
  std::fflush(stderr);
  std::abort();
}

namespace {

template <typename T>
void dev_grow(T** p, size_t* cap, size_t want) {
  if (want <= *cap && *p) return;
  if (*p) DQ_HIP(hipFree(*p));
  size_t n = std::max<size_t>(want, 1);
  DQ_HIP(hipMalloc((void**)p, n * sizeof(T)));
  *cap = n;
}

template <typename T>
void host_grow(T** p, size_t want_old_cap, size_t want) {
  (void)want_old_cap;
  if (*p) DQ_HIP(hipHostFree(*p));
  DQ_HIP(hipHostMalloc((void**)p, std::max<size_t>(want, 1) * sizeof(T), hipHostMallocDefault));
}

// Greedy order of the reference's STEP 4 (:876-887): the largest TSE wins,
// the lowest cluster index among equal TSEs (first strict '<' in index order).
struct Cand {
  double tse;
  int idx;
  int node;
};
struct CandLess {
  bool operator()(const Cand& a, const Cand& b) const {
    if (a.tse != b.tse) return a.tse < b.tse;   // max-heap on tse
    return a.idx > b.idx;                       // then lowest index first
  }
};

}  // namespace

Engine::Engine(int device) : device_(device) {
  DQ_HIP(hipSetDevice(device_));
  DQ_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  DQ_HIP(hipMalloc((void**)&d_pal_, 16384 * sizeof(uint32_t)));
  DQ_HIP(hipMalloc((void**)&d_lut_, 768 * sizeof(uint16_t)));
  DQ_HIP(hipMalloc((void**)&d_cell_cnt_, kCells * sizeof(uint16_t)));
  DQ_HIP(hipMalloc((void**)&d_cell_idx_, (size_t)kCells * kCellCap * sizeof(uint16_t)));
  DQ_HIP(hipHostMalloc((void**)&h_pal_, 16384 * sizeof(uint32_t), hipHostMallocDefault));
  DQ_HIP(hipHostMalloc((void**)&h_lut_, 768 * sizeof(uint16_t), hipHostMallocDefault));
}

Engine::~Engine() {
  // Process-lifetime object; the runtime may already be torn down at exit,
  // so release nothing here (the driver reclaims device memory).
}

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
  PendingEvent pe;
  pe.a = take_event();
  pe.b = nullptr;
  pe.kind = -1;
  pe.bytes = 0;
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

void Engine::ensure_pixels(uint32_t n) {
  // +kSweep slack: a tile's clamped loads never leave the allocation.
  const size_t want = (size_t)n + 64;
  if (want > cap_px_ || !d_p0_) {
    if (d_p0_) DQ_HIP(hipFree(d_p0_));
    if (d_p1_) DQ_HIP(hipFree(d_p1_));
    DQ_HIP(hipMalloc((void**)&d_p0_, want * sizeof(uint32_t)));
    DQ_HIP(hipMalloc((void**)&d_p1_, want * sizeof(uint32_t)));
    cap_px_ = want;
  }
}

void Engine::stage_in(const uint32_t* h_in, uint32_t n, hipStream_t stream) {
  const size_t want = (size_t)n + 64;
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
    size_t c = std::max<size_t>(nnodes, 64);
    if (d_nodes_) DQ_HIP(hipFree(d_nodes_));
    if (h_nodes_) DQ_HIP(hipHostFree(h_nodes_));
    DQ_HIP(hipMalloc((void**)&d_nodes_, c * sizeof(DevNode)));
    DQ_HIP(hipHostMalloc((void**)&h_nodes_, c * sizeof(DevNode), hipHostMallocDefault));
    cap_nodes_ = c;
  }
  if (ntiles > cap_tiles_ || !d_tiles_) {
    size_t c = std::max<size_t>(ntiles, 1024);
    if (d_tiles_) DQ_HIP(hipFree(d_tiles_));
    if (d_parts_) DQ_HIP(hipFree(d_parts_));
    if (h_tiles_) DQ_HIP(hipHostFree(h_tiles_));
    DQ_HIP(hipMalloc((void**)&d_tiles_, c * sizeof(Tile)));
    DQ_HIP(hipMalloc((void**)&d_parts_, c * sizeof(TilePartial)));
    DQ_HIP(hipHostMalloc((void**)&h_tiles_, c * sizeof(Tile), hipHostMallocDefault));
    cap_tiles_ = c;
  }
}

// One round: split every node in `active` (one launch per pass for all).
void Engine::run_round(const std::vector<int>& active, bool root_round,
                       int max_iters, double s, hipStream_t stream) {
  const int nn = (int)active.size();
  uint64_t total = 0;
  for (int id : active) total += nodes_[id].len;
  // Tile length: 4096-point steps, ~2048 tiles per round for big rounds.
  uint64_t tl = (total + 2047) / 2048;
  tl = ((tl + kSweep - 1) / kSweep) * kSweep;
  tl = std::max<uint64_t>(kSweep, std::min<uint64_t>(tl, kMaxTilePx));
  size_t ntiles = 0;
  for (int id : active) ntiles += (nodes_[id].len + tl - 1) / tl;
  ensure_round(nn, ntiles);

  int t = 0;
  for (int a = 0; a < nn; ++a) {
    const Node& n = nodes_[active[a]];
    DevNode& d = h_nodes_[a];
    std::memset(&d, 0, sizeof(d));
    d.off = n.off;
    d.len = n.len;
    d.buf = n.buf;
    d.tw = n.w;
    for (int c = 0; c < 3; ++c) { d.tm[c] = n.mean[c]; d.tv[c] = n.var[c]; }
    // Cut axis/position (:388-403): comparisons and copies only.
    double maxv = n.var[0];
    d.axis = 0;
    d.cut = n.mean[0];
    if (maxv < n.var[1]) { maxv = n.var[1]; d.axis = 1; d.cut = n.mean[1]; }
    if (maxv < n.var[2]) { d.axis = 2; d.cut = n.mean[2]; }
    d.tile_begin = t;
    for (uint64_t o = 0; o < n.len; o += tl) {
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

  PixelBufs bufs{staged_root_, d_p0_, d_p1_};
  const double bytes = 4.0 * (double)total;
  const int nt = (int)ntiles;
  auto pass = [&](int kind, int st) {
    timed_begin(stream);
    launch_pass(kind, d_tiles_, nt, d_nodes_, bufs, d_parts_, stream);
    timed_end(st, bytes, stream);
    timed_begin(stream);
    launch_epilogue(kind, d_nodes_, nn, d_tiles_, d_parts_, s, stream);
    timed_end(ST_EPILOGUE, 0.0, stream);
    last_points_swept += total;
  };
  if (root_round) pass(PASS_INIT, ST_INIT);
  pass(PASS_SPLIT, ST_SPLIT);
  for (int it = 0; it < max_iters; ++it) {
    const bool last = (it == max_iters - 1);
    pass(last ? PASS_KLAST : PASS_KMEANS, last ? ST_KLAST : ST_KMEANS);
  }
  timed_begin(stream);
  launch_partition(d_tiles_, nt, d_nodes_, bufs, stream);
  timed_end(ST_PARTITION, 2.0 * bytes, stream);

  DQ_HIP(hipMemcpyAsync(h_nodes_, d_nodes_, nn * sizeof(DevNode), hipMemcpyDeviceToHost, stream));
  DQ_HIP(hipStreamSynchronize(stream));
  collect_timing();

  for (int a = 0; a < nn; ++a) {
    const int id = active[a];
    const DevNode& d = h_nodes_[a];
    Node& p = nodes_[id];
    if (root_round) {
      for (int c = 0; c < 3; ++c) { p.mean[c] = d.tm[c]; p.var[c] = d.tv[c]; }
    }
    const uint32_t n_new = (uint32_t)d.n_new;
    const uint32_t n_old = p.len - n_new;
    Node co, cn;
    co.parent = cn.parent = id;
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

int Engine::cluster(const uint32_t* d_in, uint32_t n, int k, int max_iters,
                    uint32_t* ct, int* num_empty, hipStream_t stream) {
  DQ_CHECK(n > 0, "num_points must be > 0 (DivQuantCluster.cpp:211)");
  DQ_CHECK(k > 0, "num_colors must be > 0 (DivQuantCluster.cpp:229)");
  DQ_CHECK(max_iters >= 1, "max_iters < 1 is not supported (the reference never writes member[] then)");
  DQ_HIP(hipSetDevice(device_));
  if (!stream) stream = stream_;
  // get_double_scale (DivQuantMapColors.cpp:205-220)
  const double s = 1.0 / (std::ceil(1 / 1.0) * std::ceil(n / 1.0));

  last_means.assign((size_t)k * 3, 0.0);
  last_sizes.assign(k, 0);
  last_trace.clear();
  last_rounds = 0;
  last_points_swept = 0;
  nodes_.clear();
  nodes_.reserve(4 * (size_t)k + 8);
  Node root;
  root.w = 1.0;          // :329
  root.off = 0;
  root.len = n;
  root.buf = BUF_IN;
  nodes_.push_back(root);

  std::vector<int> leaf(k, -1);
  leaf[0] = 0;
  if (k > 1) {
    ensure_pixels(n);
    staged_root_ = d_in;
    std::priority_queue<Cand, std::vector<Cand>, CandLess> heap;
    int new_index = 1, old_index = 0;
    std::vector<int> active{0};
    bool root_round = true;
    while (true) {
      run_round(active, root_round, max_iters, s, stream);
      root_round = false;
      last_rounds++;
      // Replay the greedy order as far as the expanded tree allows.
      int need = -1;
      while (new_index < k) {
        const int x = leaf[old_index];
        if (!nodes_[x].expanded) { need = x; break; }
        const int co = nodes_[x].child_old, cn = nodes_[x].child_new;
        last_trace.push_back(new_index);
        last_trace.push_back(old_index);
        last_trace.push_back(nodes_[x].len);
        last_trace.push_back(nodes_[cn].len);
        leaf[old_index] = co;
        leaf[new_index] = cn;
        if (new_index == k - 1) { ++new_index; break; }   // :823-832
        if (nodes_[co].tse > DBL_MIN) heap.push({nodes_[co].tse, old_index, co});
        if (nodes_[cn].tse > DBL_MIN) heap.push({nodes_[cn].tse, new_index, cn});
        while (!heap.empty() && leaf[heap.top().idx] != heap.top().node) heap.pop();
        if (!heap.empty()) old_index = heap.top().idx;   // else unchanged (:876)
        ++new_index;
      }
      if (need < 0) break;
      // Next round: the leaf the replay is waiting for, plus every unexpanded
      // leaf that ranks among the next r greedy picks (r splits remain; a
      // leaf outside the top r of the current frontier can never be picked).
      const int r = k - new_index;
      std::vector<Cand> cands;
      {
        auto h2 = heap;
        while (!h2.empty() && (int)cands.size() < r) {
          Cand c = h2.top();
          h2.pop();
          if (leaf[c.idx] != c.node) continue;
          cands.push_back(c);
        }
      }
      active.clear();
      active.push_back(need);
      for (const Cand& c : cands)
        if (!nodes_[c.node].expanded && c.node != need) active.push_back(c.node);
    }
  }

  // Final centres (:1029-1094).
  int out = 0, empty = 0;
  for (int ic = 0; ic < k; ++ic) {
    const Node& nd = nodes_[leaf[ic]];
    if (k == 1) {
      // mean[0] is never assigned when no split happens: it stays 0.0.
      last_sizes[0] = n;
      ct[out++] = 0;
      break;
    }
    for (int c = 0; c < 3; ++c) last_means[3 * ic + c] = nd.mean[c];
    last_sizes[ic] = nd.len;
    if (nd.len > 0) {
      const uint32_t R = (uint8_t)(nd.mean[0] + 0.5);
      const uint32_t G = (uint8_t)(nd.mean[1] + 0.5);
      const uint32_t B = (uint8_t)(nd.mean[2] + 0.5);
      ct[out++] = (R << 16) | (G << 8) | B;
    } else {
      ++empty;
    }
  }
  if (num_empty) *num_empty = empty;
  return out;
}

void Engine::map(const uint32_t* d_in, uint32_t n, uint32_t* d_out,
                 const uint32_t* ct, int k, hipStream_t stream) {
  DQ_CHECK(k > 0, "colormapSize must be > 0 (DivQuantMapColors.cpp:264)");
  DQ_CHECK(k <= 16384, "colormapSize > 16384 is not supported by the LDS palette");
  DQ_HIP(hipSetDevice(device_));
  if (!stream) stream = stream_;
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
  int low = k >= 2 ? (int)(0.5 * (pal[0].weight + pal[1].weight) + 0.5) : 1;
  for (int v = 0; v < low; ++v) lut[v] = 0;
  int high = k >= 2 ? (int)(0.5 * (pal[k - 2].weight + pal[k - 1].weight) + 0.5) : 1;
  for (int v = high; v < 766; ++v) lut[v] = k - 1;
  for (int i = 1; i < k - 1; ++i) {
    const int lo = (int)(0.5 * (pal[i - 1].weight + pal[i].weight) + 0.5);
    const int hi = (int)(0.5 * (pal[i].weight + pal[i + 1].weight) + 0.5);
    for (int v = lo; v < hi; ++v) lut[v] = i;
  }
  for (int i = 0; i < k; ++i)
    h_pal_[i] = ((uint32_t)pal[i].red << 16) | ((uint32_t)pal[i].green << 8) | (uint32_t)pal[i].blue;
  for (int v = 0; v < 766; ++v) h_lut_[v] = (uint16_t)lut[v];
  DQ_HIP(hipMemcpyAsync(d_pal_, h_pal_, k * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
  DQ_HIP(hipMemcpyAsync(d_lut_, h_lut_, 766 * sizeof(uint16_t), hipMemcpyHostToDevice, stream));
  timed_begin(stream);
  launch_build_cells(d_pal_, k, d_cell_cnt_, d_cell_idx_, stream);
  timed_end(ST_CELLS, 0.0, stream);
  timed_begin(stream);
  launch_map(d_in, n, d_out, d_pal_, k, d_lut_, d_cell_cnt_, d_cell_idx_, stream);
  timed_end(ST_MAP, 8.0 * (double)n, stream);
  // The host staging buffers (h_pal_/h_lut_) are reused by the next call:
  // wait for the copies (and the map) before returning.
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
