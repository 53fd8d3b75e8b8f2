// dq_engine.cpp -- host side of the DivQuant hot path (see dq_engine.h).
#include "dq_engine.h"
#include "dq_weighted.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <atomic>
#include <chrono>
#include <deque>
#include <functional>
#include <string>
#include <unordered_set>

namespace dq {

// The message also goes to the file DQ_HIP_DIE_LOG names (appended, flushed
// before the abort): a test runner that captures stderr loses it otherwise.
void die(const char* what, const char* file, int line, const char* detail) {
  std::fprintf(stderr, "divquant-hip: fatal: %s (%s:%d): %s\n", what, file, line,
               detail ? detail : "");
  std::fflush(stderr);
  if (const char* path = getenv("DQ_HIP_DIE_LOG")) {
    if (FILE* f = std::fopen(path, "a")) {
      std::fprintf(f, "divquant-hip: fatal: %s (%s:%d): %s\n", what, file, line, detail ? detail : "");
      std::fflush(f);
      std::fclose(f);
    }
  }
  std::abort();
}

namespace {
constexpr uint64_t kFusePlanMaxPoints = 12u << 20;   // plansplit_kernel: rounds of <= ~one 4K frame

inline double host_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

constexpr int BUF_IN = 0, BUF_P0 = 1, BUF_P1 = 2;
inline int child_buf(int b) { return b == BUF_P0 ? BUF_P1 : BUF_P0; }
inline size_t align4(size_t x) { return (x + 3) & ~(size_t)3; }
inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }
// words of an aligned BGR24 copy of n points: whole 16-point vectors + slack,
// a multiple of 4 words (the next copy starts 16-B aligned)
inline size_t bgr_words(size_t n) { return ((3 * align16(n) + 64) / 4 + 3) & ~(size_t)3; }

// Split-pass threshold (:473): cut_pos < v <=> v >= thr for integer v.
int32_t split_threshold(double cut) {
  if (!(cut == cut)) return 256;
  if (cut < 0.0) return 0;
  if (cut >= 255.0) return 256;
  return (int32_t)std::floor(cut) + 1;
}

}  // namespace

double Engine::host_us_now() { return host_us(); }

// Experiment switches, all behind ONE entry point: DQ_HIP_TUNE is a list of
// key=value pairs ("tiles=768,lookahead=1").  Every setting leaves the
// outputs identical (they move work between launches, not arithmetic); the
// defaults are the measured best.  Unknown keys abort, so a
// misspelt experiment cannot silently measure the default.
void Engine::apply_tune(const char* spec) {
  std::string all(spec);
  size_t pos = 0;
  while (pos < all.size()) {
    size_t end = all.find(',', pos);
    if (end == std::string::npos) end = all.size();
    const std::string kv = all.substr(pos, end - pos);
    pos = end + 1;
    if (kv.empty()) continue;
    const size_t eq = kv.find('=');
    DQ_CHECK(eq != std::string::npos, "DQ_HIP_TUNE entries are key=value");
    const std::string k = kv.substr(0, eq);
    const long v = atol(kv.c_str() + eq + 1);
    if (k == "full_iters") fixed_point_ = v == 0;                       // every 2-means iteration runs
    else if (k == "plan") plan_ = v != 0;                               // device-planned rounds
    else if (k == "tiles") tiles_target_ = std::max<long>(64, v);      // tiles per big round
    else if (k == "node_tiles") node_tiles_ = std::max<long>(1, std::min<long>(65536, v));   // tiles per record at least
    else if (k == "tile_max")                                           // points per tile at most
      tile_max_ = (uint32_t)std::max<long>(kSweep, std::min<long>(kMaxTilePx, v)) / kSweep * kSweep;
    else if (k == "lds_map") use_lds_map_ = v != 0;                     // 0: the L2-gather map kernel
    else if (k == "lookahead") lookahead_ = (int)std::max<long>(0, std::min<long>(8, v));
    else if (k == "spec_kmeans") speculate_kmeans_ = v != 0;
    else if (k == "spin_sync") spin_sync_ = v != 0;
    else if (k == "eager_replan") eager_replan_ = v != 0;
    else if (k == "stats_only") stats_only_ = v != 0;
    else if (k == "stats_min") stats_min_ = (uint64_t)std::max<long>(0, v);   // last rounds above this many points: PS_STATS
    else if (k == "fuse_plan") fuse_plan_ = v != 0;
    else if (k == "fold_split") fold_split_ = v != 0;                   // split totals from the partition
    else if (k == "persist") persist_ = v != 0;                         // kpersist_kernel rounds
    else if (k == "wsmall") wsmall_ = v != 0;                           // one-launch small weighted calls
    else if (k == "kloop_max") kloop_max_ = (uint32_t)std::max<long>(0, std::min<long>(kLoopMaxLen, v));
    else die("DQ_HIP_TUNE", __FILE__, __LINE__, ("unknown key " + k).c_str());
  }
}

Engine::Engine(int device) : device_(device) {
  const char* tr = getenv("DQ_HIP_TRACE");
  trace_ = tr && (tr[0] == '1' || tr[0] == '2');
  trace_rounds_ = tr && tr[0] == '2';
  // switches of earlier rounds, now DQ_HIP_TUNE keys: refuse them rather than
  // silently measuring the default
  for (const char* old : {"DQ_HIP_FULL_ITERS", "DQ_HIP_PLAN", "DQ_HIP_KLOOP_MAX", "DQ_HIP_FUSE_PLAN"})
    if (getenv(old))
      die("environment", __FILE__, __LINE__,
          (std::string(old) + " was removed: use DQ_HIP_TUNE (full_iters=, plan=, kloop_max=, fuse_plan=)").c_str());
  if (const char* t = getenv("DQ_HIP_TUNE")) apply_tune(t);
  DQ_HIP(hipSetDevice(device_));
  DQ_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  DQ_HIP(hipDeviceGetAttribute(&num_cus_, hipDeviceAttributeMultiprocessorCount, device_));
  num_cus_ = std::max(1, num_cus_);
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
  PendingEvent pe{take_event(), nullptr, -1, 0.0, 0.0};
  DQ_HIP(hipEventRecord(pe.a, stream));
  pending_.push_back(pe);
}

void Engine::timed_end(int kind, double bytes, hipStream_t stream, double units) {
  if (!timing_) return;
  PendingEvent& pe = pending_.back();
  pe.b = take_event();
  pe.kind = kind;
  pe.bytes = bytes;
  pe.units = units;
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
    st.units += pe.units;
    event_pool_.push_back(pe.a);
    event_pool_.push_back(pe.b);
  }
  pending_.clear();
}

void Engine::debug_host_delay() const {
  if (!(debug_ & kDebugHostDelay)) return;
  const double t0 = host_us();
  while (host_us() - t0 < 200.0) __builtin_ia32_pause();
}

// kDebugArenaCheck (tests): the round arena must be all zero when a run
// starts -- every byte a planned round's fused plan + partition expects to
// find cleared (its counters, per-(tile, wave) counts, arrival words) lies
// in it, and nothing but the previous run's end-of-run clear restores it.
void Engine::check_arena_zero(hipStream_t stream) {
  DQ_HIP(hipStreamSynchronize(stream));
  DQ_HIP(hipDeviceSynchronize());   // (the previous run's clear may be on another stream)
  std::vector<uint64_t> h;
  for (size_t c = 0; c < arena_.size(); ++c) {
    h.resize(arena_[c].second / 8);
    DQ_HIP(hipMemcpy(h.data(), arena_[c].first, h.size() * 8, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < h.size(); ++i)
      if (h[i] != 0) {
        char msg[200];
        std::snprintf(msg, sizeof msg, "chunk %zu of %zu (%zu B): non-zero word 0x%016llx at byte %zu", c,
                      arena_.size(), arena_[c].second, (unsigned long long)h[i], i * 8);
        die("round arena not zero at run entry", __FILE__, __LINE__, msg);
      }
  }
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

uint32_t* Engine::scratch_words(size_t n) {
  if (n > cap_scratch_) {
    if (d_scratch_) {
      DQ_HIP(hipDeviceSynchronize());
      DQ_HIP(hipFree(d_scratch_));
    }
    DQ_HIP(hipMalloc((void**)&d_scratch_, n * sizeof(uint32_t)));
    cap_scratch_ = n;
  }
  return d_scratch_;
}

// Device arena for the per-round tables.  Chunks are kept (and reused by the
// next run); a round's block never moves once written.
char* Engine::arena_alloc(size_t bytes, hipStream_t stream) {
  bytes = (bytes + 255) & ~(size_t)255;
  while (true) {
    if (arena_chunk_ < arena_.size()) {
      auto& c = arena_[arena_chunk_];
      if (arena_used_ + bytes <= c.second) {
        char* p = c.first + arena_used_;
        arena_used_ += bytes;
        arena_hw_[arena_chunk_] = std::max(arena_hw_[arena_chunk_], arena_used_);
        return p;
      }
      ++arena_chunk_;
      arena_used_ = 0;
      continue;
    }
    const size_t sz = std::max<size_t>(bytes, (size_t)16 << 20);
    char* p = nullptr;
    DQ_HIP(hipMalloc((void**)&p, sz));
    // Zeroed on the round's stream, ahead of every launch that uses it.  (Not
    // hipMemset: for device memory it is asynchronous to the host and runs on
    // the null stream, which a non-blocking stream does not wait for -- behind
    // other lanes' work it could clear a round block after its first kernels
    // wrote it; see DESIGN.md 3c''.)
    launch_zero(p, sz, stream);
    arena_.push_back({p, sz});
    arena_hw_.push_back(0);
  }
}

template <typename T>
static void grow_device(T** p, size_t* cap, size_t want) {
  if (want <= *cap && *p) return;
  if (*p) DQ_HIP(hipFree(*p));
  const size_t c = std::max<size_t>(want, 1024);
  DQ_HIP(hipMalloc((void**)p, c * sizeof(T)));
  *cap = c;
}

// Host-coherent (fine-grained) pinned memory the kernels write with
// system-scope visibility; the device view comes from hipHostGetDevicePointer.
template <typename T>
static void grow_coherent(T** h, T** d, size_t* cap, size_t want) {
  if (want <= *cap && *h) return;
  if (*h) DQ_HIP(hipHostFree(*h));
  const size_t c = std::max<size_t>(want, 256);
  DQ_HIP(hipHostMalloc((void**)h, c * sizeof(T), hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(*h, 0, c * sizeof(T));
  DQ_HIP(hipHostGetDevicePointer((void**)d, *h, 0));
  *cap = c;
}

// Capacities of one run, set at its start (nothing of this engine is in
// flight then: the previous run ended with a stream synchronisation).
// Per slot (round parity): rec_cap results, status words for max_iters
// 2-means launches + the split epilogue, a plan list; tile partials for
// tiles_cap tiles (every round's tiles and part tiles fit: a tile holds at
// least kSweep points or is its record's last).
void Engine::ensure_round(size_t rec_cap, size_t tiles_cap, size_t, size_t staging_bytes,
                          int max_iters, hipStream_t stream) {
  const bool grow = staging_bytes > cap_stage_tab_ || !h_stage_ || !stage_ev_ || rec_cap > cap_res_ ||
                    !h_res_ || (size_t)max_iters + 1 > cap_stat_ || !h_stat_ || !h_counts_ ||
                    tiles_cap > cap_parts_ || !d_parts_ || tiles_cap > cap_parts2_ || !d_parts2_ ||
                    2 * tiles_cap > cap_sparts_ || !d_sparts_;
  if (!grow) return;
  DQ_HIP(hipStreamSynchronize(stream));
  if (staging_bytes > cap_stage_tab_ || !h_stage_) {
    if (h_stage_) DQ_HIP(hipHostFree(h_stage_));
    const size_t c = std::max<size_t>(staging_bytes, (size_t)1 << 20);
    DQ_HIP(hipHostMalloc((void**)&h_stage_, c, hipHostMallocCoherent | hipHostMallocMapped));
    DQ_HIP(hipHostGetDevicePointer((void**)&d_stage_view_, h_stage_, 0));
    cap_stage_tab_ = c;
  }
  if (!stage_ev_) DQ_HIP(hipEventCreateWithFlags(&stage_ev_, hipEventDisableTiming));
  if (rec_cap > cap_res_ || !h_res_) {
    if (h_res_) DQ_HIP(hipHostFree(h_res_));
    if (d_dres_) DQ_HIP(hipFree(d_dres_));
    if (h_plist_) DQ_HIP(hipHostFree(h_plist_));
    const size_t c = std::max<size_t>(rec_cap, 256);
    DQ_HIP(hipHostMalloc((void**)&h_res_, kSlots * c * sizeof(NodeResult), hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(h_res_, 0, kSlots * c * sizeof(NodeResult));
    DQ_HIP(hipHostGetDevicePointer((void**)&d_res_, h_res_, 0));
    DQ_HIP(hipMalloc((void**)&d_dres_, kSlots * c * sizeof(NodeResult)));
    DQ_HIP(hipHostMalloc((void**)&h_plist_, kSlots * c * sizeof(int32_t), hipHostMallocCoherent | hipHostMallocMapped));
    DQ_HIP(hipHostGetDevicePointer((void**)&d_plist_, h_plist_, 0));
    cap_res_ = c;
    cap_plist_ = c;
  }
  if ((size_t)max_iters + 1 > cap_stat_ || !h_stat_) {
    if (h_stat_) DQ_HIP(hipHostFree(h_stat_));
    cap_stat_ = std::max<size_t>((size_t)max_iters + 1, 32);
    DQ_HIP(hipHostMalloc((void**)&h_stat_, kSlots * cap_stat_ * sizeof(uint64_t), hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(h_stat_, 0, kSlots * cap_stat_ * sizeof(uint64_t));
    DQ_HIP(hipHostGetDevicePointer((void**)&d_stat_, h_stat_, 0));
  }
  if (!h_counts_) {
    DQ_HIP(hipHostMalloc((void**)&h_counts_, kSlots * 4 * sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(h_counts_, 0, kSlots * 4 * sizeof(uint32_t));
    DQ_HIP(hipHostGetDevicePointer((void**)&d_counts_h_, h_counts_, 0));
  }
  grow_device(&d_parts_, &cap_parts_, tiles_cap);
  grow_device(&d_parts2_, &cap_parts2_, tiles_cap);
  grow_device(&d_sparts_, &cap_sparts_, std::max<size_t>(2 * tiles_cap, 2));
}

// The per-logical-node totals an allreduce round sums (8 u64 per node).
void Engine::ensure_totals(size_t nlogical, hipStream_t stream) {
  if (nlogical * 8 <= cap_tot_ && d_tot_) return;
  DQ_HIP(hipStreamSynchronize(stream));
  if (d_tot_) DQ_HIP(hipFree(d_tot_));
  cap_tot_ = std::max<size_t>(nlogical * 8, 4096);
  DQ_HIP(hipMalloc((void**)&d_tot_, cap_tot_ * sizeof(uint64_t)));
}

// Wait for a status word of round `seq`; returns the number of records still
// active.  Bounded: once the stream has drained the word must be there.
// The end of a call: an event on the stream, polled with pause (the host's
// status-word waits spin the same way); hipStreamSynchronize's blocking wait
// woke the host tens of microseconds after the last kernel (DQ_HIP_TUNE spin_sync=0:
// hipStreamSynchronize).
void Engine::sync_stream(hipStream_t stream) {
  if (!spin_sync_) {
    DQ_HIP(hipStreamSynchronize(stream));
    return;
  }
  if (!sync_ev_) DQ_HIP(hipEventCreateWithFlags(&sync_ev_, hipEventDisableTiming));
  DQ_HIP(hipEventRecord(sync_ev_, stream));
  for (;;) {
    const hipError_t e = hipEventQuery(sync_ev_);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) die("hipEventQuery", __FILE__, __LINE__, hipGetErrorString(e));
    for (int i = 0; i < 16; ++i) __builtin_ia32_pause();
  }
}

uint32_t Engine::wait_status(const uint64_t* slot, uint64_t seq, hipStream_t stream) {
  const double t0 = trace_ ? host_us() : 0.0;
  struct Acc {
    Engine* e; double t0;
    ~Acc() {
      if (e->trace_) {
        e->tr_wait_us_ += host_us() - t0;
        e->tmark("w");
      }
    }
  } acc{this, t0};
  tmark("W");
  const uint32_t want = (uint32_t)seq;
  auto ready = [&](uint32_t* act) {
    const uint64_t v = __atomic_load_n(slot, __ATOMIC_ACQUIRE);
    if (!(v & 1) || (uint32_t)(v >> 32) != want) return false;
    *act = (uint32_t)((v >> 1) & 0x7FFFFFFFu);
    return true;
  };
  uint32_t act = 0;
  for (uint64_t spin = 0;; ++spin) {
    if (ready(&act)) return act;
    __builtin_ia32_pause();   // (spinning lane threads share cores)
    if ((spin & 0x3FFF) == 0x3FFF) {
      const hipError_t e = hipStreamQuery(stream);
      if (e == hipSuccess) {
        if (ready(&act)) return act;
        char msg[384];
        const uint64_t v = __atomic_load_n(slot, __ATOMIC_ACQUIRE);
        const long si = (long)(slot - h_stat_);
        int n = snprintf(msg, sizeof msg, "stream drained without the round's status (slot %ld:%ld, seq %llu, word %016llx",
                         si / (long)cap_stat_, si % (long)cap_stat_, (unsigned long long)seq, (unsigned long long)v);
        if (wait_round_ >= 0 && wait_round_ < (int)rounds_.size()) {
          const Round& R = rounds_[wait_round_];
          const uint32_t* hc = h_counts_ + 4 * R.par;
          n += snprintf(msg + n, sizeof msg - n, "; round %d planned %d prev %d nr %d tiles %zu ptiles %zu counts %u/%u/%u",
                        wait_round_, (int)R.planned, R.prev, R.nr, R.ntiles, R.nptiles, hc[0], hc[1], hc[2]);
        }
        snprintf(msg + n, sizeof msg - n, ")");
        die("status word", __FILE__, __LINE__, msg);
      }
      if (e != hipErrorNotReady) die("hipStreamQuery", __FILE__, __LINE__, hipGetErrorString(e));
    }
  }
}

// A frame shard in a buffer: the caller's packed frame (BUF_IN), or byte 0 of
// its R plane in P0 / P1 (planes cap_px_ bytes apart: DESIGN.md 4).
const uint8_t* Engine::buf_ptr(int buf, const FrameState& f, int shard) const {
  if (buf == BUF_IN) return reinterpret_cast<const uint8_t*>(f.in[shard]);
  return reinterpret_cast<const uint8_t*>(buf == BUF_P0 ? d_p0_ : d_p1_) + f.base[shard];
}

// Tile length of a round of `total` points: whole 4096-point sweeps, about
// tiles_target_ tiles, at most tile_max_ points.  A record gets at least
// node_tiles_ tiles (a node still active late in a round is then swept by
// several workgroups, not one).  plan_kernel restates both (plan_tile_len).
uint64_t Engine::round_tile_len(uint64_t total) const {
  uint64_t tl = (total + tiles_target_ - 1) / tiles_target_;
  tl = ((tl + kSweep - 1) / kSweep) * kSweep;
  return std::max<uint64_t>(kSweep, std::min<uint64_t>(tl, tile_max_));
}

uint64_t Engine::tile_len_of(uint64_t len, uint64_t tl) const {
  uint64_t t = (len + node_tiles_ - 1) / node_tiles_;
  t = ((t + kSweep - 1) / kSweep) * kSweep;
  return std::max<uint64_t>(kSweep, std::min<uint64_t>(tl, t));
}

// The source format of every node in `ids` (a partition launch's parents):
// planar working buffers, or a root's caller frame (packed / BGR24); mixed:
// FMT_ANY.
int Engine::src_fmt(const std::vector<int>& ids) const {
  int f = -1;
  for (int id : ids) {
    const Node& n = nodes_[id];
    const int g = n.buf != BUF_IN ? FMT_PLANAR : (frames_[n.frame].job->bgr ? FMT_BGR : FMT_PACKED);
    if (f >= 0 && g != f) return FMT_ANY;
    f = g;
  }
  return f < 0 ? FMT_ANY : f;
}

// ---------------------------------------------------------------------------
// Host-built round: split every node in `active` (one launch per pass for
// all), launched up to its split epilogue; finish_round waits for it.
//
// Every logical node has one RECORD per shard (record r = node * S + shard):
// the passes run over each record's own (local) points; the FP64 update
// needs the node's sums over all shards and all processes -- one fused
// epilogue when S == 1 and no communicator, else nodesum (over the records)
// + RCCL allreduce (over the processes) + epilogue from the totals.
//
// A node whose parent was split in an earlier round but not yet partitioned
// gets its points and its split-pass statistics from ONE fused launch over
// the parent's tiles (partsplit_kernel); every other node (the roots, and
// nodes whose sibling already forced the partition) has its own split pass.
// Partitions are lazy: a node is partitioned only when one of its children is
// split, so the leaves of the last round never are.
int Engine::enqueue_host_round(const std::vector<int>& active_in, bool root_round, int max_iters,
                               hipStream_t stream) {
  debug_host_delay();
  const double tb0 = trace_ ? host_us() : 0.0;
  const int S = nshard_;
  const int mode = tot_mode();
  rounds_.emplace_back();
  const int ri = (int)rounds_.size() - 1;
  Round& R = rounds_[ri];
  R.root = root_round;
  std::vector<int>& order = R.order;
  std::vector<int>& parents = R.parents;
  // node id -> logical slot in the round / position in `parents` (-1: none)
  slot_of_.assign(nodes_.size(), -1);
  parent_pos_.assign(nodes_.size(), -1);
  for (int id : active_in)
    if (root_round || nodes_[nodes_[id].parent].partitioned) order.push_back(id);
  const int n_own = (int)order.size();
  for (int id : active_in) {
    if (root_round || nodes_[nodes_[id].parent].partitioned) continue;
    order.push_back(id);
    const int p = nodes_[id].parent;
    if (parent_pos_[p] < 0) {
      parent_pos_[p] = (int)parents.size();
      parents.push_back(p);
    }
  }
  const int nl = (int)order.size();   // logical nodes
  const int nr = nl * S;              // records
  R.n_own = n_own;
  // Segments this round reads that a PS_STATS round left unwritten (own
  // split passes read a node's segment, fused partitions its parent's):
  // written first by a PS_WRITE partition of their parents, parents first.
  std::vector<int> mat;
  std::function<void(int)> need = [&](int x) {
    if (nodes_[x].points) return;
    const int p = nodes_[x].parent;
    need(p);
    if (std::find(mat.begin(), mat.end(), p) == mat.end()) mat.push_back(p);
    nodes_[nodes_[p].child_old].points = true;
    nodes_[nodes_[p].child_new].points = true;
  };
  for (int a = 0; a < n_own; ++a) need(order[a]);
  for (int p : parents) need(p);
  size_t nmat = 0;
  for (int p : mat)
    for (int sh = 0; sh < S; ++sh) nmat += seg(p, sh).ntiles;
  R.nl = nl;
  R.nr = nr;
  DQ_CHECK((size_t)nr <= cap_res_, "round larger than the run's record capacity");

  uint64_t total = 0, own_total = 0, parent_total = 0;   // local points
  double own_bytes = 0.0, part_bytes = 0.0;               // engine work model
  for (int a = 0; a < nl; ++a)
    for (int sh = 0; sh < S; ++sh) {
      total += seg(order[a], sh).len;
      if (a < n_own) {
        own_total += seg(order[a], sh).len;
        own_bytes += point_bytes(order[a]) * seg(order[a], sh).len;
      }
    }
  for (int p : parents)
    for (int sh = 0; sh < S; ++sh) {
      parent_total += seg(p, sh).len;
      part_bytes += (point_bytes(p) + 3.0) * seg(p, sh).len;
    }
  const uint64_t tl = round_tile_len(total);
  size_t ntiles = 0, nt_own = 0;
  for (int a = 0; a < nl; ++a) {   // empty records get one empty tile (their epilogue still runs)
    for (int sh = 0; sh < S; ++sh) {
      const uint64_t len = seg(order[a], sh).len;
      const uint64_t tln = tile_len_of(len, tl);
      ntiles += std::max<size_t>(1, (len + tln - 1) / tln);
    }
    if (a == n_own - 1) nt_own = ntiles;
  }
  size_t nptiles = 0;
  for (int p : parents)
    for (int sh = 0; sh < S; ++sh) nptiles += seg(p, sh).ntiles;
  DQ_CHECK(ntiles <= cap_parts_ && 2 * nptiles <= cap_sparts_, "round larger than the run's tile capacity");
  R.total = total;
  R.own_total = own_total;
  R.parent_total = parent_total;
  R.tl = tl;
  R.ntiles = R.tiles_cap = ntiles;
  R.nptiles = R.ptiles_cap = nptiles;
  R.nt_own = nt_own;

  // the round's block: [DevNode nr | Tile ntiles | PartTile nptiles | LaunchCtr max_iters+1 | wparts | rdone]
  auto al = [](size_t x) { return (x + 63) & ~(size_t)63; };
  const size_t o_tiles = al(nr * sizeof(DevNode));
  const size_t o_pt = o_tiles + al(ntiles * sizeof(Tile));
  const size_t o_mpt = o_pt + al(nptiles * sizeof(PartTile));
  const size_t o_ctr = o_mpt + al(nmat * sizeof(PartTile));
  // (LaunchCtr and status word max_iters: the split epilogue's); then the
  // per-(tile, wave) counts, zero from the staging memset (partsplit adds
  // the fused children's up)
  const size_t o_wp = o_ctr + al((size_t)(max_iters + 1) * sizeof(LaunchCtr));
  // then the fused 2-means passes' arrival words, per (iteration, record)
  const size_t o_rd = o_wp + al(ntiles * kTileWaves * sizeof(uint32_t));
  // then the records' summaries (written as each becomes final; the next plan's scan)
  const size_t o_sum = o_rd + al((size_t)max_iters * nr * sizeof(uint32_t));
  // then the partition's per-parent arrival words (split totals folded in)
  const size_t o_sd = o_sum + al((size_t)nr * sizeof(RecSummary));
  const size_t bytes = o_sd + al((size_t)nr * sizeof(uint32_t));
  R.bytes = bytes;
  if (mode == TOT_ALLREDUCE) ensure_totals(nl, stream);
  // the staging is rewritten: its previous upload must have run
  if (stage_pending_) {
    DQ_HIP(hipEventSynchronize(stage_ev_));
    stage_pending_ = false;
  }
  if (bytes > cap_stage_tab_) {
    DQ_HIP(hipHostFree(h_stage_));
    const size_t c = std::max<size_t>(bytes, 2 * cap_stage_tab_);
    DQ_HIP(hipHostMalloc((void**)&h_stage_, c, hipHostMallocCoherent | hipHostMallocMapped));
    DQ_HIP(hipHostGetDevicePointer((void**)&d_stage_view_, h_stage_, 0));
    cap_stage_tab_ = c;
  }
  char* dblk = arena_alloc(bytes, stream);
  std::memset(h_stage_, 0, bytes);
  DevNode* hn = reinterpret_cast<DevNode*>(h_stage_);
  Tile* ht = reinterpret_cast<Tile*>(h_stage_ + o_tiles);
  PartTile* hp = reinterpret_cast<PartTile*>(h_stage_ + o_pt);
  DevNode* dn = reinterpret_cast<DevNode*>(dblk);
  Tile* dt = reinterpret_cast<Tile*>(dblk + o_tiles);
  R.dn = dn;
  R.dt = dt;
  R.tbeg.assign(nr, 0);
  R.tend.assign(nr, 0);

  // first PartTile of each (parent, shard)
  std::vector<int> pt_first(parents.size() * S);
  {
    int q = 0;
    for (size_t i = 0; i < parents.size(); ++i)
      for (int sh = 0; sh < S; ++sh) {
        pt_first[i * S + sh] = q;
        q += seg(parents[i], sh).ntiles;
      }
  }
  int t = 0;
  for (int a = 0; a < nl; ++a) {
    Node& n = nodes_[order[a]];
    n.queued = true;
    slot_of_[order[a]] = a;
    frames_[n.frame].splits_queued++;
    const FrameState& fs = frames_[n.frame];
    int32_t thr = 0, shift = 0;
    if (!root_round) {
      // Cut axis/position (:388-403): comparisons and copies only.  (The
      // root's come from its PASS_INIT epilogue on the device.)
      double maxv = n.var[0], cut = n.mean[0];
      int axis = 0;
      if (maxv < n.var[1]) { maxv = n.var[1]; axis = 1; cut = n.mean[1]; }
      if (maxv < n.var[2]) { axis = 2; cut = n.mean[2]; }
      thr = split_threshold(cut);
      shift = 16 - 8 * axis;
    }
    n.axis = (int16_t)((16 - shift) >> 3);
    n.thr = (int16_t)thr;
    for (int sh = 0; sh < S; ++sh) {
      DevNode& d = hn[a * S + sh];
      d.src = buf_ptr(n.buf, fs, sh);
      d.dst = const_cast<uint8_t*>(buf_ptr(child_buf(n.buf), fs, sh));
      d.planar = n.buf != BUF_IN ? SRC_PLANAR : (fs.job->bgr ? SRC_BGR24 : SRC_PACKED);
      const Seg& sg = seg(order[a], sh);
      d.off = sg.off;
      d.len = sg.len;
      d.s = fs.s;
      d.tw = n.w;
      d.split_pb = -1;
      d.split_pe = -1;
      if (a >= n_own) {
        const int pi = parent_pos_[n.parent];
        d.split_pb = pt_first[pi * S + sh];
        d.split_pe = d.split_pb + seg(n.parent, sh).ntiles;
        d.split_side = nodes_[n.parent].child_new == order[a] ? 1 : 0;
      }
      for (int c = 0; c < 3; ++c) { d.tm[c] = n.mean[c]; d.tv[c] = n.var[c]; }
      d.prm.thr = thr;
      d.prm.shift = shift;
      for (int c = 0; c < 3; ++c) { d.box_lo[c] = n.lo[c]; d.box_hi[c] = n.hi[c]; }
      d.tile_begin = t;
      const uint64_t tln = tile_len_of(sg.len, tl);
      d.tile_len = (uint32_t)tln;
      for (uint64_t o = 0; o == 0 || o < sg.len; o += tln) {
        Tile& tt = ht[t++];
        tt.node = a * S + sh;
        tt.start = sg.off + (uint32_t)o;
        tt.end = sg.off + (uint32_t)std::min<uint64_t>(sg.len, o + tln);
      }
      d.tile_end = t;
      R.tbeg[a * S + sh] = d.tile_begin;
      R.tend[a * S + sh] = d.tile_end;
    }
  }
  {
    int q = 0;
    for (int p : parents) {
      Node& pn = nodes_[p];
      pn.partitioned = true;
      int32_t thr[2], shift[2];
      const int ch[2] = {pn.child_old, pn.child_new};
      for (int c = 0; c < 2; ++c) {
        const int sl = slot_of_[ch[c]];
        thr[c] = sl >= 0 ? hn[sl * S].prm.thr : 256;   // 256: nothing counted
        shift[c] = sl >= 0 ? hn[sl * S].prm.shift : 0;
      }
      for (int sh = 0; sh < S; ++sh) {
        const Seg& ps = seg(p, sh);
        for (int i = 0; i < ps.ntiles; ++i) {
          PartTile& pt = hp[q++];
          pt.tile = ps.dtiles + i;
          pt.parent = ps.dnode;
          pt.thr[0] = thr[0];
          pt.thr[1] = thr[1];
          pt.shift[0] = shift[0];
          pt.shift[1] = shift[1];
          for (int c = 0; c < 2; ++c) {
            const int sl = slot_of_[ch[c]];
            pt.child[c] = sl >= 0 ? sl * S + sh : -1;
          }
        }
      }
    }
  }
  {   // the PS_WRITE partition's part tiles (no children split: nothing summed or counted)
    PartTile* hm = reinterpret_cast<PartTile*>(h_stage_ + o_mpt);
    int q = 0;
    for (int p : mat)
      for (int sh = 0; sh < S; ++sh) {
        const Seg& ps = seg(p, sh);
        for (int i = 0; i < ps.ntiles; ++i) {
          PartTile& pt = hm[q++];
          pt.tile = ps.dtiles + i;
          pt.parent = ps.dnode;
          pt.thr[0] = pt.thr[1] = 256;
          pt.shift[0] = pt.shift[1] = 0;
          pt.child[0] = pt.child[1] = -1;
        }
      }
  }
  const double tb1 = trace_ ? host_us() : 0.0;
  // one upload kernel on the round's stream (no copy-engine hop)
  if (trace_ && root_round) tr_first_us_ = host_us() - tr_entry_t0_;
  tmark("host:tables");
  launch_upload(dblk, d_stage_view_, bytes, stream);
  tmark("upload");
  if (trace_) tr_build_us_ += host_us() - tb0;

  R.seq = ++seq_;
  R.par = (int)(R.seq % kSlots);
  RoundArgs& ra = R.ra;
  ra.tiles = dt;
  ra.nodes = dn;
  ra.parts = d_parts_;
  ra.parts2 = d_parts2_;
  ra.wparts = reinterpret_cast<uint32_t*>(dblk + o_wp);
  ra.ptiles = reinterpret_cast<const PartTile*>(dblk + o_pt);
  ra.sparts = d_sparts_;
  ra.hres = d_res_ + (size_t)R.par * cap_res_;
  ra.ctr = reinterpret_cast<LaunchCtr*>(dblk + o_ctr);
  ra.hstat = d_stat_ + (size_t)R.par * cap_stat_;
  ra.seq = R.seq;
  ra.fixed_point = fixed_point_ ? 1 : 0;
  ra.it = 0;
  ra.nn = nr;
  ra.tot = d_tot_;
  ra.nshard = S;
  ra.debug = debug_;
  ra.rdone = reinterpret_cast<uint32_t*>(dblk + o_rd);
  ra.rsum = reinterpret_cast<RecSummary*>(dblk + o_sum);
  ra.dres = d_dres_ + (size_t)R.par * cap_res_;
  ra.counts = nullptr;
  ra.plane = cap_px_;
  ra.tot_mode = mode;
  ra.ps_mode = PS_FULL;
  // allreduced totals with one shard and every record a partitioned parent's
  // child: the partition's last workgroups write the split totals (no
  // nodesum_kernel launch)
  const bool fold = fold_split_ && mode == TOT_ALLREDUCE && S == 1 && n_own == 0 && nptiles > 0;
  ra.sdone = fold ? reinterpret_cast<uint32_t*>(dblk + o_sd) : nullptr;
  if (nmat > 0) {
    RoundArgs ma = ra;
    ma.sdone = nullptr;
    ma.ptiles = reinterpret_cast<const PartTile*>(dblk + o_mpt);
    ma.ps_mode = PS_WRITE;
    timed_begin(stream);
    launch_partsplit(ma, (int)nmat, src_fmt(mat), stream);
    timed_end(ST_PARTITION, 0.0, stream);
  }
  // parents finalised at a PS_STATS round's split: their cursors first
  // (their points exist by now: PS_WRITE above), before this round's own
  // split pass reuses the tile-partial scratch the count pass writes
  for (int p : parents)
    if (nodes_[p].cursors_pending) fix_cursors(p, stream);
  const double bytes_all = 4.0 * (double)total;
  const int nt = (int)ntiles;
  auto pass = [&](int kind, int st, int tiles, double pbytes, double units) {
    ra.it = 0;
    if (tiles > 0) {
      timed_begin(stream);
      launch_pass(kind, ra, tiles, stream);
      tmark(kind == PASS_INIT ? "init" : "split");
      timed_end(st, pbytes, stream, units);
    }
  };
  auto epilogue = [&](int kind, int it) {
    ra.it = it < 0 ? 0 : it;
    timed_begin(stream);
    if (mode == TOT_ALLREDUCE) {
      if (!(kind == PASS_SPLIT && fold)) launch_nodesum(kind, ra, nl, stream);
      allreduce_totals(nl, stream);
    }
    launch_epilogue(kind, ra, nr, stream);
    tmark("epi");
    timed_end(ST_EPILOGUE, 0.0, stream);
  };
  if (root_round) {
    pass(PASS_INIT, ST_INIT, nt, bytes_all, (double)total);
    epilogue(PASS_INIT, -1);
  }
  pass(PASS_SPLIT, ST_SPLIT, (int)nt_own, own_bytes, (double)own_total);
  if (nptiles > 0) {
    timed_begin(stream);
    launch_partsplit(ra, (int)nptiles, src_fmt(parents), stream);
    timed_end(ST_PARTITION, part_bytes, stream, (double)parent_total);
  }
  epilogue(PASS_SPLIT, max_iters);
  // the staging's reuse waits for this event; recorded behind the round's
  // kernels (stream order: after the upload) so that the host submits the
  // first kernels without it in between (~6-15 us of GPU idle at a call's start)
  DQ_HIP(hipEventRecord(stage_ev_, stream));
  tmark("stage_ev");
  stage_pending_ = true;
  R.t_enq = tb1;
  return ri;
}

// Which logical nodes of round ri the next round may split before ri's
// results exist (speculation): every node of a frame whose splits queued so
// far stay below k - 1 (the greedy replay may need more).  Returns false
// when nothing is planned.
bool Engine::plan_list(int ri, std::vector<int32_t>* plist) {
  const Round& R = rounds_[ri];
  plist->clear();
  if (!plan_ || !fixed_point_) return false;
  // frames of the round: speculate when the frame may need more splits
  for (int a = 0; a < R.nl; ++a) {
    const FrameState& f = frames_[nodes_[R.order[a]].frame];
    if (f.splits_queued < f.job->k - 1) plist->push_back(a);
  }
  if (plist->empty() || 2 * plist->size() * (size_t)nshard_ > cap_res_ ||
      plist->size() > (size_t)kPlanMaxParents) {
    plist->clear();
    return false;
  }
  return true;
}

// Planned round: the children of `plist`'s records of round `prev`, tables
// built on the device by plan_kernel, enqueued now -- before `prev`'s
// results exist.  Grids are upper bounds (the kernels read the plan's
// counts); if a listed record is not final after its split epilogue the plan
// aborts the round (the host plans it again once `prev` has converged).
int Engine::enqueue_planned_round(int prev, const std::vector<int32_t>& plist, int max_iters,
                                  hipStream_t stream, const uint32_t* cancel) {
  const double tb0 = trace_ ? host_us() : 0.0;
  tmark("plan:begin");
  rounds_.emplace_back();
  const int ri = (int)rounds_.size() - 1;
  Round& R = rounds_[ri];
  const Round& P = rounds_[prev];
  R.planned = true;
  R.prev = prev;
  R.plist = plist;
  const int S = nshard_;
  const int mode = tot_mode();
  const int np = (int)plist.size();
  R.nl = 2 * np;
  R.nr = R.nl * S;
  R.n_own = 0;
  uint64_t total = 0;
  double part_bytes = 0.0;
  for (int32_t a : plist) {
    const int id = P.order[a];
    for (int sh = 0; sh < S; ++sh) {
      total += seg(id, sh).len;
      part_bytes += (point_bytes(id) + 3.0) * seg(id, sh).len;
    }
    Node& pn = nodes_[id];
    pn.partitioned = true;
    frames_[pn.frame].splits_queued += 2;
  }
  for (int32_t a : plist) R.parents.push_back(P.order[a]);
  // the last round of every frame it holds: its nodes' children are leaves
  // unless the greedy replay needs more splits than were speculated -- the
  // partition only sums (PS_STATS); the points of parents with a child left
  // active go out after the split epilogue (PS_LATE), the rest only if a
  // later round reads them (enqueue_host_round, PS_WRITE)
  // (rounds of at most one 4K frame's points write them all instead: the
  // single-frame chain's PS_STATS + PS_LATE launches cost more than PS_FULL's
  // writes -- C3 -1.5-2 %, C2 -0.5 %; batches keep the stats-only form)
  R.stats_only = stats_only_ && total > stats_min_;
  for (int32_t a : plist) {
    const FrameState& f = frames_[nodes_[P.order[a]].frame];
    R.stats_only = R.stats_only && f.splits_queued >= f.job->k - 1;
  }
  if (R.stats_only) part_bytes = 0.0;
  if (R.stats_only)
    for (int32_t a : plist)
      for (int sh = 0; sh < S; ++sh) part_bytes += point_bytes(P.order[a]) * seg(P.order[a], sh).len;
  R.total = R.parent_total = total;
  R.own_total = 0;
  R.tl = round_tile_len(total);
  // (a record has at most len / kSweep + 1 tiles, and at most
  // len / tl + node_tiles + 1)
  R.tiles_cap = std::min<size_t>(total / kSweep + (size_t)R.nr + 1,
                                 total / R.tl + (size_t)R.nr * (node_tiles_ + 1) + 1);
  R.ptiles_cap = P.tiles_cap;
  DQ_CHECK(R.tiles_cap <= cap_parts_ && 2 * R.ptiles_cap <= cap_sparts_, "planned round above the tile capacity");
  auto al = [](size_t x) { return (x + 63) & ~(size_t)63; };
  const size_t nr = (size_t)R.nr;
  const size_t o_tiles = al(nr * sizeof(DevNode));
  const size_t o_pt = o_tiles + al(R.tiles_cap * sizeof(Tile));
  const size_t o_cnt = o_pt + al(R.ptiles_cap * sizeof(PartTile));
  const size_t o_ctr = o_cnt + 64;
  const size_t o_wp = o_ctr + al((size_t)(max_iters + 1) * sizeof(LaunchCtr));
  const size_t o_rd = o_wp + al(R.tiles_cap * kTileWaves * sizeof(uint32_t));
  const size_t o_sum = o_rd + al((size_t)max_iters * nr * sizeof(uint32_t));
  const size_t o_sd = o_sum + al(nr * sizeof(RecSummary));   // (the partition's per-parent arrivals)
  const size_t bytes = o_sd + al(nr * sizeof(uint32_t));     // ([o_ctr, bytes): zero on entry)
  R.bytes = bytes;
  char* dblk = arena_alloc(bytes, stream);
  R.dn = reinterpret_cast<DevNode*>(dblk);
  R.dt = reinterpret_cast<Tile*>(dblk + o_tiles);
  R.dcounts = reinterpret_cast<uint32_t*>(dblk + o_cnt);
  R.seq = ++seq_;
  R.par = (int)(R.seq % kSlots);
  // the plan list: identity unless some frames do not speculate
  bool ident = true;
  for (int i = 0; i < np; ++i) ident = ident && plist[i] == i && np == P.nl;
  int32_t* hpl = h_plist_ + (size_t)R.par * cap_plist_;
  if (!ident) std::memcpy(hpl, plist.data(), (size_t)np * sizeof(int32_t));

  PlanArgs pa;
  pa.pn = P.dn;
  pa.psum = P.ra.rsum;
  pa.pres = d_dres_ + (size_t)P.par * cap_res_;
  pa.ptiles = P.dt;
  pa.plist = ident ? nullptr : d_plist_ + (size_t)R.par * cap_plist_;
  pa.np = np;
  pa.node_tiles = node_tiles_;
  pa.tl = (uint32_t)R.tl;
  pa.tiles_cap = (uint32_t)R.tiles_cap;
  pa.ptiles_cap = (uint32_t)R.ptiles_cap;
  pa.cn = R.dn;
  pa.ct = R.dt;
  pa.cpt = reinterpret_cast<PartTile*>(dblk + o_pt);
  pa.counts = R.dcounts;
  pa.hcounts = d_counts_h_ + 4 * R.par;
  pa.p0 = reinterpret_cast<const uint8_t*>(d_p0_);
  pa.p1 = reinterpret_cast<const uint8_t*>(d_p1_);
  pa.cap_bytes = 4 * cap_px_;
  pa.debug = debug_;
  pa.nshard = S;
  pa.cancel = cancel;
  RoundArgs& ra = R.ra;
  ra.tiles = R.dt;
  ra.nodes = R.dn;
  ra.parts = d_parts_;
  ra.parts2 = d_parts2_;
  ra.wparts = reinterpret_cast<uint32_t*>(dblk + o_wp);
  ra.ptiles = pa.cpt;
  ra.sparts = d_sparts_;
  ra.hres = d_res_ + (size_t)R.par * cap_res_;
  ra.ctr = reinterpret_cast<LaunchCtr*>(dblk + o_ctr);
  ra.hstat = d_stat_ + (size_t)R.par * cap_stat_;
  ra.seq = R.seq;
  ra.fixed_point = fixed_point_ ? 1 : 0;
  ra.it = max_iters;
  ra.nn = R.nr;
  if (mode == TOT_ALLREDUCE) ensure_totals(R.nl, stream);
  ra.tot = d_tot_;
  ra.nshard = S;
  ra.debug = debug_;
  ra.rdone = reinterpret_cast<uint32_t*>(dblk + o_rd);
  ra.rsum = reinterpret_cast<RecSummary*>(dblk + o_sum);
  ra.dres = d_dres_ + (size_t)R.par * cap_res_;
  ra.counts = R.dcounts;
  ra.plane = cap_px_;
  ra.tot_mode = mode;
  ra.ps_mode = R.stats_only ? PS_STATS : PS_FULL;
  // (split totals folded into the partition, as in enqueue_host_round)
  const bool fold = fold_split_ && mode == TOT_ALLREDUCE && S == 1;
  ra.sdone = fold ? reinterpret_cast<uint32_t*>(dblk + o_sd) : nullptr;
  // the plan and the partition in one launch (arena block zero) for rounds of
  // about one wave of partition workgroups (4 per CU) over at most one 4K
  // frame's points: there the plan's launch and round trips are on the
  // critical path (C3 median 0.557-0.585 -> 0.537-0.544 ms); in the lanes of
  // a batch (2-3 frames per round) the workgroups' repeated parent scans cost
  // more than the plan launch they save (8 x 4K: 1.35 -> 1.40-1.42 ms)
  size_t ptiles = 0;   // the part tiles (the listed records' tiles; prev is assigned)
  if (P.tbeg.size() == (size_t)P.nr && P.tend.size() == (size_t)P.nr) {
    for (int32_t a : plist)
      for (int sh = 0; sh < S; ++sh) ptiles += (size_t)(P.tend[a * S + sh] - P.tbeg[a * S + sh]);
  } else {
    ptiles = R.ptiles_cap;
  }
  if (fuse_plan_ && S == 1 && ptiles <= (size_t)(6 * num_cus_) && total <= kFusePlanMaxPoints) {
    timed_begin(stream);
    launch_plansplit(pa, ra, (int)R.ptiles_cap, src_fmt(R.parents), stream);
    timed_end(ST_PARTITION, part_bytes, stream, (double)total);
  } else {
    timed_begin(stream);
    launch_plan(pa, stream);
    timed_end(ST_PLAN, 0.0, stream);
    timed_begin(stream);
    launch_partsplit(ra, (int)R.ptiles_cap, src_fmt(R.parents), stream);
    timed_end(ST_PARTITION, part_bytes, stream, (double)total);
  }
  timed_begin(stream);
  if (mode == TOT_ALLREDUCE) {   // (an aborted round's nodesum writes nothing; every rank
    if (!fold) launch_nodesum(PASS_SPLIT, ra, R.nl, stream);   //  aborts the same rounds: same totals)
    allreduce_totals(R.nl, stream);
  }
  launch_epilogue(PASS_SPLIT, ra, R.nr, stream);
  timed_end(ST_EPILOGUE, 0.0, stream);
  if (R.stats_only) {   // the points of every parent with a child still active
    RoundArgs la = ra;
    la.ps_mode = PS_LATE;
    la.sdone = nullptr;
    timed_begin(stream);
    launch_partsplit(la, (int)R.ptiles_cap, src_fmt(R.parents), stream);
    timed_end(ST_PARTITION, 0.0, stream);
  }
  tmark("plan:end");
  if (trace_) tr_build_us_ += host_us() - tb0;
  R.t_enq = trace_ ? host_us() : 0.0;
  return ri;
}

// Once the round a planned round is planned from is finished (its children
// exist): the planned round's nodes, records and tiles on the host, as the
// plan built them on the device (plan_kernel's layout rules).
void Engine::assign_planned(int ri) {
  Round& R = rounds_[ri];
  const Round& P = rounds_[R.prev];
  R.order.clear();
  for (int32_t a : R.plist) {
    const Node& pn = nodes_[P.order[a]];
    R.order.push_back(pn.child_old);
    R.order.push_back(pn.child_new);
  }
  const int S = nshard_;
  R.tbeg.assign(R.nr, 0);
  R.tend.assign(R.nr, 0);
  int32_t t = 0;
  size_t npt = 0;
  for (int a = 0; a < R.nl; ++a) {
    Node& n = nodes_[R.order[a]];
    n.queued = true;
    for (int sh = 0; sh < S; ++sh) {   // records a * S + sh, tiles in record order
      const uint64_t len = seg(R.order[a], sh).len;
      const uint64_t tln = tile_len_of(len, R.tl);
      R.tbeg[a * S + sh] = t;
      t += (int32_t)std::max<uint64_t>(1, (len + tln - 1) / tln);
      R.tend[a * S + sh] = t;
    }
    // the cut the plan chose (:388-403), for the children's boxes
    double maxv = n.var[0], cut = n.mean[0];
    int axis = 0;
    if (maxv < n.var[1]) { maxv = n.var[1]; axis = 1; cut = n.mean[1]; }
    if (maxv < n.var[2]) { axis = 2; cut = n.mean[2]; }
    n.axis = (int16_t)axis;
    n.thr = (int16_t)split_threshold(cut);
  }
  for (int p : R.parents)
    for (int sh = 0; sh < S; ++sh) npt += seg(p, sh).ntiles;
  R.ntiles = (size_t)t;
  R.nptiles = npt;
}

// 2-means iteration `it` of a round: the pass with the node's epilogue fused
// (kpass_kernel); across processes the pass writes this process's node
// totals, then the allreduce and the epilogue kernel.
void Engine::kmeans_iter(Round& R, int it, int max_iters, hipStream_t stream) {
  const bool last = it == max_iters - 1;
  const int kind = last ? PASS_KLAST : PASS_KMEANS;
  const int st = last ? ST_KLAST : ST_KMEANS;
  RoundArgs& ra = R.ra;
  ra.it = it;
  const double bytes_all = 3.0 * (double)R.total;   // (exact per node: finish_round)
  timed_begin(stream);
  launch_kpass(kind, ra, (int)R.ntiles, stream);
  tmark("kpass");
  timed_end(st, bytes_all, stream);
  if (timing_) R.km_events.push_back({pending_.size() - 1, it});
  if (ra.tot_mode == TOT_ALLREDUCE) {
    timed_begin(stream);
    allreduce_totals(R.nl, stream);
    launch_epilogue(kind, ra, R.nr, stream);
    timed_end(ST_EPILOGUE, 0.0, stream);
  }
}

bool Engine::loop_ok(const Round& R) const {
  // (one workgroup per record on one CU: a 2-means pass costs it ~0.1 us per
  // 1000 points of VALU work, so only small records in rounds of at most one
  // record per CU beat the ~11 us of a kpass launch per iteration)
  if (kloop_max_ == 0 || nshard_ != 1 || cross_process() || R.root || R.nr > num_cus_) return false;
  for (int a = 0; a < R.nl; ++a) {
    const int id = R.order[a];
    if (nodes_[id].buf == BUF_IN) return false;   // (a root's packed / BGR24 frame)
    if (segs_[id].len > kloop_max_ || R.tend[a] - R.tbeg[a] > (int32_t)kLoopMaxTiles) return false;
  }
  return true;
}

// Rounds kloop does not take (records above kloop_max_ points) whose tiles
// all fit the device's resident workgroups: every 2-means iteration in one
// kpersist_kernel launch (its records' workgroups must be co-resident: at
// most kPersistWgsPerCu pass workgroups per CU -- the kernel's occupancy is
// at least that -- whatever else runs).
bool Engine::persist_ok(const Round& R) const {
  if (!persist_ || nshard_ != 1 || cross_process() || R.root || R.ntiles > (size_t)kPersistWgsPerCu * num_cus_)
    return false;
  return persist_ok_layout(R);
}

bool Engine::persist_ok_layout(const Round& R) const {
  for (int a = 0; a < R.nl; ++a)
    if (nodes_[R.order[a]].buf == BUF_IN) return false;   // (a root's packed / BGR24 frame)
  return true;
}

size_t Engine::max_record_tiles(const Round& R) const {
  size_t m = 1;
  for (int r = 0; r < R.nr && r < (int)R.tbeg.size() && r < (int)R.tend.size(); ++r)
    m = std::max<size_t>(m, (size_t)(R.tend[r] - R.tbeg[r]));
  return m;
}

void Engine::kmeans_loop(Round& R, int max_iters, hipStream_t stream, int kind) {
  if (kind == 2) ++last_persist_rounds;
  else ++last_loop_rounds;
  timed_begin(stream);
  if (kind == 2) launch_kpersist(R.ra, (int)R.ntiles, max_iters, stream);
  else launch_kloop(R.ra, R.nr, max_iters, stream);
  tmark(kind == 2 ? "kpersist" : "kloop");
  timed_end(ST_KLOOP, 0.0, stream);
  if (timing_) R.loop_event = (long)pending_.size() - 1;
}

// Wait for a round's split epilogue, run its 2-means iterations if any record
// is still active (host-polled, `lookahead_` launched past the one awaited),
// then take its results: children nodes, segments, the parents' tiles.
int Engine::finish_round(int ri, int max_iters, hipStream_t stream, bool speculate, int successor) {
  Round& R = rounds_[ri];   // (rounds_ is a deque: enqueueing below keeps R valid)
  const int S = nshard_;
  const double tw0 = tr_wait_us_;
  wait_round_ = ri;   // (named by wait_status's diagnostics)
  const double tf0 = trace_ ? host_us() : 0.0;
  const uint64_t* stat = h_stat_ + (size_t)R.par * cap_stat_;
  const NodeResult* res = h_res_ + (size_t)R.par * cap_res_;
  int launched = 0, known = 0;
  bool all_proven = false;
  // Late rounds (small records): every 2-means iteration in one launch,
  // waited for on the status word of iteration max_iters - 1
  // (kpersist_kernel, the same contract, for rounds of larger records)
  int loop = !fixed_point_ ? 0 : loop_ok(R) ? 1 : persist_ok(R) ? 2 : 0;
  // a round too big for kpersist's co-residency bound (its tiles) may still
  // take it once the split status says how few records are active: its
  // final records' workgroups exit at once, so the active records' tiles are
  // what must fit.  Then the speculative first iterations are not launched.
  const bool persist_later = fixed_point_ && loop == 0 && persist_ && nshard_ == 1 && !cross_process() &&
                             !R.root && persist_ok_layout(R);
  if (persist_later) speculate = false;
  // Nothing else queued behind this round (a frame's last rounds): its first
  // 2-means iterations go in before its split status is known -- a record
  // final at the split makes them exit at once (~4 us each); C3's last round
  // needs them and otherwise waited ~15 us for the host to see the status.
  if (speculate && fixed_point_) {
    if (loop) {
      kmeans_loop(R, max_iters, stream, loop);
      launched = max_iters;
    } else {
      for (; launched < max_iters && launched <= lookahead_; ++launched) kmeans_iter(R, launched, max_iters, stream);
    }
  }
  uint32_t split_active = 0;
  if (fixed_point_) {
    split_active = wait_status(stat + max_iters, R.seq, stream);
    all_proven = split_active == 0;
  }
  if (persist_later && !all_proven && (size_t)split_active * max_record_tiles(R) <= (size_t)kPersistWgsPerCu * num_cus_)
    loop = 2;
  if (R.planned) {   // the plan's counts equal the host's mirror of its layout
    const uint32_t* hc = h_counts_ + 4 * R.par;
    const uint32_t ab = __atomic_load_n(hc + 2, __ATOMIC_ACQUIRE);
    DQ_CHECK(ab == 0, "a finished planned round was aborted or overflowed");
    DQ_CHECK(__atomic_load_n(hc + 0, __ATOMIC_ACQUIRE) == (uint32_t)R.ntiles &&
                 __atomic_load_n(hc + 1, __ATOMIC_ACQUIRE) == (uint32_t)R.nptiles,
             "plan_kernel's tile counts differ from the host's mirror");
  }
  debug_host_delay();
  R.kmeans = !all_proven;
  // A planned successor queued behind this round aborts when a record it
  // splits is still active after the split epilogue (nearly always so when
  // 2-means runs).  Then every remaining iteration goes in now (a record final
  // earlier makes them exit at once, ~2 us each) and the successor is planned
  // again right behind them: the GPU moves on without waiting for the host to
  // see the last iteration (~25 us per 2-means round).  The re-plan cancels
  // itself if the first plan ran after all; run() keeps whichever is live.
  int replan = -1;
  if (!all_proven && successor >= 0 && eager_replan_) {
    if (loop && launched == 0) {
      kmeans_loop(R, max_iters, stream, loop);
      launched = max_iters;
    }
    for (; launched < max_iters; ++launched) kmeans_iter(R, launched, max_iters, stream);
    const std::vector<int32_t> pl = rounds_[successor].plist;
    for (int32_t a : pl) frames_[nodes_[R.order[a]].frame].splits_queued -= 2;   // (re-counted below)
    replan = enqueue_planned_round(ri, pl, max_iters, stream, rounds_[successor].dcounts);
  }
  if (!all_proven && loop) {
    if (launched == 0) {
      kmeans_loop(R, max_iters, stream, loop);
      launched = max_iters;
    }
    DQ_CHECK(wait_status(stat + (max_iters - 1), R.seq, stream) == 0, "kloop / kpersist left a record active");
    all_proven = true;   // (every record final: the loop below has nothing to wait for)
  }
  while (!all_proven) {
    while (launched < max_iters && launched <= known + lookahead_) {
      kmeans_iter(R, launched, max_iters, stream);
      ++launched;
    }
    const uint32_t act = wait_status(stat + known, R.seq, stream);
    ++known;
    if (act == 0) break;
    DQ_CHECK(known < max_iters, "nodes still active after the last 2-means iteration");
  }
  debug_host_delay();
  const double tp0 = trace_ ? host_us() : 0.0;
  const int nl = R.nl;
  // Every record's result carries the round's tag, stored after its other
  // words: read a record only once its tag is there (bounded by the stream
  // draining).  Then check the device's view of the round against the
  // host's: the record's points (the layout mirror) and, below the root, the
  // node's own mean / variance the round ran with.
  for (int r = 0; r < R.nr; ++r) {
    const uint32_t* tag = &res[r].tag;
    for (uint64_t spin = 0; __atomic_load_n(tag, __ATOMIC_ACQUIRE) != (uint32_t)R.seq; ++spin) {
      __builtin_ia32_pause();
      if ((spin & 0xFFFF) == 0xFFFF && hipStreamQuery(stream) == hipSuccess &&
          __atomic_load_n(tag, __ATOMIC_ACQUIRE) != (uint32_t)R.seq)
        die("node result", __FILE__, __LINE__, "a record's result never arrived");
    }
    const int a = r / S;
    const Node& nd = nodes_[R.order[a]];
    bool ok = res[r].len_local == seg(R.order[a], r % S).len;
    if (!R.root)
      for (int c = 0; c < 3; ++c)
        ok = ok && std::memcmp(&res[r].tm[c], &nd.mean[c], 8) == 0 && std::memcmp(&res[r].tv[c], &nd.var[c], 8) == 0;
    if (!ok) {
      char msg[200];
      std::snprintf(msg, sizeof msg, "round seq %llu (%s) record %d: device and host views differ (len %u vs %u)",
                    (unsigned long long)R.seq, R.planned ? "planned" : "host", r, res[r].len_local,
                    seg(R.order[a], r % S).len);
      die("round check", __FILE__, __LINE__, msg);
    }
  }
  // points actually swept: iteration `it` reads a node iff it is not final
  // before it (done_it <= 0: final at the last iteration, or it < done_it)
  auto swept_in = [&](int it) {
    uint64_t px = 0;
    for (int a = 0; a < nl; ++a) {
      const int di = res[a * S].done_it;
      if (!res[a * S].proven && (di <= 0 || it < di))
        for (int sh = 0; sh < S; ++sh) px += seg(R.order[a], sh).len;
    }
    return px;
  };
  auto swept_bytes = [&](int it) {
    double bytes = 0.0;
    for (int a = 0; a < nl; ++a) {
      const int di = res[a * S].done_it;
      if (!res[a * S].proven && (di <= 0 || it < di))
        for (int sh = 0; sh < S; ++sh) bytes += point_bytes(R.order[a]) * seg(R.order[a], sh).len;
    }
    return bytes;
  };
  last_points_full += R.total * (uint64_t)((R.root ? 2 : 1) + max_iters);
  last_points_swept += R.total * (uint64_t)(R.root ? 2 : 1);
  for (int it = 0; it < max_iters; ++it) last_points_swept += swept_in(it);
  if (timing_) {
    DQ_HIP(hipStreamSynchronize(stream));
    for (auto& e : R.km_events) {
      pending_[e.first].bytes = swept_bytes(e.second);
      pending_[e.first].units = (double)swept_in(e.second);
    }
    if (R.loop_event >= 0) {   // kloop reads every active record's points once
      pending_[R.loop_event].bytes = swept_bytes(0);
      pending_[R.loop_event].units = (double)swept_in(0);
    }
    collect_timing();
  }

  if (R.stats_only)   // written by PS_LATE iff the node or its sibling was active after its split
    for (int a = 0; a + 1 < nl; a += 2) {
      const bool written = !(res[a * S].proven && res[(a + 1) * S].proven);
      nodes_[R.order[a]].points = written;
      nodes_[R.order[a + 1]].points = written;
    }
  for (int a = 0; a < nl; ++a) {
    const int id = R.order[a];
    const NodeResult& r = res[a * S];   // global results: every record agrees
    if (R.root) {
      for (int c = 0; c < 3; ++c) { nodes_[id].mean[c] = r.tm[c]; nodes_[id].var[c] = r.tv[c]; }
      // the cut the INIT epilogue chose on the device, same comparisons
      double maxv = r.tv[0], cut = r.tm[0];
      int axis = 0;
      if (maxv < r.tv[1]) { maxv = r.tv[1]; axis = 1; cut = r.tm[1]; }
      if (maxv < r.tv[2]) { axis = 2; cut = r.tm[2]; }
      nodes_[id].axis = (int16_t)axis;
      nodes_[id].thr = (int16_t)split_threshold(cut);
    }
    Node co, cn;
    const int io = (int)nodes_.size();
    {
      const Node& p = nodes_[id];
      co.frame = cn.frame = p.frame;
      co.parent = cn.parent = id;
      co.w = r.ow;
      cn.w = r.nw;
      for (int c = 0; c < 3; ++c) {
        co.mean[c] = r.om[c];
        cn.mean[c] = r.nm[c];
        co.var[c] = r.ov[c];
        cn.var[c] = r.nv[c];
      }
      co.tse = r.tse_old;
      cn.tse = r.tse_new;
      cn.glen = r.n_new;
      co.glen = p.glen - r.n_new;
      co.buf = cn.buf = child_buf(p.buf);
      for (int c = 0; c < 3; ++c) {
        co.lo[c] = cn.lo[c] = p.lo[c];
        co.hi[c] = cn.hi[c] = p.hi[c];
      }
      if (r.proven) {   // the halves are the cut's: v_axis < thr | >= thr
        co.hi[p.axis] = (int16_t)std::min<int>(p.hi[p.axis], p.thr - 1);
        cn.lo[p.axis] = (int16_t)std::max<int>(p.lo[p.axis], p.thr);
      }
    }
    nodes_.push_back(co);
    nodes_.push_back(cn);
    segs_.resize((size_t)(io + 2) * S);
    nodes_[id].cursors_pending = R.stats_only && r.proven;   // (PS_STATS counts no cursors)
    for (int sh = 0; sh < S; ++sh) {
      Seg& ps = seg(id, sh);
      ps.dnode = R.dn + a * S + sh;
      ps.dtiles = R.dt + R.tbeg[a * S + sh];
      ps.dwparts = R.ra.wparts + (size_t)R.tbeg[a * S + sh] * kTileWaves;
      ps.rec = a * S + sh;
      ps.ntiles = R.tend[a * S + sh] - R.tbeg[a * S + sh];
      const uint32_t n_new = res[a * S + sh].n_new_local;
      const uint32_t n_old = ps.len - n_new;
      Seg& so = seg(io, sh);
      Seg& sn = seg(io + 1, sh);
      so.off = ps.off;
      so.len = n_old;
      sn.off = ps.off + n_old;
      sn.len = n_new;
    }
    Node& pp = nodes_[id];
    pp.child_old = io;
    pp.child_new = io + 1;
    pp.expanded = true;
    pp.queued = false;
  }
  if (trace_rounds_) {
    const double tp1 = host_us();
    std::fprintf(stderr,
                 "divquant-hip round %s: nodes=%d records=%d tiles=%zu parttiles=%zu bytes=%zu "
                 "enq->finish %.1fus (wait %.1f, 2-means its %d) post=%.1fus%s\n",
                 R.planned ? "planned" : "host", nl, R.nr, R.ntiles, R.nptiles, R.bytes,
                 tf0 - R.t_enq, tr_wait_us_ - tw0, launched, tp1 - tp0, R.kmeans ? " kmeans" : "");
  }
  return replan;
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
    f.trace.push_back((int64_t)nodes_[x].glen);
    f.trace.push_back((int64_t)nodes_[cn].glen);
    f.leaf[f.old_index] = co;
    f.leaf[f.new_index] = cn;
    if (f.new_index == k - 1) { ++f.new_index; return; }     // :823-832
    // STEP 4 (:876-887): max TSE above DBL_MIN, lowest index among equals;
    // if none qualifies old_index stays (the old half is split again).
    auto push = [&](double tse, int idx, int node) {
      f.heap.push_back({{tse, -idx}, node});
      std::push_heap(f.heap.begin(), f.heap.end());
    };
    if (nodes_[co].tse > DBL_MIN) push(nodes_[co].tse, f.old_index, co);
    if (nodes_[cn].tse > DBL_MIN) push(nodes_[cn].tse, f.new_index, cn);
    // drop stale entries (a leaf index now holding another node)
    while (!f.heap.empty() && f.leaf[-f.heap.front().first.second] != f.heap.front().second) {
      std::pop_heap(f.heap.begin(), f.heap.end());
      f.heap.pop_back();
    }
    if (!f.heap.empty()) f.old_index = -f.heap.front().first.second;
    ++f.new_index;
  }
}

// Next round's nodes of a frame: the node the replay waits for plus every
// unexpanded leaf among the top r = (splits left) of the greedy order -- a
// leaf outside the current top r can never be picked in the remaining splits.
// Nodes already queued in an enqueued round are left out.
void Engine::next_active(FrameState& f, std::vector<int>* active) {
  if (f.need < 0) return;
  const size_t r = (size_t)(f.job->k - f.new_index);
  if (!nodes_[f.need].queued) active->push_back(f.need);
  // the valid leaves of the greedy order, then its top r (keys are unique)
  top_.clear();
  for (const auto& e : f.heap)
    if (f.leaf[-e.first.second] == e.second) top_.push_back(e);
  if (top_.size() > r) {
    std::nth_element(top_.begin(), top_.begin() + r, top_.end(),
                     [](const HeapEnt& a, const HeapEnt& b) { return b < a; });
    top_.resize(r);
  }
  for (const auto& e : top_)
    if (!nodes_[e.second].expanded && !nodes_[e.second].queued && e.second != f.need)
      active->push_back(e.second);
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
    if (last) last_sizes[0] = (int64_t)(job.n_global ? job.n_global : job.n);
  } else {
    for (int ic = 0; ic < k; ++ic) {
      const Node& nd = nodes_[f.leaf[ic]];
      if (last) {
        for (int c = 0; c < 3; ++c) last_means[3 * ic + c] = nd.mean[c];
        last_sizes[ic] = (int64_t)nd.glen;
      }
      if (nd.glen > 0) {   // round, then shift back up (:1030, :1050-1052)
        const uint32_t sh = (uint32_t)(8 - job.num_bits);
        const uint32_t R = (uint32_t)(uint8_t)(nd.mean[0] + 0.5) << sh;
        const uint32_t G = (uint32_t)(uint8_t)(nd.mean[1] + 0.5) << sh;
        const uint32_t B = (uint32_t)(uint8_t)(nd.mean[2] + 0.5) << sh;
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
  tr_entry_t0_ = trace_ ? host_us() : 0.0;
  DQ_HIP(hipSetDevice(device_));
  if (!stream) stream = stream_;
  debug_ = debug_flags();
  if (debug_ & kDebugArenaCheck) check_arena_zero(stream);
  if (debug_ & kDebugFreshArena) {   // (nothing of this engine in flight: the previous run synced)
    for (auto& c : arena_) DQ_HIP(hipFree(c.first));
    arena_.clear();
    arena_hw_.clear();
  }

  frames_.assign(nframes, FrameState());
  nodes_.clear();
  segs_.clear();
  arena_chunk_ = 0;   // the previous run's tables are dead (its launches were drained)
  arena_used_ = 0;
  // (the arena is zero here: cleared behind the previous run's last kernel)
  last_rounds = 0;
  last_points_swept = 0;
  last_points_full = 0;
  last_cursor_fixes = 0;
  nshard_ = jobs[0].nshard;
  DQ_CHECK(nshard_ >= 1 && nshard_ <= kMaxShard, "shards per frame must be in [1, 8]");
  const int S = nshard_;
  size_t total = 0, align_need = 0;
  for (int i = 0; i < nframes; ++i) {
    FrameJob& j = jobs[i];
    DQ_CHECK(j.n > 0, "num_points must be > 0 (DivQuantCluster.cpp:211)");
    DQ_CHECK(j.k > 0, "num_colors must be > 0 (DivQuantCluster.cpp:229)");
    DQ_CHECK(j.d_in && j.ct, "null buffer");
    DQ_CHECK(j.nshard == S, "every frame of a batch must have the same shard count");
    DQ_CHECK(j.n_global == 0 || j.n_global >= j.n, "n_global < n");
    DQ_CHECK(j.n_global == 0 || j.n_global == j.n || cross_process(),
             "n_global > n needs a communicator (dq_hip_comm_init)");
    DQ_CHECK(!j.bgr || (S == 1 && (j.n_global == 0 || j.n_global == j.n)), "BGR24 frames are one shard");
    FrameState& f = frames_[i];
    f.job = &j;
    // shard boundaries: whole rows when the width is known, else 4-point multiples
    for (int sh = 0; sh <= S; ++sh) {
      uint64_t b;
      if (j.width > 0 && j.n % j.width == 0) {
        const uint64_t rows = j.n / j.width;
        b = (rows * (uint64_t)sh / S) * j.width;
      } else {
        b = ((uint64_t)j.n * sh / S) & ~(uint64_t)3;
      }
      if (sh == S) b = j.n;
      if (sh < S) f.first[sh] = (uint32_t)b;
      if (sh > 0) f.n[sh - 1] = (uint32_t)b - f.first[sh - 1];
    }
    for (int sh = 0; sh < S; ++sh) {
      // planar shards start 16-point aligned, 16 points of slack after each
      // (the sweeps' 16-B plane loads)
      f.base[sh] = (uint32_t)total;
      total += align16(f.n[sh]) + 16;
      const uint32_t* p = j.d_in + f.first[sh];
      if (j.bgr) {   // 48-B sweep vectors: 16-B aligned, no vector past the frame's end
        if (((uintptr_t)j.d_in & 15) != 0 || (j.n & 15) != 0) align_need += bgr_words(j.n);
      } else if (((uintptr_t)p & 15) != 0 || (f.n[sh] & 3) != 0) {
        align_need += align4(f.n[sh]) + 4;
      }
    }
  }
  DQ_CHECK(total < (1ull << 32), "batch larger than 2^32 points");
  for (int i = 0; i < nframes; ++i)
    for (int sh = 0; sh < S; ++sh)   // partition stores use 32-bit byte offsets
      DQ_CHECK(frames_[i].n[sh] < (1u << 29), "a frame shard holds at most 2^29 points");
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
    const uint64_t ng = j.n_global ? j.n_global : j.n;
    // get_double_scale (DivQuantMapColors.cpp:205-220), on the whole frame
    f.s = 1.0 / (std::ceil(1 / 1.0) * std::ceil((double)ng / 1.0));
    Node root;
    Seg root_seg[kMaxShard];
    root.frame = i;
    root.w = 1.0;          // :329
    root.glen = ng;
    root.buf = BUF_IN;
    if (j.bgr) {
      f.in[0] = j.d_in;
      if (((uintptr_t)j.d_in & 15) != 0 || (j.n & 15) != 0) {   // aligned copy, zero tail to 16 points
        const size_t w = bgr_words(j.n);
        uint8_t* dst = reinterpret_cast<uint8_t*>(d_align_ + aoff);
        DQ_HIP(hipMemcpyAsync(dst, j.d_in, (size_t)j.n * 3, hipMemcpyDeviceToDevice, stream));
        DQ_HIP(hipMemsetAsync(dst + (size_t)j.n * 3, 0, w * 4 - (size_t)j.n * 3, stream));
        f.in[0] = d_align_ + aoff;
        aoff += w;
      }
      root_seg[0].off = 0;
      root_seg[0].len = f.n[0];
    }
    for (int sh = 0; sh < S && !j.bgr; ++sh) {
      const uint32_t* p = j.d_in + f.first[sh];
      f.in[sh] = p;
      if (((uintptr_t)p & 15) != 0 || (f.n[sh] & 3) != 0) {   // 16-B loads may read up to align4(n)
        DQ_HIP(hipMemcpyAsync(d_align_ + aoff, p, (size_t)f.n[sh] * 4, hipMemcpyDeviceToDevice, stream));
        f.in[sh] = d_align_ + aoff;
        aoff += align4(f.n[sh]) + 4;
      }
      root_seg[sh].off = 0;
      root_seg[sh].len = f.n[sh];
    }
    f.leaf.assign(j.k, -1);
    f.leaf[0] = (int)nodes_.size();
    nodes_.push_back(root);
    for (int sh = 0; sh < S; ++sh) segs_.push_back(root_seg[sh]);
    if (j.k > 1) active.push_back(f.leaf[0]);
  }

  const double t_run0 = trace_ ? host_us() : 0.0;
  tr_wait_us_ = tr_build_us_ = tr_replay_us_ = 0.0;
  tr_log_.clear();
  tmark("run");
  last_planned = last_aborted = 0;
  last_loop_rounds = 0;
  last_persist_rounds = 0;
  {   // this run's capacities (nothing in flight now)
    size_t rec_cap = 64, px = 0;
    for (int i = 0; i < nframes; ++i) {
      rec_cap += 2 * (size_t)jobs[i].k * S;
      px += jobs[i].n;
    }
    const size_t tiles_cap = px / kSweep + rec_cap * (size_t)node_tiles_ + 64;
    ensure_round(rec_cap, tiles_cap, 0, 0, max_iters, stream);
    if (tot_mode() == TOT_ALLREDUCE) ensure_totals(rec_cap / S + 64, stream);
  }
  rounds_.clear();
  // Rounds in flight, oldest first.  While the oldest is the only one, the
  // next is planned on the device before its results exist; the host then
  // finishes the oldest (waits, 2-means iterations if needed, results),
  // replays the greedy order, and enqueues a host-built round for whatever
  // the replay needs that no enqueued round covers.
  std::deque<int> q;
  if (!active.empty()) q.push_back(enqueue_host_round(active, true, max_iters, stream));
  std::vector<int32_t> plist;
  while (!q.empty()) {
    const int ri = q.front();
    if (q.size() == 1 && plan_list(ri, &plist)) q.push_back(enqueue_planned_round(ri, plist, max_iters, stream));
    const int succ = q.size() >= 2 && rounds_[q[1]].planned && rounds_[q[1]].prev == ri ? q[1] : -1;
    tmark("finish:begin");
    const int replan = finish_round(ri, max_iters, stream, q.size() == 1 && speculate_kmeans_, succ);
    tmark("finish:end");
    q.pop_front();
    last_rounds++;
    if (rounds_[ri].planned) last_planned++;
    if (!q.empty() && rounds_[q.front()].planned && rounds_[q.front()].prev == ri && rounds_[ri].kmeans) {
      // The plan ran after ri's split epilogue: if a listed record was still
      // active then, it aborted its round.  (ri's 2-means launches came
      // after the plan in stream order, so its counts are visible now.)
      const int pi = q.front();
      const uint32_t ab = __atomic_load_n(h_counts_ + 4 * rounds_[pi].par + 2, __ATOMIC_ACQUIRE);
      DQ_CHECK(ab != 2, "plan_kernel: tables above the round's capacity");
      if (ab == 1) {
        q.pop_front();
        last_aborted++;
        if (replan >= 0) {   // already planned again behind ri's iterations
          q.push_front(replan);
        } else {
          const std::vector<int32_t> pl = rounds_[pi].plist;
          for (int32_t a : pl) frames_[nodes_[rounds_[ri].order[a]].frame].splits_queued -= 2;
          q.push_front(enqueue_planned_round(ri, pl, max_iters, stream));
        }
      }
      // (ab == 0 with a re-plan: the re-plan cancels itself on the device;
      // the split accounting moved to it is the first plan's)
    }
    for (int p : q)
      if (rounds_[p].planned && rounds_[p].prev == ri) assign_planned(p);
    active.clear();
    const double tr0 = trace_ ? host_us() : 0.0;
    for (auto& f : frames_) {
      if (f.job->k <= 1 || (f.need < 0 && f.new_index >= f.job->k)) continue;
      replay(f);
      next_active(f, &active);
    }
    if (trace_) tr_replay_us_ += host_us() - tr0;
    if (!active.empty()) q.push_back(enqueue_host_round(active, false, max_iters, stream));
  }
  const double t_clu = trace_ ? host_us() : 0.0;
  // The next run's planned rounds find their blocks zero: clear what this run
  // used, behind the last round's kernels -- here, before the host's colour
  // table work, so the clear runs while the host dedups instead of behind the
  // map (at the next run's start it delayed the first round by ~8 us).
  for (size_t c = 0; c < arena_.size(); ++c)
    if (arena_hw_[c] > 0) {
      launch_zero(arena_[c].first, arena_hw_[c], stream);   // (chunks and allocations: 256-B multiples)
      arena_hw_[c] = 0;
    }

  tmark("zero");
  for (int i = 0; i < nframes; ++i) finish_frame(frames_[i], i == nframes - 1);
  tmark("finish_frame");

  if (dedup_map) {
    std::vector<MapJob> mj;
    std::vector<uint32_t> table;
    for (auto& f : frames_) {
      FrameJob& j = *f.job;
      // First-occurrence colortable dedup (quant_util.cpp:93-118) with a flat
      // open-addressing set (a node-allocating unordered_set cost ~100 us per
      // 8-frame call); slot value = colour + 1, 0 = empty.
      size_t cap = 16;
      while (cap < 2 * (size_t)j.k_out) cap <<= 1;
      table.assign(cap, 0u);
      int m = 0;
      for (int i = 0; i < j.k_out; ++i) {
        const uint32_t c = j.ct[i];
        size_t h = (size_t)((c * 2654435761u) >> 7) & (cap - 1);
        while (table[h] != 0 && table[h] != c + 1) h = (h + 1) & (cap - 1);
        if (table[h] == 0) {
          table[h] = c + 1;
          j.ct[m++] = c;
        }
      }
      j.k_out = m;
      if (j.d_out)   // every shard's rows with the frame's palette
        for (int sh = 0; sh < S; ++sh)
          if (f.n[sh] > 0) mj.push_back(MapJob{f.in[sh], f.n[sh], j.d_out + f.first[sh], j.ct, m, j.bgr});
    }
    if (!mj.empty()) map_many(mj.data(), (int)mj.size(), stream, false);
    tmark("map:enqueued");
  }
  // Synchronous on return: lookahead launches of the last round may still be
  // queued, and they read the caller's input.
  const double ts0 = trace_ ? host_us() : 0.0;
  sync_stream(stream);
  tmark("synced");
  if (trace_) tr_mapsync_us_ = host_us() - ts0;
  collect_timing();
  if (trace_) {
    const double t_end = host_us();
    std::string lg;
    char buf[64];
    for (auto& e : tr_log_) {
      std::snprintf(buf, sizeof buf, " %s@%.1f", e.first, e.second - tr_entry_t0_);
      lg += buf;
    }
    std::fprintf(stderr, "divquant-hip trace: launches%s\n", lg.c_str());
    std::fprintf(stderr, "divquant-hip trace: map prep %.1fus, map launch+sync %.1fus\n",
                 tr_mapprep_us_, tr_mapsync_us_);
    std::fprintf(stderr,
                 "divquant-hip trace: frames=%d shards=%d rounds=%d entry->first launch %.1fus "
                 "cluster=%.1fus (build %.1f, wait %.1f, replay %.1f) map+sync=%.1fus total=%.1fus\n",
                 nframes, S, last_rounds, tr_first_us_, t_clu - t_run0, tr_build_us_, tr_wait_us_,
                 tr_replay_us_, t_end - t_clu, t_end - tr_entry_t0_);
  }
}

// ---------------------------------------------------------------------------
// Partition cursors of a node finalised at a PS_STATS round's split (that
// partition counts none): its split decision's per-(tile, wave) counts over
// its points and the cursor scan, into its round's tiles -- what the
// children's chunk walk would have left there.
void Engine::fix_cursors(int id, hipStream_t stream) {
  for (int sh = 0; sh < nshard_; ++sh) {
    const Seg& sg = seg(id, sh);
    RoundArgs fa{};
    fa.tiles = const_cast<Tile*>(sg.dtiles);
    fa.nodes = const_cast<DevNode*>(sg.dnode) - sg.rec;
    fa.wparts = sg.dwparts;
    fa.parts = d_parts_;
    fa.plane = cap_px_;
    launch_fix_cursors(fa, sg.ntiles, stream);
  }
  nodes_[id].cursors_pending = false;
  last_cursor_fixes++;
}

// ---------------------------------------------------------------------------
// The colour table's scratch (dq_weighted.hip launch_color_table).
void Engine::ensure_color_scratch(uint32_t n, hipStream_t stream) {
  const size_t need_scratch = color_table_scratch_bytes(n);
  if (need_scratch > cap_wscratch_) {
    DQ_HIP(hipStreamSynchronize(stream));
    if (d_wscratch_) DQ_HIP(hipFree(d_wscratch_));
    DQ_HIP(hipMalloc(&d_wscratch_, need_scratch));
    cap_wscratch_ = need_scratch;
  }
}

// calc_color_table for a host caller: the points staged (the reference reads
// inPixels[ic + ir*numRows] whatever numPixels says, :124 -- the staged range
// ends at the last index it reads), gathered when decimated or 2-D, the
// device colour table, the records back.
uint32_t Engine::color_table(const uint32_t* h_in, uint32_t rows, uint32_t cols, uint32_t dec, uint32_t* h_colors,
                             double* h_weights, hipStream_t stream) {
  DQ_HIP(hipSetDevice(device_));
  if (!stream) stream = stream_;
  DQ_CHECK(dec >= 1, "dec_factor >= 1");
  if (rows == 0 || cols == 0) return 0;
  const uint64_t nr = (rows + (uint64_t)dec - 1) / dec, nc = (cols + (uint64_t)dec - 1) / dec;
  const uint64_t last = (nc - 1) * dec + (nr - 1) * (uint64_t)dec * rows;
  DQ_CHECK(last < 0xFFFFFFF0ull && nr * nc <= 0xFFFFFFF0ull, "too many points");
  const uint32_t m = (uint32_t)(nr * nc);
  stage_in(h_in, (uint32_t)(last + 1), stream);
  ensure_color_scratch(m, stream);
  ensure_pixels(2 * (size_t)m + 8);
  const uint32_t* pts = staged_in();
  if (nr != 1 || nc != last + 1) {   // not the plain run [0, m)
    launch_cut_gather(staged_in(), d_p1_, (uint32_t)nr, (uint32_t)nc, dec, rows, 0, 0, 0, stream);
    pts = d_p1_;
  }
  uint32_t nu = 0;
  const int rc = launch_color_table(pts, m, d_wscratch_, cap_wscratch_, reinterpret_cast<uint64_t*>(d_p0_), &nu,
                                    stream);
  DQ_CHECK(rc == 0, "colour table failed");
  std::vector<uint64_t> rec(nu);
  if (nu) DQ_HIP(hipMemcpyAsync(rec.data(), d_p0_, (size_t)nu * 8, hipMemcpyDeviceToHost, stream));
  DQ_HIP(hipStreamSynchronize(stream));
  // norm_factor (:184), the weight norm_factor * count (:195)
  const double norm = 1.0 / (std::ceil((double)rows / (double)dec) * std::ceil((double)cols / (double)dec));
  for (uint32_t i = 0; i < nu; ++i) {
    h_colors[i] = (uint32_t)rec[i];
    h_weights[i] = norm * (double)(uint32_t)(rec[i] >> 32);
  }
  return nu;
}

// ---------------------------------------------------------------------------
// The weighted path: quant_varpart_fast's calc_color_table dedup and
// DivQuantCluster<false,*,true> (DivQuantCluster.cpp:1133-1138, :1163-1166).
// Rounds as run(): a round splits every node the greedy replay needs, its
// passes' folds exact parallel folds over tiles (dq_weighted.hip), the host
// replaying the reference's greedy order over the results.  An input the
// one-workgroup kernel holds takes it instead (run_weighted_small).
void Engine::run_weighted(FrameJob& job, int max_iters, bool dedup_map, hipStream_t stream) {
  DQ_CHECK(job.n > 0, "num_points must be > 0 (DivQuantCluster.cpp:211)");
  DQ_CHECK(job.k > 0, "num_colors must be > 0 (DivQuantCluster.cpp:229)");
  DQ_CHECK(job.d_in && job.ct, "null buffer");
  DQ_CHECK(max_iters >= 1, "max_iters < 1 is not supported (the reference never writes member[] then)");
  DQ_CHECK(job.nshard == 1 && (job.n_global == 0 || job.n_global == job.n),
           "the weighted path takes whole frames in one process");
  DQ_HIP(hipSetDevice(device_));
  DQ_CHECK(job.num_bits >= 1 && job.num_bits <= 8 && job.dec >= 1, "num_bits in [1,8], dec_factor >= 1");
  if (!stream) stream = stream_;
  // calc_color_table's points: every dec-th row and column of the rows x cols
  // frame (the whole input when dec = 1 and rows = 1), cut to num_bits
  const uint64_t rows = job.rows ? job.rows : 1, cols = job.cols ? job.cols : job.n;
  const uint64_t nr = (rows + job.dec - 1) / job.dec, nc = (cols + job.dec - 1) / job.dec;
  const bool gather = job.num_bits != 8 || job.dec != 1 || rows != 1 || cols != job.n;
  if (gather) {   // the reference's index ic + ir*numRows must stay inside in[0..n)
    const uint64_t last = (nc - 1) * job.dec + (nr - 1) * job.dec * rows;
    DQ_CHECK(last < job.n, "calc_color_table would read past the input (index ic + ir*numRows, :124)");
    DQ_CHECK(nr * nc <= 0xFFFFFFF0ull, "too many points");
  }
  const uint32_t n = gather ? (uint32_t)(nr * nc) : job.n;
  last_wsmall_prof.clear();
  // a small input (a superpixel region: ClusteringSegmentation.cpp:1779-1803)
  // in one launch; more colours than it holds -> the rounds below
  if (wsmall_ && !gather && n <= kWsMaxN && job.k <= kWsMaxK && run_weighted_small(job, max_iters, dedup_map, stream))
    return;
  ensure_round(2 * (size_t)job.k + 64, 1024, 0, 0, max_iters, stream);   // staging, results
  ensure_color_scratch(n, stream);
  // P0 / P1 hold the points' 8-B records (colour | count << 32): 2 words each
  ensure_pixels(2 * (size_t)n + 8);
  // norm_factor = 1 / (ceil(numRows / dec) * ceil(numCols / dec)) (:184)
  const double norm = 1.0 / (std::ceil((double)rows / (double)job.dec) * std::ceil((double)cols / (double)job.dec));
  const uint32_t* pts = job.d_in;
  if (gather) {   // cut_bits (DivQuantUni.cpp:28-100) + the decimated walk, into P1 (free until the rounds)
    const uint32_t sh = (uint32_t)(8 - job.num_bits);
    launch_cut_gather(job.d_in, d_p1_, (uint32_t)nr, (uint32_t)nc, (uint32_t)job.dec, (uint32_t)rows,
                      sh, sh, sh, stream);
    pts = d_p1_;
  }
  uint32_t nu = 0;
  // (the root's points, in calc_color_table's order, straight into P0: the
  // colour table has read P1's decimated points by then)
  const int rc = launch_color_table(pts, n, d_wscratch_, cap_wscratch_, reinterpret_cast<uint64_t*>(d_p0_), &nu,
                                    stream);
  DQ_CHECK(rc == 0, "colour table failed");

  frames_.assign(1, FrameState());
  nodes_.clear();
  segs_.clear();
  nshard_ = 1;
  last_rounds = last_planned = last_aborted = 0;
  last_points_swept = last_points_full = 0;
  last_seq_tiles = 0;
  FrameState& f = frames_[0];
  f.job = &job;
  f.s = 0.0;
  Node root;
  root.w = 1.0;        // :329
  root.glen = nu;
  root.buf = BUF_P0;
  f.leaf.assign(job.k, -1);
  f.leaf[0] = 0;
  nodes_.push_back(root);
  Seg rs;
  rs.off = 0;
  rs.len = nu;
  segs_.push_back(rs);
  std::vector<int> active;
  if (job.k > 1) active.push_back(0);
  std::vector<NodeResult> res;
  std::vector<WTile> tiles;
  while (!active.empty()) {
    // the round's records and tiles (kWTile points each, at least one per node)
    const int nn = (int)active.size();
    tiles.clear();
    for (int a = 0; a < nn; ++a) {
      const Seg& sg = seg(active[a], 0);
      for (uint32_t o = 0; o == 0 || o < sg.len; o += kWTile)
        tiles.push_back(WTile{a, sg.off + o, sg.off + std::min<uint32_t>(sg.len, o + kWTile), 0u});
    }
    const int nt = (int)tiles.size();
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_tiles = al((size_t)nn * sizeof(WState));
    const size_t up_bytes = o_tiles + al((size_t)nt * sizeof(WTile));
    const size_t o_tsum = up_bytes;
    const size_t o_tpre = o_tsum + al((size_t)nt * 8 * sizeof(double));
    const size_t o_fold = o_tpre + al((size_t)nt * 8 * sizeof(double));
    const size_t o_quick = o_fold + al((size_t)nt * kWCh * sizeof(WFold));
    const size_t o_pbase = o_quick + al((size_t)nt * kWCh * sizeof(WQuick));
    const size_t o_gen = o_pbase + al((size_t)nt * 2 * sizeof(uint32_t));
    const size_t o_res = o_gen + al((size_t)nt * sizeof(uint32_t));
    const size_t o_act = o_res + al((size_t)nn * sizeof(NodeResult));
    const size_t bytes = o_act + 256;
    if (bytes > cap_wnodes_) {
      DQ_HIP(hipStreamSynchronize(stream));
      if (d_wnodes_) DQ_HIP(hipFree(d_wnodes_));
      cap_wnodes_ = std::max<size_t>(bytes, 1 << 20);
      DQ_HIP(hipMalloc(&d_wnodes_, cap_wnodes_));
    }
    if (stage_pending_) {
      DQ_HIP(hipEventSynchronize(stage_ev_));
      stage_pending_ = false;
    }
    if (up_bytes > cap_stage_tab_) {
      DQ_HIP(hipHostFree(h_stage_));
      const size_t c = std::max<size_t>(up_bytes, 2 * cap_stage_tab_);
      DQ_HIP(hipHostMalloc((void**)&h_stage_, c, hipHostMallocCoherent | hipHostMallocMapped));
      DQ_HIP(hipHostGetDevicePointer((void**)&d_stage_view_, h_stage_, 0));
      cap_stage_tab_ = c;
    }
    WState* hw = reinterpret_cast<WState*>(h_stage_);
    int t = 0;
    bool has_root = false;
    for (int a = 0; a < nn; ++a) {
      Node& nd = nodes_[active[a]];
      const Seg& sg = seg(active[a], 0);
      WState& w = hw[a];
      std::memset(&w, 0, sizeof w);
      w.src = reinterpret_cast<const uint64_t*>(nd.buf == BUF_P0 ? d_p0_ : d_p1_);
      w.dst = reinterpret_cast<uint64_t*>(nd.buf == BUF_P0 ? d_p1_ : d_p0_);
      w.off = sg.off;
      w.len = sg.len;
      w.tile_begin = t;
      while (t < nt && tiles[t].node == a) ++t;
      w.tile_end = t;
      w.root = active[a] == 0 ? 1 : 0;
      has_root |= w.root != 0;
      w.tw = nd.w;
      for (int c = 0; c < 3; ++c) {
        w.tm[c] = nd.mean[c];
        w.tv[c] = nd.var[c];
        w.box_lo[c] = nd.lo[c];
        w.box_hi[c] = nd.hi[c];
      }
      if (!w.root) {   // the cut (:388-403); the root's comes from its init folds
        double maxv = nd.var[0], cut = nd.mean[0];
        int axis = 0;
        if (maxv < nd.var[1]) { maxv = nd.var[1]; axis = 1; cut = nd.mean[1]; }
        if (maxv < nd.var[2]) { axis = 2; cut = nd.mean[2]; }
        w.axis = axis;
        w.cut = cut;
      }
      w.done_it = -1;
    }
    std::memcpy(h_stage_ + o_tiles, tiles.data(), (size_t)nt * sizeof(WTile));
    char* db = static_cast<char*>(d_wnodes_);
    launch_upload(db, d_stage_view_, up_bytes, stream);
    DQ_HIP(hipEventRecord(stage_ev_, stream));
    stage_pending_ = true;
    // the round's results and its "still active" word in host-coherent memory
    // (written by the kernels; read by the host after a stream sync -- no
    // copies; the stream is idle here: the previous round ended with a sync)
    const size_t wres_bytes = 64 + (size_t)nn * sizeof(NodeResult);
    if (wres_bytes > cap_wres_) {
      if (h_wres_) DQ_HIP(hipHostFree(h_wres_));
      cap_wres_ = std::max<size_t>(wres_bytes, 64 + 256 * sizeof(NodeResult));
      DQ_HIP(hipHostMalloc((void**)&h_wres_, cap_wres_, hipHostMallocCoherent | hipHostMallocMapped));
      DQ_HIP(hipHostGetDevicePointer((void**)&d_wres_view_, h_wres_, 0));
    }
    volatile uint32_t* h_active = reinterpret_cast<volatile uint32_t*>(h_wres_);
    *h_active = 0u;
    WArgs wa;
    wa.nodes = reinterpret_cast<WState*>(db);
    wa.tiles = reinterpret_cast<const WTile*>(db + o_tiles);
    wa.norm = norm;
    wa.tsum = reinterpret_cast<double*>(db + o_tsum);
    wa.tpre = reinterpret_cast<double*>(db + o_tpre);
    wa.fold = reinterpret_cast<WFold*>(db + o_fold);
    wa.quick = reinterpret_cast<WQuick*>(db + o_quick);
    wa.pbase = reinterpret_cast<uint32_t*>(db + o_pbase);
    wa.gen = reinterpret_cast<uint32_t*>(db + o_gen);
    wa.res = reinterpret_cast<NodeResult*>(d_wres_view_ + 64);
    wa.active = reinterpret_cast<uint32_t*>(d_wres_view_);
    wa.nn = nn;
    wa.ntiles = nt;
    wa.max_iters = max_iters;
    wa.fixed_point = fixed_point_ ? 1 : 0;
    wa.it = 0;
    wa.pad = 0;
    if (has_root) launch_wpass(WP_INIT, wa, stream);   // (a round holding the root holds only it)
    launch_wpass(WP_SPLIT, wa, stream);
    // 2-means passes only when some split is not proven final at the split
    DQ_HIP(hipStreamSynchronize(stream));
    if (*h_active != 0) {
      for (int it = 0; it < max_iters; ++it) {
        wa.it = it;
        launch_wpass(WP_KM, wa, stream);
      }
    }
    launch_wfinish(wa, stream);
    DQ_HIP(hipStreamSynchronize(stream));
    res.resize(nn);
    std::memcpy(res.data(), h_wres_ + 64, (size_t)nn * sizeof(NodeResult));
    last_rounds++;
    for (int a = 0; a < nn; ++a) {
      const int id = active[a];
      const NodeResult& r = res[a];
      last_points_swept += seg(id, 0).len;
      last_seq_tiles += (uint32_t)r.pad;
      if (id == 0)
        for (int c = 0; c < 3; ++c) { nodes_[0].mean[c] = r.tm[c]; nodes_[0].var[c] = r.tv[c]; }
      {   // the cut the split ran with (the children's boxes)
        const Node& n = nodes_[id];
        double maxv = n.var[0], cut = n.mean[0];
        int axis = 0;
        if (maxv < n.var[1]) { maxv = n.var[1]; axis = 1; cut = n.mean[1]; }
        if (maxv < n.var[2]) { axis = 2; cut = n.mean[2]; }
        nodes_[id].axis = (int16_t)axis;
        nodes_[id].thr = (int16_t)split_threshold(cut);
      }
      DQ_CHECK(r.n_new_local == (uint32_t)r.n_new, "weighted partition count differs from the fold count");
      Node co, cn;
      const int io = (int)nodes_.size();
      const Node& p = nodes_[id];
      co.frame = cn.frame = 0;
      co.parent = cn.parent = id;
      co.w = r.ow;
      cn.w = r.nw;
      for (int c = 0; c < 3; ++c) {
        co.mean[c] = r.om[c];
        cn.mean[c] = r.nm[c];
        co.var[c] = r.ov[c];
        cn.var[c] = r.nv[c];
        co.lo[c] = cn.lo[c] = p.lo[c];
        co.hi[c] = cn.hi[c] = p.hi[c];
      }
      if (r.proven) {   // the halves are the cut's: v_axis < thr | >= thr
        co.hi[p.axis] = (int16_t)std::min<int>(p.hi[p.axis], p.thr - 1);
        cn.lo[p.axis] = (int16_t)std::max<int>(p.lo[p.axis], p.thr);
      }
      co.tse = r.tse_old;
      cn.tse = r.tse_new;
      cn.glen = r.n_new;
      co.glen = p.glen - r.n_new;
      co.buf = cn.buf = child_buf(p.buf);
      nodes_.push_back(co);
      nodes_.push_back(cn);
      segs_.resize((size_t)(io + 2));
      Seg& ps = seg(id, 0);
      Seg& so = seg(io, 0);
      Seg& sn = seg(io + 1, 0);
      so.off = ps.off;
      so.len = ps.len - (uint32_t)r.n_new;
      sn.off = ps.off + so.len;
      sn.len = (uint32_t)r.n_new;
      Node& pp = nodes_[id];
      pp.child_old = io;
      pp.child_new = io + 1;
      pp.expanded = true;
    }
    active.clear();
    if (!(f.need < 0 && f.new_index >= job.k)) {
      replay(f);
      next_active(f, &active);
    }
  }
  finish_frame(f, true);
  if (dedup_map) {
    size_t cap = 16;
    while (cap < 2 * (size_t)job.k_out) cap <<= 1;
    std::vector<uint32_t> table(cap, 0u);
    int m = 0;
    for (int i = 0; i < job.k_out; ++i) {   // first-occurrence dedup (quant_util.cpp:93-118)
      const uint32_t c = job.ct[i];
      size_t h = (size_t)((c * 2654435761u) >> 7) & (cap - 1);
      while (table[h] != 0 && table[h] != c + 1) h = (h + 1) & (cap - 1);
      if (table[h] == 0) {
        table[h] = c + 1;
        job.ct[m++] = c;
      }
    }
    job.k_out = m;
    if (job.d_out) map(job.d_in, job.n, job.d_out, job.ct, m, stream);
  }
  DQ_HIP(hipStreamSynchronize(stream));
}

// The whole weighted call in one workgroup (dq_wsmall.hip): colour table,
// DivQuantCluster<false,*,true> split by split, final centres, dedup and --
// for at most kWsMapMax colours -- the map.  Returns false when the input has
// more colours than the kernel holds (nothing written; the caller runs the
// rounds).  Synchronous, as run_weighted.
bool Engine::run_weighted_small(FrameJob& job, int max_iters, bool dedup_map, hipStream_t stream) {
  if (!h_wsres_) {
    DQ_HIP(hipHostMalloc((void**)&h_wsres_, sizeof(WSmallResult), hipHostMallocCoherent | hipHostMallocMapped));
    DQ_HIP(hipHostGetDevicePointer((void**)&d_wsres_, h_wsres_, 0));
    DQ_HIP(hipMalloc((void**)&d_wsmap_, sizeof(WsMapTab)));
  }
  __atomic_store_n(&h_wsres_->status, 0u, __ATOMIC_RELEASE);
  WSmallArgs wa;
  wa.px = job.d_in;
  wa.out = dedup_map ? job.d_out : nullptr;
  wa.res = d_wsres_;
  wa.maptab = d_wsmap_;
  // norm_factor = 1 / (ceil(numRows / dec) * ceil(numCols / dec)) (:184), rows = dec = 1
  wa.norm = 1.0 / (std::ceil(1.0 / 1.0) * std::ceil((double)job.n / 1.0));
  wa.n = job.n;
  wa.k = job.k;
  wa.max_iters = max_iters;
  wa.fixed_point = fixed_point_ ? 1 : 0;
  DQ_HIP(launch_wsmall(wa, stream));
  sync_stream(stream);
  const WSmallResult& r = *h_wsres_;
  const uint32_t st = __atomic_load_n(&r.status, __ATOMIC_ACQUIRE);
  if (st == 2) return false;
  DQ_CHECK(st == 1, st == 3 ? "small weighted kernel: partition count differs from the fold count"
                            : "small weighted kernel: no result");
  const int k = job.k;
  job.k_out = (int)r.k_raw;
  job.num_empty = (int)r.num_empty;
  for (uint32_t i = 0; i < r.k_raw; ++i) job.ct[i] = r.ct[i];
  last_means.assign(r.means, r.means + (size_t)k * 3);
  last_sizes.assign(r.sizes, r.sizes + k);
  last_trace.assign(r.trace, r.trace + (size_t)(k - 1) * 4);
  last_rounds = 1;
  last_planned = last_aborted = 0;
  last_points_swept = last_points_full = 0;
  last_seq_tiles = 0;
  last_wsmall_prof.assign(r.prof, r.prof + 8);
  if (dedup_map) {   // first-occurrence dedup (quant_util.cpp:93-118), as run_weighted
    int m = 0;
    for (int i = 0; i < job.k_out; ++i) {
      bool seen = false;
      for (int j = 0; j < m && !seen; ++j) seen = job.ct[j] == job.ct[i];
      if (!seen) job.ct[m++] = job.ct[i];
    }
    DQ_CHECK(m == (int)r.m, "small weighted kernel: dedup count differs from the host's");
    job.k_out = m;
    if (job.d_out && !r.mapped) map(job.d_in, job.n, job.d_out, job.ct, m, stream);
  }
  return true;
}

// A batch of weighted calls (superpixel regions): one launch, one workgroup
// per region the small-path kernel holds; the results read back as
// run_weighted_small's, the rest through run_weighted.
int Engine::run_weighted_regions(FrameJob* jobs, int njobs, int max_iters, hipStream_t stream) {
  DQ_HIP(hipSetDevice(device_));
  if (!stream) stream = stream_;
  std::vector<int> take, rest;
  for (int i = 0; i < njobs; ++i) {
    const FrameJob& j = jobs[i];
    const bool plain = j.num_bits == 8 && j.dec == 1 && (j.rows == 0 || j.rows == 1) && (j.cols == 0 || j.cols == j.n);
    if (wsmall_ && plain && j.n >= 1 && j.n <= kWsMaxN && j.k >= 1 && j.k <= kWsMaxK) take.push_back(i);
    else rest.push_back(i);
  }
  const size_t nb = take.size();
  if (nb > cap_wb_) {
    DQ_HIP(hipStreamSynchronize(stream));
    if (h_wbargs_) DQ_HIP(hipHostFree(h_wbargs_));
    if (h_wbres_) DQ_HIP(hipHostFree(h_wbres_));
    cap_wb_ = std::max<size_t>(nb, 64);
    DQ_HIP(hipHostMalloc((void**)&h_wbargs_, cap_wb_ * sizeof(WSmallArgs), hipHostMallocCoherent | hipHostMallocMapped));
    DQ_HIP(hipHostGetDevicePointer((void**)&d_wbargs_, h_wbargs_, 0));
    DQ_HIP(hipHostMalloc((void**)&h_wbres_, cap_wb_ * sizeof(WSmallResult), hipHostMallocCoherent | hipHostMallocMapped));
    DQ_HIP(hipHostGetDevicePointer((void**)&d_wbres_, h_wbres_, 0));
  }
  for (size_t t = 0; t < nb; ++t) {
    const FrameJob& j = jobs[take[t]];
    WSmallArgs& wa = h_wbargs_[t];
    wa.px = j.d_in;
    wa.out = j.d_out;
    wa.res = d_wbres_ + t;
    wa.maptab = nullptr;
    wa.norm = 1.0 / (std::ceil(1.0 / 1.0) * std::ceil((double)j.n / 1.0));   // (:184), rows = dec = 1
    wa.n = j.n;
    wa.k = j.k;
    wa.max_iters = max_iters;
    wa.fixed_point = fixed_point_ ? 1 : 0;
    __atomic_store_n(&h_wbres_[t].status, 0u, __ATOMIC_RELEASE);
  }
  if (nb > 0) {
    DQ_HIP(launch_wsmall_batch(d_wbargs_, (int)nb, stream));
    sync_stream(stream);
  }
  int taken = 0;
  for (size_t t = 0; t < nb; ++t) {
    FrameJob& job = jobs[take[t]];
    const WSmallResult& r = h_wbres_[t];
    const uint32_t st = __atomic_load_n(&r.status, __ATOMIC_ACQUIRE);
    if (st == 2) {   // more colours than the kernel holds
      rest.push_back(take[t]);
      continue;
    }
    DQ_CHECK(st == 1, st == 3 ? "small weighted kernel: partition count differs from the fold count"
                              : "small weighted kernel: no result");
    ++taken;
    job.k_out = (int)r.k_raw;
    job.num_empty = (int)r.num_empty;
    for (uint32_t i = 0; i < r.k_raw; ++i) job.ct[i] = r.ct[i];
    int m = 0;   // first-occurrence dedup (quant_util.cpp:93-118), as run_weighted
    for (int i = 0; i < job.k_out; ++i) {
      bool seen = false;
      for (int q = 0; q < m && !seen; ++q) seen = job.ct[q] == job.ct[i];
      if (!seen) job.ct[m++] = job.ct[i];
    }
    DQ_CHECK(m == (int)r.m, "small weighted kernel: dedup count differs from the host's");
    job.k_out = m;
    if (job.d_out && !r.mapped) map(job.d_in, job.n, job.d_out, job.ct, m, stream);
  }
  for (int i : rest) run_weighted(jobs[i], max_iters, true, stream);
  return taken;
}

// ---------------------------------------------------------------------------
// RCCL communicator (row-tile sharding across processes, one GPU each).
void Engine::comm_unique_id(char id[128]) {
  ncclUniqueId u;
  DQ_CHECK(ncclGetUniqueId(&u) == ncclSuccess, "ncclGetUniqueId failed");
  std::memcpy(id, u.internal, 128);
}

void Engine::comm_init(int nranks, int rank, const char id[128]) {
  DQ_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / world size");
  DQ_HIP(hipSetDevice(device_));
  comm_destroy();
  ncclUniqueId u;
  std::memcpy(u.internal, id, 128);
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRank(&c, nranks, u, rank);
  if (r != ncclSuccess) die("ncclCommInitRank", __FILE__, __LINE__, ncclGetErrorString(r));
  comm_ = c;
  comm_ranks_ = nranks;
  comm_rank_ = rank;
}

void Engine::comm_destroy() {
  if (!comm_) return;
  ncclCommDestroy((ncclComm_t)comm_);
  comm_ = nullptr;
  comm_ranks_ = 1;
  comm_rank_ = 0;
}

// The per-pass exchange of row-tile sharding: the logical nodes' 8 u64
// totals summed over all processes, in place, on the round's stream.
void Engine::allreduce_totals(int nlogical, hipStream_t stream) {
  if (loop_) {
    loop_->allreduce(loop_rank_, d_tot_, (size_t)nlogical * 8, stream);
    return;
  }
  const ncclResult_t r = ncclAllReduce(d_tot_, d_tot_, (size_t)nlogical * 8, ncclUint64, ncclSum,
                                       (ncclComm_t)comm_, stream);
  if (r != ncclSuccess) die("ncclAllReduce", __FILE__, __LINE__, ncclGetErrorString(r));
}

// ---------------------------------------------------------------------------
// Loopback collective (tests; dq_engine.h).  One allreduce, per rank r:
//   1. record in_ev[r] behind r's producers (nodesum / kpass) on r's stream;
//   2. barrier: every rank has recorded its in_ev and published its buffer;
//   3. r's stream waits for every in_ev, sums all ranks' buffers into its own
//      scratch, records rd_ev[r];
//   4. barrier: every rank has enqueued its reads (and waits on in_ev);
//   5. r's stream waits for every rd_ev, copies its scratch into its buffer.
// Every stream wait refers to an event recorded before a barrier the waiting
// host thread passed after it, so all dependencies point back in enqueue
// order (no cycle, whichever hardware queues the streams share), and an
// event is re-recorded only after every wait on its previous record was
// enqueued (in_ev before barrier 4 of the previous collective, rd_ev before
// barrier 2 of the next).
Loopback::Loopback(int nranks, int device) : n_(nranks) {
  DQ_CHECK(nranks >= 1 && nranks <= kMaxShard, "loopback ranks must be in [1, 8]");
  DQ_HIP(hipSetDevice(device));
  log.assign(n_, {});
  in_ev_.resize(n_);
  rd_ev_.resize(n_);
  bufs_.assign(n_, nullptr);
  scratch_.assign(n_, nullptr);
  counts_.assign(n_, 0);
  cap_.assign(n_, 0);
  for (int r = 0; r < n_; ++r) {
    DQ_HIP(hipEventCreateWithFlags(&in_ev_[r], hipEventDisableTiming));
    DQ_HIP(hipEventCreateWithFlags(&rd_ev_[r], hipEventDisableTiming));
  }
}

void Loopback::reset_log() {
  for (auto& l : log) l.clear();
}

void Loopback::barrier(int rank, const char* where) {
  std::unique_lock<std::mutex> l(mu_);
  const uint64_t g = gen_;
  if (++arrived_ == n_) {
    arrived_ = 0;
    ++gen_;
    cv_.notify_all();
    return;
  }
  const auto limit = std::chrono::duration<double>(kLoopbackTimeoutS);
  if (!cv_.wait_for(l, limit, [&] { return gen_ != g; })) {
    char msg[200];
    std::snprintf(msg, sizeof msg, "rank %d waited %.0f s at %s of collective #%zu (%d of %d ranks there)",
                  rank, kLoopbackTimeoutS, where, log[rank].size(), arrived_, n_);
    die("loopback collective", __FILE__, __LINE__, msg);
  }
}

void Loopback::allreduce(int rank, uint64_t* buf, size_t count, hipStream_t stream) {
  log[rank].push_back(count);
  if (count > cap_[rank]) {   // (first use: a sized scratch, no stream is waiting on it yet)
    DQ_HIP(hipStreamSynchronize(stream));
    if (scratch_[rank]) DQ_HIP(hipFree(scratch_[rank]));
    cap_[rank] = std::max<size_t>(count, (size_t)1 << 16);
    DQ_HIP(hipMalloc((void**)&scratch_[rank], cap_[rank] * sizeof(uint64_t)));
  }
  bufs_[rank] = buf;
  counts_[rank] = count;
  DQ_HIP(hipEventRecord(in_ev_[rank], stream));
  barrier(rank, "entry");
  SumSrcs src{};
  for (int q = 0; q < n_; ++q) {
    if (counts_[q] != count) {
      char msg[160];
      std::snprintf(msg, sizeof msg, "collective #%zu: rank %d has %zu elements, rank %d %zu", log[rank].size(),
                    rank, count, q, counts_[q]);
      die("loopback collective", __FILE__, __LINE__, msg);
    }
    src.p[q] = bufs_[q];
    if (q != rank) DQ_HIP(hipStreamWaitEvent(stream, in_ev_[q], 0));
  }
  launch_sum_u64(src, n_, scratch_[rank], count, stream);
  DQ_HIP(hipEventRecord(rd_ev_[rank], stream));
  barrier(rank, "reads");
  for (int q = 0; q < n_; ++q)
    if (q != rank) DQ_HIP(hipStreamWaitEvent(stream, rd_ev_[q], 0));
  DQ_HIP(hipMemcpyAsync(buf, scratch_[rank], count * sizeof(uint64_t), hipMemcpyDeviceToDevice, stream));
}

// ---------------------------------------------------------------------------
namespace {
// The palette sorted by R+G+B with std::sort and the reference comparator
// (DivQuantMapColors.cpp:227-238, :314-323) -- same algorithm, same input =>
// same tie order -- and the start-entry LUT from rounded midpoints (:331-383).
// Writes k sorted colours to pal and 766 LUT entries to lut.
void sorted_palette(const uint32_t* ct, int k, uint32_t* pal_out, uint16_t* lut_out) {
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
  for (int i = 0; i < k; ++i)
    pal_out[i] = ((uint32_t)pal[i].red << 16) | ((uint32_t)pal[i].green << 8) | (uint32_t)pal[i].blue;
  for (int v = 0; v < 766; ++v) lut_out[v] = (uint16_t)lut[v];
}

// Per-map block of the map staging: [LUT: 768 u16 | palette: k words,
// padded to 16 B], blocks packed; the staging starts with the MapTask table
// of the launch.
constexpr size_t kMapPal = 16384;
constexpr size_t kMapBlockWords = kMapPal + 768 / 2;
constexpr int kMapChunk = 16;   // tasks per batched launch (cell tables: 2.5 MB each)
}  // namespace

void Engine::ensure_map_stage(size_t nmaps) {
  if (nmaps <= cap_mapstage_ && h_mapstage_) return;
  if (map_pending_) {
    DQ_HIP(hipEventSynchronize(map_ev_));
    map_pending_ = false;
  }
  if (h_mapstage_) DQ_HIP(hipHostFree(h_mapstage_));
  if (d_mapstage_) DQ_HIP(hipFree(d_mapstage_));
  const size_t words = nmaps * (kMapBlockWords + sizeof(MapTask) / 4);
  DQ_HIP(hipHostMalloc((void**)&h_mapstage_, words * 4, hipHostMallocCoherent | hipHostMallocMapped));
  DQ_HIP(hipHostGetDevicePointer((void**)&d_mapstage_view_, h_mapstage_, 0));
  DQ_HIP(hipMalloc((void**)&d_mapstage_, words * 4));
  if (!map_ev_) DQ_HIP(hipEventCreateWithFlags(&map_ev_, hipEventDisableTiming));
  cap_mapstage_ = nmaps;
}

// map_colors_mps (DivQuantMapColors.cpp:243-539) for several (input, output,
// colortable) triples: host palettes for all of them, ONE upload, then ONE
// cell-build launch and ONE map launch per chunk of up to kMapChunk tasks,
// ONE synchronisation at the end.
void Engine::map_many(const MapJob* jobs, int njobs, hipStream_t stream, bool sync) {
  DQ_HIP(hipSetDevice(device_));
  if (!stream) stream = stream_;
  for (int i = 0; i < njobs; ++i) {
    DQ_CHECK(jobs[i].k > 0, "colormapSize must be > 0 (DivQuantMapColors.cpp:264)");
    DQ_CHECK(jobs[i].k <= (int)kMapPal, "colormapSize > 16384 is not supported by the LDS palette");
  }
  // A task maps at most kMapTaskMax pixels: map_lds_kernel stores through a
  // buffer resource whose byte range (4 n) must stay below 2^31.  Larger jobs
  // become consecutive tasks over the same colortable (they then share one
  // palette block and cell table, as a frame's row shards do).
  std::vector<MapJob> split;
  {
    bool big = false;
    for (int i = 0; i < njobs; ++i) big |= jobs[i].n > kMapTaskMax;
    if (big) {
      for (int i = 0; i < njobs; ++i)
        for (uint32_t o = 0; o == 0 || o < jobs[i].n; o += kMapTaskMax) {
          MapJob j = jobs[i];
          j.n = std::min<uint32_t>(kMapTaskMax, jobs[i].n - o);
          j.d_in = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(jobs[i].d_in) +
                                                     (size_t)o * (jobs[i].bgr ? 3 : 4));
          j.d_out = jobs[i].d_out + o;
          split.push_back(j);
        }
      jobs = split.data();
      njobs = (int)split.size();
    }
  }
  // BGR24 frames: map_lds_kernel reads them directly (K <= 1024, 8-B aligned
  // in, 16-B aligned out); otherwise they are packed first (bgr24_pack)
  std::vector<MapJob> packed;
  {
    int kmax_all = 0;
    bool any_bgr = false, any_staged = false;   // (a staged chunk runs map_kernel task by task)
    bool all_bgr = true;                        // (one launch maps one pixel format)
    for (int i = 0; i < njobs; ++i) {
      kmax_all = std::max(kmax_all, jobs[i].k);
      any_bgr |= jobs[i].bgr;
      all_bgr &= jobs[i].bgr;
      any_staged |= !jobs[i].bgr && (((uintptr_t)jobs[i].d_in & 15) != 0 || ((uintptr_t)jobs[i].d_out & 15) != 0);
    }
    if (any_bgr) {
      size_t need = 0;
      bool direct_all = kmax_all <= 1024 && use_lds_map_ && !any_staged && all_bgr;
      for (int i = 0; i < njobs; ++i)
        direct_all &= ((uintptr_t)jobs[i].d_in & 7) == 0 && ((uintptr_t)jobs[i].d_out & 15) == 0;
      auto direct = [&](const MapJob&) { return direct_all; };
      for (int i = 0; i < njobs; ++i)
        if (jobs[i].bgr && !direct(jobs[i])) need += align4(jobs[i].n) + 4;
      if (need > 0) {
        if (need > cap_bgr_pack_) {
          DQ_HIP(hipStreamSynchronize(stream));
          if (d_bgr_pack_) DQ_HIP(hipFree(d_bgr_pack_));
          DQ_HIP(hipMalloc((void**)&d_bgr_pack_, need * sizeof(uint32_t)));
          cap_bgr_pack_ = need;
        }
        packed.assign(jobs, jobs + njobs);
        size_t off = 0;
        for (MapJob& j : packed)
          if (j.bgr && !direct(j)) {
            launch_bgr24_pack(reinterpret_cast<const uint8_t*>(j.d_in), j.n, 1, 3 * j.n, d_bgr_pack_ + off, stream);
            j.d_in = d_bgr_pack_ + off;
            j.bgr = false;
            off += align4(j.n) + 4;
          }
        jobs = packed.data();
      }
    }
  }
  // the staging is reused: the previous map's upload must have run
  const double tm0 = trace_ ? host_us() : 0.0;
  if (map_pending_) {
    DQ_HIP(hipEventSynchronize(map_ev_));
    map_pending_ = false;
  }
  const double tm1 = trace_ ? host_us() : 0.0;
  const int chunk = std::min(njobs, kMapChunk);
  ensure_map_stage(chunk);
  if ((size_t)chunk > cap_cells_) {
    if (d_cell_rec_) DQ_HIP(hipFree(d_cell_rec_));
    if (d_cell_idx_) DQ_HIP(hipFree(d_cell_idx_));
    if (d_cell_c32_) DQ_HIP(hipFree(d_cell_c32_));
    DQ_HIP(hipMalloc((void**)&d_cell_rec_, (size_t)chunk * kCells * kCellRecWords * sizeof(uint32_t)));
    DQ_HIP(hipMalloc((void**)&d_cell_idx_, (size_t)chunk * kCells * kCellCap * sizeof(uint16_t)));
    DQ_HIP(hipMalloc((void**)&d_cell_c32_, (size_t)chunk * kCells * sizeof(uint32_t)));
    cap_cells_ = chunk;
  }
  if (num_cus_ == 0) {
    DQ_HIP(hipDeviceGetAttribute(&num_cus_, hipDeviceAttributeMultiprocessorCount, device_));
    num_cus_ = std::max(1, num_cus_);
  }
  for (int c0 = 0; c0 < njobs; c0 += chunk) {
    const int nt = std::min(chunk, njobs - c0);
    if (c0 > 0 && map_pending_) {   // staging reuse
      DQ_HIP(hipEventSynchronize(map_ev_));
      map_pending_ = false;
    }
    MapTask* ht = reinterpret_cast<MapTask*>(h_mapstage_);
    uint32_t* hblk0 = h_mapstage_ + (size_t)chunk * sizeof(MapTask) / 4;
    uint32_t* dblk0 = d_mapstage_ + (size_t)chunk * sizeof(MapTask) / 4;
    int kmax = 1;
    uint32_t nblocks = 0;
    std::vector<int> staged;   // tasks whose in/out needed aligned staging
    double ntot = 0;
    for (int t = 0; t < nt; ++t) {
      ntot += jobs[c0 + t].n;
      kmax = std::max(kmax, jobs[c0 + t].k);
    }
    // K <= 1024: the LDS-table map, one workgroup per CU over all tasks
    const bool lds_map = kmax <= 1024 && use_lds_map_;
    auto misaligned = [](const MapJob& j) {
      return !j.bgr && (((uintptr_t)j.d_in & 15) != 0 || ((uintptr_t)j.d_out & 15) != 0);
    };
    // Tasks with the same colortable (a frame's row shards) share one palette
    // block and one cell table: the table lists the first of each colortable
    // first (the cell build covers those only), the others after them (block
    // ranges follow table order).  Not with misaligned buffers (task by task).
    bool any_mis = false;
    for (int t = 0; t < nt; ++t) any_mis |= misaligned(jobs[c0 + t]);
    std::vector<int> order, first(nt, -1), slot(nt);
    for (int t = 0; t < nt && !any_mis; ++t)
      for (int u = 0; u < t; ++u)
        if (first[u] < 0 && jobs[c0 + u].ct == jobs[c0 + t].ct && jobs[c0 + u].k == jobs[c0 + t].k) {
          first[t] = u;
          break;
        }
    for (int t = 0; t < nt; ++t) if (first[t] < 0) order.push_back(t);
    const int nbuild = (int)order.size();
    for (int t = 0; t < nt; ++t) if (first[t] >= 0) order.push_back(t);
    for (int x = 0; x < nt; ++x) slot[order[x]] = x;
    size_t woff = 0;   // packed blocks
    std::vector<size_t> blk_off(nt), blk_words(nt);
    for (int x = 0; x < nt; ++x) {
      const int t = order[x];
      const MapJob& j = jobs[c0 + t];
      MapTask& m = ht[x];
      if (first[t] >= 0) {
        const MapTask& f = ht[slot[first[t]]];
        blk_off[x] = blk_off[slot[first[t]]];
        blk_words[x] = blk_words[slot[first[t]]];
        m.pal = f.pal;
        m.lut = f.lut;
        m.cell_rec = f.cell_rec;
        m.cell_idx = f.cell_idx;
        m.cell_c32 = f.cell_c32;
      } else {
        blk_off[x] = woff;
        blk_words[x] = 768 / 2 + (((size_t)j.k + 3) & ~(size_t)3);
        woff += blk_words[x];
        uint32_t* hb = hblk0 + blk_off[x];
        const uint32_t* db = dblk0 + blk_off[x];
        sorted_palette(j.ct, j.k, hb + 768 / 2, reinterpret_cast<uint16_t*>(hb));
        m.pal = db + 768 / 2;
        m.lut = reinterpret_cast<const uint16_t*>(db);
        m.cell_rec = d_cell_rec_ + (size_t)x * kCells * kCellRecWords;
        m.cell_idx = d_cell_idx_ + (size_t)x * kCells * kCellCap;
        m.cell_c32 = d_cell_c32_ + (size_t)x * kCells;
      }
      m.in = j.d_in;
      m.out = j.d_out;
      m.bgr = j.bgr ? 1 : 0;   // (aligned and K <= 1024: never staged)
      if (misaligned(j)) staged.push_back(x);   // (identity order)
      m.n = j.n;
      m.k = j.k;
      const uint32_t groups = j.n / 8;
      if (lds_map) {
        const uint32_t want = std::max<uint32_t>(1, (uint32_t)std::lround(num_cus_ * (double)j.n / ntot));
        m.grp_per_block = std::max<uint32_t>(1, (groups + want - 1) / want);
      } else {
        m.grp_per_block = map_groups_per_block(j.n);
      }
      m.block_begin = nblocks;
      nblocks += std::max<uint32_t>(1, (groups + m.grp_per_block - 1) / m.grp_per_block);
    }
    // misaligned in/out (the kernel uses 16-B accesses): aligned staging, one
    // task at a time through a private buffer
    size_t need = 0;
    for (int t : staged) need = std::max<size_t>(need, 2 * (align4(ht[t].n) + 4));
    if (need > cap_map_align_) {
      DQ_HIP(hipStreamSynchronize(stream));
      if (d_map_align_) DQ_HIP(hipFree(d_map_align_));
      DQ_HIP(hipMalloc((void**)&d_map_align_, need * sizeof(uint32_t)));
      cap_map_align_ = need;
    }
    const size_t bytes = (size_t)chunk * sizeof(MapTask) + woff * 4;
    if (trace_) tr_mapprep_us_ = host_us() - tm1;
    if (staged.empty()) {
      launch_upload(d_mapstage_, d_mapstage_view_, bytes, stream);
      const MapTask* dt = reinterpret_cast<const MapTask*>(d_mapstage_);
      timed_begin(stream);
      launch_build_cells(dt, nbuild, kmax, stream);
      timed_end(ST_CELLS, 0.0, stream);
      // (the staging-reuse event behind the map's kernels, as for round tables)
      double px = 0, mb = 0;   // pixels; bytes: 4 (BGR24: 3) read + 4 written per pixel
      for (int t = 0; t < nt; ++t) {
        px += ht[t].n;
        mb += (ht[t].bgr ? 7.0 : 8.0) * ht[t].n;
      }
      timed_begin(stream);
      if (lds_map) launch_map_lds(dt, nt, kmax, nblocks, ht[0].bgr != 0, stream);
      else launch_map(dt, nt, kmax, nblocks, stream);
      timed_end(ST_MAP, mb, stream, px);
      DQ_HIP(hipEventRecord(map_ev_, stream));
      map_pending_ = true;
    } else {
      // rare path: run the chunk task by task, staging misaligned buffers
      for (int t = 0; t < nt; ++t) {
        const MapJob& j = jobs[c0 + t];
        MapTask one = ht[t];
        const bool st = ((uintptr_t)j.d_in & 15) != 0 || ((uintptr_t)j.d_out & 15) != 0;
        const size_t want = align4(j.n) + 4;
        if (st) {
          DQ_HIP(hipMemcpyAsync(d_map_align_, j.d_in, (size_t)j.n * 4, hipMemcpyDeviceToDevice, stream));
          one.in = d_map_align_;
          one.out = d_map_align_ + want;
        }
        one.block_begin = 0;
        one.grp_per_block = map_groups_per_block(j.n);
        one.cell_rec = d_cell_rec_;
        one.cell_idx = d_cell_idx_;
        one.cell_c32 = d_cell_c32_;
        DQ_HIP(hipStreamSynchronize(stream));   // staging slot 0 reuse
        map_pending_ = false;
        ht[0] = one;
        if (t != 0) std::memmove(hblk0, hblk0 + blk_off[t], blk_words[t] * 4);
        ht[0].pal = dblk0 + 768 / 2;
        ht[0].lut = reinterpret_cast<const uint16_t*>(dblk0);
        launch_upload(d_mapstage_, d_mapstage_view_, (size_t)chunk * sizeof(MapTask) + blk_words[t] * 4,
                      stream);
        const MapTask* dt = reinterpret_cast<const MapTask*>(d_mapstage_);
        const uint32_t nb = std::max<uint32_t>(1, (j.n / 8 + one.grp_per_block - 1) / one.grp_per_block);
        timed_begin(stream);
        launch_build_cells(dt, 1, j.k, stream);
        timed_end(ST_CELLS, 0.0, stream);
        timed_begin(stream);
        launch_map(dt, 1, j.k, nb, stream);
        timed_end(ST_MAP, 8.0 * (double)j.n, stream, (double)j.n);
        if (st)
          DQ_HIP(hipMemcpyAsync(j.d_out, d_map_align_ + want, (size_t)j.n * 4, hipMemcpyDeviceToDevice, stream));
      }
    }
  }
  if (!sync) return;   // (run(): its end-of-run clear goes in first, then one sync)
  const double tm2 = trace_ ? host_us() : 0.0;
  sync_stream(stream);
  if (trace_) {
    tr_mapsync_us_ = host_us() - tm2;
    std::fprintf(stderr, "divquant-hip map: first sync %.1fus\n", tm1 - tm0);
  }
  collect_timing();
}

void Engine::map(const uint32_t* d_in, uint32_t n, uint32_t* d_out,
                 const uint32_t* ct, int k, hipStream_t stream) {
  MapJob j{d_in, n, d_out, ct, k};
  map_many(&j, 1, stream);
}

Engine& engine_for(int device, int lane) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, Engine*> engines;
  std::lock_guard<std::mutex> g(mu);
  auto it = engines.find({device, lane});
  if (it != engines.end()) return *it->second;
  Engine* e = new Engine(device);
  engines[{device, lane}] = e;
  return *e;
}

static std::atomic<int> g_lanes_override{0};

int batch_lanes() {
  static int lanes = [] {
    const char* v = getenv("DQ_HIP_LANES");
    // 3 lanes: 1.29 ms per 8 x 4K vs 1.33 with 2 (each lane's chain of
    // partition -> plan -> 2-means launches overlaps two others); 4 lanes
    // exceed HIP's default 4 hardware queues with the caller's stream (1.6 ms)
    // -- with GPU_MAX_HW_QUEUES >= 6 every lane's stream has a queue of its
    // own and 4 lanes win (1.21 -> 1.18-1.19 ms; 5 or 6 lanes: 1.64-1.75)
    const char* q = getenv("GPU_MAX_HW_QUEUES");
    const int dflt = q && atoi(q) >= 6 ? 4 : 3;
    return v && v[0] ? std::max(1, std::min(kMaxLanes, atoi(v))) : dflt;
  }();
  const int o = g_lanes_override.load();
  return o > 0 ? std::min(o, kMaxLanes) : lanes;
}

void set_batch_lanes(int lanes) { g_lanes_override.store(std::max(0, lanes)); }

static std::atomic<int> g_debug_flags{0};
void set_debug_flags(int flags) { g_debug_flags.store(flags); }
int debug_flags() { return g_debug_flags.load(); }

}  // namespace dq
