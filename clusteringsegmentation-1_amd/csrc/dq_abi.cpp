// dq_abi.cpp -- the exported surface of libdivquant_hip.so:
//   * the C ABI of include/dq_hip.h (device- and host-pointer entry points);
//   * the reference signatures of include/DivQuantHeader.h and
//     include/quant_util.h, implemented on top of it.
// The product path has no CPU fallback: without a HIP device every compute
// entry point aborts with a message.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/DivQuantHeader.h"
#include "../../include/dq_hip.h"
#include "../../include/quant_util.h"
#include "dq_engine.h"
#include "dq_weighted.h"

#include <rccl/rccl.h>
#include <map>
#include <tuple>

using dq::Engine;
using dq::engine_for;

namespace {

int current_device() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    dq::die("no HIP device", __FILE__, __LINE__,
            "libdivquant_hip has no CPU fallback; run on an MI355X (gfx950)");
  int d = 0;
  DQ_HIP(hipGetDevice(&d));
  return d;
}

bool quiet() {
  const char* q = std::getenv("DQ_HIP_QUIET");
  return q && *q && *q != '0';
}

// First-occurrence colortable dedup (quant_util.cpp:93-118).
uint32_t dedup_colortable(uint32_t* ct, uint32_t k) {
  std::unordered_set<uint32_t> seen;
  seen.reserve(k * 2 + 1);
  uint32_t m = 0;
  for (uint32_t i = 0; i < k; ++i)
    if (seen.insert(ct[i]).second) ct[m++] = ct[i];
  return m;
}

void report_empty(int num_empty) {
  if (num_empty) std::fprintf(stderr, "# empty clusters: %d\n", num_empty);   // :1067-1069
}

// Persistent host threads for the batch lanes 1..L-1 (a std::thread per lane
// per call cost tens of microseconds of every call's host time).  run()
// hands job(i) to worker i, runs job(0) on the caller and returns when all
// are done.  A worker reads the generation, the job and the lane count
// together under mu_ (run() publishes them together under mu_), so it runs
// each generation's job at most once; a thread starts with `seen` = the
// generation current when it was created.  Workers spin briefly on the
// generation word before sleeping on the condition variable.
class LaneWorkers {
 public:
  void run(int n, const std::function<void(int)>& job) {
    std::lock_guard<std::mutex> call(call_mu_);
    while ((int)threads_.size() < n - 1) {
      const int id = (int)threads_.size() + 1;
      const uint64_t g0 = gen_.load(std::memory_order_acquire);   // (no publish in flight: call_mu_)
      threads_.emplace_back([this, id, g0] { loop(id, g0); });
      threads_.back().detach();
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &job;
      nact_ = n;
      pending_.store(n - 1, std::memory_order_relaxed);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    job(0);
    for (uint64_t spin = 0; pending_.load(std::memory_order_acquire) != 0; ++spin) {
      if (spin < (1u << 16)) {
        __builtin_ia32_pause();
      } else {
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [this] { return pending_.load(std::memory_order_acquire) == 0; });
      }
    }
  }

 private:
  void loop(int id, uint64_t seen) {
    for (;;) {
      for (uint32_t spin = 0; gen_.load(std::memory_order_acquire) == seen && spin < (1u << 14); ++spin)
        __builtin_ia32_pause();
      const std::function<void(int)>* job;
      int n;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return gen_.load(std::memory_order_relaxed) != seen; });
        seen = gen_.load(std::memory_order_relaxed);   // the generation job_ / nact_ belong to
        job = job_;
        n = nact_;
      }
      if (id < n) {
        (*job)(id);
        if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
          std::lock_guard<std::mutex> l(mu_);
          done_cv_.notify_all();
        }
      }
    }
  }
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> pending_{0};
  const std::function<void(int)>* job_ = nullptr;
  int nact_ = 0;
  std::vector<std::thread> threads_;
};

// Events for one-shot cross-stream joins (a call's "inputs ready" mark, a
// NULL-stream call's completion), one per use: concurrent calls never share
// one (an event re-recorded by another call before a stream waited on it
// would order the wait after the wrong work).  A stream wait captures the
// event's state when it is enqueued, so the event returns to the pool as
// soon as every wait on it has been enqueued.
class EventPool {
 public:
  hipEvent_t get() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!free_.empty()) {
        hipEvent_t e = free_.back();
        free_.pop_back();
        return e;
      }
    }
    hipEvent_t e = nullptr;
    DQ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
  }
  void put(hipEvent_t e) {
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(e);
  }

 private:
  std::mutex mu_;
  std::vector<hipEvent_t> free_;
};

EventPool& events() {
  static EventPool* p = new EventPool();   // (never destroyed, like the engines)
  return *p;
}

// The stream a device-pointer entry runs on: the caller's, or (NULL) the
// engine's non-blocking stream made to wait for the legacy default stream
// first -- the caller's inputs may still be in flight there (a torch
// host-to-device copy on the default stream, say).
hipStream_t dev_stream(Engine& e, void* stream) {
  if (stream) return (hipStream_t)stream;
  hipEvent_t ev = events().get();
  DQ_HIP(hipEventRecord(ev, nullptr));
  DQ_HIP(hipStreamWaitEvent(e.stream(), ev, 0));
  events().put(ev);
  return e.stream();
}

// An asynchronous entry called with stream NULL ran on the engine's stream:
// order the legacy default stream after it, so work the caller queues there
// next (a framework's copy of the outputs) sees the results.
void join_default_stream(void* stream, hipStream_t used) {
  if (stream) return;
  hipEvent_t ev = events().get();
  DQ_HIP(hipEventRecord(ev, used));
  DQ_HIP(hipStreamWaitEvent(nullptr, ev, 0));
  events().put(ev);
}

LaneWorkers& lane_workers() {
  static LaneWorkers* w = new LaneWorkers();   // (never destroyed: its threads are detached)
  return *w;
}

}  // namespace

// =========================================================================
// C ABI (include/dq_hip.h)
// =========================================================================
extern "C" {

int dq_hip_abi_version(void) { return DQ_HIP_ABI_VERSION; }

int dq_hip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int dq_hip_cluster_dev(int device, const uint32_t* d_in, uint32_t n, uint32_t* k,
                       uint32_t* ct, int max_iters, void* stream) {
  if (!d_in || !k || !ct || n == 0 || *k == 0 || max_iters < 1) return -1;
  Engine& e = engine_for(device);
  std::lock_guard<std::mutex> g(e.mutex());
  dq::FrameJob j;
  j.d_in = d_in;
  j.n = n;
  j.k = (int)*k;
  j.ct = ct;
  e.run(&j, 1, max_iters, false, dev_stream(e, stream));
  *k = (uint32_t)j.k_out;
  return j.num_empty;
}

int dq_hip_quant_weighted_dev(int device, const uint32_t* d_in, uint32_t n, uint32_t* d_out,
                              uint32_t* k, uint32_t* ct, int max_iters, void* stream) {
  if (!d_in || !k || !ct || n == 0 || *k == 0 || max_iters < 1) return -1;
  Engine& e = engine_for(device);
  std::lock_guard<std::mutex> g(e.mutex());
  dq::FrameJob j;
  j.d_in = d_in;
  j.n = n;
  j.d_out = d_out;
  j.k = (int)*k;
  j.ct = ct;
  e.run_weighted(j, max_iters, d_out != nullptr, dev_stream(e, stream));
  *k = (uint32_t)j.k_out;
  return j.num_empty;
}

// Many weighted quant_recurse calls (the app's per-superpixel-region calls,
// ClusteringSegmentation.cpp:1779-1803) in one: region i = d_ins[i][0..ns[i])
// -> d_outs[i], K = ks[i], colortable at cts + i * ct_stride, its size at
// k_outs[i].  Returns the total of empty clusters, or < 0.
int dq_hip_quant_weighted_regions_dev(int device, int nregions, const uint32_t* const* d_ins, const uint32_t* ns,
                                      uint32_t* const* d_outs, const uint32_t* ks, uint32_t* cts,
                                      uint32_t ct_stride, uint32_t* k_outs, int max_iters, void* stream) {
  if (nregions < 0 || (nregions > 0 && (!d_ins || !ns || !ks || !cts || !k_outs)) || max_iters < 1) return -1;
  std::vector<dq::FrameJob> jobs((size_t)nregions);
  for (int i = 0; i < nregions; ++i) {
    if (!d_ins[i] || ns[i] == 0 || ks[i] == 0 || ks[i] > ct_stride) return -1;
    jobs[i].d_in = d_ins[i];
    jobs[i].n = ns[i];
    jobs[i].d_out = d_outs ? d_outs[i] : nullptr;
    jobs[i].k = (int)ks[i];
    jobs[i].ct = cts + (size_t)i * ct_stride;
  }
  Engine& e = engine_for(device);
  std::lock_guard<std::mutex> g(e.mutex());
  e.run_weighted_regions(jobs.data(), nregions, max_iters, dev_stream(e, stream));
  int empty = 0;
  for (int i = 0; i < nregions; ++i) {
    k_outs[i] = (uint32_t)jobs[i].k_out;
    empty += jobs[i].num_empty;
  }
  return empty;
}

static hipStream_t engine_stream(int device, void* stream);

int dq_hip_varpart_dev(int device, const uint32_t* d_in, uint32_t n, uint32_t rows, uint32_t cols,
                       uint32_t* k, uint32_t* ct, int num_bits, int dec_factor, int max_iters,
                       int uniq, void* stream) {
  if (!d_in || !k || !ct || n == 0 || *k == 0 || max_iters < 1 || num_bits < 1 || num_bits > 8 ||
      dec_factor < 1 || rows == 0 || cols == 0)
    return -1;
  // the reference's index ic + ir*numRows must stay inside the input (:124)
  const uint64_t nr = (rows + (uint64_t)dec_factor - 1) / dec_factor;
  const uint64_t nc = (cols + (uint64_t)dec_factor - 1) / dec_factor;
  if ((nc - 1) * dec_factor + (nr - 1) * dec_factor * (uint64_t)rows >= n) return -2;
  Engine& e = engine_for(device);
  std::lock_guard<std::mutex> g(e.mutex());
  dq::FrameJob j;
  j.d_in = d_in;
  j.n = n;
  j.k = (int)*k;
  j.ct = ct;
  j.num_bits = num_bits;
  j.dec = dec_factor;
  j.rows = rows;
  j.cols = cols;
  if (uniq && num_bits == 8 && dec_factor == 1) e.run(&j, 1, max_iters, false, dev_stream(e, stream));
  else e.run_weighted(j, max_iters, false, dev_stream(e, stream));
  *k = (uint32_t)j.k_out;
  return j.num_empty;
}

int dq_hip_cut_bits_dev(int device, const uint32_t* d_in, uint32_t n, uint32_t* d_out, int nbr,
                        int nbg, int nbb, void* stream) {
  if (!d_in || !d_out || nbr < 1 || nbr > 8 || nbg < 1 || nbg > 8 || nbb < 1 || nbb > 8) return -1;
  if (n == 0) return 0;
  hipStream_t st = engine_stream(device, stream);
  dq::launch_cut_gather(d_in, d_out, 1, n, 1, 1, (uint32_t)(8 - nbr), (uint32_t)(8 - nbg),
                        (uint32_t)(8 - nbb), st);
  join_default_stream(stream, st);
  return 0;
}

int dq_hip_map_dev(int device, const uint32_t* d_in, uint32_t n, uint32_t* d_out,
                   const uint32_t* ct, int k, void* stream) {
  if (!d_in || !d_out || !ct || k <= 0) return -1;
  if (n == 0) return 0;
  Engine& e = engine_for(device);
  std::lock_guard<std::mutex> g(e.mutex());
  e.map(d_in, n, d_out, ct, k, dev_stream(e, stream));
  return 0;
}

static bool block_hist_shape_ok(uint32_t w, uint32_t h, uint32_t dim, uint32_t bw, uint32_t bh) {
  // every block must hold a pixel (the reference asserts it, :468)
  return w > 0 && h > 0 && dim >= 1 && dim <= 4 && bw > 0 && bh > 0 &&
         (uint64_t)(bw - 1) * dim < w && (uint64_t)(bh - 1) * dim < h &&
         (uint64_t)w * h <= 0xFFFFFFFFull && (uint64_t)bw * bh < 0xFFFFFF00ull;
}

int dq_hip_block_hist_dev(int device, const uint32_t* d_in, uint32_t width, uint32_t height,
                          const uint32_t* palette, int npal, uint32_t dim, uint32_t block_w,
                          uint32_t block_h, uint32_t* d_quant, uint32_t* d_mode,
                          uint32_t* d_ndistinct, uint32_t* d_keys, uint32_t* d_counts,
                          void* stream) {
  if (!d_in || !palette || npal <= 0 || !d_quant || !d_mode || (!d_keys) != (!d_counts) ||
      !block_hist_shape_ok(width, height, dim, block_w, block_h))
    return -1;
  Engine& e = engine_for(device);
  std::lock_guard<std::mutex> g(e.mutex());
  hipStream_t st = dev_stream(e, stream);
  e.map(d_in, width * height, d_quant, palette, npal, st);
  // the tie queues are private to this call (stream-ordered allocation): the
  // kernels are still running when the call returns, and another call may
  // run on another stream meanwhile
  uint32_t* work = nullptr;
  DQ_HIP(hipMallocAsync((void**)&work, dq::block_hist_scratch_words(block_w, block_h) * 4, st));
  dq::BlockHistArgs a{d_quant, width, height, block_w, block_h, d_mode, d_ndistinct, d_keys, d_counts,
                      work, nullptr, 0};
  const int rc = dq::launch_block_hist(a, (int)dim, st);
  DQ_HIP(hipFreeAsync(work, st));
  join_default_stream(stream, st);
  return rc;
}

static bool bgr24_shape_ok(uint32_t width, uint32_t height, uint32_t stride) {
  return width > 0 && height > 0 && width <= 0xFFFFFFFFu / 3u && stride >= 3u * width &&
         (uint64_t)width * height <= 0xFFFFFFFFull;
}

static hipStream_t engine_stream(int device, void* stream) {
  Engine& e = engine_for(device);
  DQ_HIP(hipSetDevice(device));
  return dev_stream(e, stream);
}

int dq_hip_pack_bgr24_dev(int device, const uint8_t* d_bgr, uint32_t width, uint32_t height,
                          uint32_t stride, uint32_t* d_out, void* stream) {
  if (!d_bgr || !d_out || !bgr24_shape_ok(width, height, stride)) return -1;
  hipStream_t st = engine_stream(device, stream);
  dq::launch_bgr24_pack(d_bgr, width, height, stride, d_out, st);
  join_default_stream(stream, st);
  DQ_HIP(hipGetLastError());
  return 0;
}

int dq_hip_unpack_bgr24_dev(int device, const uint32_t* d_in, uint32_t width, uint32_t height,
                            uint32_t stride, uint8_t* d_bgr, void* stream) {
  if (!d_in || !d_bgr || !bgr24_shape_ok(width, height, stride)) return -1;
  hipStream_t st = engine_stream(device, stream);
  dq::launch_bgr24_unpack(d_in, width, height, stride, d_bgr, st);
  join_default_stream(stream, st);
  DQ_HIP(hipGetLastError());
  return 0;
}

int dq_hip_gather_bgr24_dev(int device, const uint8_t* d_bgr, uint32_t stride,
                            const uint32_t* d_coords, uint32_t n, uint32_t* d_out, void* stream) {
  if (!d_bgr || !d_coords || !d_out || stride < 3u) return -1;
  if (n == 0) return 0;
  hipStream_t st = engine_stream(device, stream);
  dq::launch_bgr24_gather(d_bgr, stride, d_coords, n, d_out, st);
  join_default_stream(stream, st);
  DQ_HIP(hipGetLastError());
  return 0;
}

// The uniform-weight batch over the engine lanes (frames split over the
// lanes' engines and streams).
static int quant_batch(int device, std::vector<dq::FrameJob>& jobs, int max_iters, void* stream) {
  const int nframes = (int)jobs.size();
  const int lanes = std::min(nframes, dq::batch_lanes());
  Engine& e0 = engine_for(device);
  if (lanes <= 1) {
    std::lock_guard<std::mutex> g(e0.mutex());
    e0.run(jobs.data(), nframes, max_iters, true, dev_stream(e0, stream));
  } else {
    // frames [f0(l), f0(l+1)) on lane l; every lane first waits for the
    // caller's stream (the frames may have been produced there)
    DQ_HIP(hipSetDevice(device));
    hipEvent_t ready = events().get();   // this call's own (concurrent calls: one each)
    DQ_HIP(hipEventRecord(ready, (hipStream_t)stream));
    for (int l = 1; l < lanes; ++l) {   // lanes inherit lane 0's switches
      Engine& e = engine_for(device, l);
      e.set_fixed_point(e0.fixed_point());
      e.set_plan(e0.plan());
      e.set_timing(e0.timing());
    }
    const std::function<void(int)> work = [&](int l) {
      const int f0 = nframes * l / lanes, f1 = nframes * (l + 1) / lanes;
      Engine& e = engine_for(device, l);
      DQ_HIP(hipSetDevice(device));
      std::lock_guard<std::mutex> g(e.mutex());
      DQ_HIP(hipStreamWaitEvent(e.stream(), ready, 0));
      e.run(jobs.data() + f0, f1 - f0, max_iters, true, e.stream());
    };
    lane_workers().run(lanes, work);
    events().put(ready);   // (every lane's wait on it is enqueued)
    // lane 0 reports for the batch: the last frame's diagnostics, summed counters
    Engine& el = engine_for(device, lanes - 1);
    std::lock_guard<std::mutex> g(e0.mutex());
    uint64_t swept = 0, full = 0, fixes = 0;
    int rounds = 0;
    for (int l = 0; l < lanes; ++l) {
      Engine& e = engine_for(device, l);
      swept += e.last_points_swept;
      full += e.last_points_full;
      fixes += e.last_cursor_fixes;
      rounds = std::max(rounds, e.last_rounds);
      if (l > 0) e0.absorb_stats(e);
    }
    e0.last_means = el.last_means;
    e0.last_sizes = el.last_sizes;
    e0.last_trace = el.last_trace;
    e0.last_rounds = rounds;
    e0.last_points_swept = swept;
    e0.last_points_full = full;
    e0.last_cursor_fixes = fixes;
  }
  int empty = 0;
  for (int i = 0; i < nframes; ++i) empty += jobs[i].num_empty;
  return empty;
}

int dq_hip_quant_batch_dev(int device, int nframes, const uint32_t* const* d_in,
                           const uint32_t* n, uint32_t* const* d_out, uint32_t k,
                           uint32_t* ct, uint32_t* k_out, int max_iters, void* stream) {
  if (nframes <= 0 || !d_in || !n || !d_out || !ct || !k_out || k == 0 || max_iters < 1)
    return -1;
  for (int i = 0; i < nframes; ++i)
    if (!d_in[i] || !d_out[i] || n[i] == 0) return -1;
  std::vector<dq::FrameJob> jobs(nframes);
  for (int i = 0; i < nframes; ++i) {
    jobs[i].d_in = d_in[i];
    jobs[i].n = n[i];
    jobs[i].d_out = d_out[i];
    jobs[i].k = (int)k;
    jobs[i].ct = ct + (size_t)i * k;
  }
  const int empty = quant_batch(device, jobs, max_iters, stream);
  for (int i = 0; i < nframes; ++i) k_out[i] = (uint32_t)jobs[i].k_out;
  return empty;
}

int dq_hip_quant_bgr24_batch_dev(int device, int nframes, const uint8_t* const* d_bgr, uint32_t width,
                                 uint32_t height, uint32_t stride, uint32_t* const* d_out, uint32_t k,
                                 uint32_t* ct, uint32_t* k_out, int uniq, int max_iters, void* stream) {
  if (nframes <= 0 || !d_bgr || !d_out || !ct || !k_out || k == 0 || max_iters < 1 ||
      !bgr24_shape_ok(width, height, stride))
    return -1;
  for (int i = 0; i < nframes; ++i)
    if (!d_bgr[i] || !d_out[i]) return -1;
  const uint32_t n = width * height;
  if (!uniq || stride != 3 * width) {
    // the weighted path's colour table (and padded rows) take packed pixels:
    // Vec3BToUID on the GPU into a scratch frame, then the packed entries
    int empty = 0;
    for (int i = 0; i < nframes; ++i) {
      uint32_t* px = nullptr;
      hipStream_t st = engine_stream(device, stream);
      DQ_HIP(hipMallocAsync((void**)&px, (size_t)n * 4 + 16, st));
      dq::launch_bgr24_pack(d_bgr[i], width, height, stride, px, st);
      uint32_t kk = k;
      int r;
      if (uniq) {
        const uint32_t* pin = px;
        r = dq_hip_quant_batch_dev(device, 1, &pin, &n, &d_out[i], k, ct + (size_t)i * k, &kk, max_iters, stream);
      } else {
        r = dq_hip_quant_weighted_dev(device, px, n, d_out[i], &kk, ct + (size_t)i * k, max_iters, stream);
      }
      DQ_HIP(hipFreeAsync(px, st));
      if (r < 0) return r;
      k_out[i] = kk;
      empty += r;
    }
    return empty;
  }
  std::vector<dq::FrameJob> jobs(nframes);
  for (int i = 0; i < nframes; ++i) {
    jobs[i].d_in = reinterpret_cast<const uint32_t*>(d_bgr[i]);
    jobs[i].bgr = true;
    jobs[i].n = n;
    jobs[i].d_out = d_out[i];
    jobs[i].k = (int)k;
    jobs[i].ct = ct + (size_t)i * k;
  }
  const int empty = quant_batch(device, jobs, max_iters, stream);
  for (int i = 0; i < nframes; ++i) k_out[i] = (uint32_t)jobs[i].k_out;
  return empty;
}

int dq_hip_quant_bgr24_dev(int device, const uint8_t* d_bgr, uint32_t width, uint32_t height,
                           uint32_t stride, uint32_t* d_out, uint32_t* k, uint32_t* ct, int uniq,
                           int max_iters, void* stream) {
  if (!k || *k == 0) return -1;
  uint32_t kk = 0;
  const int r = dq_hip_quant_bgr24_batch_dev(device, 1, &d_bgr, width, height, stride, &d_out, *k, ct, &kk,
                                             uniq, max_iters, stream);
  if (r >= 0) *k = kk;
  return r;
}

int dq_hip_map_bgr24_dev(int device, const uint8_t* d_bgr, uint32_t width, uint32_t height,
                         uint32_t stride, uint32_t* d_out, const uint32_t* ct, int k, void* stream) {
  if (!d_bgr || !d_out || !ct || k <= 0 || !bgr24_shape_ok(width, height, stride)) return -1;
  Engine& e = engine_for(device);
  std::lock_guard<std::mutex> g(e.mutex());
  hipStream_t st = dev_stream(e, stream);
  if (stride != 3 * width) {   // padded rows: packed first
    uint32_t* px = nullptr;
    const uint32_t n = width * height;
    DQ_HIP(hipMallocAsync((void**)&px, (size_t)n * 4 + 16, st));
    dq::launch_bgr24_pack(d_bgr, width, height, stride, px, st);
    e.map(px, n, d_out, ct, k, st);
    DQ_HIP(hipFreeAsync(px, st));
    return 0;
  }
  Engine::MapJob j{reinterpret_cast<const uint32_t*>(d_bgr), width * height, d_out, ct, k, true};
  e.map_many(&j, 1, st);
  return 0;
}

int dq_hip_quant_rows_dev(int device, int nframes, const uint32_t* const* d_in,
                          const uint32_t* n, const uint32_t* width, const uint64_t* n_global,
                          int nshard, uint32_t* const* d_out, uint32_t k, uint32_t* ct,
                          uint32_t* k_out, int max_iters, void* stream) {
  if (nframes <= 0 || !d_in || !n || !ct || !k_out || k == 0 || max_iters < 1) return -1;
  if (nshard < 1 || nshard > dq::kMaxShard) return -1;
  Engine& e = engine_for(device);
  for (int i = 0; i < nframes; ++i) {
    if (!d_in[i] || n[i] == 0) return -1;
    const uint64_t ng = n_global ? n_global[i] : 0;
    if (ng != 0 && ng < n[i]) return -1;
    if (ng > n[i] && e.comm_ranks() < 2) return -2;   // other rows live in other processes
  }
  std::lock_guard<std::mutex> g(e.mutex());
  std::vector<dq::FrameJob> jobs(nframes);
  for (int i = 0; i < nframes; ++i) {
    jobs[i].d_in = d_in[i];
    jobs[i].n = n[i];
    jobs[i].d_out = d_out ? d_out[i] : nullptr;
    jobs[i].k = (int)k;
    jobs[i].ct = ct + (size_t)i * k;
    jobs[i].nshard = nshard;
    jobs[i].width = width ? width[i] : 0;
    jobs[i].n_global = n_global ? n_global[i] : 0;
  }
  e.run(jobs.data(), nframes, max_iters, true, dev_stream(e, stream));
  int empty = 0;
  for (int i = 0; i < nframes; ++i) {
    k_out[i] = (uint32_t)jobs[i].k_out;
    empty += jobs[i].num_empty;
  }
  return empty;
}

// Test-only (dq_hip.h): row-tile sharding over nranks in-process ranks of
// one device, joined by the loopback collective (dq_engine.h Loopback).
// Rank r holds rows [r*H/N, (r+1)*H/N) of every frame (bench.py row_range),
// runs them on its own engine, stream and host thread with n_global = W*H,
// and maps them into its rows of d_out.
int dq_hip_loopback_rows_dev(int device, int nranks, int nframes, const uint32_t* const* d_in,
                             uint32_t width, uint32_t height, uint32_t* const* d_out, uint32_t k,
                             uint32_t* ct, uint32_t* k_out, int max_iters, uint64_t* coll_log,
                             int log_cap, int* log_len) {
  if (nranks < 1 || nranks > dq::kMaxShard || nframes <= 0 || !d_in || !d_out || !ct || !k_out || k == 0 ||
      max_iters < 1 || width == 0 || height < (uint32_t)nranks || (uint64_t)width * height >= (1ull << 32))
    return -1;
  for (int i = 0; i < nframes; ++i)
    if (!d_in[i] || !d_out[i]) return -1;
  // (rank engines are shared by every rank count: rank r of any group reuses
  // the same engine -- kMaxShard per device at most, not one per (N, r))
  static std::mutex mu;
  static std::map<std::pair<int, int>, Engine*> engines;
  static std::map<std::pair<int, int>, dq::Loopback*> groups;
  std::lock_guard<std::mutex> call(mu);
  DQ_HIP(hipSetDevice(device));
  dq::Loopback*& grp = groups[{device, nranks}];
  if (!grp) grp = new dq::Loopback(nranks, device);
  grp->reset_log();
  std::vector<Engine*> es(nranks);
  for (int r = 0; r < nranks; ++r) {
    Engine*& e = engines[std::make_pair(device, r)];
    if (!e) e = new Engine(device);
    es[r] = e;
  }
  // inputs may still be in flight on the legacy default stream
  hipEvent_t ready = events().get();
  DQ_HIP(hipEventRecord(ready, nullptr));
  for (Engine* e : es) DQ_HIP(hipStreamWaitEvent(e->stream(), ready, 0));
  events().put(ready);
  const uint64_t ng = (uint64_t)width * height;
  std::vector<int> empty(nranks, 0);
  auto work = [&](int r) {
    Engine& e = *es[r];
    DQ_HIP(hipSetDevice(device));
    std::lock_guard<std::mutex> g(e.mutex());
    const uint32_t r0 = (uint32_t)((uint64_t)height * r / nranks), r1 = (uint32_t)((uint64_t)height * (r + 1) / nranks);
    std::vector<dq::FrameJob> jobs(nframes);
    for (int i = 0; i < nframes; ++i) {
      jobs[i].d_in = d_in[i] + (size_t)r0 * width;
      jobs[i].n = (r1 - r0) * width;
      jobs[i].d_out = d_out[i] + (size_t)r0 * width;
      jobs[i].k = (int)k;
      jobs[i].ct = ct + ((size_t)r * nframes + i) * k;
      jobs[i].width = width;
      jobs[i].n_global = ng;
    }
    e.set_loopback(grp, r);
    e.run(jobs.data(), nframes, max_iters, true, e.stream());
    e.set_loopback(nullptr, 0);
    for (int i = 0; i < nframes; ++i) {
      k_out[(size_t)r * nframes + i] = (uint32_t)jobs[i].k_out;
      empty[r] += jobs[i].num_empty;
    }
  };
  std::vector<std::thread> th;
  for (int r = 1; r < nranks; ++r) th.emplace_back(work, r);
  work(0);
  for (auto& t : th) t.join();
  for (int r = 0; r < nranks; ++r) {
    if (log_len) log_len[r] = (int)grp->log[r].size();
    if (coll_log)
      for (int c = 0; c < log_cap && c < (int)grp->log[r].size(); ++c) coll_log[(size_t)r * log_cap + c] = grp->log[r][c];
  }
  {   // rank 0's diagnostics of its last frame on the device's lane-0 engine (dq_hip_last_*)
    Engine& e0 = engine_for(device);
    std::lock_guard<std::mutex> g(e0.mutex());
    e0.last_means = es[0]->last_means;
    e0.last_sizes = es[0]->last_sizes;
    e0.last_trace = es[0]->last_trace;
    e0.last_rounds = es[0]->last_rounds;
  }
  return empty[0];
}

int dq_hip_comm_unique_id(void* id128) {
  if (!id128) return -1;
  Engine::comm_unique_id(static_cast<char*>(id128));
  return 0;
}

int dq_hip_comm_init(int device, int nranks, int rank, const void* id128) {
  if (!id128 || nranks < 1 || rank < 0 || rank >= nranks) return -1;
  Engine& e = engine_for(device);
  std::lock_guard<std::mutex> g(e.mutex());
  e.comm_init(nranks, rank, static_cast<const char*>(id128));
  return 0;
}

int dq_hip_comm_size(int device) { return engine_for(device).comm_ranks(); }

int dq_hip_comm_destroy(int device) {
  Engine& e = engine_for(device);
  std::lock_guard<std::mutex> g(e.mutex());
  e.comm_destroy();
  return 0;
}

int dq_hip_quant_dev(int device, const uint32_t* d_in, uint32_t n, uint32_t* d_out,
                     uint32_t* k, uint32_t* ct, int max_iters, void* stream) {
  if (!d_in || !d_out || !k || !ct || n == 0 || *k == 0 || max_iters < 1) return -1;
  uint32_t kk = 0;
  const int r = dq_hip_quant_batch_dev(device, 1, &d_in, &n, &d_out, *k, ct, &kk, max_iters, stream);
  if (r >= 0) *k = kk;
  return r;
}

// dq_hip_quant over ngpus devices of this process: the frame's pixels split
// into ngpus row ranges (4-point multiples), one per device, every pass's node
// totals allreduced over an in-process RCCL communicator set
// (ncclCommInitAll, created once per device count); each device maps its own
// range.  Uniform-weight path only (the weighted path's folds are sequential).
static int quant_multi_gpu(const uint32_t* in, uint32_t n, uint32_t* out, uint32_t* k, uint32_t* ct,
                           int G) {
  static std::mutex mu;
  static std::map<int, std::vector<ncclComm_t>> sets;
  std::vector<ncclComm_t>* comms;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = sets.find(G);
    if (it == sets.end()) {
      std::vector<ncclComm_t> c(G);
      std::vector<int> devs(G);
      for (int d = 0; d < G; ++d) devs[d] = d;
      const ncclResult_t r = ncclCommInitAll(c.data(), G, devs.data());
      if (r != ncclSuccess) dq::die("ncclCommInitAll", __FILE__, __LINE__, ncclGetErrorString(r));
      it = sets.emplace(G, std::move(c)).first;
    }
    comms = &it->second;
  }
  std::vector<uint32_t> first(G + 1);
  for (int g = 0; g <= G; ++g) first[g] = g == G ? n : (uint32_t)(((uint64_t)n * g / G) & ~(uint64_t)3);
  std::vector<std::vector<uint32_t>> cts(G, std::vector<uint32_t>(*k));
  std::vector<int> kout(G, 0), empty(G, 0);
  auto work = [&](int g) {
    Engine& e = engine_for(g);
    std::lock_guard<std::mutex> lk(e.mutex());
    DQ_HIP(hipSetDevice(g));
    hipStream_t st = e.stream();
    const uint32_t len = first[g + 1] - first[g];
    const Engine::CommState prev = e.swap_comm({(*comms)[g], G, g});
    dq::FrameJob j;
    if (len > 0) {
      e.stage_in(in + first[g], len, st);
      j.d_in = e.staged_in();
      j.d_out = e.staged_out();
    } else {   // (n < 4 G: an empty range still takes part in every allreduce)
      e.stage_in(in, 1, st);
      j.d_in = e.staged_in();
    }
    j.n = len > 0 ? len : 1;
    j.n_global = n;
    j.k = (int)*k;
    j.ct = cts[g].data();
    e.run(&j, 1, 10, true, st);
    if (len > 0)
      DQ_HIP(hipMemcpyAsync(out + first[g], e.staged_out(), (size_t)len * 4, hipMemcpyDeviceToHost, st));
    DQ_HIP(hipStreamSynchronize(st));
    e.swap_comm(prev);
    kout[g] = j.k_out;
    empty[g] = j.num_empty;
  };
  std::vector<std::thread> th;
  for (int g = 1; g < G; ++g) th.emplace_back(work, g);
  work(0);
  for (auto& t : th) t.join();
  for (int g = 1; g < G; ++g)   // every device ran the identical FP64 updates on identical totals
    if (kout[g] != kout[0] || cts[g] != cts[0]) dq::die("dq_hip_quant", __FILE__, __LINE__, "devices disagree");
  std::memcpy(ct, cts[0].data(), (size_t)kout[0] * 4);
  *k = (uint32_t)kout[0];
  return empty[0];
}

int dq_hip_quant(const uint32_t* in, uint32_t n, uint32_t* out, uint32_t* k,
                 uint32_t* ct, int uniq, int ngpus) {
  if (!in || !out || !k || !ct || n == 0 || *k == 0) return -1;
  const int G = std::min(std::max(ngpus, 1), dq_hip_device_count());
  // (DQ_HIP_MULTI_1=1: the in-process communicator path even on one device -- tests)
  const char* m1 = std::getenv("DQ_HIP_MULTI_1");
  const bool force = m1 && m1[0] == '1' && ngpus >= 1;
  if ((G > 1 || force) && uniq && n >= 4u * (uint32_t)G) return quant_multi_gpu(in, n, out, k, ct, G);
  Engine& e = engine_for(current_device());
  std::lock_guard<std::mutex> g(e.mutex());
  hipStream_t st = e.stream();
  e.stage_in(in, n, st);
  dq::FrameJob j;
  j.d_in = e.staged_in();
  j.n = n;
  j.d_out = e.staged_out();
  j.k = (int)*k;
  j.ct = ct;
  if (uniq) e.run(&j, 1, 10, true, st);
  else e.run_weighted(j, 10, true, st);
  DQ_HIP(hipMemcpyAsync(out, e.staged_out(), (size_t)n * 4, hipMemcpyDeviceToHost, st));
  DQ_HIP(hipStreamSynchronize(st));
  *k = (uint32_t)j.k_out;
  return j.num_empty;
}

int dq_hip_map(const uint32_t* in, uint32_t n, uint32_t* out, const uint32_t* ct, int k) {
  if (!in || !out || !ct || k <= 0) return -1;
  if (n == 0) return 0;
  Engine& e = engine_for(current_device());
  std::lock_guard<std::mutex> g(e.mutex());
  hipStream_t st = e.stream();
  e.stage_in(in, n, st);
  e.map(e.staged_in(), n, e.staged_out(), ct, k, st);
  DQ_HIP(hipMemcpyAsync(out, e.staged_out(), (size_t)n * 4, hipMemcpyDeviceToHost, st));
  DQ_HIP(hipStreamSynchronize(st));
  return 0;
}

// Synthetic frames of the benchmark configs (SURVEY 8c/8d generator) and the
// output checksum the golden fixtures are keyed by.
void dq_synth_xorshift(uint32_t* out, uint64_t n, uint64_t seed) {
  uint64_t s = seed;
  for (uint64_t i = 0; i < n; ++i) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    out[i] = (uint32_t)(s & 0xFFFFFFu);
  }
}

uint64_t dq_fnv1a64(const uint32_t* w, uint64_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint64_t i = 0; i < n; ++i) {
    h ^= w[i];
    h *= 0x100000001b3ull;
  }
  return h;
}

void dq_subdivided_colors(uint32_t* out125) {
  static const uint32_t v[5] = {0, 63, 127, 191, 255};
  for (int i = 0; i < 125; ++i)   // R outermost, B innermost, alpha 0xFF (:874-888)
    out125[i] = 0xFF000000u | (v[i / 25] << 16) | (v[i / 5 % 5] << 8) | v[i % 5];
}

int dq_hip_block_hist(const uint32_t* in, uint32_t width, uint32_t height, const uint32_t* palette,
                      int npal, uint32_t dim, uint32_t block_w, uint32_t block_h, uint32_t* quant,
                      uint32_t* mode, uint32_t* ndistinct, uint32_t* keys, uint32_t* counts) {
  if (!in || !palette || npal <= 0 || !mode || (!keys) != (!counts) ||
      !block_hist_shape_ok(width, height, dim, block_w, block_h))
    return -1;
  const int dev = current_device();
  Engine& e = engine_for(dev);
  hipStream_t st = e.stream();
  const size_t n = (size_t)width * height, nb = (size_t)block_w * block_h, cap = (size_t)dim * dim;
  uint32_t *d_mode = nullptr, *d_nd = nullptr, *d_keys = nullptr, *d_counts = nullptr;
  DQ_HIP(hipMallocAsync((void**)&d_mode, nb * 4, st));
  if (ndistinct) DQ_HIP(hipMallocAsync((void**)&d_nd, nb * 4, st));
  if (keys) {
    DQ_HIP(hipMallocAsync((void**)&d_keys, nb * cap * 4, st));
    DQ_HIP(hipMallocAsync((void**)&d_counts, nb * cap * 4, st));
    DQ_HIP(hipMemsetAsync(d_keys, 0, nb * cap * 4, st));
    DQ_HIP(hipMemsetAsync(d_counts, 0, nb * cap * 4, st));
  }
  int rc;
  {
    std::lock_guard<std::mutex> g(e.mutex());
    e.stage_in(in, (uint32_t)n, st);
    e.map(e.staged_in(), (uint32_t)n, e.staged_out(), palette, npal, st);
    uint32_t* work = nullptr;
    DQ_HIP(hipMallocAsync((void**)&work, dq::block_hist_scratch_words(block_w, block_h) * 4, st));
    dq::BlockHistArgs a{e.staged_out(), width, height, block_w, block_h, d_mode, d_nd, d_keys, d_counts,
                        work, nullptr, 0};
    rc = dq::launch_block_hist(a, (int)dim, st);
    DQ_HIP(hipFreeAsync(work, st));
    if (quant) DQ_HIP(hipMemcpyAsync(quant, e.staged_out(), n * 4, hipMemcpyDeviceToHost, st));
    DQ_HIP(hipMemcpyAsync(mode, d_mode, nb * 4, hipMemcpyDeviceToHost, st));
    if (ndistinct) DQ_HIP(hipMemcpyAsync(ndistinct, d_nd, nb * 4, hipMemcpyDeviceToHost, st));
    if (keys) {
      DQ_HIP(hipMemcpyAsync(keys, d_keys, nb * cap * 4, hipMemcpyDeviceToHost, st));
      DQ_HIP(hipMemcpyAsync(counts, d_counts, nb * cap * 4, hipMemcpyDeviceToHost, st));
    }
    DQ_HIP(hipStreamSynchronize(st));
  }
  for (uint32_t* p : {d_mode, d_nd, d_keys, d_counts})
    if (p) DQ_HIP(hipFreeAsync(p, st));
  return rc;
}

int dq_hip_last_centroids(int device, double* means, int64_t* sizes, int k) {
  Engine& e = engine_for(device);
  std::lock_guard<std::mutex> g(e.mutex());
  if ((size_t)k != e.last_sizes.size()) return -1;
  if (means) std::memcpy(means, e.last_means.data(), sizeof(double) * 3 * k);
  if (sizes) std::memcpy(sizes, e.last_sizes.data(), sizeof(int64_t) * k);
  return 0;
}

int dq_hip_last_trace(int device, int64_t* trace, int k) {
  Engine& e = engine_for(device);
  std::lock_guard<std::mutex> g(e.mutex());
  if (k < 1 || (size_t)(k - 1) * 4 != e.last_trace.size()) return -1;
  if (trace && k > 1) std::memcpy(trace, e.last_trace.data(), sizeof(int64_t) * 4 * (k - 1));
  return 0;
}

int dq_hip_last_rounds(int device) { return engine_for(device).last_rounds; }

uint64_t dq_hip_last_points_swept(int device) { return engine_for(device).last_points_swept; }
uint64_t dq_hip_last_points_full(int device) { return engine_for(device).last_points_full; }
uint64_t dq_hip_last_seq_tiles(int device) { return engine_for(device).last_seq_tiles; }
uint64_t dq_hip_last_cursor_fixes(int device) { return engine_for(device).last_cursor_fixes; }

int dq_hip_last_wsmall_profile(int device, uint64_t* out, int nout) {
  const std::vector<uint64_t>& p = engine_for(device).last_wsmall_prof;
  const int n = std::min<int>(nout, (int)p.size());
  for (int i = 0; i < n; ++i) out[i] = p[i];
  return n;
}
void dq_hip_set_fixed_point(int device, int on) { engine_for(device).set_fixed_point(on != 0); }
void dq_hip_set_planned_rounds(int device, int on) {
  for (int l = 0; l < dq::kMaxLanes; ++l) engine_for(device, l).set_plan(on != 0);
}
int dq_hip_last_planned_rounds(int device) { return engine_for(device).last_planned; }

void dq_hip_set_loop_max(int device, uint32_t max_points) {
  for (int l = 0; l < dq::kMaxLanes; ++l) engine_for(device, l).set_loop_max(max_points);
}

int dq_hip_last_loop_rounds(int device) { return engine_for(device).last_loop_rounds; }

void dq_hip_set_persist(int device, int on) {
  for (int l = 0; l < dq::kMaxLanes; ++l) engine_for(device, l).set_persist(on != 0);
}

int dq_hip_last_persist_rounds(int device) { return engine_for(device).last_persist_rounds; }

void dq_hip_set_wsmall(int device, int on) {
  for (int l = 0; l < dq::kMaxLanes; ++l) engine_for(device, l).set_wsmall(on != 0);
}

void dq_hip_set_timing(int device, int on) { engine_for(device).set_timing(on != 0); }

void dq_hip_set_debug(int device, int flags) {
  (void)device;   // (process-wide: every engine reads it when a run starts)
  dq::set_debug_flags(flags);
}

void dq_hip_set_lanes(int lanes) { dq::set_batch_lanes(lanes); }
int dq_hip_get_lanes(void) { return dq::batch_lanes(); }

void dq_hip_reset_stats(int device) { engine_for(device).reset_stats(); }

int dq_hip_get_stat(int device, int kind, uint64_t* launches, double* ms, double* bytes) {
  if (kind < 0 || kind >= dq::ST_COUNT) return -1;
  const dq::KernelStat& s = engine_for(device).stats[kind];
  if (launches) *launches = s.launches;
  if (ms) *ms = s.ms;
  if (bytes) *bytes = s.bytes;
  return 0;
}

int dq_hip_get_stat_units(int device, int kind, double* units) {
  if (kind < 0 || kind >= dq::ST_COUNT) return -1;
  if (units) *units = engine_for(device).stats[kind].units;
  return 0;
}

const char* dq_hip_stat_name(int kind) {
  static const char* names[] = {"pass_init", "pass_split", "pass_kmeans", "pass_klast",
                                "epilogue", "partition", "map_cells", "map", "plan", "kloop"};
  if (kind < 0 || kind >= dq::ST_COUNT) return "";
  return names[kind];
}

// =========================================================================
// Reference signatures (include/quant_util.h, include/DivQuantHeader.h)
// =========================================================================

// quant_util.cpp:20-158.
void quant_recurse(uint32_t numPixels, const uint32_t* inPixelsPtr, uint32_t* outPixelsPtr,
                   uint32_t* numClustersPtr, uint32_t* outColortablePtr, int allPixelsUnique) {
  if (numPixels == 0 || *numClustersPtr == 0)
    dq::die("quant_recurse", __FILE__, __LINE__, "numPixels and *numClustersPtr must be > 0");
  Engine& e = engine_for(current_device());
  std::lock_guard<std::mutex> g(e.mutex());
  hipStream_t st = e.stream();
  // the reference's timing lines (quant_util.cpp:48-66, 141-145): clock()
  // CPU time of this process from t1, the map line cumulative from t1 too
  const clock_t t1 = clock();
  e.stage_in(inPixelsPtr, numPixels, st);
  dq::FrameJob j;
  j.d_in = e.staged_in();
  j.n = numPixels;
  j.k = (int)*numClustersPtr;
  j.ct = outColortablePtr;
  if (allPixelsUnique) e.run(&j, 1, 10, false, st);   // uniform weights (:1130-1132)
  else e.run_weighted(j, 10, false, st);               // calc_color_table + weighted (:1133-1138)
  report_empty(j.num_empty);
  uint32_t k = (uint32_t)j.k_out;
  *numClustersPtr = k;
  clock_t t2 = clock();
  if (!quiet()) {
    const long el = timediff(t1, t2);
    std::printf("quant_varpart_fast() elapsed: %ld ms aka %0.2f s\n", el, el / 1000.0f);
  }
  k = dedup_colortable(outColortablePtr, k);
  *numClustersPtr = k;
  e.map(e.staged_in(), numPixels, e.staged_out(), outColortablePtr, (int)k, st);
  DQ_HIP(hipMemcpyAsync(outPixelsPtr, e.staged_out(), (size_t)numPixels * 4,
                        hipMemcpyDeviceToHost, st));
  DQ_HIP(hipStreamSynchronize(st));
  t2 = clock();
  if (!quiet()) {
    const long el = timediff(t1, t2);
    std::printf("map_colors_mps() elapsed: %ld ms aka %0.2f s\n", el, el / 1000.0f);
  }
}

}  // extern "C"

// DivQuantMapColors.cpp:243-539.
void map_colors_mps(const uint32_t* inPixelsPtr, uint32_t numPixels, uint32_t* outPixelsPtr,
                    uint32_t* outColortablePtr, int colormapSize) {
  if (colormapSize <= 0)
    dq::die("map_colors_mps", __FILE__, __LINE__, "colormapSize must be > 0");
  dq_hip_map(inPixelsPtr, numPixels, outPixelsPtr, outColortablePtr, colormapSize);
}

// DivQuantCluster.cpp:1099-1179.
void quant_varpart_fast(const uint32_t numPixels, const uint32_t* inPixels, uint32_t* tmpPixels,
                        const uint32_t numRows, const uint32_t numCols, uint32_t* numClustersPtr,
                        uint32_t* colortablePtr, const int num_bits, const int dec_factor,
                        const int max_iters, const int allPixelsUnique) {
  (void)tmpPixels;
  if (!validate_num_bits((uchar)num_bits))   // (:1115-1118 asserts)
    dq::die("quant_varpart_fast", __FILE__, __LINE__, "invalid num_bits");
  if (dec_factor <= 0)   // calc_color_table's message (:103-108); the reference then runs on garbage
    dq::die("quant_varpart_fast", __FILE__, __LINE__, "Decimation factor should be positive");
  if (max_iters < 1)
    dq::die("quant_varpart_fast", __FILE__, __LINE__, "max_iters < 1 is not supported");
  Engine& e = engine_for(current_device());
  std::lock_guard<std::mutex> g(e.mutex());
  hipStream_t st = e.stream();
  e.stage_in(inPixels, numPixels, st);
  dq::FrameJob j;
  j.d_in = e.staged_in();
  j.n = numPixels;
  j.k = (int)*numClustersPtr;
  j.ct = colortablePtr;
  j.num_bits = num_bits;
  j.dec = dec_factor;
  j.rows = numRows;
  j.cols = numCols;
  // uniform weights only for unique 8-bit undecimated input (:1130-1132);
  // else calc_color_table (after cut_bits unless !unique && 8 bits, :1133-1146)
  if (allPixelsUnique && num_bits == 8 && dec_factor == 1) {
    e.run(&j, 1, max_iters, false, st);
  } else {
    if (numRows == 0 || numCols == 0)   // calc_color_table visits no pixel; DivQuantCluster asserts (:211)
      dq::die("quant_varpart_fast", __FILE__, __LINE__, "numRows and numCols must be > 0 for calc_color_table");
    e.run_weighted(j, max_iters, false, st);
  }
  report_empty(j.num_empty);
  const int k = j.k_out;
  *numClustersPtr = (uint32_t)k;
}

// DivQuantMapColors.cpp:205-220.
double get_double_scale(const uint32_t* inPixels, const uint32_t numPixels) {
  (void)inPixels;
  const int numRows = 1, dec = 1;
  const int numCols = (int)numPixels;
  return 1.0 / (ceil(numRows / (double)dec) * ceil(numCols / (double)dec));
}

// DivQuantMapColors.cpp:43-51.
void check_mem(const int x) {
  if (x != 0) {
    std::fprintf(stderr, "Insufficient memory !\n");
    std::abort();
  }
}

// DivQuantMisc.cpp:18-46.
clock_t start_timer(void) { return clock(); }
double stop_timer(const clock_t start_time) {
  return ((double)(clock() - start_time)) / CLOCKS_PER_SEC;
}
long timediff(clock_t t1, clock_t t2) {
  return (long)(((double)t2 - t1) / CLOCKS_PER_SEC * 1000);
}
int validate_num_bits(const uchar num_bits) {
  if (!(0 < num_bits && num_bits <= 8)) {
    std::fprintf(stderr, "Number of bits per channel ( %d ) must be in [1,8] !\n", num_bits);
    return 0;
  }
  return 1;
}

// DivQuantUni.cpp:28-100: drop the low (8 - num_bits) bits of each channel
// and shift the rest down (in place allowed).
void cut_bits(const uint32_t* inPixels, const uint32_t numPixels, uint32_t* outPixels,
              const uchar num_bits_red, const uchar num_bits_green, const uchar num_bits_blue) {
  if (!validate_num_bits(num_bits_red) || !validate_num_bits(num_bits_green) ||
      !validate_num_bits(num_bits_blue))
    return;
  const uint32_t sr = 8 - num_bits_red, sg = 8 - num_bits_green, sb = 8 - num_bits_blue;
  for (uint32_t i = 0; i < numPixels; ++i) {
    const uint32_t p = inPixels[i];
    const uint32_t R = ((p >> 16) & 0xFF) >> sr;
    const uint32_t G = ((p >> 8) & 0xFF) >> sg;
    const uint32_t B = (p & 0xFF) >> sb;
    outPixels[i] = (R << 16) | (G << 8) | B;
  }
}

// DivQuantMapColors.cpp:82-203 on the device (dq_weighted.hip's colour
// table, the weighted path's own): unique colours with weights count*norm in
// the reference's output order -- hash buckets ascending (HASH(R,G,B) =
// (R*33023 + G*30013 + B*27011) & 0x7fffffff) % 20023), and inside a bucket
// the most recently first-seen colour first (the chains are prepended).  The
// pixel index quirk inPixels[ic + ir*numRows] is kept (:124); numPixels is
// not read, as in the reference.
double* calc_color_table(const uint32_t* inPixels, const uint32_t numPixels, uint32_t* outPixels,
                         const uint32_t numRows, const uint32_t numCols, const int dec_factor,
                         int* num_colors) {
  (void)numPixels;
  if (dec_factor <= 0) {
    std::fprintf(stderr, "Decimation factor ( %d ) should be positive !\n", dec_factor);
    return NULL;
  }
  const uint64_t nr = (numRows + (uint64_t)dec_factor - 1) / dec_factor;
  const uint64_t nc = (numCols + (uint64_t)dec_factor - 1) / dec_factor;
  double* weights = new double[std::max<uint64_t>(1, nr * nc)];
  Engine& e = engine_for(current_device());
  std::lock_guard<std::mutex> g(e.mutex());
  *num_colors = (int)e.color_table(inPixels, numRows, numCols, (uint32_t)dec_factor, outPixels, weights, e.stream());
  return weights;
}
