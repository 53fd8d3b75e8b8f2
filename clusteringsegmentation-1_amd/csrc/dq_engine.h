// dq_engine.h -- C++ host engine behind the DivQuant drop-in.
//
// The reference splits K-1 clusters one after another, each split costing one
// split pass plus `max_iters` 2-means passes over that cluster's points
// (DivQuant/DivQuantCluster.cpp:346-1027).  The split of a cluster depends
// only on that cluster's points and its stored weight/mean/variance, never on
// the order in which clusters are split.  The engine therefore expands the
// binary split tree in ROUNDS: a round splits a whole batch of leaves at once
// (every pass of the round is ONE kernel launch over all their points), and
// a host-side replay of the reference's greedy max-TSE order (:873-892)
// decides which leaves the next round must expand.  The replay needs no
// floating point of its own: the TSEs it compares come from the device
// epilogue, which evaluates the reference's FP64 expressions verbatim.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <string>
#include <vector>

#include "dq_internal.h"
#include "dq_kernels.h"

namespace dq {

[[noreturn]] void die(const char* what, const char* file, int line, const char* detail);
#define DQ_HIP(expr)                                                      \
  do {                                                                    \
    hipError_t e_ = (expr);                                               \
    if (e_ != hipSuccess) ::dq::die(#expr, __FILE__, __LINE__, hipGetErrorString(e_)); \
  } while (0)
#define DQ_CHECK(cond, msg)                                               \
  do {                                                                    \
    if (!(cond)) ::dq::die(#cond, __FILE__, __LINE__, msg);               \
  } while (0)

// A node of the split tree: one cluster as it exists between two splits.
struct Node {
  int parent = -1;
  int child_old = -1, child_new = -1;
  bool expanded = false;
  double w = 0.0;                    // weight[]   (:290, :862-863)
  double mean[3] = {0, 0, 0};        // mean[]     (:309)
  double var[3] = {0, 0, 0};         // var[]      (:314)
  double tse = 0.0;                  // tse[]      (:304)
  uint32_t off = 0, len = 0;         // segment (len == size[] of the cluster)
  int32_t buf = BUF_IN;
};

// Per-kernel-kind timing (filled only when timing is enabled).
struct KernelStat {
  uint64_t launches = 0;
  double ms = 0.0;
  double bytes = 0.0;   // algorithmic bytes (4 B per point read, +4 B written)
};
enum StatKind { ST_INIT = 0, ST_SPLIT, ST_KMEANS, ST_KLAST, ST_EPILOGUE, ST_PARTITION,
                ST_CELLS, ST_MAP, ST_COUNT };

class Engine {
 public:
  explicit Engine(int device);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  // DivQuantCluster<true,*,true> (:133-1097) over n device-resident points.
  // Writes the non-empty cluster colours to ct (host, >= k entries) in
  // cluster-index order and returns their number; *num_empty gets the
  // number of empty clusters (:1067-1069).
  int cluster(const uint32_t* d_in, uint32_t n, int k, int max_iters,
              uint32_t* ct, int* num_empty, hipStream_t stream);

  // map_colors_mps (DivQuantMapColors.cpp:243-539) on device buffers.
  void map(const uint32_t* d_in, uint32_t n, uint32_t* d_out,
           const uint32_t* ct, int k, hipStream_t stream);

  // Host-pointer convenience (copies in and out through the engine's buffers).
  void stage_in(const uint32_t* h_in, uint32_t n, hipStream_t stream);
  const uint32_t* staged_in() const { return d_stage_in_; }
  uint32_t* staged_out() { return d_stage_out_; }

  hipStream_t stream() const { return stream_; }
  int device() const { return device_; }
  std::mutex& mutex() { return mu_; }

  // Diagnostics of the last cluster() call.
  std::vector<double> last_means;     // K*3 centroid doubles per cluster index
  std::vector<int64_t> last_sizes;    // K sizes
  std::vector<int64_t> last_trace;    // (K-1)*4: new_index old_index |C| |new|
  int last_rounds = 0;
  uint64_t last_points_swept = 0;     // sum over passes of points read

  void set_timing(bool on) { timing_ = on; }
  void reset_stats();
  KernelStat stats[ST_COUNT];

 private:
  void ensure_pixels(uint32_t n);
  void ensure_round(size_t nnodes, size_t ntiles);
  void run_round(const std::vector<int>& active, bool root_round, int max_iters,
                 double s, hipStream_t stream);
  void timed_begin(hipStream_t stream);
  void timed_end(int kind, double bytes, hipStream_t stream);
  void collect_timing();

  int device_ = 0;
  hipStream_t stream_ = nullptr;
  std::mutex mu_;
  bool timing_ = false;

  // pixel working buffers (segments of the split tree)
  uint32_t* d_p0_ = nullptr;
  uint32_t* d_p1_ = nullptr;
  size_t cap_px_ = 0;
  uint32_t* d_stage_in_ = nullptr;
  uint32_t* d_stage_out_ = nullptr;
  size_t cap_stage_ = 0;

  // per-round node/tile tables
  DevNode* d_nodes_ = nullptr;
  Tile* d_tiles_ = nullptr;
  TilePartial* d_parts_ = nullptr;
  DevNode* h_nodes_ = nullptr;   // pinned
  Tile* h_tiles_ = nullptr;      // pinned
  size_t cap_nodes_ = 0, cap_tiles_ = 0;

  // map tables
  uint32_t* d_pal_ = nullptr;
  uint16_t* d_lut_ = nullptr;
  uint16_t* d_cell_cnt_ = nullptr;
  uint16_t* d_cell_idx_ = nullptr;
  uint32_t* h_pal_ = nullptr;    // pinned
  uint16_t* h_lut_ = nullptr;    // pinned

  std::vector<Node> nodes_;
  const uint32_t* staged_root_ = nullptr;   // the caller's input (root segment)
  struct PendingEvent { hipEvent_t a, b; int kind; double bytes; };
  std::vector<PendingEvent> pending_;
  std::vector<hipEvent_t> event_pool_;
  hipEvent_t take_event();
};

// Process-wide engine for a device (created on first use).
Engine& engine_for(int device);

}  // namespace dq
