// dq_engine.h -- C++ host engine behind the DivQuant drop-in.
//
// The reference splits K-1 clusters one after another, each split costing one
// split pass plus `max_iters` 2-means passes over that cluster's points
// (DivQuant/DivQuantCluster.cpp:346-1027).  The split of a cluster depends
// only on that cluster's points and its stored weight/mean/variance, never on
// the order in which clusters are split.  The engine therefore expands the
// binary split tree in ROUNDS: a round splits a whole batch of leaves at once
// -- of every frame in the batch -- and every pass of the round is ONE kernel
// launch over all their points.  A host-side replay of the reference's greedy
// max-TSE order (:873-892) decides which leaves the next round must expand.
// The replay needs no floating point of its own: the TSEs it compares come
// from the device, which evaluates the reference's FP64 expressions verbatim.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <condition_variable>
#include <mutex>
#include <queue>
#include <deque>
#include <vector>

#include "dq_internal.h"
#include "dq_kernels.h"
#include "dq_weighted.h"

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


// A node of a frame's split tree: one cluster as it exists between splits.
// Its points are spread over the frame's shards: one local segment per
// shard, kept in Engine::segs_ (entry node * nshard + shard).
struct Node {
  int frame = 0;
  int child_old = -1, child_new = -1;
  int parent = -1;
  int32_t buf = 0;                   // 0: caller's input, 1: P0, 2: P1
  bool expanded = false;
  bool queued = false;               // in a round enqueued but not yet finished
  bool partitioned = false;          // children's segments assigned in child_buf(buf)
  bool points = true;                // its segment holds its points (false: a PS_STATS round
                                     //   computed its split without writing them)
  bool cursors_pending = false;      // final at a PS_STATS round's split: its partition cursors
                                     //   were not counted (fix_cursors before it is partitioned)
  double w = 0.0;                    // weight[]   (:290, :862-863)
  double mean[3] = {0, 0, 0};        // mean[]     (:309)
  double var[3] = {0, 0, 0};         // var[]      (:314)
  double tse = 0.0;                  // tse[]      (:304)
  uint64_t glen = 0;                 // size[] of the cluster (all shards, all processes)
  // a box holding every point (channel R, G, B): the cube for a root, the
  // parent's for a child, clipped at the parent's cut when the parent's
  // halves are proven to be the cut's (DevNode::box_lo)
  int16_t lo[3] = {0, 0, 0}, hi[3] = {255, 255, 255};
  int16_t axis = 0, thr = 0;         // the split's cut, once run (for the children's boxes)
};

// A node's local segment in one shard, and -- once the node has been split --
// its record and tiles on the device (kept for the whole run so that a later
// round can partition it, fused with its children's split pass).
struct Seg {
  uint32_t off = 0, len = 0;
  int32_t ntiles = 0;
  const DevNode* dnode = nullptr;
  const Tile* dtiles = nullptr;
  uint32_t* dwparts = nullptr;       // its tiles' per-(tile, wave) count words in its round's block
  int32_t rec = 0;                   // its record's index in its round (Tile::node)
};

// One quant_recurse / DivQuantCluster input.
struct FrameJob {
  const uint32_t* d_in = nullptr;    // device, n points (this process's rows)
  uint32_t n = 0;
  uint32_t* d_out = nullptr;         // device, mapped colours (nullptr: cluster only)
  int k = 0;                         // requested clusters
  uint32_t* ct = nullptr;            // host, >= k entries
  // row-tile sharding
  int nshard = 1;                    // row ranges of d_in processed as separate shards
  uint32_t width = 0;                // row length: shard boundaries on whole rows (0: any)
  uint64_t n_global = 0;             // points of the whole frame over all processes (0: n)
  // quant_varpart_fast's cut_bits / decimation inputs (weighted path only,
  // DivQuantCluster.cpp:1139-1146): channels cut to num_bits, every dec-th
  // row and column of a rows x cols frame read with the reference's numRows
  // stride (calc_color_table :124); cols 0: n; centres << (8 - num_bits).
  // d_in is a BGR24 frame (OpenCV CV_8UC3, continuous rows: 3 B per point,
  // B G R) read directly by the root's passes, its partition and the map
  // (uniform-weight path, one shard)
  bool bgr = false;
  int num_bits = 8;
  int dec = 1;
  uint32_t rows = 1, cols = 0;
  // outputs
  int k_out = 0;                     // colours written to ct
  int num_empty = 0;                 // empty clusters (:1067-1069)
};

// Per-kernel-kind timing (filled only when timing is enabled).
struct KernelStat {
  uint64_t launches = 0;
  double ms = 0.0;
  double bytes = 0.0;   // engine-model bytes (4 B per packed point read,
                        //   3 B per planar point read or written, 8 B per mapped pixel)
  double units = 0.0;   // points (pixels) the launches processed
};
enum StatKind { ST_INIT = 0, ST_SPLIT, ST_KMEANS, ST_KLAST, ST_EPILOGUE, ST_PARTITION,
                ST_CELLS, ST_MAP, ST_PLAN, ST_KLOOP, ST_COUNT };

// Test-only stand-in for the RCCL communicator of row-tile sharding: N
// engines of ONE process on one device, each driven by its own host thread
// and stream (rank r = the engine holding rows row_range(h, r, N)), sum their
// node totals with a reduction kernel ordered by cross-stream events.  The
// engines run the TOT_ALLREDUCE path exactly as N processes would (local
// counts != global totals), which a 1-rank RCCL communicator cannot show.
// Every rank must enqueue the same collective sequence (RCCL's contract): the
// loopback checks the element counts of each collective against each other
// and records them per rank (`log`), and a rank left waiting at a collective
// for kLoopbackTimeoutS aborts with the sequence number instead of hanging.
class Loopback {
 public:
  explicit Loopback(int nranks, int device);
  int ranks() const { return n_; }
  // rank's part of one in-place u64 sum allreduce of `count` words on `stream`
  void allreduce(int rank, uint64_t* buf, size_t count, hipStream_t stream);
  void reset_log();
  std::vector<std::vector<uint64_t>> log;   // per rank: element count of each collective
  static constexpr double kLoopbackTimeoutS = 120.0;

 private:
  void barrier(int rank, const char* where);
  int n_;
  std::mutex mu_;
  std::condition_variable cv_;
  int arrived_ = 0;
  uint64_t gen_ = 0;
  std::vector<hipEvent_t> in_ev_, rd_ev_;   // per rank: its inputs ready / its reads done
  std::vector<uint64_t*> bufs_, scratch_;
  std::vector<size_t> counts_, cap_;
};

class Engine {
 public:
  explicit Engine(int device);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  // DivQuantCluster<true,*,true> (:133-1097) over every frame of the batch;
  // with dedup_map, also the colortable dedup (quant_util.cpp:93-118) and
  // map_colors_mps into each frame's d_out.  All frames use max_iters.
  void run(FrameJob* jobs, int nframes, int max_iters, bool dedup_map, hipStream_t stream);
  // The weighted path (allPixelsUnique = 0): calc_color_table on the device,
  // then DivQuantCluster<false,*,true> with the reference's ordered FP64 folds
  // (dq_weighted.hip); dedup + map as run().  last_sizes / last_trace count
  // points = unique colours, as the reference's size[].
  void run_weighted(FrameJob& job, int max_iters, bool dedup_map, hipStream_t stream);
  // Many weighted calls (the app's superpixel regions, each with its own
  // pixels, output and K; dedup + map as run_weighted(.., true, ..)): every
  // region the one-workgroup kernel holds in ONE launch, one workgroup each;
  // the others (and any with more colours than it holds) one by one through
  // run_weighted.  Returns how many the batch launch took.
  int run_weighted_regions(FrameJob* jobs, int njobs, int max_iters, hipStream_t stream);
  // calc_color_table (DivQuantMapColors.cpp:82-203) on the device for a host
  // input: the points inPixels[ic + ir*numRows] (ir < rows, ic < cols, step
  // dec), their unique colours and weights norm * count in the reference's
  // order into h_colors / h_weights (room for rows * cols / dec^2 entries).
  // Returns the number of colours.
  uint32_t color_table(const uint32_t* h_in, uint32_t rows, uint32_t cols, uint32_t dec, uint32_t* h_colors,
                       double* h_weights, hipStream_t stream);

  // map_colors_mps (DivQuantMapColors.cpp:243-539) on device buffers.
  void map(const uint32_t* d_in, uint32_t n, uint32_t* d_out,
           const uint32_t* ct, int k, hipStream_t stream);
  // pixels per map task (map_many splits larger jobs; 4 n < 2^31 for the
  // output's buffer resource, 16-B aligned sub-jobs)
  static constexpr uint32_t kMapTaskMax = 1u << 28;
  struct MapJob {
    const uint32_t* d_in;
    uint32_t n;
    uint32_t* d_out;
    const uint32_t* ct;   // host colortable
    int k;
    bool bgr = false;     // d_in is a BGR24 frame (3 B per pixel)
  };
  // sync = false: enqueue only (the caller synchronises and collects the timing)
  void map_many(const MapJob* jobs, int njobs, hipStream_t stream, bool sync = true);

  // Host-pointer convenience (copies in and out through the engine's buffers).
  void stage_in(const uint32_t* h_in, uint32_t n, hipStream_t stream);
  const uint32_t* staged_in() const { return d_stage_in_; }
  uint32_t* staged_out() { return d_stage_out_; }
  // Device scratch of at least n words for stream-ordered helpers (block
  // histogram queue); growing it waits for the device.
  uint32_t* scratch_words(size_t n);

  hipStream_t stream() const { return stream_; }

  // Row-tile sharding across processes (one GPU each): an RCCL communicator
  // over which every pass's node totals are allreduced.
  static void comm_unique_id(char id[128]);
  void comm_init(int nranks, int rank, const char id[128]);
  void comm_destroy();
  // In-process multi-GPU (dq_hip_quant's ngpus): borrow a communicator of a
  // set created by ncclCommInitAll for the duration of one run; returns the
  // engine's previous one (restore with the same call).
  struct CommState { void* comm; int ranks, rank; };
  CommState swap_comm(CommState c) {
    CommState old{comm_, comm_ranks_, comm_rank_};
    comm_ = c.comm;
    comm_ranks_ = c.ranks;
    comm_rank_ = c.rank;
    return old;
  }
  int comm_ranks() const { return loop_ ? loop_->ranks() : comm_ranks_; }
  // Tests: join the in-process loopback group `l` as `rank` (nullptr: leave).
  void set_loopback(Loopback* l, int rank) {
    loop_ = l;
    loop_rank_ = rank;
  }
  void allreduce_totals(int nlogical, hipStream_t stream);
  int device() const { return device_; }
  std::mutex& mutex() { return mu_; }

  // Diagnostics of the last frame of the last run().
  std::vector<double> last_means;     // K*3 centroid doubles per cluster index
  std::vector<int64_t> last_sizes;    // K sizes
  std::vector<int64_t> last_trace;    // (K-1)*4: new_index old_index |C| |new|
  int last_rounds = 0;
  int last_planned = 0;               // rounds planned on the device (of last_rounds)
  int last_aborted = 0;               // planned rounds whose plan found a parent unfinished
  int last_loop_rounds = 0;           // rounds whose 2-means iterations ran in one kloop_kernel launch
  int last_persist_rounds = 0;        // ... in one kpersist_kernel launch
  uint64_t last_points_swept = 0;     // sum over passes of points read (all frames)
  uint64_t last_points_full = 0;      // the same without fixed-point finalisation
  uint64_t last_seq_tiles = 0;        // weighted: tiles folded one summand at a time
  uint64_t last_cursor_fixes = 0;     // records whose cursors a later round counted (fix_cursors)
  std::vector<uint64_t> last_wsmall_prof;   // weighted, one launch: WSmallResult::prof (empty: not taken)

  void set_timing(bool on) { timing_ = on; }
  bool timing() const { return timing_; }
  // add another engine's kernel stats to this one's (and clear them there)
  void absorb_stats(Engine& o) {
    for (int i = 0; i < ST_COUNT; ++i) {
      stats[i].launches += o.stats[i].launches;
      stats[i].ms += o.stats[i].ms;
      stats[i].bytes += o.stats[i].bytes;
      stats[i].units += o.stats[i].units;
    }
    o.reset_stats();
  }
  // Finalise a split when its 2-means reaches an exact fixed point (default
  // on; results are identical either way -- dq_kernels.hip, node_update).
  void set_fixed_point(bool on) { fixed_point_ = on; }
  // Device-planned rounds (default on; DQ_HIP_TUNE plan=0 turns the default off).
  void set_plan(bool on) { plan_ = on; }
  // kloop_kernel eligibility: records of at most n points (0: never)
  void set_loop_max(uint32_t n) { kloop_max_ = std::min<uint32_t>(n, kLoopMaxLen); }
  void set_persist(bool on) { persist_ = on; }
  // the one-workgroup weighted path for small inputs (launch_wsmall; default on)
  void set_wsmall(bool on) { wsmall_ = on; }
  bool plan() const { return plan_; }
  bool fixed_point() const { return fixed_point_; }
  void reset_stats();
  KernelStat stats[ST_COUNT];

 private:
  using HeapEnt = std::pair<std::pair<double, int>, int>;
  std::vector<HeapEnt> top_;          // next_active scratch
  struct FrameState {
    FrameJob* job = nullptr;
    double s = 0.0;                   // get_double_scale
    // per shard: offset in P0/P1 (16-B aligned), 16-B aligned input (maybe a
    // staged copy), points, and offset of the shard's rows in the frame
    uint32_t base[kMaxShard] = {};
    const uint32_t* in[kMaxShard] = {};
    uint32_t n[kMaxShard] = {};
    uint32_t first[kMaxShard] = {};
    std::vector<int> leaf;            // cluster index -> node id
    std::vector<HeapEnt> heap;        // max-heap of ((tse, -idx), node) (std::push_heap)
    int new_index = 1, old_index = 0;
    int need = -1;                    // node the replay waits for (-1: done)
    int splits_queued = 0;            // nodes expanded or queued for expansion
    std::vector<int64_t> trace;
  };

  // One enqueued split round.  Host-built rounds get their
  // tables from the host (staging + upload kernel); planned rounds from
  // plan_kernel, enqueued before the results of the round they are planned
  // from exist (their records: the children of `plist`'s records of `prev`).
  struct Round {
    uint64_t seq = 0;
    int par = 0;                      // status / result slot (seq % kSlots)
    bool root = false, planned = false;
    int prev = -1;                    // planned: the round it is planned from
    std::vector<int32_t> plist;       // planned: records of `prev` split in it
    std::vector<int> order;           // node id per logical slot (planned: once prev is done)
    std::vector<int> parents;         // nodes the round's partsplit partitions
    int n_own = 0, nl = 0, nr = 0;
    size_t ntiles = 0, nptiles = 0, nt_own = 0;
    size_t tiles_cap = 0, ptiles_cap = 0;
    uint64_t tl = 0;
    uint64_t total = 0, own_total = 0, parent_total = 0;
    std::vector<int32_t> tbeg, tend;  // per record: its tiles
    size_t bytes = 0;
    DevNode* dn = nullptr;
    Tile* dt = nullptr;
    uint32_t* dcounts = nullptr;      // planned: plan_kernel's counts (device)
    RoundArgs ra{};
    bool kmeans = false;              // its split epilogue left records active
    bool stats_only = false;          // planned, a frame's last: partsplit PS_STATS (+ PS_LATE)
    std::vector<std::pair<size_t, int>> km_events;
    long loop_event = -1;             // kloop_kernel's timing event (pending_ index)
    double t_enq = 0;
  };
  std::deque<Round> rounds_;          // (a deque: references stay valid while rounds are added)
  int wait_round_ = -1;               // the round finish_round waits on (diagnostics)

  void ensure_pixels(size_t total);
  void ensure_round(size_t nnodes, size_t ntiles, size_t nptiles, size_t staging_bytes,
                    int max_iters, hipStream_t stream);
  char* arena_alloc(size_t bytes, hipStream_t stream);
  uint32_t wait_status(const uint64_t* slot, uint64_t seq, hipStream_t stream);
  int enqueue_host_round(const std::vector<int>& active, bool root_round, int max_iters,
                         hipStream_t stream);
  bool plan_list(int ri, std::vector<int32_t>* plist);
  int enqueue_planned_round(int prev, const std::vector<int32_t>& plist, int max_iters,
                            hipStream_t stream, const uint32_t* cancel = nullptr);
  void assign_planned(int ri);
  // successor: a planned round queued from ri (-1: none).  Returns the index
  // of a re-plan of it enqueued behind ri's 2-means iterations, or -1.
  int finish_round(int ri, int max_iters, hipStream_t stream, bool speculate = false, int successor = -1);
  void kmeans_iter(Round& R, int it, int max_iters, hipStream_t stream);
  // All 2-means iterations of round R in one launch (kloop_kernel): every
  // record one shard, planar, at most kloop_max_ points and kLoopMaxTiles tiles.
  bool loop_ok(const Round& R) const;
  bool persist_ok(const Round& R) const;
  bool persist_ok_layout(const Round& R) const;   // planar records (not a root's frame)
  size_t max_record_tiles(const Round& R) const;
  // kind 1: kloop_kernel, 2: kpersist_kernel
  void kmeans_loop(Round& R, int max_iters, hipStream_t stream, int kind);
  void apply_tune(const char* spec);
  int src_fmt(const std::vector<int>& ids) const;
  void check_arena_zero(hipStream_t stream);
  uint64_t tile_len_of(uint64_t len, uint64_t tl) const;
  uint64_t round_tile_len(uint64_t total) const;
  void replay(FrameState& f);
  void next_active(FrameState& f, std::vector<int>* active);
  void finish_frame(FrameState& f, bool last);
  const uint8_t* buf_ptr(int buf, const FrameState& f, int shard) const;
  // bytes a pass reads per point of a node: the caller's packed frame (a
  // root) or the planar working buffers
  double point_bytes(int node) const {
    return nodes_[node].buf == 0 && !frames_[nodes_[node].frame].job->bgr ? 4.0 : 3.0;
  }
  void timed_begin(hipStream_t stream);
  void timed_end(int kind, double bytes, hipStream_t stream, double units = 0.0);
  void collect_timing();

  int device_ = 0;
  int debug_ = 0;                     // debug_flags() of the current run
  void debug_host_delay() const;
  uint32_t* d_bgr_pack_ = nullptr;   // BGR24 frames the map cannot read directly, packed
  size_t cap_bgr_pack_ = 0;
  bool fixed_point_ = true;
  hipStream_t stream_ = nullptr;
  std::mutex mu_;
  bool timing_ = false;

  // pixel working buffers (segments of the split trees of all frames)
  uint32_t* d_p0_ = nullptr;
  uint32_t* d_p1_ = nullptr;
  size_t cap_px_ = 0;
  uint32_t* d_stage_in_ = nullptr;
  uint32_t* d_stage_out_ = nullptr;
  size_t cap_stage_ = 0;
  uint32_t* d_scratch_ = nullptr;
  size_t cap_scratch_ = 0;
  uint32_t* d_align_ = nullptr;       // aligned copies of misaligned inputs
  size_t cap_align_ = 0;
  uint32_t* d_map_align_ = nullptr;   // map staging for misaligned in/out
  size_t cap_map_align_ = 0;

  // Per-round tables: every round's [DevNode | Tile | PartTile | LaunchCtr]
  // block is carved from a device arena that is only recycled by the next
  // run (a later round partitions nodes through their records and tiles) and
  // written with ONE copy from the pinned staging buffer.
  std::vector<std::pair<char*, size_t>> arena_;   // chunks
  size_t arena_chunk_ = 0, arena_used_ = 0;
  // bytes of each chunk the last run used: cleared when the next run starts
  // (a planned round's counters and counts must be zero on entry to the
  // fused plan + partition launch, plansplit_kernel)
  std::vector<size_t> arena_hw_;
  bool fuse_plan_ = true;             // plansplit_kernel for one-shard planned rounds (DQ_HIP_TUNE fuse_plan)
  bool fold_split_ = true;            // allreduced one-shard rounds: the partition's last workgroups
                                      //   write the split totals, no nodesum_kernel (DQ_HIP_TUNE fold_split)
  char* h_stage_ = nullptr;           // pinned
  size_t cap_stage_tab_ = 0;
  TilePartial* d_parts_ = nullptr;    // per tile of the round
  TilePartial* d_parts2_ = nullptr;   // per tile: kpersist_kernel's odd iterations
  size_t cap_parts2_ = 0;
  TilePartial* d_sparts_ = nullptr;   // per PartTile of the round
  size_t cap_parts_ = 0, cap_sparts_ = 0;
  // host-coherent pinned memory the epilogues write (results, status words),
  // kSlots slots by round sequence (a planned round runs while the host
  // finishes the previous one; a re-plan can be queued behind a planned
  // round the host has not resolved yet); the results' device copy the plans
  // read
  static constexpr int kSlots = 3;
  NodeResult* h_res_ = nullptr;
  NodeResult* d_res_ = nullptr;       // device view of h_res_
  NodeResult* d_dres_ = nullptr;      // device memory
  size_t cap_res_ = 0;                // records per slot
  uint64_t* h_stat_ = nullptr;
  uint64_t* d_stat_ = nullptr;
  size_t cap_stat_ = 0;               // words per slot
  int32_t* h_plist_ = nullptr;        // per slot: a planned round's parent records
  int32_t* d_plist_ = nullptr;
  size_t cap_plist_ = 0;
  uint32_t* h_counts_ = nullptr;      // per slot: plan_kernel's counts (host mirror)
  uint32_t* d_counts_h_ = nullptr;
  char* d_stage_view_ = nullptr;      // device view of h_stage_ (host-coherent)
  hipEvent_t stage_ev_ = nullptr;     // the last upload of h_stage_
  bool stage_pending_ = false;
  bool plan_ = true;                  // device-planned rounds (DQ_HIP_TUNE plan=0: host only)
  bool stats_only_ = true;            // a frame's last planned round: PS_STATS + PS_LATE (DQ_HIP_TUNE stats_only)
  uint64_t stats_min_ = 12u << 20;    // ... when the round has more points than this (DQ_HIP_TUNE stats_min)
  bool eager_replan_ = true;          // finish_round: all 2-means iterations + the re-plan at
                                      //   once when a planned successor waits (DQ_HIP_TUNE eager_replan)
  uint64_t seq_ = 0;                  // round sequence number
  int lookahead_ = 2;                 // 2-means iterations queued past the one awaited
                                      //   (1: C3 0.543-0.554 ms, 2: 0.518-0.525, 4: 0.520-0.532)
  bool spin_sync_ = true;             // sync_stream polls an event (DQ_HIP_TUNE spin_sync)
  hipEvent_t sync_ev_ = nullptr;
  void sync_stream(hipStream_t stream);
  bool speculate_kmeans_ = true;      // a round with nothing queued behind it starts its
                                      //   2-means iterations before its split status (DQ_HIP_TUNE spec_kmeans)
  bool persist_ = true;                // kpersist_kernel for eligible rounds (DQ_HIP_TUNE persist)
  static constexpr int kPersistWgsPerCu = 4;
  uint32_t kloop_max_ = 49152;        // a record's points at most for kloop_kernel (DQ_HIP_TUNE kloop_max; 0: off)
  int tiles_target_ = 512;            // tiles per big round (DQ_HIP_TUNE tiles; 512 vs 1024: C3 -4 %)
  int node_tiles_ = 8;                // tiles per node at least (DQ_HIP_TUNE node_tiles)
  uint32_t tile_max_ = kMaxTilePx / 2;   // points per tile at most (DQ_HIP_TUNE tile_max; 32K vs 64K: C5 -2 %)
  // host-side trace (DQ_HIP_TRACE=1): per-run phase times on stderr
  bool trace_ = false, trace_rounds_ = false;   // DQ_HIP_TRACE=1 / 2 (per round)
  double tr_wait_us_ = 0, tr_build_us_ = 0, tr_replay_us_ = 0;
  double tr_mapprep_us_ = 0, tr_mapsync_us_ = 0;
  double tr_entry_t0_ = 0, tr_first_us_ = 0;   // run() entry; entry -> the root round's first launch
  // DQ_HIP_TRACE: host timestamps of the call's launches and waits (printed
  // relative to run() entry as one line per call)
  std::vector<std::pair<const char*, double>> tr_log_;
  void tmark(const char* what) {
    if (trace_) tr_log_.emplace_back(what, host_us_now());
  }
  static double host_us_now();

  // map tables
  uint32_t* d_cell_c32_ = nullptr;    // compact records per map task of a chunk
  int num_cus_ = 0;
  bool use_lds_map_ = true;           // DQ_HIP_TUNE lds_map=0: the L2-gather map kernel
  uint32_t* d_cell_rec_ = nullptr;    // per map task of a chunk
  size_t cap_cells_ = 0;
  uint16_t* d_cell_idx_ = nullptr;
  uint32_t* h_mapstage_ = nullptr;   // pinned: per map [sorted palette | start LUT]
  uint32_t* d_mapstage_ = nullptr;
  uint32_t* d_mapstage_view_ = nullptr;   // device view of h_mapstage_ (host-coherent)
  hipEvent_t map_ev_ = nullptr;           // the last upload of h_mapstage_
  bool map_pending_ = false;
  size_t cap_mapstage_ = 0;
  void ensure_map_stage(size_t nmaps);
  // weighted path buffers
  void* d_wscratch_ = nullptr;        // colour-table scratch (runs, group tables)
  size_t cap_wscratch_ = 0;
  void* d_wnodes_ = nullptr;          // a round's WState records, tiles, fold tables, results
  char* h_wres_ = nullptr;            // host-coherent: a weighted round's "still active" word, then its results
  char* d_wres_view_ = nullptr;
  size_t cap_wres_ = 0;
  bool wsmall_ = true;                // small weighted calls in one launch (DQ_HIP_TUNE wsmall)
  WSmallResult* h_wsres_ = nullptr;   // host-coherent: its result
  WSmallArgs* h_wbargs_ = nullptr;    // host-coherent: a region batch's argument records
  WSmallArgs* d_wbargs_ = nullptr;
  WSmallResult* h_wbres_ = nullptr;   // ... and their results
  WSmallResult* d_wbres_ = nullptr;
  size_t cap_wb_ = 0;
  WSmallResult* d_wsres_ = nullptr;
  WsMapTab* d_wsmap_ = nullptr;       // device: its palette for the grid map
  bool run_weighted_small(FrameJob& job, int max_iters, bool dedup_map, hipStream_t stream);
  void ensure_color_scratch(uint32_t n, hipStream_t stream);
  void fix_cursors(int id, hipStream_t stream);
  size_t cap_wnodes_ = 0;

  std::vector<Node> nodes_;
  std::vector<Seg> segs_;             // node * nshard_ + shard
  Seg& seg(int node, int shard) { return segs_[(size_t)node * nshard_ + shard]; }
  int nshard_ = 1;                    // shard records per logical node in this run
  // where a pass's node totals come from (TotMode): own record, the node's
  // shard records in this process, or an allreduce across processes
  bool cross_process() const { return comm_ != nullptr || loop_ != nullptr; }
  int tot_mode() const { return cross_process() ? TOT_ALLREDUCE : (nshard_ > 1 ? TOT_NODE : TOT_OWN); }
  void ensure_totals(size_t nlogical, hipStream_t stream);
  uint64_t* d_tot_ = nullptr;         // sharded rounds: per logical node totals
  size_t cap_tot_ = 0;
  void* comm_ = nullptr;              // ncclComm_t across processes (row-tile sharding)
  int comm_ranks_ = 1, comm_rank_ = 0;
  Loopback* loop_ = nullptr;          // tests: in-process ranks instead of comm_
  int loop_rank_ = 0;
  std::vector<int> slot_of_, parent_pos_;   // enqueue_host_round scratch, indexed by node id
  std::vector<FrameState> frames_;
  struct PendingEvent { hipEvent_t a, b; int kind; double bytes, units; };
  std::vector<PendingEvent> pending_;
  std::vector<hipEvent_t> event_pool_;
  hipEvent_t take_event();
};

// Process-wide engines of a device (created on first use).  Lane 0 serves
// every call and holds the diagnostics; a batch of frames is split over
// batch_lanes() lanes, each an engine with its own stream driven by its own
// host thread, so one group's kernels fill the GPU while another group's host
// replays its round (DQ_HIP_LANES, default 3: measured best for 8 4K frames, interleaved A/B).
constexpr int kMaxLanes = 8;
Engine& engine_for(int device, int lane = 0);
int batch_lanes();
void set_batch_lanes(int lanes);   // 0: the default
// Test-only interleaving knobs (kDebug* in dq_kernels.h; 0 in production),
// read by every engine when a run starts.
void set_debug_flags(int flags);
int debug_flags();

}  // namespace dq
