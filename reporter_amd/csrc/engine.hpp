// engine.hpp — MI355X map-matching engine: the graph resident in HBM and the
// per-batch device workspace that the gfx950 kernels (engine.hip) run over.
//
// One Engine per process/GPU holds the read-only graph.  Each Matcher (one per
// calling thread, the threading contract of reference py/reporter_service.py:28-64)
// owns a HIP stream and a grow-only Workspace, so distinct matchers run
// concurrently without sharing mutable device state.
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "balls.hpp"
#include "graph.hpp"
#include "rm_common.hpp"
#include "serve_policy.hpp"

namespace rm {

#define RM_HIP(x)                                                                                \
  do {                                                                                           \
    hipError_t _e = (x);                                                                         \
    if (_e != hipSuccess)                                                                        \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " #x);   \
  } while (0)

// hipMalloc found too little free HBM (the engine's allocator; callers decide whether a smaller
// request can succeed: workspaces turn it into BatchTooLarge, the route-ball build steps down)
struct OutOfDeviceMemory : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct DevGraph {  // POD view of the graph in HBM, passed by value to kernels
  const uint32_t* node_off;
  const uint4* edges;            // EdgeRec
  const uint32_t* edge_src;      // source node of each directed edge
  const uint32_t* in_off;        // in-edge CSR offsets (N+1)
  const uint32_t* in_edge;       // edge ids by target node, ascending
  const uint4* in_rec;           // per in-edge: {edge, source node, road << 1 | rev, len_cm}
  const uint32_t* in_info;       // per in-edge: the edge's info word
  const uint32_t* edge_seg;
  const uint32_t* edge_seg_off;
  const uint32_t* edge_way;
  const uint32_t* road_node0;
  const uint32_t* road_node1;
  const uint32_t* road_fwd;
  const uint32_t* road_rev;
  const uint32_t* road_len;
  const uint4* verts;            // VertRec
  const unsigned long long* seg_id;
  const uint32_t* seg_len;
  const uint32_t* cell_off;
  const uint32_t* cell_item;
  const uint4* cell_rec;         // per cell item, 2 x uint4: {A.lon, A.lat, B.lon, B.lat}, {A.cum, B.cum, road | acc << 29, vertex}
  const uint4* road_rec;         // per road, 2 x uint4: {node0, node1, len_cm, fwd edge}, {rev edge, info fwd, info rev, 0}
  const uint4* relax[5];         // per travel mode, per directed edge: {target, len_cm | 0xffffffff if the mode
                                 // cannot use it, time_ms at the mode's speed, CSR range of the target}
  const uint32_t* node_rng;      // per node: first out-edge << 5 | out-degree
  const uint4* seg_rec;          // per directed edge, for K4: {len_cm | reversed << 31 | internal << 30, segment, offset, way}
  // route balls per travel mode (balls.hpp): per node {first entry, log2 table size or 0},
  // entries {node | kNone, dist cm, time ms, 0}; radius 0 = not built (K2 searches instead)
  const uint2* ball_hdr[5];
  const uint4* ball_ent[5];
  uint32_t ball_radius[5];
  uint32_t ball_mask;            // modes whose balls are built
  uint32_t ball_road_mask;       // road-id bits of a row's first word (rm_common.hpp ball_road_mask)
  // turn costs (rule 3b): per road its two headings (rm_common.hpp head_start / head_back), the
  // turn weight of each turn degree 0..180, and per mode the turn rows parallel to ball_ent
  // ({node0 word, node1 word} per slot: the turn weight of the canonical route from the table's
  // node to the road's endpoint, entering the road there, without the turn at the table's node
  // | the heading the route leaves that node with << 23; k_ball_turns)
  const uint32_t* road_head;
  const uint32_t* turn_w;
  const uint2* ball_turn[5];
  uint32_t ball_turn_mask;       // modes whose turn rows are built
  double lon0, lat0, dlon, dlat;
  uint32_t ncx, ncy, n_nodes, n_edges, n_segments, pad;
};

// Host-side description of one batch of traces (arrays live in host memory).
struct HostBatch {
  uint32_t n_traces = 0;
  const uint32_t* trace_off = nullptr;  // n_traces + 1
  const float* lon = nullptr;
  const float* lat = nullptr;
  const double* time = nullptr;
  const float* accuracy = nullptr;      // < 0 when absent
  uint32_t n_opts = 0;
  const MatchOptions* opts = nullptr;
  const uint32_t* trace_opt = nullptr;  // per trace
};

struct RunParams {
  double threshold_sec = 15.0;          // reporter_service.py:55-58
  uint32_t report_mask = 0b0110;        // levels {0,1}: bit (level+1)
  uint32_t transition_mask = 0b0110;
  uint32_t* hist = nullptr;             // device, n_segments * 16 u32 (may be null)
  int do_report = 1;
  int zero_hist = 0;                    // memset hist (and dur) on the stream before the epilogue
  unsigned long long* dur = nullptr;    // device, n_segments u64 duration sums in whole seconds (may be null)
  // a small batch (Matcher::run_small) also lays out and compacts its segments on the device
  // before its one read-back, so get_segments is a single copy (the service's reply path)
  int prefetch_segments = 0;
};

// Device addresses of a batch's inputs: the workspace's arrays, or (a small run()) the one
// block its single upload filled
struct InputView {
  const uint32_t* trace_off = nullptr;
  const float* lon = nullptr;
  const float* lat = nullptr;
  const double* time = nullptr;
  const float* acc = nullptr;
  const MatchOptions* opts = nullptr;
  const uint32_t* trace_opt = nullptr;
};

// Kernel ids for per-kernel HIP-event timing.
enum KernelId { kKStates = 0, kKCandidates, kKScan, kKRoutes, kKViterbi, kKPaths, kKSegments, kKReport, kKLocality,
                kNumKernels };
extern const char* const kKernelNames[kNumKernels];

// Device workspace of one batch.  All arrays are indexed by point slot p
// (state s of trace k lives at slot trace_off[k] + s).
constexpr int kCtlWords = 16;

struct Workspace {
  uint64_t cap_points = 0, cap_traces = 0, cap_trans = 0, cap_path = 0, cap_opts = 0, cap_segs = 0, cap_src = 0;
  // inputs
  uint32_t* trace_off = nullptr; float* lon = nullptr; float* lat = nullptr; double* time = nullptr;
  float* acc = nullptr; MatchOptions* opts = nullptr; uint32_t* trace_opt = nullptr;
  // per slot
  uint32_t* slot_trace = nullptr; uint32_t* n_states = nullptr; uint32_t* state_orig = nullptr;
  double* state_time = nullptr;     // epoch time of the state at each slot (K4 interpolation)
  // candidate descriptors, 2 x uint4 per (slot, rank): {road, s_cm, len_cm, spf | spr << 16},
  // {node0, node1, time_ms(s_cm) forward from node0, time_ms(len_cm - s_cm) reverse from node1}
  // (sp* = mode-capped speed of the directed edge in 0.1 km/h, 0 when the mode cannot use it)
  uint8_t* cand_n = nullptr; uint4* cand_desc = nullptr; float* cand_sq = nullptr;
  uint32_t* trans_cnt = nullptr; uint32_t* trans_off = nullptr; double* gc = nullptr; uint32_t* route = nullptr;
  double* route_d = nullptr;   // per transition: turn_m + |route_m - gc| (rule 3b), batches with turn costs only
  uint64_t cap_turn = 0;
  uint32_t* walk = nullptr;    // K2 -> k_turn_walks: transitions whose turn weight is walked (item << 4 | target)
  uint64_t cap_walk = 0;
  uint4* pair_info = nullptr;  // per layer pair slot: {route bound cm, time bound ms, KA | KB << 8 | mode << 16, 0}
  uint32_t* src_cnt = nullptr; uint32_t* src_off = nullptr; uint32_t* src_item = nullptr;
  int8_t* choice = nullptr; uint8_t* chain_start = nullptr; uint8_t* bp = nullptr;
  uint32_t* path_off = nullptr; uint32_t* path_cnt = nullptr; uint32_t* path_pool = nullptr; uint32_t* route_dist = nullptr;
  uint2* path_sab = nullptr;        // per chosen transition: source / target candidate offsets on their roads (cm)
  uint32_t* path_inline = nullptr;  // kInlinePath edges per slot
  // per trace outputs
  SegmentRec* segs = nullptr; uint32_t* seg_base = nullptr; uint32_t* seg_cnt = nullptr;
  uint32_t* trav_off = nullptr;     // first traversal record of each slot (scan of path_cnt)
  uint32_t* rec_slot = nullptr;     // K4: transition slot of each traversal record (k_rec_slot)
  ReportRec* reps = nullptr; uint32_t* rep_cnt = nullptr; ReportStats* stats = nullptr;
  // control words (kCtlWords): [0] path pool used [1] K2 ball-tier hand-over list [2] error flags [3] routes list A [4] paths list A
  // [5] routes list B [6] paths list B [7] candidates list (overflow lists of the lane tiers)
  // [8] path ball-tier hand-overs [9] routes list C [10] paths list C (global-memory tier)
  uint32_t* ctl = nullptr;
  uint32_t* rl_routes_a = nullptr; uint32_t* rl_routes_b = nullptr; uint32_t* rl_routes_0 = nullptr;
  uint32_t* rl_paths_a = nullptr; uint32_t* rl_paths_b = nullptr; uint32_t* rl_cand = nullptr;
  // global-memory search tier: its hand-over lists (ctl[9] routes, ctl[10] paths) and scratch
  uint32_t* rl_routes_c = nullptr; uint32_t* rl_paths_c = nullptr; void* gsearch = nullptr;
  uint32_t* trace_err = nullptr;            // per trace: error bits (kErr*) of that trace alone
  unsigned long long* tot64 = nullptr;      // u64 totals: [0] transitions [1] sources [2] path edges
  unsigned long long* tot_part = nullptr;   // per-block partial pairs of those totals (k_sum_parts folds them)
  // locality order (engine.hip k_loc_count / k_loc_scatter): the sorted state slots, each slot's
  // region bucket, the bucket cursors and the item counts in sorted order; allocated on the first
  // run that uses it (cap_sort slots)
  uint64_t cap_sort = 0;
  uint32_t* perm = nullptr; uint16_t* loc_key = nullptr; uint32_t* loc_cursor = nullptr; uint32_t* pcnt = nullptr;
  std::vector<void*> allocs;
  ~Workspace();
  void release();
};

// Raw per-vehicle point stream (the trace files simple_reporter's download phase writes:
// uuid, time, lat, lon, accuracy per line, reference py/simple_reporter.py:113,139-140).
struct PointsDesc {
  uint64_t n_points = 0;
  const uint32_t* uuid = nullptr;      // dense vehicle index per point
  const double* time = nullptr;        // epoch seconds (integers in the reference)
  const float* lon = nullptr;
  const float* lat = nullptr;
  const float* accuracy = nullptr;     // < 0 when absent
  double inactivity = 120.0;           // --inactivity (simple_reporter.py:344)
  uint32_t n_uuids = 0;
  uint32_t n_opts = 0;
  const MatchOptions* opts = nullptr;
  const uint32_t* uuid_opt = nullptr;  // per vehicle index into opts (NULL: all use opts[0])
};

// Time-tile stage parameters (simple_reporter.py:176-196, 211-254; CLI defaults :343,345,346)
struct TileParams {
  uint32_t quantisation = 3600;
  uint32_t privacy = 2;
  std::string source = "smpl_rprt";
  std::string mode = "AUTO";
};

// one CSV row of a time tile (simple_reporter.py:192-195) plus its sort keys
struct TileRow {
  uint64_t id, next_id;
  int64_t start, end;                  // floor(t0), ceil(t1)
  int32_t duration, length, queue;
  uint32_t bucket;                     // floor(time / quantisation)
  uint32_t tile;                       // level | tile index << 3 (id & 0x1FFFFFF)
  uint32_t pad[3];
};
static_assert(sizeof(TileRow) == 64, "TileRow is four dwordx4");

struct StageBufs {  // grow-only device buffers of the windowing and tile stages
  std::vector<void*> allocs;
  uint64_t cap_pts = 0, cap_rows = 0;
  uint32_t cap_tr = 0;
  uint32_t* derr = nullptr;
  uint32_t* p_uuid = nullptr; double* p_time = nullptr; float* p_lon = nullptr; float* p_lat = nullptr;
  float* p_acc = nullptr; uint32_t* p_uopt = nullptr; MatchOptions* p_opts = nullptr;
  unsigned long long* k0 = nullptr; unsigned long long* k1 = nullptr; uint32_t* v0 = nullptr; uint32_t* v1 = nullptr;
  uint32_t* flag = nullptr; uint32_t* idx = nullptr; uint32_t* wstart = nullptr; uint32_t* wcnt = nullptr;
  uint32_t* wofs = nullptr; uint32_t* wflag = nullptr; uint32_t* widx = nullptr;
  uint32_t* trace_uuid = nullptr;
  TileRow* rows = nullptr; TileRow* rows2 = nullptr;
  unsigned long long* rk = nullptr; unsigned long long* rk2 = nullptr;
  uint32_t* rperm = nullptr; uint32_t* rperm2 = nullptr; uint32_t* rflag = nullptr; uint32_t* ridx = nullptr;
  uint32_t* gpos = nullptr; uint8_t* gkeep = nullptr; uint32_t* tcnt = nullptr; uint32_t* tofs = nullptr;
  void* tmp = nullptr; size_t tmp_bytes = 0;
  uint32_t* hctl = nullptr;            // pinned read-back words
  uint32_t cap_uuids = 0;
  ~StageBufs();
};

// error bits in ctl[2] (and, except the path pool, per trace in Workspace::trace_err)
constexpr uint32_t kErrCandOverflow = 1u, kErrSearchOverflow = 2u, kErrPathOverflow = 4u, kErrRounds = 8u;
// message of the first error bit set in `bits` ("" for none)
const char* error_text(uint32_t bits);

class Engine;

// report() (reference py/reporter_service.py:79-179) on the device over host-supplied segment
// lists: trace k's segments are segs[seg_off[k] .. seg_off[k+1]); reports come back compacted
// (rep_off, T+1) with per-trace stats.  reps must hold seg_off[T] records.
void report_segments(int device, uint32_t T, const uint32_t* seg_off, const SegmentRec* segs, const double* end_time,
                     const double* threshold, const uint32_t* rmask, const uint32_t* tmask, uint32_t* rep_off,
                     ReportRec* reps, ReportStats* stats);

// The tile stage's collectives (one process per GPU): RCCL over xGMI, or a host transport the
// caller injects (capi.cpp rm_comm_init_host).  Both are blocking on `st`.
struct TileComm {
  int rank = 0, nranks = 1;
  virtual ~TileComm() = default;
  virtual uint64_t max_u64(uint64_t v, hipStream_t st) = 0;
  // every rank's `bytes` device bytes at send, in rank order, into recv (nranks * bytes)
  virtual void allgather(const void* send, void* recv, size_t bytes, hipStream_t st) = 0;
};

class Matcher {
 public:
  explicit Matcher(Engine* e);
  ~Matcher();
  Matcher(const Matcher&) = delete;
  Matcher& operator=(const Matcher&) = delete;

  // Upload a batch and run every stage on this matcher's stream; returns when the run's control
  // words are back (a large batch also reads its transition and path totals back between the
  // stages; a small one sizes its pools from upper bounds instead: run_small).  Throws on error.
  void run(const HostBatch& b, const RunParams& rp);
  // Run every stage over the batch already resident in HBM (inputs of the last run()).
  void run_device(const RunParams& rp);
  // rm_match_batch's device JSON path (engine.hip k_parse_json): reserve the byte buffer, upload
  // the trace-array bytes (from the parse threads, as their arenas fill), reserve the workspace,
  // parse them into the point arrays (flags[k] != 0:
  // trace k was not in the compact layout and must be parsed on the host; tspan[2k], [2k+1]: its
  // first and last times), place host-parsed traces' points, then run with the points in place
  void json_reserve_bytes(uint64_t bytes);                               // the byte buffer
  void json_reserve(uint64_t points, uint32_t traces, uint32_t nopts);     // workspace + per-trace arrays
  void json_upload(uint64_t off, const void* src, uint64_t n);             // thread-safe
  // span[2k], span[2k+1]: trace k's bytes [begin, end) in the buffer (begin == end: host-parsed)
  void json_parse(const uint64_t* span, const uint32_t* trace_off, uint32_t T, uint32_t* flags, double* tspan);
  void upload_points(uint64_t first, uint64_t n, const float* lon, const float* lat, const double* time, const float* acc);
  void run_parsed(const uint32_t* trace_off, uint32_t T, const MatchOptions* opts, uint32_t n_opts,
                  const uint32_t* trace_opt, const double* tspan, const RunParams& rp);
  void sync();
  // sizes of the last run
  uint32_t n_traces() const { return n_traces_; }
  uint64_t n_points() const { return n_points_; }
  uint64_t n_trans() const { return n_trans_; }
  uint64_t n_path_edges() const { return n_path_; }
  uint64_t seg_pool_used() const { return seg_used_; }
  // downloads of the last run (host buffers sized by the caller)
  void get_states(uint32_t* n_states, uint32_t* state_orig);
  void get_candidates(uint8_t* cand_n, uint32_t* road, uint32_t* s_cm, float* sq);
  void get_routes(uint32_t* trans_off, double* gc, uint32_t* route);
  // the distance terms K3 used (n_trans() doubles); 0 (nothing written) when the batch had no turn costs
  int get_route_terms(double* route_d);
  void get_viterbi(int8_t* choice, uint8_t* chain_start);
  void get_paths(uint32_t* path_off, uint32_t* path_cnt, uint32_t* pool, uint32_t* route_dist);
  // segments compacted per trace: seg_off (T+1), segs (seg_off[T])
  void get_segments(uint32_t* seg_off, SegmentRec* segs);
  // the same with the buffers sized from the device counts (one count read-back, not two)
  void get_segments(std::vector<uint32_t>& seg_off, std::vector<SegmentRec>& segs);
  uint64_t count_segments();
  void get_reports(uint32_t* rep_off, ReportRec* reps, ReportStats* stats);
  uint64_t count_reports();
  // accumulated kernel time (ms) per KernelId since the last reset
  void kernel_times(double* ms, uint64_t* launches);
  // overflow-list sizes of the last run: routes A, routes B, paths A, candidates
  void tier_counts(uint32_t* out4);
  // the kCtlWords control words of the last run (zeros before any run)
  void ctl_words(uint32_t* out);
  void reset_kernel_times();
  void set_timing(bool on) { timing_mask_ = on ? ~0u : 0u; }
  void set_timing_mask(uint32_t mask) { timing_mask_ = mask; }   // bit k: stage k (kernel_name)
  // Failure isolation: off (default), a trace that fails (kErrCandOverflow / kErrSearchOverflow /
  // kErrRounds) makes run() throw; on, run() returns, the failed traces carry no segments or
  // reports and their bits are in get_trace_errors().  The reference fails one request
  // (py/reporter_service.py:244-245) or skips one window (py/simple_reporter.py:169-173).
  void set_isolation(bool on) { isolate_ = on; }
  // Locality order of the stages that read the graph's regional data: 0 slot order, 1 K1 and K2
  // sorted by region, 2 the path stage too, -1 auto (2 on graphs of Engine::locality_default, 1
  // for batches sampled every >= 10 s on smaller ones, else 0).  Results are identical in every
  // mode.  Env RM_LOCALITY sets the initial value.
  void set_locality(int mode) { locality_ = mode; }
  bool locality_used() const { return locality_used_; }
  uint32_t error_bits() const { return err_bits_; }   // OR of the last run's per-trace errors
  void get_trace_errors(uint32_t* out);                // n_traces() words
  hipStream_t stream() const { return stream_; }
  const Engine& engine() const { return *eng_; }

  // Raw point stream -> per-vehicle time sort and inactivity windows of >= 2 points on the
  // GPU (simple_reporter.py:137-164), then every matching stage over the windows.
  void run_points(const PointsDesc& pd, const RunParams& rp);
  // vehicle index of every window of the last run_points (n_traces entries)
  void get_trace_uuid(uint32_t* out);
  // the batch the last run matched (after run_points: the windows built on the device)
  void get_batch(uint32_t* trace_off, float* lon, float* lat, double* time, float* acc);
  // Time tiles of the last run's reports: hour buckets, sort, privacy cull of (id, next_id)
  // runs and CSV text (simple_reporter.py:176-254).  Returns "name\0body\0" per file.  With
  // a communicator, rows of every rank are all-gathered and each rank emits the files it owns.
  std::string tiles(const TileParams& tp, struct TileComm* comm = nullptr);

 private:
  void ensure(uint64_t points, uint32_t traces, uint32_t nopts);
  void check_batch(uint32_t T, const uint32_t* trace_off, const MatchOptions* opts, uint32_t n_opts,
                   const uint32_t* trace_opt);
  void scan_options(const MatchOptions* opts, uint32_t n_opts);
  char* jdev_ = nullptr;        // device JSON path: trace-array bytes (grow-only), per-trace spans,
  uint64_t jcap_ = 0;           // flags and first / last times
  void* jspan_ = nullptr;
  uint32_t* jflag_ = nullptr;
  void* jtsp_ = nullptr;
  uint32_t jtcap_ = 0;
  void ensure_trans(uint64_t n, uint64_t n_src);
  void ensure_path(uint64_t n);
  void ensure_segs(uint64_t n);
  void ensure_turns();
  // the same, throwing OutOfDeviceMemory (ensure() retries a failed grown size at the exact one)
  void alloc_points(uint64_t cp, uint64_t ct, uint64_t co, uint64_t keep_trans, uint64_t keep_path, uint64_t keep_segs,
                    uint64_t keep_src);
  void ensure_trans_raw(uint64_t n, uint64_t n_src);
  void ensure_path_raw(uint64_t n);
  void ensure_segs_raw(uint64_t n);
  void ensure_global_search();
  void read_ctl();
  void tic(int k);
  void toc(int k);
  void harvest_times();
  // per-trace record lists (base[k], cnt[k] in units of `words` u64) compacted on the device and
  // downloaded through pinned memory into dst; off gets the T+1 offsets
  void download_compacted(const uint32_t* d_base, const uint32_t* d_cnt, const void* d_src, uint32_t words,
                          uint32_t* off, void* dst, const std::function<void*(uint64_t)>& dst_for);
  void grow_dl_host(size_t need);
  bool download_prefetched(uint32_t* off, void* dst, const std::function<void*(uint64_t)>& dst_for);
  void grow_dl_dev(size_t need);
  // small batches (run_small): no size read-back between the stages, one upload, one read-back
  bool run_small(const RunParams& rp, const DevGraph& g);
  // large batches once a run has sized the pools: no read-back between the stages (run_steady)
  bool run_steady(const RunParams& rp, const DevGraph& g);
  uint64_t steady_src_ = 0;    // the last ordinary / steady run's K2 sources (0: no steady run yet)
  uint32_t steady_ctl_[16] = {0};   // ... and its control words (the hand-over lists' lengths)
  void zero_hist(const RunParams& rp);
  void use_ws_inputs();
  void ensure_pack(uint64_t bytes);

  Engine* eng_;
  InputView in_;
  char* hpack_ = nullptr;      // pinned staging and device block of a small run()'s inputs (grow-only)
  char* dpack_ = nullptr;
  uint64_t pack_cap_ = 0;
  uint32_t* hoff_ = nullptr;   // pinned: a small run's per-trace segment offsets (T + 1), prefetched
  uint64_t hoff_cap_ = 0;
  bool seg_prefetched_ = false;
  void* dl_dev_ = nullptr;     // grow-only device / pinned host buffers of download_compacted
  void* dl_host_ = nullptr;
  size_t dl_dev_bytes_ = 0, dl_host_bytes_ = 0;
  hipStream_t stream_ = nullptr;
  Workspace ws_;
  uint32_t n_traces_ = 0;
  uint64_t n_points_ = 0, n_trans_ = 0, n_path_ = 0, seg_used_ = 0;
  uint32_t timing_mask_ = 0;   // stages timed by HIP events
  bool has_report_ = false;
  bool isolate_ = false;
  int locality_ = -1;
  bool batch_sparse_ = false;     // the last run()'s batch is sampled sparsely (kLocalitySparseS)
  bool locality_used_ = false;
  void ensure_sort(uint64_t n);
  uint32_t err_bits_ = 0;
  uint32_t* hctl_ = nullptr;  // pinned host mirror of the control words
  StageBufs sb_;
  bool from_points_ = false;
  uint32_t mode_mask_ = 0;   // travel modes of the batch (bit per Mode): which route balls K2 needs
  uint32_t turn_mask_ = 0;   // modes of the batch with a turn_penalty_factor > 0: turn rows, route_d
  float batch_radius_ = 0.f; // the batch's largest search_radius (m): K1's grid (Engine::k1_grid)
  void ensure_points(uint64_t n, uint32_t n_uuids, uint32_t n_opts);
  void ensure_rows(uint64_t n, uint32_t traces);
  struct Ev { hipEvent_t a, b; int k; };
  std::vector<Ev> pending_, free_ev_;
  double kms_[kNumKernels] = {0};
  uint64_t klaunch_[kNumKernels] = {0};
};

// K1's grid refinement for a graph (host only; engine.hip): each graph-file cell split f x f
uint32_t choose_grid_split(const Graph& g);
// the same for queries of radius_m (the padded box of that radius)
uint32_t choose_grid_split_for(const Graph& g, float radius_m);

// one K1 grid in HBM: its cell ranges, self-contained cell records and geometry
struct K1Grid {
  const uint32_t* cell_off = nullptr;
  const uint4* cell_rec = nullptr;
  double lon0 = 0, lat0 = 0, dlon = 0, dlat = 0;
  uint32_t ncx = 0, ncy = 0, split = 1;
};

class Engine {
 public:
  Engine(const Graph& g, int device);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;
  const DevGraph& dev() const { return dg_; }
  // copy of the device view taken under the ball lock (tables may be added concurrently)
  DevGraph dev_snapshot() const;
  int device() const { return device_; }
  const Graph& host() const { return host_; }
  uint32_t n_segments() const { return host_.num_segments(); }
  // build (once) the route balls of every mode in `mode_mask` (bit per Mode); thread-safe
  void ensure_balls(uint32_t mode_mask);
  // build (once) the turn rows of the built tables of every mode in `mode_mask`; thread-safe
  void ensure_turn_rows(uint32_t mode_mask);
  uint32_t turn_row_mask() const { return dg_.ball_turn_mask; }
  double turn_build_ms(int mode) const { return mode >= 0 && mode <= kModePedestrian ? turn_ms_[mode] : 0.0; }
  // ball radius in cm for modes built from now on (0 disables the ball tier)
  void set_ball_radius(uint32_t radius_cm);
  uint32_t ball_radius() const { return ball_radius_cm_; }
  // stats of one mode's tables: {keys, table entries, nodes without a table, build ms}
  void ball_stats(int mode, double* out4) const;
  // radius (cm) the mode's tables were built at (0: none; its transitions use the search tiers)
  uint32_t mode_ball_radius(int mode) const;
  // modes whose tables were built on the GPU (bit per Mode)
  uint32_t ball_gpu_mask() const { return ball_gpu_; }
  // keys[2i], keys[2i+1] from node from[i] to road[i]'s node0 / node1 through the built tables
  // of `mode`, probed on the device as K2 does (all-ones: outside the ball / no table)
  void ball_lookup(int mode, uint64_t n, const uint32_t* from, const uint32_t* road, uint64_t* keys, uint8_t* preds);
  // K1's grid: each cell of the graph's grid split f x f (1 = the graph's grid)
  uint32_t grid_split() const { return grid_split_; }
  // K1's grid for a batch whose largest query radius is radius_m: the default one, or a second
  // split built when wider queries read fewer items on it (grid_alt_radius() and up)
  void k1_grid(float radius_m, DevGraph& g) const;
  uint32_t grid_alt_split() const { return n_grids_ > 1 ? grids_[1].split : 0u; }
  float grid_alt_radius() const { return grid_alt_radius_; }
  // locality order by default (Matcher::set_locality -1): graphs whose route tables and cell
  // records outgrow the L2s; and the shift from K1 grid cells to the coarse sort cells (~500 m)
  bool locality_default() const { return locality_default_; }
  uint32_t locality_shift() const { return locality_shift_; }
  uint32_t locality_bits() const { return locality_bits_; }

 private:
  int device_;
  Graph host_;
  DevGraph dg_{};
  std::vector<void*> allocs_;
  mutable std::mutex ball_mu_;
  uint32_t ball_radius_cm_ = 40000;   // set from auto_ball_radius_cm(graph) at construction
  uint32_t ball_built_ = 0;             // mode bits
  uint32_t ball_gpu_ = 0;               // mode bits built on the GPU
  uint32_t grid_split_ = 1;
  K1Grid grids_[2];
  int n_grids_ = 1;
  float grid_alt_radius_ = 0.f;         // batches with a query radius from this take grids_[1]
  bool locality_default_ = false;
  uint32_t locality_shift_ = 0, locality_bits_ = 0;
  uint64_t ball_bytes_ = 0;             // bytes of the tables built so far (all modes)
  uint32_t turn_tried_ = 0;             // modes whose turn rows were attempted (ensure_turn_rows)
  double turn_ms_[5] = {};
  bool build_balls_gpu(int mode, uint32_t radius_cm, uint32_t max_keys, uint64_t avail_bytes);
  double ball_info_[5][4] = {};
};

}  // namespace rm
