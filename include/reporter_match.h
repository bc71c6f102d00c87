/* reporter_match.h — C-ABI of libreporter_match.so, the MI355X (gfx950) map
 * matcher that replaces Valhalla/meili behind Open Traffic Reporter.
 *
 * Drop-in boundary (what the reference binds):
 *   valhalla.Configure(conf)             reference py/reporter_service.py:284, py/simple_reporter.py:132
 *       -> rm_configure
 *   valhalla.SegmentMatcher()            reference py/reporter_service.py:52,  py/simple_reporter.py:133
 *       -> rm_matcher_create / rm_matcher_destroy
 *   SegmentMatcher.Match(json) -> json   reference py/reporter_service.py:240, py/simple_reporter.py:166
 *       -> rm_match (+ rm_free for the returned string)
 * The Python package `valhalla/` in this repository binds exactly these through
 * ctypes, so reporter_service.py runs unchanged.
 *
 * Conventions: plain pointers and sizes, no C++ or torch types.  Return 0 on
 * success, non-zero on error; the message is in rm_last_error() (thread-local).
 * Distinct matchers/runners may be used concurrently from different threads;
 * one handle must not be used by two threads at once (the reference keeps one
 * SegmentMatcher per thread, py/reporter_service.py:28-29,51-52).
 */
#ifndef REPORTER_MATCH_H
#define REPORTER_MATCH_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RM_ABI_VERSION 1

/* ---------------- errors / device ---------------- */
const char* rm_last_error(void);
int rm_abi_version(void);
int rm_set_device(int device);  /* device used by the next rm_configure / rm_engine_create */
int rm_device_count(int* count);

/* ---------------- drop-in boundary (valhalla module) ---------------- */
typedef struct rm_matcher rm_matcher;
/* Reads a Valhalla-style JSON config: "meili" defaults (+ per-mode sections) and
 * the graph file ("reporter_amd": {"graph": path} or "mjolnir": {"tile_extract": *.rmg}),
 * loads the graph into HBM.  err/errlen may be NULL. */
int rm_configure(const char* conf_json_path, char* err, size_t errlen);
rm_matcher* rm_matcher_create(void);            /* NULL on error (no configure yet) */
void rm_matcher_destroy(rm_matcher* m);
/* trace_json: {"uuid", "trace":[{"lat","lon","time"[,"accuracy"]}...], "match_options":{...}}
 * *out_json: {"segments":[...]} allocated by the library; release with rm_free. */
int rm_match(rm_matcher* m, const char* trace_json, char** out_json);
/* n traces at once (one GPU launch sequence); outs[i] must each be freed with rm_free. */
int rm_match_batch(rm_matcher* m, const char* const* traces, size_t n, char** outs);
/* rm_match_batch with the n replies in one malloc'd, NUL-terminated buffer: reply i is
 * (*buf)[off[i], off[i+1]) (off: n+1 entries, caller-allocated).  One allocation and one free
 * (rm_free(*buf)) instead of n: the Python binding reads the replies out of one memoryview. */
int rm_match_batch_packed(rm_matcher* m, const char* const* traces, size_t n, char** buf, uint64_t* off);
void rm_free(char* p);
/* Host wall times (ms) of the matcher's last uncoalesced rm_match_batch: out[0] JSON parse
 * (single pass, up to 16 host threads), [1] staging into pinned host arrays, [2] engine run
 * (H2D of the batch + every kernel + its size read-backs), [3] segment download (D2H),
 * [4] reply formatting, [5] total. */
int rm_matcher_timing(const rm_matcher* m, double out[6]);
/* Request coalescing (on unless the config sets "reporter_amd": {"coalesce": false}):
 * concurrent rm_match calls from many threads are queued and run as one GPU batch by a
 * dispatcher thread; "coalesce_window_ms" (default 0: take whatever queued while the
 * previous batch ran) and "coalesce_max_traces" (16384) shape the batches.
 * out: [0] batches run [1] requests served [2] largest batch [3] requests queued now. */
int rm_coalesce_stats(uint64_t out[4]);
/* Dispatcher wall time (ms, summed over the batches since rm_configure): [0] staging the parsed
 * points into pinned memory, [1] the engine run (uploads, kernels, size read-backs), [2] the
 * segment download, [3] reply formatting.  Parsing runs on the calling threads, not here. */
int rm_coalesce_timing(double out[4]);

/* ---------------- matcher options (layout of rm::MatchOptions) ---------------- */
typedef struct {
  int32_t mode;  /* 0 auto, 1 bus, 2 motor_scooter, 3 bicycle, 4 pedestrian */
  float sigma_z, beta, search_radius, gps_accuracy, breakage_distance, interpolation_distance,
      max_route_distance_factor, max_route_time_factor, turn_penalty_factor;
} rm_options;
void rm_default_options(rm_options* o);

/* ---------------- synthetic world (host only; no GPU needed) ---------------- */
typedef struct {
  uint32_t rows, cols;
  double block_m;
  uint64_t seed;
  double center_lat, center_lon, jitter;
  uint32_t arterial_every, highway_every;
  double segment_max_m, internal_m, service_frac, oneway_frac, curve_frac, cell_m;
} rm_world_params;
void rm_default_world_params(rm_world_params* p);
int rm_world_build(const rm_world_params* p, const char* out_path);
/* counts of a graph file: nodes, edges, roads, verts, segments, cells, cell items */
int rm_graph_info(const char* graph_path, uint64_t out[7]);
/* OpenStreetMap exchange (graph_osm.cpp; the reference builds its Valhalla tiles from OSM,
 * py/get_tiles.py:30-102, py/simple_reporter.py:36-49).  rm_graph_export_osm writes an .rmg
 * graph as OSM XML: routing tags (highway, maxspeed, oneway, access) on one way per road,
 * exact reporter:* tags, one type=osmlr relation per OSMLR segment, the grid geometry in a
 * type=reporter_grid relation.  rm_graph_import_osm reads OSM XML into an .rmg: an exported
 * file comes back bit-identical; any other OSM XML is split into roads at intersections with
 * speeds / access from its tags and a grid index of cell_m metres (OSMLR segments only where
 * osmlr relations give them). */
int rm_graph_export_osm(const char* graph_path, const char* osm_path);
/* The same OSM elements as OSM PBF (the input valhalla_build_tiles reads, reference
 * Dockerfile:42-49): zlib-deflated blobs, an OSMHeader (OsmSchema-V0.6, DenseNodes), dense
 * nodes at nanodegree granularity (exact float coordinates; a reporter:ll tag where nanodegrees
 * would not bring a float back), ways and relations with packed delta-coded refs. */
int rm_graph_export_pbf(const char* graph_path, const char* pbf_path);
/* OSM XML or PBF (told apart by content) -> .rmg. */
int rm_graph_import_osm(const char* osm_path, const char* graph_path, double cell_m);
/* A seeded irregular city written as generic OSM (osm_city.cpp), with no reporter:* tags, so
 * rm_graph_import_osm ingests it as it would an extract: a jittered junction lattice of curved
 * multi-vertex ways, diagonal avenues crossing at 9-road hubs, roundabouts, boulevards of one-way
 * carriageway pairs, one-way streets, dead ends, service loops, foot / cycle paths, a trunk road
 * on bridges joined at ramps, type=osmlr relations on part of the ways only, OSM ids in shuffled
 * chunks.  pbf != 0 writes PBF, else XML (the same elements). */
typedef struct {
  uint32_t rows, cols;
  double block_m;
  uint64_t seed;
  double center_lat, center_lon, jitter;
  uint32_t primary_every, secondary_every, boulevard_every, diagonal_every;
  double roundabout_frac, drop_frac, oneway_frac, spur_frac, service_frac, footway_frac, osmlr_local_frac,
      way_max_m;
  uint32_t trunk;
} rm_city_params;
void rm_default_city_params(rm_city_params* p);
int rm_osm_city_write(const rm_city_params* p, const char* osm_path, int pbf);

typedef struct {
  uint32_t n_traces, n_points;
  double rate_s, noise_m;
  uint64_t seed;
  int32_t mode;
  int64_t start_epoch;
  uint32_t threads;
} rm_trace_params;
void rm_default_trace_params(rm_trace_params* p);
/* Arrays sized n_traces*n_points; truth_* may be NULL. */
int rm_traces_generate(const char* graph_path, const rm_trace_params* p, double* lon, double* lat, double* time,
                       float* accuracy, uint32_t* truth_edge, uint32_t* truth_off_cm);
/* p->n_traces traces; slot k holds trace ids[k] of the seeded set (identical to what
 * rm_traces_generate puts at index ids[k]): one rank generates just its uuid shard. */
int rm_traces_generate_ids(const char* graph_path, const rm_trace_params* p, const uint32_t* ids, double* lon,
                           double* lat, double* time, float* accuracy, uint32_t* truth_edge, uint32_t* truth_off_cm);

/* ---------------- batched array API (bench / batch pipeline / parity tests) ---------------- */
typedef struct rm_engine rm_engine;
typedef struct rm_runner rm_runner;

rm_engine* rm_engine_create(const char* graph_path, int device);
void rm_engine_destroy(rm_engine* e);
uint32_t rm_engine_n_segments(const rm_engine* e);
int rm_engine_segment_ids(const rm_engine* e, uint64_t* ids); /* n_segments ids (dense index -> OSMLR id) */
/* Route balls (K2's lookup tier): per node and travel mode, exact shortest (dist, time) keys
 * to every node within `radius_m`, built once per mode on first use.  Transitions whose
 * route bound fits the radius are answered by table probes instead of a bounded search;
 * results are identical either way.  radius_m 0 disables the tier.  Set before the first
 * run (modes already built keep their tables).  0..10000 m.  Default: env RM_BALL_RADIUS_M,
 * else rm_graph_auto_ball_radius of the graph. */
int rm_engine_set_ball_radius(rm_engine* e, double radius_m);
/* Host-only: the engine's automatic radius for a graph file — the largest of 2000 m (meili's
 * default breakage distance, so every default-bounded transition is a table probe), 1500,
 * 1000, 700, 500 m whose estimated tables stay within 72 GiB per mode (RM_BALL_BUDGET_GB) and
 * 2^33 rows; else 400 m. */
int rm_graph_auto_ball_radius(const char* graph_path, double* radius_m);
/* Host-only: the radius a travel mode's tables are built at when avail_gb GiB of HBM are left
 * for them — the largest of start_m and the radii below it (2000, 1500, 1000, 700, 500, 400,
 * 300, 200 m) whose sampled tables for that mode (+10 %) fit avail_gb and 2^33 rows; 0 when none
 * does (the mode's transitions then run in the search tiers).  The engine applies it per mode
 * with avail = min(per-mode budget, half the device's HBM less earlier modes' tables, free HBM
 * less 4 GiB); auto and bus share one build. */
int rm_graph_fit_ball_radius(const char* graph_path, int mode, double start_m, double avail_gb, double* radius_m);
/* Host-only: sampled ball statistics of `mode` at radius_m (bounded searches from 256 nodes):
 * out[3] = mean nodes per ball, estimated table bytes of all nodes, fraction of balls above
 * 4096 nodes. */
int rm_graph_ball_sample(const char* graph_path, int mode, double radius_m, double out[3]);
/* out[6]: radius m, keys stored, table entries (16 B each), nodes without a table, build ms,
 * 1 when the tables were built on the GPU (small balls on large graphs; env RM_BALL_BUILD=host|gpu) */
int rm_engine_ball_stats(const rm_engine* e, int mode, double out[6]);
/* K1's spatial index: the graph file's grid with each cell split f x f (*f = 1: the file's grid),
 * chosen at upload to minimise the items a default-radius query reads (RM_GRID_SPLIT overrides).
 * It changes which grid items are read, never which roads are found. */
int rm_engine_grid_split(const rm_engine* e, uint32_t* f);
/* K1's second grid (engine.hip Engine::k1_grid): its split f (0: none) and the batch query
 * radius (m) from which a batch takes it instead of the default one.  New in round 5: no
 * reference call site (the reference has no grid index; Valhalla's meili owns its own). */
int rm_engine_grid_alt(const rm_engine* e, uint32_t* f, float* radius_m);
/* turn rows (DESIGN.md §3 rule 3b) built so far: bit per travel mode, and each mode's build ms */
int rm_engine_turn_rows(const rm_engine* e, uint32_t* mode_mask, double* build_ms /*5*/);
/* Host-only: the grid refinement an engine would choose for a graph file. */
int rm_graph_grid_split(const char* graph_path, uint32_t* f);
/* The engine's own tables of `mode` (built by a run that used the mode), probed on the device as
 * K2 probes them: keys[2i], keys[2i+1] from node from[i] to road[i]'s node0 / node1, all-ones
 * outside the ball or for a node without a table; preds (may be NULL) gets the rows' canonical
 * predecessor indices of node0 / node1 (7: none stored).  Compare with rm_balls_lookup. */
int rm_engine_ball_lookup(rm_engine* e, int mode, uint64_t n, const uint32_t* from, const uint32_t* road,
                          uint64_t* keys, uint8_t* preds);
/* Host-only check of the ball tables (no GPU): builds the balls of `mode` for the graph
 * file and looks up n (from node, road) pairs the way the K2 kernel probes them;
 * keys[2i], keys[2i+1] = dist_cm << 32 | time_ms from `from` to the road's node0 / node1,
 * all-ones for an endpoint outside the ball (or `from` without a table).  preds (may be NULL):
 * preds[2i], preds[2i+1] = the index, among the endpoint's in-edges in edge-id order, of its
 * canonical predecessor in the search from `from` (smallest-id usable in-edge u -> v with
 * key(from -> u) + key(u -> v) == key(from -> v)); 7 when the endpoint is `from`, outside the
 * ball, or the index is 7 or more.  Returns 0 / -1. */
int rm_balls_lookup(const char* graph_path, int mode, double radius_m, uint64_t n, const uint32_t* from,
                    const uint32_t* road, uint64_t* keys, uint8_t* preds);

rm_runner* rm_runner_create(rm_engine* e);
void rm_runner_destroy(rm_runner* r);

typedef struct {
  uint32_t n_traces;
  const uint32_t* trace_off;  /* n_traces+1 */
  const float* lon;           /* degrees */
  const float* lat;
  const double* time;         /* epoch seconds */
  const float* accuracy;      /* metres, < 0 when absent */
  uint32_t n_opts;
  const rm_options* opts;
  const uint32_t* trace_opt;  /* per trace index into opts */
} rm_batch_desc;

typedef struct {
  double threshold_sec;       /* reporter_service.py:55-58 (default 15) */
  uint32_t report_mask;       /* bit (level+1) set when level is reported; {0,1} = 0x6 */
  uint32_t transition_mask;
  uint32_t* hist_dev;         /* device pointer, n_segments*16 u32 speed histogram, may be NULL */
  int32_t do_report;          /* run the report() epilogue */
  int32_t zero_hist;          /* zero hist_dev (and dur_dev) on the runner's stream before the epilogue */
  uint64_t* dur_dev;          /* device pointer, n_segments u64: per OSMLR segment the sum of the reports'
                                 whole-second durations int(round(t1 - t0)) (the tile rows' duration
                                 column, py/simple_reporter.py:179) over the reports the histogram counts;
                                 may be NULL.  Integer sums, so the multi-GPU all-reduce is exact */
} rm_run_params;
void rm_default_run_params(rm_run_params* p);

/* upload + run every kernel; blocks until done */
int rm_runner_run(rm_runner* r, const rm_batch_desc* b, const rm_run_params* p);
/* run again over the batch already resident in HBM (bench steps) */
int rm_runner_rerun(rm_runner* r, const rm_run_params* p);
/* rerun n runners (contiguous parts of one batch, same engine) concurrently, one host thread
 * per part, so their kernels overlap on their streams; with zero_hist the shared histogram is
 * zeroed once before any part reports.  Returns the first part's error. */
int rm_runners_rerun(rm_runner* const* rs, uint32_t n, const rm_run_params* p);
/* out: [0] points [1] traces [2] transitions [3] path edges [4] segments [5] reports
 *      [6] route pairs sent to the wave tier [7] ... to the single-source tier
 *      [8] transitions sent to the path wave tier [9] states sent to the candidate wave tier */
int rm_runner_sizes(rm_runner* r, uint64_t out[10]);
/* K2 tier hand-overs of the last run: [0] items the ball tier passed to the search tiers,
 * [1] items the register search tier passed on, [2] items the second register tier passed on,
 * [3] chosen transitions the path ball tier passed to the path search tiers,
 * [4] route items the LDS wave tier passed to the global-memory tier, [5] likewise for paths,
 * [6] route items the 16-lane group tier passed to the 512-slot wave tier, [7] likewise for paths,
 * [8] route items the 512-slot wave tier passed to the 4096-slot one, [9] likewise for paths */
int rm_runner_route_tiers(rm_runner* r, uint64_t out[10]);
int rm_runner_get_states(rm_runner* r, uint32_t* n_states, uint32_t* state_orig);
int rm_runner_get_candidates(rm_runner* r, uint8_t* cand_n, uint32_t* road, uint32_t* s_cm, float* sq);
int rm_runner_get_routes(rm_runner* r, uint32_t* trans_off, double* gc, uint32_t* route_cm);
/* with turn costs (DESIGN.md §3 rule 3b): every transition's distance term turn_m + |route_m - gc|
 * in metres (+inf when invalid), as the Viterbi adds it; *present = 0 (nothing written) when no
 * trace of the last run had turn costs */
int rm_runner_get_route_terms(rm_runner* r, double* route_d, int* present);
int rm_runner_get_viterbi(rm_runner* r, int8_t* choice, uint8_t* chain_start);
int rm_runner_get_paths(rm_runner* r, uint32_t* path_off, uint32_t* path_cnt, uint32_t* path_edges, uint32_t* route_dist);
/* segments: 56-byte records (rm::SegmentRec); seg_off has n_traces+1 entries */
int rm_runner_get_segments(rm_runner* r, uint32_t* seg_off, void* segs);
/* reports: 48-byte records (rm::ReportRec); stats: 40-byte rm::ReportStats per trace */
int rm_runner_get_reports(rm_runner* r, uint32_t* rep_off, void* reps, void* stats);
/* Failure isolation (default off: a trace that fails makes rm_runner_run return non-zero).
 * On: a trace that fails on its own — more than 192 roads inside its search radius, a route
 * search beyond every tier's capacity, a path that cannot be rebuilt — gets no segments and no
 * reports, the run succeeds for every other trace, and rm_runner_trace_errors gives the bits
 * (1 candidates, 2 route search, 8 path reconstruction) per trace.  The reference fails just
 * that request (py/reporter_service.py:244-245) or skips just that window
 * (py/simple_reporter.py:169-173). */
int rm_runner_set_isolation(rm_runner* r, int on);
int rm_runner_trace_errors(rm_runner* r, uint32_t* errs);   /* n_traces words of the last run */
/* Locality order of the stages that read regional graph data (K1 cell records, K2 route-ball
 * tables, the path walk): the state slots are sorted each step into the Morton-ordered cells of a
 * 64 x 64 grid over the graph (a counting sort) and those stages take their work in that order,
 * XCD-contiguously, so one region's tables meet in one L2.  mode 0: slot order; 1: K1 and K2 in
 * locality order; 2: the path stage too; -1 (default): 2 on graphs of >= 150 k nodes (env
 * RM_LOCALITY_NODES), 1 for batches sampled every >= 10 s on average on smaller graphs, else 0.
 * Env RM_LOCALITY sets the initial mode.  Results are identical in every mode.  *used: whether
 * the last run used it. */
int rm_runner_set_locality(rm_runner* r, int mode);
int rm_runner_locality_used(rm_runner* r, int* used);
/* per-kernel HIP-event timing on the runner's stream */
int rm_runner_set_timing(rm_runner* r, int on);
/* time only the stages whose bit is set (bit k = rm_kernel_name(k)): fewer event records in a timed region */
int rm_runner_set_timing_mask(rm_runner* r, uint32_t mask);
int rm_runner_kernel_times(rm_runner* r, double* ms, uint64_t* launches, int n);
int rm_runner_reset_times(rm_runner* r);
const char* rm_kernel_name(int k);
int rm_num_kernels(void);

/* ---------------- report() on host-supplied segment lists ----------------
 * The device report() epilogue (reference py/reporter_service.py:79-179) over segment lists
 * that did not come from the matcher: trace k's segments are segs[seg_off[k] .. seg_off[k+1])
 * (56-byte rm::SegmentRec), its last point's time trace_end_time[k] (:81), its threshold and
 * level masks per trace.  Reports come back compacted per trace (rep_off: n_traces+1 offsets,
 * reps: room for seg_off[n_traces] 48-byte records), stats: 40-byte rm::ReportStats per trace.
 * Uses the device of rm_set_device. */
typedef struct {
  uint32_t n_traces;
  const uint32_t* seg_off;
  const void* segs;
  const double* trace_end_time;
  const double* threshold_sec;
  const uint32_t* report_mask;      /* bit (level+1) per reported level */
  const uint32_t* transition_mask;
} rm_report_desc;
int rm_report_segments(const rm_report_desc* d, uint32_t* rep_off, void* reps, void* stats);

/* ---------------- batch-pipeline stages around the matcher (reference py/simple_reporter.py) ----------------
 * rm_runner_run_points replaces the per-vehicle grouping, time sort and inactivity
 * windowing of simple_reporter.match (py/simple_reporter.py:137-164) with a device sort,
 * then matches every window of >= 2 points (as rm_runner_run).
 * rm_runner_tiles replaces the hour bucketing of the valid reports (:176-196) and the
 * report phase's sort, privacy cull and CSV (:211-254): it returns, per tile file,
 * "name\0body\0" where name is "<start>_<end>/<level>/<tile index>" and body the text
 * the reference uploads.  With a communicator the rows of every rank are all-gathered
 * and each rank returns the files it owns (file key hashed over ranks). */
typedef struct rm_comm rm_comm;
typedef struct {
  uint64_t n_points;
  const uint32_t* uuid;       /* dense vehicle index per point (< n_uuids) */
  const double* time;         /* epoch seconds (integers in the reference, :140) */
  const float* lon;
  const float* lat;
  const float* accuracy;      /* may be NULL */
  double inactivity_sec;      /* --inactivity, default 120 (:344) */
  uint32_t n_uuids;
  uint32_t n_opts;
  const rm_options* opts;
  const uint32_t* uuid_opt;   /* per vehicle index into opts; NULL = opts[0] for all */
} rm_points_desc;
int rm_runner_run_points(rm_runner* r, const rm_points_desc* d, const rm_run_params* p);
/* vehicle index of each matched window of the last rm_runner_run_points (n_traces entries) */
int rm_runner_get_trace_uuid(rm_runner* r, uint32_t* uuid);
/* the batch the last run matched: trace_off (n_traces+1), lon, lat, time, accuracy (n_points) */
int rm_runner_get_batch(rm_runner* r, uint32_t* trace_off, float* lon, float* lat, double* time, float* accuracy);
typedef struct {
  uint32_t quantisation;      /* --quantisation, default 3600 (:343) */
  uint32_t privacy;           /* --privacy, default 2 (:345) */
  const char* source;         /* --source-id, default "smpl_rprt" (:346) */
  const char* mode;           /* vehicle type column, upper-cased (:194) */
} rm_tile_params;
void rm_default_tile_params(rm_tile_params* p);
/* blob is library-allocated (free with rm_free); comm may be NULL */
int rm_runner_tiles(rm_runner* r, const rm_tile_params* p, rm_comm* comm, char** blob, size_t* len);

/* ---------------- RCCL over xGMI (multi-GPU histogram exchange) ----------------
 * One process per GPU.  Replaces the reference's keyed Kafka repartition of
 * "id next_id" reports (BatchingProcessor.java:126) with one all-reduce of the
 * per-OSMLR-segment speed histogram.  Rank 0 creates the id, every rank inits. */
int rm_comm_unique_id(uint8_t id_out[128]);
rm_comm* rm_comm_init(int nranks, int rank, const uint8_t id[128], int device);
void rm_comm_destroy(rm_comm* c);
/* dtype: 0 u32, 1 u64, 2 f64; op: 0 sum, 1 max.  In place on a device buffer (a host buffer on a
 * device -1 host-transport communicator); blocks until done. */
int rm_comm_allreduce(rm_comm* c, void* dev_buf, size_t count, int dtype, int op);
/* The optional exchange of SURVEY §8(e): each rank owns one segment-id range.  buf holds nranks
 * chunks of count_per_rank elements; on return chunk `rank` holds the reduction of every rank's
 * chunk `rank` (RCCL reduce-scatter, in place), the other chunks are unspecified.  Half the bytes
 * per rank of an all-reduce; buffers as rm_comm_allreduce.  For the speed histogram (16 bins per
 * segment) count_per_rank must be 16 x the segments per rank, so no segment's bins are split. */
int rm_comm_reduce_scatter(rm_comm* c, void* buf, size_t count_per_rank, int dtype, int op);
/* all-reduce of one host double (op as above) */
int rm_comm_allreduce_host_f64(rm_comm* c, double* value, int op);
int rm_comm_barrier(rm_comm* c);
/* A communicator over a host transport the caller supplies (e.g. the gloo backend of an
 * existing job, or a test harness): fn must be a blocking all-gather across the nranks callers,
 * placing every rank's `bytes` bytes of send at recv + rank * bytes, and return 0.  Every rm_comm
 * operation then runs over it (device buffers staged through host memory); device -1 makes a
 * host-only communicator (rm_comm_allreduce_host_f64 and rm_comm_barrier work without a GPU). */
typedef int (*rm_host_allgather_fn)(void* ctx, const void* send, size_t bytes, void* recv);
rm_comm* rm_comm_init_host(int nranks, int rank, rm_host_allgather_fn fn, void* ctx, int device);
/* Host-only: the rank that culls and writes time-tile file (bucket, level | tile index << 3) when
 * rm_runner_tiles runs with an nranks communicator (the device filter uses the same function). */
int rm_tile_file_owner(uint64_t bucket, uint32_t tile, int nranks);

/* ---------------- device memory helpers (histograms without a framework) ---------------- */
int rm_device_alloc(size_t bytes, void** dev_ptr);
int rm_device_free(void* dev_ptr);
int rm_device_memset(void* dev_ptr, int value, size_t bytes);
int rm_device_download(void* host_dst, const void* dev_src, size_t bytes);
int rm_device_upload(void* dev_dst, const void* host_src, size_t bytes);
int rm_device_synchronize(void);

#ifdef __cplusplus
}
#endif
#endif
