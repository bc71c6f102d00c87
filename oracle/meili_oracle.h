/* ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py
 * cpu_baseline).  Never linked into or called by the product path.
 *
 * meili_oracle: plain-C, single-threaded CPU restatement of the map matcher
 * that Valhalla 2.4.5's meili runs behind valhalla.SegmentMatcher().Match
 * (reference call sites py/reporter_service.py:240, py/simple_reporter.py:166;
 * version pin Dockerfile:7).  meili's source is NOT under /root/reference and
 * cannot be fetched offline, so this file restates its
 * published HMM design — candidate search, bounded route search, Viterbi,
 * segment forming — with every tie-break and rounding rule written out
 * (DESIGN.md §3).  PARITY vs REAL MEILI: UNPINNED.  What is pinned:
 *   - og_report_trace() against the reference's own report() golden vectors
 *     (tests/golden/report_golden.json);
 *   - the GPU engine against this oracle, bit-exact, on identical inputs.
 */
#ifndef MEILI_ORACLE_H
#define MEILI_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint32_t n_nodes, n_edges, n_roads, n_verts, n_segments;
  const uint32_t* node_off;      /* N+1 CSR offsets */
  const uint32_t* edges;         /* 4*E: target, len_cm, info, road<<1|rev */
  const uint32_t* edge_seg;      /* E: dense segment index or 0xffffffff */
  const uint32_t* edge_seg_off;  /* E */
  const uint32_t* edge_way;      /* E */
  const uint32_t *road_node0, *road_node1, *road_fwd, *road_rev, *road_len_cm, *road_vert_off;
  const uint32_t* verts;         /* 4*V: lon (f32 bits), lat (f32 bits), cum_cm, road */
  const uint64_t* seg_id;        /* S */
  const uint32_t* seg_len_cm;    /* S */
  double lon0, lat0, dlon, dlat;
  uint32_t ncx, ncy;
  const uint32_t* cell_off;
  const uint32_t* cell_item;
} og_graph;

typedef struct {
  int32_t mode;
  float sigma_z, beta, search_radius, gps_accuracy, breakage_distance, interpolation_distance,
      max_route_distance_factor, max_route_time_factor, turn_penalty_factor;
} og_options;

typedef struct {
  uint32_t n_traces;
  const uint32_t* trace_off;  /* T+1 */
  const float* lon;
  const float* lat;
  const double* time;
  const float* accuracy;      /* < 0: absent */
  const og_options* opts;
  const uint32_t* trace_opt;  /* per trace option index */
} og_batch;

typedef struct {             /* same layout as rm::SegmentRec */
  uint64_t segment_id;
  double start_time, end_time;
  int32_t length, queue_length;
  uint32_t flags;             /* bit0 internal, bit1 has id */
  uint32_t begin_shape_index, end_shape_index;
  uint32_t seg_dense, way_first, way_last;
} og_segment;

typedef struct {             /* same layout as rm::ReportRec */
  uint64_t id, next_id;
  double t0, t1;
  int32_t length, queue_length;
  uint32_t seg_dense, pad;
} og_report;

typedef struct {             /* same layout as rm::ReportStats */
  int32_t successful_count, unreported_count;
  int32_t successful_length_m, unreported_length_m;
  int32_t discontinuities, invalid_speeds, invalid_times, unassociated;
  int32_t shape_used, n_reports;
} og_stats;

typedef struct og_result og_result;

/* Runs the full matcher over a batch. Returns NULL on allocation failure. */
og_result* og_match(const og_graph* g, const og_batch* b);
void og_free(og_result* r);

/* sizes of the variable-length outputs */
void og_sizes(const og_result* r, uint64_t* n_points, uint64_t* n_trans, uint64_t* n_path_edges,
              uint64_t* n_segments);

/* Per-layer arrays (indexed by point slot: state s of trace k at trace_off[k]+s). */
void og_get_states(const og_result* r, uint32_t* n_states /*T*/, uint32_t* state_orig /*P*/);
void og_get_candidates(const og_result* r, uint8_t* cand_n /*P*/, uint32_t* road /*P*16*/,
                       uint32_t* s_cm /*P*16*/, float* sq /*P*16*/);
void og_get_routes(const og_result* r, uint32_t* trans_off /*P*/, double* gc /*P*/, uint32_t* route_cm /*n_trans*/);
/* turn weight U of every transition (0 without turn costs or along one road; DESIGN.md §3 rule 3b) */
void og_get_route_turns(const og_result* r, uint32_t* route_turn /*n_trans*/);
/* every transition's distance term turn_m + |route_m - gc| (metres; +inf invalid), as S3 adds it */
void og_get_route_terms(const og_result* r, double* route_d /*n_trans*/);
/* per road: the headings (whole degrees, 8-bit Valhalla steps) at node0 and node1 into the road */
void og_road_heads(const og_graph* g, uint16_t* h0 /*n_roads*/, uint16_t* h1 /*n_roads*/);
void og_get_viterbi(const og_result* r, int8_t* choice /*P*/, uint8_t* chain_start /*P*/);
void og_get_paths(const og_result* r, uint32_t* path_off /*P*/, uint32_t* path_cnt /*P*/,
                  uint32_t* path_edges /*n_path_edges*/, uint32_t* route_key_dist /*P*/);
void og_get_segments(const og_result* r, uint32_t* seg_off /*T+1*/, og_segment* segs /*n_segments*/);

/* Post-match report() restatement (reference py/reporter_service.py:79-179).
 * levels are bitmasks: bit (level+1) set when level is in the set (bit 0 = None/-1).
 * Writes at most n_segs reports; returns the count. */
int og_report_trace(const og_segment* segs, uint32_t n_segs, double trace_end_time, double threshold_sec,
                    uint32_t report_mask, uint32_t transition_mask, og_report* out, og_stats* stats);

/* Whole CPU pipeline for the baseline: match + report + speed histogram.
 * hist: n_segments*16 u32 (may be NULL). Returns the number of reports. */
uint64_t og_pipeline(const og_graph* g, const og_batch* b, double threshold_sec, uint32_t report_mask,
                     uint32_t transition_mask, uint32_t* hist);

/* as og_pipeline; dur (may be NULL): n_segments u64 sums of the whole-second durations
 * int(round(t1 - t0)) of the reports the histogram counts */
uint64_t og_pipeline2(const og_graph* g, const og_batch* b, double threshold_sec, uint32_t report_mask,
                      uint32_t transition_mask, uint32_t* hist, uint64_t* dur);
/* build the in-edge index that the path-walk counters [15]/[16] need (once per graph) */
void og_prepare_path_counters(const og_graph* g);

/* Algorithmic work of the stages since the last reset (meili_oracle.c lists all 17):
 * [0] searches [1] settled nodes [2] scanned edges [3] label writes
 * [4] target label lookups [5] route writes [6] candidate items tested [7] states ... */
void og_reset_counters(void);
void og_get_counters(uint64_t* out8);

#ifdef __cplusplus
}
#endif
#endif
