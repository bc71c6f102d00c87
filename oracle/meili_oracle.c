/* ORACLE — test infrastructure only.  See meili_oracle.h for the contract and
 * the parity status (real meili: UNPINNED; report(): PINNED by golden vectors).
 *
 * Stages (DESIGN.md §3 is the written spec; each stage cites the meili step it
 * restates — meili is external to /root/reference):
 *   S0 states      MapMatcher::OfflineMatch interpolation rule
 *   S1 candidates  CandidateGridQuery::Query + EmissionCostModel
 *   S2 routes      TransitionCostModel / find_shortest_path (bounded label setting)
 *   S3 viterbi     ViterbiSearch + breakage (OfflineMatch)
 *   S4 paths       FindMatchResults / ConstructRoute
 *   S5 segments    TrafficSegmentMatcher interpolate_matches + form_segments
 *   S6 report      reference py/reporter_service.py:79-179
 *
 * Compile with -ffp-contract=off (see oracle/Makefile): every float/double
 * expression is written in the exact operation order the GPU kernels use.
 */
#include "meili_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define OG_NONE 0xffffffffu
#define OG_K 16
#define OG_ROUTE_INVALID 0xffffffffu
#define OG_KEY_INF 0xffffffffffffffffull
#define OG_INVALID_SEGMENT_ID 0x3fffffffffffull
#define OG_MAX_RADIUS 200.0f
#define OG_MAX_BOUND_CM 100000000u
#define OG_FLAG_INTERNAL (1u << 19)

static const double MPD_LAT = 110567.0;
static const double MPD_LON_EQ = 111320.0;
static const double DEG2RAD = 0.017453292519943295;
static const double OG_PI = 3.141592653589793;
static const double RAD_EARTH_M = 6378160.187; /* Valhalla midgard kRadEarthMeters */
static const double QUEUE_SPEED_MPS = 2.7777777777777777; /* 10 km/h */

/* ---------------- deterministic math (identical op order on the GPU) ---------------- */
static double og_cos(double x) {
  const double z = x * x;
  double p = 1.0 / 2432902008176640000.0;
  p = p * z - 1.0 / 6402373705728000.0;
  p = p * z + 1.0 / 20922789888000.0;
  p = p * z - 1.0 / 87178291200.0;
  p = p * z + 1.0 / 479001600.0;
  p = p * z - 1.0 / 3628800.0;
  p = p * z + 1.0 / 40320.0;
  p = p * z - 1.0 / 720.0;
  p = p * z + 1.0 / 24.0;
  p = p * z - 0.5;
  p = p * z + 1.0;
  return p;
}
/* sin(x), |x| <= pi/2: odd Taylor series to x^21 in Horner form (exact hex coefficients) */
static double og_sin(double x) {
  const double z = x * x;
  double p = 0x1.71b8ef6dcf572p-66;
  p = p * z + -0x1.2f49b46814157p-57;
  p = p * z + 0x1.952c77030ad4ap-49;
  p = p * z + -0x1.ae7f3e733b81fp-41;
  p = p * z + 0x1.6124613a86d09p-33;
  p = p * z + -0x1.ae64567f544e4p-26;
  p = p * z + 0x1.71de3a556c734p-19;
  p = p * z + -0x1.a01a01a01a01ap-13;
  p = p * z + 0x1.1111111111111p-7;
  p = p * z + -0x1.5555555555555p-3;
  p = p * z + 0x1.0000000000000p+0;
  return x * p;
}

// cos(x) for |x| <= 2 pi (differences of longitudes), reduced onto det_cos's range.
static double og_cos_wide(double x) {
  double a = x < 0.0 ? -x : x;
  if (a > OG_PI) a = 2.0 * OG_PI - a;
  if (a > 0.5 * OG_PI) return -og_cos(OG_PI - a);
  return og_cos(a);
}

// asin(y) for |y| <= 1/2: Taylor series to y^55 (coefficients (2n)!/(4^n n!^2 (2n+1)) as exact
// hex literals), Horner in y^2.
static double og_asin_half(double y) {
  const double z = y * y;
  double p = 0x1.018f963c229bfp-9;
  p = p * z + 0x1.1052bc5fa960ap-9;
  p = p * z + 0x1.208d3570ae5a6p-9;
  p = p * z + 0x1.3275586c5f2f0p-9;
  p = p * z + 0x1.464c0950f7d47p-9;
  p = p * z + 0x1.5c5f56efaaaabp-9;
  p = p * z + 0x1.750de64d7d05fp-9;
  p = p * z + 0x1.90cb77f60c7cep-9;
  p = p * z + 0x1.b026f57b13b14p-9;
  p = p * z + 0x1.d3d2a8e0dd67dp-9;
  p = p * z + 0x1.fcaf8fb6db6dbp-9;
  p = p * z + 0x1.15ee9d45d1746p-8;
  p = p * z + 0x1.31683bdef7bdfp-8;
  p = p * z + 0x1.51ba308d3dcb1p-8;
  p = p * z + 0x1.782dda12f684cp-8;
  p = p * z + 0x1.a6863d70a3d71p-8;
  p = p * z + 0x1.df3bd37a6f4dfp-8;
  p = p * z + 0x1.12ef3cf3cf3cfp-7;
  p = p * z + 0x1.3fde50d79435ep-7;
  p = p * z + 0x1.7a87878787878p-7;
  p = p * z + 0x1.c99999999999ap-7;
  p = p * z + 0x1.1c4ec4ec4ec4fp-6;
  p = p * z + 0x1.6e8ba2e8ba2e9p-6;
  p = p * z + 0x1.f1c71c71c71c7p-6;
  p = p * z + 0x1.6db6db6db6db7p-5;
  p = p * z + 0x1.3333333333333p-4;
  p = p * z + 0x1.5555555555555p-3;
  p = p * z + 0x1.0000000000000p+0;
  return y * p;
}

// acos(c) for -1 < c < 1 from det_asin_half: 2 asin(sqrt((1-c)/2)) near 1, pi/2 - asin(c) in the
// middle, pi - 2 asin(sqrt((1+c)/2)) near -1 (IEEE sqrt: correctly rounded on both sides).
static double og_acos(double c) {
  if (c > 0.5) return 2.0 * og_asin_half(sqrt((1.0 - c) * 0.5));
  if (c < -0.5) return OG_PI - 2.0 * og_asin_half(sqrt((1.0 + c) * 0.5));
  return 0.5 * OG_PI - og_asin_half(c);
}
static float og_mlon(float lat) { return (float)(MPD_LON_EQ * og_cos((double)lat * DEG2RAD)); }

static float f32_of(uint32_t bits);
/* ---------------- turn costs (DESIGN.md §3 rule 3b; meili TransitionCostModel's turn term) ----------------
 * meili adds turn_penalty_factor * exp(-degree / 45) per turn of a transition's route (degree 0 = a
 * U-turn, 180 = straight on) to |route - gc| before dividing by beta.  Restated in integers: a turn
 * of `d` degrees weighs og_tu[d] = round(65536 exp(-d/45)), a route's turns sum to an integer U, and
 * the transition's turn cost is U * factor / 65536 metres. */
/* atan(t), 0 <= t <= 1: atan(t) = pi/4 + atan((t-1)/(t+1)) above tan(pi/8), then the odd Taylor
 * series to z^45 in Horner form in z^2 (coefficients (-1)^n/(2n+1)) */
static double og_atan_unit(double t) {
  double off = 0.0, z = t;
  if (t > 0.41421356237309503) { z = (t - 1.0) / (t + 1.0); off = 0.25 * OG_PI; }
  const double s = z * z;
  double p = 1.0 / 45.0;
  for (int n = 21; n >= 0; --n) p = p * s + ((n & 1) ? -1.0 : 1.0) / (double)(2 * n + 1);
  return off + z * p;
}
/* compass bearing in degrees [0, 360] of (dx east, dy north) */
static double og_bearing_deg(double dx, double dy) {
  const double ax = fabs(dx), ay = fabs(dy);
  if (ax == 0.0 && ay == 0.0) return 0.0;
  const double a = ax <= ay ? og_atan_unit(ax / ay) : 0.5 * OG_PI - og_atan_unit(ay / ax);
  double th;
  if (dx >= 0.0) th = dy >= 0.0 ? a : OG_PI - a;
  else th = dy < 0.0 ? OG_PI + a : 2.0 * OG_PI - a;
  return th * (180.0 / OG_PI);
}
/* ---- headings: Valhalla's NodeInfo edge headings (mjolnir graph builder: round(PointLL::
 * HeadingAlongPolyline(shape, kMetersOffsetForHeading = 30 m)), 8-bit storage round(h * 255/359),
 * read back as round(h8 * 359/255)).  External (Valhalla 2.x, absent here) and restated from its
 * published behaviour; DESIGN.md rule 3b.  PointLL::Heading is the initial great-circle bearing. */
static double og_gc(float lon_a, float lat_a, float lon_b, float lat_b);
static double og_initial_bearing(float lon_a, float lat_a, float lon_b, float lat_b) {
  if (lon_a == lon_b && lat_a == lat_b) return 0.0;
  const double p1 = (double)lat_a * DEG2RAD, p2 = (double)lat_b * DEG2RAD;
  const double dl = ((double)lon_b - (double)lon_a) * DEG2RAD;
  const double east = og_sin(dl) * og_cos(p2);
  const double north = og_cos(p1) * og_sin(p2) - og_sin(p1) * og_cos(p2) * og_cos_wide(dl);
  return og_bearing_deg(east, north);
}
/* HeadingAlongPolyline over n >= 2 shape points xs/ys (start node first) */
static double og_heading_along(const float* xs, const float* ys, uint32_t n) {
  if (n == 2) return og_initial_bearing(xs[0], ys[0], xs[1], ys[1]);
  double d = 0.0;
  for (uint32_t i = 0; i + 1 < n && d < 30.0; ++i) {
    const double seg = og_gc(xs[i], ys[i], xs[i + 1], ys[i + 1]);
    if (d + seg > 30.0) {
      const double f = (30.0 - d) / seg;
      const float x = (float)((double)xs[i] + ((double)xs[i + 1] - (double)xs[i]) * f);
      const float y = (float)((double)ys[i] + ((double)ys[i + 1] - (double)ys[i]) * f);
      return og_initial_bearing(xs[0], ys[0], x, y);
    }
    d += seg;
  }
  return og_initial_bearing(xs[0], ys[0], xs[n - 1], ys[n - 1]);
}
static uint32_t og_node_heading(double h) {
  const uint32_t hd = (uint32_t)floor(h + 0.5) % 360u;
  const uint32_t h8 = (uint32_t)floorf((float)hd * (255.0f / 359.0f) + 0.5f);
  return (uint32_t)floorf((float)h8 * (359.0f / 255.0f) + 0.5f);
}
/* per road: the heading of its forward edge at node0 (H0) and of its reverse edge at node1 (H1) */
static void og_road_headings(const og_graph* g, uint16_t* H0, uint16_t* H1) {
  uint32_t cap = 0;
  float *xs = NULL, *ys = NULL;
  for (uint32_t r = 0; r < g->n_roads; ++r) {
    const uint32_t a = g->road_vert_off[r], n = g->road_vert_off[r + 1] - a;
    if (n > cap) {
      cap = n * 2;
      xs = (float*)realloc(xs, cap * sizeof(float));
      ys = (float*)realloc(ys, cap * sizeof(float));
    }
    const uint32_t* V = g->verts;
    for (uint32_t i = 0; i < n; ++i) { xs[i] = f32_of(V[4 * (a + i)]); ys[i] = f32_of(V[4 * (a + i) + 1]); }
    H0[r] = (uint16_t)og_node_heading(og_heading_along(xs, ys, n));
    for (uint32_t i = 0; i < n; ++i) { xs[i] = f32_of(V[4 * (a + n - 1 - i)]); ys[i] = f32_of(V[4 * (a + n - 1 - i) + 1]); }
    H1[r] = (uint16_t)og_node_heading(og_heading_along(xs, ys, n));
  }
  free(xs);
  free(ys);
}
static uint32_t og_tu[181];
static void og_turn_table(void) {
  for (int d = 0; d <= 180; ++d) og_tu[d] = (uint32_t)lround(65536.0 * exp(-(double)d / 45.0));
}
/* turn between an edge arriving with back heading hb (at the node, toward where it came from) and
 * an edge leaving with heading hs */
static uint32_t og_turn(uint32_t hb, uint32_t hs) {
  uint32_t d = hb > hs ? hb - hs : hs - hb;
  if (d > 180u) d = 360u - d;
  return og_tu[d];
}
/* measurement distance: Valhalla PointLL::Distance (meili GreatCircleDistance), spherical law of
   cosines on the float coordinates, radius RAD_EARTH_M, rounded to float */
static double og_gc(float lon_a, float lat_a, float lon_b, float lat_b) {
  if (lon_a == lon_b && lat_a == lat_b) return 0.0;
  const double a = (double)lat_a * DEG2RAD, c = (double)lat_b * DEG2RAD;
  const double dl = ((double)lon_b - (double)lon_a) * DEG2RAD;
  const double cosb = og_sin(a) * og_sin(c) + og_cos(a) * og_cos(c) * og_cos_wide(dl);
  if (cosb >= 1.0) return 0.0;
  if (cosb <= -1.0) return (double)(float)(OG_PI * RAD_EARTH_M);
  return (double)(float)(og_acos(cosb) * RAD_EARTH_M);
}
static float f32_of(uint32_t bits) { float f; memcpy(&f, &bits, 4); return f; }

/* ---------------- graph helpers ---------------- */
static uint32_t e_target(const og_graph* g, uint32_t e) { return g->edges[4 * (size_t)e]; }
static uint32_t e_len(const og_graph* g, uint32_t e) { return g->edges[4 * (size_t)e + 1]; }
static uint32_t e_info(const og_graph* g, uint32_t e) { return g->edges[4 * (size_t)e + 2]; }
static uint32_t mode_access(int mode) { return mode == 3 ? 2u : (mode == 4 ? 4u : 1u); }
static uint32_t mode_speed(int mode, uint32_t edge_dkph) {
  uint32_t cap = 0xffffu;
  if (mode == 3) cap = 180; else if (mode == 4) cap = 51; else if (mode == 2) cap = 450;
  return edge_dkph < cap ? edge_dkph : cap;
}
static uint32_t t_ms(uint32_t d_cm, uint32_t dkph) {
  return (uint32_t)(((uint64_t)d_cm * 360ull) / (uint64_t)(dkph ? dkph : 1u));
}
static int e_ok(const og_graph* g, uint32_t e, uint32_t acc) {
  return e != OG_NONE && (((e_info(g, e) >> 16) & 7u) & acc) != 0;
}
static uint32_t e_speed(const og_graph* g, uint32_t e, int mode) { return mode_speed(mode, e_info(g, e) & 0xffffu); }
static uint64_t mk(uint32_t d, uint32_t t) { return ((uint64_t)d << 32) | t; }

/* ---------------- algorithmic work counters (rooflines of K1..K4) ----------------
 * [0] searches [1] settled nodes [2] scanned edges [3] label writes
 * [4] target label lookups [5] route writes [6] candidate items tested [7] states
 * [8] route-ball rows a table formulation of K2 reads: per (source, target with a usable
 *     direction), one per usable exit of the source [9] candidate descriptors read by K2
 *     (KA sources + KB targets per layer pair) [10] candidates kept (sum of K over states)
 * [11] grid rows visited by the candidate search (one item range per row) [12] chained
 * transitions (a path is built) [13] path edges [14] segments formed
 * [15] in-edge records the path walk reads (per walked node the canonical predecessor's record,
 *      located by the index stored in the route-ball rows; when that index is 7 or more, the
 *      node's in-edges in edge-id order up to it) [16] route-ball rows the path stage reads, one
 *      per usable exit: the target road's once per chained transition, the predecessor road's
 *      per walked node, and each usable in-edge's on a scan (counted only after
 *      og_prepare_path_counters)
 * [17] [18] [19] settled nodes, scanned edges and label writes of the same K2 searches stopped at
 *      their targets (engine.hip SearchTargets): label-setting order settles nodes by key, and a
 *      search that stops once every target's route key is below the next key settles exactly the
 *      nodes with keys <= the largest target route key (all of them when a target is unreached)
 * [20] transitions whose turn weight a turn row gives when turn_penalty_factor > 0 (a valid route
 *      entering its target road from a node: one 8 B turn row each in the table formulation);
 *      counted at any factor (the routes do not depend on it)
 * [21] nodes those routes turn at (the canonical-path walk of the search formulation) */
#define OG_NCNT 22
static uint64_t og_cnt[OG_NCNT];
static uint32_t og_roots;   /* usable exits of the last search_from */
static int og_counting = 0;
void og_reset_counters(void) { memset(og_cnt, 0, sizeof og_cnt); }
void og_get_counters(uint64_t* out) { memcpy(out, og_cnt, sizeof og_cnt); }

/* in-edge index of one graph for counters [15]/[16] (in-edges of a node in edge-id order, the
 * order the GPU path walk visits them); built outside any timed region */
static const uint32_t* pc_node_off = NULL;
static uint32_t pc_nodes = 0;
static uint32_t* pc_in_off = NULL;
static uint32_t* pc_in_edge = NULL;

/* ---------------- result container ---------------- */
struct og_result {
  uint64_t P, T, n_trans, n_path, n_seg;
  uint32_t* n_states; uint32_t* state_orig;
  uint8_t* cand_n; uint32_t* cand_road; uint32_t* cand_s; float* cand_sq;
  uint32_t* trans_off; double* gc; uint32_t* route; uint32_t* route_turn; double* route_d;
  int8_t* choice; uint8_t* chain_start;
  uint32_t* path_off; uint32_t* path_cnt; uint32_t* path_edges; uint32_t* route_dist;
  uint32_t* seg_off; og_segment* segs;
};

/* ---------------- bounded search workspace ---------------- */
typedef struct { uint64_t key; uint32_t node; } hitem;
typedef struct {
  uint32_t n;            /* nodes */
  uint64_t* label;       /* per node */
  uint64_t* rootkey;     /* per node: init key when a root, else inf */
  uint32_t* stamp;       /* per node: generation of label */
  uint32_t gen;
  hitem* heap; uint32_t hn, hcap;
  uint32_t* touched; uint32_t nt, tcap;
  uint32_t* pred;        /* per node */
  /* per settle, in settle order (counting only): key, cumulative scanned edges, label writes */
  uint64_t* skey; uint64_t* sscan; uint64_t* swrite; uint32_t ns, scap;
} search_ws;

static int ws_init(search_ws* w, uint32_t n) {
  memset(w, 0, sizeof(*w));
  w->n = n;
  w->label = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
  w->rootkey = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
  w->stamp = (uint32_t*)calloc(n ? n : 1, sizeof(uint32_t));
  w->pred = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  w->hcap = 1024; w->heap = (hitem*)malloc(sizeof(hitem) * w->hcap);
  w->tcap = 1024; w->touched = (uint32_t*)malloc(sizeof(uint32_t) * w->tcap);
  w->scap = 1024;
  w->skey = (uint64_t*)malloc(sizeof(uint64_t) * w->scap);
  w->sscan = (uint64_t*)malloc(sizeof(uint64_t) * w->scap);
  w->swrite = (uint64_t*)malloc(sizeof(uint64_t) * w->scap);
  return w->label && w->rootkey && w->stamp && w->pred && w->heap && w->touched && w->skey && w->sscan && w->swrite;
}
static void ws_free(search_ws* w) {
  free(w->label); free(w->rootkey); free(w->stamp); free(w->pred); free(w->heap); free(w->touched);
  free(w->skey); free(w->sscan); free(w->swrite);
}
static uint64_t ws_get(const search_ws* w, uint32_t v) { return w->stamp[v] == w->gen ? w->label[v] : OG_KEY_INF; }
static void ws_touch(search_ws* w, uint32_t v) {
  if (w->stamp[v] != w->gen) {
    w->stamp[v] = w->gen; w->label[v] = OG_KEY_INF; w->rootkey[v] = OG_KEY_INF; w->pred[v] = OG_NONE;
    if (w->nt == w->tcap) { w->tcap *= 2; w->touched = (uint32_t*)realloc(w->touched, sizeof(uint32_t) * w->tcap); }
    w->touched[w->nt++] = v;
  }
}
static void heap_push(search_ws* w, uint64_t key, uint32_t node) {
  if (w->hn == w->hcap) { w->hcap *= 2; w->heap = (hitem*)realloc(w->heap, sizeof(hitem) * w->hcap); }
  uint32_t i = w->hn++;
  while (i) {
    uint32_t p = (i - 1) / 2;
    if (w->heap[p].key <= key) break;
    w->heap[i] = w->heap[p]; i = p;
  }
  w->heap[i].key = key; w->heap[i].node = node;
}
static hitem heap_pop(search_ws* w) {
  hitem top = w->heap[0], last = w->heap[--w->hn];
  uint32_t i = 0;
  for (;;) {
    uint32_t c = 2 * i + 1;
    if (c >= w->hn) break;
    if (c + 1 < w->hn && w->heap[c + 1].key < w->heap[c].key) c++;
    if (w->heap[c].key >= last.key) break;
    w->heap[i] = w->heap[c]; i = c;
  }
  if (w->hn) w->heap[i] = last;
  return top;
}

/* Exact lexicographic (dist, time) shortest keys from the exits of candidate
 * (road, s) to every node whose distance is <= bound.  Label-setting
 * Dijkstra on a binary heap (meili uses a bucket queue; any exact method
 * yields the same keys since integer keys make the minimum unique). */
static void search_from(const og_graph* g, search_ws* w, uint32_t road, uint32_t s, int mode, uint32_t bound) {
  const uint32_t acc = mode_access(mode);
  w->gen++; w->nt = 0; w->hn = 0; w->ns = 0;
  if (w->gen == 0) { memset(w->stamp, 0, sizeof(uint32_t) * w->n); w->gen = 1; }
  const uint32_t L = g->road_len_cm[road];
  const uint32_t ef = g->road_fwd[road], er = g->road_rev[road];
  og_roots = (uint32_t)(e_ok(g, ef, acc) && L - s <= bound) + (uint32_t)(e_ok(g, er, acc) && s <= bound);
  if (e_ok(g, ef, acc) && L - s <= bound) {          /* exit forward to node1 */
    const uint32_t v = g->road_node1[road];
    const uint64_t k = mk(L - s, t_ms(L - s, e_speed(g, ef, mode)));
    ws_touch(w, v);
    w->rootkey[v] = k;
    if (k < w->label[v]) { w->label[v] = k; heap_push(w, k, v); }
  }
  if (e_ok(g, er, acc) && s <= bound) {              /* exit reverse to node0 */
    const uint32_t v = g->road_node0[road];
    const uint64_t k = mk(s, t_ms(s, e_speed(g, er, mode)));
    ws_touch(w, v);
    w->rootkey[v] = k;
    if (k < w->label[v]) { w->label[v] = k; heap_push(w, k, v); }
  }
  if (og_counting) og_cnt[0]++;
  while (w->hn) {
    hitem it = heap_pop(w);
    if (it.key != w->label[it.node]) continue;       /* stale */
    const uint32_t u = it.node;
    if (og_counting) { og_cnt[1]++; og_cnt[2] += g->node_off[u + 1] - g->node_off[u]; }
    uint64_t writes = 0;
    for (uint32_t e = g->node_off[u]; e < g->node_off[u + 1]; ++e) {
      if (!e_ok(g, e, acc)) continue;
      const uint32_t len = e_len(g, e);
      const uint64_t nk = it.key + mk(len, t_ms(len, e_speed(g, e, mode)));
      if ((uint32_t)(nk >> 32) > bound) continue;
      const uint32_t v = e_target(g, e);
      ws_touch(w, v);
      if (nk < w->label[v]) { w->label[v] = nk; heap_push(w, nk, v); if (og_counting) og_cnt[3]++; ++writes; }
    }
    if (og_counting) {
      if (w->ns == w->scap) {
        w->scap *= 2;
        w->skey = (uint64_t*)realloc(w->skey, sizeof(uint64_t) * w->scap);
        w->sscan = (uint64_t*)realloc(w->sscan, sizeof(uint64_t) * w->scap);
        w->swrite = (uint64_t*)realloc(w->swrite, sizeof(uint64_t) * w->scap);
      }
      const uint64_t ps = w->ns ? w->sscan[w->ns - 1] : 0, pw = w->ns ? w->swrite[w->ns - 1] : 0;
      w->skey[w->ns] = it.key;
      w->sscan[w->ns] = ps + (g->node_off[u + 1] - g->node_off[u]);
      w->swrite[w->ns] = pw + writes;
      w->ns++;
    }
  }
}

/* counters [17..19]: the prefix of the last search's settles with keys <= kmax */
static void count_to_targets(const search_ws* w, uint64_t kmax) {
  uint32_t lo = 0, hi = w->ns;   /* first settle with key > kmax (keys settle in order) */
  while (lo < hi) {
    const uint32_t mid = (lo + hi) / 2;
    if (w->skey[mid] <= kmax) lo = mid + 1; else hi = mid;
  }
  og_cnt[17] += lo;
  if (lo) { og_cnt[18] += w->sscan[lo - 1]; og_cnt[19] += w->swrite[lo - 1]; }
}

/* canonical predecessor: a root keeps its init key; otherwise the smallest
 * directed edge id among the tight in-edges from labelled nodes. */
static void canonical_preds(const og_graph* g, search_ws* w, int mode) {
  const uint32_t acc = mode_access(mode);
  for (uint32_t i = 0; i < w->nt; ++i) w->pred[w->touched[i]] = OG_NONE;
  for (uint32_t i = 0; i < w->nt; ++i) {
    const uint32_t u = w->touched[i];
    const uint64_t ku = w->label[u];
    if (ku == OG_KEY_INF) continue;
    for (uint32_t e = g->node_off[u]; e < g->node_off[u + 1]; ++e) {
      if (!e_ok(g, e, acc)) continue;
      const uint32_t v = e_target(g, e);
      if (w->stamp[v] != w->gen) continue;
      const uint64_t kv = w->label[v];
      if (kv == OG_KEY_INF || kv == w->rootkey[v]) continue;
      const uint32_t len = e_len(g, e);
      if (ku + mk(len, t_ms(len, e_speed(g, e, mode))) == kv && e < w->pred[v]) w->pred[v] = e;
    }
  }
}

/* source node of directed edge e: binary search in the CSR */
static uint32_t og_edge_src(const og_graph* g, uint32_t e) {
  uint32_t lo = 0, hi = g->n_nodes;
  while (hi - lo > 1) { const uint32_t mid = (lo + hi) / 2; if (g->node_off[mid] <= e) lo = mid; else hi = mid; }
  return lo;
}

/* Turn weight U of the route from a searched source on road ra to a target entered by combination
 * combo (2: road rb forward from its node0, 3: rb reverse from its node1): the route's canonical
 * path (canonical_preds must have run) walked back from the entry node; every node on it is a
 * turn, from the edge that arrives to the edge that leaves, the exit node's arriving edge being
 * the source road in its exit direction (as the path stage's exit edge: forward when the node is
 * ra's node1).  Direct combinations turn nowhere: U = 0. */
static uint32_t og_turn_walk(const og_graph* g, const search_ws* w, const uint16_t* H0, const uint16_t* H1,
                             uint32_t ra, uint32_t rb, int combo) {
  if (combo < 2) return 0u;
  uint32_t hs = combo == 2 ? H0[rb] : H1[rb];   /* heading of the entry edge where it leaves the node */
  uint32_t v = combo == 2 ? g->road_node0[rb] : g->road_node1[rb];
  uint32_t U = 0;
  while (w->label[v] != w->rootkey[v]) {
    const uint32_t e = w->pred[v];
    const uint32_t rr = g->edges[4 * (size_t)e + 3] >> 1, rev = g->edges[4 * (size_t)e + 3] & 1u;
    U += og_turn(rev ? H0[rr] : H1[rr], hs);     /* e arrives at v: its back heading there */
    hs = rev ? H1[rr] : H0[rr];                  /* e leaves its source */
    v = og_edge_src(g, e);
    og_cnt[21]++;
  }
  U += og_turn(v == g->road_node1[ra] ? H1[ra] : H0[ra], hs);
  og_cnt[21]++;
  return U;
}

typedef struct { uint32_t road, s, sq_bits; float sq; uint32_t v; } cand_t;

/* route key from a searched source to target candidate (road_b, s_b), plus the
 * winning combination: 0 direct-fwd, 1 direct-rev, 2 entry-fwd (via node0),
 * 3 entry-rev (via node1); ties keep the earliest combination in that order. */
static uint64_t route_to(const og_graph* g, const search_ws* w, uint32_t road_a, uint32_t s_a, uint32_t road_b,
                         uint32_t s_b, int mode, int* combo) {
  const uint32_t acc = mode_access(mode);
  const uint32_t ef = g->road_fwd[road_b], er = g->road_rev[road_b], L = g->road_len_cm[road_b];
  uint64_t best = OG_KEY_INF;
  int bc = -1;
  if (road_a == road_b) {
    if (e_ok(g, ef, acc) && s_b >= s_a) {
      const uint64_t k = mk(s_b - s_a, t_ms(s_b - s_a, e_speed(g, ef, mode)));
      if (k < best) { best = k; bc = 0; }
    }
    if (e_ok(g, er, acc) && s_a >= s_b) {
      const uint64_t k = mk(s_a - s_b, t_ms(s_a - s_b, e_speed(g, er, mode)));
      if (k < best) { best = k; bc = 1; }
    }
  }
  if (e_ok(g, ef, acc)) {
    const uint64_t lab = ws_get(w, g->road_node0[road_b]);
    if (lab != OG_KEY_INF) {
      const uint64_t k = lab + mk(s_b, t_ms(s_b, e_speed(g, ef, mode)));
      if (k < best) { best = k; bc = 2; }
    }
  }
  if (e_ok(g, er, acc)) {
    const uint64_t lab = ws_get(w, g->road_node1[road_b]);
    if (lab != OG_KEY_INF) {
      const uint64_t k = lab + mk(L - s_b, t_ms(L - s_b, e_speed(g, er, mode)));
      if (k < best) { best = k; bc = 3; }
    }
  }
  if (combo) *combo = bc;
  return best;
}

/* ---------------- S1: candidate search for one state point ---------------- */
static int cand_cmp_road(const void* a, const void* b) {
  const cand_t* x = (const cand_t*)a; const cand_t* y = (const cand_t*)b;
  if (x->road != y->road) return x->road < y->road ? -1 : 1;
  if (x->sq_bits != y->sq_bits) return x->sq_bits < y->sq_bits ? -1 : 1;
  return x->v < y->v ? -1 : (x->v > y->v);
}
static int cand_cmp_rank(const void* a, const void* b) {
  const cand_t* x = (const cand_t*)a; const cand_t* y = (const cand_t*)b;
  if (x->sq_bits != y->sq_bits) return x->sq_bits < y->sq_bits ? -1 : 1;
  return x->road < y->road ? -1 : (x->road > y->road);
}

static float point_radius(const og_options* o, float acc) {
  float r = o->search_radius;
  if (acc >= 0.0f && acc > r) r = acc;
  if (r > OG_MAX_RADIUS) r = OG_MAX_RADIUS;
  if (!(r > 0.0f)) r = 0.0f;
  return r;
}

static uint32_t find_candidates(const og_graph* g, float lon, float lat, float r, int mode, cand_t** buf,
                                uint32_t* cap, cand_t* out) {
  const uint32_t acc = mode_access(mode);
  const float mlon = og_mlon(lat);
  const float mlat = (float)MPD_LAT;
  const float r2 = r * r;
  const float pad = r * 1.01f + 0.5f;
  const float qlon = pad / mlon, qlat = pad / mlat;
  const double fx0 = floor(((double)(lon - qlon) - g->lon0) / g->dlon);
  const double fx1 = floor(((double)(lon + qlon) - g->lon0) / g->dlon);
  const double fy0 = floor(((double)(lat - qlat) - g->lat0) / g->dlat);
  const double fy1 = floor(((double)(lat + qlat) - g->lat0) / g->dlat);
  if (fx1 < 0 || fy1 < 0 || fx0 > (double)(g->ncx - 1) || fy0 > (double)(g->ncy - 1)) return 0;
  const uint32_t x0 = fx0 < 0 ? 0 : (uint32_t)fx0, y0 = fy0 < 0 ? 0 : (uint32_t)fy0;
  const uint32_t x1 = fx1 > (double)(g->ncx - 1) ? g->ncx - 1 : (uint32_t)fx1;
  const uint32_t y1 = fy1 > (double)(g->ncy - 1) ? g->ncy - 1 : (uint32_t)fy1;
  uint32_t n = 0;
  og_cnt[11] += y1 - y0 + 1;
  for (uint32_t cy = y0; cy <= y1; ++cy)
    for (uint32_t cx = x0; cx <= x1; ++cx) {
      const uint32_t c = cy * g->ncx + cx;
      for (uint32_t it = g->cell_off[c]; it < g->cell_off[c + 1]; ++it) {
        const uint32_t v = g->cell_item[it];
        const uint32_t* A = g->verts + 4 * (size_t)v;
        const uint32_t* B = A + 4;
        const uint32_t road = A[3];
        og_cnt[6]++;
        if (!e_ok(g, g->road_fwd[road], acc) && !e_ok(g, g->road_rev[road], acc)) continue;
        const float ax = (f32_of(A[0]) - lon) * mlon, ay = (f32_of(A[1]) - lat) * mlat;
        const float bx = (f32_of(B[0]) - lon) * mlon, by = (f32_of(B[1]) - lat) * mlat;
        const float dx = bx - ax, dy = by - ay;
        const float l2 = dx * dx + dy * dy;
        float t = 0.0f;
        if (l2 > 0.0f) {
          t = -(ax * dx + ay * dy) / l2;
          if (t < 0.0f) t = 0.0f;
          if (t > 1.0f) t = 1.0f;
        }
        const float cxp = ax + t * dx, cyp = ay + t * dy;
        const float sq = cxp * cxp + cyp * cyp;
        if (!(sq <= r2)) continue;
        const float along = (float)A[2] + t * (float)(B[2] - A[2]);
        uint32_t s = (uint32_t)rintf(along);
        if (s < A[2]) s = A[2];
        if (s > B[2]) s = B[2];
        if (n == *cap) { *cap *= 2; *buf = (cand_t*)realloc(*buf, sizeof(cand_t) * *cap); }
        cand_t* cd = &(*buf)[n++];
        cd->road = road; cd->s = s; cd->sq = sq; memcpy(&cd->sq_bits, &sq, 4); cd->v = v;
      }
    }
  if (!n) return 0;
  /* per road: keep min (sq, vertex) */
  qsort(*buf, n, sizeof(cand_t), cand_cmp_road);
  uint32_t m = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (i == 0 || (*buf)[i].road != (*buf)[i - 1].road) (*buf)[m++] = (*buf)[i];
  qsort(*buf, m, sizeof(cand_t), cand_cmp_rank);
  if (m > OG_K) m = OG_K;
  memcpy(out, *buf, sizeof(cand_t) * m);
  return m;
}

/* ---------------- S5 helpers: traversals and runs ---------------- */
typedef struct {
  uint32_t e, b, en;       /* directed edge, [b, en] cm along it */
  double tb, te;
  uint32_t sb, se;         /* state orig index at/before begin / end */
} trav_t;

typedef struct { trav_t* v; uint32_t n, cap; } trav_vec;
static void tv_push(trav_vec* tv, trav_t t) {
  if (tv->n == tv->cap) { tv->cap = tv->cap ? 2 * tv->cap : 64; tv->v = (trav_t*)realloc(tv->v, sizeof(trav_t) * tv->cap); }
  tv->v[tv->n++] = t;
}
typedef struct { og_segment* v; uint64_t n, cap; } seg_vec;
static void sv_push(seg_vec* sv, og_segment s) {
  if (sv->n == sv->cap) { sv->cap = sv->cap ? 2 * sv->cap : 1024; sv->v = (og_segment*)realloc(sv->v, sizeof(og_segment) * sv->cap); }
  sv->v[sv->n++] = s;
}

/* append a traversal, merging with the previous one when it continues the same
 * directed edge from the same offset (a state point passed straight through) */
static void add_trav(trav_vec* tv, trav_t t) {
  if (t.en == t.b) return;  /* zero-length pieces carry no information */
  if (tv->n) {
    trav_t* p = &tv->v[tv->n - 1];
    if (p->e == t.e && p->en == t.b) { p->en = t.en; p->te = t.te; p->se = t.se; return; }
  }
  tv_push(tv, t);
}

static double interp_time(double ta, double tb, uint64_t x, uint64_t D) {
  if (D == 0) return ta;
  return ta + (tb - ta) * ((double)x / (double)D);
}

static void form_runs(const og_graph* g, const trav_vec* tv, seg_vec* out) {
  uint32_t i = 0;
  while (i < tv->n) {
    const trav_t* f = &tv->v[i];
    const uint32_t sd = g->edge_seg[f->e];
    const int internal = (e_info(g, f->e) & OG_FLAG_INTERNAL) != 0;
    uint32_t j = i + 1;
    while (j < tv->n) {
      const trav_t* p = &tv->v[j - 1];
      const trav_t* c = &tv->v[j];
      const uint32_t sd2 = g->edge_seg[c->e];
      const int int2 = (e_info(g, c->e) & OG_FLAG_INTERNAL) != 0;
      if (sd2 != sd) break;
      if (sd == OG_NONE && int2 != internal) break;
      if (p->en != e_len(g, p->e) || c->b != 0) break;
      if (sd != OG_NONE && g->edge_seg_off[c->e] != g->edge_seg_off[p->e] + e_len(g, p->e)) break;
      ++j;
    }
    const trav_t* l = &tv->v[j - 1];
    og_segment s;
    memset(&s, 0, sizeof(s));
    const int start_ok = f->b == 0 && (sd == OG_NONE || g->edge_seg_off[f->e] == 0);
    const int end_ok = l->en == e_len(g, l->e) &&
                       (sd == OG_NONE || g->edge_seg_off[l->e] + e_len(g, l->e) == g->seg_len_cm[sd]);
    s.segment_id = sd == OG_NONE ? OG_INVALID_SEGMENT_ID : g->seg_id[sd];
    s.start_time = start_ok ? f->tb : -1.0;
    s.end_time = end_ok ? l->te : -1.0;
    if (sd != OG_NONE) {
      s.length = (start_ok && end_ok) ? (int32_t)((g->seg_len_cm[sd] + 50u) / 100u) : -1;
    } else {
      uint64_t tot = 0;
      for (uint32_t k = i; k < j; ++k) tot += tv->v[k].en - tv->v[k].b;
      s.length = (int32_t)((tot + 50u) / 100u);
    }
    uint64_t q = 0;
    for (uint32_t k = j; k-- > i;) {
      const trav_t* t = &tv->v[k];
      const double dt = t->te - t->tb;
      const uint32_t d = t->en - t->b;
      if (dt > 0.0 && ((double)d * 0.01) / dt < QUEUE_SPEED_MPS) q += d; else break;
    }
    s.queue_length = (int32_t)((q + 50u) / 100u);
    s.flags = (sd == OG_NONE && internal ? 1u : 0u) | (sd != OG_NONE ? 2u : 0u);
    s.begin_shape_index = f->sb;
    s.end_shape_index = l->se;
    s.seg_dense = sd;
    s.way_first = g->edge_way[f->e];
    s.way_last = s.way_first;
    for (uint32_t k = i + 1; k < j; ++k)
      if (g->edge_way[tv->v[k].e] != s.way_first) s.way_last = g->edge_way[tv->v[k].e];
    sv_push(out, s);
    i = j;
  }
}

/* ---------------- the matcher ---------------- */
og_result* og_match(const og_graph* g, const og_batch* b) {
  og_result* R = (og_result*)calloc(1, sizeof(og_result));
  if (!R) return NULL;
  const uint64_t T = b->n_traces, P = b->trace_off[T];
  R->P = P; R->T = T;
  R->n_states = (uint32_t*)calloc(T ? T : 1, 4);
  R->state_orig = (uint32_t*)calloc(P ? P : 1, 4);
  R->cand_n = (uint8_t*)calloc(P ? P : 1, 1);
  R->cand_road = (uint32_t*)calloc(P * OG_K + 1, 4);
  R->cand_s = (uint32_t*)calloc(P * OG_K + 1, 4);
  R->cand_sq = (float*)calloc(P * OG_K + 1, 4);
  R->trans_off = (uint32_t*)calloc(P ? P : 1, 4);
  R->gc = (double*)calloc(P ? P : 1, 8);
  R->choice = (int8_t*)malloc(P ? P : 1);
  R->chain_start = (uint8_t*)calloc(P ? P : 1, 1);
  R->path_off = (uint32_t*)calloc(P ? P : 1, 4);
  R->path_cnt = (uint32_t*)calloc(P ? P : 1, 4);
  R->route_dist = (uint32_t*)calloc(P ? P : 1, 4);
  R->seg_off = (uint32_t*)calloc(T + 1, 4);
  if (P) memset(R->choice, -1, P);

  search_ws ws;
  if (!ws_init(&ws, g->n_nodes)) { og_free(R); return NULL; }
  uint32_t cap = 256;
  cand_t* cbuf = (cand_t*)malloc(sizeof(cand_t) * cap);
  cand_t top[OG_K];

  /* S0 + S1 */
  for (uint64_t k = 0; k < T; ++k) {
    const uint32_t o = b->trace_off[k], n = b->trace_off[k + 1] - o;
    const og_options* op = &b->opts[b->trace_opt[k]];
    uint32_t ns = 0, last = 0;
    for (uint32_t i = 0; i < n; ++i) {
      if (i > 0) {
        const double d = og_gc(b->lon[o + last], b->lat[o + last], b->lon[o + i], b->lat[o + i]);
        if (d < (double)op->interpolation_distance) continue;
      }
      R->state_orig[o + ns++] = i;
      last = i;
    }
    R->n_states[k] = ns;
    og_cnt[7] += ns;
    for (uint32_t s = 0; s < ns; ++s) {
      const uint32_t p = o + R->state_orig[o + s];
      const float r = point_radius(op, b->accuracy[p]);
      const uint32_t m = find_candidates(g, b->lon[p], b->lat[p], r, op->mode, &cbuf, &cap, top);
      R->cand_n[o + s] = (uint8_t)m;
      og_cnt[10] += m;
      for (uint32_t j = 0; j < m; ++j) {
        R->cand_road[(o + s) * (uint64_t)OG_K + j] = top[j].road;
        R->cand_s[(o + s) * (uint64_t)OG_K + j] = top[j].s;
        R->cand_sq[(o + s) * (uint64_t)OG_K + j] = top[j].sq;
      }
    }
  }
  /* transition offsets (exclusive scan over layer slots, in slot order) */
  uint64_t nt = 0;
  for (uint64_t k = 0; k < T; ++k) {
    const uint32_t o = b->trace_off[k];
    for (uint32_t s = 1; s < R->n_states[k]; ++s) {
      R->trans_off[o + s] = (uint32_t)nt;
      nt += (uint64_t)R->cand_n[o + s - 1] * R->cand_n[o + s];
    }
  }
  R->n_trans = nt;
  R->route = (uint32_t*)malloc(sizeof(uint32_t) * (nt ? nt : 1));
  R->route_turn = (uint32_t*)calloc(nt ? nt : 1, sizeof(uint32_t));
  R->route_d = (double*)malloc(sizeof(double) * (nt ? nt : 1));
  uint16_t* H0 = (uint16_t*)malloc(sizeof(uint16_t) * (g->n_roads ? g->n_roads : 1));
  uint16_t* H1 = (uint16_t*)malloc(sizeof(uint16_t) * (g->n_roads ? g->n_roads : 1));
  og_road_headings(g, H0, H1);
  og_turn_table();

  /* S2 routes */
  for (uint64_t k = 0; k < T; ++k) {
    const uint32_t o = b->trace_off[k];
    const og_options* op = &b->opts[b->trace_opt[k]];
    const int turns = op->turn_penalty_factor > 0.0f;
    const double tscale = (double)op->turn_penalty_factor * 0x1p-16;   /* metres per unit of turn weight */
    for (uint32_t s = 1; s < R->n_states[k]; ++s) {
      const uint32_t la = o + s - 1, lb = o + s;
      const uint32_t pa = o + R->state_orig[la], pb = o + R->state_orig[lb];
      const double gc = og_gc(b->lon[pa], b->lat[pa], b->lon[pb], b->lat[pb]);
      R->gc[lb] = gc;
      const uint32_t KA = R->cand_n[la], KB = R->cand_n[lb];
      if (!KA || !KB) continue;
      double maxd = gc * (double)op->max_route_distance_factor;
      if ((double)op->breakage_distance < maxd) maxd = (double)op->breakage_distance;
      double bcm = floor(maxd * 100.0);
      if (!(bcm >= 0.0)) bcm = 0.0;
      const uint32_t bound = bcm > (double)OG_MAX_BOUND_CM ? OG_MAX_BOUND_CM : (uint32_t)bcm;
      const double dt = b->time[pb] - b->time[pa];
      uint32_t tmax = 0xffffffffu;
      if (dt > 0.0) {
        const double tm = floor(dt * (double)op->max_route_time_factor * 1000.0);
        tmax = tm >= 4294967295.0 ? 0xffffffffu : (uint32_t)tm;
      }
      og_cnt[4] += 2ull * KA * KB;
      og_cnt[5] += (uint64_t)KA * KB;
      og_cnt[9] += (uint64_t)KA + KB;
      og_counting = 1;
      for (uint32_t i = 0; i < KA; ++i) {
        const uint32_t ra = R->cand_road[la * (uint64_t)OG_K + i], sa = R->cand_s[la * (uint64_t)OG_K + i];
        search_from(g, &ws, ra, sa, op->mode, bound);
        uint64_t kmax = 0;
        int preds = 0;
        for (uint32_t j = 0; j < KB; ++j) {
          const uint32_t rb = R->cand_road[lb * (uint64_t)OG_K + j], sb = R->cand_s[lb * (uint64_t)OG_K + j];
          if (e_ok(g, g->road_fwd[rb], mode_access(op->mode)) || e_ok(g, g->road_rev[rb], mode_access(op->mode)))
            og_cnt[8] += og_roots;
          int combo = -1;
          const uint64_t key = route_to(g, &ws, ra, sa, rb, sb, op->mode, &combo);
          if (key > kmax) kmax = key;
          uint32_t out = OG_ROUTE_INVALID;
          if (key != OG_KEY_INF && (uint32_t)(key >> 32) <= bound && (uint32_t)key <= tmax) out = (uint32_t)(key >> 32);
          R->route[R->trans_off[lb] + i * KB + j] = out;
          if (out != OG_ROUTE_INVALID && combo >= 2) og_cnt[20]++;   /* factor-independent: counted always */
          if (turns && out != OG_ROUTE_INVALID && combo >= 2) {
            if (!preds) { canonical_preds(g, &ws, op->mode); preds = 1; }
            R->route_turn[R->trans_off[lb] + i * KB + j] = og_turn_walk(g, &ws, H0, H1, ra, rb, combo);
          }
          /* the transition's distance term (rule 3b): turn_m + |route_m - gc|, turn_m = U * factor /
           * 65536 (+0 without turn costs, and +0 + x == x); +inf for an invalid route */
          R->route_d[R->trans_off[lb] + i * KB + j] =
              out == OG_ROUTE_INVALID ? INFINITY
                                      : (double)R->route_turn[R->trans_off[lb] + i * KB + j] * tscale +
                                            fabs((double)out * 0.01 - gc);
        }
        count_to_targets(&ws, kmax);
      }
    }
  }

  og_counting = 0;
  /* S3 viterbi */
  double* cost = (double*)malloc(sizeof(double) * (P * OG_K + 1));
  uint8_t* bp = (uint8_t*)malloc(P * OG_K + 1);
  for (uint64_t k = 0; k < T; ++k) {
    const uint32_t o = b->trace_off[k], S = R->n_states[k];
    const og_options* op = &b->opts[b->trace_opt[k]];
    const double inv2s2 = 1.0 / (2.0 * (double)op->sigma_z * (double)op->sigma_z);
    const double inv_beta = 1.0 / (double)op->beta;
    int prev_ok = 0;
    for (uint32_t s = 0; s < S; ++s) {
      const uint32_t l = o + s, KB = R->cand_n[l];
      if (!KB) { R->chain_start[l] = 1; prev_ok = 0; continue; }
      int start = !prev_ok || (s > 0 && R->gc[l] > (double)op->breakage_distance);
      const uint32_t KA = s > 0 ? R->cand_n[l - 1] : 0;
      if (!start) {
        int any = 0;
        for (uint32_t j = 0; j < KB; ++j) {
          double best = INFINITY; int arg = -1;
          for (uint32_t i = 0; i < KA; ++i) {
            const double ci = cost[(l - 1) * (uint64_t)OG_K + i];
            const uint32_t rc = R->route[R->trans_off[l] + i * KB + j];
            if (ci == INFINITY || rc == OG_ROUTE_INVALID) continue;
            /* one fused multiply-add: cost_i + (turn_m + |route_m - gc|) / beta, rounded once (the
             * distance term formed with the route in S2) */
            const double c = fma(R->route_d[R->trans_off[l] + i * KB + j], inv_beta, ci);
            if (c < best) { best = c; arg = (int)i; }
          }
          const double em = (double)R->cand_sq[l * (uint64_t)OG_K + j] * inv2s2;
          cost[l * (uint64_t)OG_K + j] = arg >= 0 ? best + em : INFINITY;
          bp[l * (uint64_t)OG_K + j] = arg >= 0 ? (uint8_t)arg : 255;
          any |= arg >= 0;
        }
        if (!any) start = 1;
      }
      if (start) {
        R->chain_start[l] = 1;
        for (uint32_t j = 0; j < KB; ++j) {
          cost[l * (uint64_t)OG_K + j] = (double)R->cand_sq[l * (uint64_t)OG_K + j] * inv2s2;
          bp[l * (uint64_t)OG_K + j] = 255;
        }
      }
      prev_ok = 1;
    }
    /* backtrace every chain: a chain ends at s when the next layer starts one */
    for (uint32_t s = S; s-- > 0;) {
      const uint32_t l = o + s, KB = R->cand_n[l];
      if (!KB) continue;
      const int is_end = (s + 1 == S) || R->chain_start[l + 1];
      if (!is_end) continue;
      int w = 0;
      for (uint32_t j = 1; j < KB; ++j)
        if (cost[l * (uint64_t)OG_K + j] < cost[l * (uint64_t)OG_K + w]) w = (int)j;
      uint32_t t = s;
      for (;;) {
        R->choice[o + t] = (int8_t)w;
        if (R->chain_start[o + t]) break;
        w = bp[(o + t) * (uint64_t)OG_K + w];
        --t;
      }
    }
  }
  free(cost); free(bp);

  /* S4 paths + S5 segments */
  uint64_t pcap = 1024, pn = 0;
  uint32_t* pool = (uint32_t*)malloc(sizeof(uint32_t) * pcap);
  seg_vec sv = {0, 0, 0};
  trav_vec tv = {0, 0, 0};
  uint32_t* stack = (uint32_t*)malloc(sizeof(uint32_t) * 1024);
  uint32_t scap = 1024;
  for (uint64_t k = 0; k < T; ++k) {
    const uint32_t o = b->trace_off[k], S = R->n_states[k];
    const og_options* op = &b->opts[b->trace_opt[k]];
    const uint32_t acc = mode_access(op->mode);
    R->seg_off[k] = (uint32_t)sv.n;
    tv.n = 0;
    for (uint32_t s = 0; s < S; ++s) {
      const uint32_t l = o + s;
      if (R->chain_start[l] || R->choice[l] < 0) {  /* chain boundary: flush runs */
        form_runs(g, &tv, &sv); tv.n = 0;
        continue;
      }
      const uint32_t la = l - 1;
      const uint32_t i = (uint32_t)R->choice[la], j = (uint32_t)R->choice[l];
      const uint32_t ra = R->cand_road[la * (uint64_t)OG_K + i], sa = R->cand_s[la * (uint64_t)OG_K + i];
      const uint32_t rb = R->cand_road[l * (uint64_t)OG_K + j], sb = R->cand_s[l * (uint64_t)OG_K + j];
      const uint32_t pa = o + R->state_orig[la], pbt = o + R->state_orig[l];
      double maxd = R->gc[l] * (double)op->max_route_distance_factor;
      if ((double)op->breakage_distance < maxd) maxd = (double)op->breakage_distance;
      double bcm = floor(maxd * 100.0);
      if (!(bcm >= 0.0)) bcm = 0.0;
      const uint32_t bound = bcm > (double)OG_MAX_BOUND_CM ? OG_MAX_BOUND_CM : (uint32_t)bcm;
      search_from(g, &ws, ra, sa, op->mode, bound);
      int combo = -1;
      const uint64_t key = route_to(g, &ws, ra, sa, rb, sb, op->mode, &combo);
      const uint32_t D = (uint32_t)(key >> 32);
      R->route_dist[l] = D;
      /* directed edge sequence: exit edge, graph edges, entry edge */
      uint32_t ns = 0;
      const int pcount = pc_node_off == g->node_off && pc_nodes == g->n_nodes;
      if (pcount && (e_ok(g, g->road_fwd[rb], acc) || e_ok(g, g->road_rev[rb], acc)))
        og_cnt[16] += og_roots;   /* entry labels: the exits' rows of the target road, read once */
      if (combo <= 1) {
        stack[ns++] = combo == 0 ? g->road_fwd[ra] : g->road_rev[ra];
      } else {
        canonical_preds(g, &ws, op->mode);
        const uint32_t entry_e = combo == 2 ? g->road_fwd[rb] : g->road_rev[rb];
        uint32_t v = combo == 2 ? g->road_node0[rb] : g->road_node1[rb];
        stack[ns++] = entry_e;
        while (ws.label[v] != ws.rootkey[v]) {
          const uint32_t e = ws.pred[v];
          if (pcount) {
            /* the GPU walk (k_paths_ball) reads the canonical predecessor's in-edge record straight
             * from the index stored in the route-ball rows when it is below 7, else it scans the
             * in-edges in edge-id order up to it, probing both exits' rows of each usable one; then
             * the exits' rows of the predecessor's road give the next node's label */
            uint32_t idx = 0;
            while (pc_in_off[v] + idx < pc_in_off[v + 1] && pc_in_edge[pc_in_off[v] + idx] != e) ++idx;
            if (idx < 7) {
              og_cnt[15]++;
            } else {
              for (uint32_t q = pc_in_off[v]; q <= pc_in_off[v] + idx; ++q) {
                og_cnt[15]++;
                if (e_ok(g, pc_in_edge[q], acc)) og_cnt[16] += og_roots;
              }
            }
            og_cnt[16] += og_roots;
          }
          if (ns == scap) { scap *= 2; stack = (uint32_t*)realloc(stack, sizeof(uint32_t) * scap); }
          stack[ns++] = e;
          /* source node of e: binary search in CSR */
          uint32_t lo = 0, hi = g->n_nodes;
          while (hi - lo > 1) { const uint32_t mid = (lo + hi) / 2; if (g->node_off[mid] <= e) lo = mid; else hi = mid; }
          v = lo;
        }
        if (ns == scap) { scap *= 2; stack = (uint32_t*)realloc(stack, sizeof(uint32_t) * scap); }
        stack[ns++] = (v == g->road_node1[ra]) ? g->road_fwd[ra] : g->road_rev[ra];
        /* reverse into travel order */
        for (uint32_t x = 0; x < ns / 2; ++x) { const uint32_t t = stack[x]; stack[x] = stack[ns - 1 - x]; stack[ns - 1 - x] = t; }
      }
      R->path_off[l] = (uint32_t)pn;
      R->path_cnt[l] = ns;
      og_cnt[12]++;
      og_cnt[13] += ns;
      if (pn + ns > pcap) { while (pn + ns > pcap) pcap *= 2; pool = (uint32_t*)realloc(pool, sizeof(uint32_t) * pcap); }
      memcpy(pool + pn, stack, sizeof(uint32_t) * ns);
      pn += ns;
      /* traversals with distance-interpolated times */
      const double ta = b->time[pa], tb = b->time[pbt];
      const uint32_t oa = R->state_orig[la], ob = R->state_orig[l];
      uint64_t x = 0;
      for (uint32_t q = 0; q < ns; ++q) {
        const uint32_t e = stack[q];
        const uint32_t len = e_len(g, e);
        const int rev = (g->edges[4 * (size_t)e + 3] & 1u) != 0;
        const uint32_t L = len;
        uint32_t b0 = 0, b1 = L;
        if (q == 0) b0 = rev ? L - sa : sa;                 /* exit point in edge coords */
        if (q + 1 == ns) b1 = rev ? L - sb : sb;            /* entry point in edge coords */
        if (ns == 1 && combo <= 1) { b0 = rev ? L - sa : sa; b1 = rev ? L - sb : sb; }
        trav_t t;
        t.e = e; t.b = b0; t.en = b1;
        t.tb = interp_time(ta, tb, x, D);
        x += (uint64_t)(b1 - b0);
        t.te = interp_time(ta, tb, x, D);
        t.sb = oa;
        t.se = (q + 1 == ns) ? ob : oa;
        add_trav(&tv, t);
      }
      (void)acc;
    }
    form_runs(g, &tv, &sv);
  }
  R->seg_off[T] = (uint32_t)sv.n;
  og_cnt[14] += sv.n;
  R->path_edges = pool; R->n_path = pn;
  R->segs = sv.v; R->n_seg = sv.n;
  free(tv.v); free(stack); free(cbuf); free(H0); free(H1);
  ws_free(&ws);
  return R;
}

void og_free(og_result* r) {
  if (!r) return;
  free(r->n_states); free(r->state_orig); free(r->cand_n); free(r->cand_road); free(r->cand_s); free(r->cand_sq);
  free(r->trans_off); free(r->gc); free(r->route); free(r->route_turn); free(r->route_d); free(r->choice); free(r->chain_start);
  free(r->path_off); free(r->path_cnt); free(r->path_edges); free(r->route_dist); free(r->seg_off); free(r->segs);
  free(r);
}

void og_sizes(const og_result* r, uint64_t* n_points, uint64_t* n_trans, uint64_t* n_path_edges, uint64_t* n_segments) {
  *n_points = r->P; *n_trans = r->n_trans; *n_path_edges = r->n_path; *n_segments = r->n_seg;
}
void og_get_states(const og_result* r, uint32_t* n_states, uint32_t* state_orig) {
  memcpy(n_states, r->n_states, 4 * r->T); memcpy(state_orig, r->state_orig, 4 * r->P);
}
void og_get_candidates(const og_result* r, uint8_t* cand_n, uint32_t* road, uint32_t* s_cm, float* sq) {
  memcpy(cand_n, r->cand_n, r->P); memcpy(road, r->cand_road, 4 * r->P * OG_K);
  memcpy(s_cm, r->cand_s, 4 * r->P * OG_K); memcpy(sq, r->cand_sq, 4 * r->P * OG_K);
}
void og_get_routes(const og_result* r, uint32_t* trans_off, double* gc, uint32_t* route_cm) {
  memcpy(trans_off, r->trans_off, 4 * r->P); memcpy(gc, r->gc, 8 * r->P); memcpy(route_cm, r->route, 4 * r->n_trans);
}
void og_get_route_turns(const og_result* r, uint32_t* route_turn) { memcpy(route_turn, r->route_turn, 4 * r->n_trans); }
void og_get_route_terms(const og_result* r, double* route_d) { memcpy(route_d, r->route_d, 8 * r->n_trans); }
void og_road_heads(const og_graph* g, uint16_t* h0, uint16_t* h1) { og_road_headings(g, h0, h1); }
void og_get_viterbi(const og_result* r, int8_t* choice, uint8_t* chain_start) {
  memcpy(choice, r->choice, r->P); memcpy(chain_start, r->chain_start, r->P);
}
void og_get_paths(const og_result* r, uint32_t* path_off, uint32_t* path_cnt, uint32_t* path_edges, uint32_t* route_key_dist) {
  memcpy(path_off, r->path_off, 4 * r->P); memcpy(path_cnt, r->path_cnt, 4 * r->P);
  memcpy(path_edges, r->path_edges, 4 * r->n_path); memcpy(route_key_dist, r->route_dist, 4 * r->P);
}
void og_get_segments(const og_result* r, uint32_t* seg_off, og_segment* segs) {
  memcpy(seg_off, r->seg_off, 4 * (r->T + 1)); memcpy(segs, r->segs, sizeof(og_segment) * r->n_seg);
}

/* ---------------- S6: report() restatement ---------------- */
static int in_mask(uint32_t mask, int level) { return (mask >> (level + 1)) & 1u; }

int og_report_trace(const og_segment* segs, uint32_t n, double end_time, double threshold, uint32_t rmask,
                    uint32_t tmask, og_report* out, og_stats* st) {
  memset(st, 0, sizeof(*st));
  st->successful_length_m = -1; st->unreported_length_m = -1; st->shape_used = -1;
  int last = (int)n - 1;                                        /* :86-87 */
  while (last >= 0 && end_time - segs[last].start_time < threshold) --last;
  if (last >= 0 && segs[last].begin_shape_index != 0) st->shape_used = (int32_t)segs[last].begin_shape_index;
  int have_prior = 0, nrep = 0;
  uint64_t p_id = 0; double p_t0 = 0, p_t1 = 0; int32_t p_len = 0, p_q = 0; int p_lvl = -1; uint32_t p_dense = 0;
  int p_has_id = 0;
  for (int k = 0; k <= last; ++k) {
    const og_segment* s = &segs[k];
    const int has_id = (s->flags & 2u) != 0, internal = (s->flags & 1u) != 0;
    if (k != 0 && s->start_time == -1.0 && segs[k - 1].end_time == -1.0) st->discontinuities++;  /* :115-116 */
    const int lvl = has_id ? (int)(s->segment_id & 7u) : -1;                                     /* :119 */
    if (have_prior && p_has_id && p_len > 0 && !internal) {                                      /* :122 */
      if (p_lvl >= 0 && in_mask(rmask, p_lvl)) {
        const int to_next = in_mask(tmask, lvl);
        og_report r;
        r.id = p_id; r.t0 = p_t0; r.t1 = to_next ? s->start_time : p_t1;
        r.length = p_len; r.queue_length = p_q; r.seg_dense = p_dense; r.pad = 0;
        r.next_id = (to_next && has_id) ? s->segment_id : OG_INVALID_SEGMENT_ID;
        const double dt = r.t1 - r.t0;
        if (dt <= 0 || isinf(dt) || isnan(dt)) st->invalid_times++;
        else if (((double)p_len / dt) * 3.6 > 160.0) st->invalid_speeds++;
        else { out[nrep++] = r; st->successful_count++; st->successful_length_m = p_len; }
      } else {
        st->unreported_count++; st->unreported_length_m = p_len;
      }
    }
    if (!(internal && k != 0)) {                                                                  /* :145-154 */
      have_prior = 1; p_has_id = has_id; p_id = s->segment_id; p_t0 = s->start_time; p_t1 = s->end_time;
      p_len = s->length; p_q = s->queue_length; p_lvl = lvl; p_dense = s->seg_dense;
    }
    if (!has_id && !internal) st->unassociated++;                                                 /* :161-162 */
  }
  st->n_reports = nrep;
  return nrep;
}

void og_prepare_path_counters(const og_graph* g) {
  free(pc_in_off); free(pc_in_edge);
  pc_nodes = g->n_nodes;
  pc_in_off = (uint32_t*)calloc((size_t)g->n_nodes + 1, sizeof(uint32_t));
  pc_in_edge = (uint32_t*)malloc(sizeof(uint32_t) * (g->n_edges ? g->n_edges : 1));
  uint32_t* fill = (uint32_t*)malloc(sizeof(uint32_t) * (g->n_nodes ? g->n_nodes : 1));
  if (!pc_in_off || !pc_in_edge || !fill) { free(fill); pc_node_off = NULL; return; }
  for (uint32_t e = 0; e < g->n_edges; ++e) pc_in_off[e_target(g, e) + 1]++;
  for (uint32_t n = 0; n < g->n_nodes; ++n) pc_in_off[n + 1] += pc_in_off[n];
  memcpy(fill, pc_in_off, sizeof(uint32_t) * g->n_nodes);
  for (uint32_t e = 0; e < g->n_edges; ++e) pc_in_edge[fill[e_target(g, e)]++] = e;
  free(fill);
  pc_node_off = g->node_off;
}

uint64_t og_pipeline(const og_graph* g, const og_batch* b, double threshold, uint32_t rmask, uint32_t tmask,
                     uint32_t* hist) {
  return og_pipeline2(g, b, threshold, rmask, tmask, hist, NULL);
}

uint64_t og_pipeline2(const og_graph* g, const og_batch* b, double threshold, uint32_t rmask, uint32_t tmask,
                      uint32_t* hist, uint64_t* dur) {
  og_result* r = og_match(g, b);
  if (!r) return 0;
  uint64_t total = 0;
  og_report* rep = (og_report*)malloc(sizeof(og_report) * (r->n_seg + 1));
  for (uint64_t k = 0; k < r->T; ++k) {
    const uint32_t s0 = r->seg_off[k], s1 = r->seg_off[k + 1];
    const uint32_t o = b->trace_off[k], n = b->trace_off[k + 1] - o;
    og_stats st;
    if (!n) continue;
    const int m = og_report_trace(r->segs + s0, s1 - s0, b->time[o + n - 1], threshold, rmask, tmask, rep, &st);
    for (int q = 0; q < m; ++q) {
      const og_report* x = &rep[q];
      const double dt = x->t1 - x->t0;
      if (!(x->t0 > 0 && x->t1 > 0 && dt > 0.5 && x->length > 0 && x->queue_length >= 0)) continue;  /* simple_reporter.py:177 */
      if (hist && x->seg_dense != OG_NONE) {
        int bin = (int)(((double)x->length / dt) * 3.6 / 10.0);
        if (bin > 15) bin = 15;
        if (bin < 0) bin = 0;
        hist[(uint64_t)x->seg_dense * 16u + (uint32_t)bin] += 1u;
      }
      /* duration column of the tile row, int(round(t1 - t0)) (simple_reporter.py:179):
       * Python 2 round() is half away from zero, as C round() */
      if (dur && x->seg_dense != OG_NONE) dur[x->seg_dense] += (uint64_t)round(dt);
      total++;
    }
  }
  free(rep);
  og_free(r);
  return total;
}
