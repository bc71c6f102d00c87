// rm_common.hpp — constants, record layouts and deterministic math shared by
// the host runtime and the gfx950 kernels of the reporter map-matching engine.
//
// The matcher replaces valhalla.SegmentMatcher().Match (called at
// reference py/reporter_service.py:240 and py/simple_reporter.py:166).  Every
// numeric rule below is part of the engine's written specification
// (DESIGN.md §3); oracle/meili_oracle.c restates the same rules independently.
//
// Build rule: every translation unit is compiled with -ffp-contract=off and
// without fast-math, so fp32/fp64 results are bit-identical between the host
// oracle (gcc, SSE) and the device (hipcc, gfx950).
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIP__) || defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RM_HD __host__ __device__ __forceinline__
#else
#define RM_HD static inline
#endif

namespace rm {

// ---- id semantics (reference py/simple_reporter.py:37-49, Segment.java:16) ----
constexpr int kLevelBits = 3;
constexpr int kTileIndexBits = 22;
constexpr int kSegmentIndexBits = 21;
constexpr uint64_t kInvalidSegmentId = 0x3fffffffffffull;  // Segment.java:16
constexpr uint32_t kNone = 0xffffffffu;

// ---- distance approximation (Valhalla-2.x-style PointLL float geometry) ----
constexpr double kMetersPerDegLat = 110567.0;  // meters per degree latitude
constexpr double kMetersPerDegLonEq = 111320.0;  // meters per degree longitude at the equator
constexpr double kDegToRad = 0.017453292519943295;
constexpr double kPi = 3.141592653589793;
constexpr double kRadEarthMeters = 6378160.187;   // Valhalla midgard kRadEarthMeters

// cos(x) for |x| <= pi/2 by a fixed Horner polynomial in x^2 (Taylor to x^20).
// Pure IEEE add/mul in a fixed order: identical bits on host and device.
RM_HD double det_cos(double x) {
  const double z = x * x;
  double p = 1.0 / 2432902008176640000.0;   // 1/20!
  p = p * z - 1.0 / 6402373705728000.0;     // 1/18!
  p = p * z + 1.0 / 20922789888000.0;       // 1/16!
  p = p * z - 1.0 / 87178291200.0;          // 1/14!
  p = p * z + 1.0 / 479001600.0;            // 1/12!
  p = p * z - 1.0 / 3628800.0;              // 1/10!
  p = p * z + 1.0 / 40320.0;                // 1/8!
  p = p * z - 1.0 / 720.0;                  // 1/6!
  p = p * z + 1.0 / 24.0;                   // 1/4!
  p = p * z - 0.5;                          // 1/2!
  p = p * z + 1.0;
  return p;
}

// sin(x) for |x| <= pi/2: odd Taylor series to x^21, Horner in x^2 (coefficients as exact
// hex literals of (-1)^k/(2k+1)!); same contract as det_cos.
RM_HD double det_sin(double x) {
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
RM_HD double det_cos_wide(double x) {
  double a = x < 0.0 ? -x : x;
  if (a > kPi) a = 2.0 * kPi - a;
  if (a > 0.5 * kPi) return -det_cos(kPi - a);
  return det_cos(a);
}

// asin(y) for |y| <= 1/2: Taylor series to y^55 (coefficients (2n)!/(4^n n!^2 (2n+1)) as exact
// hex literals), Horner in y^2.
RM_HD double det_asin_half(double y) {
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
RM_HD double det_acos(double c) {
  if (c > 0.5) return 2.0 * det_asin_half(__builtin_sqrt((1.0 - c) * 0.5));
  if (c < -0.5) return kPi - 2.0 * det_asin_half(__builtin_sqrt((1.0 + c) * 0.5));
  return 0.5 * kPi - det_asin_half(c);
}

// meters per degree of longitude at latitude lat (degrees), as float.
RM_HD float meters_per_lon(float lat) {
  return (float)(kMetersPerDegLonEq * det_cos((double)lat * kDegToRad));
}

// Great-circle distance between two measurements, as Valhalla's PointLL::Distance (meili's
// GreatCircleDistance): spherical law of cosines on the float lon/lat, Earth radius
// kRadEarthMeters, the result rounded to float; deterministic sin/cos/acos so both sides agree.
// gc_trig takes sin/cos of both latitudes (lat_sin / lat_cos below), so kernels that measure a
// point against several others evaluate them once per point; same operations, same bits.
RM_HD double lat_sin(float lat) { return det_sin((double)lat * kDegToRad); }
RM_HD double lat_cos(float lat) { return det_cos((double)lat * kDegToRad); }
RM_HD double gc_trig(float lon_a, float lat_a, double sa, double ca, float lon_b, float lat_b, double sb, double cb) {
  if (lon_a == lon_b && lat_a == lat_b) return 0.0;
  const double dl = ((double)lon_b - (double)lon_a) * kDegToRad;
  const double cosb = sa * sb + ca * cb * det_cos_wide(dl);
  if (cosb >= 1.0) return 0.0;
  if (cosb <= -1.0) return (double)(float)(kPi * kRadEarthMeters);
  return (double)(float)(det_acos(cosb) * kRadEarthMeters);
}
RM_HD double gc_distance(float lon_a, float lat_a, float lon_b, float lat_b) {
  return gc_trig(lon_a, lat_a, lat_sin(lat_a), lat_cos(lat_a), lon_b, lat_b, lat_sin(lat_b), lat_cos(lat_b));
}

// ---- turn costs (meili TransitionCostModel's turn term; DESIGN.md §3 rule 3b) ----
// meili adds turn_penalty_factor * exp(-d / 45) for every turn of d degrees (0 = U-turn, 180 =
// straight on) of a transition's route to |route - gc| before dividing by beta.  Here a turn of d
// degrees weighs kTurnWeight(d) = round(65536 exp(-d/45)) (turn_weight_table), a route's turns sum
// to an integer U (associative: the route tables store partial sums), and the transition's turn
// cost is U * factor * 2^-16 metres.  Headings are Valhalla NodeInfo headings: 8-bit steps of
// 360/255 degrees, expanded back to whole degrees.
//
// atan(t), 0 <= t <= 1: atan(t) = pi/4 + atan((t-1)/(t+1)) above tan(pi/8), then the odd Taylor
// series to z^45, Horner in z^2 with coefficients (-1)^n/(2n+1) computed by one IEEE division each
RM_HD double det_atan_unit(double t) {
  double off = 0.0, z = t;
  if (t > 0.41421356237309503) { z = (t - 1.0) / (t + 1.0); off = 0.25 * kPi; }
  const double s = z * z;
  double p = 1.0 / 45.0;
  for (int n = 21; n >= 0; --n) p = p * s + ((n & 1) ? -1.0 : 1.0) / (double)(2 * n + 1);
  return off + z * p;
}
// compass bearing in degrees [0, 360] of (dx east, dy north), metres
RM_HD double det_bearing_deg(double dx, double dy) {
  const double ax = dx < 0.0 ? -dx : dx, ay = dy < 0.0 ? -dy : dy;
  if (ax == 0.0 && ay == 0.0) return 0.0;
  const double a = ax <= ay ? det_atan_unit(ax / ay) : 0.5 * kPi - det_atan_unit(ay / ax);
  double th;
  if (dx >= 0.0) th = dy >= 0.0 ? a : kPi - a;
  else th = dy < 0.0 ? kPi + a : 2.0 * kPi - a;
  return th * (180.0 / kPi);
}
// Round 6: an edge's heading at its start node as Valhalla's graph builder stores
// it in NodeInfo -- round(PointLL::HeadingAlongPolyline(shape, kMetersOffsetForHeading = 30 m)):
// the initial great-circle bearing from the node to the point 30 m along the edge's shape (the
// segment that passes 30 m, by PointLL::Distance, interpolated linearly in lon/lat), or to the
// shape's last point when the edge is shorter (two-point shapes: to the other end) -- kept in 8 bits
// (round(h * 255/359)) and expanded back to degrees (round(h8 * 359/255)).  Curved ways turn by
// their direction 30 m out, not by their first vertex.  Restated from Valhalla 2.x (external,
// absent here): parity of these degrees with meili is unpinned (DESIGN.md rule 3b).
constexpr double kHeadingOffsetM = 30.0;
RM_HD double det_heading(float lon_a, float lat_a, float lon_b, float lat_b) {   // PointLL::Heading
  if (lon_a == lon_b && lat_a == lat_b) return 0.0;
  const double la = (double)lat_a * kDegToRad, lb = (double)lat_b * kDegToRad;
  const double dl = ((double)lon_b - (double)lon_a) * kDegToRad;
  const double y = det_sin(dl) * det_cos(lb);                                     // east
  const double x = det_cos(la) * det_sin(lb) - det_sin(la) * det_cos(lb) * det_cos_wide(dl);   // north
  return det_bearing_deg(y, x);
}
// pt(i, lon, lat): shape point i of the edge (0 = its start node), n >= 2 points
template <class P>
RM_HD double heading_along(const P& pt, uint32_t n) {   // PointLL::HeadingAlongPolyline
  float lon0, lat0, lon1, lat1;
  pt(0u, lon0, lat0);
  if (n == 2u) {
    pt(1u, lon1, lat1);
    return det_heading(lon0, lat0, lon1, lat1);
  }
  double d = 0.0;
  float la = lon0, ta = lat0;
  for (uint32_t i = 0; i + 1u < n && d < kHeadingOffsetM; ++i) {
    pt(i + 1u, lon1, lat1);
    const double seg = gc_distance(la, ta, lon1, lat1);
    if (d + seg > kHeadingOffsetM) {
      const double pct = (kHeadingOffsetM - d) / seg;
      const float lon = (float)((double)la + ((double)lon1 - (double)la) * pct);
      const float lat = (float)((double)ta + ((double)lat1 - (double)ta) * pct);
      return det_heading(lon0, lat0, lon, lat);
    }
    d += seg;
    la = lon1;
    ta = lat1;
  }
  pt(n - 1u, lon1, lat1);
  return det_heading(lon0, lat0, lon1, lat1);
}
// whole degrees -> NodeInfo's 8 bits -> degrees 0..359
RM_HD uint32_t node_heading_deg(double h) {
  const uint32_t hd = (uint32_t)floor(h + 0.5) % 360u;
  const uint32_t h8 = (uint32_t)floorf((float)hd * (255.0f / 359.0f) + 0.5f);
  return (uint32_t)floorf((float)h8 * (359.0f / 255.0f) + 0.5f);
}
// turn angle class between an edge arriving with back heading hb (at the node, pointing the way
// it came) and an edge leaving with heading hs: 0 (U-turn) .. 180 (straight on)
RM_HD uint32_t turn_degree(uint32_t hb, uint32_t hs) {
  const uint32_t d = hb > hs ? hb - hs : hs - hb;
  return d > 180u ? 360u - d : d;
}
constexpr int kTurnDegrees = 181;
constexpr uint32_t kTurnScaleLog = 16;   // turn weight units per metre at factor 1: 2^16
// a road's headings packed in one word: H0 (at node0, into the road) | H1 (at node1) << 16.  A
// forward edge leaves node0 with H0 and arrives at node1 with back heading H1; a reverse edge the
// other way round.
RM_HD uint32_t head_start(uint32_t hw, uint32_t rev) { return rev ? hw >> 16 : hw & 0xffffu; }
RM_HD uint32_t head_back(uint32_t hw, uint32_t rev) { return rev ? hw & 0xffffu : hw >> 16; }
// Turn row word (route tables with turn costs, k_ball_turns): for the table of node x and an
// endpoint v of the row's road, the turn weight T of the canonical route x -> v entering the road
// at v (every turn on it but the one at x) | the heading the route leaves x with << 23.
// T = kTurnNone: not stored (the route's transitions go to the search tiers).
constexpr uint32_t kTurnTMask = 0x7fffffu, kTurnNone = 0x7fffffu, kTurnHeadShift = 23;

// ---- directed-edge record (16 B, one dwordx4 load in the route kernel) ----
// info bits: [0,16) speed in 0.1 km/h, [16,19) access mask, bit 19 internal, bit 20 service
struct EdgeRec {
  uint32_t target;   // end node
  uint32_t len_cm;   // integer centimetres (>= 1)
  uint32_t info;     // speed / access / flags
  uint32_t road;     // (road id << 1) | reversed
};
constexpr uint32_t kAccessAuto = 1u, kAccessBicycle = 2u, kAccessPedestrian = 4u;
constexpr uint32_t kFlagInternal = 1u << 19, kFlagService = 1u << 20;
RM_HD uint32_t edge_speed_dkph(uint32_t info) { return info & 0xffffu; }
RM_HD uint32_t edge_access(uint32_t info) { return (info >> 16) & 7u; }

// ---- shape vertex record (16 B) ----
struct VertRec {
  float lon, lat;
  uint32_t cum_cm;   // distance of this vertex from the road's first vertex (cm)
  uint32_t road;     // owning road; kNone for the last vertex of a road
};

// ---- travel modes ----
enum Mode : int { kModeAuto = 0, kModeBus = 1, kModeMotorScooter = 2, kModeBicycle = 3, kModePedestrian = 4 };
RM_HD uint32_t mode_access(int mode) {
  return mode == kModeBicycle ? kAccessBicycle : (mode == kModePedestrian ? kAccessPedestrian : kAccessAuto);
}
// speed used for routing time on an edge, in 0.1 km/h
RM_HD uint32_t mode_speed_dkph(int mode, uint32_t edge_dkph) {
  uint32_t cap = 0xffffu;
  if (mode == kModeBicycle) cap = 180;
  else if (mode == kModePedestrian) cap = 51;
  else if (mode == kModeMotorScooter) cap = 450;
  return edge_dkph < cap ? edge_dkph : cap;
}
// milliseconds to cover d_cm at speed dkph (floor)
RM_HD uint32_t time_ms(uint32_t d_cm, uint32_t dkph) {
  return (uint32_t)(((uint64_t)d_cm * 360ull) / (uint64_t)(dkph ? dkph : 1u));
}

// ---- route keys: lexicographic (distance cm, time ms) in one u64 ----
RM_HD uint64_t make_key(uint32_t d_cm, uint32_t t_ms) { return ((uint64_t)d_cm << 32) | t_ms; }
RM_HD uint32_t key_dist(uint64_t k) { return (uint32_t)(k >> 32); }
RM_HD uint32_t key_time(uint64_t k) { return (uint32_t)k; }
constexpr uint64_t kKeyInf = ~0ull;

// home slot of node v in a route-ball table of 2^bits entries (balls.hpp; bits >= 1)
#ifdef RM_BALL_SLOT_RANDOM
RM_HD uint32_t ball_slot(uint32_t v, uint32_t bits) { return (v * 2654435761u) >> (32u - bits); }
#else
// In a large table (>= 1024 slots) roads with ids in one aligned group of 8 keep adjacent rows
// (one 128-byte line): the target roads of a transition lie around one GPS point and
// neighbouring roads have neighbouring ids, so a transition's probes share lines; the groups
// are spread by a Fibonacci hash.  Small tables hash every road (few groups would collide into
// long probe chains: C4's 700 m tables ran K2 2x slower grouped).  C2 K2 1.10 -> 1.04 ms,
// C3 4.11 -> 3.58 ms on 200 k traces.
#ifndef RM_BALL_GROUP_LOG
#define RM_BALL_GROUP_LOG 3
#endif
#ifndef RM_BALL_GROUP_BITS
#define RM_BALL_GROUP_BITS 10
#endif
constexpr uint32_t kBallGroupBits = RM_BALL_GROUP_BITS, kBallGroupLog = RM_BALL_GROUP_LOG;
#ifndef RM_BALL_SLOTS_PER_ROW
#define RM_BALL_SLOTS_PER_ROW 2
#endif
constexpr uint32_t kBallSlotsPerRow = RM_BALL_SLOTS_PER_ROW;   // table size >= this x rows (load <= 1/this)
RM_HD uint32_t ball_slot(uint32_t v, uint32_t bits) {
  if (bits < kBallGroupBits) return (v * 2654435761u) >> (32u - bits);
  return ((((v >> kBallGroupLog) * 2654435761u) >> (32u + kBallGroupLog - bits)) << kBallGroupLog) |
         (v & ((1u << kBallGroupLog) - 1u));
}
// Canonical predecessors in the rows (round 3).  Above a 26-bit road id, a row's road word
// carries the canonical predecessor of each endpoint v of the road in the search from the
// table's node x: bits 26-28 for node0, 29-31 for node1, each the index, among v's in-edges in
// edge-id order (the engine's in_rec order), of the smallest-id edge u -> v usable by the mode
// with key(x -> u) + key(u -> v) == key(x -> v); kBallPredNone when v is x, or that index is 7 or
// more (the path walk then scans v's in-edges).  The path walk follows these one probe per node
// instead of probing every in-edge (k_paths_ball).  A graph of 2^26 - 1 roads or more keeps the
// whole word for the road: mask all-ones and no predecessors.
constexpr uint32_t kBallRoadBits = 26;
constexpr uint32_t kBallPredNone = 7u;
RM_HD uint32_t ball_road_mask(uint32_t n_roads) {
  return n_roads < (1u << kBallRoadBits) - 1u ? (1u << kBallRoadBits) - 1u : ~0u;
}
RM_HD uint32_t ball_road_word(uint32_t road, uint32_t p0, uint32_t p1, uint32_t mask) {
  return mask == ~0u ? road : road | p0 << kBallRoadBits | p1 << (kBallRoadBits + 3u);
}
// predecessor index of endpoint `side` (0: node0, 1: node1) in a row's road word
RM_HD uint32_t ball_pred(uint32_t word, uint32_t side, uint32_t mask) {
  return mask == ~0u ? kBallPredNone : (word >> (kBallRoadBits + 3u * side)) & 7u;
}

// Rank that writes a time-tile file (bucket, level | tile index << 3) in the multi-rank batch
// reporter: the rows of every rank are all-gathered and each file is culled and written by one
// rank (Fibonacci hash of the file key), so the privacy count sees every vehicle.  Shared by the
// device filter (stages.hip k_tile_own) and the host export rm_tile_file_owner.
RM_HD int tile_file_owner(uint64_t bucket, uint32_t tile, int nranks) {
  const unsigned long long h = (((unsigned long long)bucket << 25) | tile) * 0x9e3779b97f4a7c15ull;
  return (int)((h >> 33) % (unsigned long long)(nranks > 0 ? nranks : 1));
}

#endif

// A node's table starts at row 2 * hdr.x of its mode's entry array (hdr = {first row / 2,
// log2 size}): every table has a power-of-two size >= 2 and the tables are laid out back to
// back, so every first row is even, and a u32 hdr.x addresses 2^33 rows (128 GiB) per mode.
constexpr uint64_t kBallMaxRows = 1ull << 33;
RM_HD uint64_t ball_row0(uint32_t hx) { return (uint64_t)hx << 1; }

// Route-ball row (balls.hpp), 16 bytes: the keys from the table's node to both endpoints
// of road x, as 24-bit cm distances and 24-bit ms times split over the words:
//   x = road (kNone: free slot)
//   y = d0 | t0[7:0] << 24      z = d1 | t1[7:0] << 24      w = t0[23:8] | t1[23:8] << 16
// d = kBallNoDist: that endpoint is outside the ball.  24 bits hold 167 km / 4.6 h, so any
// radius up to the breakage distance fits in one row (the build gives a node no table when
// a key does not fit).
constexpr uint32_t kBallNoDist = 0xffffffu;
constexpr uint32_t kBallMaxField = 0xfffffeu;   // largest storable distance / time
RM_HD uint64_t ball_key0(uint32_t x, uint32_t y, uint32_t w) {
  const uint32_t d = y & 0xffffffu;
  return (x == 0xffffffffu || d == kBallNoDist) ? ~0ull : make_key(d, (y >> 24) | ((w & 0xffffu) << 8));
}
RM_HD uint64_t ball_key1(uint32_t x, uint32_t z, uint32_t w) {
  const uint32_t d = z & 0xffffffu;
  return (x == 0xffffffffu || d == kBallNoDist) ? ~0ull : make_key(d, (z >> 24) | ((w >> 16) << 8));
}
// pack the keys k0 / k1 (kKeyInf: outside) of one row; both fit (callers check ball_key_fits)
RM_HD void ball_pack(uint64_t k0, uint64_t k1, uint32_t& y, uint32_t& z, uint32_t& w) {
  const uint32_t d0 = k0 == ~0ull ? kBallNoDist : key_dist(k0), t0 = k0 == ~0ull ? 0u : key_time(k0);
  const uint32_t d1 = k1 == ~0ull ? kBallNoDist : key_dist(k1), t1 = k1 == ~0ull ? 0u : key_time(k1);
  y = d0 | (t0 & 0xffu) << 24;
  z = d1 | (t1 & 0xffu) << 24;
  w = (t0 >> 8) | (t1 >> 8) << 16;
}
RM_HD bool ball_key_fits(uint64_t k) { return key_dist(k) <= kBallMaxField && key_time(k) <= kBallMaxField; }

// ---- matcher limits ----
constexpr int kMaxCand = 16;            // K: candidates kept per state (nearest first)
constexpr float kMaxSearchRadius = 200.f;
constexpr uint32_t kRouteInvalid = 0xffffffffu;

// Per-request matcher options (meili defaults: Dockerfile:14-17, generate_test_trace.py:36-38).
struct MatchOptions {
  int32_t mode;
  float sigma_z;                    // 4.07
  float beta;                       // 3
  float search_radius;              // 50 m
  float gps_accuracy;               // 5 m (default accuracy when a point has none)
  float breakage_distance;          // 2000 m
  float interpolation_distance;     // 10 m
  float max_route_distance_factor;  // 5
  float max_route_time_factor;      // 2
  float turn_penalty_factor;        // meili's turn costs (rule 3b): 0 none; stock per-mode defaults 200 / 140 / 100
};
// meili's TransitionCostModel refuses a negative factor; infinities and NaN would poison the costs
constexpr const char* kTurnPenaltyError = "turn_penalty_factor must be non-negative and finite";
RM_HD bool turn_factor_ok(float f) { return f >= 0.f && f - f == 0.f; }   // f - f is NaN for +inf

RM_HD MatchOptions default_options() {
  MatchOptions o;
  o.mode = kModeAuto; o.sigma_z = 4.07f; o.beta = 3.f; o.search_radius = 50.f; o.gps_accuracy = 5.f;
  o.breakage_distance = 2000.f; o.interpolation_distance = 10.f; o.max_route_distance_factor = 5.f;
  o.max_route_time_factor = 2.f; o.turn_penalty_factor = 0.f;
  return o;
}

// ---- segment record produced by the engine (one matched OSMLR run) ----
struct SegmentRec {
  uint64_t segment_id;      // kInvalidSegmentId when the run has no OSMLR id
  double start_time;        // -1 when entered mid-segment
  double end_time;          // -1 when left mid-segment
  int32_t length;           // metres; -1 when partial
  int32_t queue_length;     // metres
  uint32_t flags;           // bit0 internal, bit1 has_id
  uint32_t begin_shape_index;
  uint32_t end_shape_index;
  uint32_t seg_dense;       // dense segment index (kNone if none)
  uint32_t way_first;       // way id of the run's first traversal
  uint32_t way_last;        // last way id differing from way_first (== way_first if none)
};
static_assert(sizeof(SegmentRec) == 56, "SegmentRec layout is shared with oracle/meili_oracle.h");

// ---- report record produced by the report epilogue (reporter_service.py:79-179) ----
struct ReportRec {
  uint64_t id;
  uint64_t next_id;         // kInvalidSegmentId when absent
  double t0, t1;
  int32_t length, queue_length;
  uint32_t seg_dense;
  uint32_t pad;
};
static_assert(sizeof(ReportRec) == 48, "ReportRec layout is shared with oracle/meili_oracle.h");

// ---- traversal record: one piece of a chosen path with its times and OSMLR tags ----
struct TravRec {
  uint32_t e, b, en, slot;          // directed edge, [b, en] cm along it, transition slot | flags below
  double tb, te;                    // interpolated epoch times at b and en
  uint32_t sd, soff, len, way;      // dense segment, edge offset in segment, edge length, way id
};
static_assert(sizeof(TravRec) == 48, "TravRec is three dwordx4");
// TravRec::slot flags: the edge is internal; the record is the last of its transition (its end
// state is the transition's target state, otherwise its source state)
constexpr uint32_t kTravInternal = 1u << 31, kTravLast = 1u << 30, kTravSlotMask = kTravLast - 1u;

struct ReportStats {        // per trace (reporter_service.py:164-177)
  int32_t successful_count, unreported_count;
  int32_t successful_length_m, unreported_length_m;  // last assigned length (m), -1 if never
  int32_t discontinuities, invalid_speeds, invalid_times, unassociated;
  int32_t shape_used;       // -1 when absent
  int32_t n_reports;
};

constexpr int kHistBins = 16;           // 10 km/h bins, 0..160 (reporter_service.py:133)

}  // namespace rm
