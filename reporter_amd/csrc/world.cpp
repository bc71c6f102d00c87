// world.cpp — seeded synthetic road world + GPS trace generator.
//
// The reference matches against Valhalla tiles built from OSM; none exist
// offline, so the engine ships its own world (SURVEY.md §8d "Synthetic world"):
//   * perturbed grid, every 10th line arterial (level 1), every 40th highway (level 0)
//   * internal edges (15 m) at intersections of two major lines (turn-channel analogue)
//   * OSMLR segments chained along each line and direction up to 1 km
//   * ~5 % local service roads with no OSMLR association, ~10 % one-way local roads
//   * segment ids: level | tile_index << 3 | segment_index << 25 with Valhalla's
//     tile sizes 4/1/0.25 degrees (reference py/get_tiles.py:35-39, py/simple_reporter.py:37-49)
// The trace generator restates reference py/generate_test_trace.py:35-104 (noise),
// :120-149 (1 s resampling at edge speed) and :151-164 (routed drives) on this world.
#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <thread>
#include <unordered_map>
#include "graph.hpp"

namespace rm {

namespace {

struct Rng {  // splitmix64-seeded xoshiro256**
  uint64_t s[4];
  static uint64_t sm(uint64_t& x) {
    uint64_t z = (x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  explicit Rng(uint64_t seed) { for (auto& v : s) v = sm(seed); }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t below(uint32_t n) { return (uint32_t)(uniform() * n) % (n ? n : 1); }
  double normal(double sigma) {
    double u1 = uniform(), u2 = uniform();
    if (u1 < 1e-300) u1 = 1e-300;
    return sigma * std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
};

uint64_t mix(uint64_t a, uint64_t b) { uint64_t x = a * 0x9e3779b97f4a7c15ull ^ (b + 0x632be59bd9b4e019ull); return Rng::sm(x); }

double round6(double x) { return std::round(x * 1e6) / 1e6; }

int line_level(uint32_t idx, const WorldParams& p) {
  if (p.highway_every && idx % p.highway_every == 0) return 0;
  if (p.arterial_every && idx % p.arterial_every == 0) return 1;
  return 2;
}

uint32_t level_speed(int level) { return level == 0 ? 900u : (level == 1 ? 500u : 300u); }

struct RoadSpec {
  uint32_t n0, n1;
  std::vector<std::pair<float, float>> shape;  // lon, lat incl. endpoints
  uint32_t info_fwd, info_rev;
  uint32_t way;
  int level;
  bool associable_fwd, associable_rev;
};

}  // namespace

// length of a straight shape piece, metres (equirectangular at its mean latitude)
double piece_m(float lon0, float lat0, float lon1, float lat1) {
  const double ml = 0.5 * ((double)lat0 + (double)lat1);
  const double dy = ((double)lat1 - (double)lat0) * kMetersPerDegLat;
  const double dx = ((double)lon1 - (double)lon0) * (kMetersPerDegLonEq * std::cos(ml * kDegToRad));
  return std::sqrt(dx * dx + dy * dy);
}

void assemble_roads(Graph& g, const std::vector<RoadInput>& roads) {
  // roads -> shapes, lengths
  const uint32_t R = (uint32_t)roads.size();
  g.road_node0.resize(R); g.road_node1.resize(R); g.road_len_cm.resize(R);
  g.road_vert_off.resize(R + 1);
  g.road_fwd.assign(R, kNone); g.road_rev.assign(R, kNone);
  g.verts.clear();
  for (uint32_t r = 0; r < R; ++r) {
    const RoadInput& rs = roads[r];
    g.road_node0[r] = rs.n0; g.road_node1[r] = rs.n1;
    g.road_vert_off[r] = (uint32_t)g.verts.size();
    double cum = 0;
    uint32_t last_cm = 0;
    for (size_t k = 0; k < rs.shape.size(); ++k) {
      if (k) cum += piece_m(rs.shape[k - 1].first, rs.shape[k - 1].second, rs.shape[k].first, rs.shape[k].second);
      uint32_t cm = (uint32_t)std::llround(cum * 100.0);
      if (k && cm <= last_cm) cm = last_cm + 1;  // strictly increasing
      last_cm = cm;
      VertRec v;
      v.lon = rs.shape[k].first; v.lat = rs.shape[k].second; v.cum_cm = cm;
      v.road = (k + 1 < rs.shape.size()) ? r : kNone;
      g.verts.push_back(v);
    }
    g.road_len_cm[r] = last_cm;
  }
  g.road_vert_off[R] = (uint32_t)g.verts.size();

  // directed edges -> CSR (stable by source node)
  const uint32_t N = (uint32_t)g.node_lon.size();
  struct DE { uint32_t from; EdgeRec rec; uint32_t way; };
  std::vector<DE> des;
  des.reserve(2 * (size_t)R);
  for (uint32_t r = 0; r < R; ++r) {
    des.push_back({roads[r].n0, {roads[r].n1, g.road_len_cm[r], roads[r].info_fwd, r << 1}, roads[r].way_fwd});
    des.push_back({roads[r].n1, {roads[r].n0, g.road_len_cm[r], roads[r].info_rev, (r << 1) | 1u}, roads[r].way_rev});
  }
  std::stable_sort(des.begin(), des.end(), [](const DE& a, const DE& b) { return a.from < b.from; });
  const uint32_t E = (uint32_t)des.size();
  g.node_off.assign(N + 1, 0);
  g.edges.resize(E);
  g.edge_way.resize(E);
  for (uint32_t e = 0; e < E; ++e) {
    g.node_off[des[e].from + 1]++;
    g.edges[e] = des[e].rec;
    g.edge_way[e] = des[e].way;
    const uint32_t road = des[e].rec.road >> 1;
    if (des[e].rec.road & 1u) g.road_rev[road] = e; else g.road_fwd[road] = e;
  }
  for (uint32_t n = 0; n < N; ++n) g.node_off[n + 1] += g.node_off[n];
  g.edge_seg.assign(E, kNone);
  g.edge_seg_off.assign(E, 0);
}

void build_grid_index(Graph& g) { build_grid_index(g.verts, g.grid); }

void build_grid_index(const std::vector<VertRec>& verts, GridIndex& gi) {
  const size_t ncell = (size_t)gi.ncx * gi.ncy;
  if (ncell > 400000000ull) throw std::runtime_error("grid index too large; raise cell_m");
  std::vector<uint32_t> cnt(ncell + 1, 0);
  auto cell_range = [&](const VertRec& a, const VertRec& b, uint32_t& x0, uint32_t& x1, uint32_t& y0, uint32_t& y1) {
    const double lo0 = std::min(a.lon, b.lon), lo1 = std::max(a.lon, b.lon);
    const double la0 = std::min(a.lat, b.lat), la1 = std::max(a.lat, b.lat);
    x0 = (uint32_t)std::floor((lo0 - gi.lon0) / gi.dlon); x1 = (uint32_t)std::floor((lo1 - gi.lon0) / gi.dlon);
    y0 = (uint32_t)std::floor((la0 - gi.lat0) / gi.dlat); y1 = (uint32_t)std::floor((la1 - gi.lat0) / gi.dlat);
    x1 = std::min(x1, gi.ncx - 1); y1 = std::min(y1, gi.ncy - 1);
  };
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) {
      gi.cell_off.assign(ncell + 1, 0);
      for (size_t c = 0; c < ncell; ++c) gi.cell_off[c + 1] = gi.cell_off[c] + cnt[c];
      gi.cell_item.resize(gi.cell_off[ncell]);
      std::fill(cnt.begin(), cnt.end(), 0);
    }
    for (uint32_t v = 0; v + 1 < (uint32_t)verts.size(); ++v) {
      if (verts[v].road == kNone) continue;
      uint32_t x0, x1, y0, y1;
      cell_range(verts[v], verts[v + 1], x0, x1, y0, y1);
      for (uint32_t y = y0; y <= y1; ++y)
        for (uint32_t x = x0; x <= x1; ++x) {
          const size_t c = (size_t)y * gi.ncx + x;
          if (pass == 1) gi.cell_item[gi.cell_off[c] + cnt[c]] = v;
          cnt[c]++;
        }
    }
  }
}

Graph build_world(const WorldParams& p) {
  if (p.rows < 2 || p.cols < 2) throw std::runtime_error("world needs at least 2x2 nodes");
  if ((uint64_t)p.rows * p.cols > 200000000ull) throw std::runtime_error("world too large");
  Graph g;
  const double mlon0 = kMetersPerDegLonEq * std::cos(p.center_lat * kDegToRad);
  const double y_half = 0.5 * p.block_m * (p.rows - 1), x_half = 0.5 * p.block_m * (p.cols - 1);
  auto to_ll = [&](double x, double y, float& lon, float& lat) {
    lat = (float)round6(p.center_lat + (y - y_half) / kMetersPerDegLat);
    lon = (float)round6(p.center_lon + (x - x_half) / mlon0);
  };
  // grid nodes
  const uint32_t nbase = p.rows * p.cols;
  std::vector<double> nx(nbase), ny(nbase);
  g.node_lon.resize(nbase);
  g.node_lat.resize(nbase);
  for (uint32_t i = 0; i < p.rows; ++i)
    for (uint32_t j = 0; j < p.cols; ++j) {
      Rng r(mix(p.seed, (uint64_t)i * p.cols + j));
      const uint32_t n = i * p.cols + j;
      nx[n] = j * p.block_m + (2 * r.uniform() - 1) * p.jitter * p.block_m;
      ny[n] = i * p.block_m + (2 * r.uniform() - 1) * p.jitter * p.block_m;
      to_ll(nx[n], ny[n], g.node_lon[n], g.node_lat[n]);
    }
  auto major = [&](uint32_t i, uint32_t j) { return line_level(i, p) <= 1 && line_level(j, p) <= 1; };
  auto add_node = [&](double x, double y) {
    float lo, la;
    to_ll(x, y, lo, la);
    g.node_lon.push_back(lo);
    g.node_lat.push_back(la);
    return (uint32_t)(g.node_lon.size() - 1);
  };

  std::vector<RoadSpec> roads;
  // per line and direction, the ordered list of road ids (for OSMLR chaining)
  std::vector<std::vector<uint32_t>> line_roads(p.rows + p.cols);

  auto make_piece = [&](uint32_t a, uint32_t b, bool a_major, bool b_major, int level, uint32_t way,
                        uint32_t line, uint64_t key) {
    Rng r(mix(p.seed ^ 0xabcdefull, key));
    const double ax = nx[a], ay = ny[a], bx = nx[b], by = ny[b];
    const double dx = bx - ax, dy = by - ay, len = std::sqrt(dx * dx + dy * dy);
    const double ux = dx / len, uy = dy / len;
    uint32_t na = a, nb = b;
    double sax = ax, say = ay, sbx = bx, sby = by;
    const bool split = len > 3 * p.internal_m;
    const uint32_t acc_line = level == 0 ? kAccessAuto : (kAccessAuto | kAccessBicycle | kAccessPedestrian);
    auto internal_road = [&](uint32_t n0, uint32_t n1) {
      RoadSpec rs;
      rs.n0 = n0; rs.n1 = n1;
      rs.shape = {{g.node_lon[n0], g.node_lat[n0]}, {g.node_lon[n1], g.node_lat[n1]}};
      const uint32_t info = 200u | (acc_line << 16) | kFlagInternal;
      rs.info_fwd = rs.info_rev = info;
      rs.way = way; rs.level = level; rs.associable_fwd = rs.associable_rev = false;
      roads.push_back(rs);
      line_roads[line].push_back((uint32_t)roads.size() - 1);
    };
    if (a_major && split) {
      sax = ax + ux * p.internal_m; say = ay + uy * p.internal_m;
      na = add_node(sax, say);
      internal_road(a, na);
    }
    if (b_major && split) {
      sbx = bx - ux * p.internal_m; sby = by - uy * p.internal_m;
      nb = add_node(sbx, sby);
    }
    RoadSpec rs;
    rs.n0 = na; rs.n1 = nb; rs.way = way; rs.level = level;
    rs.shape.push_back({g.node_lon[na], g.node_lat[na]});
    if (r.uniform() < p.curve_frac) {
      const double off = (2 * r.uniform() - 1) * 4.0;
      float lo, la;
      to_ll(0.5 * (sax + sbx) - uy * off, 0.5 * (say + sby) + ux * off, lo, la);
      rs.shape.push_back({lo, la});
    }
    rs.shape.push_back({g.node_lon[nb], g.node_lat[nb]});
    uint32_t speed = level_speed(level), acc_f = acc_line, acc_r = acc_line;
    bool service = false;
    rs.associable_fwd = rs.associable_rev = true;
    if (level == 2) {
      if (r.uniform() < p.service_frac) {
        service = true; speed = 150u;
        rs.associable_fwd = rs.associable_rev = false;
      } else if (r.uniform() < p.oneway_frac) {
        if (r.uniform() < 0.5) { acc_r = kAccessPedestrian; rs.associable_rev = false; }
        else { acc_f = kAccessPedestrian; rs.associable_fwd = false; }
      }
    }
    const uint32_t flags = service ? kFlagService : 0u;
    rs.info_fwd = speed | (acc_f << 16) | flags;
    rs.info_rev = speed | (acc_r << 16) | flags;
    roads.push_back(rs);
    line_roads[line].push_back((uint32_t)roads.size() - 1);
    if (b_major && split) internal_road(nb, b);
  };

  for (uint32_t i = 0; i < p.rows; ++i)  // horizontal lines
    for (uint32_t j = 0; j + 1 < p.cols; ++j)
      make_piece(i * p.cols + j, i * p.cols + j + 1, major(i, j), major(i, j + 1), line_level(i, p),
                 1000u + i, i, ((uint64_t)i << 32) | j);
  for (uint32_t j = 0; j < p.cols; ++j)  // vertical lines
    for (uint32_t i = 0; i + 1 < p.rows; ++i)
      make_piece(i * p.cols + j, (i + 1) * p.cols + j, major(i, j), major(i + 1, j), line_level(j, p),
                 1000u + p.rows + j, p.rows + j, (1ull << 62) | ((uint64_t)j << 32) | i);

  {
    std::vector<RoadInput> in(roads.size());
    for (size_t r = 0; r < roads.size(); ++r)
      in[r] = {roads[r].n0, roads[r].n1, roads[r].shape, roads[r].info_fwd, roads[r].info_rev, roads[r].way, roads[r].way};
    assemble_roads(g, in);
  }
  const uint32_t N = (uint32_t)g.node_lon.size();

  // OSMLR chaining along each line and direction
  const double tile_size[3] = {4.0, 1.0, 0.25};
  std::unordered_map<uint32_t, uint32_t> tile_counter[3];
  auto next_index = [&](int level, uint32_t tile) -> uint32_t { return tile_counter[level][tile]++; };
  auto close_segment = [&](std::vector<uint32_t>& run, uint32_t len_cm, int level) {
    if (run.empty()) return;
    const uint32_t e0 = run[0];
    // tile of the segment's first node
    uint32_t from = 0;
    {
      // source node of e0: search CSR (edges are sorted by source)
      uint32_t lo = 0, hi = N;
      while (hi - lo > 1) { uint32_t mid = (lo + hi) / 2; if (g.node_off[mid] <= e0) lo = mid; else hi = mid; }
      from = lo;
    }
    const double sz = tile_size[level];
    const uint32_t ncols = (uint32_t)std::llround(360.0 / sz);
    const uint32_t row = (uint32_t)std::floor(((double)g.node_lat[from] + 90.0) / sz);
    const uint32_t col = (uint32_t)std::floor(((double)g.node_lon[from] + 180.0) / sz);
    const uint32_t tile = row * ncols + col;
    const uint32_t idx = next_index(level, tile);
    const uint64_t id = (uint64_t)level | ((uint64_t)tile << kLevelBits) | ((uint64_t)idx << (kLevelBits + kTileIndexBits));
    const uint32_t s = (uint32_t)g.seg_id.size();
    g.seg_id.push_back(id);
    g.seg_len_cm.push_back(len_cm);
    uint32_t off = 0;
    for (uint32_t e : run) { g.edge_seg[e] = s; g.edge_seg_off[e] = off; off += g.edges[e].len_cm; }
    run.clear();
  };
  const uint32_t seg_max_cm = (uint32_t)std::llround(p.segment_max_m * 100.0);
  for (uint32_t line = 0; line < p.rows + p.cols; ++line) {
    const auto& lr = line_roads[line];
    for (int dir = 0; dir < 2; ++dir) {
      std::vector<uint32_t> run;
      uint32_t run_cm = 0;
      int run_level = 2;
      for (size_t k = 0; k < lr.size(); ++k) {
        const uint32_t r = dir == 0 ? lr[k] : lr[lr.size() - 1 - k];
        const bool assoc = dir == 0 ? roads[r].associable_fwd : roads[r].associable_rev;
        const uint32_t e = dir == 0 ? g.road_fwd[r] : g.road_rev[r];
        if (!assoc) { close_segment(run, run_cm, run_level); run_cm = 0; continue; }
        const uint32_t len = g.edges[e].len_cm;
        if (!run.empty() && run_cm + len > seg_max_cm) { close_segment(run, run_cm, run_level); run_cm = 0; }
        run.push_back(e);
        run_cm += len;
        run_level = roads[r].level;
      }
      close_segment(run, run_cm, run_level);
    }
  }

  // uniform grid index over shape segments
  float min_lon = 1e30f, min_lat = 1e30f, max_lon = -1e30f, max_lat = -1e30f;
  for (const auto& v : g.verts) {
    min_lon = std::min(min_lon, v.lon); max_lon = std::max(max_lon, v.lon);
    min_lat = std::min(min_lat, v.lat); max_lat = std::max(max_lat, v.lat);
  }
  GridIndex& gi = g.grid;
  gi.dlat = p.cell_m / kMetersPerDegLat;
  gi.dlon = p.cell_m / mlon0;
  gi.lon0 = (double)min_lon - gi.dlon;
  gi.lat0 = (double)min_lat - gi.dlat;
  gi.ncx = (uint32_t)std::ceil(((double)max_lon - gi.lon0) / gi.dlon) + 2;
  gi.ncy = (uint32_t)std::ceil(((double)max_lat - gi.lat0) / gi.dlat) + 2;
  build_grid_index(g);
  g.validate();
  return g;
}

// ---------------------------------------------------------------------------
// trace generator

namespace {

void position_on_edge(const Graph& g, uint32_t e, uint32_t off_cm, double& lon, double& lat) {
  const EdgeRec& er = g.edges[e];
  const uint32_t r = er.road >> 1;
  const bool rev = er.road & 1u;
  const uint32_t L = g.road_len_cm[r];
  const uint32_t s = rev ? L - std::min(off_cm, L) : std::min(off_cm, L);  // offset from road start
  const uint32_t v0 = g.road_vert_off[r], v1 = g.road_vert_off[r + 1];
  for (uint32_t v = v0; v + 1 < v1; ++v) {
    const VertRec& a = g.verts[v];
    const VertRec& b = g.verts[v + 1];
    if (s <= b.cum_cm || v + 2 == v1) {
      const double t = b.cum_cm > a.cum_cm ? (double)(s - std::min(s, a.cum_cm)) / (double)(b.cum_cm - a.cum_cm) : 0.0;
      const double tc = std::min(1.0, std::max(0.0, t));
      lon = (double)a.lon + tc * ((double)b.lon - (double)a.lon);
      lat = (double)a.lat + tc * ((double)b.lat - (double)a.lat);
      return;
    }
  }
  lon = g.verts[v1 - 1].lon; lat = g.verts[v1 - 1].lat;
}

// Fastest-route planner for the trace generator.  The reference generator drives a
// Valhalla /route answer between two locations with auto costing
// (py/generate_test_trace.py:151-164, then the :166-179 edge walk); here the same role
// is played by an A* search on edge travel time (mode speeds) to a random destination,
// so traces follow the fast road classes the way routed traffic does.
struct RoutePlanner {
  const Graph& g;
  int mode;
  uint32_t acc, vmax_dkph;
  std::vector<uint32_t> stamp, done, cost, pedge;
  std::vector<std::pair<uint64_t, uint32_t>> heap;
  uint32_t gen = 0;
  static constexpr uint32_t kSettleCap = 400000;

  RoutePlanner(const Graph& gr, int m)
      : g(gr), mode(m), acc(mode_access(m)), vmax_dkph(mode_speed_dkph(m, 900u)),
        stamp(gr.num_nodes(), 0), done(gr.num_nodes(), 0), cost(gr.num_nodes(), 0), pedge(gr.num_nodes(), kNone) {}

  uint32_t h_ms(uint32_t n, uint32_t dst) const {
    const double d = piece_m(g.node_lon[n], g.node_lat[n], g.node_lon[dst], g.node_lat[dst]);
    return (uint32_t)(0.95 * d * 36000.0 / (double)vmax_dkph);
  }

  // a uniform draw among the nodes whose straight-line distance from `from` is in
  // [lo_m, hi_m], found by a breadth-first walk that stops at hi_m (kNone when empty)
  uint32_t ring_node(uint32_t from, double lo_m, double hi_m, Rng& r) {
    if (++gen == 0) {
      std::fill(stamp.begin(), stamp.end(), 0u);
      std::fill(done.begin(), done.end(), 0u);
      gen = 1;
    }
    std::vector<uint32_t> q{from}, hits;
    stamp[from] = gen;
    for (size_t h = 0; h < q.size() && q.size() < 400000; ++h) {
      const uint32_t u = q[h];
      for (uint32_t e = g.node_off[u]; e < g.node_off[u + 1]; ++e) {
        const uint32_t v = g.edges[e].target;
        if (stamp[v] == gen) continue;
        stamp[v] = gen;
        const double d = piece_m(g.node_lon[from], g.node_lat[from], g.node_lon[v], g.node_lat[v]);
        if (d > hi_m) continue;
        q.push_back(v);
        if (d >= lo_m) hits.push_back(v);
      }
    }
    return hits.empty() ? kNone : hits[r.below((uint32_t)hits.size())];
  }

  // edges of the fastest route src -> dst whose first edge is not on road `avoid_road`
  bool plan(uint32_t src, uint32_t avoid_road, uint32_t dst, std::vector<uint32_t>& out) {
    out.clear();
    if (src == dst) return false;
    if (++gen == 0) {
      std::fill(stamp.begin(), stamp.end(), 0u);
      std::fill(done.begin(), done.end(), 0u);
      gen = 1;
    }
    typedef std::pair<uint64_t, uint32_t> Item;  // ((f << 32) | node) orders ties by node id
    heap.clear();
    auto push = [&](uint32_t v, uint32_t gcost) {
      const uint64_t f = (uint64_t)gcost + h_ms(v, dst);
      heap.push_back(Item((f << 32) | v, v));
      std::push_heap(heap.begin(), heap.end(), std::greater<Item>());
    };
    stamp[src] = gen; cost[src] = 0; pedge[src] = kNone;
    push(src, 0);
    uint32_t settled = 0;
    while (!heap.empty()) {
      std::pop_heap(heap.begin(), heap.end(), std::greater<Item>());
      const uint32_t u = heap.back().second;
      heap.pop_back();
      if (done[u] == gen) continue;
      done[u] = gen;
      if (u == dst) break;
      if (++settled > kSettleCap) return false;
      for (uint32_t e = g.node_off[u]; e < g.node_off[u + 1]; ++e) {
        const EdgeRec& er = g.edges[e];
        if (!(edge_access(er.info) & acc)) continue;
        if (u == src && (er.road >> 1) == avoid_road) continue;
        const uint32_t v = er.target;
        if (done[v] == gen) continue;
        const uint32_t nc = cost[u] + time_ms(er.len_cm, mode_speed_dkph(mode, edge_speed_dkph(er.info)));
        if (stamp[v] != gen || nc < cost[v]) {
          stamp[v] = gen; cost[v] = nc; pedge[v] = e;
          push(v, nc);
        }
      }
    }
    if (done[dst] != gen) return false;
    for (uint32_t x = dst; x != src;) {
      const uint32_t e = pedge[x];
      out.push_back(e);
      const uint32_t road = g.edges[e].road >> 1;  // source node of e = far end of its twin
      x = (g.edges[e].road & 1u) ? g.road_node1[road] : g.road_node0[road];
    }
    std::reverse(out.begin(), out.end());
    return true;
  }
};

// random destination node at a driving distance that fits the rest of the trace
uint32_t pick_destination(const Graph& g, Rng& r, uint32_t from, double remaining_s, RoutePlanner& planner) {
  const double want = std::min(6000.0, std::max(400.0, remaining_s * 12.0));
  uint32_t best = kNone;
  double best_err = 1e300;
  for (int tries = 0; tries < 24; ++tries) {
    const uint32_t n = r.below(g.num_nodes());
    if (n == from) continue;
    const double d = piece_m(g.node_lon[from], g.node_lat[from], g.node_lon[n], g.node_lat[n]);
    const double err = std::fabs(d - want);
    if (err < best_err) { best_err = err; best = n; }
    if (d >= 0.5 * want && d <= 1.5 * want) return n;
  }
  // graphs much wider than the trace's reach (C4 country scale): uniform draws miss the
  // distance window, and the nearest miss may be hundreds of km away (an A* to it would
  // settle the planner's whole cap).  Draw from the ring of nodes around `from` instead.
  const uint32_t ring = planner.ring_node(from, 0.5 * want, 1.5 * want, r);
  return ring != kNone ? ring : best;
}

// trace number k of the seeded set (its own RNG stream), written to output slot `slot`
void gen_one(const Graph& g, const TraceParams& p, uint32_t k, uint32_t slot, TraceSet& ts,
             const std::vector<uint32_t>& starts, RoutePlanner& planner) {
  Rng r(mix(p.seed, 0x7472616365ull + k));
  const uint32_t acc = mode_access(p.mode);
  const uint32_t base = ts.trace_off[slot];
  // start edge
  uint32_t e = starts[r.below((uint32_t)starts.size())];
  double off_m = r.uniform() * g.edges[e].len_cm * 0.01;
  std::vector<uint32_t> route;
  size_t ri = 0;
  const double t_total = (p.n_points ? p.n_points - 1 : 0) * p.rate_s;
  const int lookback = (int)std::ceil(30.0 / (p.rate_s + 2.0));
  std::vector<double> hx, hy;
  int qx = 0, qy = 0;
  double t_now = 0.0;
  const double accuracy = std::round(std::min(100.0, 1.6448536269514722 * std::max(1.0, p.noise_m)) * 100.0) / 100.0;
  const int64_t t0 = p.start_epoch + (int64_t)(k % 3600u);
  for (uint32_t s = 0; s < p.n_points; ++s) {
    const double t_target = s * p.rate_s;
    // drive forward to t_target
    while (true) {
      const double len_m = g.edges[e].len_cm * 0.01;
      const double v = mode_speed_dkph(p.mode, edge_speed_dkph(g.edges[e].info)) / 36.0;  // m/s
      const double t_end = t_now + (len_m - off_m) / v;
      if (t_end >= t_target) { off_m += (t_target - t_now) * v; t_now = t_target; break; }
      t_now = t_end;
      const uint32_t node = g.edges[e].target;
      const uint32_t road = g.edges[e].road >> 1;
      // follow the planned route; plan a new one to a fresh destination when it ends
      if (ri >= route.size()) {
        route.clear();
        ri = 0;
        const uint32_t dst = pick_destination(g, r, node, t_total - t_now, planner);
        if (dst != kNone) planner.plan(node, road, dst, route);
      }
      if (ri < route.size()) { e = route[ri++]; off_m = 0.0; continue; }
      // no route from here (island / one-way trap): random continuation as a fallback,
      // straight on the same way with p=0.6, else uniform; avoid U-turns
      uint32_t opts[16]; uint32_t no = 0; uint32_t straight = kNone;
      for (uint32_t x = g.node_off[node]; x < g.node_off[node + 1] && no < 16; ++x) {
        if (!(edge_access(g.edges[x].info) & acc) || (g.edges[x].road >> 1) == road) continue;
        opts[no++] = x;
        if (g.edge_way[x] == g.edge_way[e]) straight = x;
      }
      uint32_t ne;
      if (no == 0) {  // dead end: U-turn
        ne = kNone;
        for (uint32_t x = g.node_off[node]; x < g.node_off[node + 1]; ++x)
          if ((g.edges[x].road >> 1) == road && (edge_access(g.edges[x].info) & acc)) ne = x;
        if (ne == kNone) { off_m = len_m; t_now = t_target; break; }  // stuck: stay put
      } else if (straight != kNone && r.uniform() < 0.6) {
        ne = straight;
      } else {
        ne = opts[r.below(no)];
      }
      e = ne; off_m = 0.0;
    }
    uint32_t off_cm = (uint32_t)std::min<double>(g.edges[e].len_cm, std::floor(off_m * 100.0));
    double lon, lat;
    position_on_edge(g, e, off_cm, lon, lat);
    if (p.noise_m > 0) {  // generate_test_trace.py:77-92
      double ax, ay;
      while (true) {
        ax = r.normal(p.noise_m); ay = r.normal(p.noise_m);
        const int sx = ax > 0 ? 1 : (ax < 0 ? -1 : 0), sy = ay > 0 ? 1 : (ay < 0 ? -1 : 0);
        if (s == 0) { qx = sx; qy = sy; break; }
        if (sx == qx && sy == qy) break;
      }
      hx.push_back(ax); hy.push_back(ay);
      const size_t n = hx.size(), m = std::min<size_t>(n, (size_t)lookback);
      double mx = 0, my = 0;
      for (size_t i = n - m; i < n; ++i) { mx += hx[i]; my += hy[i]; }
      mx /= (double)m; my /= (double)m;
      lon += mx / (kMetersPerDegLonEq * std::cos(lat * kDegToRad));
      lat += my / kMetersPerDegLat;
    }
    ts.lon[base + s] = round6(lon);
    ts.lat[base + s] = round6(lat);
    ts.time[base + s] = (double)(t0 + (int64_t)std::llround(t_target));
    ts.accuracy[base + s] = (float)accuracy;
    ts.truth_edge[base + s] = e;
    ts.truth_off_cm[base + s] = off_cm;
  }
}

}  // namespace

TraceSet generate_traces(const Graph& g, const TraceParams& p, const uint32_t* ids) {
  TraceSet ts;
  const uint64_t P = (uint64_t)p.n_traces * p.n_points;
  if (P > 0xffffffffull) throw std::runtime_error("too many points for one trace set");
  ts.lon.resize(P); ts.lat.resize(P); ts.time.resize(P); ts.accuracy.resize(P);
  ts.truth_edge.resize(P); ts.truth_off_cm.resize(P);
  ts.trace_off.resize(p.n_traces + 1);
  for (uint32_t k = 0; k <= p.n_traces; ++k) ts.trace_off[k] = k * p.n_points;
  const uint32_t acc = mode_access(p.mode);
  std::vector<uint32_t> starts;
  for (uint32_t e = 0; e < g.num_edges(); ++e)
    if ((edge_access(g.edges[e].info) & acc) && !(g.edges[e].info & kFlagInternal)) starts.push_back(e);
  if (starts.empty()) throw std::runtime_error("no edge usable by this mode");
  unsigned nt = p.threads ? p.threads : std::max(1u, std::thread::hardware_concurrency());
  nt = std::min<unsigned>(nt, 64);
  if (p.n_traces < 64) nt = 1;
  // each thread owns a route planner (16 B per node); keep them within ~4 GiB
  const uint64_t per = 16ull * std::max<uint32_t>(g.num_nodes(), 1u);
  nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nt, (4ull << 30) / per));
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      RoutePlanner planner(g, p.mode);
      for (uint32_t k = t; k < p.n_traces; k += nt) gen_one(g, p, ids ? ids[k] : k, k, ts, starts, planner);
    });
  for (auto& x : th) x.join();
  return ts;
}

}  // namespace rm
