// osm_city.cpp — a seeded irregular city written as generic OpenStreetMap (PBF or XML).
//
// The reference matches on Valhalla tiles that valhalla_build_tiles makes from an OSM extract
// (reference Dockerfile:42-49; tile hierarchy py/get_tiles.py:30-102, OSMLR ids
// py/simple_reporter.py:36-49).  The engine's own world generator (world.cpp) lays a perturbed
// grid out as roads directly; this file instead writes a city the way an OSM extract describes
// one, with no reporter:* tags, so rm_graph_import_osm takes its generic path (split at shared
// nodes, speeds and access from tags, OSMLR only where relations name it).  It carries what a
// real extract has and the grid never does:
//   * curved multi-vertex ways (quadratic Bezier links, 0-8 interior vertices per block), long
//     ways over many blocks and grid cells that only the importer splits into roads;
//   * diagonal and anti-diagonal avenues: where they cross, four ways meet in one node (8 roads)
//     and a cul-de-sac starts there too (9 in-edges: beyond the 3-bit stored predecessor index
//     of the route-ball rows, rm_common.hpp kBallPredNone);
//   * roundabouts (closed junction=roundabout ways, one-way by OSM convention) where the
//     streets end on the ring;
//   * boulevards as pairs of one-way carriageways, the cross streets passing both;
//   * one-way residential streets, dead-end spurs, service loops (a second road between the
//     same two nodes), footways and cycleways through blocks, links left out of the lattice;
//   * a trunk road crossing the city on bridges (no shared nodes with the streets under it),
//     joined to them only at interchanges by trunk_link ramps;
//   * type=osmlr relations on the classified roads and on a fraction of residential ways only,
//     one or two member ways, forward and backward;
//   * OSM ids in the shuffled chunks of consecutive ids real extracts have (node and way order
//     is not spatial order).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <map>
#include <memory>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

#include "osm_model.hpp"

namespace rm {

namespace {

struct Rng {  // splitmix64
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9e3779b97f4a7c15ull + 0x2545f4914f6cdd1dull) {}
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t below(uint32_t n) { return n ? (uint32_t)(next() % n) : 0u; }
  bool chance(double p) { return uniform() < p; }
};

// lattice sides a link leaves a junction by
enum Side { kW = 0, kE = 1, kS = 2, kN = 3, kBelow = 4, kAbove = 5 };

struct Way {
  std::vector<uint32_t> refs;   // node indices
  std::string hw;
  int level = 2;                // OSMLR level: 0 trunk/primary, 1 secondary/tertiary, 2 local
  int oneway = 0;               // 1 forward only, -1 reverse only (for vehicles)
  bool roundabout = false, osmlr = false, bridge = false;
  std::string maxspeed, access;
  int line = -1;                // lattice line the way was cut from (-1: none)
  double len_m = 0;
};

class City {
 public:
  explicit City(const CityParams& p) : p_(p), rng_(p.seed) {
    if (p.rows < 3 || p.cols < 3) throw std::runtime_error("city needs at least 3x3 junctions");
    if ((uint64_t)p.rows * p.cols > 4000000ull) throw std::runtime_error("city too large");
    if (!(p.block_m >= 40.0)) throw std::runtime_error("city block_m must be >= 40 m");
    if (p.diagonal_every % 2) throw std::runtime_error("diagonal_every must be even (no mid-block crossings)");
    W_ = p.block_m * (p.cols - 1);
    H_ = p.block_m * (p.rows - 1);
    mlon_ = kMetersPerDegLonEq * std::cos(p.center_lat * kDegToRad);
  }

  void build() {
    junctions();
    streets();
    diagonals();
    if (p_.trunk) trunk();
    extras();
    relations();
  }

  void emit(OsmSink& sink) {
    // ids in the order an edited map accumulates them: chunks of consecutive ids, the chunks
    // themselves not in spatial order
    const std::vector<uint64_t> nid = shuffled_ids(nodes_x_.size(), 256, 2100000000ull);
    const std::vector<uint64_t> wid = shuffled_ids(ways_.size(), 48, 150000000ull);
    std::vector<float> lat(nodes_x_.size()), lon(nodes_x_.size());
    float la0 = 1e30f, la1 = -1e30f, lo0 = 1e30f, lo1 = -1e30f;
    for (size_t i = 0; i < nodes_x_.size(); ++i) {
      // OSM's 7 decimal places, then the float the graph keeps
      lat[i] = (float)(std::round((p_.center_lat + (nodes_y_[i] - 0.5 * H_) / kMetersPerDegLat) * 1e7) / 1e7);
      lon[i] = (float)(std::round((p_.center_lon + (nodes_x_[i] - 0.5 * W_) / mlon_) * 1e7) / 1e7);
      la0 = std::min(la0, lat[i]); la1 = std::max(la1, lat[i]);
      lo0 = std::min(lo0, lon[i]); lo1 = std::max(lo1, lon[i]);
    }
    sink.bounds(la0, lo0, la1, lo1);
    std::vector<uint32_t> order(nodes_x_.size());
    std::iota(order.begin(), order.end(), 0u);
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return nid[a] < nid[b]; });
    for (uint32_t i : order) sink.node(nid[i], lat[i], lon[i]);
    std::vector<uint32_t> word(ways_.size());
    std::iota(word.begin(), word.end(), 0u);
    std::sort(word.begin(), word.end(), [&](uint32_t a, uint32_t b) { return wid[a] < wid[b]; });
    std::vector<uint64_t> refs;
    for (uint32_t w : word) {
      const Way& wy = ways_[w];
      refs.clear();
      for (uint32_t r : wy.refs) refs.push_back(nid[r]);
      OsmTags t;
      t.push_back({"highway", wy.hw});
      if (!wy.maxspeed.empty()) t.push_back({"maxspeed", wy.maxspeed});
      if (wy.roundabout) t.push_back({"junction", "roundabout"});
      if (wy.oneway == 1) t.push_back({"oneway", "yes"});
      if (wy.oneway == -1) t.push_back({"oneway", "-1"});
      if (wy.bridge) { t.push_back({"bridge", "yes"}); t.push_back({"layer", "1"}); }
      if (!wy.access.empty()) t.push_back({"access", wy.access});
      if (wy.hw == "residential" && rng_.chance(0.5)) t.push_back({"name", "Street " + std::to_string(w)});
      sink.way(wid[w], refs, t);
    }
    std::vector<OsmMember> mem;
    for (size_t k = 0; k < rels_.size(); ++k) {
      const Rel& rl = rels_[k];
      mem.clear();
      for (const auto& m : rl.members) mem.push_back({"way", m.second ? "backward" : "forward", wid[m.first]});
      OsmTags t{{"type", "osmlr"}, {"osmlr:id", std::to_string(rl.id)}};
      sink.relation(7000000ull + k, mem, t);
    }
    sink.finish();
  }

 private:
  struct Rel {
    uint64_t id;
    std::vector<std::pair<uint32_t, bool>> members;   // (way, backward)
  };
  const CityParams& p_;
  Rng rng_;
  double W_, H_, mlon_;
  std::vector<double> nodes_x_, nodes_y_;
  std::vector<Way> ways_;
  std::vector<Rel> rels_;
  // per junction: kind 0 plain, 1 roundabout, 2 split (boulevard row); its node(s)
  std::vector<uint8_t> kind_;
  std::vector<uint32_t> center_, ring_;   // ring_: 4 nodes per junction (W, E, S, N) or split S/N at [2], [3]
  std::vector<double> jx_, jy_;
  // interior vertices of every lattice link (for things that attach mid-block); key: line, index
  std::map<std::pair<int, uint32_t>, std::vector<uint32_t>> link_interior_;

  uint32_t add_node(double x, double y) {
    nodes_x_.push_back(x);
    nodes_y_.push_back(y);
    return (uint32_t)nodes_x_.size() - 1;
  }
  uint32_t J(uint32_t i, uint32_t j) const { return i * p_.cols + j; }
  bool on_diag(uint32_t i, uint32_t j) const {
    const uint32_t k = p_.diagonal_every;
    return k && (((int64_t)j - (int64_t)i) % (int64_t)k == 0 || (i + j) % k == 0);
  }
  bool hub(uint32_t i, uint32_t j) const {
    const uint32_t k = p_.diagonal_every;
    return k && ((int64_t)j - (int64_t)i) % (int64_t)k == 0 && (i + j) % k == 0;
  }
  bool boulevard_row(uint32_t i) const {
    return p_.boulevard_every && i % p_.boulevard_every == p_.boulevard_every / 2 && i > 0 && i + 1 < p_.rows;
  }
  std::string row_class(uint32_t i, int& level) const {
    if (boulevard_row(i) || (p_.primary_every && i % p_.primary_every == 0)) { level = 0; return "primary"; }
    if (p_.secondary_every && i % p_.secondary_every == 0) { level = 1; return i % (2 * p_.secondary_every) ? "tertiary" : "secondary"; }
    level = 2;
    return "residential";
  }

  // the node a link leaving junction (i, j) by `side` starts or ends at
  uint32_t jn(uint32_t i, uint32_t j, int side) const {
    const uint32_t q = J(i, j);
    if (kind_[q] == 1) return ring_[4 * q + (side >= 4 ? (side == kBelow ? kS : kN) : side)];
    if (kind_[q] == 2) {
      if (side == kS || side == kBelow) return ring_[4 * q + 2];
      if (side == kN || side == kAbove) return ring_[4 * q + 3];
    }
    return center_[q];
  }

  void junctions() {
    const uint32_t n = p_.rows * p_.cols;
    kind_.assign(n, 0);
    center_.assign(n, kNone);
    ring_.assign(4 * (size_t)n, kNone);
    jx_.resize(n);
    jy_.resize(n);
    for (uint32_t i = 0; i < p_.rows; ++i)
      for (uint32_t j = 0; j < p_.cols; ++j) {
        const uint32_t q = J(i, j);
        const bool border = i == 0 || j == 0 || i + 1 == p_.rows || j + 1 == p_.cols;
        jx_[q] = j * p_.block_m + (border ? 0.0 : (2 * rng_.uniform() - 1) * p_.jitter * p_.block_m);
        jy_[q] = i * p_.block_m + (border ? 0.0 : (2 * rng_.uniform() - 1) * p_.jitter * p_.block_m);
        if (boulevard_row(i)) {
          kind_[q] = 2;
          const double half = 8.0 + 2.0 * rng_.uniform();
          ring_[4 * q + 2] = add_node(jx_[q], jy_[q] - half);
          ring_[4 * q + 3] = add_node(jx_[q], jy_[q] + half);
        } else if (!border && !on_diag(i, j) && !boulevard_row(i - 1) && !boulevard_row(i + 1) &&
                   rng_.chance(p_.roundabout_frac)) {
          kind_[q] = 1;
        } else {
          center_[q] = add_node(jx_[q], jy_[q]);
        }
      }
    // roundabouts: a ring of radius 15-22 m; the streets end on it at W / E / S / N, with two
    // shape vertices between neighbouring entries; one closed way, counter-clockwise
    for (uint32_t q = 0; q < n; ++q) {
      if (kind_[q] != 1) continue;
      const double r = 15.0 + 7.0 * rng_.uniform();
      Way w;
      w.hw = "tertiary";
      w.level = 1;
      w.roundabout = true;
      const int entry_side[4] = {kE, kN, kW, kS};   // at 0, 90, 180, 270 degrees
      uint32_t first = kNone;
      for (int k = 0; k < 4; ++k) {
        const double a = k * 0.5 * kPi;
        const uint32_t e = add_node(jx_[q] + r * std::cos(a), jy_[q] + r * std::sin(a));
        ring_[4 * q + entry_side[k]] = e;
        if (!k) first = e;
        w.refs.push_back(e);
        for (int m = 1; m <= 2; ++m) {
          const double b = a + m * (0.5 * kPi / 3.0);
          w.refs.push_back(add_node(jx_[q] + r * std::cos(b), jy_[q] + r * std::sin(b)));
        }
      }
      w.refs.push_back(first);
      ways_.push_back(w);
    }
  }

  // interior vertices of a curved link a -> b: a quadratic Bezier whose control point sits
  // `bend` x length off the chord's midpoint
  void link_shape(uint32_t a, uint32_t b, uint32_t nv, double bend, std::vector<uint32_t>& out) {
    const double ax = nodes_x_[a], ay = nodes_y_[a], bx = nodes_x_[b], by = nodes_y_[b];
    const double dx = bx - ax, dy = by - ay, len = std::sqrt(dx * dx + dy * dy);
    const double cx = 0.5 * (ax + bx) - dy / len * bend * len, cy = 0.5 * (ay + by) + dx / len * bend * len;
    for (uint32_t k = 1; k <= nv; ++k) {
      const double t = (double)k / (nv + 1), u = 1 - t;
      out.push_back(add_node(u * u * ax + 2 * u * t * cx + t * t * bx, u * u * ay + 2 * u * t * cy + t * t * by));
    }
  }

  double dist(uint32_t a, uint32_t b) const {
    return std::hypot(nodes_x_[a] - nodes_x_[b], nodes_y_[a] - nodes_y_[b]);
  }

  // A lattice line walked link by link into ways: a way ends where the next link does not start
  // at its last node (a roundabout, a boulevard crossed diagonally), where a link is missing, and
  // once it is longer than way_max_m.
  struct LineWalker {
    City& c;
    int line;
    std::string hw;
    int level;
    int oneway;
    std::string maxspeed;
    Way cur;
    void close() {
      if (cur.refs.size() >= 2) {
        cur.hw = hw; cur.level = level; cur.line = line; cur.maxspeed = maxspeed;
        cur.oneway = oneway;
        if (hw == "residential" && !oneway && c.rng_.chance(c.p_.oneway_frac)) cur.oneway = c.rng_.chance(0.5) ? 1 : -1;
        c.ways_.push_back(cur);
      }
      cur = Way();
    }
    void link(uint32_t a, uint32_t b, uint32_t idx, uint32_t nv, double bend) {
      if (!cur.refs.empty() && (cur.refs.back() != a || cur.len_m > c.p_.way_max_m)) close();
      if (cur.refs.empty()) cur.refs.push_back(a);
      std::vector<uint32_t> in;
      c.link_shape(a, b, nv, bend, in);
      c.link_interior_[{line, idx}] = in;
      uint32_t prev = a;
      for (uint32_t v : in) { cur.refs.push_back(v); cur.len_m += c.dist(prev, v); prev = v; }
      cur.refs.push_back(b);
      cur.len_m += c.dist(prev, b);
    }
  };

  uint32_t nverts(int level) {
    if (rng_.chance(0.25)) return 0;
    return level == 2 ? 1 + rng_.below(3) : 2 + rng_.below(6);
  }
  double bend() { return rng_.chance(0.3) ? 0.0 : (2 * rng_.uniform() - 1) * 0.12; }

  void streets() {
    // rows (lines 0..rows-1): ways west to east; boulevard rows as two one-way carriageways
    for (uint32_t i = 0; i < p_.rows; ++i) {
      int level;
      const std::string hw = row_class(i, level);
      const std::string ms = level == 0 ? "60" : (level == 1 ? "50" : (rng_.chance(0.5) ? "30" : ""));
      if (boulevard_row(i)) {
        // south carriageway eastbound, north carriageway westbound (its ways run east to west)
        LineWalker s{*this, (int)i, hw, level, 1, ms, Way()};
        for (uint32_t j = 0; j + 1 < p_.cols; ++j)
          s.link(ring_[4 * J(i, j) + 2], ring_[4 * J(i, j + 1) + 2], j, nverts(level), bend());
        s.close();
        LineWalker nw{*this, (int)(p_.rows + p_.cols + i), hw, level, 1, ms, Way()};
        for (uint32_t j = p_.cols - 1; j > 0; --j)
          nw.link(ring_[4 * J(i, j) + 3], ring_[4 * J(i, j - 1) + 3], j, nverts(level), bend());
        nw.close();
        continue;
      }
      LineWalker w{*this, (int)i, hw, level, 0, ms, Way()};
      for (uint32_t j = 0; j + 1 < p_.cols; ++j) {
        const bool keep = level < 2 || !rng_.chance(p_.drop_frac) || i == 0 || i + 1 == p_.rows;
        if (!keep) { w.close(); continue; }
        w.link(jn(i, j, kE), jn(i, j + 1, kW), j, nverts(level), bend());
      }
      w.close();
    }
    // columns (lines rows..rows+cols-1): ways south to north; a boulevard's two carriageway
    // nodes are joined by the column itself
    for (uint32_t j = 0; j < p_.cols; ++j) {
      int level;
      const std::string hw = row_class(j, level);
      const std::string ms = level == 0 ? "60" : (level == 1 ? "50" : (rng_.chance(0.5) ? "30" : ""));
      const int line = (int)(p_.rows + j);
      LineWalker w{*this, line, hw, level, 0, ms, Way()};
      for (uint32_t i = 0; i + 1 < p_.rows; ++i) {
        if (kind_[J(i, j)] == 2) w.link(ring_[4 * J(i, j) + 2], ring_[4 * J(i, j) + 3], 2 * p_.rows + i, 0, 0.0);
        const bool keep = level < 2 || !rng_.chance(p_.drop_frac) || j == 0 || j + 1 == p_.cols ||
                          kind_[J(i, j)] == 2 || kind_[J(i + 1, j)] == 2;
        if (!keep) { w.close(); continue; }
        w.link(jn(i, j, kN), jn(i + 1, j, kS), i, nverts(level), bend());
      }
      w.close();
    }
  }

  void diagonals() {
    const uint32_t k = p_.diagonal_every;
    if (!k) return;
    int line = (int)(2 * (p_.rows + p_.cols));
    // diagonals j - i = d (south-west to north-east)
    for (int64_t d = -(int64_t)(p_.rows - 1) / k * k; d < (int64_t)p_.cols; d += k, ++line) {
      LineWalker w{*this, line, "secondary", 1, 0, "50", Way()};
      for (int64_t i = std::max<int64_t>(0, -d); i + 1 < (int64_t)p_.rows && i + d + 1 < (int64_t)p_.cols; ++i)
        w.link(jn(i, i + d, kAbove), jn(i + 1, i + d + 1, kBelow), (uint32_t)i, 2 + rng_.below(6), 0.5 * bend());
      w.close();
    }
    // anti-diagonals i + j = s (south-east to north-west)
    for (int64_t s = 0; s < (int64_t)(p_.rows + p_.cols - 1); s += k, ++line) {
      LineWalker w{*this, line, "secondary", 1, 0, "50", Way()};
      for (int64_t i = std::max<int64_t>(0, s - (int64_t)p_.cols + 1); i + 1 < (int64_t)p_.rows && s - i - 1 >= 0; ++i)
        w.link(jn(i, s - i, kAbove), jn(i + 1, s - i - 1, kBelow), (uint32_t)i, 2 + rng_.below(6), 0.5 * bend());
      w.close();
    }
  }

  // A trunk road on bridges across the city, west to east, with a vertex every ~90 m; it meets
  // the streets only at interchanges (a trunk_link ramp from a trunk vertex to the nearest plain
  // junction) every ~2.5 km and at both ends.
  void trunk() {
    const double y0 = 0.3 * H_, y1 = 0.7 * H_, amp = 0.03 * H_;
    const uint32_t nv = std::max<uint32_t>(4, (uint32_t)(W_ / 90.0));
    std::vector<uint32_t> verts;
    for (uint32_t k = 0; k <= nv; ++k) {
      const double t = (double)k / nv;
      verts.push_back(add_node(-0.02 * W_ + t * 1.04 * W_, y0 + t * (y1 - y0) + amp * std::sin(6.0 * t)));
    }
    auto ramp = [&](uint32_t tv) {
      // nearest plain junction (a junction node the streets share; none on a ring or a split)
      uint32_t best = kNone;
      double bd = 1e300;
      for (uint32_t q = 0; q < kind_.size(); ++q) {
        if (kind_[q] != 0) continue;
        const double d = std::hypot(jx_[q] - nodes_x_[tv], jy_[q] - nodes_y_[tv]);
        if (d < bd) { bd = d; best = q; }
      }
      if (best == kNone || bd < 20.0) return;
      Way r;
      r.hw = "trunk_link";
      r.level = 0;
      r.refs.push_back(tv);
      link_shape(tv, center_[best], 2, 0.1, r.refs);
      r.refs.push_back(center_[best]);
      ways_.push_back(r);
    };
    const uint32_t every = std::max<uint32_t>(2, (uint32_t)(2500.0 / (W_ * 1.04 / nv)));
    Way cur;
    auto flush = [&]() {
      if (cur.refs.size() >= 2) {
        cur.hw = "trunk"; cur.level = 0; cur.bridge = true; cur.maxspeed = "90";
        ways_.push_back(cur);
      }
      cur = Way();
    };
    for (uint32_t k = 0; k <= nv; ++k) {
      cur.refs.push_back(verts[k]);
      if (k == 0 || k == nv || k % every == 0) ramp(verts[k]);
      if (k && k < nv && k % 8 == 0) { flush(); cur.refs.push_back(verts[k]); }
    }
    flush();
  }

  void extras() {
    const uint32_t R = p_.rows, C = p_.cols;
    // dead-end spurs: from every hub and a fraction of plain junctions, into a block
    for (uint32_t i = 1; i + 1 < R; ++i)
      for (uint32_t j = 1; j + 1 < C; ++j) {
        const uint32_t q = J(i, j);
        if (kind_[q] != 0 || (on_diag(i, j) && !hub(i, j)) || !(hub(i, j) || rng_.chance(p_.spur_frac))) continue;
        const double a = (hub(i, j) ? 0.35 : 0.25 + 0.5 * rng_.below(4)) * kPi + 0.1 * rng_.uniform();
        const double L = 35.0 + 35.0 * rng_.uniform();
        const uint32_t e = add_node(jx_[q] + L * std::cos(a), jy_[q] + L * std::sin(a));
        Way w;
        w.hw = "residential";
        w.refs.push_back(center_[q]);
        link_shape(center_[q], e, rng_.below(3), 0.1, w.refs);
        w.refs.push_back(e);
        ways_.push_back(w);
      }
    // service loops off residential links (two roads between the same pair of street nodes),
    // footways and cycleways across blocks between the interior vertices of opposite links
    for (const auto& kv : link_interior_) {
      const std::vector<uint32_t>& in = kv.second;
      if (in.size() < 2 || kv.first.first >= (int)(R + C) || !rng_.chance(p_.service_frac)) continue;
      int level;
      const uint32_t li = kv.first.first < (int)R ? (uint32_t)kv.first.first : (uint32_t)kv.first.first - R;
      row_class(li, level);
      if (level != 2) continue;
      const uint32_t a = in.front(), b = in.back();
      const double dx = nodes_x_[b] - nodes_x_[a], dy = nodes_y_[b] - nodes_y_[a], l = std::hypot(dx, dy);
      if (l < 10.0) continue;
      const double off = rng_.chance(0.5) ? 25.0 : -25.0;
      Way w;
      w.hw = "service";
      if (rng_.chance(0.3)) w.access = "private";
      w.refs = {a, add_node(nodes_x_[a] - dy / l * off, nodes_y_[a] + dx / l * off),
                add_node(nodes_x_[b] - dy / l * off, nodes_y_[b] + dx / l * off), b};
      ways_.push_back(w);
    }
    for (uint32_t i = 0; i + 1 < R; ++i)
      for (uint32_t j = 0; j + 1 < C; ++j) {
        if (!rng_.chance(p_.footway_frac)) continue;
        auto s = link_interior_.find({(int)i, j}), n = link_interior_.find({(int)(i + 1), j});
        if (s == link_interior_.end() || n == link_interior_.end() || s->second.empty() || n->second.empty()) continue;
        if (boulevard_row(i) || boulevard_row(i + 1)) continue;
        const uint32_t a = s->second[s->second.size() / 2], b = n->second[n->second.size() / 2];
        Way w;
        w.hw = rng_.chance(0.25) ? "cycleway" : "footway";
        w.refs.push_back(a);
        link_shape(a, b, 1 + rng_.below(2), 0.15, w.refs);
        w.refs.push_back(b);
        ways_.push_back(w);
      }
  }

  // type=osmlr relations: classified roads always, residential ways with osmlr_local_frac;
  // never rings, ramps, service roads or paths.  A way and the next of its line (sharing its
  // last node) form one two-member segment when both qualify and their length allows.
  void relations() {
    const double tile_size[3] = {4.0, 1.0, 0.25};
    std::map<std::pair<int, uint32_t>, uint32_t> next_idx;
    auto seg_id = [&](int level, uint32_t node) {
      const double lat = p_.center_lat + (nodes_y_[node] - 0.5 * H_) / kMetersPerDegLat;
      const double lon = p_.center_lon + (nodes_x_[node] - 0.5 * W_) / mlon_;
      const double sz = tile_size[level];
      const uint32_t ncols = (uint32_t)std::llround(360.0 / sz);
      const uint32_t tile = (uint32_t)std::floor((lat + 90.0) / sz) * ncols + (uint32_t)std::floor((lon + 180.0) / sz);
      const uint32_t idx = next_idx[{level, tile}]++;
      return (uint64_t)level | ((uint64_t)tile << kLevelBits) | ((uint64_t)idx << (kLevelBits + kTileIndexBits));
    };
    std::vector<uint8_t> ok(ways_.size(), 0);
    for (size_t w = 0; w < ways_.size(); ++w) {
      const Way& wy = ways_[w];
      const bool cls = wy.hw == "trunk" || wy.hw == "primary" || wy.hw == "secondary" || wy.hw == "tertiary";
      ok[w] = !wy.roundabout && (cls || (wy.hw == "residential" && wy.line >= 0 && rng_.chance(p_.osmlr_local_frac)));
    }
    for (size_t w = 0; w < ways_.size(); ++w) {
      if (!ok[w]) continue;
      std::vector<uint32_t> grp{(uint32_t)w};
      if (w + 1 < ways_.size() && ok[w + 1] && ways_[w + 1].line == ways_[w].line && ways_[w].line >= 0 &&
          ways_[w + 1].refs.front() == ways_[w].refs.back() && ways_[w + 1].oneway == ways_[w].oneway &&
          ways_[w].len_m + ways_[w + 1].len_m < 1000.0 && rng_.chance(0.4)) {
        grp.push_back((uint32_t)w + 1);
        ok[w + 1] = 0;
      }
      const Way& f = ways_[grp.front()];
      const Way& l = ways_[grp.back()];
      if (f.oneway >= 0) {
        Rel r{seg_id(f.level, f.refs.front()), {}};
        for (uint32_t g : grp) r.members.push_back({g, false});
        rels_.push_back(r);
      }
      if (f.oneway <= 0) {
        Rel r{seg_id(f.level, l.refs.back()), {}};
        for (size_t k = grp.size(); k-- > 0;) r.members.push_back({grp[k], true});
        rels_.push_back(r);
      }
    }
  }

  std::vector<uint64_t> shuffled_ids(size_t n, size_t chunk, uint64_t base) {
    const size_t nch = (n + chunk - 1) / chunk;
    std::vector<size_t> perm(nch);
    std::iota(perm.begin(), perm.end(), (size_t)0);
    for (size_t k = nch; k > 1; --k) std::swap(perm[k - 1], perm[rng_.below((uint32_t)k)]);
    std::vector<uint64_t> id(n);
    uint64_t next = base;
    for (size_t c : perm)
      for (size_t i = c * chunk; i < std::min(n, (c + 1) * chunk); ++i) {
        next += 1 + (rng_.chance(0.1) ? rng_.below(5) : 0);
        id[i] = next;
      }
    return id;
  }
};

}  // namespace

void write_osm_city(const CityParams& p, OsmSink& sink) {
  City c(p);
  c.build();
  c.emit(sink);
}

}  // namespace rm
