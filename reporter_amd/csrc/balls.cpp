// balls.cpp — host build of the per-node route balls (see balls.hpp).
//
// One Dijkstra per node over the mode's directed edges, keys (dist cm, time ms) packed in
// a u64 exactly as the matcher's searches add them (rm_common.hpp make_key), pruned at
// distance > radius; the settled nodes are then folded into one row per incident road.
// Two passes over the nodes (count, then fill) so the tables are laid out contiguously
// without holding every ball in memory at once.
#include "balls.hpp"

#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstdlib>
#include <functional>
#include <queue>
#include <unordered_map>
#include <unordered_set>
#include <stdexcept>
#include <thread>
#include <utility>

namespace rm {
namespace {

struct EdgeKey {
  uint32_t target;
  uint64_t key;   // kKeyInf when the mode cannot use the edge
};

// per-thread Dijkstra scratch: dense labels, touched list for O(ball) reset
struct Scratch {
  std::vector<uint64_t> lab;
  std::vector<uint32_t> touched;
  std::vector<std::pair<uint32_t, uint64_t>> out;  // settled (node, key)
  using Item = std::pair<uint64_t, uint32_t>;
  std::priority_queue<Item, std::vector<Item>, std::greater<Item>> pq;
  explicit Scratch(uint32_t n) : lab(n, kKeyInf) {}

  // settled keys of the ball of u; false when it holds more than max_keys nodes
  bool run(const Graph& g, const std::vector<EdgeKey>& ek, uint32_t u, uint32_t radius, uint32_t max_keys) {
    for (uint32_t v : touched) lab[v] = kKeyInf;
    touched.clear();
    out.clear();
    while (!pq.empty()) pq.pop();
    lab[u] = 0;
    touched.push_back(u);
    pq.push({0ull, u});
    bool ok = true;
    while (!pq.empty()) {
      const Item it = pq.top();
      pq.pop();
      if (it.first != lab[it.second]) continue;   // stale entry
      out.push_back({it.second, it.first});
      if (out.size() > max_keys) { ok = false; break; }
      for (uint32_t e = g.node_off[it.second]; e < g.node_off[it.second + 1]; ++e) {
        if (ek[e].key == kKeyInf) continue;
        const uint64_t nk = it.first + ek[e].key;
        if (key_dist(nk) > radius) continue;
        const uint32_t v = ek[e].target;
        if (nk < lab[v]) {
          if (lab[v] == kKeyInf) touched.push_back(v);
          lab[v] = nk;
          pq.push({nk, v});
        }
      }
    }
    return ok;
  }
};

// in-edges of every node in edge-id order (the engine's in_rec order) and each edge's source
struct InEdges {
  std::vector<uint32_t> off, edge, src;
  explicit InEdges(const Graph& g) {
    const uint32_t N = g.num_nodes(), E = g.num_edges();
    off.assign(N + 1, 0);
    edge.resize(E);
    src.resize(E);
    for (uint32_t u = 0; u < N; ++u)
      for (uint32_t e = g.node_off[u]; e < g.node_off[u + 1]; ++e) src[e] = u;
    for (uint32_t e = 0; e < E; ++e) off[g.edges[e].target + 1]++;
    for (uint32_t n = 0; n < N; ++n) off[n + 1] += off[n];
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    for (uint32_t e = 0; e < E; ++e) edge[fill[g.edges[e].target]++] = e;
  }
};

// canonical predecessor of settled node v (key kv) in the search from root (rm_common.hpp
// kBallRoadBits): index among v's in-edges of the first usable tight one, kBallPredNone when
// v is the root or the index is 7 or more
uint32_t pred_index(const InEdges& ie, const std::vector<EdgeKey>& ek, const std::vector<uint64_t>& lab,
                    uint32_t root, uint32_t v, uint64_t kv) {
  if (v == root) return kBallPredNone;
  for (uint32_t q = ie.off[v], i = 0; q < ie.off[v + 1] && i < kBallPredNone; ++q, ++i) {
    const uint32_t e = ie.edge[q];
    if (ek[e].key == kKeyInf) continue;
    const uint64_t lu = lab[ie.src[e]];
    if (lu != kKeyInf && lu + ek[e].key == kv) return i;
  }
  return kBallPredNone;
}

// roads touched by a ball: every road with an endpoint in it, with the keys of both
// endpoints (kKeyInf for an endpoint outside the ball) and their predecessor indices
struct RoadAcc {
  std::vector<uint32_t> pos;      // road -> index in rows (kNone when untouched)
  std::vector<uint32_t> roads;
  std::vector<uint64_t> k0, k1;
  std::vector<uint8_t> p0, p1;
  explicit RoadAcc(uint32_t n_roads) : pos(n_roads, kNone) {}
  // pred(i): predecessor index of settled[i] (only called when `with_pred`)
  template <class Pred>
  void collect(const Graph& g, const std::vector<uint32_t>& inc_off, const std::vector<uint32_t>& inc,
               const std::vector<std::pair<uint32_t, uint64_t>>& settled, bool with_pred, Pred&& pred) {
    for (uint32_t r : roads) pos[r] = kNone;
    roads.clear(); k0.clear(); k1.clear(); p0.clear(); p1.clear();
    for (size_t i = 0; i < settled.size(); ++i) {
      const auto& kv = settled[i];
      const uint8_t pv = with_pred ? (uint8_t)pred(i) : (uint8_t)kBallPredNone;
      for (uint32_t q = inc_off[kv.first]; q < inc_off[kv.first + 1]; ++q) {
        const uint32_t r = inc[q];
        if (pos[r] == kNone) {
          pos[r] = (uint32_t)roads.size(); roads.push_back(r); k0.push_back(kKeyInf); k1.push_back(kKeyInf);
          p0.push_back((uint8_t)kBallPredNone); p1.push_back((uint8_t)kBallPredNone);
        }
        if (g.road_node0[r] == kv.first) { k0[pos[r]] = kv.second; p0[pos[r]] = pv; }
        if (g.road_node1[r] == kv.first) { k1[pos[r]] = kv.second; p1[pos[r]] = pv; }
      }
    }
  }
  void collect(const Graph& g, const std::vector<uint32_t>& inc_off, const std::vector<uint32_t>& inc,
               const std::vector<std::pair<uint32_t, uint64_t>>& settled) {
    collect(g, inc_off, inc, settled, false, [](size_t) { return kBallPredNone; });
  }
};

uint32_t table_bits(uint64_t keys) {
  uint32_t bits = 1;
  while ((1ull << bits) < kBallSlotsPerRow * keys) ++bits;
  return bits;
}

template <class F>
void parallel_nodes(uint32_t n, int threads, F&& f) {
  threads = std::max(1, std::min<int>(threads, (int)((n + 1023) / 1024)));
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      for (uint32_t u = (uint32_t)t; u < n; u += (uint32_t)threads) f(t, u);
    });
  for (auto& th : pool) th.join();
}

}  // namespace


// Ball size by sampling: the bounded search (auto mode) from 256 nodes spread over the node
// ids, with sparse labels (no per-graph arrays: cheap on a 16.6 M-node graph).  Rows are the
// roads of the settled nodes' out-edges (a one-way road entering the ball from outside is the
// only row it misses).  A density-times-disc estimate overshoots route-distance balls (a grid's
// network ball is a diamond) and power-of-two tables amplify that: it put C4's 1000 m tables
// at 136 GB (they are 68 GB) and picked 700 m.
struct BallSampler {
  const Graph& g;
  int mode;
  BallSampler(const Graph& gr, int m) : g(gr), mode(m) {}
  BallSample at(uint32_t radius_cm, uint32_t max_keys) const {
    BallSample out;
    const uint32_t N = g.num_nodes();
    const uint32_t S = std::min<uint32_t>(N, 256u);
    const uint32_t acc = mode_access(mode);
    double nodes = 0, slots = 0;
    uint32_t skipped = 0;
    std::unordered_map<uint32_t, uint64_t> lab;
    std::unordered_set<uint32_t> roads;
    using Item = std::pair<uint64_t, uint32_t>;
    for (uint32_t i = 0; i < S; ++i) {
      const uint32_t u = (uint32_t)(((uint64_t)i * N) / S);
      lab.clear();
      roads.clear();
      std::priority_queue<Item, std::vector<Item>, std::greater<Item>> pq;
      lab[u] = 0;
      pq.push({0ull, u});
      uint32_t settled = 0;
      bool ok = true;
      while (!pq.empty()) {
        const Item it = pq.top();
        pq.pop();
        if (it.first != lab[it.second]) continue;
        if (++settled > max_keys) { ok = false; break; }
        for (uint32_t e = g.node_off[it.second]; e < g.node_off[it.second + 1]; ++e) {
          const EdgeRec& r = g.edges[e];
          roads.insert(r.road >> 1);
          if (!(edge_access(r.info) & acc)) continue;
          const uint64_t nk = it.first + make_key(r.len_cm, time_ms(r.len_cm, mode_speed_dkph(mode, edge_speed_dkph(r.info))));
          if (key_dist(nk) > radius_cm) continue;
          auto f = lab.find(r.target);
          if (f == lab.end() || nk < f->second) {
            lab[r.target] = nk;
            pq.push({nk, r.target});
          }
        }
      }
      if (!ok) { ++skipped; nodes += max_keys; continue; }
      nodes += settled;
      slots += (double)(1ull << table_bits(std::max<size_t>(1, roads.size())));
    }
    out.nodes = S ? nodes / S : 0.0;
    out.table_bytes = S ? slots / S * (double)N * 16.0 : 0.0;
    out.skipped_frac = S ? (double)skipped / S : 0.0;
    return out;
  }
};

BallSample sample_balls(const Graph& g, uint32_t radius_cm, uint32_t max_keys, int mode) {
  if (g.num_nodes() == 0) return BallSample{};
  BallSampler bs(g, mode);
  return bs.at(radius_cm, max_keys);
}

namespace {
// sampled tables of one mode fit `avail` bytes (+10 %) and the row cap, and most balls fit
bool sample_fits(const BallSample& bs, uint64_t avail_bytes) {
  const double bytes = bs.table_bytes * 1.1;
  return bs.skipped_frac <= 0.05 && bytes <= (double)avail_bytes && bytes <= (double)kBallMaxRows * 16.0;
}
double env_gb(const char* name) {
  const char* s = std::getenv(name);
  return s ? std::atof(s) : 0.0;
}
}  // namespace

uint64_t ball_mode_budget() {
  const double gb = env_gb("RM_BALL_BUDGET_GB");
  return gb > 0.0 ? (uint64_t)(gb * (double)(1ull << 30)) : kBallAutoBudget;
}

uint64_t ball_total_budget(uint64_t hbm_total) {
  const double gb = env_gb("RM_BALL_TOTAL_GB");
  return gb > 0.0 ? (uint64_t)(gb * (double)(1ull << 30)) : hbm_total / 2;
}

uint32_t next_ball_radius_cm(uint32_t r_cm) {
  for (const uint32_t r : kBallRadii)
    if (r < r_cm) return r;
  return 0u;
}

uint32_t fit_ball_radius_cm(const Graph& g, int mode, uint32_t start_cm, uint64_t avail_bytes, BallSample* sample) {
  if (g.num_nodes() < 2 || start_cm == 0) return start_cm;
  BallSampler sampler(g, mode);
  for (uint32_t r = start_cm; r; r = next_ball_radius_cm(r)) {
    const BallSample bs = sampler.at(r, kBallMaxKeysHost);
    if (!sample_fits(bs, avail_bytes)) continue;
    if (sample) *sample = bs;
    return r;
  }
  return 0u;
}

int ball_twin_mode(int mode) {
  // bus routes exactly as auto: same access bit, no speed cap (rm_common.hpp mode_speed_dkph)
  if (mode == kModeBus) return kModeAuto;
  if (mode == kModeAuto) return kModeBus;
  return -1;
}

double est_ball_nodes(const Graph& g, uint32_t radius_cm) {
  if (g.num_nodes() < 2) return (double)g.num_nodes();
  return sample_balls(g, radius_cm, kBallMaxKeysHost).nodes;
}

void road_incidence(const Graph& g, std::vector<uint32_t>& inc_off, std::vector<uint32_t>& inc) {
  const uint32_t N = g.num_nodes(), R = g.num_roads();
  inc_off.assign(N + 1, 0);
  for (uint32_t r = 0; r < R; ++r) {
    inc_off[g.road_node0[r] + 1]++;
    if (g.road_node1[r] != g.road_node0[r]) inc_off[g.road_node1[r] + 1]++;
  }
  for (uint32_t n = 0; n < N; ++n) inc_off[n + 1] += inc_off[n];
  inc.resize(inc_off[N]);
  std::vector<uint32_t> fill(inc_off.begin(), inc_off.end() - 1);
  for (uint32_t r = 0; r < R; ++r) {
    inc[fill[g.road_node0[r]]++] = r;
    if (g.road_node1[r] != g.road_node0[r]) inc[fill[g.road_node1[r]]++] = r;
  }
}

uint32_t auto_ball_radius_cm(const Graph& g, uint64_t budget_bytes) {
  if (budget_bytes == 0) budget_bytes = ball_mode_budget();
  const uint32_t N = g.num_nodes();
  if (N < 2) return 40000u;
  BallSampler sampler(g, kModeAuto);
  for (const uint32_t r : {200000u, 150000u, 100000u, 70000u, 50000u})
    if (sample_fits(sampler.at(r, kBallMaxKeysHost), budget_bytes)) return r;
  return 40000u;
}

void build_balls(const Graph& g, int mode, uint32_t radius_cm, uint32_t max_keys, int threads, BallTables& out,
                 uint64_t max_rows) {
  const auto t0 = std::chrono::steady_clock::now();
  const uint32_t N = g.num_nodes(), E = g.num_edges();
  const uint32_t acc = mode_access(mode);
  std::vector<EdgeKey> ek(E);
  for (uint32_t e = 0; e < E; ++e) {
    const EdgeRec& r = g.edges[e];
    const bool ok = (edge_access(r.info) & acc) != 0u;
    ek[e] = {r.target, ok ? make_key(r.len_cm, time_ms(r.len_cm, mode_speed_dkph(mode, edge_speed_dkph(r.info)))) : kKeyInf};
  }
  if (radius_cm > kBallMaxRadiusCm) throw std::runtime_error("ball radius above 10 km");
  // node -> incident roads
  const uint32_t R = g.num_roads();
  std::vector<uint32_t> inc_off, inc;
  road_incidence(g, inc_off, inc);
  threads = std::max(1, threads);
  std::vector<Scratch> scr;
  std::vector<RoadAcc> acc_r;
  scr.reserve(threads);
  acc_r.reserve(threads);
  for (int t = 0; t < threads; ++t) { scr.emplace_back(N); acc_r.emplace_back(R); }
  // pass 1: table size per node
  std::vector<uint32_t> bits(N, 0);
  parallel_nodes(N, threads, [&](int t, uint32_t u) {
    if (!scr[t].run(g, ek, u, radius_cm, max_keys)) { bits[u] = 0; return; }
    for (const auto& kv : scr[t].out)
      if (!ball_key_fits(kv.second)) { bits[u] = 0; return; }
    acc_r[t].collect(g, inc_off, inc, scr[t].out);
    bits[u] = acc_r[t].roads.size() > 2 * (size_t)max_keys ? 0u : table_bits(acc_r[t].roads.size());
  });
  out.hdr.assign(2 * (size_t)N, 0);
  uint64_t total = 0;
  out.n_skipped = 0;
  for (uint32_t u = 0; u < N; ++u) {
    out.hdr[2 * (size_t)u] = (uint32_t)(total >> 1);   // first row / 2 (rm_common.hpp ball_row0)
    out.hdr[2 * (size_t)u + 1] = bits[u];
    if (bits[u]) total += 1ull << bits[u];
    else out.n_skipped++;
    if (total > std::min(kBallMaxRows, max_rows)) throw BallsTooLarge("route balls too large for their budget; lower the radius");
  }
  out.ent.assign(4 * total, 0);
  for (uint64_t i = 0; i < total; ++i) out.ent[4 * i] = kNone;
  // pass 2: fill (tables are disjoint, so threads write without locks); rows carry the
  // endpoints' canonical predecessors when the road ids leave room (rm_common.hpp)
  const uint32_t rmask = ball_road_mask(R);
  const bool with_pred = rmask != ~0u;
  InEdges ie(g);
  std::vector<uint64_t> keys(threads, 0);
  parallel_nodes(N, threads, [&](int t, uint32_t u) {
    if (!bits[u]) return;
    Scratch& sc = scr[t];
    sc.run(g, ek, u, radius_cm, max_keys);
    RoadAcc& ra = acc_r[t];
    ra.collect(g, inc_off, inc, sc.out, with_pred,
               [&](size_t i) { return pred_index(ie, ek, sc.lab, u, sc.out[i].first, sc.out[i].second); });
    const uint32_t b = bits[u], mask = (1u << b) - 1u;
    uint32_t* tab = out.ent.data() + 4 * ball_row0(out.hdr[2 * (size_t)u]);
    for (size_t q = 0; q < ra.roads.size(); ++q) {
      uint32_t s = ball_slot(ra.roads[q], b);
      while (tab[4 * s] != kNone) s = (s + 1) & mask;
      tab[4 * s] = ball_road_word(ra.roads[q], ra.p0[q], ra.p1[q], rmask);
      ball_pack(ra.k0[q], ra.k1[q], tab[4 * s + 1], tab[4 * s + 2], tab[4 * s + 3]);
    }
    keys[t] += ra.roads.size();
  });
  out.road_mask = rmask;
  out.n_keys = 0;
  for (uint64_t k : keys) out.n_keys += k;
  out.radius_cm = radius_cm;
  out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace rm
