// balls.hpp — per-node route balls: exact lexicographic (distance cm, time ms) shortest
// keys from every node to every node within a radius, per travel mode, stored as one
// small open-addressed table per node.
//
// Why: K2 (transition costs) answers, for every pair of consecutive states, "shortest
// route from each candidate of A to each candidate of B within `bound`" (meili's
// bounded one-to-many Dijkstra; reference call site simple_reporter.py:166 ->
// valhalla::meili::MapMatcher).  With labels keyed by exact u64 (dist, time) sums, a
// multi-root bounded search from the two exits of a source candidate equals
//     label(v) = min over exits x of  rk_x + key(x -> v)
// for every v whose key has distance <= bound, so when bound <= radius the search is
// replaced by table probes.  A node's table is keyed by ROAD: the row of road r holds the
// keys to both of r's endpoints, so one 16-byte probe per (exit, target candidate) gives
// both entry labels the target's route combinations need.  Built once per graph and mode
// (the engine's graph-load step); the tables live in HBM next to the graph.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "graph.hpp"

namespace rm {

struct BallTables {
  std::vector<uint32_t> hdr;   // 2 per node: first entry, log2(table size) (0: no table, node's ball too big)
  std::vector<uint32_t> ent;   // 4 per row: road (kNone when free) and the keys to the road's node0 / node1
                               // (24-bit cm distances and ms times, rm_common.hpp ball_pack)
  uint32_t radius_cm = 0;
  uint64_t n_keys = 0;         // (node, road) rows stored
  uint32_t n_skipped = 0;      // nodes whose ball exceeded max_keys (their searches use the search tiers)
  uint32_t road_mask = ~0u;    // road-id bits of a row's first word (rm_common.hpp ball_road_mask)
  double build_ms = 0;
};

// Balls of `mode` with radius `radius_cm` (keys with distance <= radius are kept),
// tables sized to the next power of two >= 2 x keys; nodes with more than `max_keys`
// keys, or a key beyond the row's 24-bit fields, get no table.  `threads` host threads.
constexpr uint32_t kBallMaxKeysHost = 4096;   // ball nodes above which a node gets no table
constexpr uint32_t kBallMaxRadiusCm = 1000000;   // 10 km knob cap (rows hold 24-bit distances)

// Tables that would exceed kBallMaxRows (rm_common.hpp) or the memory granted to them: the
// caller steps the radius down instead of failing.
struct BallsTooLarge : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Default radius for a graph: the largest of {2000 (meili's default breakage distance, so
// every default-bounded transition is a table probe), 1500, 1000, 700, 500} m whose tables
// (sampled: sample_balls, +10 %) stay within `budget_bytes` per mode and whose balls mostly
// fit kBallMaxKeysHost; 400 m when none does.
constexpr uint64_t kBallAutoBudget = 72ull << 30;   // per mode; C4: 1000 m (68 GB built)
// budget 0: ball_mode_budget() (kBallAutoBudget, or RM_BALL_BUDGET_GB when set)
uint32_t auto_ball_radius_cm(const Graph& g, uint64_t budget_bytes = 0);
uint64_t ball_mode_budget();
// bytes all modes' tables together may take on a device with `hbm_total` bytes: half of it
// (the other half holds the graph and the batch workspaces: ~0.75 KB per point), or
// RM_BALL_TOTAL_GB when set
uint64_t ball_total_budget(uint64_t hbm_total);

// Radii (cm) the per-mode choice steps down through, largest first.
constexpr uint32_t kBallRadii[] = {200000u, 150000u, 100000u, 70000u, 50000u, 40000u, 30000u, 20000u};
// The radius a mode's tables are built at: the largest of kBallRadii at or below start_cm
// (start_cm itself first when it is not on the ladder) whose sampled tables for THIS mode
// (+10 %) fit both `avail_bytes` and kBallMaxRows, and whose balls mostly fit
// kBallMaxKeysHost; 0 when none does (the mode's transitions use the search tiers).
uint32_t fit_ball_radius_cm(const Graph& g, int mode, uint32_t start_cm, uint64_t avail_bytes,
                            struct BallSample* sample = nullptr);
// next radius below r_cm on the ladder (0 when none)
uint32_t next_ball_radius_cm(uint32_t r_cm);
// Travel modes whose tables are identical (same access mask and routing speeds: auto and
// bus) share one build: the mode whose tables `mode` can reuse, or -1.
int ball_twin_mode(int mode);

// throws BallsTooLarge (before allocating the rows) when the tables need more than max_rows rows
void build_balls(const Graph& g, int mode, uint32_t radius_cm, uint32_t max_keys, int threads, BallTables& out,
                 uint64_t max_rows = kBallMaxRows);

// node -> incident roads CSR (every road listed at node0 and at node1)
void road_incidence(const Graph& g, std::vector<uint32_t>& inc_off, std::vector<uint32_t>& inc);

// sampled ball statistics at a radius (exact bounded searches of `mode` from 256 nodes)
struct BallSample {
  double nodes = 0;          // mean nodes per ball
  double table_bytes = 0;    // estimated bytes of all nodes' power-of-two tables
  double skipped_frac = 0;   // sampled balls above max_keys (no table)
};
BallSample sample_balls(const Graph& g, uint32_t radius_cm, uint32_t max_keys, int mode = 0);
// nodes an average ball of radius_cm holds (sampled); the engine builds small balls on the GPU
double est_ball_nodes(const Graph& g, uint32_t radius_cm);

}  // namespace rm
