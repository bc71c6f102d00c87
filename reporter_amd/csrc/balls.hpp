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
// replaced by two table probes per target entry node.  Built once per graph and mode
// (the engine's graph-load step); the tables live in HBM next to the graph.
#pragma once
#include <cstdint>
#include <vector>

#include "graph.hpp"

namespace rm {

struct BallTables {
  std::vector<uint32_t> hdr;   // 2 per node: first entry, log2(table size) (0: no table, node's ball too big)
  std::vector<uint32_t> ent;   // 4 per entry: node (kEmpty when free), dist cm, time ms, 0
  uint32_t radius_cm = 0;
  uint64_t n_keys = 0;         // (node, node) keys stored
  uint32_t n_skipped = 0;      // nodes whose ball exceeded max_keys (their searches use the search tiers)
  double build_ms = 0;
};

// Balls of `mode` with radius `radius_cm` (keys with distance <= radius are kept),
// tables sized to the next power of two >= 2 x keys; nodes with more than `max_keys`
// keys get no table.  `threads` host threads.
constexpr uint32_t kBallMaxKeysHost = 4096;   // keys per node above which a node gets no table

void build_balls(const Graph& g, int mode, uint32_t radius_cm, uint32_t max_keys, int threads, BallTables& out);

}  // namespace rm
