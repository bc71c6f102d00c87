// graph.hpp — host-side road graph: CSR of directed edges tagged with OSMLR
// segment ids, road shapes, and a uniform spatial grid index.
//
// This is the engine's replacement for the Valhalla tile/graph layer the
// reference reads through meili (tile hierarchy: reference py/get_tiles.py:30-39;
// segment-id bit layout: py/simple_reporter.py:37-49).  The same arrays are
// written to a flat binary file (".rmg") that the GPU runtime uploads to HBM
// and that oracle/ reads as plain arrays.
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>
#include "rm_common.hpp"

namespace rm {

struct GridIndex {
  double lon0 = 0, lat0 = 0, dlon = 1, dlat = 1;  // origin + cell size (degrees)
  uint32_t ncx = 1, ncy = 1;
  std::vector<uint32_t> cell_off;   // ncx*ncy + 1
  std::vector<uint32_t> cell_item;  // vertex index of a shape segment's first vertex
};

struct Graph {
  // nodes
  std::vector<float> node_lon, node_lat;
  std::vector<uint32_t> node_off;       // CSR offsets, size N+1
  // directed edges (CSR order)
  std::vector<EdgeRec> edges;
  std::vector<uint32_t> edge_seg;       // dense OSMLR segment index or kNone
  std::vector<uint32_t> edge_seg_off;   // cm from the segment's start to this edge's start
  std::vector<uint32_t> edge_way;       // way id
  // roads (undirected shape owners)
  std::vector<uint32_t> road_node0, road_node1, road_fwd, road_rev, road_len_cm, road_vert_off;
  // shape vertices
  std::vector<VertRec> verts;
  // OSMLR segments
  std::vector<uint64_t> seg_id;
  std::vector<uint32_t> seg_len_cm;
  GridIndex grid;

  uint32_t num_nodes() const { return (uint32_t)node_lon.size(); }
  uint32_t num_edges() const { return (uint32_t)edges.size(); }
  uint32_t num_roads() const { return (uint32_t)road_len_cm.size(); }
  uint32_t num_verts() const { return (uint32_t)verts.size(); }
  uint32_t num_segments() const { return (uint32_t)seg_id.size(); }

  void save(const std::string& path) const;     // throws std::runtime_error
  static Graph load(const std::string& path);   // throws std::runtime_error
  void validate() const;                        // throws on a malformed graph
};

struct WorldParams {
  uint32_t rows = 40, cols = 40;
  double block_m = 100.0;
  uint64_t seed = 1;
  double center_lat = 47.0, center_lon = 8.0;
  double jitter = 0.15;            // node jitter, fraction of a block
  uint32_t arterial_every = 10;    // every 10th line is level 1
  uint32_t highway_every = 40;     // every 40th line is level 0
  double segment_max_m = 1000.0;   // OSMLR segments are chained up to this length
  double internal_m = 15.0;        // internal edge length at major intersections
  double service_frac = 0.05;      // local edges without OSMLR association
  double oneway_frac = 0.10;       // local roads that are one-way for vehicles
  double curve_frac = 0.30;        // roads given a curved mid vertex
  double cell_m = 100.0;           // grid-index cell size
};

Graph build_world(const WorldParams& p);

// Graph assembly shared by the world builder and the OSM importer (graph_osm.cpp).
// A road: its two graph nodes, its shape (lon, lat incl. both endpoints), the info words
// and way ids of its forward (n0 -> n1) and reverse directed edges.
struct RoadInput {
  uint32_t n0, n1;
  std::vector<std::pair<float, float>> shape;
  uint32_t info_fwd, info_rev, way_fwd, way_rev;
};
// shape vertices (cumulative cm), road lengths, CSR of directed edges (stable by source
// node, forward before reverse per road), road -> edge maps; node arrays must be set.
// edge_seg / edge_seg_off are reset to "no OSMLR segment".
void assemble_roads(Graph& g, const std::vector<RoadInput>& roads);
// cell_off / cell_item of g.grid from its origin, cell size and dimensions
void build_grid_index(Graph& g);
// (re)build the cell -> shape piece CSR of `gi` (origin, cell size and extent already set):
// every piece is listed in each cell its lon/lat bounding box overlaps
void build_grid_index(const std::vector<VertRec>& verts, GridIndex& gi);
// length of a straight shape piece, metres (equirectangular at its mean latitude)
double piece_m(float lon0, float lat0, float lon1, float lat1);

// OpenStreetMap exchange of a graph (graph_osm.cpp).  export_osm writes OSM XML (".osm")
// whose ways, tags and relations carry everything an .rmg holds; import_osm reads it back
// bit-identically, or builds a graph from a generic OSM XML file (intersections split ways,
// highway / maxspeed / oneway / access tags give speeds and access, no OSMLR segments
// unless osmlr relations are present; cell_m sizes the grid index then).
void export_osm(const Graph& g, const std::string& path);
// the same elements as OSM PBF (osm_pbf.cpp: zlib blobs, dense nodes, nanodegree granularity)
void export_osm_pbf(const Graph& g, const std::string& path);
// XML or PBF, told apart by content
Graph import_osm(const std::string& path, double cell_m = 100.0);

// Synthetic GPS traces (restating reference py/generate_test_trace.py:35-104,120-164):
// fastest routes (A* on travel time) to random destinations, driven at edge speed and
// resampled every `rate_s` seconds, with the generator's correlated noise
// (first-quadrant lock + moving average).
struct TraceParams {
  uint32_t n_traces = 1, n_points = 100;
  double rate_s = 1.0;
  double noise_m = 5.0;
  uint64_t seed = 1;
  int32_t mode = kModeAuto;
  int64_t start_epoch = 1483228800;  // fixed (replaces time.time()-86400 at line 60)
  uint32_t threads = 0;              // 0 = hardware concurrency
};

struct TraceSet {
  std::vector<double> lon, lat, time;   // 6-dp rounded degrees, epoch seconds
  std::vector<float> accuracy;          // per point (generate_test_trace.py:40)
  std::vector<uint32_t> trace_off;      // n_traces + 1
  std::vector<uint32_t> truth_edge;     // directed edge under the true position
  std::vector<uint32_t> truth_off_cm;   // offset along that edge
};

// p.n_traces traces; with ids, slot k holds trace ids[k] of the seeded set (the same trace
// the full set has at index ids[k]): a rank generates exactly its uuid shard
TraceSet generate_traces(const Graph& g, const TraceParams& p, const uint32_t* ids = nullptr);

}  // namespace rm
