// osm_model.hpp — the OSM element stream and parsed model shared by the XML (graph_osm.cpp) and
// PBF (osm_pbf.cpp) encodings of the engine's graph.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "graph.hpp"

namespace rm {

using OsmTags = std::vector<std::pair<std::string, std::string>>;   // in emission order

struct OsmMember {
  std::string type, role;   // type: "node" | "way" | "relation"
  uint64_t ref;
};

// Receives a graph's OSM elements in file order: bounds, nodes (ascending id), ways, relations.
class OsmSink {
 public:
  virtual ~OsmSink() = default;
  virtual void bounds(float minlat, float minlon, float maxlat, float maxlon) = 0;
  virtual void node(uint64_t id, float lat, float lon) = 0;
  virtual void way(uint64_t id, const std::vector<uint64_t>& refs, const OsmTags& tags) = 0;
  virtual void relation(uint64_t id, const std::vector<OsmMember>& members, const OsmTags& tags) = 0;
  virtual void finish() = 0;
};

// a graph's OSM elements (graph_osm.cpp); the generator string names the exact-round-trip format
extern const char* const kOsmGenerator;
void emit_osm(const Graph& g, OsmSink& sink);

// What a reader hands the importer (either encoding).
struct OsmParsedWay {
  uint64_t id;
  std::vector<uint64_t> refs;
  std::map<std::string, std::string> tags;
};
struct OsmParsedRelation {
  uint64_t id;
  std::vector<OsmMember> members;
  std::map<std::string, std::string> tags;
};
struct OsmParsed {
  std::vector<std::pair<uint64_t, std::pair<float, float>>> nodes;   // id -> (lon, lat) as float
  std::vector<OsmParsedWay> ways;
  std::vector<OsmParsedRelation> rels;
};

OsmParsed parse_osm_xml(const std::string& path);
OsmParsed parse_osm_pbf(const std::string& path);
Graph graph_from_osm(OsmParsed& osm, double cell_m);

// writers of either encoding (graph_osm.cpp, osm_pbf.cpp)
std::unique_ptr<OsmSink> make_osm_xml_sink(const std::string& path);
std::unique_ptr<OsmSink> make_osm_pbf_sink(const std::string& path);

// A seeded irregular city as generic OSM (osm_city.cpp): a jittered junction lattice whose
// streets are curved multi-vertex ways, diagonal avenues meeting at 9-road hubs, roundabouts,
// boulevards of one-way carriageway pairs, one-way streets, dead ends, service loops, paths, a
// bridged trunk road with ramps, OSMLR relations on part of the ways only.  No reporter:* tags.
struct CityParams {
  uint32_t rows = 40, cols = 40;    // junction lattice
  double block_m = 120.0;
  uint64_t seed = 1;
  double center_lat = 47.0, center_lon = 8.0;
  double jitter = 0.25;             // junction jitter, fraction of a block
  uint32_t primary_every = 8, secondary_every = 4, boulevard_every = 12;
  uint32_t diagonal_every = 10;     // even: diagonals cross each other only at junctions
  double roundabout_frac = 0.05, drop_frac = 0.06, oneway_frac = 0.15;
  double spur_frac = 0.05, service_frac = 0.05, footway_frac = 0.05;
  double osmlr_local_frac = 0.3;    // residential ways with OSMLR segments
  double way_max_m = 700.0;         // a street's OSM ways end at a junction past this length
  uint32_t trunk = 1;               // the bridged trunk road
};
void write_osm_city(const CityParams& p, OsmSink& sink);

}  // namespace rm
