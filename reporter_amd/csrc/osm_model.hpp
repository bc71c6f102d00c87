// osm_model.hpp — the OSM element stream and parsed model shared by the XML (graph_osm.cpp) and
// PBF (osm_pbf.cpp) encodings of the engine's graph.
#pragma once
#include <cstdint>
#include <map>
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

}  // namespace rm
