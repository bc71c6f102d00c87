// graph_osm.cpp — OpenStreetMap exchange of the engine's road graph.
//
// The reference matches on Valhalla tiles that valhalla_build_tiles makes from an OSM
// extract (Dockerfile:42-49, README.md:129-130), and reads its tile hierarchy / OSMLR ids as
// get_tiles.py:30-102 and simple_reporter.py:36-49 describe.  No tile builder runs offline, so
// the engine's graph is its own .rmg; this file makes that graph expressible as OSM and back,
// in both encodings the tile builder reads (XML here, PBF in osm_pbf.cpp):
//
//   emit_osm     .rmg -> OSM elements, streamed to a sink (XML or PBF writer): graph nodes
//                (id = index + 1), interior shape vertices (id = N + 1 + vertex index), one way
//                per road carrying the usual routing tags (highway, maxspeed, oneway, access)
//                plus exact reporter:* tags, one type=osmlr relation per OSMLR segment (its
//                directed edges as forward / backward way members, id and length tags) and a
//                type=reporter_grid relation holding the spatial index geometry.
//   graph_from_osm  parsed OSM (either encoding) -> .rmg.  A file written by export_osm /
//                export_osm_pbf comes back bit-identical.  Any other OSM is ingested the way a
//                router does it: highway ways are split at intersections (nodes shared by ways
//                or way ends), speeds from maxspeed or the highway class, access from oneway /
//                access tags; OSMLR segments only where osmlr relations name them (a member way
//                that was split contributes all of its roads, in order).
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "graph.hpp"
#include "osm_model.hpp"

namespace rm {

namespace {


std::string xml_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    switch (c) {
      case '&': o += "&amp;"; break;
      case '<': o += "&lt;"; break;
      case '>': o += "&gt;"; break;
      case '"': o += "&quot;"; break;
      case '\'': o += "&apos;"; break;
      default: o += c;
    }
  }
  return o;
}

void put_tag(FILE* f, const std::string& k, const std::string& v) {
  std::fprintf(f, "  <tag k=\"%s\" v=\"%s\"/>\n", xml_escape(k).c_str(), xml_escape(v).c_str());
}

// OSM XML writer
class XmlSink : public OsmSink {
 public:
  explicit XmlSink(const std::string& path) : path_(path) {
    f_ = std::fopen(path.c_str(), "wb");
    if (!f_) throw std::runtime_error("cannot open OSM file for writing: " + path);
    std::fprintf(f_, "<?xml version='1.0' encoding='UTF-8'?>\n<osm version=\"0.6\" generator=\"%s\">\n", kOsmGenerator);
  }
  ~XmlSink() override {
    if (f_) std::fclose(f_);
  }
  void bounds(float minlat, float minlon, float maxlat, float maxlon) override {
    std::fprintf(f_, " <bounds minlat=\"%.9g\" minlon=\"%.9g\" maxlat=\"%.9g\" maxlon=\"%.9g\"/>\n", (double)minlat,
                 (double)minlon, (double)maxlat, (double)maxlon);
  }
  // float coordinates as 9 significant digits: parsing them back (strtod, then to float)
  // gives the same float
  void node(uint64_t id, float lat, float lon) override {
    std::fprintf(f_, " <node id=\"%llu\" version=\"1\" lat=\"%.9g\" lon=\"%.9g\"/>\n", (unsigned long long)id,
                 (double)lat, (double)lon);
  }
  void way(uint64_t id, const std::vector<uint64_t>& refs, const OsmTags& tags) override {
    std::fprintf(f_, " <way id=\"%llu\" version=\"1\">\n", (unsigned long long)id);
    for (uint64_t r : refs) std::fprintf(f_, "  <nd ref=\"%llu\"/>\n", (unsigned long long)r);
    for (const auto& kv : tags) put_tag(f_, kv.first, kv.second);
    std::fprintf(f_, " </way>\n");
  }
  void relation(uint64_t id, const std::vector<OsmMember>& members, const OsmTags& tags) override {
    std::fprintf(f_, " <relation id=\"%llu\" version=\"1\">\n", (unsigned long long)id);
    for (const OsmMember& m : members)
      std::fprintf(f_, "  <member type=\"%s\" ref=\"%llu\" role=\"%s\"/>\n", m.type.c_str(), (unsigned long long)m.ref,
                   xml_escape(m.role).c_str());
    for (const auto& kv : tags) put_tag(f_, kv.first, kv.second);
    std::fprintf(f_, " </relation>\n");
  }
  void finish() override {
    std::fprintf(f_, "</osm>\n");
    const int rc = std::fclose(f_);
    f_ = nullptr;
    if (rc != 0) throw std::runtime_error("short write on OSM file: " + path_);
  }

 private:
  std::string path_;
  FILE* f_ = nullptr;
};

std::string highway_of(uint32_t info_f, uint32_t info_r) {
  const uint32_t flags = info_f | info_r;
  const uint32_t sp = std::max(edge_speed_dkph(info_f), edge_speed_dkph(info_r));
  if (flags & kFlagInternal) return "primary_link";
  if (flags & kFlagService) return "service";
  if (sp >= 800) return "motorway";
  if (sp >= 450) return "primary";
  return "residential";
}

std::string kmh(uint32_t dkph) {
  char b[32];
  if (dkph % 10 == 0) std::snprintf(b, sizeof b, "%u", dkph / 10);
  else std::snprintf(b, sizeof b, "%u.%u", dkph / 10, dkph % 10);
  return b;
}

// ---------------------------------------------------------------- minimal OSM XML reader
struct XmlElem {
  std::string name;
  std::vector<std::pair<std::string, std::string>> attrs;
  bool closing = false, self_closing = false;
  const std::string* attr(const char* k) const {
    for (const auto& a : attrs) if (a.first == k) return &a.second;
    return nullptr;
  }
};

std::string xml_unescape(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] != '&') { o += s[i]; continue; }
    const size_t e = s.find(';', i);
    if (e == std::string::npos) { o += s[i]; continue; }
    const std::string ent = s.substr(i + 1, e - i - 1);
    if (ent == "amp") o += '&';
    else if (ent == "lt") o += '<';
    else if (ent == "gt") o += '>';
    else if (ent == "quot") o += '"';
    else if (ent == "apos") o += '\'';
    else if (!ent.empty() && ent[0] == '#') {
      const long cp = ent.size() > 1 && (ent[1] == 'x' || ent[1] == 'X') ? std::strtol(ent.c_str() + 2, nullptr, 16)
                                                                           : std::strtol(ent.c_str() + 1, nullptr, 10);
      if (cp < 0x80) o += (char)cp;
      else o += '?';   // non-ASCII character references do not occur in routing tags we read
    } else {
      o += s.substr(i, e - i + 1);
    }
    i = e;
  }
  return o;
}

// next element starting at pos (skips text, comments, declarations); false at end
bool next_elem(const std::string& x, size_t& pos, XmlElem& el) {
  for (;;) {
    const size_t lt = x.find('<', pos);
    if (lt == std::string::npos) return false;
    if (x.compare(lt, 4, "<!--") == 0) {
      const size_t e = x.find("-->", lt + 4);
      if (e == std::string::npos) throw std::runtime_error("unterminated XML comment");
      pos = e + 3;
      continue;
    }
    if (x[lt + 1] == '?' || x[lt + 1] == '!') {
      const size_t e = x.find('>', lt);
      if (e == std::string::npos) throw std::runtime_error("unterminated XML declaration");
      pos = e + 1;
      continue;
    }
    const size_t gt = x.find('>', lt);
    if (gt == std::string::npos) throw std::runtime_error("unterminated XML element");
    size_t i = lt + 1;
    el = XmlElem();
    if (x[i] == '/') { el.closing = true; ++i; }
    const size_t ns = i;
    while (i < gt && !std::isspace((unsigned char)x[i]) && x[i] != '/') ++i;
    el.name = x.substr(ns, i - ns);
    while (i < gt) {
      while (i < gt && std::isspace((unsigned char)x[i])) ++i;
      if (i >= gt) break;
      if (x[i] == '/') { el.self_closing = true; ++i; continue; }
      const size_t ks = i;
      while (i < gt && x[i] != '=' && !std::isspace((unsigned char)x[i])) ++i;
      const std::string key = x.substr(ks, i - ks);
      while (i < gt && x[i] != '=') ++i;
      ++i;
      while (i < gt && std::isspace((unsigned char)x[i])) ++i;
      if (i >= gt || (x[i] != '"' && x[i] != '\'')) throw std::runtime_error("malformed XML attribute");
      const char q = x[i++];
      const size_t vs = i;
      const size_t ve = x.find(q, vs);
      if (ve == std::string::npos || ve > gt) throw std::runtime_error("unterminated XML attribute");
      el.attrs.push_back({key, xml_unescape(x.substr(vs, ve - vs))});
      i = ve + 1;
    }
    pos = gt + 1;
    return true;
  }
}

uint64_t to_u64(const std::string* s, const char* what) {
  if (!s) throw std::runtime_error(std::string("OSM element without ") + what);
  char* end = nullptr;
  const long long v = std::strtoll(s->c_str(), &end, 10);
  if (end == s->c_str() || v < 0) throw std::runtime_error(std::string("bad OSM ") + what + ": " + *s);
  return (uint64_t)v;
}

const std::string* tag(const std::map<std::string, std::string>& t, const char* k) {
  auto it = t.find(k);
  return it == t.end() ? nullptr : &it->second;
}

bool is_no(const std::string* v) { return v && (*v == "no" || *v == "private"); }

// routing attributes of a generic highway way (speeds 0.1 km/h, access bits per direction)
void derive_info(const std::map<std::string, std::string>& t, uint32_t& info_f, uint32_t& info_r) {
  const std::string hw = *tag(t, "highway");
  uint32_t sp = 300;
  if (hw == "motorway") sp = 900;
  else if (hw == "trunk") sp = 700;
  else if (hw == "primary" || hw == "secondary") sp = 500;
  else if (hw == "tertiary") sp = 400;
  else if (hw == "service") sp = 150;
  else if (hw.size() > 5 && hw.compare(hw.size() - 5, 5, "_link") == 0) sp = 200;
  else if (hw == "footway" || hw == "path" || hw == "pedestrian" || hw == "steps" || hw == "cycleway") sp = 50;
  auto speed_of = [&](const char* k, uint32_t dflt) {
    const std::string* v = tag(t, k);
    if (!v) return dflt;
    const double kph = std::atof(v->c_str());
    return kph > 0 ? (uint32_t)std::lround(kph * 10.0) : dflt;
  };
  const uint32_t sp_any = speed_of("maxspeed", sp);
  const uint32_t sp_f = speed_of("maxspeed:forward", sp_any), sp_r = speed_of("maxspeed:backward", sp_any);
  const bool foot_only = hw == "footway" || hw == "path" || hw == "pedestrian" || hw == "steps";
  const bool cycle_only = hw == "cycleway";
  const bool fast = hw == "motorway" || hw == "trunk" || hw == "motorway_link" || hw == "trunk_link";
  uint32_t a = 0;
  if (!foot_only && !cycle_only && !is_no(tag(t, "motor_vehicle")) && !is_no(tag(t, "access"))) a |= kAccessAuto;
  if (!fast && !foot_only && !is_no(tag(t, "bicycle"))) a |= kAccessBicycle;
  if (!fast && !cycle_only && !is_no(tag(t, "foot"))) a |= kAccessPedestrian;
  if (cycle_only) a |= kAccessBicycle;
  if (foot_only) a |= kAccessPedestrian;
  uint32_t af = a, ar = a;
  const std::string* ow = tag(t, "oneway");
  // a roundabout is one-way in its drawing direction unless tagged otherwise (OSM convention)
  const std::string* jc = tag(t, "junction");
  const bool ring = jc && (*jc == "roundabout" || *jc == "circular") && !(ow && *ow == "no");
  // an explicit oneway=-1 wins over the roundabout's implied drawing direction
  if (ow && *ow == "-1") af &= kAccessPedestrian;
  else if (ring || (ow && (*ow == "yes" || *ow == "true" || *ow == "1"))) ar &= kAccessPedestrian;
  uint32_t flags = 0;
  if (hw == "service") flags |= kFlagService;
  if (hw.size() > 5 && hw.compare(hw.size() - 5, 5, "_link") == 0) flags |= kFlagInternal;
  info_f = std::min<uint32_t>(sp_f, 0xffffu) | (af << 16) | flags;
  info_r = std::min<uint32_t>(sp_r, 0xffffu) | (ar << 16) | flags;
}

}  // namespace

const char* const kOsmGenerator = "reporter_amd rmg-osm 1";

void emit_osm(const Graph& g, OsmSink& sink) {
  const uint32_t N = g.num_nodes(), R = g.num_roads(), S = g.num_segments();
  if (N) {
    float lo0 = g.node_lon[0], lo1 = lo0, la0 = g.node_lat[0], la1 = la0;
    for (uint32_t n = 1; n < N; ++n) {
      lo0 = std::min(lo0, g.node_lon[n]); lo1 = std::max(lo1, g.node_lon[n]);
      la0 = std::min(la0, g.node_lat[n]); la1 = std::max(la1, g.node_lat[n]);
    }
    sink.bounds(la0, lo0, la1, lo1);
  }
  for (uint32_t n = 0; n < N; ++n) sink.node(n + 1ull, g.node_lat[n], g.node_lon[n]);
  for (uint32_t r = 0; r < R; ++r)
    for (uint32_t v = g.road_vert_off[r] + 1; v + 1 < g.road_vert_off[r + 1]; ++v)
      sink.node((uint64_t)N + 1 + v, g.verts[v].lat, g.verts[v].lon);
  std::vector<uint64_t> refs;
  OsmTags tags;
  for (uint32_t r = 0; r < R; ++r) {
    refs.clear();
    tags.clear();
    refs.push_back(g.road_node0[r] + 1ull);
    for (uint32_t v = g.road_vert_off[r] + 1; v + 1 < g.road_vert_off[r + 1]; ++v) refs.push_back((uint64_t)N + 1 + v);
    refs.push_back(g.road_node1[r] + 1ull);
    const uint32_t ef = g.road_fwd[r], er = g.road_rev[r];
    const uint32_t inf = ef == kNone ? 0u : g.edges[ef].info, inr = er == kNone ? 0u : g.edges[er].info;
    tags.push_back({"highway", highway_of(inf, inr)});
    const uint32_t sf = edge_speed_dkph(inf), sr = edge_speed_dkph(inr);
    if (ef != kNone && er != kNone && sf != sr) {
      tags.push_back({"maxspeed:forward", kmh(sf)});
      tags.push_back({"maxspeed:backward", kmh(sr)});
    } else {
      tags.push_back({"maxspeed", kmh(ef != kNone ? sf : sr)});
    }
    const uint32_t af = ef == kNone ? 0u : edge_access(inf), ar = er == kNone ? 0u : edge_access(inr);
    if ((af & kAccessAuto) && !(ar & kAccessAuto)) tags.push_back({"oneway", "yes"});
    else if (!(af & kAccessAuto) && (ar & kAccessAuto)) tags.push_back({"oneway", "-1"});
    else if (!((af | ar) & kAccessAuto)) tags.push_back({"motor_vehicle", "no"});
    if (!((af | ar) & kAccessBicycle)) tags.push_back({"bicycle", "no"});
    if (!((af | ar) & kAccessPedestrian)) tags.push_back({"foot", "no"});
    tags.push_back({"reporter:info", (ef == kNone ? std::string("-") : std::to_string(inf)) + ";" +
                                         (er == kNone ? std::string("-") : std::to_string(inr))});
    tags.push_back({"reporter:way", std::to_string(ef == kNone ? 0u : g.edge_way[ef]) + ";" +
                                        std::to_string(er == kNone ? 0u : g.edge_way[er])});
    sink.way(r + 1ull, refs, tags);
  }
  // OSMLR segments: their directed edges in offset order
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> seg_edges(S);   // (offset cm, edge)
  for (uint32_t e = 0; e < g.num_edges(); ++e)
    if (g.edge_seg[e] != kNone) seg_edges[g.edge_seg[e]].push_back({g.edge_seg_off[e], e});
  std::vector<OsmMember> members;
  for (uint32_t s = 0; s < S; ++s) {
    auto& v = seg_edges[s];
    std::stable_sort(v.begin(), v.end());
    members.clear();
    tags.clear();
    std::string offs;
    for (const auto& oe : v) {
      const uint32_t road = g.edges[oe.second].road >> 1;
      members.push_back({"way", (g.edges[oe.second].road & 1u) ? "backward" : "forward", road + 1ull});
      if (!offs.empty()) offs += ';';
      offs += std::to_string(oe.first);
    }
    tags.push_back({"type", "osmlr"});
    tags.push_back({"osmlr:id", std::to_string(g.seg_id[s])});
    tags.push_back({"osmlr:length_cm", std::to_string(g.seg_len_cm[s])});
    tags.push_back({"osmlr:offsets_cm", offs});
    sink.relation(s + 1ull, members, tags);
  }
  {
    char b[256];
    std::snprintf(b, sizeof b, "%a %a %a %a %u %u", g.grid.lon0, g.grid.lat0, g.grid.dlon, g.grid.dlat, g.grid.ncx,
                  g.grid.ncy);
    members.clear();
    tags.clear();
    tags.push_back({"type", "reporter_grid"});
    tags.push_back({"reporter:grid", b});
    sink.relation(S + 1ull, members, tags);
  }
  sink.finish();
}

void export_osm(const Graph& g, const std::string& path) {
  XmlSink x(path);
  emit_osm(g, x);
}

std::unique_ptr<OsmSink> make_osm_xml_sink(const std::string& path) { return std::make_unique<XmlSink>(path); }

OsmParsed parse_osm_xml(const std::string& path) {
  std::string x;
  {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open OSM file: " + path);
    char buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) x.append(buf, n);
    std::fclose(f);
  }
  OsmParsed o;
  size_t pos = 0;
  XmlElem el;
  int ctx = 0;   // 1 way, 2 relation
  bool saw_osm = false;
  while (next_elem(x, pos, el)) {
    if (el.name == "osm") { saw_osm = true; continue; }
    if (el.closing) {
      if (el.name == "way" || el.name == "relation") ctx = 0;
      continue;
    }
    if (el.name == "node") {
      const std::string *la = el.attr("lat"), *lo = el.attr("lon");
      if (!la || !lo) throw std::runtime_error("OSM node without lat/lon");
      o.nodes.push_back({to_u64(el.attr("id"), "node id"),
                         {(float)std::strtod(lo->c_str(), nullptr), (float)std::strtod(la->c_str(), nullptr)}});
      ctx = 0;
    } else if (el.name == "way") {
      o.ways.push_back(OsmParsedWay{to_u64(el.attr("id"), "way id"), {}, {}});
      ctx = el.self_closing ? 0 : 1;
    } else if (el.name == "relation") {
      o.rels.push_back(OsmParsedRelation{to_u64(el.attr("id"), "relation id"), {}, {}});
      ctx = el.self_closing ? 0 : 2;
    } else if (el.name == "nd" && ctx == 1) {
      o.ways.back().refs.push_back(to_u64(el.attr("ref"), "nd ref"));
    } else if (el.name == "tag" && ctx) {
      const std::string *k = el.attr("k"), *v = el.attr("v");
      if (!k || !v) throw std::runtime_error("OSM tag without k/v");
      (ctx == 1 ? o.ways.back().tags : o.rels.back().tags)[*k] = *v;
    } else if (el.name == "member" && ctx == 2) {
      const std::string *t = el.attr("type"), *role = el.attr("role");
      o.rels.back().members.push_back({t ? *t : "", role ? *role : "", to_u64(el.attr("ref"), "member ref")});
    }
  }
  if (!saw_osm) throw std::runtime_error("not an OSM XML file: " + path);
  return o;
}

Graph graph_from_osm(OsmParsed& osm, double cell_m) {
  auto& nodes = osm.nodes;
  auto& ways = osm.ways;
  auto& rels = osm.rels;
  std::stable_sort(nodes.begin(), nodes.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::unordered_map<uint64_t, uint32_t> nidx;   // OSM node id -> position in `nodes`
  nidx.reserve(nodes.size() * 2);
  for (uint32_t i = 0; i < nodes.size(); ++i) nidx[nodes[i].first] = i;
  std::stable_sort(ways.begin(), ways.end(), [](const OsmParsedWay& a, const OsmParsedWay& b) { return a.id < b.id; });
  std::stable_sort(rels.begin(), rels.end(),
                   [](const OsmParsedRelation& a, const OsmParsedRelation& b) { return a.id < b.id; });
  // routable ways: highway-tagged with >= 2 known nodes
  std::vector<const OsmParsedWay*> hw;
  for (const OsmParsedWay& w : ways) {
    if (!tag(w.tags, "highway") || w.refs.size() < 2) continue;
    for (uint64_t r : w.refs)
      if (!nidx.count(r)) throw std::runtime_error("OSM way " + std::to_string(w.id) + " names a missing node");
    hw.push_back(&w);
  }
  bool exact = !hw.empty();
  for (const OsmParsedWay* w : hw) exact = exact && tag(w->tags, "reporter:info") && tag(w->tags, "reporter:way");
  // ---- graph nodes: way ends and nodes used more than once; ascending OSM id
  std::vector<uint32_t> uses(nodes.size(), 0);
  std::vector<uint8_t> is_end(nodes.size(), 0);
  for (const OsmParsedWay* w : hw) {
    for (uint64_t r : w->refs) uses[nidx[r]]++;
    is_end[nidx[w->refs.front()]] = is_end[nidx[w->refs.back()]] = 1;
  }
  Graph g;
  std::vector<uint32_t> gidx(nodes.size(), kNone);
  for (uint32_t i = 0; i < nodes.size(); ++i)
    if (is_end[i] || uses[i] > 1) {
      gidx[i] = (uint32_t)g.node_lon.size();
      g.node_lon.push_back(nodes[i].second.first);
      g.node_lat.push_back(nodes[i].second.second);
    }
  // ---- roads: ways split at graph nodes
  std::vector<RoadInput> roads;
  std::unordered_map<uint64_t, std::vector<uint32_t>> way_roads;   // way id -> its roads in way order
  for (const OsmParsedWay* w : hw) {
    uint32_t inf, inr, wf = (uint32_t)w->id, wr = (uint32_t)w->id;
    if (exact) {
      const std::string& s = *tag(w->tags, "reporter:info");
      const size_t sc = s.find(';');
      if (sc == std::string::npos) throw std::runtime_error("bad reporter:info tag");
      inf = s.substr(0, sc) == "-" ? 0u : (uint32_t)std::strtoul(s.c_str(), nullptr, 10);
      inr = s.substr(sc + 1) == "-" ? 0u : (uint32_t)std::strtoul(s.c_str() + sc + 1, nullptr, 10);
      if (std::sscanf(tag(w->tags, "reporter:way")->c_str(), "%u;%u", &wf, &wr) != 2)
        throw std::runtime_error("bad reporter:way tag");
    } else {
      derive_info(w->tags, inf, inr);
    }
    size_t start = 0;
    for (size_t k = 1; k < w->refs.size(); ++k) {
      const uint32_t ni = nidx[w->refs[k]];
      if (gidx[ni] == kNone && k + 1 < w->refs.size()) continue;
      RoadInput rd;
      rd.n0 = gidx[nidx[w->refs[start]]];
      rd.n1 = gidx[ni];
      for (size_t q = start; q <= k; ++q) rd.shape.push_back(nodes[nidx[w->refs[q]]].second);
      rd.info_fwd = inf; rd.info_rev = inr; rd.way_fwd = wf; rd.way_rev = wr;
      start = k;
      if (rd.n0 == rd.n1) {
        if (exact) throw std::runtime_error("exported way closes on itself");
        continue;   // a closed loop between one intersection: no route uses it end to end
      }
      std::vector<uint32_t>& wr_list = way_roads[w->id];
      if (exact && !wr_list.empty()) throw std::runtime_error("exported way spans several roads");
      wr_list.push_back((uint32_t)roads.size());
      roads.push_back(std::move(rd));
    }
  }
  if (roads.empty()) throw std::runtime_error("OSM file has no routable highway ways");
  assemble_roads(g, roads);
  // ---- OSMLR segments.  A member way that the import split into several roads contributes
  // all of them in travel order (forward: the way's order; backward: reversed), so the
  // segment's edges and offsets follow the whole way, never its first piece alone.
  for (const OsmParsedRelation& rl : rels) {
    const std::string* t = tag(rl.tags, "type");
    if (!t || *t != "osmlr") continue;
    const std::string *id = tag(rl.tags, "osmlr:id"), *len = tag(rl.tags, "osmlr:length_cm");
    if (!id) throw std::runtime_error("osmlr relation without osmlr:id");
    const uint32_t s = (uint32_t)g.seg_id.size();
    g.seg_id.push_back(std::strtoull(id->c_str(), nullptr, 10));
    std::vector<uint32_t> offs;
    if (const std::string* o = tag(rl.tags, "osmlr:offsets_cm")) {
      const char* p = o->c_str();
      while (*p) {
        char* e = nullptr;
        offs.push_back((uint32_t)std::strtoul(p, &e, 10));
        p = *e == ';' ? e + 1 : e;
        if (e == p && *p) throw std::runtime_error("bad osmlr:offsets_cm");
      }
    }
    uint32_t acc = 0;
    size_t piece = 0;   // edges assigned so far (offsets index, exact files: one per member)
    for (size_t m = 0; m < rl.members.size(); ++m) {
      const OsmMember& mb = rl.members[m];
      auto it = way_roads.find(mb.ref);
      if (mb.type != "way" || it == way_roads.end()) throw std::runtime_error("osmlr relation names a non-road member");
      const bool back = mb.role == "backward";
      const std::vector<uint32_t>& rs = it->second;
      for (size_t q = 0; q < rs.size(); ++q) {
        const uint32_t road = rs[back ? rs.size() - 1 - q : q];
        const uint32_t e = back ? g.road_rev[road] : g.road_fwd[road];
        if (e == kNone) throw std::runtime_error("osmlr member direction has no edge");
        if (g.edge_seg[e] != kNone) throw std::runtime_error("an edge belongs to two osmlr segments");
        g.edge_seg[e] = s;
        g.edge_seg_off[e] = piece < offs.size() ? offs[piece] : acc;
        acc += g.edges[e].len_cm;
        ++piece;
      }
    }
    g.seg_len_cm.push_back(len ? (uint32_t)std::strtoul(len->c_str(), nullptr, 10) : acc);
  }
  // ---- spatial index: the exported geometry, or cells of cell_m metres
  bool have_grid = false;
  for (const OsmParsedRelation& rl : rels) {
    const std::string* t = tag(rl.tags, "type");
    const std::string* gs = tag(rl.tags, "reporter:grid");
    if (!t || *t != "reporter_grid" || !gs) continue;
    if (std::sscanf(gs->c_str(), "%la %la %la %la %u %u", &g.grid.lon0, &g.grid.lat0, &g.grid.dlon, &g.grid.dlat,
                    &g.grid.ncx, &g.grid.ncy) != 6)
      throw std::runtime_error("bad reporter:grid tag");
    // an untrusted file: the cell count must stay plausible for the graph (the index holds one
    // offset per cell) and the cells must be finite and positive
    const double cells = (double)g.grid.ncx * (double)g.grid.ncy;
    if (!(g.grid.dlon > 0) || !(g.grid.dlat > 0) || !std::isfinite(g.grid.lon0) || !std::isfinite(g.grid.lat0) ||
        g.grid.ncx == 0 || g.grid.ncy == 0 || cells > std::max(1e6, 64.0 * (double)g.verts.size()))
      throw std::runtime_error("implausible reporter:grid geometry");
    have_grid = true;
  }
  if (!have_grid) {
    if (!(cell_m > 0)) throw std::runtime_error("cell_m must be positive");
    float min_lon = 1e30f, min_lat = 1e30f, max_lon = -1e30f, max_lat = -1e30f;
    for (const auto& v : g.verts) {
      min_lon = std::min(min_lon, v.lon); max_lon = std::max(max_lon, v.lon);
      min_lat = std::min(min_lat, v.lat); max_lat = std::max(max_lat, v.lat);
    }
    const double mid = 0.5 * ((double)min_lat + (double)max_lat);
    GridIndex& gi = g.grid;
    gi.dlat = cell_m / kMetersPerDegLat;
    gi.dlon = cell_m / (kMetersPerDegLonEq * std::cos(mid * kDegToRad));
    gi.lon0 = (double)min_lon - gi.dlon;
    gi.lat0 = (double)min_lat - gi.dlat;
    gi.ncx = (uint32_t)std::ceil(((double)max_lon - gi.lon0) / gi.dlon) + 2;
    gi.ncy = (uint32_t)std::ceil(((double)max_lat - gi.lat0) / gi.dlat) + 2;
    if ((double)gi.ncx * (double)gi.ncy > std::max(1e6, 64.0 * (double)g.verts.size()))
      throw std::runtime_error("cell_m too small for the extent of the OSM file");
  }
  build_grid_index(g);
  g.validate();
  return g;
}

// XML or PBF by content: a PBF file starts with the 4-byte length of its first BlobHeader
Graph import_osm(const std::string& path, double cell_m) {
  unsigned char head[8] = {};
  {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open OSM file: " + path);
    const size_t n = std::fread(head, 1, sizeof head, f);
    std::fclose(f);
    if (n < 5) throw std::runtime_error("OSM file too short: " + path);
  }
  const bool pbf = head[0] == 0 && head[4] == 0x0a;   // BlobHeader field 1 (type) first
  OsmParsed osm = pbf ? parse_osm_pbf(path) : parse_osm_xml(path);
  return graph_from_osm(osm, cell_m);
}

}  // namespace rm
