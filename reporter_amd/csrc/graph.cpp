// graph.cpp — ".rmg" flat graph file: header + named, 64-byte aligned sections.
//
//   bytes 0..7   "RMGRAPH1"
//   u32 version (=1), u32 nsections
//   nsections x { char name[24]; u64 offset; u64 bytes; }
//   section payloads (little-endian arrays), each 64-byte aligned
//
// reporter_amd/graphfile.py reads the same layout with numpy for tests/oracle.
#include "graph.hpp"

#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace rm {

namespace {

struct SecHdr {
  char name[24];
  uint64_t offset;
  uint64_t bytes;
};

struct GridMeta {
  double lon0, lat0, dlon, dlat;
  uint32_t ncx, ncy;
  uint32_t pad[2];
};

struct Writer {
  struct Item { std::string name; const void* p; uint64_t n; };
  std::vector<Item> items;
  template <class T> void add(const char* name, const std::vector<T>& v) {
    items.push_back({name, v.data(), (uint64_t)(v.size() * sizeof(T))});
  }
  void add_raw(const char* name, const void* p, uint64_t n) { items.push_back({name, p, n}); }
  void write(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot open graph file for writing: " + path);
    const uint32_t version = 1, ns = (uint32_t)items.size();
    std::vector<SecHdr> hdr(ns);
    uint64_t off = 16 + sizeof(SecHdr) * ns;
    off = (off + 63) & ~63ull;
    for (uint32_t i = 0; i < ns; ++i) {
      std::memset(hdr[i].name, 0, sizeof(hdr[i].name));
      std::strncpy(hdr[i].name, items[i].name.c_str(), sizeof(hdr[i].name) - 1);
      hdr[i].offset = off;
      hdr[i].bytes = items[i].n;
      off = (off + items[i].n + 63) & ~63ull;
    }
    bool ok = std::fwrite("RMGRAPH1", 1, 8, f) == 8;
    ok = ok && std::fwrite(&version, 4, 1, f) == 1 && std::fwrite(&ns, 4, 1, f) == 1;
    ok = ok && std::fwrite(hdr.data(), sizeof(SecHdr), ns, f) == ns;
    uint64_t pos = 16 + sizeof(SecHdr) * ns;
    static const char zeros[64] = {0};
    for (uint32_t i = 0; ok && i < ns; ++i) {
      while (pos < hdr[i].offset) {
        uint64_t k = hdr[i].offset - pos; if (k > 64) k = 64;
        ok = std::fwrite(zeros, 1, k, f) == k; pos += k;
      }
      if (items[i].n) ok = ok && std::fwrite(items[i].p, 1, items[i].n, f) == items[i].n;
      pos += items[i].n;
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) throw std::runtime_error("short write on graph file: " + path);
  }
};

struct Reader {
  std::vector<char> buf;
  std::vector<SecHdr> hdr;
  explicit Reader(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open graph file: " + path);
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (n < 16) { std::fclose(f); throw std::runtime_error("graph file too short: " + path); }
    buf.resize((size_t)n);
    size_t got = std::fread(buf.data(), 1, (size_t)n, f);
    std::fclose(f);
    if (got != (size_t)n) throw std::runtime_error("short read on graph file: " + path);
    if (std::memcmp(buf.data(), "RMGRAPH1", 8) != 0) throw std::runtime_error("not an .rmg graph file: " + path);
    uint32_t version, ns;
    std::memcpy(&version, buf.data() + 8, 4);
    std::memcpy(&ns, buf.data() + 12, 4);
    if (version != 1) throw std::runtime_error("unsupported .rmg version");
    if (16 + (uint64_t)ns * sizeof(SecHdr) > (uint64_t)n) throw std::runtime_error("corrupt .rmg header");
    hdr.resize(ns);
    std::memcpy(hdr.data(), buf.data() + 16, sizeof(SecHdr) * ns);
    for (auto& h : hdr)
      if (h.offset + h.bytes > (uint64_t)n) throw std::runtime_error("corrupt .rmg section bounds");
  }
  const SecHdr& find(const char* name) const {
    for (auto& h : hdr) if (std::strncmp(h.name, name, sizeof(h.name)) == 0) return h;
    throw std::runtime_error(std::string("graph file lacks section ") + name);
  }
  template <class T> void get(const char* name, std::vector<T>& v) const {
    const SecHdr& h = find(name);
    if (h.bytes % sizeof(T)) throw std::runtime_error(std::string("bad section size ") + name);
    v.resize(h.bytes / sizeof(T));
    if (h.bytes) std::memcpy(v.data(), buf.data() + h.offset, h.bytes);
  }
};

}  // namespace

void Graph::save(const std::string& path) const {
  GridMeta gm{grid.lon0, grid.lat0, grid.dlon, grid.dlat, grid.ncx, grid.ncy, {0, 0}};
  Writer w;
  w.add("node_lon", node_lon); w.add("node_lat", node_lat); w.add("node_off", node_off);
  w.add("edges", edges); w.add("edge_seg", edge_seg); w.add("edge_seg_off", edge_seg_off);
  w.add("edge_way", edge_way);
  w.add("road_node0", road_node0); w.add("road_node1", road_node1); w.add("road_fwd", road_fwd);
  w.add("road_rev", road_rev); w.add("road_len_cm", road_len_cm); w.add("road_vert_off", road_vert_off);
  w.add("verts", verts); w.add("seg_id", seg_id); w.add("seg_len_cm", seg_len_cm);
  w.add_raw("grid_meta", &gm, sizeof(gm));
  w.add("cell_off", grid.cell_off); w.add("cell_item", grid.cell_item);
  w.write(path);
}

Graph Graph::load(const std::string& path) {
  Reader r(path);
  Graph g;
  r.get("node_lon", g.node_lon); r.get("node_lat", g.node_lat); r.get("node_off", g.node_off);
  r.get("edges", g.edges); r.get("edge_seg", g.edge_seg); r.get("edge_seg_off", g.edge_seg_off);
  r.get("edge_way", g.edge_way);
  r.get("road_node0", g.road_node0); r.get("road_node1", g.road_node1); r.get("road_fwd", g.road_fwd);
  r.get("road_rev", g.road_rev); r.get("road_len_cm", g.road_len_cm); r.get("road_vert_off", g.road_vert_off);
  r.get("verts", g.verts); r.get("seg_id", g.seg_id); r.get("seg_len_cm", g.seg_len_cm);
  std::vector<GridMeta> gm;
  r.get("grid_meta", gm);
  if (gm.size() != 1) throw std::runtime_error("bad grid_meta section");
  g.grid.lon0 = gm[0].lon0; g.grid.lat0 = gm[0].lat0; g.grid.dlon = gm[0].dlon; g.grid.dlat = gm[0].dlat;
  g.grid.ncx = gm[0].ncx; g.grid.ncy = gm[0].ncy;
  r.get("cell_off", g.grid.cell_off); r.get("cell_item", g.grid.cell_item);
  g.validate();
  return g;
}

void Graph::validate() const {
  const uint32_t N = num_nodes(), E = num_edges(), R = num_roads(), V = num_verts(), S = num_segments();
  auto fail = [](const char* m) { throw std::runtime_error(std::string("invalid graph: ") + m); };
  if (node_lat.size() != N || node_off.size() != (size_t)N + 1) fail("node arrays");
  if (node_off[0] != 0 || node_off[N] != E) fail("CSR bounds");
  for (uint32_t n = 0; n < N; ++n) if (node_off[n] > node_off[n + 1]) fail("CSR not monotone");
  if (edge_seg.size() != E || edge_seg_off.size() != E || edge_way.size() != E) fail("edge arrays");
  for (uint32_t e = 0; e < E; ++e) {
    const EdgeRec& r = edges[e];
    if (r.target >= N || r.len_cm == 0 || (r.road >> 1) >= R || edge_speed_dkph(r.info) == 0) fail("edge record");
    if (edge_seg[e] != kNone && edge_seg[e] >= S) fail("edge segment index");
  }
  if (road_node1.size() != R || road_fwd.size() != R || road_rev.size() != R || road_node0.size() != R ||
      road_vert_off.size() != (size_t)R + 1 || road_vert_off[R] != V) fail("road arrays");
  for (uint32_t r = 0; r < R; ++r) {
    if (road_vert_off[r + 1] < road_vert_off[r] + 2) fail("road needs >= 2 vertices");
    if (road_fwd[r] != kNone && road_fwd[r] >= E) fail("road fwd edge");
    if (road_rev[r] != kNone && road_rev[r] >= E) fail("road rev edge");
    if (road_node0[r] >= N || road_node1[r] >= N || road_node0[r] == road_node1[r]) fail("road nodes");
    if (verts[road_vert_off[r + 1] - 1].cum_cm != road_len_cm[r]) fail("road length / shape");
  }
  if (seg_len_cm.size() != S) fail("segment arrays");
  if (grid.cell_off.size() != (size_t)grid.ncx * grid.ncy + 1 || grid.cell_off.back() != grid.cell_item.size())
    fail("grid index");
  for (uint32_t it : grid.cell_item) if (it + 1 >= V || verts[it].road == kNone) fail("grid item");
}

}  // namespace rm
