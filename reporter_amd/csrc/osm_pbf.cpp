// osm_pbf.cpp — OSM PBF ("OpenStreetMap protocol buffer binary") writer and reader for the
// engine's graph.  BASELINE.json's north star builds the Valhalla tiles of
// both paths "from a synthetic OSM .pbf"; valhalla_build_tiles (reference Dockerfile:42-49,
// README.md:129-130) reads this format.  Hand-written: protobuf varints / zigzag / packed
// fields and zlib-deflated blobs, no protobuf library.
//
// File layout (the OSM PBF format):
//   repeated { int32 big-endian length of BlobHeader; BlobHeader; Blob }
//   BlobHeader { 1: string type ("OSMHeader" | "OSMData"), 3: int32 datasize }
//   Blob       { 2: int32 raw_size, 3: bytes zlib_data }        (1: raw, also read)
//   HeaderBlock   { 1: HeaderBBox {1 left, 2 right, 3 top, 4 bottom: sint64 nanodegrees},
//                   4: required_features "OsmSchema-V0.6" "DenseNodes", 16: writingprogram }
//   PrimitiveBlock { 1: StringTable { 1: repeated bytes s }, 2: repeated PrimitiveGroup,
//                    17: granularity (nanodegrees per unit), 19/20: lat/lon offset }
//   PrimitiveGroup { 1: Node, 2: DenseNodes {1 id, 8 lat, 9 lon: packed delta sint64,
//                    10 keys_vals}, 3: Way {1 id, 2 keys, 3 vals, 8 refs: delta sint64},
//                    4: Relation {1 id, 2 keys, 3 vals, 8 roles_sid, 9 memids: delta sint64,
//                    10 types} }
// The writer uses granularity 1 (nanodegrees) so every float coordinate of magnitude >= ~0.01
// degree survives exactly; a node whose float would not is given a reporter:ll tag with its
// exact hex floats, which the reader prefers.  Blocks hold up to 8000 entities.
#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "graph.hpp"
#include "osm_model.hpp"

namespace rm {

namespace {

// ---------------------------------------------------------------- protobuf encoding
void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) { o += (char)(uint8_t)(v | 0x80); v >>= 7; }
  o += (char)(uint8_t)v;
}
uint64_t zigzag(int64_t v) { return ((uint64_t)v << 1) ^ (uint64_t)(v >> 63); }
int64_t unzigzag(uint64_t v) { return (int64_t)(v >> 1) ^ -(int64_t)(v & 1); }
void put_key(std::string& o, uint32_t field, uint32_t wire) { put_varint(o, ((uint64_t)field << 3) | wire); }
void put_uint(std::string& o, uint32_t field, uint64_t v) { put_key(o, field, 0); put_varint(o, v); }
void put_sint(std::string& o, uint32_t field, int64_t v) { put_key(o, field, 0); put_varint(o, zigzag(v)); }
void put_bytes(std::string& o, uint32_t field, const std::string& b) {
  put_key(o, field, 2);
  put_varint(o, b.size());
  o += b;
}

// ---------------------------------------------------------------- protobuf decoding
struct Pb {
  const uint8_t* p;
  const uint8_t* e;
  Pb(const void* b, size_t n) : p((const uint8_t*)b), e((const uint8_t*)b + n) {}
  explicit Pb(const std::string& s) : Pb(s.data(), s.size()) {}
  bool more() const { return p < e; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int sh = 0; sh < 64; sh += 7) {
      if (p >= e) throw std::runtime_error("truncated varint in OSM PBF");
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << sh;
      if (!(b & 0x80)) return v;
    }
    throw std::runtime_error("varint too long in OSM PBF");
  }
  // next field: its number and wire type; length-delimited payloads in (lp, ln)
  bool field(uint32_t& num, uint32_t& wire, uint64_t& val, const uint8_t*& lp, size_t& ln) {
    if (p >= e) return false;
    const uint64_t k = varint();
    num = (uint32_t)(k >> 3);
    wire = (uint32_t)(k & 7);
    switch (wire) {
      case 0: val = varint(); break;
      case 1: if (e - p < 8) throw std::runtime_error("truncated OSM PBF"); p += 8; break;
      case 5: if (e - p < 4) throw std::runtime_error("truncated OSM PBF"); p += 4; break;
      case 2: {
        const uint64_t n = varint();
        if (n > (uint64_t)(e - p)) throw std::runtime_error("truncated OSM PBF field");
        lp = p;
        ln = (size_t)n;
        p += n;
        break;
      }
      default: throw std::runtime_error("unsupported protobuf wire type in OSM PBF");
    }
    return true;
  }
};

// packed varints (wire 2) or one varint (wire 0) into out
void unpack(uint32_t wire, uint64_t val, const uint8_t* lp, size_t ln, std::vector<uint64_t>& out) {
  if (wire == 0) { out.push_back(val); return; }
  if (wire != 2) throw std::runtime_error("bad packed field in OSM PBF");
  Pb q(lp, ln);
  while (q.more()) out.push_back(q.varint());
}

std::string deflate_bytes(const std::string& raw) {
  uLongf n = compressBound((uLong)raw.size());
  std::string out(n, '\0');
  if (compress2((Bytef*)&out[0], &n, (const Bytef*)raw.data(), (uLong)raw.size(), 6) != Z_OK)
    throw std::runtime_error("zlib compress failed");
  out.resize(n);
  return out;
}

std::string inflate_bytes(const uint8_t* z, size_t n, size_t raw_size) {
  if (raw_size > (64u << 20)) throw std::runtime_error("OSM PBF blob above 64 MiB");
  std::string out(raw_size, '\0');
  uLongf got = (uLongf)raw_size;
  if (uncompress((Bytef*)&out[0], &got, (const Bytef*)z, (uLong)n) != Z_OK || got != raw_size)
    throw std::runtime_error("zlib inflate failed on an OSM PBF blob");
  return out;
}

// ---------------------------------------------------------------- writer
class PbfSink : public OsmSink {
 public:
  explicit PbfSink(const std::string& path) : path_(path) {
    f_ = std::fopen(path.c_str(), "wb");
    if (!f_) throw std::runtime_error("cannot open OSM PBF file for writing: " + path);
  }
  ~PbfSink() override {
    if (f_) std::fclose(f_);
  }
  void bounds(float minlat, float minlon, float maxlat, float maxlon) override {
    have_bounds_ = true;
    bb_[0] = minlon; bb_[1] = maxlon; bb_[2] = maxlat; bb_[3] = minlat;
  }
  void node(uint64_t id, float lat, float lon) override {
    header();
    if (kind_ != 1) flush();
    kind_ = 1;
    const int64_t la = std::llround((double)lat * 1e9), lo = std::llround((double)lon * 1e9);
    nid_.push_back((int64_t)id);
    nlat_.push_back(la);
    nlon_.push_back(lo);
    // exact float bits when nanodegrees do not bring the float back (|x| below ~0.01 degree)
    if ((float)((double)la * 1e-9) != lat || (float)((double)lo * 1e-9) != lon) {
      char b[96];
      std::snprintf(b, sizeof b, "%a %a", (double)lat, (double)lon);
      nkv_.push_back(sid("reporter:ll"));
      nkv_.push_back(sid(b));
    }
    nkv_.push_back(0);
    if (nid_.size() >= kBlock) flush();
  }
  void way(uint64_t id, const std::vector<uint64_t>& refs, const OsmTags& tags) override {
    header();
    if (kind_ != 2) flush();
    kind_ = 2;
    std::string w;
    put_uint(w, 1, id);
    pack_tags(w, tags);
    std::string r;
    int64_t prev = 0;
    for (uint64_t x : refs) { put_varint(r, zigzag((int64_t)x - prev)); prev = (int64_t)x; }
    put_bytes(w, 8, r);
    put_bytes(group_, 3, w);
    if (++count_ >= kBlock) flush();
  }
  void relation(uint64_t id, const std::vector<OsmMember>& members, const OsmTags& tags) override {
    header();
    if (kind_ != 3) flush();
    kind_ = 3;
    std::string rl;
    put_uint(rl, 1, id);
    pack_tags(rl, tags);
    std::string roles, ids, types;
    int64_t prev = 0;
    for (const OsmMember& m : members) {
      put_varint(roles, sid(m.role));
      put_varint(ids, zigzag((int64_t)m.ref - prev));
      prev = (int64_t)m.ref;
      put_varint(types, m.type == "node" ? 0u : (m.type == "way" ? 1u : 2u));
    }
    put_bytes(rl, 8, roles);
    put_bytes(rl, 9, ids);
    put_bytes(rl, 10, types);
    put_bytes(group_, 4, rl);
    if (++count_ >= kBlock) flush();
  }
  void finish() override {
    header();
    flush();
    const int rc = std::fclose(f_);
    f_ = nullptr;
    if (rc != 0) throw std::runtime_error("short write on OSM PBF file: " + path_);
  }

 private:
  static constexpr size_t kBlock = 8000;   // entities per PrimitiveBlock (the format's convention)
  std::string path_;
  FILE* f_ = nullptr;
  bool header_done_ = false, have_bounds_ = false;
  float bb_[4] = {};
  int kind_ = 0;   // 1 dense nodes, 2 ways, 3 relations
  size_t count_ = 0;
  std::string group_;
  std::vector<int64_t> nid_, nlat_, nlon_;
  std::vector<uint32_t> nkv_;
  std::vector<std::string> strings_{std::string()};   // index 0: the empty string (delimiter)
  std::unordered_map<std::string, uint32_t> sidx_;

  uint32_t sid(const std::string& s) {
    auto it = sidx_.find(s);
    if (it != sidx_.end()) return it->second;
    const uint32_t k = (uint32_t)strings_.size();
    strings_.push_back(s);
    sidx_.emplace(s, k);
    return k;
  }
  void pack_tags(std::string& o, const OsmTags& tags) {
    std::string ks, vs;
    for (const auto& kv : tags) { put_varint(ks, sid(kv.first)); put_varint(vs, sid(kv.second)); }
    put_bytes(o, 2, ks);
    put_bytes(o, 3, vs);
  }
  void blob(const char* type, const std::string& raw) {
    std::string b;
    put_uint(b, 2, raw.size());
    put_bytes(b, 3, deflate_bytes(raw));
    std::string h;
    put_bytes(h, 1, type);
    put_uint(h, 3, b.size());
    const uint32_t n = (uint32_t)h.size();
    const unsigned char len[4] = {(unsigned char)(n >> 24), (unsigned char)(n >> 16), (unsigned char)(n >> 8),
                                  (unsigned char)n};
    if (std::fwrite(len, 1, 4, f_) != 4 || std::fwrite(h.data(), 1, h.size(), f_) != h.size() ||
        std::fwrite(b.data(), 1, b.size(), f_) != b.size())
      throw std::runtime_error("short write on OSM PBF file: " + path_);
  }
  void header() {
    if (header_done_) return;
    header_done_ = true;
    std::string hb;
    if (have_bounds_) {
      std::string bb;
      put_sint(bb, 1, std::llround((double)bb_[0] * 1e9));
      put_sint(bb, 2, std::llround((double)bb_[1] * 1e9));
      put_sint(bb, 3, std::llround((double)bb_[2] * 1e9));
      put_sint(bb, 4, std::llround((double)bb_[3] * 1e9));
      put_bytes(hb, 1, bb);
    }
    put_bytes(hb, 4, "OsmSchema-V0.6");
    put_bytes(hb, 4, "DenseNodes");
    put_bytes(hb, 16, kOsmGenerator);
    blob("OSMHeader", hb);
  }
  void flush() {
    if (kind_ == 1 && !nid_.empty()) {
      std::string d, a;
      int64_t p = 0;
      for (int64_t x : nid_) { put_varint(a, zigzag(x - p)); p = x; }
      put_bytes(d, 1, a);
      a.clear(); p = 0;
      for (int64_t x : nlat_) { put_varint(a, zigzag(x - p)); p = x; }
      put_bytes(d, 8, a);
      a.clear(); p = 0;
      for (int64_t x : nlon_) { put_varint(a, zigzag(x - p)); p = x; }
      put_bytes(d, 9, a);
      a.clear();
      for (uint32_t x : nkv_) put_varint(a, x);
      put_bytes(d, 10, a);
      put_bytes(group_, 2, d);
      nid_.clear(); nlat_.clear(); nlon_.clear(); nkv_.clear();
    }
    if (!group_.empty()) {
      std::string st, blk;
      for (const std::string& x : strings_) put_bytes(st, 1, x);
      put_bytes(blk, 1, st);
      put_bytes(blk, 2, group_);
      put_uint(blk, 17, 1);   // granularity: nanodegrees
      blob("OSMData", blk);
    }
    group_.clear();
    count_ = 0;
    strings_.assign(1, std::string());
    sidx_.clear();
  }
};

}  // namespace

void export_osm_pbf(const Graph& g, const std::string& path) {
  PbfSink s(path);
  emit_osm(g, s);
}

std::unique_ptr<OsmSink> make_osm_pbf_sink(const std::string& path) { return std::make_unique<PbfSink>(path); }

// ---------------------------------------------------------------- reader
OsmParsed parse_osm_pbf(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open OSM PBF file: " + path);
  struct Closer { FILE* f; ~Closer() { std::fclose(f); } } closer{f};
  OsmParsed o;
  bool saw_header = false;
  std::vector<uint64_t> a, b, c, kv;
  std::vector<std::string> st;
  for (;;) {
    unsigned char len[4];
    const size_t got = std::fread(len, 1, 4, f);
    if (got == 0) break;
    if (got != 4) throw std::runtime_error("truncated OSM PBF blob header length");
    const uint32_t hn = (uint32_t)len[0] << 24 | (uint32_t)len[1] << 16 | (uint32_t)len[2] << 8 | len[3];
    if (hn > 64 * 1024) throw std::runtime_error("OSM PBF blob header above 64 KiB");
    std::string h(hn, '\0');
    if (std::fread(&h[0], 1, hn, f) != hn) throw std::runtime_error("truncated OSM PBF blob header");
    std::string type;
    uint64_t datasize = 0;
    {
      Pb q(h);
      uint32_t num, wire;
      uint64_t val = 0;
      const uint8_t* lp = nullptr;
      size_t ln = 0;
      while (q.field(num, wire, val, lp, ln)) {
        if (num == 1 && wire == 2) type.assign((const char*)lp, ln);
        else if (num == 3 && wire == 0) datasize = val;
      }
    }
    if (datasize > (64u << 20)) throw std::runtime_error("OSM PBF blob above 64 MiB");
    std::string bl(datasize, '\0');
    if (datasize && std::fread(&bl[0], 1, datasize, f) != datasize) throw std::runtime_error("truncated OSM PBF blob");
    std::string raw;
    {
      Pb q(bl);
      uint32_t num, wire;
      uint64_t val = 0, raw_size = 0;
      const uint8_t* lp = nullptr;
      size_t ln = 0;
      const uint8_t* zp = nullptr;
      size_t zn = 0;
      bool have_raw = false;
      while (q.field(num, wire, val, lp, ln)) {
        if (num == 1 && wire == 2) { raw.assign((const char*)lp, ln); have_raw = true; }
        else if (num == 2 && wire == 0) raw_size = val;
        else if (num == 3 && wire == 2) { zp = lp; zn = ln; }
        else if (num >= 4 && num <= 7) throw std::runtime_error("OSM PBF blob compression other than zlib");
      }
      if (!have_raw) {
        if (!zp) throw std::runtime_error("OSM PBF blob without data");
        raw = inflate_bytes(zp, zn, (size_t)raw_size);
      }
    }
    if (type == "OSMHeader") {
      Pb q(raw);
      uint32_t num, wire;
      uint64_t val = 0;
      const uint8_t* lp = nullptr;
      size_t ln = 0;
      while (q.field(num, wire, val, lp, ln)) {
        if (num == 4 && wire == 2) {
          const std::string feat((const char*)lp, ln);
          if (feat != "OsmSchema-V0.6" && feat != "DenseNodes" && feat != "HistoricalInformation")
            throw std::runtime_error("OSM PBF requires an unsupported feature: " + feat);
        }
      }
      saw_header = true;
      continue;
    }
    if (type != "OSMData") continue;   // unknown blob types are skipped, as the format allows
    if (!saw_header) throw std::runtime_error("OSM PBF data before its OSMHeader");
    // PrimitiveBlock
    st.clear();
    std::vector<std::pair<const uint8_t*, size_t>> groups;
    int64_t gran = 100, lat_off = 0, lon_off = 0;
    {
      Pb q(raw);
      uint32_t num, wire;
      uint64_t val = 0;
      const uint8_t* lp = nullptr;
      size_t ln = 0;
      while (q.field(num, wire, val, lp, ln)) {
        if (num == 1 && wire == 2) {
          Pb s(lp, ln);
          uint32_t n2, w2;
          uint64_t v2 = 0;
          const uint8_t* p2 = nullptr;
          size_t l2 = 0;
          while (s.field(n2, w2, v2, p2, l2))
            if (n2 == 1 && w2 == 2) st.emplace_back((const char*)p2, l2);
        } else if (num == 2 && wire == 2) {
          groups.push_back({lp, ln});
        } else if (num == 17 && wire == 0) {
          gran = (int64_t)val;
        } else if (num == 19 && wire == 0) {
          lat_off = (int64_t)val;
        } else if (num == 20 && wire == 0) {
          lon_off = (int64_t)val;
        }
      }
    }
    auto str = [&](uint64_t k) -> const std::string& {
      if (k >= st.size()) throw std::runtime_error("OSM PBF string index out of range");
      return st[k];
    };
    auto coord = [&](int64_t off, int64_t v) { return 1e-9 * (double)(off + gran * v); };
    for (const auto& gp : groups) {
      Pb q(gp.first, gp.second);
      uint32_t num, wire;
      uint64_t val = 0;
      const uint8_t* lp = nullptr;
      size_t ln = 0;
      while (q.field(num, wire, val, lp, ln)) {
        if (wire != 2) continue;
        Pb e(lp, ln);
        uint32_t n2, w2;
        uint64_t v2 = 0;
        const uint8_t* p2 = nullptr;
        size_t l2 = 0;
        if (num == 2) {   // DenseNodes
          a.clear(); b.clear(); c.clear(); kv.clear();
          while (e.field(n2, w2, v2, p2, l2)) {
            if (n2 == 1) unpack(w2, v2, p2, l2, a);
            else if (n2 == 8) unpack(w2, v2, p2, l2, b);
            else if (n2 == 9) unpack(w2, v2, p2, l2, c);
            else if (n2 == 10) unpack(w2, v2, p2, l2, kv);
          }
          if (b.size() != a.size() || c.size() != a.size()) throw std::runtime_error("malformed OSM PBF dense nodes");
          int64_t id = 0, la = 0, lo = 0;
          size_t k = 0;
          for (size_t i = 0; i < a.size(); ++i) {
            id += unzigzag(a[i]);
            la += unzigzag(b[i]);
            lo += unzigzag(c[i]);
            float flat = (float)coord(lat_off, la), flon = (float)coord(lon_off, lo);
            while (k < kv.size() && kv[k] != 0) {   // this node's tags, then its 0 delimiter
              if (k + 1 >= kv.size()) throw std::runtime_error("malformed OSM PBF dense node tags");
              if (str(kv[k]) == "reporter:ll") {
                double dla = 0, dlo = 0;
                if (std::sscanf(str(kv[k + 1]).c_str(), "%la %la", &dla, &dlo) != 2)
                  throw std::runtime_error("bad reporter:ll tag");
                flat = (float)dla;
                flon = (float)dlo;
              }
              k += 2;
            }
            ++k;
            if (id < 0) throw std::runtime_error("negative OSM node id");
            o.nodes.push_back({(uint64_t)id, {flon, flat}});
          }
        } else if (num == 1) {   // plain Node
          int64_t id = 0, la = 0, lo = 0;
          while (e.field(n2, w2, v2, p2, l2)) {
            if (n2 == 1 && w2 == 0) id = unzigzag(v2);
            else if (n2 == 8 && w2 == 0) la = unzigzag(v2);
            else if (n2 == 9 && w2 == 0) lo = unzigzag(v2);
          }
          if (id < 0) throw std::runtime_error("negative OSM node id");
          o.nodes.push_back({(uint64_t)id, {(float)coord(lon_off, lo), (float)coord(lat_off, la)}});
        } else if (num == 3) {   // Way
          OsmParsedWay w{0, {}, {}};
          a.clear(); b.clear(); c.clear();
          while (e.field(n2, w2, v2, p2, l2)) {
            if (n2 == 1 && w2 == 0) w.id = v2;
            else if (n2 == 2) unpack(w2, v2, p2, l2, a);
            else if (n2 == 3) unpack(w2, v2, p2, l2, b);
            else if (n2 == 8) unpack(w2, v2, p2, l2, c);
          }
          if (a.size() != b.size()) throw std::runtime_error("malformed OSM PBF way tags");
          for (size_t i = 0; i < a.size(); ++i) w.tags[str(a[i])] = str(b[i]);
          int64_t r = 0;
          for (uint64_t d : c) {
            r += unzigzag(d);
            if (r < 0) throw std::runtime_error("negative OSM node ref");
            w.refs.push_back((uint64_t)r);
          }
          o.ways.push_back(std::move(w));
        } else if (num == 4) {   // Relation
          OsmParsedRelation rl{0, {}, {}};
          std::vector<uint64_t> roles, ids, types;
          a.clear(); b.clear();
          while (e.field(n2, w2, v2, p2, l2)) {
            if (n2 == 1 && w2 == 0) rl.id = v2;
            else if (n2 == 2) unpack(w2, v2, p2, l2, a);
            else if (n2 == 3) unpack(w2, v2, p2, l2, b);
            else if (n2 == 8) unpack(w2, v2, p2, l2, roles);
            else if (n2 == 9) unpack(w2, v2, p2, l2, ids);
            else if (n2 == 10) unpack(w2, v2, p2, l2, types);
          }
          if (a.size() != b.size() || roles.size() != ids.size() || types.size() != ids.size())
            throw std::runtime_error("malformed OSM PBF relation");
          for (size_t i = 0; i < a.size(); ++i) rl.tags[str(a[i])] = str(b[i]);
          int64_t m = 0;
          for (size_t i = 0; i < ids.size(); ++i) {
            m += unzigzag(ids[i]);
            if (m < 0) throw std::runtime_error("negative OSM member ref");
            const char* ty = types[i] == 0 ? "node" : (types[i] == 1 ? "way" : "relation");
            rl.members.push_back({ty, str(roles[i]), (uint64_t)m});
          }
          o.rels.push_back(std::move(rl));
        }
      }
    }
  }
  if (!saw_header) throw std::runtime_error("not an OSM PBF file: " + path);
  return o;
}

}  // namespace rm
