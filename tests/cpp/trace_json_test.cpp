// Host test of the single-pass Match-request reader (reporter_amd/csrc/trace_json.hpp): over
// generated requests, mutations and every prefix of small documents it must return exactly
// what the DOM reader path (json.hpp + the checks capi.cpp made before round 3, restated in
// dom_parse below) returns — the same points bit for bit and the same options, or the same
// error message.  Also: replies formatted with to_chars parse back to the doubles "%.17g" gives.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "json.hpp"
#include "json_points.hpp"
#include "trace_json.hpp"

using namespace rm;

namespace {

struct Parsed {
  bool ok = false;
  std::string err;
  std::vector<float> lon, lat, acc;
  std::vector<double> time;
  MatchOptions opt{};
};

const char* kModes[5] = {"auto", "bus", "motor_scooter", "bicycle", "pedestrian"};

// the DOM path (capi.cpp parse_trace / apply_options of round 2)
void dom_apply(const json::Value* o, MatchOptions& m) {
  if (!o || o->type != json::Value::Object) return;
  auto num = [&](const char* k, float& dst) {
    const json::Value* v = o->get(k);
    if (v && v->is_num()) dst = (float)v->num;
    else if (v && v->type != json::Value::Null) throw std::runtime_error(std::string("match option ") + k + " must be a number");
  };
  num("sigma_z", m.sigma_z);
  num("beta", m.beta);
  num("search_radius", m.search_radius);
  num("gps_accuracy", m.gps_accuracy);
  num("breakage_distance", m.breakage_distance);
  num("interpolation_distance", m.interpolation_distance);
  num("max_route_distance_factor", m.max_route_distance_factor);
  num("max_route_time_factor", m.max_route_time_factor);
  num("turn_penalty_factor", m.turn_penalty_factor);
  if (!(m.sigma_z > 0.f) || !std::isfinite(m.sigma_z)) throw std::runtime_error("sigma_z must be positive");
  if (!(m.beta > 0.f) || !std::isfinite(m.beta)) throw std::runtime_error("beta must be positive");
  if (!(m.search_radius >= 0.f)) throw std::runtime_error("search_radius must be non-negative");
  if (!turn_factor_ok(m.turn_penalty_factor)) throw std::runtime_error(kTurnPenaltyError);
}

Parsed dom_parse(const char* text, const MatchOptions* defaults) {
  Parsed t;
  try {
    json::Value v = json::parse(text);
    if (v.type != json::Value::Object) throw std::runtime_error("trace request must be a JSON object");
    const json::Value* mo = v.get("match_options");
    int mode = kModeAuto;
    if (mo && mo->type == json::Value::Object) {
      const json::Value* mv = mo->get("mode");
      if (mv && mv->type == json::Value::String) {
        mode = -1;
        for (int m = 0; m < 5; ++m)
          if (mv->str == kModes[m]) mode = m;
        if (mode < 0) throw std::runtime_error("unsupported mode: " + mv->str);
      }
    }
    t.opt = defaults[mode];
    t.opt.mode = mode;
    dom_apply(mo, t.opt);
    const json::Value* tr = v.get("trace");
    if (!tr || tr->type != json::Value::Array) throw std::runtime_error("trace must be an array of points");
    if (tr->arr.empty()) throw std::runtime_error("trace must contain at least one point");
    for (const json::Value& p : tr->arr) {
      const json::Value* la = p.get("lat");
      const json::Value* lo = p.get("lon");
      if (!la || !lo || !la->is_num() || !lo->is_num()) throw std::runtime_error("each trace point needs numeric lat and lon");
      if (!(la->num >= -90.0 && la->num <= 90.0 && lo->num >= -180.0 && lo->num <= 180.0))
        throw std::runtime_error("trace point out of range");
      t.lat.push_back((float)la->num);
      t.lon.push_back((float)lo->num);
      const json::Value* tm = p.get("time");
      t.time.push_back((tm && tm->is_num()) ? tm->num : -1.0);
      const json::Value* ac = p.get("accuracy");
      t.acc.push_back((ac && ac->is_num()) ? (float)ac->num : -1.0f);
    }
    t.ok = true;
  } catch (const std::exception& e) {
    t.err = e.what();
  }
  return t;
}

Parsed fast_parse(const char* text, const MatchOptions* defaults, tj::PointSink& sink) {
  Parsed t;
  const size_t n0 = sink.size();
  try {
    t.opt = tj::parse_request(text, defaults, sink);
    t.ok = true;
    t.lon.assign(sink.lon.begin() + n0, sink.lon.end());
    t.lat.assign(sink.lat.begin() + n0, sink.lat.end());
    t.acc.assign(sink.acc.begin() + n0, sink.acc.end());
    t.time.assign(sink.time.begin() + n0, sink.time.end());
  } catch (const std::exception& e) {
    t.err = e.what();
    if (sink.size() != n0) t.err += " [sink changed on error]";
  }
  return t;
}

// rm_match_batch's device path for one request (capi.cpp match_json_batch_device): the host reads
// the structure leaving a compact-looking trace array to the device, the device rules
// (json_points.hpp, here run on the host in k_parse_json's order) read its points, and anything
// they reject is parsed again by the generic reader.  `accepted` counts requests the device kept.
Parsed device_parse(const char* text, const MatchOptions* defaults, size_t& accepted) {
  tj::PointSink sk;
  tj::TraceSpan sp;
  Parsed t;
  try {
    t.opt = tj::parse_request_deferred(text, std::strlen(text), defaults, sk, sp);
  } catch (const std::exception&) {
    tj::PointSink fresh;
    return fast_parse(text, defaults, fresh);
  }
  if (!sp.on) {
    t.ok = true;
    t.lon = sk.lon; t.lat = sk.lat; t.acc = sk.acc; t.time = sk.time;
    return t;
  }
  const uint8_t* s = reinterpret_cast<const uint8_t*>(sp.b);
  const uint64_t e = (uint64_t)(sp.e - sp.b);
  bool bad = false;
  uint32_t idx = 0;
  for (uint64_t i = 0; i < e && !bad; ++i) {
    if (s[i] != '{') continue;
    uint64_t q = i;
    double la = 0, lo = 0, tm = 0, ac = 0;
    if (!jp::point(s, q, e, la, lo, tm, ac) || !jp::point_follows(s, q, e) || !jp::in_range(la, lo) || idx >= sp.n_open) {
      bad = true;
      break;
    }
    t.lat.push_back((float)la); t.lon.push_back((float)lo); t.time.push_back(tm); t.acc.push_back((float)ac);
    ++idx;
  }
  if (bad || idx != sp.n_open) {
    tj::PointSink fresh;
    return fast_parse(text, defaults, fresh);
  }
  ++accepted;
  t.ok = true;
  return t;
}

// requests in the layout bench.py and json.dumps(separators=(',', ':')) write: every trace compact
std::string gen_compact(std::mt19937_64& rng, int npts) {
  std::uniform_real_distribution<double> ulat(-89.0, 89.0), ulon(-179.0, 179.0), uacc(0.0, 120.0);
  std::string s = "{\"uuid\":\"" + std::to_string(rng() % 100000) + "\",\"trace\":[";
  char b[64];
  for (int i = 0; i < npts; ++i) {
    std::vector<std::string> kv;
    const int f = (int)(rng() % 4);
    auto num = [&](double x) {
      if (f == 0) std::snprintf(b, sizeof b, "%.6f", x);
      else if (f == 1) std::snprintf(b, sizeof b, "%.13g", x);
      else if (f == 2) std::snprintf(b, sizeof b, "%.0f", x);
      else std::snprintf(b, sizeof b, "%.9f", x);
      return std::string(b);
    };
    kv.push_back("\"lat\":" + num(ulat(rng)));
    kv.push_back("\"lon\":" + num(ulon(rng)));
    kv.push_back("\"time\":" + std::to_string(1483228800 + i * (1 + rng() % 30)));
    kv.push_back("\"accuracy\":" + num(uacc(rng)));
    if (rng() % 3 == 0)
      for (size_t a = kv.size(); a > 1; --a) std::swap(kv[a - 1], kv[rng() % a]);
    s += i ? ",{" : "{";
    for (size_t a = 0; a < kv.size(); ++a) s += (a ? "," : "") + kv[a];
    s += "}";
  }
  s += "],\"match_options\":{\"mode\":\"" + std::string(kModes[rng() % 5]) + "\",\"report_levels\":[0,1]}}";
  return s;
}

bool same_bits(const void* a, const void* b, size_t n) { return std::memcmp(a, b, n) == 0; }

bool same(const Parsed& a, const Parsed& b, std::string& why) {
  if (a.ok != b.ok) { why = "ok " + std::to_string(a.ok) + " vs " + std::to_string(b.ok) + " (" + a.err + " | " + b.err + ")"; return false; }
  if (!a.ok) {
    if (a.err != b.err) { why = "error '" + a.err + "' vs '" + b.err + "'"; return false; }
    return true;
  }
  if (a.lon.size() != b.lon.size()) { why = "point count"; return false; }
  const size_t n = a.lon.size();
  if (!same_bits(a.lon.data(), b.lon.data(), n * 4) || !same_bits(a.lat.data(), b.lat.data(), n * 4) ||
      !same_bits(a.acc.data(), b.acc.data(), n * 4) || !same_bits(a.time.data(), b.time.data(), n * 8)) {
    why = "point values";
    return false;
  }
  if (!same_bits(&a.opt, &b.opt, sizeof(MatchOptions))) { why = "options"; return false; }
  return true;
}

std::string fmt_num(std::mt19937_64& rng, double x) {
  char b[64];
  switch (rng() % 6) {
    case 0: std::snprintf(b, sizeof b, "%.6f", x); break;
    case 1: std::snprintf(b, sizeof b, "%.17g", x); break;
    case 2: std::snprintf(b, sizeof b, "%.9e", x); break;
    case 3: std::snprintf(b, sizeof b, "%.3f", x); break;
    case 4: std::snprintf(b, sizeof b, "%.12g", x); break;
    default: std::snprintf(b, sizeof b, "%.20f", x); break;
  }
  return b;
}

std::string gen_request(std::mt19937_64& rng, int npts) {
  std::uniform_real_distribution<double> ulat(-89.0, 89.0), ulon(-179.0, 179.0), uacc(0.0, 120.0);
  std::string s = "{\"uuid\":\"veh" + std::to_string(rng() % 100000) + "\"";
  auto sep = [&]() { return (rng() % 5 == 0) ? std::string(" \n\t") : std::string(); };
  std::string pts = "\"trace\":" + sep() + "[";
  for (int i = 0; i < npts; ++i) {
    if (i) pts += "," + sep();
    std::vector<std::string> kv;
    kv.push_back("\"lat\":" + fmt_num(rng, ulat(rng)));
    kv.push_back("\"lon\":" + fmt_num(rng, ulon(rng)));
    if (rng() % 8) kv.push_back("\"time\":" + std::to_string(1483228800 + i * (1 + rng() % 30)));
    if (rng() % 4) kv.push_back("\"accuracy\":" + fmt_num(rng, uacc(rng)));
    if (rng() % 20 == 0) kv.push_back("\"extra\":{\"a\":[1,2,{\"b\":null}],\"c\":\"x\\u00e9\"}");
    if (rng() % 30 == 0) kv.push_back("\"l\\u0061t\":" + fmt_num(rng, ulat(rng)));   // escaped duplicate
    for (size_t a = kv.size(); a > 1; --a) std::swap(kv[a - 1], kv[rng() % a]);
    pts += "{";
    for (size_t a = 0; a < kv.size(); ++a) pts += (a ? "," : "") + sep() + kv[a];
    pts += "}";
  }
  pts += "]";
  std::string mo = "\"match_options\":{";
  std::vector<std::string> opts;
  opts.push_back("\"mode\":\"" + std::string(kModes[rng() % 5]) + "\"");
  opts.push_back("\"report_levels\":[0,1]");
  opts.push_back("\"transition_levels\":[0,1]");
  if (rng() % 2) opts.push_back("\"sigma_z\":" + fmt_num(rng, 1.0 + (rng() % 1000) / 100.0));
  if (rng() % 2) opts.push_back("\"beta\":" + fmt_num(rng, 0.5 + (rng() % 100) / 10.0));
  if (rng() % 2) opts.push_back("\"search_radius\":" + std::to_string(rng() % 200));
  if (rng() % 3 == 0) opts.push_back("\"breakage_distance\":" + std::to_string(500 + rng() % 5000));
  if (rng() % 4 == 0) opts.push_back(rng() % 3 ? "\"turn_penalty_factor\":0" : "\"turn_penalty_factor\":200");
  if (rng() % 6 == 0) opts.push_back("\"gps_accuracy\":null");
  for (size_t a = opts.size(); a > 1; --a) std::swap(opts[a - 1], opts[rng() % a]);
  for (size_t a = 0; a < opts.size(); ++a) mo += (a ? "," : "") + opts[a];
  mo += "}";
  std::vector<std::string> top = {pts, mo};
  if (rng() % 2) std::swap(top[0], top[1]);
  for (auto& x : top) s += "," + sep() + x;
  s += "}";
  return s;
}

}  // namespace

#define CHECK(c, msg)                                                              \
  do {                                                                             \
    if (!(c)) {                                                                    \
      std::fprintf(stderr, "FAILED %s: %s\n", #c, std::string(msg).c_str());       \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

int main() {
  MatchOptions defaults[5];
  for (int m = 0; m < 5; ++m) {
    defaults[m] = default_options();
    defaults[m].mode = m;
    defaults[m].search_radius = 50.f + 10.f * m;
  }
  std::mt19937_64 rng(12345);
  tj::PointSink sink;
  std::string why;
  size_t n_ok = 0, n_err = 0, n_docs = 0, dev_kept = 0;
  // every document also through the device path: the same result as the DOM reader
  auto check_device = [&](const char* doc, const Parsed& want) {
    const Parsed d = device_parse(doc, defaults, dev_kept);
    return same(want, d, why);
  };
  // 1. generated valid requests (+ their options), appended one after another to one sink
  for (int it = 0; it < 3000; ++it) {
    const std::string doc = gen_request(rng, 1 + (int)(rng() % 40));
    const Parsed a = dom_parse(doc.c_str(), defaults), b = fast_parse(doc.c_str(), defaults, sink);
    CHECK(same(a, b, why), why + " in " + doc.substr(0, 300));
    CHECK(check_device(doc.c_str(), a), "device path: " + why + " in " + doc.substr(0, 300));
    ++n_docs;
    (a.ok ? n_ok : n_err)++;
  }
  CHECK(n_ok > 2300, "too few valid documents");
  // turn costs (DESIGN.md rule 3b): any non-negative finite factor is accepted (0, null, meili's
  // per-mode 200 / 140 / 100); a negative one fails as meili's TransitionCostModel does, and so
  // does one that overflows to infinity
  {
    const char* base = "{\"uuid\":\"1\",\"trace\":[{\"lat\":1,\"lon\":2,\"time\":3}],\"match_options\":{%s}}";
    char doc[256];
    for (const char* o : {"\"turn_penalty_factor\":200", "\"turn_penalty_factor\":-1e-30", "\"turn_penalty_factor\":0",
                          "\"turn_penalty_factor\":null", "\"turn_penalty_factor\":1e39", "\"turn_penalty_factor\":140.5"}) {
      std::snprintf(doc, sizeof doc, base, o);
      const Parsed a = dom_parse(doc, defaults), b = fast_parse(doc, defaults, sink);
      CHECK(same(a, b, why), why + " in " + doc);
      const bool want_ok = !std::strstr(o, ":-") && !std::strstr(o, "e39");
      CHECK(b.ok == want_ok && (want_ok || b.err == kTurnPenaltyError), std::string(doc) + " -> " + b.err);
    }
  }
  // 2. mutations: one byte replaced / deleted / inserted, and every prefix of small documents
  const char* alphabet = "{}[]\":,0123456789.-eE+ \\ulnt\x01";
  for (int it = 0; it < 4000; ++it) {
    std::string doc = gen_request(rng, 1 + (int)(rng() % 4));
    const size_t pos = rng() % doc.size();
    const char ch = alphabet[rng() % std::strlen(alphabet)];
    switch (rng() % 3) {
      case 0: doc[pos] = ch; break;
      case 1: doc.erase(pos, 1); break;
      default: doc.insert(doc.begin() + (long)pos, ch); break;
    }
    const Parsed a = dom_parse(doc.c_str(), defaults), b = fast_parse(doc.c_str(), defaults, sink);
    CHECK(same(a, b, why), why + " in " + doc);
    CHECK(check_device(doc.c_str(), a), "device path: " + why + " in " + doc);
    ++n_docs;
    (a.ok ? n_ok : n_err)++;
  }
  // compact requests (the device parser's layout), whole and mutated
  const size_t kept0 = dev_kept;
  for (int it = 0; it < 3000; ++it) {
    std::string doc = gen_compact(rng, 1 + (int)(rng() % 30));
    if (it % 2) {
      const size_t pos = rng() % doc.size();
      const char ch = alphabet[rng() % std::strlen(alphabet)];
      switch (rng() % 3) {
        case 0: doc[pos] = ch; break;
        case 1: doc.erase(pos, 1); break;
        default: doc.insert(doc.begin() + (long)pos, ch); break;
      }
    }
    const Parsed a = dom_parse(doc.c_str(), defaults), b = fast_parse(doc.c_str(), defaults, sink);
    CHECK(same(a, b, why), why + " in " + doc.substr(0, 300));
    CHECK(check_device(doc.c_str(), a), "device path: " + why + " in " + doc.substr(0, 300));
    ++n_docs;
    (a.ok ? n_ok : n_err)++;
  }
  CHECK(dev_kept - kept0 > 1400, "the device path kept too few compact requests: " + std::to_string(dev_kept - kept0));
  for (int it = 0; it < 60; ++it) {
    const std::string doc = gen_request(rng, 2);
    for (size_t k = 0; k <= doc.size(); ++k) {
      const std::string pre = doc.substr(0, k);
      const Parsed a = dom_parse(pre.c_str(), defaults), b = fast_parse(pre.c_str(), defaults, sink);
      CHECK(same(a, b, why), why + " in prefix " + pre);
      CHECK(check_device(pre.c_str(), a), "device path: " + why + " in prefix " + pre);
      ++n_docs;
    }
  }
  // 3. hand-written semantic cases
  const char* cases[] = {
      "[1,2]", "\"x\"", "{}", "{\"trace\":[]}", "{\"trace\":{}}", "{\"trace\":[1]}", "{\"trace\":[{\"lat\":1}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":\"2\"}]}", "{\"trace\":[{\"lat\":91,\"lon\":2}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}],\"match_options\":{\"mode\":\"boat\"}}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}],\"match_options\":{\"mode\":7}}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}],\"match_options\":{\"sigma_z\":\"a\"}}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}],\"match_options\":{\"sigma_z\":0}}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}],\"match_options\":{\"beta\":-1,\"sigma_z\":\"x\"}}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}],\"match_options\":{\"search_radius\":-1}}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}],\"match_options\":[]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}],\"match_options\":{\"beta\":null}}",
      "{\"trace\":[{\"lat\":1,\"lon\":2,\"time\":\"t\",\"accuracy\":null}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2,\"lat\":3}]}", "{\"trace\":[{\"lat\":\"a\",\"lon\":2,\"lat\":3}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}],\"trace\":5}", "{\"trace\":5,\"trace\":[{\"lat\":1,\"lon\":2}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2},{\"lat\":100,\"lon\":2},{\"lon\":1}]}",
      "{\"trace\":[{\"lat\":1e400,\"lon\":2}]}", "{\"trace\":[{\"lat\":-0,\"lon\":-0.0}]}",
      "{\"trace\":[{\"lat\":12.345678901234567890123,\"lon\":1.7976931348623157e308}]}",
      "{\"trace\":[{\"lat\":0.000000000000000000000000001,\"lon\":1e-400}]}",
      "{\"trace\":[{\"lat\":01,\"lon\":2}]}", "{\"trace\":[{\"lat\":1.,\"lon\":2}]}", "{\"trace\":[{\"lat\":.5,\"lon\":2}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}]} x", "{\"trace\":[{\"lat\":1,\"lon\":2}],}", " \n{\"trace\":[{\"lat\":1,\"lon\":2}]}\n ",
      "{\"tr\\u0061ce\":[{\"lat\":1,\"lon\":2}],\"match_options\":{\"mo\\u0064e\":\"bicycle\"}}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}],\"match_options\":{\"mode\":\"bicycle\",\"mode\":\"boat\"}}",
      "{\"trace\":[{\"lat\":1,\"lon\":2}],\"match_options\":{\"mode\":\"pedestrian\"},\"match_options\":{\"mode\":\"boat\"}}",
      "{\"a\":[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[1]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]],\"trace\":[{\"lat\":1,\"lon\":2}]}",
      "{\"s\":\"\\ud83d\\ude00\\n\\t\\\"\",\"trace\":[{\"lat\":1,\"lon\":2}]}", "{\"s\":\"\\x\"}", "{\"s\":\"ab", "",
      "{\"trace\":[{\"lat\":4.9e-324,\"lon\":123456789012345678}]}", "{\"trace\":[{\"lat\":1E+2,\"lon\":2e-0}]}",
      // the compact point layout (trace_json.hpp point_compact) and its fall-backs
      "{\"trace\":[{\"lat\":1.5,\"lon\":2,\"time\":3,\"accuracy\":4}]}",
      "{\"trace\":[{\"accuracy\":4,\"time\":3.25,\"lon\":-2.125,\"lat\":-1.5}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2,\"time\":3,\"accuracy\":4,\"lat\":5}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2,\"time\":3,\"accuracy\":4,\"x\":5}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2,\"time\":null,\"accuracy\":4}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2,\"time\":3,\"accuracy\":4 }]}",
      "{\"trace\":[{\"lat\":-,\"lon\":2,\"time\":3,\"accuracy\":4}]}",
      "{\"trace\":[{\"lat\":1.,\"lon\":2,\"time\":3,\"accuracy\":4}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2e1,\"time\":3,\"accuracy\":4}]}",
      "{\"trace\":[{\"lat\":91,\"lon\":2,\"time\":3,\"accuracy\":4},{\"lat\":1,\"lon\":2,\"time\":3,\"accuracy\":4}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2,\"time\":1234567890.12345,\"accuracy\":4}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2,\"time\":1234567890.123456,\"accuracy\":4}]}",
      "{\"trace\":[{\"lat\":1,\"lon\":2,\"time\":3,\"accuracy\":4}",
  };
  for (const char* c : cases) {
    const Parsed a = dom_parse(c, defaults), b = fast_parse(c, defaults, sink);
    CHECK(same(a, b, why), why + " in " + c);
    CHECK(check_device(c, a), std::string("device path: ") + why + " in " + c);
    ++n_docs;
  }
  // 4. replies: to_chars digits parse back to the same doubles as %.17g
  std::uniform_real_distribution<double> ut(1.4e9, 1.6e9);
  for (int it = 0; it < 200000; ++it) {
    double x = ut(rng);
    if (it % 3 == 0) x = std::floor(x);
    if (it % 7 == 0) x = std::ldexp((double)(rng() >> 11), -(int)(rng() % 60));
    std::string o;
    tj::put_num(o, x);
    char b17[40];
    std::snprintf(b17, sizeof b17, "%.17g", x);
    const double y = std::strtod(o.c_str(), nullptr), z = std::strtod(b17, nullptr);
    CHECK(std::memcmp(&y, &z, 8) == 0 && std::memcmp(&y, &x, 8) == 0, o + " vs " + b17);
  }
  std::printf("trace json ok: %zu documents (%zu valid, %zu errors), %zu kept by the device path\n", n_docs, n_ok,
              n_err, dev_kept);
  return 0;
}
