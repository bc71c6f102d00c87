// trace_json.hpp — the /report boundary's hot host path: one validating pass over a Match
// request that writes its points straight into batch arrays, and the reply formatter.
//
// Match's request is the JSON reporter_service.py:240 sends (json.dumps of the /report trace,
// separators ',' ':'): {"uuid", "trace": [{"lat","lon","time","accuracy"}...], "match_options":
// {mode, sigma_z, ...}}.  The DOM reader (json.hpp) allocated a string per key
// and a vector per value; at 600 points per trace that made host parsing ~1 % of the engine's
// rate.  This reader keeps the DOM reader's contract exactly (tests/cpp/trace_json_test.cpp runs
// both over the same documents):
//   * the whole document is validated first; a syntax error is reported as "invalid JSON (...)
//     at offset N" before any semantic error;
//   * keys compare after unescaping, the FIRST occurrence of a key counts;
//   * numbers convert to the double a correctly rounded strtod gives (Clinger's exact fast path
//     for <= 15 significant digits and |10-exponent| <= 22, strtod otherwise), then lat/lon/
//     accuracy to float as Valhalla's PointLL does;
//   * semantic errors in the DOM reader's order: not an object, mode, options, trace, points.
// Replies are formatted with std::to_chars (shortest round-trip digits: the same doubles as
// "%.17g" once parsed — the consumer is json.loads, reporter_service.py:241).
#pragma once
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "rm_common.hpp"
#include <limits>

namespace rm {

// the 16-19 digit number path below reads an x87 extended significand
constexpr bool kX87LongDouble = std::numeric_limits<long double>::digits == 64 && sizeof(long double) >= 10;
namespace tj {

// A trace array left for the device parser (rm_match_batch, round 4): the bytes strictly between
// its '[' and the first ']' after it, and the number of '{' in them.  Only a compact trace
// (point_compact's layout, points separated by single commas) is kept by the device parser; it
// flags anything else, and the request is then parsed again by the generic reader.
struct TraceSpan {
  const char* b = nullptr;
  const char* e = nullptr;
  uint32_t n_open = 0;
  bool on = false;
};

// points of many traces, appended in order (one sink per host thread)
struct PointSink {
  std::vector<float> lon, lat, acc;
  std::vector<double> time;
  void clear() { lon.clear(); lat.clear(); acc.clear(); time.clear(); }
  size_t size() const { return lon.size(); }
};

inline int mode_index(const char* s, size_t n) {
  auto eq = [&](const char* m) { return std::strlen(m) == n && std::memcmp(s, m, n) == 0; };
  if (eq("auto")) return kModeAuto;
  if (eq("bus")) return kModeBus;
  if (eq("motor_scooter")) return kModeMotorScooter;
  if (eq("bicycle")) return kModeBicycle;
  if (eq("pedestrian")) return kModePedestrian;
  return -1;
}

class Reader {
 public:
  Reader(const char* s, size_t len, const MatchOptions* mode_defaults, TraceSpan* defer = nullptr)
      : p_(s), s0_(s), end_(s + len), defaults_(mode_defaults), defer_(defer) {}

  // Parse one request; its points are appended to `sink` (only when the request is valid).
  MatchOptions request(PointSink& sink) {
    const size_t n0 = sink.size();
    try {
      parse_document(sink);
    } catch (...) {
      truncate(sink, n0);
      throw;
    }
    // semantic errors, in the order the DOM reader checks them
    std::string err;
    if (!top_object_) err = "trace request must be a JSON object";
    else if (!mode_err_.empty()) err = mode_err_;
    if (err.empty()) {
      MatchOptions o = defaults_[mode_];
      o.mode = mode_;
      for (int k = 0; k < kNumOpt; ++k) {
        if (opt_state_[k] == 2) { err = std::string("match option ") + kOptNames[k] + " must be a number"; break; }
        if (opt_state_[k] == 1) *opt_field(o, k) = (float)opt_val_[k];
      }
      if (err.empty()) {
        if (!(o.sigma_z > 0.f) || !std::isfinite(o.sigma_z)) err = "sigma_z must be positive";
        else if (!(o.beta > 0.f) || !std::isfinite(o.beta)) err = "beta must be positive";
        else if (!(o.search_radius >= 0.f)) err = "search_radius must be non-negative";
        else if (!turn_factor_ok(o.turn_penalty_factor)) err = kTurnPenaltyError;
      }
      if (err.empty()) {
        if (trace_state_ == 0 || trace_state_ == 2) err = "trace must be an array of points";
        else if (sink.size() == n0 && point_err_.empty() && !(defer_ && defer_->on))
          err = "trace must contain at least one point";
        else if (!point_err_.empty()) err = point_err_;
      }
      if (err.empty()) return o;
    }
    truncate(sink, n0);
    throw std::runtime_error(err);
  }

 private:
  static constexpr int kNumOpt = 9;
  static constexpr const char* kOptNames[kNumOpt] = {"sigma_z", "beta", "search_radius", "gps_accuracy",
                                                     "breakage_distance", "interpolation_distance",
                                                     "max_route_distance_factor", "max_route_time_factor",
                                                     "turn_penalty_factor"};
  static float* opt_field(MatchOptions& o, int k) {
    float* f[kNumOpt] = {&o.sigma_z, &o.beta, &o.search_radius, &o.gps_accuracy, &o.breakage_distance,
                         &o.interpolation_distance, &o.max_route_distance_factor, &o.max_route_time_factor,
                         &o.turn_penalty_factor};
    return f[k];
  }

  const char* p_;
  const char* s0_;
  const char* end_;   // the terminating NUL (word-wide reads stay before it)
  const MatchOptions* defaults_;
  TraceSpan* defer_;             // non-null: a trace array that may be compact is left to the device
  bool top_object_ = false;
  int trace_state_ = 0;          // 0 absent, 1 array seen, 2 first "trace" value not an array
  bool opts_seen_ = false;       // first "match_options" handled
  bool mode_seen_ = false;
  int mode_ = kModeAuto;
  std::string mode_err_, point_err_;
  int opt_state_[kNumOpt] = {};  // 0 absent / null, 1 number, 2 wrong type (first occurrence)
  double opt_val_[kNumOpt] = {};
  bool opt_seen_[kNumOpt] = {};

  static void truncate(PointSink& s, size_t n) {
    s.lon.resize(n); s.lat.resize(n); s.acc.resize(n); s.time.resize(n);
  }
  [[noreturn]] void fail(const char* m) {
    throw std::runtime_error(std::string("invalid JSON (") + m + ") at offset " + std::to_string(p_ - s0_));
  }
  void ws() { while (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r') ++p_; }

  // ---- strings: a key is decoded into `out` (small), a skipped string only validated
  static void utf8(std::string& o, uint32_t c) {
    if (c < 0x80) o += (char)c;
    else if (c < 0x800) { o += (char)(0xc0 | (c >> 6)); o += (char)(0x80 | (c & 0x3f)); }
    else if (c < 0x10000) { o += (char)(0xe0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 0x3f)); o += (char)(0x80 | (c & 0x3f)); }
    else { o += (char)(0xf0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 0x3f)); o += (char)(0x80 | ((c >> 6) & 0x3f)); o += (char)(0x80 | (c & 0x3f)); }
  }
  uint32_t hex4() {
    uint32_t c = 0;
    for (int i = 0; i < 4; ++i) {
      const char h = *p_++;
      c <<= 4;
      if (h >= '0' && h <= '9') c |= h - '0';
      else if (h >= 'a' && h <= 'f') c |= h - 'a' + 10;
      else if (h >= 'A' && h <= 'F') c |= h - 'A' + 10;
      else fail("bad \\u escape");
    }
    return c;
  }
  // string at p_ (on its opening quote).  Fast path: no escape -> [*b, *e) points into the text.
  // With escapes the decoded text goes to `tmp` and [*b, *e) points into it.
  void string(const char** b, const char** e, std::string& tmp) {
    ++p_;
    const char* st = p_;
    for (;;) {
      const unsigned char c = (unsigned char)*p_;
      if (c == '"') { *b = st; *e = p_; ++p_; return; }
      if (c == '\\') break;
      if (c == 0) { ++p_; fail("unterminated string"); }
      if (c < 0x20) { ++p_; fail("control character in string"); }
      ++p_;
    }
    tmp.assign(st, p_);
    for (;;) {
      const char c = *p_++;
      if (c == '"') { *b = tmp.data(); *e = tmp.data() + tmp.size(); return; }
      if (c == 0) fail("unterminated string");
      if ((unsigned char)c < 0x20) fail("control character in string");
      if (c != '\\') { tmp += c; continue; }
      const char x = *p_++;
      switch (x) {
        case '"': tmp += '"'; break;
        case '\\': tmp += '\\'; break;
        case '/': tmp += '/'; break;
        case 'b': tmp += '\b'; break;
        case 'f': tmp += '\f'; break;
        case 'n': tmp += '\n'; break;
        case 'r': tmp += '\r'; break;
        case 't': tmp += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xd800 && cp < 0xdc00 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            const uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xd800) << 10) + (lo - 0xdc00);
          }
          utf8(tmp, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
  }

  // ---- numbers: the token is validated exactly as the DOM reader does, and converted to the
  // correctly rounded double (what strtod returns) without strtod in the common cases
  static bool digit(char c) { return (unsigned)(c - '0') < 10u; }
  // the value of eight ASCII digits (SWAR; p_[0], the low byte, is the most significant)
  static uint32_t eight_value(uint64_t v) {
    v -= 0x3030303030303030ull;
    v = v * 10u + (v >> 8);
    v = (((v & 0x000000FF000000FFull) * 0x000F424000000064ull) +
         (((v >> 16) & 0x000000FF000000FFull) * 0x0000271000000001ull)) >> 32;
    return (uint32_t)v;
  }
  // digits at p_ into m (wrapping past 19 digits: the caller checks the count).  Eight bytes at
  // a time: the run of digits at the front of the word is found from a per-byte non-digit mask
  // and converted in one go (the bytes after it replaced by leading '0's), no loop per digit.
  void digits(uint64_t& m) {
    static const uint64_t kPow10u[9] = {1u, 10u, 100u, 1000u, 10000u, 100000u, 1000000u, 10000000u, 100000000u};
    uint64_t v;
    while (end_ - p_ >= 8) {
      std::memcpy(&v, p_, 8);   // little-endian: p_[0] is the low byte
      const uint64_t a = v ^ 0x3030303030303030ull;   // a digit byte becomes 0..9
      const uint64_t bad = (a & 0xF0F0F0F0F0F0F0F0ull) | (((a & 0x0F0F0F0F0F0F0F0Full) + 0x0606060606060606ull) & 0x1010101010101010ull);
      if (!bad) {
        m = m * 100000000u + eight_value(v);
        p_ += 8;
        continue;
      }
      const unsigned n = (unsigned)__builtin_ctzll(bad) >> 3;   // digits before the first non-digit
      if (n) {
        m = m * kPow10u[n] + eight_value((v << (64 - 8 * n)) | (0x3030303030303030ull >> (8 * n)));
        p_ += n;
      }
      return;
    }
    while (digit(*p_)) { m = m * 10u + (uint64_t)(*p_ - '0'); ++p_; }
  }
  // up to eight digits at q into m (m * 10^n + their value); returns n (8: all eight were digits).
  // The caller guarantees 8 readable bytes at q.
  static unsigned run8(const char* q, uint64_t& m) {
    static const uint64_t kPow10u[9] = {1u, 10u, 100u, 1000u, 10000u, 100000u, 1000000u, 10000000u, 100000000u};
    uint64_t v;
    std::memcpy(&v, q, 8);
    const uint64_t a = v ^ 0x3030303030303030ull;
    const uint64_t bad = (a & 0xF0F0F0F0F0F0F0F0ull) | (((a & 0x0F0F0F0F0F0F0F0Full) + 0x0606060606060606ull) & 0x1010101010101010ull);
    const unsigned n = bad ? (unsigned)__builtin_ctzll(bad) >> 3 : 8u;
    if (n == 8u) m = m * 100000000u + eight_value(v);
    else if (n) m = m * kPow10u[n] + eight_value((v << (64 - 8 * n)) | (0x3030303030303030ull >> (8 * n)));
    return n;
  }
  // number() for the common token, word-wide: [-]digits[.digits], at most 15 digits, no exponent,
  // with 40 bytes readable at p_; false (p_ unchanged) for anything else, which number() reads
  bool number_swar(double& out) {
    if (end_ - p_ < 40) return false;
    const char* q = p_;
    const bool neg = *q == '-';
    q += neg;
    uint64_t m = 0;
    unsigned ni = run8(q, m);
    if (ni == 8u) { const unsigned x = run8(q + 8, m); if (x == 8u) return false; ni += x; }
    if (!ni) return false;
    q += ni;
    unsigned fr = 0;
    if (*q == '.') {
      ++q;
      fr = run8(q, m);
      if (fr == 8u) { const unsigned x = run8(q + 8, m); if (x == 8u) return false; fr += x; }
      if (!fr) return false;
      q += fr;
    }
    if (ni + fr > 15u || *q == 'e' || *q == 'E') return false;
    static const double kPow10s[16] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15};
    const double v = fr ? (double)m / kPow10s[fr] : (double)m;
    out = neg ? -v : v;
    p_ = q;
    return true;
  }
  double number() {
    // the common token first — [-]digits[.digits], at most 15 digits, no exponent: one pass, one
    // exact operation (Clinger); anything else (including every malformed token) is re-read by
    // the general path below from the same start, so errors and values are the general path's
    {
      const char* q = p_;
      const bool neg = *q == '-';
      q += neg;
      const char* d0 = q;
      uint64_t m = 0;
      while (digit(*q)) { m = m * 10u + (uint64_t)(*q - '0'); ++q; }
      int nd = (int)(q - d0), fr = 0;
      if (nd && *q == '.') {
        const char* f0 = ++q;
        while (digit(*q)) { m = m * 10u + (uint64_t)(*q - '0'); ++q; }
        fr = (int)(q - f0);
        nd = fr ? nd + fr : 99;
      }
      if (nd && nd <= 15 && *q != 'e' && *q != 'E') {
        static const double kPow10s[16] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15};
        p_ = q;
        const double v = fr ? (double)m / kPow10s[fr] : (double)m;
        return neg ? -v : v;
      }
    }
    const char* st = p_;
    const bool neg = *p_ == '-';
    p_ += neg;
    if (!digit(*p_)) fail("bad number");
    const char* d0 = p_;
    uint64_t m = 0;
    digits(m);
    size_t ndig = (size_t)(p_ - d0);
    int exp10 = 0;
    if (*p_ == '.') {
      ++p_;
      const char* f0 = p_;
      digits(m);
      ndig += (size_t)(p_ - f0);
      exp10 = -(int)std::min<size_t>((size_t)(p_ - f0), 100000);
    }
    if (*p_ == 'e' || *p_ == 'E') {
      ++p_;
      bool eneg = false;
      if (*p_ == '+' || *p_ == '-') { eneg = *p_ == '-'; ++p_; }
      if (!digit(*p_)) fail("bad exponent");
      int ev = 0;
      while (digit(*p_)) { if (ev < 100000) ev = ev * 10 + (*p_ - '0'); ++p_; }
      exp10 += eneg ? -ev : ev;
    }
    bool exact = ndig <= 19;   // m holds every digit (< 10^19 < 2^64)
    if (!exact) {              // leading zeros do not count
      size_t lead = 0;
      for (const char* q = d0; q < p_ && (*q == '0' || *q == '.'); ++q) lead += *q == '0';
      exact = ndig - lead <= 19;
    }
    if (exact) {
      if (m == 0) return neg ? -0.0 : 0.0;
      // Clinger: an exact integer (< 2^53) times / divided by an exact power of ten rounds once
      static const double kPow10[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                                        1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
      if (m < (1ull << 53) && exp10 >= -22 && exp10 <= 22) {
        const double v = exp10 < 0 ? (double)m / kPow10[-exp10] : (double)m * kPow10[exp10];
        return neg ? -v : v;
      }
      // 16-19 digits (Python's repr of a float32 widened to double has 17): one x87 operation on
      // exact operands (m < 2^64 and 10^k, k <= 27, fit the 64-bit significand) is within half
      // an extended ulp of the true value, so rounding it to double is correct unless it lies
      // within one extended ulp of a double halfway point; those go to strtod
      static const long double kPow10L[28] = {
          1e0L, 1e1L, 1e2L, 1e3L, 1e4L, 1e5L, 1e6L, 1e7L, 1e8L, 1e9L, 1e10L, 1e11L, 1e12L, 1e13L,
          1e14L, 1e15L, 1e16L, 1e17L, 1e18L, 1e19L, 1e20L, 1e21L, 1e22L, 1e23L, 1e24L, 1e25L, 1e26L, 1e27L};
      // x87 80-bit extended only (64-bit significand in the low 8 bytes); IEEE quad long double
      // (aarch64, ppc64le) lays its significand out differently and takes strtod
      if (kX87LongDouble && exp10 >= -27 && exp10 <= 27) {
        const long double q = exp10 < 0 ? (long double)m / kPow10L[-exp10] : (long double)m * kPow10L[exp10];
        uint64_t sig;
        std::memcpy(&sig, &q, 8);   // x87 extended: the 64-bit significand is the low 8 bytes
        const uint32_t low = (uint32_t)sig & 0x7ffu;
        if (low < 0x3ffu || low > 0x401u) {
          const double v = (double)q;
          return neg ? -v : v;
        }
      }
    }
    char buf[128];
    const size_t n = (size_t)(p_ - st);
    if (n < sizeof buf) {
      std::memcpy(buf, st, n);
      buf[n] = 0;
      return std::strtod(buf, nullptr);
    }
    return std::strtod(std::string(st, p_).c_str(), nullptr);
  }

  // ---- generic value skipper (validates, stores nothing)
  void skip(int depth) {
    if (depth > 64) fail("nesting too deep");
    ws();
    switch (*p_) {
      case '{': {
        ++p_; ws();
        if (*p_ == '}') { ++p_; return; }
        std::string tmp;
        for (;;) {
          ws();
          if (*p_ != '"') fail("expected key");
          const char *b, *e;
          string(&b, &e, tmp);
          ws();
          if (*p_ != ':') fail("expected ':'");
          ++p_;
          skip(depth + 1);
          ws();
          if (*p_ == ',') { ++p_; continue; }
          if (*p_ == '}') { ++p_; return; }
          fail("expected ',' or '}'");
        }
      }
      case '[': {
        ++p_; ws();
        if (*p_ == ']') { ++p_; return; }
        for (;;) {
          skip(depth + 1);
          ws();
          if (*p_ == ',') { ++p_; continue; }
          if (*p_ == ']') { ++p_; return; }
          fail("expected ',' or ']'");
        }
      }
      case '"': { std::string tmp; const char *b, *e; string(&b, &e, tmp); return; }
      case 't': if (!std::strncmp(p_, "true", 4)) { p_ += 4; return; } fail("bad literal");
      case 'f': if (!std::strncmp(p_, "false", 5)) { p_ += 5; return; } fail("bad literal");
      case 'n': if (!std::strncmp(p_, "null", 4)) { p_ += 4; return; } fail("bad literal");
      default: (void)number(); return;
    }
  }

  // value kinds the semantic checks distinguish
  enum Kind { kNull, kNum, kOther };
  // parse a scalar-or-anything value: numbers are converted, anything else skipped
  Kind scalar(int depth, double& num) {
    ws();
    const char c = *p_;
    if (c == '-' || (c >= '0' && c <= '9')) { num = number(); return kNum; }
    if (c == 'n' && !std::strncmp(p_, "null", 4)) { p_ += 4; return kNull; }
    skip(depth);
    return kOther;
  }

  static bool key_is(const char* b, const char* e, const char* k) {
    const size_t n = std::strlen(k);
    return (size_t)(e - b) == n && std::memcmp(b, k, n) == 0;
  }

  void parse_document(PointSink& sink) {
    ws();
    if (*p_ != '{') {
      skip(0);
      ws();
      if (*p_) fail("trailing characters");
      return;
    }
    top_object_ = true;
    ++p_; ws();
    if (*p_ == '}') { ++p_; } else {
      std::string tmp;
      for (;;) {
        ws();
        if (*p_ != '"') fail("expected key");
        const char *b, *e;
        string(&b, &e, tmp);
        ws();
        if (*p_ != ':') fail("expected ':'");
        ++p_;
        if (key_is(b, e, "trace") && trace_state_ == 0) trace_value(sink);
        else if (key_is(b, e, "match_options") && !opts_seen_) options_value();
        else skip(1);
        ws();
        if (*p_ == ',') { ++p_; continue; }
        if (*p_ == '}') { ++p_; break; }
        fail("expected ',' or '}'");
      }
    }
    ws();
    if (*p_) fail("trailing characters");
  }

  void options_value() {
    opts_seen_ = true;
    ws();
    if (*p_ != '{') { skip(1); return; }   // not an object: no options apply (DOM: apply_options returns)
    ++p_; ws();
    if (*p_ == '}') { ++p_; return; }
    std::string tmp;
    for (;;) {
      ws();
      if (*p_ != '"') fail("expected key");
      const char *b, *e;
      string(&b, &e, tmp);
      ws();
      if (*p_ != ':') fail("expected ':'");
      ++p_;
      int k = -1;
      for (int q = 0; q < kNumOpt; ++q)
        if (key_is(b, e, kOptNames[q])) { k = q; break; }
      if (k >= 0 && !opt_seen_[k]) {
        opt_seen_[k] = true;
        double v = 0.0;
        const Kind kd = scalar(2, v);
        opt_state_[k] = kd == kNum ? 1 : (kd == kNull ? 0 : 2);
        opt_val_[k] = v;
      } else if (key_is(b, e, "mode") && !mode_seen_) {
        mode_seen_ = true;
        ws();
        if (*p_ == '"') {
          std::string mt;
          const char *mb, *me;
          string(&mb, &me, mt);
          const int m = mode_index(mb, (size_t)(me - mb));
          if (m < 0) mode_err_ = "unsupported mode: " + std::string(mb, me);
          else mode_ = m;
        } else {
          skip(2);   // a non-string mode is ignored (DOM: mode stays auto)
        }
      } else {
        skip(2);
      }
      ws();
      if (*p_ == ',') { ++p_; continue; }
      if (*p_ == '}') { ++p_; return; }
      fail("expected ',' or '}'");
    }
  }

  void trace_value(PointSink& sink) {
    ws();
    if (*p_ != '[') { trace_state_ = 2; skip(1); return; }
    trace_state_ = 1;
    if (defer_) {
      // a compact trace starts with its first point and has no ']' before its end, so the first
      // ']' closes it; whether the bytes between are compact points is the device parser's check
      const char* b = p_ + 1;
      const char* close = *b == '{' ? static_cast<const char*>(std::memchr(b, ']', (size_t)(end_ - b))) : nullptr;
      if (close) {
        defer_->b = b;
        defer_->e = close;
        defer_->n_open = (uint32_t)std::count(b, close, '{');
        defer_->on = true;
        p_ = close + 1;
        return;
      }
    }
    ++p_; ws();
    if (*p_ == ']') { ++p_; return; }
    std::string tmp;
    for (;;) {
      ws();
      if (*p_ == '{') {
        if (!point_compact(sink)) point(sink, tmp);
      } else {
        skip(2);
        if (point_err_.empty()) point_err_ = "each trace point needs numeric lat and lon";
      }
      ws();
      if (*p_ == ',') { ++p_; continue; }
      if (*p_ == ']') { ++p_; return; }
      fail("expected ',' or ']'");
    }
  }

  // The point layout json.dumps(separators=(',', ':')) writes, in any key order: exactly the
  // keys lat, lon, time, accuracy, once each, unescaped, with number values and no whitespace.
  // Anything else (another key, a repeat, a non-number, whitespace, an earlier failed point)
  // rewinds to the '{' and takes the generic point() below, so the result, the validation and
  // the error offsets are the generic path's: a number that fails here fails there at the same
  // offset, since both reach it through the same bytes.
  bool point_compact(PointSink& sink) {
    if (!point_err_.empty()) return false;
    const char* st = p_;
    double v[4];
    unsigned seen = 0;
    ++p_;
    auto lit = [&](const char* s, size_t n) {   // the text at p_ starts with s[0, n) (never reads past the NUL)
      if ((size_t)(end_ - p_) < n || std::memcmp(p_, s, n) != 0) return false;
      p_ += n;
      return true;
    };
    // the four keys as little-endian words ("lat": and "lon": 6 bytes, "time": 7, "accuracy": 11)
    constexpr uint64_t kLat = 0x3a2274616c22ull, kLon = 0x3a226e6f6c22ull, kTime = 0x3a22656d697422ull;
    constexpr uint64_t kAcc0 = 0x6361727563636122ull, kAcc1 = 0x3a2279ull;
    for (;;) {
      int k;
      if (end_ - p_ >= 16) {   // one word compare per key
        uint64_t w;
        uint32_t w2;
        std::memcpy(&w, p_, 8);
        std::memcpy(&w2, p_ + 8, 4);
        const uint64_t w6 = w & 0xffffffffffffull, w7 = w & 0xffffffffffffffull;
        if (w6 == kLat) { k = 0; p_ += 6; }
        else if (w6 == kLon) { k = 1; p_ += 6; }
        else if (w7 == kTime) { k = 2; p_ += 7; }
        else if (w == kAcc0 && (w2 & 0xffffffu) == kAcc1) { k = 3; p_ += 11; }
        else break;
      } else if (lit("\"lat\":", 6)) k = 0;
      else if (lit("\"lon\":", 6)) k = 1;
      else if (lit("\"time\":", 7)) k = 2;
      else if (lit("\"accuracy\":", 11)) k = 3;
      else break;
      if (seen & (1u << k) || !(*p_ == '-' || digit(*p_))) break;
      seen |= 1u << k;
      if (!number_swar(v[k])) v[k] = number();
      if (*p_ == ',') { ++p_; continue; }
      if (*p_ == '}' && seen == 15u) {
        ++p_;
        if (!(v[0] >= -90.0 && v[0] <= 90.0 && v[1] >= -180.0 && v[1] <= 180.0)) {
          point_err_ = "trace point out of range";
          return true;
        }
        sink.lat.push_back((float)v[0]);
        sink.lon.push_back((float)v[1]);
        sink.time.push_back(v[2]);
        sink.acc.push_back((float)v[3]);
        return true;
      }
      break;
    }
    p_ = st;
    return false;
  }

  void point(PointSink& sink, std::string& tmp) {
    ++p_; ws();
    // first occurrence of each key (DOM get): 0 absent, 1 number, 2 other / null
    int st_lat = 0, st_lon = 0, st_t = 0, st_a = 0;
    double lat = 0, lon = 0, tm = -1.0, ac = -1.0;
    if (*p_ == '}') { ++p_; } else {
      for (;;) {
        ws();
        if (*p_ != '"') fail("expected key");
        const char *b, *e;
        string(&b, &e, tmp);
        ws();
        if (*p_ != ':') fail("expected ':'");
        ++p_;
        int* st = nullptr;
        double* dst = nullptr;
        const size_t n = (size_t)(e - b);
        if (n == 3 && b[0] == 'l' && b[1] == 'a' && b[2] == 't') { st = &st_lat; dst = &lat; }
        else if (n == 3 && b[0] == 'l' && b[1] == 'o' && b[2] == 'n') { st = &st_lon; dst = &lon; }
        else if (n == 4 && std::memcmp(b, "time", 4) == 0) { st = &st_t; dst = &tm; }
        else if (n == 8 && std::memcmp(b, "accuracy", 8) == 0) { st = &st_a; dst = &ac; }
        if (st && *st == 0) {
          double v = 0.0;
          const Kind kd = scalar(3, v);
          *st = kd == kNum ? 1 : 2;
          if (kd == kNum) *dst = v;
        } else {
          skip(3);
        }
        ws();
        if (*p_ == ',') { ++p_; continue; }
        if (*p_ == '}') { ++p_; break; }
        fail("expected ',' or '}'");
      }
    }
    if (!point_err_.empty()) return;   // an earlier point failed: the request fails with its error
    if (st_lat != 1 || st_lon != 1) { point_err_ = "each trace point needs numeric lat and lon"; return; }
    if (!(lat >= -90.0 && lat <= 90.0 && lon >= -180.0 && lon <= 180.0)) { point_err_ = "trace point out of range"; return; }
    sink.lat.push_back((float)lat);   // Valhalla PointLL is float
    sink.lon.push_back((float)lon);
    sink.time.push_back(st_t == 1 ? tm : -1.0);
    sink.acc.push_back(st_a == 1 ? (float)ac : -1.0f);
  }
};

// Parse one Match request (NUL-terminated), appending its points to `sink`.  Returns the
// trace's options (its mode's defaults with the request's match_options applied).  Throws with
// the DOM reader's messages; on error nothing is appended.
inline MatchOptions parse_request(const char* text, const MatchOptions mode_defaults[5], PointSink& sink) {
  Reader r(text, std::strlen(text), mode_defaults);
  return r.request(sink);
}
// Parse one request leaving its trace array to the device parser where it may be compact
// (span.on); throws on anything the structure alone fails (the caller then parses the request
// with parse_request, which reports the generic reader's error).
inline MatchOptions parse_request_deferred(const char* text, size_t len, const MatchOptions mode_defaults[5],
                                           PointSink& sink, TraceSpan& span) {
  span = TraceSpan();
  Reader r(text, len, mode_defaults, &span);
  return r.request(sink);
}
// the same, with the text's length known (len = strlen(text): the NUL at text[len] ends it)
inline MatchOptions parse_request(const char* text, size_t len, const MatchOptions mode_defaults[5], PointSink& sink) {
  Reader r(text, len, mode_defaults);
  return r.request(sink);
}

// ---- reply formatting ----
inline void put_u64(std::string& o, uint64_t x) {
  char b[24];
  const auto r = std::to_chars(b, b + sizeof b, x);
  o.append(b, r.ptr);
}
inline void put_i64(std::string& o, int64_t x) {
  char b[24];
  const auto r = std::to_chars(b, b + sizeof b, x);
  o.append(b, r.ptr);
}
inline void put_num(std::string& o, double x) {
  if (x == -1.0) { o += "-1"; return; }
  char b[40];
  const auto r = std::to_chars(b, b + sizeof b, x);   // shortest digits that round-trip
  o.append(b, r.ptr);
}

// {"segments":[...]} of one trace: the schema of README.md:288-301 (segment_id omitted without
// an OSMLR id; -1 for a time / length that is not known)
inline void format_segments(const SegmentRec* s, uint32_t n, std::string& o) {
  o.clear();
  o.reserve(16 + (size_t)n * 200);
  o += "{\"segments\":[";
  for (uint32_t k = 0; k < n; ++k) {
    const SegmentRec& r = s[k];
    if (k) o += ',';
    o += '{';
    if (r.flags & 2u) { o += "\"segment_id\":"; put_u64(o, r.segment_id); o += ','; }
    o += "\"way_ids\":[";
    put_u64(o, r.way_first);
    if (r.way_last != r.way_first) { o += ','; put_u64(o, r.way_last); }
    o += "],\"start_time\":"; put_num(o, r.start_time);
    o += ",\"end_time\":"; put_num(o, r.end_time);
    o += ",\"queue_length\":"; put_i64(o, r.queue_length);
    o += ",\"length\":"; put_i64(o, r.length);
    o += ",\"internal\":"; o += (r.flags & 1u) ? "true" : "false";
    o += ",\"begin_shape_index\":"; put_u64(o, r.begin_shape_index);
    o += ",\"end_shape_index\":"; put_u64(o, r.end_shape_index);
    o += '}';
  }
  o += "]}";
}

}  // namespace tj
}  // namespace rm
