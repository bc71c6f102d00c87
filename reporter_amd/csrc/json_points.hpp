// json_points.hpp — the compact trace layout read by the device JSON parser (engine.hip
// k_parse_json), as host/device functions so the host test (tests/cpp/trace_json_test.cpp) runs
// the same rules against the generic reader.
//
// A compact trace array holds points in point_compact's layout (trace_json.hpp): '{', the keys
// "lat", "lon", "time", "accuracy" once each in any order, each followed by ':' and a number of at
// most 15 significant digits ([-]digits[.digits], no exponent), ',' between members, '}'; points
// are separated by single commas; no whitespace.  Such a number converts exactly as the host
// reader's Clinger path does: the digits as an exact integer m < 10^15, one IEEE division by
// 10^fraction digits.  Anything else is "not compact": the host reader parses that request.
#pragma once
#include <cstdint>

#include "rm_common.hpp"

namespace rm {
namespace jp {

RM_HD bool digit(uint8_t c) { return (uint32_t)(c - '0') < 10u; }

RM_HD double pow10_exact(uint32_t k) {   // 10^k, k <= 15 (exact doubles)
  double p = 1.0;
  for (uint32_t i = 0; i < k; ++i) p *= 10.0;
  return p;
}

// the number at s[q..e) (q on '-' or a digit); q moves past it
RM_HD bool number(const uint8_t* s, uint64_t& q, uint64_t e, double& out) {
  uint64_t i = q;
  const bool neg = i < e && s[i] == '-';
  i += neg;
  uint64_t m = 0;
  uint32_t ni = 0, fr = 0;
  while (i < e && digit(s[i])) {
    if (ni >= 15u) return false;
    m = m * 10u + (uint64_t)(s[i] - '0');
    ++i;
    ++ni;
  }
  if (!ni) return false;
  if (i < e && s[i] == '.') {
    ++i;
    while (i < e && digit(s[i])) {
      if (ni + fr >= 15u) return false;
      m = m * 10u + (uint64_t)(s[i] - '0');
      ++i;
      ++fr;
    }
    if (!fr) return false;
  }
  if (i < e && (s[i] == 'e' || s[i] == 'E')) return false;
  const double v = fr ? (double)m / pow10_exact(fr) : (double)m;
  out = neg ? -v : v;
  q = i;
  return true;
}

// the key at s[i..e): 0 lat, 1 lon, 2 time, 3 accuracy (n: its bytes with the quotes and ':'),
// -1 for anything else.  Immediate compares: a key string in memory would cost the device a
// dependent load per byte.
RM_HD int key(const uint8_t* s, uint64_t i, uint64_t e, uint32_t& n) {
  if (e - i < 6 || s[i] != '"') return -1;
  const uint8_t c1 = s[i + 1];
  if (c1 == 'l') {
    const uint8_t c2 = s[i + 2], c3 = s[i + 3];
    if (s[i + 4] != '"' || s[i + 5] != ':') return -1;
    n = 6;
    if (c2 == 'a' && c3 == 't') return 0;
    if (c2 == 'o' && c3 == 'n') return 1;
    return -1;
  }
  if (c1 == 't') {
    if (e - i < 7 || s[i + 2] != 'i' || s[i + 3] != 'm' || s[i + 4] != 'e' || s[i + 5] != '"' || s[i + 6] != ':') return -1;
    n = 7;
    return 2;
  }
  if (c1 == 'a') {
    if (e - i < 11 || s[i + 2] != 'c' || s[i + 3] != 'c' || s[i + 4] != 'u' || s[i + 5] != 'r' || s[i + 6] != 'a' ||
        s[i + 7] != 'c' || s[i + 8] != 'y' || s[i + 9] != '"' || s[i + 10] != ':')
      return -1;
    n = 11;
    return 3;
  }
  return -1;
}

// the compact point whose '{' is at s[q]; q moves past its '}'.  v: lat, lon, time, accuracy
RM_HD bool point(const uint8_t* s, uint64_t& q, uint64_t e, double& la, double& lo, double& tm, double& ac) {
  uint64_t i = q + 1;
  uint32_t seen = 0;
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
  for (int m = 0; m < 4; ++m) {   // four members, then '}'
    uint32_t n = 0;
    const int k = key(s, i, e, n);
    if (k < 0 || (seen & (1u << k))) return false;
    seen |= 1u << k;
    i += n;
    double x = 0.0;
    if (i >= e || !(s[i] == '-' || digit(s[i])) || !number(s, i, e, x)) return false;
    v0 = k == 0 ? x : v0;
    v1 = k == 1 ? x : v1;
    v2 = k == 2 ? x : v2;
    v3 = k == 3 ? x : v3;
    if (i >= e) return false;
    const uint8_t c = s[i++];
    if (m < 3 ? c != ',' : c != '}') return false;
  }
  q = i;
  la = v0; lo = v1; tm = v2; ac = v3;
  return true;
}

// what follows a point that ended at q: ",{" (the next point) or the end of the span
RM_HD bool point_follows(const uint8_t* s, uint64_t q, uint64_t e) {
  return q == e || (s[q] == ',' && q + 1 < e && s[q + 1] == '{');
}

// lat / lon within range (the host reader's "trace point out of range" otherwise)
RM_HD bool in_range(double la, double lo) { return la >= -90.0 && la <= 90.0 && lo >= -180.0 && lo <= 180.0; }

}  // namespace jp
}  // namespace rm
