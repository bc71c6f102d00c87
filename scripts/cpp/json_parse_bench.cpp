// Single-thread timing of the /report request parser (trace_json.hpp) on bench.py-style requests
// (request_jsons: %.6f lat/lon, integer time, %g accuracy; 600 points per request).  Diagnostic.
//   g++ -O3 -march=native -std=c++17 scripts/cpp/json_parse_bench.cpp -o /tmp/jpb && /tmp/jpb [requests]
#include <chrono>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

#include "../../reporter_amd/csrc/trace_json.hpp"

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 1000;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  std::vector<std::string> reqs;
  size_t bytes = 0, pts = 0;
  char buf[160];
  for (int k = 0; k < n; ++k) {
    std::string s = "{\"uuid\":\"" + std::to_string(k) + "\",\"trace\":[";
    double lat = 47.0 + u(rng) * 0.2, lon = 8.0 + u(rng) * 0.2;
    for (int i = 0; i < 600; ++i) {
      lat += (u(rng) - 0.5) * 1e-4; lon += (u(rng) - 0.5) * 1e-4;
      std::snprintf(buf, sizeof buf, "%s{\"lat\":%.6f,\"lon\":%.6f,\"time\":%d,\"accuracy\":%g}", i ? "," : "",
                    (double)(float)lat, (double)(float)lon, 1500000000 + i, 5.0);
      s += buf;
    }
    s += "],\"match_options\":{\"mode\":\"auto\",\"report_levels\":[0,1],\"transition_levels\":[0,1]}}";
    bytes += s.size();
    pts += 600;
    reqs.push_back(std::move(s));
  }
  rm::MatchOptions defs[5];
  for (int m = 0; m < 5; ++m) { defs[m] = rm::default_options(); defs[m].mode = m; }
  rm::tj::PointSink sk;
  double best = 1e30, chk = 0;
  for (int rep = 0; rep < 7; ++rep) {
    sk.clear();
    sk.lon.reserve(pts); sk.lat.reserve(pts); sk.acc.reserve(pts); sk.time.reserve(pts);
    const auto t0 = std::chrono::steady_clock::now();
    for (const auto& r : reqs) rm::tj::parse_request(r.c_str(), r.size(), defs, sk);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    best = std::min(best, s);
    chk = 0;
    for (size_t i = 0; i < sk.size(); ++i) chk += sk.lat[i] + sk.lon[i] * 3 + sk.time[i] * 1e-9 + sk.acc[i];
  }
  std::printf("%zu points, %.1f MB: %.2f ms, %.1f ns/point, %.2f GB/s (checksum %.6f)\n", pts, bytes / 1e6, best * 1e3,
              best * 1e9 / pts, bytes / best / 1e9, chk);
}
