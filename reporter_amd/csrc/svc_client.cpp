// svc_client.cpp — a multi-threaded /report client of the C-ABI with no interpreter in the way
// (VERDICT r03 item 4): N threads, one rm_matcher each (the reference service's threading,
// py/reporter_service.py:28-64), each calling rm_match on the next request of a shared list, as
// the service's worker threads call SegmentMatcher.Match (:240) for concurrent HTTP requests.
// The library coalesces the concurrent calls into GPU batches.  What this measures is the
// library's own ceiling for the service: requests/s and points/s with N requests in flight,
// latency percentiles, and the coalescer's batch statistics.  bench.py runs it; it does not
// format HTTP or JSON beyond what Match itself does.
//
//   rm_svc_client <config.json> <requests.txt> <clients> <requests> [warmup]
//   requests.txt: one /report request JSON per line; the number of points of a request is the
//   number of "lat" keys on its line.  Prints one JSON object.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include <sys/resource.h>

#include "../../include/reporter_match.h"

namespace {

size_t count_points(const std::string& s) {
  size_t n = 0;
  for (size_t at = s.find("\"lat\""); at != std::string::npos; at = s.find("\"lat\"", at + 5)) ++n;
  return n;
}

// the process's CPU seconds (user + system) and the cgroup's CPU throttling counters (cgroup v2
// cpu.stat; zeros when absent): a service stalled by a CPU quota shows up in throttled_us
double cpu_seconds() {
  rusage u{};
  getrusage(RUSAGE_SELF, &u);
  return (double)u.ru_utime.tv_sec + u.ru_utime.tv_usec * 1e-6 + (double)u.ru_stime.tv_sec + u.ru_stime.tv_usec * 1e-6;
}
void cgroup_throttle(unsigned long long* periods, unsigned long long* usec) {
  *periods = 0; *usec = 0;
  std::ifstream f("/sys/fs/cgroup/cpu.stat");
  std::string k;
  unsigned long long v;
  while (f >> k >> v) {
    if (k == "nr_throttled") *periods = v;
    else if (k == "throttled_usec") *usec = v;
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s <config.json> <requests.txt> <clients> <requests> [warmup]\n", argv[0]);
    return 2;
  }
  const char* conf = argv[1];
  const int clients = std::max(1, std::atoi(argv[3]));
  const size_t total = (size_t)std::max(1L, std::atol(argv[4]));
  const size_t warmup = argc > 5 ? (size_t)std::atol(argv[5]) : 0;
  std::vector<std::string> reqs;
  std::vector<size_t> pts;
  {
    std::ifstream f(argv[2]);
    std::string line;
    while (std::getline(f, line))
      if (!line.empty()) {
        pts.push_back(count_points(line));
        reqs.push_back(std::move(line));
      }
  }
  if (reqs.empty()) {
    std::fprintf(stderr, "no requests in %s\n", argv[2]);
    return 2;
  }
  char err[1024] = {0};
  if (rm_configure(conf, err, sizeof err) != 0) {
    std::fprintf(stderr, "rm_configure: %s\n", err);
    return 1;
  }
  // one pass of `n` requests over `clients` threads; per-request latency in microseconds
  std::atomic<long> client_us{0};   // CPU time of the client threads themselves (parse, wait, reply)
  auto run = [&](size_t n, std::vector<double>* lat, size_t* npts, size_t* nerr) {
    std::atomic<size_t> next{0}, points{0}, errors{0};
    std::vector<std::vector<double>> lats(clients);
    std::vector<std::thread> th;
    for (int c = 0; c < clients; ++c)
      th.emplace_back([&, c] {
        rm_matcher* m = rm_matcher_create();
        if (!m) { errors += n; return; }
        for (size_t q = next++; q < n; q = next++) {
          const size_t i = q % reqs.size();
          char* out = nullptr;
          const auto t0 = std::chrono::steady_clock::now();
          const int rc = rm_match(m, reqs[i].c_str(), &out);
          const auto t1 = std::chrono::steady_clock::now();
          if (rc == 0) {
            points += pts[i];
            rm_free(out);
          } else {
            ++errors;
          }
          lats[c].push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        rm_matcher_destroy(m);
        rusage u{};
        getrusage(RUSAGE_THREAD, &u);
        client_us += u.ru_utime.tv_sec * 1000000L + u.ru_utime.tv_usec + u.ru_stime.tv_sec * 1000000L + u.ru_stime.tv_usec;
      });
    for (auto& t : th) t.join();
    if (lat) for (auto& v : lats) lat->insert(lat->end(), v.begin(), v.end());
    if (npts) *npts = points;
    if (nerr) *nerr = errors;
  };
  if (warmup) run(warmup, nullptr, nullptr, nullptr);
  uint64_t s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  double m0[4] = {0, 0, 0, 0}, m1[4] = {0, 0, 0, 0};
  rm_coalesce_stats(s0);
  rm_coalesce_timing(m0);
  std::vector<double> lat;
  size_t npts = 0, nerr = 0;
  unsigned long long thr0 = 0, thu0 = 0, thr1 = 0, thu1 = 0;
  cgroup_throttle(&thr0, &thu0);
  const double cpu0 = cpu_seconds();
  client_us = 0;
  rusage r0{};
  getrusage(RUSAGE_SELF, &r0);
  const auto t0 = std::chrono::steady_clock::now();
  run(total, &lat, &npts, &nerr);
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const double cpu1 = cpu_seconds();
  rusage r1{};
  getrusage(RUSAGE_SELF, &r1);
  cgroup_throttle(&thr1, &thu1);
  rm_coalesce_stats(s1);
  rm_coalesce_timing(m1);
  std::sort(lat.begin(), lat.end());
  auto pct = [&](double q) { return lat.empty() ? 0.0 : lat[std::min(lat.size() - 1, (size_t)(q * lat.size()))] / 1e3; };
  const double batches = (double)(s1[0] - s0[0]);
  std::printf("{\"clients\": %d, \"requests\": %zu, \"errors\": %zu, \"seconds\": %.6f, \"requests_per_s\": %.1f, "
              "\"points_per_s\": %.1f, \"points_per_request\": %.1f, \"latency_ms\": {\"p50\": %.3f, \"p90\": %.3f, "
              "\"p99\": %.3f, \"max\": %.3f}, \"batches\": %.0f, \"requests_per_batch\": %.2f, "
              "\"ms_per_batch\": %.4f, \"largest_batch\": %llu, \"dispatcher_ms_per_batch\": {\"staging\": %.4f, "
              "\"engine\": %.4f, \"download\": %.4f, \"format\": %.4f}, \"cpu_seconds\": %.3f, \"client_cpu_seconds\": %.3f, "
              "\"context_switches\": {\"voluntary\": %ld, \"involuntary\": %ld}, \"cgroup_throttled_periods\": %llu, \"cgroup_throttled_ms\": %.1f}\n",
              clients, total, nerr, sec, (double)total / sec, (double)npts / sec, (double)npts / (double)total,
              pct(0.5), pct(0.9), pct(0.99), lat.empty() ? 0.0 : lat.back() / 1e3, batches,
              batches > 0 ? (double)(s1[1] - s0[1]) / batches : 0.0, batches > 0 ? sec * 1e3 / batches : 0.0,
              (unsigned long long)s1[2], batches > 0 ? (m1[0] - m0[0]) / batches : 0.0,
              batches > 0 ? (m1[1] - m0[1]) / batches : 0.0, batches > 0 ? (m1[2] - m0[2]) / batches : 0.0,
              batches > 0 ? (m1[3] - m0[3]) / batches : 0.0, cpu1 - cpu0, client_us.load() * 1e-6,
              r1.ru_nvcsw - r0.ru_nvcsw, r1.ru_nivcsw - r0.ru_nivcsw, thr1 - thr0, (thu1 - thu0) / 1e3);
  return nerr ? 1 : 0;
}
