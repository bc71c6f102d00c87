// Host test of the coalescer's failure policy (reporter_amd/csrc/serve_policy.hpp) with a fake
// runner: a persistent whole-batch failure is attempted once; a batch too large is retried by
// halves until the parts fit, within the retry budget; per-request outcomes are kept.
#include <cstdio>
#include <string>
#include <vector>

#include "serve_policy.hpp"

struct Req {
  int id;
  std::string out, err;
};

static int g_runs = 0;

#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "FAILED %s at line %d\n", #c, __LINE__);  \
      return 1;                                                      \
    }                                                                \
  } while (0)

template <class Run>
static std::vector<Req> serve(int n, Run run, int& budget) {
  std::vector<Req> reqs(n);
  std::vector<Req*> ptr(n);
  for (int i = 0; i < n; ++i) { reqs[i].id = i; ptr[i] = &reqs[i]; }
  g_runs = 0;
  rm::serve_split(ptr.data(), ptr.size(), run, [](Req* r, const char* m) { r->err = m; }, budget);
  return reqs;
}

int main() {
  // 1. a device error on every run: one run, every request gets the message
  {
    int budget = rm::kServeRetryBudget;
    auto reqs = serve(16384, [](Req* const*, size_t) { ++g_runs; throw std::runtime_error("HIP error: device lost"); }, budget);
    CHECK(g_runs == 1);
    for (auto& r : reqs) CHECK(r.err == "HIP error: device lost" && r.out.empty());
  }
  // 2. batches above 1000 requests are too large: halves until they fit, every request answered
  {
    int budget = rm::kServeRetryBudget;
    auto reqs = serve(4096, [](Req* const* q, size_t n) {
      ++g_runs;
      if (n > 1000) throw rm::BatchTooLarge("batch too large");
      for (size_t i = 0; i < n; ++i) q[i]->out = "ok" + std::to_string(q[i]->id);
    }, budget);
    CHECK(g_runs == 1 + 2 + 4 + 8);   // 4096 -> 2 x 2048 -> 4 x 1024 (all > 1000) -> 8 x 512 fit
    for (auto& r : reqs) CHECK(r.err.empty() && r.out == "ok" + std::to_string(r.id));
  }
  // 3. too large at every size: bounded by the retry budget, then every request gets the error
  {
    int budget = rm::kServeRetryBudget;
    auto reqs = serve(16384, [](Req* const*, size_t) { ++g_runs; throw rm::BatchTooLarge("batch too large"); }, budget);
    CHECK(g_runs <= 1 + rm::kServeRetryBudget);
    CHECK(budget >= 0);
    for (auto& r : reqs) CHECK(r.err == "batch too large");
  }
  // 4. per-request errors set by the runner survive (the engine isolates one trace's failure)
  {
    int budget = rm::kServeRetryBudget;
    auto reqs = serve(96, [](Req* const* q, size_t n) {
      ++g_runs;
      for (size_t i = 0; i < n; ++i) {
        if (q[i]->id == 17) q[i]->err = "candidate roads";
        else q[i]->out = "ok";
      }
    }, budget);
    CHECK(g_runs == 1);
    for (auto& r : reqs) CHECK(r.id == 17 ? (r.err == "candidate roads") : (r.out == "ok" && r.err.empty()));
  }
  // 5. a device error inside a half after a split fails that half only
  {
    int budget = rm::kServeRetryBudget;
    auto reqs = serve(8, [](Req* const* q, size_t n) {
      ++g_runs;
      if (n > 4) throw rm::BatchTooLarge("batch too large");
      if (q[0]->id == 0) throw std::runtime_error("HIP error");
      for (size_t i = 0; i < n; ++i) q[i]->out = "ok";
    }, budget);
    CHECK(g_runs == 3);
    for (auto& r : reqs) CHECK(r.id < 4 ? r.err == "HIP error" : r.out == "ok");
  }
  std::printf("serve policy ok\n");
  return 0;
}
