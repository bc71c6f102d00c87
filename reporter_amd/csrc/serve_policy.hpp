// serve_policy.hpp — how the request coalescer (capi.cpp) answers a batch whose run failed.
//
// The reference answers each /report on its own thread, so a failing Match is one HTTP 500
// (py/reporter_service.py:244-245).  Here concurrent requests share one GPU batch.  Failures
// that belong to one trace are already isolated per trace by the engine (Matcher isolation:
// trace_err).  What can still fail a whole batch falls in two classes:
//   * the batch is too large for the device (index limits, workspace HBM): a smaller batch
//     can succeed, so the requests are retried as two halves, within a bounded number of runs;
//   * anything else (a HIP error, a route-table build that cannot fit, a sticky device fault)
//     is the same for every request in it: each gets the error at once, with no retry, so a
//     persistent fault costs one run instead of 2n - 1.
// Header-only so a host test can drive it with a fake runner (tests/cpp/serve_policy_test.cpp).
#pragma once
#include <cstddef>
#include <stdexcept>

namespace rm {

// A run that failed because of the batch's size (points, transitions or path edges beyond the
// engine's index limits, or a workspace that does not fit in HBM).
struct BatchTooLarge : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Runs kServeRetryBudget more at most after the first, whatever the batch size.
constexpr int kServeRetryBudget = 64;

// Answer requests reqs[0, n): run(reqs, n) fills every request's reply (or its own error) or
// throws; fail(req, message) gives one request an error.  `budget` is the number of further
// runs the whole batch may still take (shared by the halves).
template <class Req, class Run, class Fail>
void serve_split(Req* const* reqs, size_t n, Run&& run, Fail&& fail, int& budget) {
  if (n == 0) return;
  try {
    run(reqs, n);
    return;
  } catch (const BatchTooLarge& e) {
    if (n > 1 && budget >= 2) {
      budget -= 2;
      const size_t h = n / 2;
      serve_split(reqs, h, run, fail, budget);
      serve_split(reqs + h, n - h, run, fail, budget);
      return;
    }
    for (size_t i = 0; i < n; ++i) fail(reqs[i], e.what());
  } catch (const std::exception& e) {
    for (size_t i = 0; i < n; ++i) fail(reqs[i], e.what());
  } catch (...) {
    for (size_t i = 0; i < n; ++i) fail(reqs[i], "unknown error");
  }
}

}  // namespace rm
