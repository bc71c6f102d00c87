// host_pool.hpp — persistent host worker threads for the boundary's parse / stage / format work.
//
// The /report boundary splits a batch's JSON parsing, staging and reply formatting over up to 16
// host threads.  Spawning them per batch cost ~0.5 ms a call, and the request coalescer runs
// hundreds of batches a second, so the workers live for the process.  One job runs at a time
// (callers queue on a mutex); a job is fn(t) for t in [0, nt), t = 0 on the calling thread.
#pragma once
#include <algorithm>
#include <condition_variable>
#include <cstddef>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace rm {

class HostPool {
 public:
  // min(16, hardware threads), or RM_HOST_THREADS (1..256) for a host with more cores to give
  static HostPool& get() {
    static HostPool pool(default_size());
    return pool;
  }
  static unsigned default_size() {
    if (const char* e = std::getenv("RM_HOST_THREADS")) {
      const long v = std::strtol(e, nullptr, 10);
      if (v >= 1 && v <= 256) return (unsigned)v;
    }
    return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  }
  size_t size() const { return workers_.size() + 1; }

  // fn(t) for t in [0, nt) (nt <= size()); rethrows the lowest t's exception
  void run(size_t nt, const std::function<void(size_t)>& fn) {
    nt = std::min(nt, size());
    if (nt <= 1) { fn(0); return; }
    std::lock_guard<std::mutex> job(job_mu_);
    std::vector<std::exception_ptr> err(nt);
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      err_ = &err;
      nt_ = nt;
      next_ = 1;
      pending_ = nt - 1;
      ++gen_;
    }
    cv_.notify_all();
    try { fn(0); } catch (...) { err[0] = std::current_exception(); }
    {
      std::unique_lock<std::mutex> lk(mu_);
      done_cv_.wait(lk, [&] { return pending_ == 0; });
      fn_ = nullptr;
    }
    for (auto& e : err)
      if (e) std::rethrow_exception(e);
  }

  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  explicit HostPool(unsigned n) {
    for (unsigned i = 1; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      size_t t;
      const std::function<void(size_t)>* fn;
      std::vector<std::exception_ptr>* err;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || (gen_ != seen && next_ < nt_); });
        if (stop_) return;
        t = next_++;
        if (next_ >= nt_) seen = gen_;
        fn = fn_;
        err = err_;
      }
      try { (*fn)(t); } catch (...) { (*err)[t] = std::current_exception(); }
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--pending_ == 0) done_cv_.notify_all();
      }
    }
  }

  std::vector<std::thread> workers_;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)>* fn_ = nullptr;
  std::vector<std::exception_ptr>* err_ = nullptr;
  size_t nt_ = 0, next_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace rm
