// pst_pool.h — one process-wide pool of host worker threads for libpst's host-side work (PDB
// parsing, token-file writes). Threads are created once and reused: on the GPU boxes a thread
// start costs tens of microseconds, so a pool per call (three per parse) cost more than the work
// on a 31-file batch.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace pst {

class HostPool {
 public:
  static HostPool& get() {
    static HostPool p;
    return p;
  }
  // fn(i) for i in order[0..n) handed out dynamically; `threads` workers including the caller.
  // Calls from several host threads at once are serialised.
  void run(int n, int threads, const std::function<void(int)>& fn) {
    threads = std::max(1, std::min(threads, n));
    if (threads <= 1) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    std::lock_guard<std::mutex> call(call_mu_);
    {
      std::unique_lock<std::mutex> lk(mu_);
      while ((int)workers_.size() < threads - 1) {
        const int id = (int)workers_.size();
        workers_.emplace_back([this, id] { loop(id); });
      }
      job_ = &fn;
      n_ = n;
      limit_ = threads - 1;
      next_.store(0);
      pending_ = limit_;
      ++gen_;
    }
    cv_.notify_all();
    for (int i = next_++; i < n; i = next_++) fn(i);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* job;
      int n;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        if (id >= limit_) continue;  // not part of this call
        job = job_;
        n = n_;
      }
      for (int i = next_++; i < n; i = next_++) (*job)(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::function<void(int)>* job_ = nullptr;
  int n_ = 0, limit_ = 0, pending_ = 0;
  std::atomic<int> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace pst
