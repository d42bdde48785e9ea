// Persistent worker pool for the search engine's per-round host phases
// (gather, encode, apply).  Round 1 spawned and joined fresh std::threads four
// times per MCTS round (~64 thread creations per 2048-leaf round); here the
// workers sleep on a condition variable between rounds.  run(n, fn) calls
// fn(0..n-1), parts claimed from an atomic counter (so uneven parts balance),
// the calling thread working too.  Every part writes its own outputs, so
// results do not depend on which thread ran which part.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace ag {

class WorkPool {
 public:
  explicit WorkPool(int workers) {
    for (int i = 0; i < workers; ++i) threads_.emplace_back([this]() { loop(); });
  }
  ~WorkPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  WorkPool(const WorkPool&) = delete;
  WorkPool& operator=(const WorkPool&) = delete;

  int workers() const { return (int)threads_.size(); }

  void run(int nparts, const std::function<void(int)>& fn) {
    if (threads_.empty() || nparts <= 1) {
      for (int p = 0; p < nparts; ++p) fn(p);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(m_);
      fn_ = &fn;
      nparts_ = nparts;
      next_.store(0);
      active_ = (int)threads_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [this]() { return active_ == 0; });  // no worker still holds fn_
    fn_ = nullptr;
  }

 private:
  void work() {
    for (int p = next_.fetch_add(1); p < nparts_; p = next_.fetch_add(1)) (*fn_)(p);
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&]() { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      work();
      {
        std::lock_guard<std::mutex> lk(m_);
        if (--active_ == 0) done_.notify_one();
      }
    }
  }

  std::vector<std::thread> threads_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  uint64_t gen_ = 0;
  bool stop_ = false;
  const std::function<void(int)>* fn_ = nullptr;
  int nparts_ = 0;
  std::atomic<int> next_{0};
  int active_ = 0;
};

}  // namespace ag
