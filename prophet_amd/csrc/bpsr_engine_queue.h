// Per-lane queue of pending fold jobs for BYTEPS_SERVER_ENABLE_SCHEDULE
// (byteps/server/queue.h:31-105).  Host-only: no HIP types, unit-tested on the
// CPU (tests/cpp/engine_queue_check.cpp).
//
// Ordering.  The reference keeps a heap whose comparator (queue.h:91-97)
// reads a per-key counter `push_cnt_` that Push increments (queue.h:49-53)
// and ClearCounter zeroes once the key's round is complete (server.cc:269-271)
// or after every async push (server.cc:277): the popped message is the one
// whose key has the FEWEST counted pushes, ties broken by the smaller (older)
// message id.  The reference heap
// reads the counters at comparison time, so its pop order drifts from that
// rule once counters change under a built heap; this queue applies the rule
// itself at every pop (linear scan: a lane holds a handful of jobs).  Without
// scheduling it is FIFO, like the reference's plain queue (queue.h:80-82).
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <unordered_map>
#include <utility>

namespace bpsr {

template <class Job>
class EngineQueue {
 public:
  explicit EngineQueue(bool schedule) : schedule_(schedule) {}

  // queue.h:49-58 Push: enqueue, count one push for the key.
  uint64_t push(uint64_t key, Job job) {
    std::lock_guard<std::mutex> g(mu_);
    const uint64_t id = next_id_++;
    items_.push_back(Item{id, key, std::move(job)});
    if (schedule_) ++push_cnt_[key];
    cv_.notify_one();
    return id;
  }

  // A push the reference would have queued as a SUM_RECV message but that
  // this build folds later in one launch (fused policy): counted, not queued.
  void count(uint64_t key) {
    if (!schedule_) return;
    std::lock_guard<std::mutex> g(mu_);
    ++push_cnt_[key];
  }

  // queue.h:85-89 ClearCounter.
  void clear_counter(uint64_t key) {
    if (!schedule_) return;
    std::lock_guard<std::mutex> g(mu_);
    push_cnt_[key] = 0;
  }

  // queue.h:68-83 WaitAndPop.  Returns false once stopped and drained.  A
  // held queue pops nothing until released (debug: lets a test queue several
  // jobs and then watch the order they leave in); stopping overrides a hold.
  bool wait_pop(Job* out, uint64_t* key = nullptr, uint64_t* id = nullptr) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return stop_ || (!held_ && !items_.empty()); });
    if (items_.empty()) return false;
    size_t best = 0;
    if (schedule_) {
      for (size_t i = 1; i < items_.size(); ++i)
        if (before(items_[i], items_[best])) best = i;
    }
    if (key) *key = items_[best].key;
    if (id) *id = items_[best].id;
    *out = std::move(items_[best].job);
    items_.erase(items_.begin() + (std::ptrdiff_t)best);
    return true;
  }

  void hold(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    held_ = on;
    cv_.notify_all();
  }

  void stop() {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    cv_.notify_all();
  }

  size_t size() const {
    std::lock_guard<std::mutex> g(mu_);
    return items_.size();
  }

  uint64_t push_count(uint64_t key) const {
    std::lock_guard<std::mutex> g(mu_);
    auto it = push_cnt_.find(key);
    return it == push_cnt_.end() ? 0 : it->second;
  }

 private:
  struct Item {
    uint64_t id;
    uint64_t key;
    Job job;
  };

  // a runs before b: fewer counted pushes on its key, then the older id
  bool before(const Item& a, const Item& b) const {
    const uint64_t ca = cnt(a.key), cb = cnt(b.key);
    return ca != cb ? ca < cb : a.id < b.id;
  }

  uint64_t cnt(uint64_t key) const {
    auto it = push_cnt_.find(key);
    return it == push_cnt_.end() ? 0 : it->second;
  }

  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Item> items_;
  std::unordered_map<uint64_t, uint64_t> push_cnt_;
  uint64_t next_id_ = 0;
  bool schedule_;
  bool held_ = false;
  bool stop_ = false;
};

}  // namespace bpsr
