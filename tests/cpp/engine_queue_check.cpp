// CPU unit check of the server's engine queue (prophet_amd/csrc/bpsr_engine_queue.h),
// the BYTEPS_SERVER_ENABLE_SCHEDULE ordering of byteps/server/queue.h:68-97:
// pop the job whose key has the fewest counted pushes, then the oldest.
// Built and run by tests/test_server_host.py; prints "fails=<n>".
#include <atomic>
#include <chrono>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "bpsr_engine_queue.h"

static int fails = 0;
#define CHECK(c)                                                 \
  do {                                                           \
    if (!(c)) {                                                  \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);    \
      ++fails;                                                   \
    }                                                            \
  } while (0)

using Q = bpsr::EngineQueue<std::string>;

static std::vector<std::string> drain(Q& q) {
  std::vector<std::string> out;
  q.stop();
  std::string j;
  while (q.wait_pop(&j)) out.push_back(j);
  return out;
}

int main() {
  {  // no scheduling: FIFO (queue.h:80-82)
    Q q(false);
    q.push(1, "a1");
    q.push(1, "a2");
    q.push(2, "b1");
    q.count(1);
    CHECK(q.push_count(1) == 0);
    auto o = drain(q);
    CHECK((o == std::vector<std::string>{"a1", "a2", "b1"}));
  }
  {  // fewest counted pushes first, ties by age
    Q q(true);
    q.push(1, "a1");
    q.push(1, "a2");
    q.push(2, "b1");
    q.push(3, "c1");
    CHECK(q.push_count(1) == 2 && q.push_count(2) == 1);
    auto o = drain(q);
    CHECK((o == std::vector<std::string>{"b1", "c1", "a1", "a2"}));
  }
  {  // a finished round (ClearCounter, server.cc:269-271) jumps the queue
    Q q(true);
    q.push(1, "a_sum");
    q.push(2, "b_sum1");
    q.push(2, "b_sum2");
    q.push(2, "b_copy_merged");
    q.clear_counter(2);
    auto o = drain(q);
    CHECK((o == std::vector<std::string>{"b_sum1", "b_sum2", "b_copy_merged", "a_sum"}));
  }
  {  // count(): a push folded later (fused policy) still weighs its key
    Q q(true);
    q.push(1, "a");
    q.push(2, "b");
    q.count(1);
    auto o = drain(q);
    CHECK((o == std::vector<std::string>{"b", "a"}));
  }
  {  // counts are read at pop time: a later count reorders queued jobs
    Q q(true);
    q.push(1, "a");
    q.push(2, "b");
    std::string j;
    q.count(2);
    q.count(2);
    CHECK(q.wait_pop(&j) && j == "a");
    CHECK(q.wait_pop(&j) && j == "b");
  }
  {  // hold: nothing pops until released; stop overrides a hold
    Q q(true);
    q.hold(true);
    std::atomic<int> popped{0};
    std::thread t([&] {
      std::string j;
      while (q.wait_pop(&j)) popped++;
    });
    q.push(5, "x");
    q.push(6, "y");
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    CHECK(popped.load() == 0);
    CHECK(q.size() == 2);
    q.hold(false);
    for (int i = 0; i < 200 && popped.load() < 2; ++i)
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    CHECK(popped.load() == 2);
    q.hold(true);
    q.push(7, "z");
    q.stop();
    t.join();
    CHECK(popped.load() == 3);
  }
  std::printf("fails=%d\n", fails);
  return fails ? 1 : 0;
}
