// Host-only stress of the native Prophet scheduler (bpsr_prophet.cpp, built
// from the library's own source with g++ under a sanitizer by
// tests/test_prophet_native.py): transport threads add tasks (one keeps
// backward order for the scheduled gradients, others feed the FIFO) while an
// engine thread polls getTask and reports each release finished, and a third
// kind of thread reads pending()/state().  Every task must leave exactly once.
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "bpsr/prophet.h"

namespace bpsr {
// the library's fail() lives in bpsr_api.cpp (HIP); a host stand-in here
int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
  return code;
}
}  // namespace bpsr

int main() {
  const int32_t cps[] = {-1, 9, 22, 35, 50, 62, 77, 90, 103, 117, 130, 143, 160};
  const double ex[] = {16, 15, 9, 10, 12, 18, 15, 21, 30, 25, 20, 5, 0};
  byteps_prophet_config cfg;
  std::memset(&cfg, 0, sizeof(cfg));
  cfg.batch_size = 64;
  cfg.net_b = 3;
  cfg.credit = 1 << 20;
  cfg.checkpoints = cps;
  cfg.ncheckpoints = 13;
  cfg.backward_exec = ex;
  int fails = 0;
  for (int iter = 0; iter < 20; ++iter) {
    byteps_prophet_queue* q = nullptr;
    if (byteps_prophet_create(&cfg, &q)) return 2;
    std::vector<byteps_prophet_task> sched;
    uint64_t h = 0;
    for (int g = 160; g >= 0; --g) {
      const int np = 1 + (g % 3 == 0);
      for (int p = 0; p < np; ++p) {
        byteps_prophet_task t;
        std::memset(&t, 0, sizeof(t));
        t.grad = g;
        t.part = p;
        t.len = 1000 + 37 * g;
        t.total_partnum = np;
        t.scheduled = 1;
        t.handle = h++;
        sched.push_back(t);
      }
    }
    const uint64_t nsched = h;
    const int kFifoThreads = 3, kFifo = 200;
    const uint64_t total = nsched + (uint64_t)kFifoThreads * kFifo;
    std::vector<std::atomic<int>> seen(total);
    for (auto& s : seen) s = 0;
    std::atomic<uint64_t> got{0};
    std::atomic<bool> stop{false};
    std::thread poller([&] {
      while (got.load() < total) {
        byteps_prophet_task t;
        int32_t ph = 0;
        const int rc = byteps_prophet_get_task(q, &t, &ph);
        if (rc < 0) {
          ++fails;
          break;
        }
        if (rc == 1) {
          seen[t.handle].fetch_add(1);
          got.fetch_add(1);
          byteps_prophet_report_finish(q, t.len);
        }
      }
    });
    std::thread reader([&] {
      while (!stop.load()) {
        uint64_t n = 0;
        byteps_prophet_state st;
        byteps_prophet_pending(q, &n);
        byteps_prophet_get_state(q, &st);
      }
    });
    std::vector<std::thread> feeders;
    feeders.emplace_back([&] {
      for (auto& t : sched) byteps_prophet_add_task(q, &t);
    });
    for (int f = 0; f < kFifoThreads; ++f)
      feeders.emplace_back([&, f] {
        for (int i = 0; i < kFifo; ++i) {
          byteps_prophet_task t;
          std::memset(&t, 0, sizeof(t));
          t.grad = 5000 + i;
          t.len = 8;
          t.scheduled = 0;
          t.handle = nsched + (uint64_t)f * kFifo + i;
          byteps_prophet_add_task(q, &t);
        }
      });
    for (auto& t : feeders) t.join();
    poller.join();
    stop = true;
    reader.join();
    for (auto& s : seen) fails += s.load() != 1;
    byteps_prophet_destroy(q);
  }
  printf("fails=%d\n", fails);
  return fails ? 1 : 0;
}
