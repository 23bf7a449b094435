// Config 3 from native code (not product code): the block queue
// (byteps_reduce_blockq_*) driven through its C ABI with no Python in the
// loop, to measure the device-side bound of live Prophet block releases.
// ResNet-50 fp16, 8 workers, 165 partitions in 12 Prophet blocks
// (tools/cfg3_resnet50_table.txt from tools/cfg3_table.py), 3 rotated input
// sets.  One JSON line per variant: per-iteration ms (median / min / max of
// `reps` timed runs of `iters` iterations), fraction of the 8 TB/s roofline at
// (N+1) x bytes per iteration, run-to-run spread, and exactness against one
// plan over all partitions.
// With the task file (tools/cfg3_resnet50_tasks.txt, argv[4]) one more variant
// runs the native Prophet scheduler (include/bpsr/prophet.h) in the loop: per
// iteration the 165 partitions arrive in backward order, one per getTask poll,
// and every release group completes blocks that are released then (one
// release_range per run of consecutive blocks) — Z_BATCH_SIZE 64, Z_NET_B
// 10000, Z_CREDIT 16 MiB (tools/bench_configs.py's setting).
//   usage: cfg3_native [table] [iters] [reps] [tasks|""] [variant substring]
//   hipcc -O2 -std=c++17 -Iinclude -o tools/cfg3_native tools/cfg3_native.cpp \
//         -Lprophet_amd -lbpsr -Wl,-rpath,'$ORIGIN/../prophet_amd'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include <chrono>

#include "bpsr/prophet.h"
#include "bpsr/reduce.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)
#define CKR(x)                                                                           \
  do {                                                                                   \
    int r_ = (x);                                                                        \
    if (r_ != 0) {                                                                       \
      fprintf(stderr, "%s:%d rc=%d %s\n", __FILE__, __LINE__, r_, byteps_reduce_last_error()); \
      exit(3);                                                                           \
    }                                                                                    \
  } while (0)

namespace {
constexpr int N = 8;
constexpr int kSets = 3;

struct Table {
  size_t total = 0;
  std::vector<std::pair<size_t, size_t>> parts;  // (offset, len) in block order
  std::vector<int> block_end;
};

Table read_table(const char* path) {
  Table t;
  FILE* f = fopen(path, "r");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path);
    exit(2);
  }
  int np = 0, nb = 0;
  if (fscanf(f, "%zu %d %d", &t.total, &np, &nb) != 3) exit(2);
  for (int i = 0; i < np; ++i) {
    size_t o, l;
    if (fscanf(f, "%zu %zu", &o, &l) != 2) exit(2);
    t.parts.push_back({o, l});
  }
  for (int i = 0; i < nb; ++i) {
    int e;
    if (fscanf(f, "%d", &e) != 1) exit(2);
    t.block_end.push_back(e);
  }
  fclose(f);
  return t;
}

struct Tasks {
  std::vector<int32_t> cps;
  std::vector<byteps_prophet_task> arrivals;  // backward order; handle = table index
};

Tasks read_tasks(const char* path) {
  Tasks t;
  FILE* f = fopen(path, "r");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path);
    exit(2);
  }
  int nc = 0;
  if (fscanf(f, "%d", &nc) != 1) exit(2);
  t.cps.resize(nc);
  for (auto& c : t.cps)
    if (fscanf(f, "%d", &c) != 1) exit(2);
  int g, p, np;
  long long len;
  for (uint64_t i = 0; fscanf(f, "%d %d %d %lld", &g, &p, &np, &len) == 4; ++i) {
    byteps_prophet_task k;
    std::memset(&k, 0, sizeof(k));
    k.grad = g;
    k.part = p;
    k.total_partnum = np;
    k.len = len;
    k.scheduled = 1;
    k.key = ((uint64_t)g << 16) + (uint64_t)p;
    k.handle = i;
    t.arrivals.push_back(k);
  }
  fclose(f);
  std::sort(t.arrivals.begin(), t.arrivals.end(),
            [](const byteps_prophet_task& a, const byteps_prophet_task& b) {
              return a.grad != b.grad ? a.grad > b.grad : a.part < b.part;
            });
  return t;
}

struct Set {
  std::vector<char*> in;
  char* out = nullptr;
  char* ref = nullptr;
  byteps_reduce_blockq* q = nullptr;
  byteps_reduce_plan* plan_blocks = nullptr;  // all partitions, no block boundaries (bound)
  byteps_reduce_plan* plan_ref = nullptr;     // the same into ref (exactness check)
};

std::vector<byteps_bucket_desc> descs(const Table& t, const Set& s, char* dst) {
  std::vector<byteps_bucket_desc> d(t.parts.size());
  for (size_t i = 0; i < t.parts.size(); ++i) {
    std::memset(&d[i], 0, sizeof(d[i]));
    d[i].dst = dst + t.parts[i].first;
    for (int k = 0; k < N; ++k) d[i].srcs[k] = s.in[k] + t.parts[i].first;
    d[i].len = t.parts[i].second;
    d[i].n = N;
  }
  return d;
}
}  // namespace

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "tools/cfg3_resnet50_table.txt";
  const int iters = argc > 2 ? atoi(argv[2]) : 200;
  const int reps = argc > 3 ? atoi(argv[3]) : 7;
  const char* task_path = argc > 4 && argv[4][0] ? argv[4] : nullptr;
  // optional: run only the variants whose name contains one of argv[5]'s comma-separated substrings (a PMC pass
  // serialises dispatches, so a live variant's consumer could never see its
  // releases: profile "pre_released" / "plan" there)
  const char* only = argc > 5 ? argv[5] : nullptr;
  const Table t = read_table(path);
  const int nb = (int)t.block_end.size();
  Tasks tasks;
  byteps_prophet_queue* sched = nullptr;
  std::vector<int> block_of(t.parts.size()), block_size(nb);
  for (int b = 0, i = 0; b < nb; ++b)
    for (; i < t.block_end[b]; ++i) {
      block_of[i] = b;
      ++block_size[b];
    }
  if (task_path) {
    tasks = read_tasks(task_path);
    if (tasks.arrivals.size() != t.parts.size()) {
      fprintf(stderr, "task file has %zu partitions, table %zu\n", tasks.arrivals.size(),
              t.parts.size());
      return 2;
    }
    byteps_prophet_config pc;
    std::memset(&pc, 0, sizeof(pc));
    pc.batch_size = 64;
    pc.net_b = 10000;
    pc.credit = 16 << 20;
    pc.checkpoints = tasks.cps.data();
    pc.ncheckpoints = (int32_t)tasks.cps.size();
    std::vector<double> ex = {16, 15, 9, 10, 12, 18, 15, 21, 30, 25, 20, 5, 0};
    if (ex.size() != tasks.cps.size()) return 2;
    pc.backward_exec = ex.data();  // copied by create
    CKR(byteps_prophet_create(&pc, &sched));
  }
  // the library's PUSH loop (byteps_prophet_loop_*): one scheduler + loop per
  // input set (each set has its own block queue)
  std::vector<byteps_prophet_queue*> lq(kSets, nullptr);
  std::vector<byteps_prophet_loop*> loops(kSets, nullptr), iloops(kSets, nullptr),
      hloops(kSets, nullptr);
  std::vector<byteps_prophet_queue*> hq(kSets, nullptr);  // host-release loops' schedulers
  std::vector<byteps_reduce_blockq*> hbq(kSets, nullptr);   // and block queues
  std::vector<int> left(nb);
  double sched_us = 0;
  long sched_iters = 0, groups_seen = 0, release_calls = 0;
  CKR(byteps_reduce_init(0));
  // fp16 inputs: random signs and mantissas, exponents around 1 (finite)
  std::vector<uint16_t> host(t.total / 2);
  uint32_t x = 12345u;
  std::vector<Set> sets(kSets);
  for (auto& s : sets) {
    for (int k = 0; k < N; ++k) {
      for (auto& h : host) {
        x = x * 1664525u + 1013904223u;
        h = (uint16_t)(((x >> 16) & 0x83ffu) | (((x >> 8) & 1u) ? 0x3800u : 0x3c00u));
      }
      char* p = nullptr;
      CK(hipMalloc(&p, t.total));
      CK(hipMemcpy(p, host.data(), t.total, hipMemcpyHostToDevice));
      s.in.push_back(p);
    }
    CK(hipMalloc(&s.out, t.total));
    CK(hipMalloc(&s.ref, t.total));
    auto d = descs(t, s, s.out);
    CKR(byteps_reduce_blockq_create(d.data(), (int)d.size(), t.block_end.data(), nb,
                                    BYTEPS_REDUCE_FLOAT16, BYTEPS_REDUCE_MODE_REFERENCE, &s.q));
    CKR(byteps_reduce_blockq_config(s.q, 0, 5.0));
    CKR(byteps_reduce_plan_create(d.data(), (int)d.size(), BYTEPS_REDUCE_FLOAT16,
                                  BYTEPS_REDUCE_MODE_REFERENCE, &s.plan_blocks));
    auto r = descs(t, s, s.ref);
    CKR(byteps_reduce_plan_create(r.data(), (int)r.size(), BYTEPS_REDUCE_FLOAT16,
                                  BYTEPS_REDUCE_MODE_REFERENCE, &s.plan_ref));
  }
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t cons, rel[2];
  if (getenv("CFG3_PRIORITY_CONSUMER")) {  // A/B: a caller stream (fork/join onto the library's)
    CK(hipStreamCreateWithPriority(&cons, hipStreamNonBlocking, hi));
  } else {  // the library's consumer stream: a hardware queue of its own
    void* cs = nullptr;
    CKR(byteps_reduce_blockq_stream(sets[0].q, &cs));
    cons = reinterpret_cast<hipStream_t>(cs);
  }
  CK(hipStreamCreateWithFlags(&rel[0], hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&rel[1], hipStreamNonBlocking));
  for (auto& s : sets) CKR(byteps_reduce_plan_launch(s.plan_ref, cons));
  CK(hipDeviceSynchronize());

  using Fn = std::function<void(int)>;
  const Fn pre_released = [&](int i) {
    Set& s = sets[i % kSets];
    CKR(byteps_reduce_blockq_release(s.q, -1, cons));
    CKR(byteps_reduce_blockq_launch(s.q, cons));
  };
  // launched from a caller's own stream: the library forks the consumer onto
  // its own hardware queue and joins it back (byteps_reduce_blockq_launch)
  const Fn pre_released_forked = [&](int i) {
    Set& s = sets[i % kSets];
    CKR(byteps_reduce_blockq_release(s.q, -1, rel[1]));
    CKR(byteps_reduce_blockq_launch(s.q, rel[1]));
  };
  const Fn live = [&](int i) {  // one release per block, behind the launch, on a second stream
    Set& s = sets[i % kSets];
    CKR(byteps_reduce_blockq_launch(s.q, cons));
    for (int b = 0; b < nb; ++b) CKR(byteps_reduce_blockq_release(s.q, b, rel[0]));
  };
  const Fn live_2streams = [&](int i) {  // releases alternate between two streams
    Set& s = sets[i % kSets];
    CKR(byteps_reduce_blockq_launch(s.q, cons));
    for (int b = 0; b < nb; ++b) CKR(byteps_reduce_blockq_release(s.q, b, rel[b & 1]));
  };
  const Fn live_ranges = [&](int i) {  // release groups of 4 blocks, one kernel each
    Set& s = sets[i % kSets];
    CKR(byteps_reduce_blockq_launch(s.q, cons));
    for (int b = 0; b < nb; b += 4)
      CKR(byteps_reduce_blockq_release_range(s.q, b, std::min(4, nb - b), rel[0]));
  };
  const Fn release_first = [&](int i) {  // releases issued before the launch, other stream
    Set& s = sets[i % kSets];
    for (int b = 0; b < nb; ++b) CKR(byteps_reduce_blockq_release(s.q, b, rel[0]));
    CKR(byteps_reduce_blockq_launch(s.q, cons));
  };
  // the scheduler in the loop: arrivals one per poll, releases per group
  const Fn prophet_live = [&](int i) {
    Set& s = sets[i % kSets];
    CKR(byteps_reduce_blockq_launch(s.q, cons));
    const auto t0 = std::chrono::steady_clock::now();
    CKR(byteps_prophet_reset(sched));
    for (int b = 0; b < nb; ++b) left[b] = block_size[b];
    std::vector<char> done(nb, 0);
    int first_open = 0;  // lowest block not yet released
    size_t next = 0;
    bool in_group = false;
    for (;;) {
      if (next < tasks.arrivals.size()) CKR(byteps_prophet_add_task(sched, &tasks.arrivals[next++]));
      byteps_prophet_task got;
      const int rc = byteps_prophet_get_task(sched, &got, nullptr);
      if (rc < 0) CKR(rc);
      if (rc == 1) {
        in_group = true;
        const int b = block_of[got.handle];
        if (--left[b] == 0) done[b] = 1;
        CKR(byteps_prophet_report_finish(sched, got.len));
        continue;
      }
      if (in_group) {  // end of a release group: release the completed blocks, by runs
        ++groups_seen;
        for (int b = 0; b < nb;) {
          if (done[b] != 1) {
            ++b;
            continue;
          }
          int e = b;
          while (e < nb && done[e] == 1) done[e++] = 2;
          CKR(byteps_reduce_blockq_release_range(s.q, b, e - b, rel[0]));
          ++release_calls;
          b = e;
        }
        while (first_open < nb && done[first_open] == 2) ++first_open;
        in_group = false;
      }
      uint64_t pend = 0;
      CKR(byteps_prophet_pending(sched, &pend));
      if (next >= tasks.arrivals.size() && pend == 0) break;
    }
    if (first_open != nb) {
      fprintf(stderr, "scheduler left blocks unreleased\n");
      exit(5);
    }
    sched_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    ++sched_iters;
  };
  const Fn push_loop_inline = [&](int i) {
    const int k = i % kSets;
    const auto t0 = std::chrono::steady_clock::now();
    CKR(byteps_prophet_loop_begin(iloops[k], cons));
    for (const auto& t : tasks.arrivals) CKR(byteps_prophet_loop_push(iloops[k], &t));
    CKR(byteps_prophet_loop_end(iloops[k], 5.0));
    sched_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    ++sched_iters;
  };
  const Fn push_loop_host = [&](int i) {
    const int k = i % kSets;
    const auto t0 = std::chrono::steady_clock::now();
    CKR(byteps_prophet_loop_begin(hloops[k], cons));
    for (const auto& t : tasks.arrivals) CKR(byteps_prophet_loop_push(hloops[k], &t));
    CKR(byteps_prophet_loop_end(hloops[k], 5.0));
    sched_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    ++sched_iters;
  };
  const Fn push_loop = [&](int i) {
    const int k = i % kSets;
    const auto t0 = std::chrono::steady_clock::now();
    CKR(byteps_prophet_loop_begin(loops[k], cons));
    for (const auto& t : tasks.arrivals) CKR(byteps_prophet_loop_push(loops[k], &t));
    CKR(byteps_prophet_loop_end(loops[k], 5.0));
    sched_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    ++sched_iters;
  };
  // the same with every partition in one push_many (they have all landed):
  // one drain, the ready release groups released as one range
  const Fn push_loop_inline_many = [&](int i) {
    const int k = i % kSets;
    const auto t0 = std::chrono::steady_clock::now();
    CKR(byteps_prophet_loop_begin(iloops[k], cons));
    CKR(byteps_prophet_loop_push_many(iloops[k], tasks.arrivals.data(),
                                      (int32_t)tasks.arrivals.size()));
    CKR(byteps_prophet_loop_end(iloops[k], 5.0));
    sched_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    ++sched_iters;
  };
  const Fn plan_no_blocks = [&](int i) {
    CKR(byteps_reduce_plan_launch(sets[i % kSets].plan_blocks, cons));
  };
  struct V {
    const char* name;
    const Fn* fn;
  };
  std::vector<V> variants = {{"plan_all_partitions_no_blocks", &plan_no_blocks},
                             {"blockq_pre_released", &pre_released},
                             {"blockq_pre_released_forked", &pre_released_forked},
                             {"blockq_live_release", &live},
                             {"blockq_live_release_2streams", &live_2streams},
                             {"blockq_live_release_ranges4", &live_ranges},
                             {"blockq_releases_first_other_stream", &release_first}};
  if (sched) {
    variants.push_back({"blockq_live_prophet_scheduler", &prophet_live});
    byteps_prophet_config pc;
    std::memset(&pc, 0, sizeof(pc));
    const double ex[] = {16, 15, 9, 10, 12, 18, 15, 21, 30, 25, 20, 5, 0};
    pc.batch_size = 64;
    pc.net_b = 10000;
    pc.credit = 16 << 20;
    pc.checkpoints = tasks.cps.data();
    pc.ncheckpoints = (int32_t)tasks.cps.size();
    pc.backward_exec = ex;
    for (int k = 0; k < kSets; ++k) {
      CKR(byteps_prophet_create(&pc, &lq[k]));
      CKR(byteps_prophet_loop_create(lq[k], sets[k].q, block_of.data(), (int32_t)block_of.size(),
                                     nb, rel[0], 0, &loops[k]));
      CKR(byteps_prophet_loop_create(lq[k], sets[k].q, block_of.data(), (int32_t)block_of.size(),
                                     nb, rel[0], BYTEPS_PROPHET_LOOP_INLINE, &iloops[k]));
    }
    variants.push_back({"blockq_prophet_push_loop", &push_loop});
    variants.push_back({"blockq_prophet_push_loop_inline", &push_loop_inline});
    variants.push_back({"blockq_prophet_push_loop_inline_many", &push_loop_inline_many});
    // host releases (data resident): separate block queues, since enabling
    // host releases adds the forwarding workgroup to every later launch
    for (int k = 0; k < kSets; ++k) {
      CKR(byteps_prophet_create(&pc, &hq[k]));
      auto hd = descs(t, sets[k], sets[k].out);
      CKR(byteps_reduce_blockq_create(hd.data(), (int)hd.size(), t.block_end.data(), nb,
                                      BYTEPS_REDUCE_FLOAT16, BYTEPS_REDUCE_MODE_REFERENCE,
                                      &hbq[k]));
      CKR(byteps_reduce_blockq_config(hbq[k], 0, 5.0));
      CKR(byteps_prophet_loop_create(hq[k], hbq[k], block_of.data(), (int32_t)block_of.size(),
                                     nb, nullptr, BYTEPS_PROPHET_LOOP_HOST_RELEASE, &hloops[k]));
    }
    variants.push_back({"blockq_prophet_push_loop_host_release", &push_loop_host});
  }
  const double alg = (double)(N + 1) * (double)t.total;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const V& v : variants) {
    if (only) {  // comma-separated substrings
      bool hit = false;
      std::string list(only);
      for (size_t a = 0; a <= list.size();) {
        size_t b = list.find(',', a);
        if (b == std::string::npos) b = list.size();
        if (b > a && std::strstr(v.name, list.substr(a, b - a).c_str())) hit = true;
        a = b + 1;
      }
      if (!hit) continue;
    }
    sched_us = 0;
    sched_iters = groups_seen = release_calls = 0;
    for (int i = 0; i < 30; ++i) (*v.fn)(i);
    CK(hipDeviceSynchronize());
    std::vector<double> ms;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0, cons));
      for (int i = 0; i < iters; ++i) (*v.fn)(i);
      CK(hipEventRecord(e1, cons));
      CK(hipDeviceSynchronize());
      float el = 0;
      CK(hipEventElapsedTime(&el, e0, e1));
      ms.push_back(el / iters);
    }
    int status = 0;
    for (auto& s : sets) status |= byteps_reduce_blockq_status(s.q, cons);
    bool exact = true;
    std::vector<char> a(t.total), b(t.total);
    for (auto& s : sets) {
      CK(hipMemcpy(a.data(), s.out, t.total, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), s.ref, t.total, hipMemcpyDeviceToHost));
      exact = exact && std::memcmp(a.data(), b.data(), t.total) == 0;
      CK(hipMemset(s.out, 0, t.total));  // the next variant must write it again
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    printf("{\"config\": \"cfg3\", \"driver\": \"native C++ (tools/cfg3_native.cpp)\", "
           "\"variant\": \"%s\", \"n_workers\": %d, \"partitions\": %zu, \"blocks\": %d, "
           "\"bytes_per_worker\": %zu, \"iters\": %d, \"reps\": %d, \"ms\": %.5f, "
           "\"min_ms\": %.5f, \"max_ms\": %.5f, \"spread\": %.4f, \"hbm_frac\": %.4f, "
           "\"status\": %d, \"exact_vs_plan\": %s, \"scheduler_host_us_per_iter\": %.2f, "
           "\"release_groups_per_iter\": %.2f, \"release_calls_per_iter\": %.2f}\n",
           v.name, N, t.parts.size(), nb, t.total, iters, reps, med, ms.front(), ms.back(),
           (ms.back() - ms.front()) / med, alg / (med * 1e-3) / 8e12, status,
           exact ? "true" : "false", sched_iters ? sched_us / sched_iters : 0.0,
           sched_iters ? (double)groups_seen / sched_iters : 0.0,
           sched_iters ? (double)release_calls / sched_iters : 0.0);
    fflush(stdout);
  }
  for (int k = 0; k < kSets; ++k) {
    if (loops[k]) byteps_prophet_loop_destroy(loops[k]);
    if (iloops[k]) byteps_prophet_loop_destroy(iloops[k]);
    if (hloops[k]) byteps_prophet_loop_destroy(hloops[k]);
    if (lq[k]) byteps_prophet_destroy(lq[k]);
    if (hq[k]) byteps_prophet_destroy(hq[k]);
    if (hbq[k]) byteps_reduce_blockq_destroy(hbq[k]);
  }
  if (sched) byteps_prophet_destroy(sched);
  for (auto& s : sets) {
    byteps_reduce_blockq_destroy(s.q);
    byteps_reduce_plan_destroy(s.plan_blocks);
    byteps_reduce_plan_destroy(s.plan_ref);
    for (char* p : s.in) CK(hipFree(p));
    CK(hipFree(s.out));
    CK(hipFree(s.ref));
  }
  return 0;
}
