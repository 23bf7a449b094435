// Probe (not product code): does running consecutive config-3 iterations on
// TWO hardware queues (iteration i on queue i % 2) hide a launch's ramp and
// drain behind the neighbour's?  Round 5 adds the library's overlap mode
// (byteps_reduce_blockq_overlap: the same alternation, each launch dispatched
// once every workgroup of the previous one has started) and live releases
// (every block released on a third stream after the launch).  Block queues pre-released (no waiting), and
// the one-launch plan (no blocks), each on one stream vs alternating two
// CU-masked streams (queues of their own); 4 input sets, so iterations that
// share a set share a stream (no overlap between them).  Per-iteration wall
// time over `iters` back-to-back iterations, median of `reps`.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 -Iinclude tools/dbg/overlap_probe.cpp \
//     -o tools/dbg/overlap_probe -Lprophet_amd -lbpsr -Wl,-rpath,'$ORIGIN/../../prophet_amd'
//   tools/dbg/overlap_probe tools/cfg3_resnet50_table.txt 200 5 [skew]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "bpsr/reduce.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)
#define CKR(x)                                                                                  \
  do {                                                                                          \
    int r_ = (x);                                                                               \
    if (r_ != 0) {                                                                              \
      fprintf(stderr, "%s:%d rc=%d %s\n", __FILE__, __LINE__, r_, byteps_reduce_last_error()); \
      exit(3);                                                                                  \
    }                                                                                           \
  } while (0)

namespace {
constexpr int N = 8, kSets = 4;
struct Set {
  std::vector<char*> in;
  char* out = nullptr;
  byteps_reduce_blockq* q = nullptr;
  byteps_reduce_plan* plan = nullptr;
};
}  // namespace

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "tools/cfg3_resnet50_table.txt";
  const int iters = argc > 2 ? atoi(argv[2]) : 200;
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  // skew >= 0: each set's 8 inputs and output are slots of ONE allocation,
  // (total rounded up to 64 KiB) + skew bytes apart (prophet_amd/arena.py);
  // < 0: separate allocations
  const long skew = argc > 4 ? atol(argv[4]) : -1;
  FILE* f = fopen(path, "r");
  if (!f) return 2;
  size_t total = 0;
  int np = 0, nb = 0;
  if (fscanf(f, "%zu %d %d", &total, &np, &nb) != 3) return 2;
  std::vector<std::pair<size_t, size_t>> parts(np);
  for (auto& p : parts)
    if (fscanf(f, "%zu %zu", &p.first, &p.second) != 2) return 2;
  std::vector<int> block_end(nb);
  for (auto& e : block_end)
    if (fscanf(f, "%d", &e) != 1) return 2;
  fclose(f);
  setenv("BPSR_BQ_OWN_QUEUE", "0", 1);  // launch on the stream given (the probe picks queues)
  CKR(byteps_reduce_init(0));
  std::vector<uint16_t> host(total / 2);
  uint32_t x = 12345u;
  std::vector<Set> sets(kSets);
  const size_t stride = ((total + 65535) & ~(size_t)65535) + (size_t)(skew > 0 ? skew : 0);
  for (auto& s : sets) {
    char* slab = nullptr;
    if (skew >= 0) CK(hipMalloc(&slab, stride * (N + 1)));
    for (int k = 0; k < N; ++k) {
      for (auto& h : host) {
        x = x * 1664525u + 1013904223u;
        h = (uint16_t)(((x >> 16) & 0x83ffu) | (((x >> 8) & 1u) ? 0x3800u : 0x3c00u));
      }
      char* p = nullptr;
      if (slab) p = slab + stride * k;
      else CK(hipMalloc(&p, total));
      CK(hipMemcpy(p, host.data(), total, hipMemcpyHostToDevice));
      s.in.push_back(p);
    }
    if (slab) s.out = slab + stride * N;
    else CK(hipMalloc(&s.out, total));
    std::vector<byteps_bucket_desc> d(np);
    for (int i = 0; i < np; ++i) {
      std::memset(&d[i], 0, sizeof(d[i]));
      d[i].dst = s.out + parts[i].first;
      for (int k = 0; k < N; ++k) d[i].srcs[k] = s.in[k] + parts[i].first;
      d[i].len = parts[i].second;
      d[i].n = N;
    }
    CKR(byteps_reduce_blockq_create(d.data(), np, block_end.data(), nb, BYTEPS_REDUCE_FLOAT16,
                                    BYTEPS_REDUCE_MODE_REFERENCE, &s.q));
    CKR(byteps_reduce_blockq_config(s.q, 0, 5.0));
    CKR(byteps_reduce_plan_create(d.data(), np, BYTEPS_REDUCE_FLOAT16,
                                  BYTEPS_REDUCE_MODE_REFERENCE, &s.plan));
  }
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
  for (int c = 0; c < cus; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
  hipStream_t qs[2];
  for (auto& s : qs) CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  CK(hipDeviceSynchronize());
  const double alg = (double)(N + 1) * (double)total;
  auto run = [&](const char* name, const std::function<void(int)>& fn) {
    for (int i = 0; i < 20; ++i) fn(i);
    CK(hipDeviceSynchronize());
    std::vector<double> ts;
    for (int r = 0; r < reps; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < iters; ++i) fn(i);
      CK(hipDeviceSynchronize());
      ts.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
                       .count() / iters);
    }
    for (auto& s : sets) CKR(byteps_reduce_blockq_status(s.q, qs[0]));  // no timeout
    std::sort(ts.begin(), ts.end());
    printf("{\"variant\": \"%s\", \"ms_per_iter\": %.5f, \"min_ms\": %.5f, \"frac_of_roofline\": "
           "%.4f}\n", name, ts[ts.size() / 2], ts.front(), alg / (ts[ts.size() / 2] * 1e-3) / 8e12);
    fflush(stdout);
  };
  hipStream_t rel;
  CK(hipStreamCreateWithFlags(&rel, hipStreamNonBlocking));
  auto overlap = [&](int on) {
    for (auto& s : sets) CKR(byteps_reduce_blockq_overlap(s.q, on));
  };
  for (int pass = 0; pass < 2; ++pass) {
    overlap(0);
    run("blockq_live_1q", [&](int i) {
      Set& s = sets[i % kSets];
      CKR(byteps_reduce_blockq_launch(s.q, qs[0]));
      CKR(byteps_reduce_blockq_release(s.q, -1, rel));
    });
    overlap(1);
    run("blockq_live_overlap", [&](int i) {
      Set& s = sets[i % kSets];
      CKR(byteps_reduce_blockq_launch(s.q, qs[i & 1]));
      CKR(byteps_reduce_blockq_release(s.q, -1, rel));
    });
    run("blockq_pre_released_overlap", [&](int i) {
      Set& s = sets[i % kSets];
      CKR(byteps_reduce_blockq_release(s.q, -1, qs[i & 1]));
      CKR(byteps_reduce_blockq_launch(s.q, qs[i & 1]));
    });
    overlap(0);
    run("blockq_pre_released_1q", [&](int i) {
      Set& s = sets[i % kSets];
      CKR(byteps_reduce_blockq_release(s.q, -1, qs[0]));
      CKR(byteps_reduce_blockq_launch(s.q, qs[0]));
    });
    run("blockq_pre_released_2q", [&](int i) {
      Set& s = sets[i % kSets];
      CKR(byteps_reduce_blockq_release(s.q, -1, qs[i & 1]));
      CKR(byteps_reduce_blockq_launch(s.q, qs[i & 1]));
    });
    run("plan_1q", [&](int i) { CKR(byteps_reduce_plan_launch(sets[i % kSets].plan, qs[0])); });
    run("plan_2q", [&](int i) {
      CKR(byteps_reduce_plan_launch(sets[i % kSets].plan, qs[i & 1]));
    });
  }
  return 0;
}
