// Host cost of the HIP calls the server's per-key paths make (not product
// code): per call, from 1 thread and from 8 threads at once, on 4 streams.
//   launch_cost [iters]   -> one JSON line per call kind and thread count
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
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
#define CKR(x)                                                                             \
  do {                                                                                     \
    int r_ = (x);                                                                          \
    if (r_ != 0) {                                                                         \
      fprintf(stderr, "%s:%d rc=%d %s\n", __FILE__, __LINE__, r_, byteps_reduce_last_error()); \
      exit(3);                                                                             \
    }                                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  constexpr int kT = 8, kS = 4, kSrc = 8;
  constexpr size_t kLen = 64 * 1024;
  CK(hipSetDevice(0));
  CKR(byteps_reduce_init(0));
  std::vector<hipStream_t> st(kS);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // per thread: its own buffers and events
  struct Th {
    char* src[kSrc];
    char* dst[4];
    hipEvent_t ev, done;
  };
  std::vector<Th> th(kT);
  for (auto& t : th) {
    for (auto& p : t.src) CK(hipMalloc(&p, kLen));
    for (auto& p : t.dst) CK(hipMalloc(&p, kLen));
    CK(hipEventCreateWithFlags(&t.ev, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&t.done, hipEventDisableTiming));
    CK(hipEventRecord(t.done, st[0]));
  }
  CK(hipDeviceSynchronize());
  using Fn = std::function<void(int, int)>;  // (thread, i)
  const Fn sum_n = [&](int k, int) {
    CKR(byteps_reduce_sum_n(th[k].dst[0], (const void* const*)th[k].src, kSrc, kLen,
                            BYTEPS_REDUCE_FLOAT16, BYTEPS_REDUCE_MODE_REFERENCE, st[k % kS]));
  };
  const Fn batched4 = [&](int k, int) {
    byteps_bucket_desc d[4];
    std::memset(d, 0, sizeof(d));
    for (int b = 0; b < 4; ++b) {
      d[b].dst = th[k].dst[b];
      for (int s = 0; s < kSrc; ++s) d[b].srcs[s] = th[k].src[s];
      d[b].len = kLen;
      d[b].n = kSrc;
    }
    CKR(byteps_reduce_sum_batched(d, 4, BYTEPS_REDUCE_FLOAT16, BYTEPS_REDUCE_MODE_REFERENCE,
                                  st[k % kS]));
  };
  const Fn copy_kernel = [&](int k, int) {
    CKR(byteps_reduce_copy(th[k].dst[1], th[k].src[0], kLen, st[k % kS]));
  };
  const Fn memcpy_d2d = [&](int k, int) {
    CK(hipMemcpyAsync(th[k].dst[1], th[k].src[0], kLen, hipMemcpyDeviceToDevice, st[k % kS]));
  };
  const Fn record = [&](int k, int) { CK(hipEventRecord(th[k].ev, st[k % kS])); };
  const Fn wait_ev = [&](int k, int) { CK(hipStreamWaitEvent(st[k % kS], th[k].done, 0)); };
  const Fn sync_done = [&](int k, int) { CK(hipEventSynchronize(th[k].done)); };
  const Fn query_done = [&](int k, int) { (void)hipEventQuery(th[k].done); };
  const Fn set_device = [&](int, int) { CK(hipSetDevice(0)); };
  struct V {
    const char* name;
    const Fn* fn;
  };
  const V vs[] = {{"byteps_reduce_sum_n 8x64KiB", &sum_n},
                  {"byteps_reduce_sum_batched 4x(8x64KiB)", &batched4},
                  {"byteps_reduce_copy 64KiB", &copy_kernel},
                  {"hipMemcpyAsync D2D 64KiB", &memcpy_d2d},
                  {"hipEventRecord", &record},
                  {"hipStreamWaitEvent", &wait_ev},
                  {"hipEventSynchronize (complete)", &sync_done},
                  {"hipEventQuery (complete)", &query_done},
                  {"hipSetDevice", &set_device}};
  for (const V& v : vs) {
    for (int nt : {1, kT}) {
      for (int k = 0; k < nt; ++k) (*v.fn)(k, 0);  // warm
      CK(hipDeviceSynchronize());
      std::atomic<int> go{0};
      std::vector<double> us(nt);
      std::vector<std::thread> ts;
      for (int k = 0; k < nt; ++k)
        ts.emplace_back([&, k] {
          CK(hipSetDevice(0));
          while (!go.load()) {
          }
          const auto t0 = std::chrono::steady_clock::now();
          for (int i = 0; i < iters; ++i) {
            (*v.fn)(k, i);
            if ((i & 63) == 63 && (v.fn == &sum_n || v.fn == &batched4 || v.fn == &copy_kernel ||
                                   v.fn == &memcpy_d2d))
              CK(hipStreamSynchronize(st[k % kS]));  // bounded queue depth
          }
          us[k] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                      .count() / iters;
        });
      go = 1;
      for (auto& t : ts) t.join();
      CK(hipDeviceSynchronize());
      double mx = 0;
      for (double u : us) mx = u > mx ? u : mx;
      printf("{\"call\": \"%s\", \"threads\": %d, \"us_per_call_per_thread\": %.3f, "
             "\"calls_per_us_all_threads\": %.3f}\n",
             v.name, nt, mx, nt / mx);
      fflush(stdout);
    }
  }
  return 0;
}
