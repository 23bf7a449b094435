// Probe (not product code): latency of the pull copy service
// (bpsr_copy_service.cpp) against hipMemcpyAsync + hipStreamSynchronize, per
// copy size and number of concurrent posting threads.
//   make -C prophet_amd/csrc && hipcc -O2 -std=c++17 --offload-arch=gfx950 -I include \
//     -I prophet_amd/csrc -c tools/dbg/copysvc_probe.cpp -o prophet_amd/csrc/build/probe.o && \
//   hipcc --offload-arch=gfx950 prophet_amd/csrc/build/probe.o prophet_amd/csrc/build/bpsr_*.o \
//     -o tools/dbg/copysvc_probe -ldl -lpthread
// (linked to the objects: libbpsr.so exports only the byteps_* C ABI)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "bpsr/reduce.h"
#include "bpsr_internal.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
  bpsr::CopyService* svc = nullptr;
  if (bpsr::copysvc_create(0, &svc)) { printf("create failed\n"); return 1; }
  uint64_t* trace = nullptr;
  CK(hipMalloc(&trace, sizeof(uint64_t) * 4 * bpsr::kSvcRing));
  CK(hipMemset(trace, 0, sizeof(uint64_t) * 4 * bpsr::kSvcRing));
  bpsr::copysvc_set_trace(svc, trace);
  int khz = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  std::vector<uint64_t> tr(4 * bpsr::kSvcRing);
  const size_t sizes[] = {4096, 65536, 1u << 20, 8u << 20};
  const int threads[] = {1, 8};
  const int iters = 400;
  for (int T : threads) {
    std::vector<char*> src(T), dst(T);
    std::vector<hipStream_t> st(T);
    for (int t = 0; t < T; ++t) {
      CK(hipMalloc(&src[t], 8u << 20));
      CK(hipMalloc(&dst[t], 8u << 20));
      CK(hipMemset(src[t], t + 1, 8u << 20));
      CK(hipStreamCreateWithFlags(&st[t], hipStreamNonBlocking));
    }
    for (size_t sz : sizes) {
      for (int mode = 0; mode < 2; ++mode) {
        std::vector<std::vector<double>> lat(T);
        const uint64_t p0 = bpsr::copysvc_posted(svc);
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
          th.emplace_back([&, t] {
            for (int i = 0; i < iters; ++i) {
              const auto t0 = std::chrono::steady_clock::now();
              if (mode == 0) {
                if (bpsr::copysvc_copy(svc, dst[t], src[t], sz)) {
                  printf("copy failed: %s\n", byteps_reduce_last_error());
                  fflush(stdout);
                  std::abort();
                }
              } else {
                (void)hipMemcpyAsync(dst[t], src[t], sz, hipMemcpyDeviceToDevice, st[t]);
                (void)hipStreamSynchronize(st[t]);
              }
              lat[t].push_back(std::chrono::duration<double, std::micro>(
                                   std::chrono::steady_clock::now() - t0).count());
            }
          });
        for (auto& x : th) x.join();
        const uint64_t p1 = bpsr::copysvc_posted(svc);
        double fp50 = 0, cp50 = 0, fp90 = 0, cp90 = 0;
        if (mode == 0) {
          CK(hipMemcpy(tr.data(), trace, tr.size() * 8, hipMemcpyDeviceToHost));
          std::vector<double> f, cpy;
          for (uint64_t j = p0 + 20 * T; j < p1; ++j) {
            const uint64_t* t = &tr[(j % bpsr::kSvcRing) * 4];
            // signed: both polling waves stamp [0], so the later one may land
            // after the copier picked the job up (a negative gap, not a wrap)
            f.push_back((double)(int64_t)(t[1] - t[0]) * 1e3 / khz);
            cpy.push_back((double)(t[2] - t[1]) * 1e3 / khz);
          }
          std::sort(f.begin(), f.end());
          std::sort(cpy.begin(), cpy.end());
          if (!f.empty()) {
            fp50 = f[f.size() / 2]; fp90 = f[f.size() * 9 / 10];
            cp50 = cpy[cpy.size() / 2]; cp90 = cpy[cpy.size() * 9 / 10];
          }
        }
        std::vector<double> all;
        for (auto& v : lat) all.insert(all.end(), v.begin() + 20, v.end());
        std::sort(all.begin(), all.end());
        printf("{\"threads\": %d, \"bytes\": %zu, \"path\": \"%s\", \"p50_us\": %.1f, \"p90_us\": %.1f, \"p99_us\": %.1f, "
               "\"fetched_to_picked_p50_p90_us\": [%.1f, %.1f], \"picked_to_copied_p50_p90_us\": [%.1f, %.1f]}\n",
               T, sz, mode == 0 ? "service" : "hipMemcpyAsync+sync", all[all.size() / 2],
               all[all.size() * 9 / 10], all[all.size() * 99 / 100], fp50, fp90, cp50, cp90);
        fflush(stdout);
      }
    }
    std::vector<char> h(8u << 20);
    for (int t = 0; t < T; ++t) {
      CK(hipMemcpy(h.data(), dst[t], 8u << 20, hipMemcpyDeviceToHost));
      if (h[0] != (char)(t + 1) || h[(8u << 20) - 1] != (char)(t + 1)) printf("MISMATCH t=%d\n", t);
    }
  }
  {  // a device-wide synchronisation while 8 threads copy through the service
    const int T = 8;
    std::vector<char*> src(T), dst(T);
    for (int t = 0; t < T; ++t) {
      CK(hipMalloc(&src[t], 1u << 20));
      CK(hipMalloc(&dst[t], 1u << 20));
    }
    std::atomic<bool> stop{false};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        while (!stop.load())
          if (bpsr::copysvc_copy(svc, dst[t], src[t], 64u << 10)) std::abort();
      });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    std::vector<double> s;
    for (int i = 0; i < 200; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      CK(hipDeviceSynchronize());
      s.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
      std::this_thread::sleep_for(std::chrono::microseconds(1500));
    }
    stop.store(true);
    for (auto& x : th) x.join();
    std::sort(s.begin(), s.end());
    printf("{\"device_sync_under_8_copiers_us\": {\"p50\": %.0f, \"p90\": %.0f, \"p99\": %.0f, \"max\": %.0f}}\n",
           s[s.size() / 2], s[s.size() * 9 / 10], s[s.size() * 99 / 100], s.back());
  }
  printf("launches %llu\n", (unsigned long long)bpsr::copysvc_launches(svc));
  bpsr::copysvc_destroy(svc);
  return 0;
}
