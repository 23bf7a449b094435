// Config 1 from native threads (not product code): the GPU-resident PS server
// driven through its C ABI the way a ps-lite handler in server.cc would drive
// it — per worker one push thread (non-blocking pushes) and one pull thread
// (zero-copy views), 64 MiB fp32 per worker split into BytePS's 4,096,000-B
// partitions (17 keys).  No Python in the loop.  Prints one JSON line per mode.
// Modes 2 and 3 are the device-resident round (pushes written into the receive
// slots by an RDMA transport — byteps_server_recv_slot, filled once here —
// announced with byteps_server_push_ready; pulls as zero-copy device views,
// byteps_server_pull_device_view): 17 keys and 1 key of 64 MiB.
//   hipcc -O2 -std=c++17 -Iinclude -o tools/cfg1_native tools/cfg1_native.cpp \
//         -Lprophet_amd -lbpsr -Wl,-rpath,'$ORIGIN/../prophet_amd' -lpthread
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "bpsr/server.h"

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                \
    }                                                                         \
  } while (0)
#define CKS(x)                                                                    \
  do {                                                                            \
    int r_ = (x);                                                                 \
    if (r_ != 0) {                                                                \
      fprintf(stderr, "%s:%d rc=%d %s\n", __FILE__, __LINE__, r_, byteps_reduce_last_error()); \
      exit(3);                                                                    \
    }                                                                             \
  } while (0)

namespace {
constexpr int N = 2;
constexpr size_t B = 64u << 20;
constexpr size_t kPart = 4096000;  // global.cc:128-135 partition bound (aligned to 8*local_size)

std::atomic<int> acks{0};
void on_push(void*, uint64_t, int, int status) {
  if (status != 0) {
    fprintf(stderr, "push ack status %d\n", status);
    exit(4);
  }
  acks.fetch_add(1, std::memory_order_relaxed);
}
}  // namespace

int main(int argc, char** argv) {
  const int lanes = argc > 1 ? atoi(argv[1]) : 4;
  const int rounds = argc > 2 ? atoi(argv[2]) : 20;
  const int only = argc > 3 ? atoi(argv[3]) : -1;  // run one mode only (traces)
  std::vector<float*> host(N);
  for (int k = 0; k < N; ++k) {
    CK(hipHostMalloc(reinterpret_cast<void**>(&host[k]), B, hipHostMallocDefault));
    uint32_t x = 1000u + (uint32_t)k;
    for (size_t i = 0; i < B / 4; ++i) {
      x = x * 1664525u + 1013904223u;
      host[k][i] = (float)((int)(x >> 9) - (1 << 22)) / (float)(1 << 20);
    }
  }
  std::vector<std::pair<size_t, size_t>> parts17, parts1{{0, B}};  // (offset, len)
  for (size_t o = 0; o < B; o += kPart) parts17.push_back({o, std::min(kPart, B - o)});

  for (int mode = 0; mode < 4; ++mode) {
    if (only >= 0 && mode != only) continue;
    const int view_pulls = mode == 1;
    const bool device = mode >= 2;
    const auto& parts = mode == 3 ? parts1 : parts17;
    const int P = (int)parts.size();
    byteps_server_config cfg{N, lanes, BYTEPS_SERVER_FUSED, 0, 0};
    byteps_server* srv = nullptr;
    CKS(byteps_server_create(&cfg, &srv));
    std::vector<char*> out(N);
    for (int k = 0; k < N; ++k) CK(hipHostMalloc(reinterpret_cast<void**>(&out[k]), B, 0));
    // init round (non-blocking init pushes; the store = the last call's data)
    acks = 0;
    for (int i = 0; i < P; ++i)
      for (int k = 0; k < N; ++k)
        CKS(byteps_server_push_async(srv, (uint64_t)i, k, (char*)host[k] + parts[i].first,
                                     parts[i].second, BYTEPS_REDUCE_FLOAT32, BYTEPS_SERVER_HOST,
                                     on_push, nullptr));
    while (acks.load() < N * P) std::this_thread::yield();
    if (device)  // the transport's RDMA writes land in the slots (once here)
      for (int i = 0; i < P; ++i)
        for (int k = 0; k < N; ++k) {
          void* slot = nullptr;
          CKS(byteps_server_recv_slot(srv, (uint64_t)i, k, &slot));
          CK(hipMemcpy(slot, (char*)host[k] + parts[i].first, parts[i].second,
                       hipMemcpyHostToDevice));
        }

    std::vector<double> ts;
    for (int r = 0; r < rounds + 2; ++r) {
      std::vector<std::atomic<int>> pushed(N * P);
      for (auto& a : pushed) a = 0;
      const bool check = r == rounds + 1;
      auto t0 = std::chrono::steady_clock::now();
      std::vector<std::thread> th;
      for (int k = 0; k < N; ++k) {
        th.emplace_back([&, k] {  // PushLoop (core_loops.cc:492-528)
          for (int i = 0; i < P; ++i) {
            if (device) {
              CKS(byteps_server_push_ready(srv, (uint64_t)i, k));
              pushed[k * P + i].store(1, std::memory_order_release);
              continue;
            }
            CKS(byteps_server_push_async(srv, (uint64_t)i, k, (char*)host[k] + parts[i].first,
                                         parts[i].second, BYTEPS_REDUCE_FLOAT32,
                                         BYTEPS_SERVER_HOST, on_push, nullptr));
            pushed[k * P + i].store(1, std::memory_order_release);
          }
        });
        th.emplace_back([&, k] {  // PullLoop (core_loops.cc:530-564)
          for (int i = 0; i < P; ++i) {
            while (!pushed[k * P + i].load(std::memory_order_acquire)) std::this_thread::yield();
            if (device) {
              const void* v = nullptr;
              size_t n = 0;
              CKS(byteps_server_pull_device_view(srv, (uint64_t)i, &v, &n));
              if (check) CK(hipMemcpy(out[k] + parts[i].first, v, n, hipMemcpyDeviceToHost));
            } else if (view_pulls) {
              const void* v = nullptr;
              size_t n = 0;
              CKS(byteps_server_pull_host_view(srv, (uint64_t)i, &v, &n));
              if (check) memcpy(out[k] + parts[i].first, v, n);
            } else {
              CKS(byteps_server_pull(srv, (uint64_t)i, out[k] + parts[i].first, parts[i].second,
                                     BYTEPS_SERVER_HOST));
            }
          }
        });
      }
      for (auto& t : th) t.join();
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (r >= 1 && r <= rounds) ts.push_back(s);
    }
    // exactness: a 2-way fold is one fp32 add per element, in either order
    size_t bad = 0;
    for (int k = 0; k < N; ++k) {
      const float* o = reinterpret_cast<const float*>(out[k]);
      for (size_t i = 0; i < B / 4; ++i) {
        const float want = host[0][i] + host[1][i];
        if (memcmp(&o[i], &want, 4) != 0) ++bad;
      }
    }
    std::sort(ts.begin(), ts.end());
    const double med = ts[ts.size() / 2];
    printf("{\"config\": \"cfg1\", \"driver\": \"native C++ threads\", \"layout\": "
           "\"%dkeys_push_pull_threads\", \"pushes\": \"%s\", \"pulls\": "
           "\"%s\", \"lanes\": %d, \"n_workers\": %d, \"bucket_bytes\": %zu, \"round_ms\": %.3f, "
           "\"min_ms\": %.3f, \"gibps\": %.2f, \"exact\": %s}\n", P,
           device ? "byteps_server_push_ready (device-resident slots)" : "byteps_server_push_async",
           device ? "byteps_server_pull_device_view"
                  : view_pulls ? "byteps_server_pull_host_view" : "byteps_server_pull",
           lanes, N, B,
           med * 1e3, ts.front() * 1e3, N * (double)B / med / (1 << 30), bad ? "false" : "true");
    fflush(stdout);
    CKS(byteps_server_destroy(srv));
    for (int k = 0; k < N; ++k) CK(hipHostFree(out[k]));
  }
  for (int k = 0; k < N; ++k) CK(hipHostFree(host[k]));
  return 0;
}
