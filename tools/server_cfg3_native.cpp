// Config 3's key set through the GPU-resident PS server from native threads
// (not product code): ResNet-50 fp16, 8 workers, the 165 BytePS partitions as
// keys (tools/cfg3_resnet50_table.txt, Prophet block order), every push
// device-resident.  Measures what a round of many small keys costs in the
// server's state machine and launches, next to the block queue's one launch
// per iteration (tools/cfg3_native.cpp).  One JSON line per variant:
//   push_ready   the pushes already sit in the receive slots (an RDMA transport
//                writing into HBM, byteps_server_recv_slot): each worker thread
//                only signals arrival for its 165 keys;
//   push_d2d     each worker thread pushes from its own device buffer
//                (byteps_server_push_async, D2D copy into the slot);
//   ..._many     the same through the batched calls (byteps_server_push_ready_many
//                / push_many, then pull_many): one launch per lane per call;
//   ...+device_view  pulls as zero-copy device views of the store
//                (byteps_server_pull_device_view: what a GPUDirect transport
//                sends from); one extra round with copying pulls checks the bits.
// Every round ends when every worker has pulled every key (device pulls).
// Worker threads persist across rounds (a transport's receive threads).
//   hipcc -O2 -std=c++17 -Iinclude -o tools/server_cfg3_native tools/server_cfg3_native.cpp \
//         -Lprophet_amd -lbpsr -Wl,-rpath,'$ORIGIN/../prophet_amd' -lpthread
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "bpsr/server.h"

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
std::atomic<long> acks{0}, pulled{0};
void on_pull(void*, uint64_t, const void*, size_t, int status) {
  if (status) {
    fprintf(stderr, "pull status %d\n", status);
    exit(4);
  }
  pulled.fetch_add(1, std::memory_order_relaxed);
}
void on_push(void*, uint64_t, int, int status) {
  if (status) {
    fprintf(stderr, "push ack status %d\n", status);
    exit(4);
  }
  acks.fetch_add(1, std::memory_order_relaxed);
}
}  // namespace

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "tools/cfg3_resnet50_table.txt";
  const int rounds = argc > 2 ? atoi(argv[2]) : 20;
  const int lanes = argc > 3 ? atoi(argv[3]) : 4;
  const int only = argc > 4 ? atoi(argv[4]) : -1;  // run one variant (0..3), -1 all
  FILE* f = fopen(path, "r");
  if (!f) return 2;
  size_t total = 0;
  int np = 0, nb = 0;
  if (fscanf(f, "%zu %d %d", &total, &np, &nb) != 3) return 2;
  std::vector<std::pair<size_t, size_t>> parts(np);
  for (auto& p : parts)
    if (fscanf(f, "%zu %zu", &p.first, &p.second) != 2) return 2;
  fclose(f);
  // per worker: its gradient vector (device) and its pull destination (device)
  std::vector<char*> grad(N), out(N);
  std::vector<uint16_t> host(total / 2);
  uint32_t x = 777u;
  for (int k = 0; k < N; ++k) {
    for (auto& h : host) {
      x = x * 1664525u + 1013904223u;
      h = (uint16_t)(((x >> 16) & 0x83ffu) | (((x >> 8) & 1u) ? 0x3800u : 0x3c00u));
    }
    CK(hipMalloc(&grad[k], total));
    CK(hipMalloc(&out[k], total));
    CK(hipMemcpy(grad[k], host.data(), total, hipMemcpyHostToDevice));
  }
  const double alg = (double)(N + 1) * (double)total;
  const char* names[] = {"push_ready", "push_d2d", "push_ready_many+pull_many",
                         "push_many_d2d+pull_many", "push_ready+device_view",
                         "push_ready_many+device_view", "one_receive_thread:push_ready+device_view",
                         "one_receive_thread:push_async_d2d+pull_into_async",
                         "push_async_d2d+pull_into_async", "push_blocking_d2d"};
  constexpr int kVariants = 10;
  std::vector<uint64_t> keys(np);
  std::vector<size_t> lens(np);
  for (int i = 0; i < np; ++i) {
    keys[i] = (uint64_t)i;
    lens[i] = parts[i].second;
  }
  for (int variant = 0; variant < kVariants; ++variant) {
    if (only >= 0 && variant != only) continue;
    const bool view = variant >= 4 && variant <= 6;
    const bool many = variant == 2 || variant == 3 || variant == 5;
    const bool ready = variant != 1 && variant != 3 && variant < 7;
    byteps_server_config cfg;
    std::memset(&cfg, 0, sizeof(cfg));
    cfg.num_workers = N;
    cfg.engine_lanes = lanes;
    cfg.policy = BYTEPS_SERVER_FUSED;
    byteps_server* srv = nullptr;
    CKR(byteps_server_create(&cfg, &srv));
    // init round: blocking pushes from every worker thread, keys in order
    {
      std::vector<std::thread> th;
      for (int k = 0; k < N; ++k)
        th.emplace_back([&, k] {
          for (int i = 0; i < np; ++i)
            CKR(byteps_server_push(srv, (uint64_t)i, k, grad[k] + parts[i].first,
                                   parts[i].second, BYTEPS_REDUCE_FLOAT16, BYTEPS_SERVER_DEVICE));
        });
      for (auto& t : th) t.join();
    }
    if (ready) {  // slots hold the pushes already (written once, as by DMA)
      for (int k = 0; k < N; ++k)
        for (int i = 0; i < np; ++i) {
          void* slot = nullptr;
          CKR(byteps_server_recv_slot(srv, (uint64_t)i, k, &slot));
          CK(hipMemcpy(slot, grad[k] + parts[i].first, parts[i].second,
                       hipMemcpyDeviceToDevice));
        }
    }
    uint64_t st0[11] = {0};
    CKR(byteps_server_stats(srv, st0, 11));
    // persistent worker threads (a transport's receive threads), released per
    // round by the driver and joined by a countdown
    std::vector<double> ts;
    std::mutex m;
    std::condition_variable cv;
    int go = -1, left = 0;
    const int total_rounds = rounds + 2 + (view ? 1 : 0);  // + a checking round
    // when each worker's pushes of the round returned (ns since the epoch of
    // steady_clock): the round splits into push phase (max) and pull phase
    std::vector<std::atomic<int64_t>> push_done(N);
    auto stamp = [&](int k) {
      push_done[k].store(std::chrono::duration_cast<std::chrono::nanoseconds>(
                             std::chrono::steady_clock::now().time_since_epoch())
                             .count());
    };
    std::vector<double> push_ts;
    auto one_round = [&](int k, int r) {
      if (variant == 7 || variant == 8) {  // non-blocking device pushes and pulls into device buffers
        if (variant == 7 && k != 0) {
          stamp(k);
          return;
        }
        const int w0 = variant == 7 ? 0 : k, w1 = variant == 7 ? N : k + 1;
        for (int i = 0; i < np; ++i)
          for (int w = w0; w < w1; ++w)
            CKR(byteps_server_push_async(srv, (uint64_t)i, w, grad[w] + parts[i].first,
                                         parts[i].second, BYTEPS_REDUCE_FLOAT16,
                                         BYTEPS_SERVER_DEVICE, on_push, nullptr));
        stamp(k);
        for (int i = 0; i < np; ++i)
          for (int w = w0; w < w1; ++w)
            CKR(byteps_server_pull_into_async(srv, (uint64_t)i, out[w] + parts[i].first,
                                              parts[i].second, BYTEPS_SERVER_DEVICE, on_pull,
                                              nullptr));
        return;
      }
      if (variant == 6) {  // ps-lite's shape: ONE receive thread makes every call
        if (k != 0) {
          stamp(k);
          return;
        }
        for (int i = 0; i < np; ++i)
          for (int w = 0; w < N; ++w) CKR(byteps_server_push_ready(srv, (uint64_t)i, w));
        stamp(0);
        for (int i = 0; i < np; ++i)
          for (int w = 0; w < N; ++w) {
            if (r < rounds + 2) {
              const void* v = nullptr;
              size_t vl = 0;
              CKR(byteps_server_pull_device_view(srv, (uint64_t)i, &v, &vl));
              if (!v || vl != parts[i].second) exit(6);
            } else {  // the checking round: copies into every worker's output
              CKR(byteps_server_pull(srv, (uint64_t)i, out[w] + parts[i].first, parts[i].second,
                                     BYTEPS_SERVER_DEVICE));
            }
          }
        return;
      }
      if (view && r < rounds + 2) {  // zero-copy: every pull is a view of the store
        if (many)
          CKR(byteps_server_push_ready_many(srv, keys.data(), np, k));
        else
          for (int i = 0; i < np; ++i) CKR(byteps_server_push_ready(srv, (uint64_t)i, k));
        stamp(k);
        for (int i = 0; i < np; ++i) {
          const void* v = nullptr;
          size_t vl = 0;
          CKR(byteps_server_pull_device_view(srv, (uint64_t)i, &v, &vl));
          if (!v || vl != parts[i].second) exit(6);
        }
        return;
      }
      if (many) {
            std::vector<const void*> srcs(np);
            std::vector<void*> dsts(np);
            for (int i = 0; i < np; ++i) {
              srcs[i] = grad[k] + parts[i].first;
              dsts[i] = out[k] + parts[i].first;
            }
            if (ready)
              CKR(byteps_server_push_ready_many(srv, keys.data(), np, k));
            else
              CKR(byteps_server_push_many(srv, keys.data(), srcs.data(), lens.data(), np, k,
                                          BYTEPS_REDUCE_FLOAT16, BYTEPS_SERVER_DEVICE));
            stamp(k);
            CKR(byteps_server_pull_many(srv, keys.data(), dsts.data(), lens.data(), np,
                                        BYTEPS_SERVER_DEVICE));
            return;
          }
          for (int i = 0; i < np; ++i) {
            if (ready)
              CKR(byteps_server_push_ready(srv, (uint64_t)i, k));
            else if (variant == 9)  // a per-key blocking transport: blocking device pushes
              CKR(byteps_server_push(srv, (uint64_t)i, k, grad[k] + parts[i].first,
                                     parts[i].second, BYTEPS_REDUCE_FLOAT16, BYTEPS_SERVER_DEVICE));
            else
              CKR(byteps_server_push_async(srv, (uint64_t)i, k, grad[k] + parts[i].first,
                                           parts[i].second, BYTEPS_REDUCE_FLOAT16,
                                           BYTEPS_SERVER_DEVICE, on_push, nullptr));
          }
          stamp(k);
          for (int i = 0; i < np; ++i)
            CKR(byteps_server_pull(srv, (uint64_t)i, out[k] + parts[i].first, parts[i].second,
                                   BYTEPS_SERVER_DEVICE));
    };
    // Round hand-off between the driver and the worker threads.  The
    // one-receive-thread variants (6, 7: ps-lite's shape, a receive thread
    // that is always running) spin on atomics: a condition variable adds two
    // thread wake-ups, 20-40 us, to every round (r04s28: 0.133-0.144 vs
    // 0.114-0.117 ms for variant 6 with device releases).  The 8-thread
    // variants keep the condition variable of rounds 2-3: with 8 busy
    // workers and the server's own threads, spinning idle threads take CPU
    // from them (r04s28: variant 4 0.21 vs 0.29-0.31 ms, variant 0 1.39-1.43
    // vs 1.68-1.76).  CFG3_HANDOFF=spin|cv overrides.
    const char* ho = getenv("CFG3_HANDOFF");
    const bool cv_handoff = ho ? std::string(ho) == "cv" : !(variant == 6 || variant == 7);
    std::atomic<int> go_a{-1}, left_a{0};
    std::vector<std::thread> th;
    for (int k = 0; k < N; ++k)
      th.emplace_back([&, k] {
        for (int r = 0; r < total_rounds; ++r) {
          if (cv_handoff) {
            std::unique_lock<std::mutex> lk(m);
            cv.wait(lk, [&] { return go >= r; });
          } else {
            while (go_a.load(std::memory_order_acquire) < r) __builtin_ia32_pause();
          }
          one_round(k, r);
          if (cv_handoff) {
            std::lock_guard<std::mutex> lk(m);
            if (--left == 0) cv.notify_all();
          } else {
            left_a.fetch_sub(1, std::memory_order_acq_rel);
          }
        }
      });
    for (int r = 0; r < total_rounds; ++r) {
      acks = 0;
      pulled = 0;
      auto t0 = std::chrono::steady_clock::now();
      if (cv_handoff) {
        {
          std::lock_guard<std::mutex> lk(m);
          left = N;
          go = r;
        }
        cv.notify_all();
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return left == 0; });
      } else {
        left_a.store(N, std::memory_order_release);
        go_a.store(r, std::memory_order_release);
        while (left_a.load(std::memory_order_acquire) > 0) __builtin_ia32_pause();
      }
      if (variant == 1 || variant == 7 || variant == 8)
        while (acks.load() < (long)N * np) std::this_thread::yield();
      if (variant == 7 || variant == 8)
        while (pulled.load() < (long)N * np) std::this_thread::yield();
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (r >= 2 && r < rounds + 2) {
        ts.push_back(s);
        int64_t last = 0;
        for (int k = 0; k < N; ++k) last = std::max(last, push_done[k].load());
        const int64_t t0ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                 t0.time_since_epoch()).count();
        push_ts.push_back((double)(last - t0ns) * 1e-9);
      }
    }
    for (auto& t : th) t.join();
    // exactness: every worker's pull equals worker 0's (one store per key)
    bool same = true;
    std::vector<char> a(total), b(total);
    CK(hipMemcpy(a.data(), out[0], total, hipMemcpyDeviceToHost));
    for (int k = 1; k < N; ++k) {
      CK(hipMemcpy(b.data(), out[k], total, hipMemcpyDeviceToHost));
      same = same && std::memcmp(a.data(), b.data(), total) == 0;
    }
    std::sort(ts.begin(), ts.end());
    const double med = ts[ts.size() / 2];
    std::sort(push_ts.begin(), push_ts.end());
    const double push_med = push_ts[push_ts.size() / 2];
    uint64_t st[11] = {0};
    CKR(byteps_server_stats(srv, st, 11));
    for (int i = 0; i < 11; ++i) st[i] -= st0[i];
    const char* rel = getenv("BPSR_SERVER_RELEASE");
    printf("{\"config\": \"cfg3_via_server\", \"driver\": \"native C++ threads "
           "(tools/server_cfg3_native.cpp)\", \"variant\": \"%s\", \"n_workers\": %d, "
           "\"keys\": %d, \"lanes\": %d, \"bytes_per_worker\": %zu, \"round_ms\": %.4f, "
           "\"min_ms\": %.4f, \"us_per_key\": %.2f, \"hbm_frac_of_round\": %.4f, "
           "\"push_phase_ms\": %.4f, \"fold_launches_per_round\": %.1f, "
           "\"rounds_folded_per_round\": %.1f, \"pull_launches_per_round\": %.1f, "
           "\"issuer_ms_per_round\": %.4f, \"push_copy_launches_per_round\": %.1f, "
           "\"release\": \"%s\", \"consumer_launches_per_round\": %.2f, "
           "\"key_releases_per_round\": %.1f, \"service_pulls_per_round\": %.1f, "
           "\"service_launches\": %llu, \"service_pushes_per_round\": %.1f, \"handoff\": \"%s\", "
           "\"pulls_agree\": %s}\n",
           names[variant], N, np, lanes, total, med * 1e3,
           ts.front() * 1e3, med * 1e6 / np, alg / med / 8e12, push_med * 1e3,
           (double)st[0] / total_rounds, (double)st[1] / total_rounds,
           (double)st[2] / total_rounds, (double)st[4] * 1e-6 / total_rounds,
           (double)st[5] / total_rounds, rel ? rel : "launch", (double)st[6] / total_rounds,
           (double)st[7] / total_rounds, (double)st[8] / total_rounds,
           (unsigned long long)st[9], (double)st[10] / total_rounds, cv_handoff ? "condvar" : "spin",
           same ? "true" : "false");
    fflush(stdout);
    CKR(byteps_server_destroy(srv));
  }
  for (int k = 0; k < N; ++k) {
    CK(hipFree(grad[k]));
    CK(hipFree(out[k]));
  }
  return 0;
}
