// Probe (not product code), round 6: per hardware queue, how long a release
// takes to take effect while a block-queue-shaped consumer runs on an
// all-CU-masked queue, for three release forms: a one-wave kernel storing a
// pinned host word (the release kernel's shape), a stream write packet
// (hipStreamWriteValue32 of the word) and an event marker (hipEventRecord,
// the host polling hipEventQuery).  The host spins on the word / the event,
// so each sample is enqueue -> visible to the host.  Consumers: none, one
// (on c0) or two (c0 and c1, the overlapped pair), each a dispatch that keeps
// refilling (10-us workgroups at 2 per CU, the gated consumer's shape) for
// the whole measurement.  Streams: the NULL stream, 8 non-blocking normal
// streams (the pool's queues), one high-priority stream.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/dbg/queue_probe2.cpp -o tools/dbg/queue_probe2
//   tools/dbg/queue_probe2 [samples=40]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)

__global__ void consumer_like(const unsigned* stop, unsigned long long work_ticks) {
  extern __shared__ char lds[];
  const unsigned long long t0 = wall_clock64();
  if (threadIdx.x == 0) lds[0] = 0;
  if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return;
  while (wall_clock64() - t0 < work_ticks) __builtin_amdgcn_s_sleep(32);
}

__global__ void store_word(unsigned* w, unsigned v) {
  if (threadIdx.x == 0) __hip_atomic_store(w, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void qid_of(unsigned long long* out) {
  if (threadIdx.x == 0) {
    const size_t qp = (size_t)__builtin_amdgcn_queue_ptr();
    out[0] = *reinterpret_cast<const unsigned long long*>(qp + 32);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int samples = argc > 1 ? atoi(argv[1]) : 40;
  int cus = 0, khz = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  fprintf(stderr, "priority range: least %d greatest %d\n", least, greatest);
  std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
  for (int c = 0; c < cus; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
  unsigned *stop = nullptr, *word = nullptr;
  CK(hipHostMalloc(&stop, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc(&word, 64, hipHostMallocCoherent | hipHostMallocMapped));
  unsigned long long* qid = nullptr;
  CK(hipHostMalloc(&qid, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&consumer_like),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024));
  hipStream_t c[2];
  for (auto& s : c) CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  struct S {
    hipStream_t s;
    std::string kind;
    long long q;
  };
  std::vector<S> ss;
  ss.push_back({nullptr, "null", -1});
  for (int i = 0; i < 8; ++i) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ss.push_back({s, "normal", -1});
  }
  {
    hipStream_t s;
    CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest));
    ss.push_back({s, "high", -1});
  }
  for (int k = 0; k < 2; ++k) {
    CK(hipStreamSynchronize(c[k]));
    qid_of<<<1, 64, 0, c[k]>>>(qid);
    CK(hipStreamSynchronize(c[k]));
    fprintf(stderr, "consumer queue c%d: hsa queue %llu\n", k, qid[0]);
  }
  for (auto& st : ss) {
    qid_of<<<1, 64, 0, st.s>>>(qid);
    CK(hipDeviceSynchronize());
    st.q = (long long)qid[0];
  }
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const unsigned long long work_ticks = 10ull * (unsigned long long)khz / 1000;
  // each consumer launch refills for ~ (grid / (2 * cus)) * 10 us
  const unsigned grid = (unsigned)cus * 2 * 400;  // ~4 ms per launch
  unsigned val = 0;
  // False dependency: stream 1 waits (hipStreamWaitEvent) for a consumer on
  // c0 that runs until `stop`; a release kernel on every other stream is timed.
  {
    hipEvent_t cev;
    CK(hipEventCreateWithFlags(&cev, hipEventDisableTiming));
    for (size_t i = 0; i < ss.size(); ++i) {
      if (i == 1) continue;
      __atomic_store_n(stop, 0u, __ATOMIC_SEQ_CST);
      hipLaunchKernelGGL(consumer_like, dim3((unsigned)cus * 2), dim3(256), 80 * 1024, c[0], stop,
                         (unsigned long long)khz * 20);  // up to 20 ms
      CK(hipEventRecord(cev, c[0]));
      CK(hipStreamWaitEvent(ss[1].s, cev, 0));
      ++val;
      const double t0 = now_us();
      hipLaunchKernelGGL(store_word, dim3(1), dim3(64), 0, ss[i].s, word, val);
      while (__atomic_load_n(word, __ATOMIC_ACQUIRE) != val)
        if (now_us() - t0 > 10000) __atomic_store_n(stop, 1u, __ATOMIC_SEQ_CST);
      const double t1 = now_us();
      __atomic_store_n(stop, 1u, __ATOMIC_SEQ_CST);
      CK(hipDeviceSynchronize());
      printf("{\"test\": \"barrier_on_stream1\", \"stream1_queue\": %lld, \"stream\": %zu, "
             "\"kind\": \"%s\", \"hsa_queue\": %lld, \"release_us\": %.1f, \"blocked\": %s}\n",
             ss[1].q, i, ss[i].kind.c_str(), ss[i].q, t1 - t0, t1 - t0 > 9000 ? "true" : "false");
      fflush(stdout);
    }
  }
  const char* forms[] = {"kernel", "write_value", "event"};
  for (int ncons = 0; ncons <= 2; ++ncons) {
    for (size_t i = 0; i < ss.size(); ++i) {
      if (ncons > 0 && ss[i].s == nullptr) continue;  // the NULL stream waits for c0/c1 (blocking)
      for (const char* form : forms) {
        std::vector<double> lat;
        __atomic_store_n(stop, 0u, __ATOMIC_SEQ_CST);
        int launched = 0;
        double t_launch = 0;
        for (int k = 0; k < samples; ++k) {
          // keep the consumers' dispatch going: relaunch every ~3 ms
          if (ncons > 0 && (launched == 0 || now_us() - t_launch > 3000)) {
            for (int q = 0; q < ncons; ++q)
              hipLaunchKernelGGL(consumer_like, dim3(grid), dim3(256), 80 * 1024, c[q], stop, work_ticks);
            t_launch = now_us();
            ++launched;
            std::this_thread::sleep_for(std::chrono::microseconds(200));
          }
          ++val;
          const double t0 = now_us();
          double t1 = 0;
          if (!strcmp(form, "kernel")) {
            hipLaunchKernelGGL(store_word, dim3(1), dim3(64), 0, ss[i].s, word, val);
            while (__atomic_load_n(word, __ATOMIC_ACQUIRE) != val) {
              if (now_us() - t0 > 200000) break;
            }
            t1 = now_us();
          } else if (!strcmp(form, "write_value")) {
            CK(hipStreamWriteValue32(ss[i].s, word, val, 0));
            while (__atomic_load_n(word, __ATOMIC_ACQUIRE) != val) {
              if (now_us() - t0 > 200000) break;
            }
            t1 = now_us();
          } else {
            CK(hipEventRecord(ev, ss[i].s));
            while (hipEventQuery(ev) != hipSuccess) {
              if (now_us() - t0 > 200000) break;
            }
            t1 = now_us();
          }
          lat.push_back(t1 - t0);
          std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        __atomic_store_n(stop, 1u, __ATOMIC_SEQ_CST);
        CK(hipDeviceSynchronize());
        std::sort(lat.begin(), lat.end());
        printf("{\"consumers\": %d, \"stream\": %zu, \"kind\": \"%s\", \"hsa_queue\": %lld, "
               "\"form\": \"%s\", \"median_us\": %.1f, \"p90_us\": %.1f, \"max_us\": %.1f}\n",
               ncons, i, ss[i].kind.c_str(), ss[i].q, form, lat[lat.size() / 2],
               lat[lat.size() * 9 / 10], lat.back());
        fflush(stdout);
      }
    }
  }
  return 0;
}
