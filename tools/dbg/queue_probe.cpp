// Probe (not product code): which hardware queues can dispatch a one-wave
// kernel while a block-queue-shaped consumer occupies the GPU, and whether
// the consumer's shape (dispatch still pending vs whole grid resident)
// matters.  Round 6, VERDICT item 1 (the r05s76 stall).
//
// Streams are made the way torch and libbpsr make them: the NULL stream,
// non-blocking normal-priority streams (pooled onto GPU_MAX_HW_QUEUES
// hardware queues), high/low-priority streams, all-CU-masked streams (a
// hardware queue each).  A tiny kernel records the id of the HSA queue it was
// dispatched from (hsa_queue_t::id via the queue pointer), so each stream is
// tied to its hardware queue.  For each stream and blocker shape the host
// times the tiny kernel's completion (bounded: the blocker's flag goes up
// after hold_ms regardless).  A churn phase then creates and destroys streams
// as the server's lanes do and tests the streams made after it.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/dbg/queue_probe.cpp -o tools/dbg/queue_probe
//   tools/dbg/queue_probe [hold_ms=20]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

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

// Spins until the flag is up (or the limit); work_ticks > 0: exits after that
// long instead (a consumer whose workgroups finish and whose dispatch refills).
__global__ void blocker(const unsigned* flag, unsigned long long limit, unsigned long long work_ticks) {
  extern __shared__ char lds[];
  const unsigned long long t0 = wall_clock64();
  if (threadIdx.x == 0) lds[0] = 0;
  for (;;) {
    if (work_ticks && wall_clock64() - t0 >= work_ticks) return;
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
    if (wall_clock64() - t0 >= limit) return;
    __builtin_amdgcn_s_sleep(8);
  }
}

__global__ void tiny(unsigned long long* out) {
  if (threadIdx.x == 0) {
    const size_t qp = (size_t)__builtin_amdgcn_queue_ptr();
    out[0] = *reinterpret_cast<const unsigned long long*>(qp + 32);
  }
}

struct S {
  hipStream_t s;
  std::string kind;
};

int main(int argc, char** argv) {
  const int hold_ms = argc > 1 ? atoi(argv[1]) : 20;
  int cus = 0, khz = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
  for (int c = 0; c < cus; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
  unsigned* flag = nullptr;
  CK(hipHostMalloc(&flag, 4, hipHostMallocCoherent | hipHostMallocMapped));
  unsigned long long* qid = nullptr;
  CK(hipHostMalloc(&qid, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&blocker),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024));
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t c0, c1;
  CK(hipExtStreamCreateWithCUMask(&c0, (uint32_t)mask.size(), mask.data()));
  CK(hipExtStreamCreateWithCUMask(&c1, (uint32_t)mask.size(), mask.data()));
  std::vector<S> ss;
  ss.push_back({nullptr, "null"});
  for (int i = 0; i < 6; ++i) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ss.push_back({s, "normal"});
  }
  for (int i = 0; i < 2; ++i) {
    hipStream_t s;
    CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest));
    ss.push_back({s, "high"});
  }
  {
    hipStream_t s;
    CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, least));
    ss.push_back({s, "low"});
  }
  ss.push_back({c1, "cu_masked_c1"});
  CK(hipDeviceSynchronize());
  const unsigned long long limit = (unsigned long long)hold_ms * 4 * (unsigned long long)khz;
  const unsigned long long work_ticks = 10ull * (unsigned long long)khz / 1000;  // 10 us tiles

  // blocker shapes: none, gated (8 x resident grid, spinning), persistent
  // (exactly resident, spinning), gated_work (10-us tiles, a refilling dispatch)
  auto run = [&](const char* phase, const S& st, int idx, const char* shape) {
    unsigned grid = 0;
    unsigned long long wt = 0;
    if (!strcmp(shape, "gated")) grid = (unsigned)cus * 8;
    else if (!strcmp(shape, "persistent")) grid = (unsigned)cus * 2;
    else if (!strcmp(shape, "gated_work")) {
      grid = (unsigned)((unsigned long long)cus * 2 * hold_ms * 1000 / 10);
      wt = work_ticks;
    }
    __atomic_store_n(flag, 0u, __ATOMIC_SEQ_CST);
    qid[0] = ~0ull;
    if (grid) hipLaunchKernelGGL(blocker, dim3(grid), dim3(256), 80 * 1024, c0, flag, limit, wt);
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, st.s, qid);
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipEventRecord(ev, st.s));
    double ms = -1;
    for (;;) {
      const double el =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (hipEventQuery(ev) == hipSuccess) {
        ms = el;
        break;
      }
      if (el > hold_ms) __atomic_store_n(flag, 1u, __ATOMIC_SEQ_CST);
      if (el > 4.0 * hold_ms + 1000) break;
    }
    __atomic_store_n(flag, 1u, __ATOMIC_SEQ_CST);
    CK(hipDeviceSynchronize());
    CK(hipEventDestroy(ev));
    printf("{\"phase\": \"%s\", \"stream\": %d, \"kind\": \"%s\", \"hsa_queue\": %lld, "
           "\"blocker\": \"%s\", \"tiny_ms\": %.3f, \"blocked\": %s}\n",
           phase, idx, st.kind.c_str(), (long long)qid[0], shape, ms,
           ms >= hold_ms ? "true" : "false");
    fflush(stdout);
  };
  const char* shapes[] = {"none", "gated", "persistent", "gated_work"};
  {
    S cs{c0, "cu_masked_c0"};
    run("fresh", cs, -1, "none");
  }
  for (size_t i = 0; i < ss.size(); ++i)
    for (const char* sh : shapes) run("fresh", ss[i], (int)i, sh);
  // churn: four rounds of a 4-lane server's streams (3 per lane) made, used, destroyed
  for (int r = 0; r < 4; ++r) {
    std::vector<hipStream_t> lanes(12);
    for (auto& l : lanes) CK(hipStreamCreateWithFlags(&l, hipStreamNonBlocking));
    for (auto& l : lanes) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, l, qid + 1);
    CK(hipDeviceSynchronize());
    for (auto& l : lanes) CK(hipStreamDestroy(l));
  }
  std::vector<S> after;
  for (int i = 0; i < 6; ++i) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    after.push_back({s, "normal_after_churn"});
  }
  for (size_t i = 0; i < after.size(); ++i)
    for (const char* sh : shapes) run("churn", after[i], (int)i, sh);
  for (size_t i = 0; i < ss.size(); ++i) run("churn_old", ss[i], (int)i, "gated");
  CK(hipDeviceSynchronize());
  return 0;
}
