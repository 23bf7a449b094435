// Probe (not product code): which streams' kernels wait while a consumer-
// shaped kernel on a CU-masked stream is still dispatching.  A "blocker"
// launch on a dedicated (all-CU-masked) stream has far more workgroups than
// fit at 2 per CU (LDS-capped); each spins until a device flag is set, so the
// launch keeps dispatching for as long as the flag is down.  While it is
// stuck, a one-wave kernel is launched on each of N freshly created streams
// in turn, and the host measures how long each takes to complete (bounded:
// the flag is raised after `hold_ms` regardless).  Streams whose kernel
// completes only after the flag went up share something with the blocker's
// dispatch (a hardware queue or pipe).
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/dbg/pipe_probe.cpp -o tools/dbg/pipe_probe
//   tools/dbg/pipe_probe [nstreams=12] [hold_ms=50] [nblockers=1] [work_us=0] [low=0]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
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

// work_ticks > 0: each workgroup works that long and exits (a consumer whose
// dispatch keeps waiting for slots); 0: spins until the flag (or limit).
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

__global__ void tiny(unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

int main(int argc, char** argv) {
  const int nstreams = argc > 1 ? atoi(argv[1]) : 12;
  const int hold_ms = argc > 2 ? atoi(argv[2]) : 50;
  const int nblockers = argc > 3 ? atoi(argv[3]) : 1;
  const int work_us = argc > 4 ? atoi(argv[4]) : 0;  // > 0: consumer-like workgroups
  const int low = argc > 5 ? atoi(argv[5]) : 0;       // 1: blockers on low-priority streams
  int cus = 0, khz = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
  for (int c = 0; c < cus; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
  unsigned* flag = nullptr;
  CK(hipHostMalloc(&flag, 4, hipHostMallocCoherent | hipHostMallocMapped));
  unsigned* out = nullptr;
  CK(hipMalloc(&out, 4096));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&blocker),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024));
  std::vector<hipStream_t> blk(nblockers);
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  fprintf(stderr, "priority range least %d greatest %d\n", least, greatest);
  for (auto& b : blk) {
    if (low) CK(hipStreamCreateWithPriority(&b, hipStreamNonBlocking, least));
    else CK(hipExtStreamCreateWithCUMask(&b, (uint32_t)mask.size(), mask.data()));
  }
  // streams made the way torch's pool and the library make them
  std::vector<hipStream_t> ss(nstreams);
  for (int i = 0; i < nstreams; ++i) CK(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
  hipStream_t extra;
  CK(hipExtStreamCreateWithCUMask(&extra, (uint32_t)mask.size(), mask.data()));
  CK(hipDeviceSynchronize());
  const unsigned long long limit = (unsigned long long)hold_ms * 4 * (unsigned long long)khz;
  const unsigned long long work_ticks = (unsigned long long)work_us * (unsigned long long)khz / 1000;
  // consumer-like: enough workgroups (2 per CU resident) to keep dispatching ~hold_ms
  const unsigned grid = work_us > 0 ? (unsigned)((unsigned long long)cus * 2 * hold_ms * 1000 / work_us)
                                    : (unsigned)cus * 8;
  auto run = [&](hipStream_t s, int idx, const char* kind) {
    __atomic_store_n(flag, 0u, __ATOMIC_SEQ_CST);
    for (auto& b : blk)
      hipLaunchKernelGGL(blocker, dim3(grid), dim3(256), 80 * 1024, b, flag, limit, work_ticks);
    std::this_thread::sleep_for(std::chrono::milliseconds(2));  // the blockers are dispatching
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, out);
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipEventRecord(ev, s));
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
    printf("{\"stream\": %d, \"kind\": \"%s\", \"tiny_ms\": %.3f, \"blocked\": %s}\n", idx, kind, ms,
           ms >= hold_ms ? "true" : "false");
    fflush(stdout);
  };
  for (int i = 0; i < nstreams; ++i) run(ss[i], i, "plain");
  run(extra, nstreams, "cu_masked");
  CK(hipDeviceSynchronize());
  return 0;
}
