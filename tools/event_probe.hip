// What a completion marker between two folds costs on the device timeline
// (not product code).  The same 8-way fold (a copy of the product tile shape,
// buffer loads, nt, one workgroup per CU) back to back on one stream, with
// after each launch:
//   none        nothing
//   event       hipEventRecord (hipEventDisableTiming)
//   event_dev   hipEventRecord of an event created with hipEventReleaseToDevice
//   ext_stop    no separate record: hipExtLaunchKernel's stopEvent (the kernel's
//               own completion signal updates the event)
//   write32     hipStreamWriteValue32 of a counter into device memory
// Timed with default events around a block of launches queued behind a spin
// kernel, so host issue time is not on the clock.
//   hipcc -O3 --offload-arch=gfx950 -o tools/event_probe tools/event_probe.hip
//   tools/event_probe [MiB per source list] [reps]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));
constexpr int kN = 8, kVpt = 2, kTile = 256 * kVpt * 16;

__global__ __launch_bounds__(256) void fold(char* base, unsigned long long stride) {
  char* tb = base + (unsigned long long)blockIdx.x * kTile;
  const unsigned off = threadIdx.x * 16u;
  __amdgpu_buffer_rsrc_t r[kN + 1];
#pragma unroll
  for (int k = 0; k <= kN; ++k)
    r[k] = __builtin_amdgcn_make_buffer_rsrc(tb + (unsigned long long)k * stride, 0, kTile, 0x00020000);
  f4 acc[kVpt];
#pragma unroll
  for (int j = 0; j < kVpt; ++j)
    acc[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r[0], off + j * 4096u, 0, 2));
#pragma unroll
  for (int k = 1; k < kN; ++k) {
    f4 x[kVpt];
#pragma unroll
    for (int j = 0; j < kVpt; ++j)
      x[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r[k], off + j * 4096u, 0, 2));
#pragma unroll
    for (int j = 0; j < kVpt; ++j) acc[j] += x[j];
  }
#pragma unroll
  for (int j = 0; j < kVpt; ++j)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, acc[j]), r[kN], off + j * 4096u, 0, 2);
}

__global__ void spin(unsigned long long cycles) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
}

int main(int argc, char** argv) {
  std::vector<size_t> mibs = {1, 4, 16, 64, 256};
  if (argc > 1) {
    mibs.clear();
    std::string s(argv[1]);
    size_t p = 0;
    while (p < s.size()) {
      size_t q = s.find(',', p);
      if (q == std::string::npos) q = s.size();
      mibs.push_back((size_t)atol(s.substr(p, q - p).c_str()));
      p = q + 1;
    }
  }
  const int reps0 = argc > 2 ? atoi(argv[2]) : 100;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t t0, t1, ev, ev_dev, ev_ext;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ev_dev, hipEventDisableTiming | hipEventReleaseToDevice));
  CK(hipEventCreateWithFlags(&ev_ext, hipEventDisableTiming));
  CK(hipFuncSetAttribute((const void*)fold, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  unsigned* counter;
  CK(hipMalloc(&counter, 4096));
  const char* modes[] = {"none", "event", "event_dev", "ext_stop", "write32"};
  for (size_t mib : mibs) {
    const size_t B = mib << 20, stride = B + 16384;
    const unsigned tiles = (unsigned)(B / kTile);
    const int reps = (int)std::max<size_t>(10, std::min<size_t>(reps0, reps0 * 64 / std::max<size_t>(mib, 64)));
    std::vector<char*> slab(3);
    for (int s = 0; s < 3; ++s) {
      CK(hipMalloc(&slab[s], stride * (kN + 1)));
      CK(hipMemset(slab[s], 0, stride * (kN + 1)));
    }
    for (int round = 0; round < 2; ++round) {
      for (int m = 0; m < 5; ++m) {
        auto launch = [&](int i) {
          char* b = slab[i % 3];
          if (m == 3) {
            hipExtLaunchKernelGGL(fold, dim3(tiles), dim3(256), 160 * 1024, st, nullptr, ev_ext, 0, b,
                                  (unsigned long long)stride);
          } else {
            hipLaunchKernelGGL(fold, dim3(tiles), dim3(256), 160 * 1024, st, b, (unsigned long long)stride);
            if (m == 1) CK(hipEventRecord(ev, st));
            if (m == 2) CK(hipEventRecord(ev_dev, st));
            if (m == 4) CK(hipStreamWriteValue32(st, counter, (uint32_t)i, 0));
          }
        };
        for (int i = 0; i < 3; ++i) launch(i);
        CK(hipStreamSynchronize(st));
        float best = 1e30f, sum = 0;
        for (int rep = 0; rep < 3; ++rep) {
          hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st, 5000000ull);  // ~50 ms of lead at 100 MHz
          CK(hipEventRecord(t0, st));
          for (int i = 0; i < reps; ++i) launch(i);
          CK(hipEventRecord(t1, st));
          CK(hipEventSynchronize(t1));
          float ms;
          CK(hipEventElapsedTime(&ms, t0, t1));
          ms /= reps;
          sum += ms;
          if (ms < best) best = ms;
        }
        printf("{\"probe\": \"event_probe\", \"mib_per_source\": %zu, \"marker\": \"%s\", \"round\": %d, "
               "\"us_per_fold_avg\": %.2f, \"us_per_fold_best\": %.2f}\n",
               mib, modes[m], round, sum / 3 * 1e3, best * 1e3);
        fflush(stdout);
      }
    }
    for (int s = 0; s < 3; ++s) CK(hipFree(slab[s]));
  }
  return 0;
}
