// HBM streaming probe for the fold kernel design (not product code).
//
// Measures, on one MI355X, what a pure streaming pattern can reach so the fold
// kernel's roofline fraction can be read against an achievable ceiling:
//   read-N   : N input streams, per-lane xor into a register, one dword written per thread
//   write    : one output stream (16-B stores)
//   copy     : 1 read + 1 write stream
//   fold-N   : N reads + 1 write (the product's access pattern), fp32 adds
// for two work distributions (grid-stride interleave vs contiguous chunk per
// block), plain vs non-temporal loads/stores, and source spacing (power of
// two vs padded) in one slab.  3 rotated buffer sets defeat the Infinity Cache.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/hbm_probe tools/hbm_probe.hip
//   tools/hbm_probe [bucket_MiB] [N]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kMax = 16;
struct Srcs { const f4* p[kMax]; };

template <bool NTL>
__device__ __forceinline__ f4 ld(const f4* p) {
  if constexpr (NTL) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NTS>
__device__ __forceinline__ void st(f4* p, f4 v) {
  if constexpr (NTS) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// MODE 0 = fold, 1 = read-only, 2 = copy (N=1), 3 = write-only
template <int N, int MODE, bool CHUNK, bool NTL, bool NTS, int VPT>
__global__ __launch_bounds__(256) void probe(Srcs s, f4* dst, unsigned long long nvec,
                                             unsigned long long chunk, float* sink) {
  const unsigned long long t = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
  unsigned long long begin, end, step;
  if (CHUNK) {
    begin = (unsigned long long)blockIdx.x * chunk + threadIdx.x;
    end = (unsigned long long)(blockIdx.x + 1) * chunk;
    if (end > nvec) end = nvec;
    step = 256;
  } else {
    begin = t;
    end = nvec;
    step = (unsigned long long)gridDim.x * 256;
  }
  f4 junk = {0, 0, 0, 0};
  for (unsigned long long v = begin; v < end; v += step * VPT) {
    f4 acc[VPT];
    if constexpr (MODE == 3) {
#pragma unroll
      for (int j = 0; j < VPT; ++j) acc[j] = f4{1.f, 2.f, 3.f, (float)v};
    } else {
#pragma unroll
      for (int j = 0; j < VPT; ++j)
        acc[j] = (v + j * step < end) ? ld<NTL>(s.p[0] + v + j * step) : f4{0, 0, 0, 0};
#pragma unroll
      for (int k = 1; k < N; ++k) {
        f4 x[VPT];
#pragma unroll
        for (int j = 0; j < VPT; ++j)
          x[j] = (v + j * step < end) ? ld<NTL>(s.p[k] + v + j * step) : f4{0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < VPT; ++j) acc[j] += x[j];
      }
    }
    if constexpr (MODE == 1) {
#pragma unroll
      for (int j = 0; j < VPT; ++j) junk += acc[j];
    } else {
#pragma unroll
      for (int j = 0; j < VPT; ++j)
        if (v + j * step < end) st<NTS>(dst + v + j * step, acc[j]);
    }
  }
  if constexpr (MODE == 1) {
    if (junk.x == 1234.5f) sink[t & 1023] = junk.y + junk.z + junk.w;
  }
}

struct Cfg {
  const char* name;
  void (*launch)(Srcs, f4*, unsigned long long, unsigned long long, float*, int, hipStream_t);
  int nsrc;     // streams read
  int writes;   // streams written
  int vpt;
};

template <int N, int MODE, bool CHUNK, bool NTL, bool NTS, int VPT>
static void L(Srcs s, f4* d, unsigned long long nvec, unsigned long long chunk, float* sink,
              int grid, hipStream_t st) {
  hipLaunchKernelGGL((probe<N, MODE, CHUNK, NTL, NTS, VPT>), dim3(grid), dim3(256), 0, st, s, d,
                     nvec, chunk, sink);
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? atol(argv[1]) : 256;
  const size_t B = mib << 20;
  const unsigned long long nvec = B / 16;
  const int sets = 3;
  const size_t pads[] = {0, 65536 * 5 + 4096};
  float* sink;
  CK(hipMalloc(&sink, 4096 * sizeof(float)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  std::vector<Cfg> cfgs = {
      {"fold8_gs_vpt1_ntl_nts", L<8, 0, false, true, true, 1>, 8, 1, 1},
      {"fold8_chunk_vpt4_ntl_nts", L<8, 0, true, true, true, 4>, 8, 1, 4},
      {"fold8_chunk_vpt8_ntl_nts", L<8, 0, true, true, true, 8>, 8, 1, 8},
      {"fold8_chunk_vpt16_ntl_nts", L<8, 0, true, true, true, 16>, 8, 1, 16},
      {"fold8_chunk_vpt8_ntl", L<8, 0, true, true, false, 8>, 8, 1, 8},
      {"fold8_chunk_vpt16_ntl", L<8, 0, true, true, false, 16>, 8, 1, 16},
      {"fold8_chunk_vpt16", L<8, 0, true, false, false, 16>, 8, 1, 16},
      {"read8_gs_vpt1_ntl", L<8, 1, false, true, false, 1>, 8, 0, 1},
      {"copy_gs_vpt1_nt", L<1, 0, false, true, true, 1>, 1, 1, 1},
  };
  const int grids[] = {512, 1024, 2048, 0 /* one chunk (VPT vectors) per thread */};
  for (size_t pad : pads) {
    const size_t stride = B + pad;
    // slab per set: 8 sources + dst, each `stride` apart
    std::vector<char*> slab(sets);
    for (int s = 0; s < sets; ++s) {
      CK(hipMalloc(&slab[s], 9 * stride));
      CK(hipMemset(slab[s], 0, 9 * stride));
    }
    for (const Cfg& c : cfgs) {
      for (int g : grids) {
        const bool chunk = strstr(c.name, "chunk") != nullptr;
        const int vpt = c.vpt;
        int grid = g ? g : (int)((nvec + 256ull * vpt - 1) / (256ull * vpt));
        unsigned long long ch = (nvec + grid - 1) / grid;
        float best = 1e30f, sum = 0;
        const int reps = 20;
        for (int round = 0; round < 3; ++round) {
          CK(hipEventRecord(e0, st));
          for (int r = 0; r < reps; ++r) {
            char* base = slab[r % sets];
            Srcs srcs;
            for (int k = 0; k < kMax; ++k) srcs.p[k] = (const f4*)(base + (k % 8) * stride);
            c.launch(srcs, (f4*)(base + 8 * stride), nvec, ch, sink, grid, st);
          }
          CK(hipEventRecord(e1, st));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ms /= reps;
          if (round > 0) { best = ms < best ? ms : best; sum += ms; }
        }
        const double bytes = (double)B * (c.nsrc + c.writes);
        printf("{\"probe\": \"%s\", \"pad\": %zu, \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
               c.name, pad, grid, best, bytes / (best * 1e-3) / 1e9);
        fflush(stdout);
      }
    }
    for (int s = 0; s < sets; ++s) CK(hipFree(slab[s]));
  }
  return 0;
}
