// Third HBM probe (not product code): does the 8-way fold's rate depend on
// how far apart its 9 streams are in the address space, and does a chunk-
// interleaved slot layout (chunk c of every operand side by side) help?
// Same tile shape as the product (256 threads x VPT 2 x 16 B, one workgroup
// per CU via LDS, nt loads and stores).
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=16 \
//         -o tools/hbm_probe3 tools/hbm_probe3.hip
//   tools/hbm_probe3 <bucket MiB> [reps]
// Layouts (one slab per input set, 3 sets rotated):
//   contig:<pad MiB>   operand k at k * (B + pad + 16 KiB)   (pad 0 = the product's arena)
//   inter:<chunk KiB>  chunk c of operand k at (c * 9 + k) * (chunk + 16 KiB)
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
constexpr int kN = 8, kVpt = 2, kTile = 256 * kVpt * 16;  // 8 KiB per operand per tile

struct Geo {
  char* base;
  unsigned long long op_stride;    // bytes between operands inside a chunk group
  unsigned long long group_stride; // bytes between chunk groups
  unsigned tiles_per_chunk;
};

__global__ __launch_bounds__(256) void fold_geo(Geo g) {
  const unsigned t = blockIdx.x;
  const unsigned c = t / g.tiles_per_chunk, w = t % g.tiles_per_chunk;
  char* tb = g.base + (unsigned long long)c * g.group_stride + (unsigned long long)w * kTile;
  const unsigned off = threadIdx.x * 16u;
  __amdgpu_buffer_rsrc_t r[kN + 1];
#pragma unroll
  for (int k = 0; k <= kN; ++k)
    r[k] = __builtin_amdgcn_make_buffer_rsrc(tb + (unsigned long long)k * g.op_stride, 0, kTile,
                                             0x00020000);
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

// Same tile, arguments as scalars: with -mllvm -amdgpu-kernarg-preload-count
// they arrive in SGPRs at wave launch (a struct argument is not preloaded), so
// no kernarg round trip precedes the first data load.
__global__ __launch_bounds__(256) void fold_geo_sc(char* base, unsigned long long op_stride,
                                                   unsigned long long group_stride,
                                                   unsigned tiles_per_chunk) {
  Geo g{base, op_stride, group_stride, tiles_per_chunk};
  const unsigned t = blockIdx.x;
  const unsigned c = t / g.tiles_per_chunk, w = t % g.tiles_per_chunk;
  char* tb = g.base + (unsigned long long)c * g.group_stride + (unsigned long long)w * kTile;
  const unsigned off = threadIdx.x * 16u;
  __amdgpu_buffer_rsrc_t r[kN + 1];
#pragma unroll
  for (int k = 0; k <= kN; ++k)
    r[k] = __builtin_amdgcn_make_buffer_rsrc(tb + (unsigned long long)k * g.op_stride, 0, kTile,
                                             0x00020000);
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

// T consecutive tiles per workgroup (grid = tiles / T), one after the other:
// PIPE = false: load, add, store each tile in turn; PIPE = true: the next
// tile's loads are issued before the current tile's adds and stores (two
// register sets), so the CU's load stream does not pause at tile boundaries
// and a workgroup is launched / retired once per T tiles.
template <int T, bool PIPE>
__global__ __launch_bounds__(256) void fold_multi(char* base, unsigned long long op_stride) {
  const unsigned off = threadIdx.x * 16u;
  auto rs = [&](unsigned t, int k) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(base + (unsigned long long)t * kTile +
                                                 (unsigned long long)k * op_stride, 0, kTile, 0x00020000);
  };
  auto issue = [&](f4 (&x)[kN][kVpt], unsigned t) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < kN; ++k) {
      const auto r = rs(t, k);
#pragma unroll
      for (int j = 0; j < kVpt; ++j)
        x[k][j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off + j * 4096u, 0, 2));
    }
  };
  auto finish = [&](f4 (&x)[kN][kVpt], unsigned t) __attribute__((always_inline)) {
    const auto rd = rs(t, kN);
#pragma unroll
    for (int j = 0; j < kVpt; ++j) {
      f4 acc = x[0][j];
#pragma unroll
      for (int k = 1; k < kN; ++k) acc += x[k][j];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, acc), rd, off + j * 4096u, 0, 2);
    }
  };
  const unsigned t0 = blockIdx.x * T;
  if constexpr (!PIPE) {
#pragma unroll
    for (int i = 0; i < T; ++i) {
      f4 x[kN][kVpt];
      issue(x, t0 + i);
      finish(x, t0 + i);
    }
  } else {
    f4 a[kN][kVpt], b[kN][kVpt];
    issue(a, t0);
#pragma unroll
    for (int i = 0; i < T; i += 2) {
      if (i + 1 < T) issue(b, t0 + i + 1);
      finish(a, t0 + i);
      if (i + 1 < T) {
        if (i + 2 < T) issue(a, t0 + i + 2);
        finish(b, t0 + i + 1);
      }
    }
  }
}

__global__ void fill_random(unsigned* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    p[i] = (x & 0x807fffffu) | ((126u + (x >> 23) % 3u) << 23);
  }
}

int main(int argc, char** argv) {
  const size_t B = (size_t)(argc > 1 ? atol(argv[1]) : 256) << 20;  // multiple of the chunks
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const size_t skew = 16384;
  std::vector<std::string> layouts = {"contig:0", "inter:64",  "inter:256", "inter:1024",
                                      "inter:4096", "inter:16384", "contig:0", "contig:2",
                                      "contig:768", "inter:1024"};
  if (const char* v = getenv("PROBE3_LAYOUTS")) {
    layouts.clear();
    std::string s(v);
    size_t p = 0;
    while (p < s.size()) {
      size_t q = s.find(',', p);
      if (q == std::string::npos) q = s.size();
      layouts.push_back(s.substr(p, q - p));
      p = q + 1;
    }
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipFuncSetAttribute((const void*)fold_geo, hipFuncAttributeMaxDynamicSharedMemorySize,
                         160 * 1024));
  CK(hipFuncSetAttribute((const void*)fold_geo_sc, hipFuncAttributeMaxDynamicSharedMemorySize,
                         160 * 1024));
  for (const void* k : {(const void*)fold_multi<1, false>, (const void*)fold_multi<2, false>,
                        (const void*)fold_multi<4, false>, (const void*)fold_multi<2, true>,
                        (const void*)fold_multi<4, true>})
    CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const unsigned tiles = (unsigned)(B / kTile);
  for (std::string L : layouts) {
    // "sc-" prefix: the scalar-argument kernel
    const bool sc = L.rfind("sc-", 0) == 0;
    if (sc) L = L.substr(3);
    // "multi:T" / "pipe:T": T tiles per workgroup (contiguous slots)
    int multi = 0;
    bool pipe = false;
    if (L.rfind("multi:", 0) == 0 || L.rfind("pipe:", 0) == 0) {
      pipe = L[0] == 'p';
      multi = atoi(L.c_str() + L.find(':') + 1);
      L = "contig:0";
    }
    const bool inter = L.rfind("inter:", 0) == 0;
    const size_t arg = (size_t)atol(L.c_str() + L.find(':') + 1);
    Geo g{};
    size_t bytes;
    if (inter) {
      const size_t C = arg << 10;
      g.tiles_per_chunk = (unsigned)(C / kTile);
      g.op_stride = C + skew;
      g.group_stride = (kN + 1) * g.op_stride;
      bytes = (B / C) * g.group_stride;
    } else {
      g.tiles_per_chunk = tiles;
      g.op_stride = B + (arg << 20) + skew;
      g.group_stride = 0;
      bytes = (kN + 1) * g.op_stride;
    }
    std::vector<char*> slab(3);
    for (int s = 0; s < 3; ++s) {
      CK(hipMalloc(&slab[s], bytes));
      hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (unsigned*)slab[s], bytes / 4,
                         77u + s);
    }
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0;
    for (int round = 0; round < 4; ++round) {
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) {
        g.base = slab[r % 3];
        if (multi) {
          const unsigned grid = tiles / (unsigned)multi;
          auto k = pipe ? (multi == 2 ? (const void*)fold_multi<2, true> : (const void*)fold_multi<4, true>)
                        : (multi == 1 ? (const void*)fold_multi<1, false>
                                      : multi == 2 ? (const void*)fold_multi<2, false>
                                                   : (const void*)fold_multi<4, false>);
          void* args[] = {&g.base, &g.op_stride};
          CK(hipLaunchKernel(k, dim3(grid), dim3(256), args, 160 * 1024, st));
        } else if (sc)
          hipLaunchKernelGGL(fold_geo_sc, dim3(tiles), dim3(256), 160 * 1024, st, g.base,
                             g.op_stride, g.group_stride, g.tiles_per_chunk);
        else
          hipLaunchKernelGGL(fold_geo, dim3(tiles), dim3(256), 160 * 1024, st, g);
      }
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      if (round > 0) {
        sum += ms;
        if (ms < best) best = ms;
      }
    }
    const float avg = sum / 3;
    printf("{\"probe\": \"hbm_probe3\", \"layout\": \"%s\", \"bucket_mib\": %zu, \"ms_avg\": %.4f, "
           "\"ms_best\": %.4f, \"frac_avg\": %.4f, \"scalar_args\": %d, \"tiles_per_wg\": %d, \"pipelined\": %d}\n",
           L.c_str(), B >> 20, avg, best, (kN + 1.0) * B / (avg * 1e-3) / 8e12, (int)sc, multi ? multi : 1, (int)pipe);
    fflush(stdout);
    for (int s = 0; s < 3; ++s) CK(hipFree(slab[s]));
  }
  return 0;
}
