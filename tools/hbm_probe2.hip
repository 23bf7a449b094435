// Second HBM probe (not product code): the product's tile shape (one
// 256-thread workgroup per tile of 256*VPT 16-B vectors, 8 sources) with
//   * cache-policy bits on loads and stores (buffer ops, aux: 1 = sc0,
//     2 = nt, 16 = sc1 — MI355X_MICROARCH.md / cdna_hip_programming.md T8),
//   * in-place output (dst = source 0, the server's zero-copy accumulator,
//     server.cc:216-218) vs a separate output stream,
//   * slab spacing (skew) between the 9 operands.
//   hipcc -O3 --offload-arch=gfx950 -o tools/hbm_probe2 tools/hbm_probe2.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      exit(2);                                                                        \
    }                                                                                 \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
struct Ops { char* p[9]; };

template <int LAUX, int SAUX, int VPT, bool INPLACE>
__global__ __launch_bounds__(256) void fold8(Ops o, unsigned bytes_per_op) {
  const unsigned tile = blockIdx.x;
  const unsigned off0 = (tile * 256u * VPT + threadIdx.x) * 16u;
  __amdgpu_buffer_rsrc_t r[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) r[k] = __builtin_amdgcn_make_buffer_rsrc(o.p[k], 0, bytes_per_op, 0x00020000);
  f4 acc[VPT];
#pragma unroll
  for (int j = 0; j < VPT; ++j)
    acc[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r[0], off0 + j * 4096u, 0, LAUX));
#pragma unroll
  for (int k = 1; k < 8; ++k) {
    f4 x[VPT];
#pragma unroll
    for (int j = 0; j < VPT; ++j)
      x[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r[k], off0 + j * 4096u, 0, LAUX));
#pragma unroll
    for (int j = 0; j < VPT; ++j) acc[j] += x[j];
  }
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int j = 0; j < VPT; ++j)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, acc[j]), INPLACE ? r[0] : r[8],
                                           off0 + j * 4096u, 0, SAUX);
}

struct V {
  const char* name;
  void (*fn)(Ops, unsigned, int, hipStream_t);
};
template <int LA, int SA, int VPT, bool IP>
static void L(Ops o, unsigned b, int grid, hipStream_t s) {
  hipLaunchKernelGGL((fold8<LA, SA, VPT, IP>), dim3(grid), dim3(256), 0, s, o, b);
}

int main(int argc, char** argv) {
  const size_t B = (size_t)(argc > 1 ? atol(argv[1]) : 256) << 20;
  const int sets = 3;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<V> vs = {
      {"l0_s0", L<0, 0, 4, false>},       {"l2_s2", L<2, 2, 4, false>},
      {"l2_s0", L<2, 0, 4, false>},       {"l0_s2", L<0, 2, 4, false>},
      {"l2_s16", L<2, 16, 4, false>},     {"l2_s18", L<2, 18, 4, false>},
      {"l2_s17", L<2, 17, 4, false>},     {"l3_s2", L<3, 2, 4, false>},
      {"l16_s2", L<16, 2, 4, false>},     {"l18_s18", L<18, 18, 4, false>},
      {"l2_s2_v2", L<2, 2, 2, false>},    {"l2_s2_v8", L<2, 2, 8, false>},
      {"inpl_l2_s2", L<2, 2, 4, true>},   {"inpl_l0_s0", L<0, 0, 4, true>},
      {"inpl_l2_s0", L<2, 0, 4, true>},   {"inpl_l2_s2_v8", L<2, 2, 8, true>},
  };
  const size_t skews[] = {0, 4096, 16384, 65536};
  for (int rep = 0; rep < 2; ++rep) {
    for (size_t skew : skews) {
      const size_t stride = B + skew;
      std::vector<char*> slab(sets);
      for (int s = 0; s < sets; ++s) {
        CK(hipMalloc(&slab[s], 9 * stride));
        CK(hipMemset(slab[s], 0, 9 * stride));
      }
      for (const V& v : vs) {
        float best = 1e30f;
        for (int round = 0; round < 3; ++round) {
          const int reps = 20;
          CK(hipEventRecord(e0, st));
          for (int r = 0; r < reps; ++r) {
            Ops o;
            for (int k = 0; k < 9; ++k) o.p[k] = slab[r % sets] + k * stride;
            // grid derived from the name's VPT suffix
            int VPT = 4;
            for (const char* c = v.name; *c; ++c)
              if (c[0] == '_' && c[1] == 'v') VPT = atoi(c + 2);
            v.fn(o, (unsigned)B, (int)(B / 16 / (256 * VPT)), st);
          }
          CK(hipEventRecord(e1, st));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ms /= reps;
          if (round > 0 && ms < best) best = ms;
        }
        printf("{\"v\": \"%s\", \"skew\": %zu, \"rep\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
               v.name, skew, rep, best, 9.0 * B / (best * 1e-3) / 1e9);
        fflush(stdout);
      }
      for (int s = 0; s < sets; ++s) CK(hipFree(slab[s]));
    }
  }
  return 0;
}
