// Second HBM probe (not product code): the product's tile shape (one
// 256-thread workgroup per tile of 256*VPT 16-B vectors, 8 sources) with
//   * cache-policy bits on loads and stores (buffer ops, aux: 1 = sc0,
//     2 = nt, 16 = sc1 — MI355X_MICROARCH.md / cdna_hip_programming.md T8),
//   * in-place output (dst = source 0, the server's zero-copy accumulator,
//     server.cc:216-218) vs a separate output stream,
//   * slab spacing (skew) between the 9 operands.
//   hipcc -O3 --offload-arch=gfx950 -Iinclude -o tools/hbm_probe2 tools/hbm_probe2.hip \
//         -Lprophet_amd -lbpsr -Wl,-rpath,'$ORIGIN/../prophet_amd'   ("n8_product" = libbpsr)
#include <hip/hip_runtime.h>

#include "bpsr/reduce.h"

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
struct Ops { char* p[17]; };

// XMAP: blockIdx -> tile.  0 = identity (the product: dispatch order = address
// order); 1 = one contiguous range of tiles per XCD (workgroups go to XCDs
// round-robin, blockIdx % 8); C > 1 = chunks of C consecutive tiles per XCD,
// the 8 XCDs' chunks adjacent (needs grid % (8*C) == 0).
template <int XMAP>
__device__ __forceinline__ unsigned xcd_tile(unsigned bid, unsigned grid) {
  if (XMAP == 0) return bid;
  const unsigned x = bid % 8u, k = bid / 8u;
  if (XMAP == 1) {
    const unsigned per = grid / 8u, rem = grid % 8u;
    return x * per + (x < rem ? x : rem) + k;
  }
  return ((k / XMAP) * 8u + x) * XMAP + k % XMAP;
}

template <int LAUX, int SAUX, int VPT, bool INPLACE, int NSRC = 8, bool INDEP = false,
          int XMAP = 0>
__global__ __launch_bounds__(256) void fold8(Ops o, unsigned bytes_per_op) {
  const unsigned tile = xcd_tile<XMAP>(blockIdx.x, gridDim.x);
  const unsigned off0 = (tile * 256u * VPT + threadIdx.x) * 16u;
  __amdgpu_buffer_rsrc_t r[NSRC + 1];
#pragma unroll
  for (int k = 0; k <= NSRC; ++k) r[k] = __builtin_amdgcn_make_buffer_rsrc(o.p[k], 0, bytes_per_op, 0x00020000);
  f4 acc[VPT];
  if (INDEP) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int j = 0; j < VPT; ++j)   // store first: no dependency on this tile's loads
      __builtin_amdgcn_raw_buffer_store_b128(u4{1, 2, 3, tile}, r[NSRC], off0 + j * 4096u, 0, SAUX);
  }
#pragma unroll
  for (int j = 0; j < VPT; ++j)
    acc[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r[0], off0 + j * 4096u, 0, LAUX));
#pragma unroll
  for (int k = 1; k < NSRC; ++k) {
    f4 x[VPT];
#pragma unroll
    for (int j = 0; j < VPT; ++j)
      x[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r[k], off0 + j * 4096u, 0, LAUX));
#pragma unroll
    for (int j = 0; j < VPT; ++j) acc[j] += x[j];
  }
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  if (INDEP) {
    if (acc[0].x == 12345.f) o.p[16][threadIdx.x] = 1;   // keep the loads alive
    return;
  }
#pragma unroll
  for (int j = 0; j < VPT; ++j)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, acc[j]), INPLACE ? r[0] : r[NSRC],
                                           off0 + j * 4096u, 0, SAUX);
}

// Persistent variant: grid = CUs x k, each workgroup walks tiles with a stride
// of gridDim.x and keeps the next tile's loads in flight while it folds and
// stores the current one (software pipelining in registers).
template <int VPT, int NSRC>
__global__ __launch_bounds__(256) void fold_persist(Ops o, unsigned bytes_per_op, unsigned ntiles) {
  __amdgpu_buffer_rsrc_t r[NSRC + 1];
#pragma unroll
  for (int k = 0; k <= NSRC; ++k) r[k] = __builtin_amdgcn_make_buffer_rsrc(o.p[k], 0, bytes_per_op, 0x00020000);
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  f4 a[NSRC][VPT], b[NSRC][VPT];
  unsigned tile = blockIdx.x;
  if (tile >= ntiles) return;
  auto issue = [&](f4 (&x)[NSRC][VPT], unsigned t) __attribute__((always_inline)) {
    const unsigned off0 = (t * 256u * VPT + threadIdx.x) * 16u;
#pragma unroll
    for (int k = 0; k < NSRC; ++k)
#pragma unroll
      for (int j = 0; j < VPT; ++j)
        x[k][j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r[k], off0 + j * 4096u, 0, 2));
  };
  auto finish = [&](f4 (&x)[NSRC][VPT], unsigned t) __attribute__((always_inline)) {
    const unsigned off0 = (t * 256u * VPT + threadIdx.x) * 16u;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      f4 acc = x[0][j];
#pragma unroll
      for (int k = 1; k < NSRC; ++k) acc += x[k][j];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, acc), r[NSRC], off0 + j * 4096u, 0, 2);
    }
  };
  issue(a, tile);
  for (;;) {
    const unsigned nxt = tile + gridDim.x;
    if (nxt < ntiles) issue(b, nxt);
    finish(a, tile);
    if (nxt >= ntiles) break;
    tile = nxt;
    const unsigned nx2 = tile + gridDim.x;
    if (nx2 < ntiles) issue(a, nx2);
    finish(b, tile);
    if (nx2 >= ntiles) break;
    tile = nx2;
  }
}

__global__ void fill_random(unsigned* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    // finite fp32 in about [-2, 2]: random mantissa/sign, exponent 126..128
    p[i] = (x & 0x807fffffu) | ((126u + (x >> 23) % 3u) << 23);
  }
}

struct V {
  const char* name;
  void (*fn)(Ops, unsigned, int, hipStream_t);
};
template <int LA, int SA, int VPT, bool IP, int NS = 8, bool IND = false, int LDS_KB = 0,
          int XMAP = 0>
static void L(Ops o, unsigned b, int grid, hipStream_t s) {
  // LDS_KB of dynamic LDS per workgroup caps residency (160 KiB per CU)
  hipLaunchKernelGGL((fold8<LA, SA, VPT, IP, NS, IND, XMAP>), dim3(grid), dim3(256), LDS_KB * 1024,
                     s, o, b);
}

template <int VPT, int NS, int GRID_PER_CU, int LDS_KB>
static void P(Ops o, unsigned b, int grid, hipStream_t s) {
  const unsigned ntiles = (unsigned)grid;  // caller passes the tile count
  hipLaunchKernelGGL((fold_persist<VPT, NS>), dim3(256 * GRID_PER_CU), dim3(256), LDS_KB * 1024, s,
                     o, b, ntiles);
}

// The product kernel through the C ABI on the same operands.
template <int NS>
static void PROD(Ops o, unsigned b, int grid, hipStream_t s) {
  (void)grid;
  const void* srcs[NS];
  for (int k = 0; k < NS; ++k) srcs[k] = o.p[k];
  byteps_reduce_sum_n(o.p[NS], srcs, NS, b, BYTEPS_REDUCE_FLOAT32, 0, s);
}

int main(int argc, char** argv) {
  const size_t B = (size_t)(argc > 1 ? atol(argv[1]) : 256) << 20;
  const int sets = 3;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<V> vs_policy = {  // cache policy at the product's shape (aux 2 = nt, 16 = sc1)
      {"n8_v2_wg1cu", L<2, 2, 2, false, 8, false, 160>},
      {"n8_product", PROD<8>},
      {"n8_v2_wg1cu_l2s18", L<2, 18, 2, false, 8, false, 160>},
      {"n8_v2_wg1cu_l2s16", L<2, 16, 2, false, 8, false, 160>},
      {"n8_v2_wg1cu_l18s18", L<18, 18, 2, false, 8, false, 160>},
      {"n8_v2_wg1cu_l18s2", L<18, 2, 2, false, 8, false, 160>},
      {"n8_v2_wg1cu_l3s2", L<3, 2, 2, false, 8, false, 160>},
      {"n8_v2_wg1cu_l2s3", L<2, 3, 2, false, 8, false, 160>},
      {"n8_v2_wg1cu_l2s0", L<2, 0, 2, false, 8, false, 160>},
      {"n8_v2_wg1cu_l2s17", L<2, 17, 2, false, 8, false, 160>},
      {"n8_v2_wg1cu_l2s19", L<2, 19, 2, false, 8, false, 160>},
  };
  std::vector<V> vs = {
      {"n8", L<2, 2, 4, false, 8>},
      {"n8_v2_wg1cu", L<2, 2, 2, false, 8, false, 160>},
      {"n8_product", PROD<8>},
      {"n8_v2_wg1cu_xcdrange", L<2, 2, 2, false, 8, false, 160, 1>},
      {"n8_v2_wg1cu_xcdchunk4", L<2, 2, 2, false, 8, false, 160, 4>},
      {"n8_v2_wg1cu_xcdchunk64", L<2, 2, 2, false, 8, false, 160, 64>},
      {"n8_v2_hw_xcdrange", L<2, 2, 2, false, 8, false, 0, 1>},
      {"n8_v2_hw", L<2, 2, 2, false, 8, false, 0, 0>},
      {"n8_v1_wg2cu", L<2, 2, 1, false, 8, false, 80>},
      {"n8_v4_wg1cu", L<2, 2, 4, false, 8, false, 160>},
      {"n1_copy", L<2, 2, 4, false, 1>},
      {"n16_v2_wg1cu", L<2, 2, 2, false, 16, false, 160>},
  };
  std::vector<V> vs_xmap = {  // blockIdx -> tile maps by bucket size (round 3)
      {"n8_v2_wg1cu", L<2, 2, 2, false, 8, false, 160>},
      {"n8_product", PROD<8>},
      {"n8_v2_wg1cu_xcdchunk4", L<2, 2, 2, false, 8, false, 160, 4>},
      {"n8_v2_wg1cu_xcdchunk16", L<2, 2, 2, false, 8, false, 160, 16>},
      {"n8_v2_wg1cu_xcdchunk64", L<2, 2, 2, false, 8, false, 160, 64>},
      {"n8_v2_wg1cu_xcdchunk256", L<2, 2, 2, false, 8, false, 160, 256>},
  };
  if (getenv("PROBE_POLICY")) vs = vs_policy;
  if (getenv("PROBE_XMAP")) vs = vs_xmap;
  const size_t skews[] = {16384};
  for (int rep = 0; rep < 2; ++rep) {
    for (size_t skew : skews) {
      const size_t stride = B + skew;
      std::vector<char*> slab(sets);
      for (int s = 0; s < sets; ++s) {
        CK(hipMalloc(&slab[s], 17 * stride));
        if (getenv("PROBE_ZERO")) {
          CK(hipMemset(slab[s], 0, 17 * stride));
        } else {
          hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (unsigned*)slab[s],
                             17 * stride / 4, 77u + s);
          CK(hipDeviceSynchronize());
        }
      }
      for (const V& v : vs) {
        float best = 1e30f;
        for (int round = 0; round < 3; ++round) {
          const int reps = 20;
          CK(hipEventRecord(e0, st));
          for (int r = 0; r < reps; ++r) {
            Ops o;
            int ns = atoi(v.name + 1);
            for (int k = 0; k <= ns; ++k) o.p[k] = slab[r % sets] + k * stride;
            for (int k = ns + 1; k < 17; ++k) o.p[k] = slab[r % sets] + 16 * stride;
            // grid derived from the name's VPT suffix
            int VPT = 4;
            for (const char* c = v.name; *c; ++c)
              if (c[0] == '_' && c[1] == 'v' && c[2] >= '0' && c[2] <= '9') VPT = atoi(c + 2);
            v.fn(o, (unsigned)B, (int)(B / 16 / (256 * VPT)), st);
          }
          CK(hipEventRecord(e1, st));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ms /= reps;
          if (round > 0 && ms < best) best = ms;
        }
        const int ns = atoi(v.name + 1);
        printf("{\"v\": \"%s\", \"skew\": %zu, \"rep\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
               v.name, skew, rep, best, (ns + 1.0) * B / (best * 1e-3) / 1e9);
        fflush(stdout);
      }
      for (int s = 0; s < sets; ++s) CK(hipFree(slab[s]));
    }
  }
  return 0;
}
