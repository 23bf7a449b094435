// CDNA4 (gfx950) kernels of the gradient-bucket reduce path.
//
//   fold_kernel     dst = ((s0 + s1) + ...) + s_{n-1}, one bucket, one launch.
//                   Replaces the (N-1) CpuReducer::sum calls of one server
//                   round (server.cc:216-250, cpu_reducer.cc:86-91) with a
//                   single pass: (N+1)*B HBM bytes instead of (3N-1)*B.
//   batched_kernel  the same over a table of buckets (one Prophet block,
//                   scheduled_queue.cc:244-296) in one launch.
//   copy_kernel     CpuReducer::copy (cpu_reducer.cc:209-220).
//
// Design (pure HBM streaming, no reuse, no MFMA):
//   * 16-byte (dwordx4) loads/stores, lane i of a wave at base + 16*i, so one
//     wave-instruction moves 1 KiB contiguous;
//   * VPT independent 16-B vectors per thread per source, spaced one grid
//     stride apart, all N sources' loads of an iteration issued before the
//     dependent adds consume them (N*VPT loads in flight per lane);
//   * strict left fold in registers (no reassociation: bit-exact with the
//     reference order), one store per vector;
//   * optional non-temporal (nt) loads for the once-read inputs;
//   * head/tail elements that do not fill a 16-B vector (and the fp16
//     F16C-tail region, cpu_reducer.cc:118-125) go through the element path
//     with the reference's tail semantics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bpsr_internal.h"
#include "bpsr_ops.h"

namespace bpsr {

template <bool NT>
__device__ __forceinline__ vec16 ld16(const unsigned char* p) {
  if constexpr (NT) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    u4 v = __builtin_nontemporal_load(reinterpret_cast<const u4*>(p));
    return bitcast<vec16>(v);
  } else {
    return *reinterpret_cast<const vec16*>(p);
  }
}

__device__ __forceinline__ void st16(unsigned char* p, const vec16& v) {
  *reinterpret_cast<vec16*>(p) = v;
}

template <class E, bool ALIGNED>
__device__ __forceinline__ E ld_e(const unsigned char* p) {
  if constexpr (ALIGNED) {
    return *reinterpret_cast<const E*>(p);
  } else {
    E v;
    __builtin_memcpy(&v, p, sizeof(E));
    return v;
  }
}

template <class E, bool ALIGNED>
__device__ __forceinline__ void st_e(unsigned char* p, E v) {
  if constexpr (ALIGNED) {
    *reinterpret_cast<E*>(p) = v;
  } else {
    __builtin_memcpy(p, &v, sizeof(E));
  }
}

// Vector part of one bucket: vectors [v_begin, v_end) of the 16-B range that
// starts at byte `vec_off` of every operand, visited by `t` in steps of
// `stride` threads, VPT vectors per step.
template <class Op, int VPT, bool NT, int NS>
__device__ __forceinline__ void fold_vectors(const unsigned char* const* srcs, int n,
                                             unsigned char* dst, uint64_t vec_off,
                                             uint64_t nvec, uint64_t t, uint64_t stride) {
  const int ns = NS > 0 ? NS : n;
  uint64_t v = t;
  // Full steps: all VPT vectors in range, no guards.
  for (; v + (VPT - 1) * stride < nvec; v += VPT * stride) {
    typename Op::Acc acc[VPT];
    const uint64_t off0 = vec_off + v * 16;
#pragma unroll
    for (int j = 0; j < VPT; ++j) acc[j] = Op::init(ld16<NT>(srcs[0] + off0 + j * stride * 16));
    if constexpr (NS > 0) {
#pragma unroll
      for (int k = 1; k < NS; ++k) {
        vec16 x[VPT];
#pragma unroll
        for (int j = 0; j < VPT; ++j) x[j] = ld16<NT>(srcs[k] + off0 + j * stride * 16);
#pragma unroll
        for (int j = 0; j < VPT; ++j) Op::accum(acc[j], x[j]);
      }
    } else {
#pragma unroll 4
      for (int k = 1; k < ns; ++k) {
        vec16 x[VPT];
#pragma unroll
        for (int j = 0; j < VPT; ++j) x[j] = ld16<NT>(srcs[k] + off0 + j * stride * 16);
#pragma unroll
        for (int j = 0; j < VPT; ++j) Op::accum(acc[j], x[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < VPT; ++j) st16(dst + off0 + j * stride * 16, Op::finish(acc[j]));
  }
  // Remainder: fewer than VPT vectors left for this thread.
  for (; v < nvec; v += stride) {
    const uint64_t off = vec_off + v * 16;
    typename Op::Acc acc = Op::init(ld16<NT>(srcs[0] + off));
    for (int k = 1; k < ns; ++k) Op::accum(acc, ld16<NT>(srcs[k] + off));
    st16(dst + off, Op::finish(acc));
  }
}

// Element part: elements [0, head) and [tail_begin, n_elems) plus trailing
// bytes; `tail_sem_from` = first element index with F16C-tail semantics.
template <class Op, bool ALIGNED>
__device__ __forceinline__ void fold_elements(const unsigned char* const* srcs, int n,
                                              unsigned char* dst, const FoldGeom& g,
                                              uint64_t t, uint64_t stride) {
  using E = typename Op::E;
  const uint64_t n_head = g.head_elems;
  const uint64_t n_tail = g.n_elems - g.tail_begin;
  const uint64_t n_scalar = n_head + n_tail;
  for (uint64_t s = t; s < n_scalar; s += stride) {
    const uint64_t e = s < n_head ? s : g.tail_begin + (s - n_head);
    const bool tail = e >= g.tail_sem_from;
    const uint64_t off = e * sizeof(E);
    typename Op::EAcc acc = Op::init_e(ld_e<E, ALIGNED>(srcs[0] + off), tail);
    for (int k = 1; k < n; ++k) Op::accum_e(acc, ld_e<E, ALIGNED>(srcs[k] + off), tail);
    st_e<E, ALIGNED>(dst + off, Op::finish_e(acc, tail));
  }
  // Trailing len % sizeof(T) bytes: the fold's accumulator is the first
  // arrival (server.cc:216-218), so they come from srcs[0].
  if (g.copy_trailing) {
    const uint64_t tb = g.n_elems * sizeof(E);
    for (uint64_t b = t; b < g.trailing_bytes; b += stride) dst[tb + b] = srcs[0][tb + b];
  }
}

template <class Op, int VPT, bool NT, int NS, bool ALIGNED>
__global__ __launch_bounds__(kBlock) void fold_kernel(FoldArgs a) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  fold_vectors<Op, VPT, NT, NS>(a.srcs, a.n, a.dst, a.g.vec_off, a.g.nvec, t, stride);
  fold_elements<Op, ALIGNED>(a.srcs, a.n, a.dst, a.g, t, stride);
}

// Batched: block b works on tile b of the concatenated tile space; a bucket's
// tiles are [tile_start[i], tile_start[i+1]).  Each tile is kBlock*VPT
// vectors of one bucket.  Element work of every bucket is done by the bucket's
// first tile.
template <class Op, int VPT, bool NT>
__global__ __launch_bounds__(kBlock) void batched_kernel(const BatchEntry* __restrict__ tab,
                                                         const uint32_t* __restrict__ tile_start,
                                                         int nbuckets, uint32_t ntiles) {
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // binary search: last i with tile_start[i] <= tile
    int lo = 0, hi = nbuckets - 1;
    while (lo < hi) {
      int mid = (lo + hi + 1) >> 1;
      if (tile_start[mid] <= tile) lo = mid; else hi = mid - 1;
    }
    const BatchEntry& e = tab[lo];
    const uint32_t local = tile - tile_start[lo];
    const uint64_t tile_vecs = (uint64_t)kBlock * VPT;
    const uint64_t v0 = (uint64_t)local * tile_vecs;
    const uint64_t nv = e.g.nvec > v0 ? (e.g.nvec - v0 < tile_vecs ? e.g.nvec - v0 : tile_vecs) : 0;
    // Within the tile: kBlock threads, stride kBlock, VPT vectors each.
    fold_vectors<Op, VPT, NT, 0>(e.srcs, e.n, e.dst, e.g.vec_off + v0 * 16, nv, threadIdx.x,
                                 kBlock);
    if (local == 0) {
      if (e.aligned) fold_elements<Op, true>(e.srcs, e.n, e.dst, e.g, threadIdx.x, kBlock);
      else fold_elements<Op, false>(e.srcs, e.n, e.dst, e.g, threadIdx.x, kBlock);
    }
  }
}

__global__ __launch_bounds__(kBlock) void copy_kernel(unsigned char* __restrict__ dst,
                                                      const unsigned char* __restrict__ src,
                                                      uint64_t head, uint64_t nvec,
                                                      uint64_t len) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t v = t; v < nvec; v += stride)
    st16(dst + head + v * 16, *reinterpret_cast<const vec16*>(src + head + v * 16));
  const uint64_t tail_begin = head + nvec * 16;
  const uint64_t nscalar = head + (len - tail_begin);
  for (uint64_t s = t; s < nscalar; s += stride) {
    const uint64_t b = s < head ? s : tail_begin + (s - head);
    dst[b] = src[b];
  }
}

// ------------------------------------------------------------- launchers ----

template <class Op, int VPT, bool NT, int NS>
static hipError_t launch_fold_ns(const FoldArgs& a, int grid, hipStream_t s) {
  if (a.aligned)
    hipLaunchKernelGGL((fold_kernel<Op, VPT, NT, NS, true>), dim3(grid), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((fold_kernel<Op, VPT, NT, NS, false>), dim3(grid), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

template <class Op, int VPT, bool NT>
static hipError_t launch_fold_vpt(const FoldArgs& a, int grid, hipStream_t s) {
  switch (a.n) {  // compile-time source counts for the common worker counts
    case 2: return launch_fold_ns<Op, VPT, NT, 2>(a, grid, s);
    case 4: return launch_fold_ns<Op, VPT, NT, 4>(a, grid, s);
    case 8: return launch_fold_ns<Op, VPT, NT, 8>(a, grid, s);
    case 16: return launch_fold_ns<Op, VPT, NT, 16>(a, grid, s);
    default: return launch_fold_ns<Op, VPT, NT, 0>(a, grid, s);
  }
}

template <class Op>
static hipError_t launch_fold_op(const FoldArgs& a, const Tuning& tu, hipStream_t s) {
  const int grid = fold_grid(a.g, tu);
  if (tu.nt) {
    switch (tu.vpt) {
      case 1: return launch_fold_vpt<Op, 1, true>(a, grid, s);
      case 2: return launch_fold_vpt<Op, 2, true>(a, grid, s);
      default: return launch_fold_vpt<Op, 4, true>(a, grid, s);
    }
  }
  switch (tu.vpt) {
    case 1: return launch_fold_vpt<Op, 1, false>(a, grid, s);
    case 2: return launch_fold_vpt<Op, 2, false>(a, grid, s);
    default: return launch_fold_vpt<Op, 4, false>(a, grid, s);
  }
}

hipError_t launch_fold(const FoldArgs& a, int dtype, int mode, const Tuning& tu,
                       hipStream_t s) {
  switch (dtype) {
    case kFloat32: return launch_fold_op<OpF32>(a, tu, s);
    case kFloat64: return launch_fold_op<OpF64>(a, tu, s);
    case kFloat16:
      return mode == kModeAccumF32 ? launch_fold_op<OpAcc16<false>>(a, tu, s)
                                   : launch_fold_op<OpF16>(a, tu, s);
    case kBFloat16:
      return mode == kModeAccumF32 ? launch_fold_op<OpAcc16<true>>(a, tu, s)
                                   : launch_fold_op<OpBF16>(a, tu, s);
    case kUInt8:
    case kInt8: return launch_fold_op<OpI8>(a, tu, s);
    case kInt32: return launch_fold_op<OpI32>(a, tu, s);
    case kInt64: return launch_fold_op<OpI64>(a, tu, s);
    default: return hipErrorInvalidValue;
  }
}

template <class Op>
static hipError_t launch_batched_op(const BatchEntry* tab, const uint32_t* tile_start,
                                    int nbuckets, uint32_t ntiles, const Tuning& tu,
                                    hipStream_t s) {
  const int grid = (int)(ntiles < (uint32_t)tu.max_grid ? ntiles : (uint32_t)tu.max_grid);
  if (tu.nt)
    hipLaunchKernelGGL((batched_kernel<Op, kBatchVPT, true>), dim3(grid), dim3(kBlock), 0, s,
                       tab, tile_start, nbuckets, ntiles);
  else
    hipLaunchKernelGGL((batched_kernel<Op, kBatchVPT, false>), dim3(grid), dim3(kBlock), 0, s,
                       tab, tile_start, nbuckets, ntiles);
  return hipGetLastError();
}

hipError_t launch_batched(const BatchEntry* tab, const uint32_t* tile_start, int nbuckets,
                          uint32_t ntiles, int dtype, int mode, const Tuning& tu,
                          hipStream_t s) {
  switch (dtype) {
    case kFloat32: return launch_batched_op<OpF32>(tab, tile_start, nbuckets, ntiles, tu, s);
    case kFloat64: return launch_batched_op<OpF64>(tab, tile_start, nbuckets, ntiles, tu, s);
    case kFloat16:
      return mode == kModeAccumF32
                 ? launch_batched_op<OpAcc16<false>>(tab, tile_start, nbuckets, ntiles, tu, s)
                 : launch_batched_op<OpF16>(tab, tile_start, nbuckets, ntiles, tu, s);
    case kBFloat16:
      return mode == kModeAccumF32
                 ? launch_batched_op<OpAcc16<true>>(tab, tile_start, nbuckets, ntiles, tu, s)
                 : launch_batched_op<OpBF16>(tab, tile_start, nbuckets, ntiles, tu, s);
    case kUInt8:
    case kInt8: return launch_batched_op<OpI8>(tab, tile_start, nbuckets, ntiles, tu, s);
    case kInt32: return launch_batched_op<OpI32>(tab, tile_start, nbuckets, ntiles, tu, s);
    case kInt64: return launch_batched_op<OpI64>(tab, tile_start, nbuckets, ntiles, tu, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_copy(void* dst, const void* src, size_t len, const Tuning& tu,
                       hipStream_t s) {
  const uintptr_t d = (uintptr_t)dst, q = (uintptr_t)src;
  uint64_t head = 0, nvec = 0;
  if (((d ^ q) & 15u) == 0) {  // co-aligned: vectors between head and tail
    head = (16u - (d & 15u)) & 15u;
    if (head > len) head = len;
    nvec = (len - head) / 16;
  } else {
    head = len;  // byte path only
  }
  uint64_t work = nvec + 64;
  uint64_t blocks = (work + kBlock - 1) / kBlock;
  if (blocks > (uint64_t)tu.max_grid) blocks = tu.max_grid;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(copy_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s,
                     (unsigned char*)dst, (const unsigned char*)src, head, nvec, (uint64_t)len);
  return hipGetLastError();
}

}  // namespace bpsr
