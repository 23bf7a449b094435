// CpuReducer::copy (cpu_reducer.cc:209-220) on the device, and the dtype/mode
// dispatch of the fold and batched launchers.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bpsr_internal.h"
#include "bpsr_ops.h"

namespace bpsr {

// 16-B vectors between an unaligned head and tail (operands co-aligned mod 16),
// bytes otherwise.  Same tiling as the fold kernel: a workgroup owns
// kBlock*kCopyVPT contiguous vectors.
constexpr int kCopyVPT = 8;

__global__ __launch_bounds__(kBlock) void copy_kernel(unsigned char* __restrict__ dst,
                                                      const unsigned char* __restrict__ src,
                                                      uint64_t head, uint64_t nvec,
                                                      uint64_t len) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const uint64_t tile_vecs = (uint64_t)kBlock * kCopyVPT;
  const uint64_t ntiles = (nvec + tile_vecs - 1) / tile_vecs;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t v0 = tile * tile_vecs + threadIdx.x;
    if ((tile + 1) * tile_vecs <= nvec) {
      u4 x[kCopyVPT];
#pragma unroll
      for (int j = 0; j < kCopyVPT; ++j)
        x[j] = __builtin_nontemporal_load(
            reinterpret_cast<const u4*>(src + head + (v0 + j * kBlock) * 16));
#pragma unroll
      for (int j = 0; j < kCopyVPT; ++j)
        __builtin_nontemporal_store(x[j], reinterpret_cast<u4*>(dst + head + (v0 + j * kBlock) * 16));
    } else {
      for (uint64_t v = v0; v < nvec; v += kBlock)
        *reinterpret_cast<u4*>(dst + head + v * 16) =
            *reinterpret_cast<const u4*>(src + head + v * 16);
    }
  }
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint64_t tail_begin = head + nvec * 16;
  const uint64_t nscalar = head + (len - tail_begin);
  for (uint64_t s = t; s < nscalar; s += stride) {
    const uint64_t b = s < head ? s : tail_begin + (s - head);
    dst[b] = src[b];
  }
}

hipError_t allow_full_lds(const void* kernel) {
  return hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)kLdsPerCU);
}

hipError_t launch_copy(void* dst, const void* src, size_t len, const Tuning& tu,
                       hipStream_t s) {
  const uintptr_t d = (uintptr_t)dst, q = (uintptr_t)src;
  uint64_t head = 0, nvec = 0;
  if (((d ^ q) & 15u) == 0) {
    head = (16u - (d & 15u)) & 15u;
    if (head > len) head = len;
    nvec = (len - head) / 16;
  } else {
    head = len;  // not co-aligned: byte path (rare; a shard view at an odd offset)
  }
  const uint64_t tile_vecs = (uint64_t)kBlock * kCopyVPT;
  uint64_t blocks = (nvec + tile_vecs - 1) / tile_vecs;
  const uint64_t nscalar = head + (len - head - nvec * 16);
  const uint64_t sblocks = (nscalar + kBlock - 1) / kBlock;
  if (sblocks > blocks) blocks = sblocks;
  if (blocks > (uint64_t)tu.max_grid) blocks = tu.max_grid;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(copy_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s,
                     (unsigned char*)dst, (const unsigned char*)src, head, nvec, (uint64_t)len);
  return hipGetLastError();
}

hipError_t launch_fold(const FoldArgs& a, int dtype, int mode, const Tuning& tu,
                       hipStream_t s) {
  const bool acc = mode == kModeAccumF32;
  switch (dtype) {
    case kFloat32: return launch_fold_f32(a, tu, s);
    case kFloat64: return launch_fold_f64(a, tu, s);
    case kFloat16: return acc ? launch_fold_f16acc(a, tu, s) : launch_fold_f16(a, tu, s);
    case kBFloat16: return acc ? launch_fold_bf16acc(a, tu, s) : launch_fold_bf16(a, tu, s);
    case kUInt8:
    case kInt8: return launch_fold_i8(a, tu, s);
    case kInt32: return launch_fold_i32(a, tu, s);
    case kInt64: return launch_fold_i64(a, tu, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_batched(const BatchLaunch& L, int vpt, int dtype, int mode, const Tuning& tu,
                          hipStream_t s) {
  const bool acc = mode == kModeAccumF32;
  switch (dtype) {
    case kFloat32: return launch_batched_f32(L, vpt, tu, s);
    case kFloat64: return launch_batched_f64(L, vpt, tu, s);
    case kFloat16:
      return acc ? launch_batched_f16acc(L, vpt, tu, s) : launch_batched_f16(L, vpt, tu, s);
    case kBFloat16:
      return acc ? launch_batched_bf16acc(L, vpt, tu, s) : launch_batched_bf16(L, vpt, tu, s);
    case kUInt8:
    case kInt8: return launch_batched_i8(L, vpt, tu, s);
    case kInt32: return launch_batched_i32(L, vpt, tu, s);
    case kInt64: return launch_batched_i64(L, vpt, tu, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace bpsr
