// CpuReducer::copy (cpu_reducer.cc:209-220) on the device, and the dtype/mode
// dispatch of the fold and batched launchers.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>

#include "bpsr_kernels_impl.h"

namespace bpsr {

// The copy is the fold kernel with one byte-typed source: same tiles, buffer
// loads, nt policy and element path (unaligned head/tail bytes; operands not
// co-aligned mod 16 go through the element path entirely).  Its residency is
// its own: two streams need more workgroups per CU than the 9-stream fold to
// keep the HBM queues full: 4 per CU with 8 KiB tiles measured 0.80 of the
// roofline at 256 MiB vs 0.75 for the old grid-stride copy and 0.67 for
// torch's (profiles/r01_copy_sweep.jsonl; Tuning::copy_occ / copy_vpt).
// Cache policy as for the folds (cache_pol): write-through stores below
// Tuning::wt_max_bytes, nt above (the copy always reads nt).
template <int VPT, int NT>
static hipError_t launch_copy_vpt(const FoldArgs& a0, const Tuning& tu, hipStream_t s) {
  static KernelAttr attr;
  const hipError_t lds_ok =
      allow_lds(attr, reinterpret_cast<const void*>(&fold_kernel<OpI8, VPT, NT, 1>));
  if (lds_ok != hipSuccess) return lds_ok;
  FoldArgs a = a0;
  a.grid = (uint32_t)fold_grid(a.g, tu, VPT);
  const int occ = a.grid >= tu.occ_min_tiles ? tu.copy_occ : 0;
  hipLaunchKernelGGL((fold_kernel<OpI8, VPT, NT, 1>), dim3(a.grid), dim3(kBlock),
                     occ_lds_bytes(occ), s, a);
  return hipGetLastError();
}

template <int NT>
static hipError_t launch_copy_pol(const FoldArgs& a, int vpt, const Tuning& tu, hipStream_t s) {
  switch (vpt) {
    case 1: return launch_copy_vpt<1, NT>(a, tu, s);
    case 2: return launch_copy_vpt<2, NT>(a, tu, s);
    default: return launch_copy_vpt<4, NT>(a, tu, s);
  }
}

hipError_t allow_lds(KernelAttr& once, const void* kernel, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const uint64_t bit = dev < 64 ? (uint64_t{1} << dev) : 0;
  if (bit && (once.done.load(std::memory_order_acquire) & bit)) return hipSuccess;
  e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess && bit) once.done.fetch_or(bit, std::memory_order_release);
  return e;
}

hipError_t launch_copy(void* dst, const void* src, size_t len, const Tuning& tu,
                       hipStream_t s) {
  FoldArgs a;
  std::memset(&a, 0, sizeof(a));
  a.srcs[0] = static_cast<const unsigned char*>(src);
  a.dst = static_cast<unsigned char*>(dst);
  a.n = 1;
  make_geom(kUInt8, len, dst, &src, 1, false, &a.g, &a.aligned);
  int vpt = tu.copy_vpt;
  while (vpt > 1 && (a.g.nvec + (uint64_t)kBlock * vpt - 1) / ((uint64_t)kBlock * vpt) < kMinTiles)
    vpt >>= 1;
  Tuning tn = tu;
  tn.nt = 1;  // the copy reads non-temporal whatever the fold tuning says
  if (cache_pol(tn, a.g.nvec * 16) == kPolWt) return launch_copy_pol<kPolWt>(a, vpt, tu, s);
  return launch_copy_pol<kPolNt>(a, vpt, tu, s);
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

// Block-queue release (one wave) of blocks [first, first + count) for
// `epoch`: each block's word is raised to the epoch by a system-scope atomic
// max — the consumers poll at system scope whatever cache the writer ran
// behind (a hipMemset node inside a replayed hipGraph was not seen), and max,
// not store, because releases of consecutive epochs may run on different
// streams out of order.  Nothing is cleared between iterations: launch k
// waits for words >= k.
__global__ void blockq_release_kernel(uint32_t* flags, uint32_t first, uint32_t count,
                                      uint32_t epoch) {
  for (uint32_t i = threadIdx.x; i < count; i += 64)
    __hip_atomic_fetch_max(flags + first + i, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_blockq_release(uint32_t* flags, uint32_t first, uint32_t count, uint32_t epoch,
                                 hipStream_t s) {
  hipLaunchKernelGGL(blockq_release_kernel, dim3(1), dim3(64), 0, s, flags, first, count, epoch);
  return hipGetLastError();
}

// Keyed release behind the stream's earlier work (a round whose pushes were
// copied into their slots on that stream): one lane stores the block's word.
__global__ void key_release_kernel(uint64_t* kwords, uint32_t block, uint64_t word,
                                   uint64_t* word2_at, uint64_t word2) {
  if (threadIdx.x == 0) {
    if (word2_at) __hip_atomic_store(word2_at, word2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(kwords + block, word, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

hipError_t launch_key_release(uint64_t* kwords, uint32_t block, uint64_t word,
                              uint64_t* word2_at, uint64_t word2, hipStream_t s) {
  hipLaunchKernelGGL(key_release_kernel, dim3(1), dim3(64), 0, s, kwords, block, word, word2_at,
                     word2);
  return hipGetLastError();
}

// The HSA id of the queue this dispatch came from: hsa_queue_t::id, at byte 32
// of the queue (type, features, base_address, doorbell_signal, size,
// reserved1, id — hsa.h), which the dispatch's queue pointer addresses.
__global__ void queue_id_kernel(uint64_t* out) {
  if (threadIdx.x == 0) {
    const uint64_t* q = reinterpret_cast<const uint64_t*>((size_t)__builtin_amdgcn_queue_ptr());
    __hip_atomic_store(out, q[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

hipError_t read_queue_id(hipStream_t s, uint64_t* out) {
  hipLaunchKernelGGL(queue_id_kernel, dim3(1), dim3(64), 0, s, out);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return e;
}

// Dispatch-sequence gate: one wave, enqueued on a
// consumer launch's stream ahead of its kernel, returns once the last
// workgroups of the device's earlier launches have all started (the counter
// reaches the target; system-scope polls, the adds are system-scope
// atomics).  Bounded: past the timeout it returns anyway (the count is exact
// by construction; this only keeps a mistake from hanging the stream).
__global__ void seq_gate_kernel(const unsigned long long* started, unsigned long long target,
                                uint64_t timeout_ticks) {
  const uint64_t t0 = wall_clock64();
  for (;;) {
    const unsigned long long v =
        __hip_atomic_load(started, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v >= target || wall_clock64() - t0 > timeout_ticks) return;
    __builtin_amdgcn_s_sleep(2);
  }
}

hipError_t launch_seq_gate(const unsigned long long* started, unsigned long long target,
                           uint64_t timeout_ticks, hipStream_t s) {
  hipLaunchKernelGGL(seq_gate_kernel, dim3(1), dim3(64), 0, s, started, target, timeout_ticks);
  return hipGetLastError();
}

hipError_t launch_blockq(const BlockqLaunch& Q, int vpt, int pol, size_t lds, bool g, int dtype,
                         int mode, hipStream_t s) {
  const bool acc = mode == kModeAccumF32;
  switch (dtype) {
    case kFloat32: return launch_blockq_f32(Q, vpt, pol, lds, g, s);
    case kFloat64: return launch_blockq_f64(Q, vpt, pol, lds, g, s);
    case kFloat16:
      return acc ? launch_blockq_f16acc(Q, vpt, pol, lds, g, s)
                 : launch_blockq_f16(Q, vpt, pol, lds, g, s);
    case kBFloat16:
      return acc ? launch_blockq_bf16acc(Q, vpt, pol, lds, g, s)
                 : launch_blockq_bf16(Q, vpt, pol, lds, g, s);
    case kUInt8:
    case kInt8: return launch_blockq_i8(Q, vpt, pol, lds, g, s);
    case kInt32: return launch_blockq_i32(Q, vpt, pol, lds, g, s);
    case kInt64: return launch_blockq_i64(Q, vpt, pol, lds, g, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace bpsr
