// The pull copy service's kernel (bpsr_copy_service.cpp): persistent
// workgroups serving device-to-device copies that host threads post into a
// pinned job ring.
//   workgroup 0, the fetcher (one wave): polls the next slots of the host
//     ring; moves each newly posted job's tagged words into the same slot of
//     a device ring, so copiers never read over PCIe; decides when the
//     launch ends — after idle_ticks without a new job with every fetched job
//     completed, once max_ticks have passed, or when the host raises `stop` —
//     and raises the exit word (and the host's `exited` word).
//   workgroups 1..wgs-1, the copiers: copier g polls its next job's words in
//     the device ring until all three carry the job's tag, copies the job,
//     and stores the job's done word to the host.  16-B aligned jobs load with sc1 (L1 bypassed: no acquire
//     fence; the source was written back by its producing kernel's end) and
//     store with sc1 (write-through: no release fence); every storing wave
//     drains before the done word is stored.  Other jobs take an agent
//     acquire before and an agent release after plain copies.
// Every access to host memory and to the ring's words is a vector atomic.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bpsr_internal.h"

namespace bpsr {
namespace {

__device__ __forceinline__ uint64_t ld_host64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_dev64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_dev64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// A 16-B aligned job: sc1 loads and sc1 (write-through) stores, 8 in flight
// per lane (32 KiB per pass of the workgroup).  Buffer descriptors bound the job: lanes past its end load zeros
// and store nothing.
__device__ __forceinline__ void copy_sc1(unsigned char* dst, const unsigned char* src,
                                         uint32_t len) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  constexpr int kSc1 = 16;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(src), 0, len,
                                                    0x00020000);
  const auto rd = __builtin_amdgcn_make_buffer_rsrc(dst, 0, len, 0x00020000);
  constexpr uint32_t kStep = kBlock * 16;
  constexpr int kDepth = 8;
  for (uint32_t o = threadIdx.x * 16; o < len; o += kDepth * kStep) {
    u4 x[kDepth];
#pragma unroll
    for (int d = 0; d < kDepth; ++d)
      x[d] = __builtin_amdgcn_raw_buffer_load_b128(rs, o + d * kStep, 0, kSc1);
#pragma unroll
    for (int d = 0; d < kDepth; ++d)
      __builtin_amdgcn_raw_buffer_store_b128(x[d], rd, o + d * kStep, 0, kSc1);
  }
}

// Any other job: plain copies behind an agent acquire, words when aligned.
__device__ __forceinline__ void copy_plain(unsigned char* dst, const unsigned char* src,
                                           uint64_t len) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const uint64_t a = reinterpret_cast<uint64_t>(dst) | reinterpret_cast<uint64_t>(src);
  if (((a | len) & 3) == 0) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (uint64_t i = threadIdx.x; i < len / 4; i += kBlock) d[i] = s[i];
  } else {
    for (uint64_t i = threadIdx.x; i < len; i += kBlock) dst[i] = src[i];
  }
}

// One wave per poller: polls a window of the host ring's next slots each pass
// (one PCIe round trip; 8 slots, 64 while the last pass found a full window)
// and moves the consecutive run of posted jobs it finds into the device ring.
// kPollers waves poll the same ring half a round trip apart, so a posted job
// is seen sooner.  A wave moves only the jobs it claims by raising the shared
// `s_seen` past them, so each job's words are stored by ONE wave: a late store
// can never put job j's words back over job j + kSvcRing's (j + kSvcRing is
// posted only once j is done, i.e. once a copier read the claimed store).
// Wave 0 decides the exit — on the host's stop word (checked every pass, in
// the same round trip as the ring), at max_ticks of age even while busy, or
// after idle_ticks without a new job with every fetched job completed — and
// stores the launch's number to the host's `exited` word, so a waiting host
// thread relaunches at once; wave 1 follows the exit word.
__device__ void fetcher(const SvcArgs& a) {
  constexpr uint32_t kPollers = 2;
  __shared__ uint64_t s_seen;  // jobs below are claimed (in the device ring, or not this launch's)
  if (threadIdx.x == 0) s_seen = a.start;
  __syncthreads();
  if (threadIdx.x >= 64 * kPollers) return;
  const uint32_t wave = threadIdx.x / 64;
  const uint32_t l = threadIdx.x % 64;
  if (wave) __builtin_amdgcn_s_sleep(12);
  uint32_t kWin = 8;
  const uint64_t t_begin = wall_clock64();
  uint64_t t_idle = t_begin;
  for (;;) {
    const uint64_t base = __hip_atomic_load(&s_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint64_t j = base + l;
    const uint64_t slot = j % kSvcRing;
    const uint64_t tag = svc_tag(j);
    uint64_t w0 = 0, w1 = 0, w2 = 0, sig = 0;
    if (l < kWin) {
      const uint64_t* hw = reinterpret_cast<const uint64_t*>(a.ring + slot);
      w0 = ld_host64(hw + 0);
      w1 = ld_host64(hw + 1);
      w2 = ld_host64(hw + 2);
    }
    if (l == 0)  // the exit signal, in the same round trip
      sig = wave ? ld_dev64(a.dev + 2)
                 : __hip_atomic_load(a.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    sig = __builtin_amdgcn_readfirstlane((uint32_t)sig);
    const bool valid = l < kWin && (w0 >> 48) == tag && (w1 >> 48) == tag && (w2 >> 48) == tag;
    const uint64_t vmask = __ballot(valid);
    const uint64_t run = ~vmask ? __builtin_ctzll(~vmask) : 64;  // consecutive posted jobs
    if (run && !sig) {  // nothing more is moved once the exit is signalled
      uint64_t old = 0;
      if (l == 0)
        old = __hip_atomic_fetch_max(&s_seen, base + run, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
      old = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(old >> 32)) << 32) |
            __builtin_amdgcn_readfirstlane((uint32_t)old);
      if (valid && l < run && j >= old) {  // claimed by this wave
        uint64_t* dw = reinterpret_cast<uint64_t*>(a.dring + slot);
        st_dev64(dw + 0, w0);
        st_dev64(dw + 1, w1);
        st_dev64(dw + 2, w2);
        if (a.trace) st_dev64(a.trace + slot * 4 + 0, wall_clock64());
      }
    }
    const uint64_t now = wall_clock64();
    if (wave) {
      if (sig) return;
      if (!run) __builtin_amdgcn_s_sleep(1);
      kWin = run == kWin ? 64 : 8;
      continue;
    }
    bool quit = sig || now - t_begin > a.max_ticks;
    if (run) {
      t_idle = now;
    } else if (!quit) {
      const uint64_t seen = __hip_atomic_load(&s_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      quit = a.start + ld_dev64(a.dev + 1) >= seen && now - t_idle > a.idle_ticks;
    }
    if (quit) {
      if (l == 0) {
        st_dev64(a.dev + 2, sig ? kSvcExitStop : kSvcExitDone);
        __hip_atomic_store(a.exited, a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return;
    }
    if (!run) __builtin_amdgcn_s_sleep(1);
    kWin = run == kWin ? 64 : 8;
  }
}

__device__ void copier(const SvcArgs& a) {
  __shared__ uint64_t s_job[3];
  __shared__ uint32_t s_state;  // 1 job, 2 exit, 3 done by an earlier launch
  const uint32_t ncop = a.wgs - 1;
  uint64_t next = a.start + (blockIdx.x - 1);
  for (;;) {
    const uint64_t slot = next % kSvcRing;
    if (threadIdx.x == 0) {
      const uint64_t* dw = reinterpret_cast<const uint64_t*>(a.dring + slot);
      const uint64_t tag = svc_tag(next);
      uint32_t st = 0;
      for (;;) {
        const uint64_t w0 = ld_dev64(dw + 0), w1 = ld_dev64(dw + 1), w2 = ld_dev64(dw + 2);
        if ((w0 >> 48) == tag && (w1 >> 48) == tag && (w2 >> 48) == tag) {
          s_job[0] = w0 & kSvcMask;
          s_job[1] = w1 & kSvcMask;
          s_job[2] = w2 & kSvcMask;
          st = 1;
          // a relaunch may meet jobs an earlier launch finished
          if (next < a.check_below && ld_host64(a.done + slot * kDoneStride) >= next + 1) st = 3;
          if (a.trace) st_dev64(a.trace + slot * 4 + 1, wall_clock64());
          break;
        }
        if (ld_dev64(a.dev + 2)) {
          st = 2;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      // tests only: hold the job; a stop meanwhile drops it uncopied (the
      // host word itself: the fetcher may have left at its age limit)
      if (st == 1 && a.stall_ticks) {
        const uint64_t t0 = wall_clock64();
        while (wall_clock64() - t0 < a.stall_ticks) {
          if (ld_dev64(a.dev + 2) == kSvcExitStop ||
              __hip_atomic_load(a.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
            st = 2;
            break;
          }
          __builtin_amdgcn_s_sleep(8);
        }
      }
      s_state = st;
    }
    __syncthreads();
    const uint32_t st = s_state;
    if (st == 2) return;
    if (st == 1) {
      unsigned char* dst = reinterpret_cast<unsigned char*>(s_job[0]);
      const unsigned char* src = reinterpret_cast<const unsigned char*>(s_job[1]);
      const uint64_t len = s_job[2];
      const bool vec = ((reinterpret_cast<uint64_t>(dst) | reinterpret_cast<uint64_t>(src) |
                         len) & 15) == 0;
      if (vec) copy_sc1(dst, src, (uint32_t)len);
      else copy_plain(dst, src, len);
      drain();  // every storing wave
      __syncthreads();
      if (threadIdx.x == 0) {
        if (!vec) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          drain();
        }
        if (a.trace) st_dev64(a.trace + slot * 4 + 2, wall_clock64());
        __hip_atomic_store(a.done + slot * kDoneStride, next + 1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(a.dev + 1, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();  // s_job / s_state are rewritten next
    next += ncop;
  }
}

}  // namespace

__global__ __launch_bounds__(kBlock) void copy_service_kernel(SvcArgs a) {
  if (blockIdx.x == 0) fetcher(a);
  else copier(a);
}

hipError_t launch_copy_service(const SvcArgs& a, hipStream_t s) {
  if (a.wgs < 2) return hipErrorInvalidValue;
  hipLaunchKernelGGL(copy_service_kernel, dim3(a.wgs), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace bpsr
