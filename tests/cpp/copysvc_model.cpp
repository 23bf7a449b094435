// CPU test of the pull copy service's host side (prophet_amd/csrc/
// bpsr_copy_service.cpp, compiled unchanged with g++): the job ring, the
// launch / relaunch rules (idle exit, age exit, the `exited` word, a job
// stranded by an exit), and the give-up (stop, wait for the launch, then the
// caller falls back) — against a CPU model of the service kernel's protocol
// (bpsr_k_service.hip: fetcher claims, tagged device ring, copiers in job
// order, done words) behind a fake HIP runtime whose events track model
// launches.  Timing is randomised to shake out orderings.  Not a model of the
// GPU's memory system: the host logic is what is under test.
//   g++ -std=c++17 -O1 -pthread -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
//       -Iinclude -Iprophet_amd/csrc prophet_amd/csrc/bpsr_copy_service.cpp \
//       tests/cpp/copysvc_model.cpp -o copysvc_model
// Prints "fails=0" on success.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "bpsr_internal.h"

namespace bpsr {
int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  char buf[256];
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  (void)buf;
  return code;
}
int hip_fail(hipError_t e, const char*) { return e == hipSuccess ? 0 : BYTEPS_REDUCE_EHIP; }
}  // namespace bpsr

namespace {

std::atomic<int> g_fails{0};
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);           \
      g_fails.fetch_add(1);                                        \
    }                                                              \
  } while (0)

uint64_t now_ticks() {  // the model's wall clock: 100 MHz, as hipDeviceAttributeWallClockRate says
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count() / 10;
}

thread_local std::mt19937 t_rng{std::random_device{}()};
void jitter(int max_us) {
  if (max_us > 0 && t_rng() % 4 == 0)
    std::this_thread::sleep_for(std::chrono::microseconds(t_rng() % (max_us + 1)));
}

// ---------------------------------------------------------- model kernel --
struct Launch {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
};
std::atomic<int> g_live_launches{0}, g_max_live{0};
std::atomic<uint64_t> g_late_copies{0};  // copies the model made after a stop was seen
std::atomic<bool> g_wedge{false};        // copiers hang (a launch that does not end)
int g_jitter_us = 20;

uint64_t ld(const uint64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
void st(uint64_t* p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

void model_fetcher(bpsr::SvcArgs a) {
  uint64_t seen = a.start;
  const uint64_t t_begin = now_ticks();
  uint64_t t_idle = t_begin;
  for (;;) {
    jitter(g_jitter_us);
    const uint32_t sig = __atomic_load_n(a.stop, __ATOMIC_ACQUIRE);
    uint64_t run = 0;
    if (!sig) {
      for (; run < 64; ++run) {
        const uint64_t j = seen + run;
        const uint64_t* hw = reinterpret_cast<const uint64_t*>(a.ring + j % bpsr::kSvcRing);
        const uint64_t tag = bpsr::svc_tag(j);
        const uint64_t w0 = ld(hw), w1 = ld(hw + 1), w2 = ld(hw + 2);
        if ((w0 >> 48) != tag || (w1 >> 48) != tag || (w2 >> 48) != tag) break;
        uint64_t* dw = reinterpret_cast<uint64_t*>(a.dring + j % bpsr::kSvcRing);
        st(dw + 0, w0);
        st(dw + 1, w1);
        st(dw + 2, w2);
      }
      seen += run;
    }
    const uint64_t now = now_ticks();
    bool quit = sig || now - t_begin > a.max_ticks;
    if (run) t_idle = now;
    else if (!quit) quit = a.start + ld(a.dev + 1) >= seen && now - t_idle > a.idle_ticks;
    if (quit) {
      st(a.dev + 2, sig ? bpsr::kSvcExitStop : bpsr::kSvcExitDone);
      __atomic_store_n(a.exited, a.gen, __ATOMIC_RELEASE);
      return;
    }
    if (!run) std::this_thread::sleep_for(std::chrono::microseconds(1));
  }
}

// the 64 copiers, emulated round-robin by one thread: copier g serves jobs
// start + g - 1, + 64, ... in order, and leaves once its next job is not
// there and the exit word is up
void model_copiers(bpsr::SvcArgs a) {
  const uint32_t ncop = a.wgs - 1;
  std::vector<uint64_t> next(ncop);
  std::vector<char> gone(ncop, 0);
  for (uint32_t g = 0; g < ncop; ++g) next[g] = a.start + g;
  uint32_t left = ncop;
  while (left) {
    bool any = false;
    for (uint32_t g = 0; g < ncop; ++g) {
      if (gone[g]) continue;
      const uint64_t j = next[g];
      const uint64_t slot = j % bpsr::kSvcRing;
      const uint64_t* dw = reinterpret_cast<const uint64_t*>(a.dring + slot);
      const uint64_t tag = bpsr::svc_tag(j);
      const uint64_t w0 = ld(dw), w1 = ld(dw + 1), w2 = ld(dw + 2);
      if ((w0 >> 48) != tag || (w1 >> 48) != tag || (w2 >> 48) != tag) {
        if (ld(a.dev + 2)) {
          gone[g] = 1;
          --left;
        }
        continue;
      }
      any = true;
      while (g_wedge.load()) std::this_thread::sleep_for(std::chrono::microseconds(100));
      bool skip = j < a.check_below && ld(a.done + slot * bpsr::kDoneStride) >= j + 1;
      if (!skip && a.stall_ticks) {  // tests: hold the job, drop it on a stop
        const uint64_t t0 = now_ticks();
        while (now_ticks() - t0 < a.stall_ticks) {
          if (ld(a.dev + 2) == bpsr::kSvcExitStop || __atomic_load_n(a.stop, __ATOMIC_ACQUIRE)) {
            gone[g] = 1;
            --left;
            skip = true;
            break;
          }
          std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        if (gone[g]) continue;
      }
      if (!skip) {
        jitter(g_jitter_us);
        if (__atomic_load_n(a.stop, __ATOMIC_ACQUIRE)) g_late_copies.fetch_add(1);
        std::memcpy(reinterpret_cast<void*>(w0 & bpsr::kSvcMask),
                    reinterpret_cast<const void*>(w1 & bpsr::kSvcMask), w2 & bpsr::kSvcMask);
        st(a.done + slot * bpsr::kDoneStride, j + 1);
      }
      __atomic_fetch_add(a.dev + 1, (uint64_t)1, __ATOMIC_ACQ_REL);
      next[g] += ncop;
    }
    if (!any) std::this_thread::sleep_for(std::chrono::microseconds(2));
  }
}

struct FakeEvent {
  std::shared_ptr<Launch> launch;  // the model launch recorded into this event
};
std::mutex g_stream_mu;
std::shared_ptr<Launch> g_last_launch;  // the service stream's latest launch

}  // namespace

namespace bpsr {
hipError_t launch_copy_service(const SvcArgs& a, hipStream_t) {
  auto L = std::make_shared<Launch>();
  {
    std::lock_guard<std::mutex> g(g_stream_mu);
    // one stream: a launch starts after the previous one ended (in order)
    if (g_last_launch) {
      std::unique_lock<std::mutex> lk(g_last_launch->mu);
      if (!g_last_launch->done) {
        printf("FAIL a launch queued while the previous one still runs\n");
        g_fails.fetch_add(1);
      }
    }
    g_last_launch = L;
  }
  std::thread([a, L] {
    const int live = g_live_launches.fetch_add(1) + 1;
    int m = g_max_live.load();
    while (live > m && !g_max_live.compare_exchange_weak(m, live)) {
    }
    std::thread f(model_fetcher, a), c(model_copiers, a);
    f.join();
    c.join();
    g_live_launches.fetch_sub(1);
    std::lock_guard<std::mutex> g(L->mu);
    L->done = true;
    L->cv.notify_all();
  }).detach();
  return hipSuccess;
}
}  // namespace bpsr

// ------------------------------------------------------- fake HIP runtime --
extern "C" {
hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t, int) {
  *v = 100000;  // kHz: the model's 100 MHz clock
  return hipSuccess;
}
hipError_t hipDeviceGetStreamPriorityRange(int* lo, int* hi) {
  *lo = 0;
  *hi = -1;
  return hipSuccess;
}
hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned, int) {
  *s = reinterpret_cast<hipStream_t>(new int(1));
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
  delete reinterpret_cast<int*>(s);
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) {
  std::shared_ptr<Launch> L;
  {
    std::lock_guard<std::mutex> g(g_stream_mu);
    L = g_last_launch;
  }
  if (L) {
    std::unique_lock<std::mutex> lk(L->mu);
    L->cv.wait(lk, [&] { return L->done; });
  }
  return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  *e = reinterpret_cast<hipEvent_t>(new FakeEvent());
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) {
  delete reinterpret_cast<FakeEvent*>(e);
  return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t) {
  std::lock_guard<std::mutex> g(g_stream_mu);
  reinterpret_cast<FakeEvent*>(e)->launch = g_last_launch;
  return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t e) {
  auto L = reinterpret_cast<FakeEvent*>(e)->launch;
  if (!L) return hipSuccess;
  std::lock_guard<std::mutex> g(L->mu);
  return L->done ? hipSuccess : hipErrorNotReady;
}
hipError_t hipEventSynchronize(hipEvent_t e) {
  auto L = reinterpret_cast<FakeEvent*>(e)->launch;
  if (!L) return hipSuccess;
  std::unique_lock<std::mutex> lk(L->mu);
  L->cv.wait(lk, [&] { return L->done; });
  return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t n, unsigned) {
  *p = std::calloc(1, n);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipHostFree(void* p) {
  std::free(p);
  return hipSuccess;
}
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned) {
  *d = h;
  return hipSuccess;
}
hipError_t hipMalloc(void** p, size_t n) {
  *p = std::calloc(1, n);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) {
  std::free(p);
  return hipSuccess;
}
hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) {
  std::memset(p, v, n);  // the previous launch has ended (svc_launch waits first)
  return hipSuccess;
}
}  // extern "C"

// ------------------------------------------------------------------ tests --
namespace {

// Posters copying random sizes (1 B .. 3 chunks) between their own buffers,
// with pauses past the idle exit now and then; every byte checked.
void racing_posters(int threads, int copies, int pause_every) {
  bpsr::CopyService* svc = nullptr;
  CHECK(bpsr::copysvc_create(0, &svc) == 0);
  if (!svc) return;
  std::vector<std::thread> th;
  std::atomic<int> bad{0}, errs{0};
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      std::mt19937 rng(1000 + t);
      std::vector<unsigned char> src(200 << 10), dst(200 << 10);
      for (int i = 0; i < copies; ++i) {
        const size_t len = 1 + rng() % (rng() % 4 == 0 ? src.size() : 4096);
        for (size_t b = 0; b < len; b += 97) src[b] = (unsigned char)(rng() | 1);
        src[len - 1] = (unsigned char)(i | 1);
        std::memset(dst.data(), 0, len);
        if (bpsr::copysvc_copy(svc, dst.data(), src.data(), len)) {
          errs.fetch_add(1);
          continue;
        }
        if (std::memcmp(dst.data(), src.data(), len)) bad.fetch_add(1);
        if (pause_every && i % pause_every == pause_every - 1)
          std::this_thread::sleep_for(std::chrono::microseconds(600 + rng() % 400));
      }
    });
  for (auto& x : th) x.join();
  CHECK(bad.load() == 0);
  CHECK(errs.load() == 0);
  CHECK(!bpsr::copysvc_broken(svc));
  const uint64_t launches = bpsr::copysvc_launches(svc);
  printf("racing_posters threads=%d copies=%d launches=%llu\n", threads, copies,
         (unsigned long long)launches);
  CHECK(launches >= 2);  // the age / idle exits and their relaunches
  bpsr::copysvc_destroy(svc);
  CHECK(g_max_live.load() <= 1);  // never two launches at once
}

// The give-up: every job is held 3 x the give-up time; the first copy gives
// up (ETIMEOUT) only after the launch has ended, the held job is dropped (no
// copy after the stop), and later posts fail at once (the service is off).
void give_up() {
  setenv("BPSR_COPYSVC_TEST_STALL_MS", "40", 1);
  bpsr::CopyService* svc = nullptr;
  CHECK(bpsr::copysvc_create(0, &svc) == 0);
  unsetenv("BPSR_COPYSVC_TEST_STALL_MS");
  if (!svc) return;
  std::vector<unsigned char> src(5000, 7), dst(5000, 0);
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = bpsr::copysvc_copy(svc, dst.data(), src.data(), src.size());
  const double ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  CHECK(rc == BYTEPS_REDUCE_ETIMEOUT);
  CHECK(ms >= 40 && ms < 110);
  CHECK(bpsr::copysvc_broken(svc));
  CHECK(g_live_launches.load() == 0);  // the launch ended before the caller heard
  // the caller now copies another way and reuses its buffer: nothing late
  std::memset(dst.data(), 0x55, dst.size());
  std::this_thread::sleep_for(std::chrono::milliseconds(150));
  CHECK(dst[0] == 0x55 && dst[4999] == 0x55);
  CHECK(g_late_copies.load() == 0);
  CHECK(bpsr::copysvc_copy(svc, dst.data(), src.data(), 16) != 0);  // off for good
  printf("give_up ms=%.1f\n", ms);
  bpsr::copysvc_destroy(svc);
}

// The give-up when the launch does not end (a wedged kernel): the copy
// returns a hard error once the bounded wait for the launch has passed —
// not ETIMEOUT, and the service reports wedged rather than broken, so no
// caller copies the bytes another way while the kernel may still write them;
// later posts fail at once.  Then the launch is let go and ends.
void wedged_give_up() {
  setenv("BPSR_COPYSVC_TEST_STALL_MS", "40", 1);
  bpsr::CopyService* svc = nullptr;
  CHECK(bpsr::copysvc_create(0, &svc) == 0);
  unsetenv("BPSR_COPYSVC_TEST_STALL_MS");
  if (!svc) return;
  std::vector<unsigned char> src(5000, 7), dst(5000, 0);
  g_wedge.store(true);
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = bpsr::copysvc_copy(svc, dst.data(), src.data(), src.size());
  const double ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  CHECK(rc == BYTEPS_REDUCE_EHIP);
  CHECK(ms >= 40 + 200 && ms < 40 + 200 + 150);  // the give-up, then the bounded wait (5 x 40 ms)
  CHECK(bpsr::copysvc_wedged(svc));
  CHECK(!bpsr::copysvc_broken(svc));  // no fallback copy
  CHECK(g_live_launches.load() == 1);
  CHECK(bpsr::copysvc_copy(svc, dst.data(), src.data(), 16) == BYTEPS_REDUCE_EHIP);
  g_wedge.store(false);
  for (int i = 0; i < 200 && g_live_launches.load(); ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  CHECK(g_live_launches.load() == 0);
  CHECK(g_late_copies.load() == 0);
  printf("wedged_give_up ms=%.1f\n", ms);
  bpsr::copysvc_destroy(svc);  // leaks the wedged service's buffers by design
}

}  // namespace

int main() {
  racing_posters(1, 3000, 0);
  racing_posters(8, 600, 50);
  g_jitter_us = 200;  // slow "device": posts pile up, launches exit and relaunch busy
  racing_posters(4, 300, 0);
  g_jitter_us = 20;
  give_up();
  wedged_give_up();
  printf("fails=%d\n", g_fails.load());
  return g_fails.load() ? 1 : 0;
}
