// The pull copy service's host side (kernel: bpsr_k_service.hip).
//
// A blocking pull into device memory used to ride a lane launch: the pull
// thread handed its copy to the lane issuer, the issuer launched it, the
// lane's completer saw the launch finish and woke the thread — two thread
// hand-offs and a HIP launch per pull, about 50 us per pull at best, which a
// worker pulling 160 keys one after another pays 160 times.
// Here the pull thread writes one tagged 32-B job into a pinned ring and
// spins on the job's done word: the persistent service kernel
// picks the job up within a few microseconds, copies it, makes the bytes
// visible device-wide and stores the done word.  No HIP call on that path.
//
// The kernel runs on a non-blocking high-priority stream: a hardware queue of
// its own (the runtime shares only normal-priority queues between streams), so
// it never holds back work queued on the process's shared queues, and no
// implicit synchronisation with the legacy NULL stream, so PyTorch's default
// stream does not wait for a running service (a CU-masked stream would have
// its own queue but is a blocking stream: DESIGN.md §9).  It exits by
// itself after kIdleUs without a job or kMaxUs of age (busy or not), storing
// its launch number to the pinned `exited` word, and a waiting or posting
// thread that sees the word relaunches it at once; a job stranded by an exit
// is served by the relaunch, which starts at the oldest job still pending and
// skips jobs already done.  The age limit bounds what a device-wide
// synchronisation elsewhere in the process (torch.cuda.synchronize,
// hipDeviceSynchronize, hipFree) waits for the service: the running launch's
// remaining age plus at most one relaunch's (include/bpsr/server.h).
// A relaunch happens only after the old launch has completed, so no job is
// copied by two launches at once (a late second copy could overwrite a buffer
// its caller already reuses).  For the same reason a give-up (a job not served
// in kTimeoutMs) raises `stop` and waits for the running launch to end before
// any caller learns that the service is off and copies the bytes another way:
// the fetcher checks `stop` on every pass and moves nothing after it.  That
// wait is bounded (kStopWaitMs): a launch that has not ended by then may be
// wedged and may still write a job's buffer, so the service is then marked
// wedged — every caller gets a hard error and none falls back to another copy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <cstdlib>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "bpsr_error.h"
#include "bpsr_internal.h"

namespace bpsr {

namespace {
constexpr uint32_t kSvcWgs = 65;             // workgroups per launch: the fetcher + 64 copiers
constexpr size_t kChunk = 64 << 10;          // one job's bytes at most (a large copy spreads)
// A launch's idle exit (short: a device-wide synchronisation waits for a
// running service; a pull burst keeps it alive) and its age limit (a
// relaunch costs ~20 us of posting latency, so 1 ms keeps that near 2 %).
#ifndef BPSR_SVC_MAX_US  // (probe builds only: tools/dbg/copysvc_probe.cpp)
#define BPSR_SVC_MAX_US 1000
#endif
constexpr int kIdleUs = 500, kMaxUs = BPSR_SVC_MAX_US;
constexpr int kCheckUs = 200;                // a waiter's liveness check period
constexpr int64_t kExitPollNs = 2000;        // ... while the launch is exiting
constexpr int kTimeoutMs = 10000;            // a job's give-up (reported, not retried)
constexpr int kStopWaitMs = 1000;            // a give-up's wait for the launch to end
}  // namespace

struct CopyService {
  int device = -1;
  hipStream_t stream = nullptr;
  hipEvent_t ev = nullptr;       // the current launch's completion
  SvcJob* ring = nullptr;        // pinned host
  uint64_t* done = nullptr;      // pinned host, one 64-B line per slot (kDoneStride words)
  uint32_t* stop = nullptr;      // pinned host: [0] stop, [16] exited (its own 64-B line)
  uint32_t* exited = nullptr;
  SvcJob* ring_d = nullptr;      // their device views
  uint64_t* done_d = nullptr;
  uint32_t* stop_d = nullptr;
  uint64_t* dev = nullptr;       // device words of the kernel
  SvcJob* dring = nullptr;       // device ring
  uint64_t* trace = nullptr;     // probes only
  uint64_t idle_ticks = 0, max_ticks = 0, stall_ticks = 0;
  // Posting is lock-free (a job index from `posted`, then the slot's words);
  // `mu` serialises only launches and liveness checks.
  std::atomic<uint64_t> posted{0};      // job indices handed out
  std::atomic<int64_t> last_post_ns{0};
  std::atomic<bool> running{false};     // written under mu
  std::atomic<uint32_t> gen{0};         // the current launch's number (written under mu)
  std::atomic<bool> broken{false};      // a job timed out: the service is off for good
  std::atomic<bool> wedged{false};      // ... and its launch did not end: no fallback either
  std::mutex mu;
  uint64_t scan_from = 0;               // under mu: every job below is done
  std::atomic<uint64_t> launches{0};
  int timeout_ms = kTimeoutMs;
  int stop_wait_ms = kStopWaitMs;
};

namespace {

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Polls an event for at most `ms`: true once it has completed.
bool event_done_within(hipEvent_t ev, int ms) {
  const int64_t end = now_ns() + (int64_t)ms * 1000000;
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return e == hipSuccess;
    if (now_ns() > end) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// Live services.  A process that exits without destroying its server must not
// leave a service kernel polling pinned host memory the runtime is about to
// unmap: an exit handler, registered after the runtime's own state exists
// (so it runs before the runtime's teardown), stops every live service and
// waits for its kernel.
std::mutex g_live_mu;
std::set<CopyService*>* g_live = nullptr;

void stop_live_services() {
  std::lock_guard<std::mutex> g(g_live_mu);
  if (!g_live) return;
  for (CopyService* c : *g_live) {
    if (c->stop) __atomic_store_n(c->stop, 1u, __ATOMIC_RELEASE);
    if (c->running.load() && !c->wedged.load()) (void)event_done_within(c->ev, c->stop_wait_ms);
  }
}

void register_live(CopyService* c) {
  std::lock_guard<std::mutex> g(g_live_mu);
  if (!g_live) {
    g_live = new std::set<CopyService*>();
    std::atexit(stop_live_services);
  }
  g_live->insert(c);
}

void unregister_live(CopyService* c) {
  std::lock_guard<std::mutex> g(g_live_mu);
  if (g_live) g_live->erase(c);
}

// A slot's done word only grows (its next job is posted after this one is
// done), so a later job's value also says this one is done.
bool job_done(const CopyService* c, uint64_t j) {
  return __atomic_load_n(&c->done[(j % kSvcRing) * kDoneStride], __ATOMIC_ACQUIRE) >= j + 1;
}

// The running launch has decided to exit (its fetcher stored its number):
// a thread with a pending job relaunches now rather than at its next check.
bool svc_exiting(const CopyService* c) {
  return c->running.load() && __atomic_load_n(c->exited, __ATOMIC_ACQUIRE) == c->gen.load();
}

// With mu held: a launch is running until its event says it is gone (one
// that decided to exit finishes the copies it started first; the caller then
// polls it rather than blocking on it with mu held, so a give-up can still
// fire meanwhile).
bool svc_alive(CopyService* c) {
  if (!c->running.load()) return false;
  if (hipEventQuery(c->ev) == hipSuccess) c->running.store(false);
  return c->running.load();
}

// With mu held: give up — raise `stop`, wait until the running launch has
// ended (it moves and starts no job after seeing `stop`; copies already under
// way finish first), and only then mark the service off, so that no caller
// copies a job's bytes another way while the kernel may still write them.
// The wait is bounded: a launch still running after stop_wait_ms is wedged —
// a hard error for this and every later caller, with no fallback copy.
int svc_give_up(CopyService* c, uint64_t j) {
  __atomic_store_n(c->stop, 1u, __ATOMIC_RELEASE);
  if (c->running.load()) {
    if (!event_done_within(c->ev, c->stop_wait_ms)) {
      c->wedged.store(true);
      return fail(BYTEPS_REDUCE_EHIP,
                  "copy service: job %llu not served in %d ms, and the launch did not stop "
                  "within %d ms (it may still write the job's buffer: no fallback copy)",
                  (unsigned long long)j, c->timeout_ms, c->stop_wait_ms);
    }
    c->running.store(false);
  }
  c->broken.store(true);
  return fail(BYTEPS_REDUCE_ETIMEOUT, "copy service: job %llu not served in %d ms",
              (unsigned long long)j, c->timeout_ms);
}

// With mu held: start a launch at the oldest job not done (jobs handed out
// but not yet written count as not done: the fetcher waits for them).
int svc_launch(CopyService* c) {
  if (c->running.load()) {  // let the old launch finish first (it is stopping)
    if (!event_done_within(c->ev, c->stop_wait_ms)) {
      c->wedged.store(true);
      return fail(BYTEPS_REDUCE_EHIP, "copy service: the exiting launch did not end within %d ms",
                  c->stop_wait_ms);
    }
    c->running.store(false);
  }
  const uint64_t posted = c->posted.load();
  uint64_t start = c->scan_from;
  while (start < posted && job_done(c, start)) ++start;
  c->scan_from = start;
  SvcArgs a{};
  a.ring = c->ring_d;
  a.done = c->done_d;
  a.stop = c->stop_d;
  a.exited = c->stop_d + 16;
  a.dev = c->dev;
  a.dring = c->dring;
  a.trace = c->trace;
  a.start = start;
  a.check_below = posted;
  a.idle_ticks = c->idle_ticks;
  a.max_ticks = c->max_ticks;
  a.stall_ticks = c->stall_ticks;
  a.wgs = kSvcWgs;
  a.gen = c->gen.load() + 1;
  hipError_t e = hipMemsetAsync(c->dev, 0, 4 * sizeof(uint64_t), c->stream);
  if (e == hipSuccess) e = launch_copy_service(a, c->stream);
  if (e == hipSuccess) e = hipEventRecord(c->ev, c->stream);
  if (e != hipSuccess) return hip_fail(e, "copy service launch");
  c->gen.store(a.gen);
  c->running.store(true);
  c->launches.fetch_add(1, std::memory_order_relaxed);
  return 0;
}

}  // namespace

int copysvc_create(int device, CopyService** out) {
  *out = nullptr;
  CopyService* c = new CopyService();
  c->device = device;
  int khz = 0;
  hipError_t e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
  if (e != hipSuccess || khz <= 0) {
    delete c;
    return e != hipSuccess ? hip_fail(e, "wall clock rate")
                           : fail(BYTEPS_REDUCE_EHIP, "copy service: no wall clock rate");
  }
  c->idle_ticks = (uint64_t)khz * kIdleUs / 1000;
  // tests of the give-up path: a short give-up time, and copiers that hold
  // every job three times that long before copying it (unless stopped)
  if (const char* v = getenv("BPSR_COPYSVC_TEST_STALL_MS")) {
    c->timeout_ms = std::max(1, atoi(v));
    c->stall_ticks = (uint64_t)khz * 3 * c->timeout_ms;
    c->stop_wait_ms = std::min(kStopWaitMs, 5 * c->timeout_ms);
  }
  c->max_ticks = (uint64_t)khz * kMaxUs / 1000;
  int prio_lo = 0, prio_hi = 0;
  e = hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (e == hipSuccess && prio_lo == prio_hi) {
    delete c;
    return fail(BYTEPS_REDUCE_EHIP, "copy service: no stream priorities (no queue of its own)");
  }
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_hi);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev, hipEventDisableTiming);
  const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
  if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&c->ring), sizeof(SvcJob) * kSvcRing, fl);
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void**>(&c->done), sizeof(uint64_t) * kSvcRing * kDoneStride, fl);
  if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&c->stop), 128, fl);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&c->dev), 256);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&c->dring), sizeof(SvcJob) * kSvcRing);
  // on the service's own (non-blocking) stream: a NULL-stream memset would
  // wait for every blocking stream, a running keyed consumer's included —
  // which can be waiting for this very thread's next push
  if (e == hipSuccess) e = hipMemsetAsync(c->dring, 0, sizeof(SvcJob) * kSvcRing, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) {
    std::memset(c->ring, 0, sizeof(SvcJob) * kSvcRing);
    std::memset(c->done, 0, sizeof(uint64_t) * kSvcRing * kDoneStride);
    std::memset(c->stop, 0, 128);
    c->exited = c->stop + 16;
    e = hipHostGetDevicePointer(reinterpret_cast<void**>(&c->ring_d), c->ring, 0);
  }
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&c->done_d), c->done, 0);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&c->stop_d), c->stop, 0);
  if (e != hipSuccess) {
    const int rc = hip_fail(e, "copy service setup");
    copysvc_destroy(c);
    return rc;
  }
  register_live(c);
  *out = c;
  return 0;
}

void copysvc_destroy(CopyService* c) {
  if (!c) return;
  unregister_live(c);
  if (c->stop) __atomic_store_n(c->stop, 1u, __ATOMIC_RELEASE);
  // exits within one poll; a wedged launch may still touch the ring and the
  // job buffers: leak what it can reach rather than free it under the kernel
  if (c->running.load() && (c->wedged.load() || !event_done_within(c->ev, c->stop_wait_ms))) return;
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->ev) (void)hipEventDestroy(c->ev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->ring) (void)hipHostFree(c->ring);
  if (c->done) (void)hipHostFree(c->done);
  if (c->stop) (void)hipHostFree(c->stop);
  if (c->dev) (void)hipFree(c->dev);
  if (c->dring) (void)hipFree(c->dring);
  delete c;
}

// With mu held, for a job j not done: keep a launch serving, or give up.
int svc_check(CopyService* c, uint64_t j, int64_t now, int64_t t0) {
  if (c->broken.load() || c->wedged.load())
    return fail(BYTEPS_REDUCE_EHIP, "copy service: off after a timeout");
  if (!svc_alive(c)) {
    const int rc = svc_launch(c);
    if (rc) {
      c->broken.store(true);
      return rc;
    }
  }
  if (now - t0 > c->timeout_ms * 1000000ll) return svc_give_up(c, j);
  return 0;
}

// Waits for job j's done word: spin, then yield; every kCheckUs without it,
// or as soon as the launch signals its exit, make sure a launch is serving.
// 0, or an error (the service then stays off).
int wait_job(CopyService* c, uint64_t j, int64_t t0) {
  int64_t t_check = now_ns();
  for (;;) {
    if (job_done(c, j)) return 0;
    for (int k = 0; k < 32; ++k) __builtin_ia32_pause();
    const int64_t now = now_ns();
    if (now - t0 > 50'000) std::this_thread::yield();
    const int64_t since = now - t_check;
    if (since > kCheckUs * 1000ll || (since > kExitPollNs && svc_exiting(c))) {
      t_check = now;
      std::lock_guard<std::mutex> g(c->mu);
      if (job_done(c, j)) return 0;
      if (const int rc = svc_check(c, j, now, t0)) return rc;
    }
  }
}

int copysvc_post(CopyService* c, void* dst, const void* src, size_t len, uint64_t* first_out,
                 uint64_t* n_out) {
  *first_out = 0;
  *n_out = 0;
  if (len == 0) return 0;
  if (((reinterpret_cast<uint64_t>(dst) + len) | (reinterpret_cast<uint64_t>(src) + len)) > kSvcMask)
    return fail(BYTEPS_REDUCE_EARGS, "copy service: address beyond 48 bits");
  if (c->broken.load() || c->wedged.load())
    return fail(BYTEPS_REDUCE_EHIP, "copy service: off after a timeout");
  const uint64_t n = (len + kChunk - 1) / kChunk;
  const uint64_t first = c->posted.fetch_add(n);
  const int64_t t0 = now_ns();
  int rc = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t j = first + i;
    // the slot's previous job first (a ring's worth of jobs behind)
    if (j >= kSvcRing && (rc = wait_job(c, j - kSvcRing, t0))) return rc;
    SvcJob& r = c->ring[j % kSvcRing];
    const size_t off = (size_t)i * kChunk;
    const uint64_t tag = svc_tag(j) << 48;
    __atomic_store_n(&r.w[0], (reinterpret_cast<uint64_t>(dst) + off) | tag, __ATOMIC_RELAXED);
    __atomic_store_n(&r.w[1], (reinterpret_cast<uint64_t>(src) + off) | tag, __ATOMIC_RELAXED);
    __atomic_store_n(&r.w[2], (uint64_t)std::min(kChunk, len - off) | tag, __ATOMIC_RELEASE);
  }
  // a launch idle for most of kIdleUs may be exiting: look after posting
  const int64_t prev = c->last_post_ns.exchange(t0);
  if (!c->running.load() || t0 - prev > kIdleUs * 500ll || svc_exiting(c)) {
    std::lock_guard<std::mutex> g(c->mu);
    if (c->broken.load() || c->wedged.load())
      return fail(BYTEPS_REDUCE_EHIP, "copy service: off after a timeout");
    if (!svc_alive(c) && (rc = svc_launch(c))) {
      c->broken.store(true);
      return rc;
    }
  }
  *first_out = first;
  *n_out = n;
  return 0;
}

int copysvc_test(CopyService* c, uint64_t first, uint64_t n, int64_t posted_ns, bool* done) {
  *done = false;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t j = first + i;
    if (job_done(c, j)) continue;
    // not yet: past kCheckUs since posting (or the launch is exiting), make
    // sure a launch is serving
    const int64_t now = now_ns();
    if (now - posted_ns > kCheckUs * 1000ll || svc_exiting(c)) {  // (the caller polls)
      std::lock_guard<std::mutex> g(c->mu);
      if (job_done(c, j)) continue;
      if (const int rc = svc_check(c, j, now, posted_ns)) return rc;
    }
    return 0;
  }
  *done = true;
  return 0;
}

int64_t copysvc_now_ns() { return now_ns(); }

int copysvc_copy(CopyService* c, void* dst, const void* src, size_t len) {
  uint64_t first = 0, n = 0;
  const int64_t t0 = now_ns();
  int rc = copysvc_post(c, dst, src, len, &first, &n);
  if (rc) return rc;
  for (uint64_t i = 0; i < n; ++i)
    if ((rc = wait_job(c, first + i, t0))) return rc;
  return 0;
}

uint64_t copysvc_launches(CopyService* c) { return c ? c->launches.load() : 0; }

uint64_t copysvc_posted(CopyService* c) { return c->posted.load(); }

bool copysvc_broken(const CopyService* c) { return c->broken.load(); }

bool copysvc_wedged(const CopyService* c) { return c->wedged.load(); }

void copysvc_set_trace(CopyService* c, uint64_t* dev_trace) {
  std::lock_guard<std::mutex> g(c->mu);
  c->trace = dev_trace;
}

}  // namespace bpsr
