// The PUSH loop: Prophet's scheduler feeding the block queue from a native
// thread (include/bpsr/prophet.h, byteps_prophet_loop_*).
//
// The reference runs its PUSH stage as a background loop (core_loops.cc
// RunPushLoopOnce: getTask, send, FinishOrProceed -> reportFinish) over the
// scheduled queue.  Here the "send" of a released partition is the device
// fold of its block: the loop thread polls the scheduler whenever partitions
// arrive, counts released partitions per block, reports each release group's
// partitions finished at the group's end (credit back to the scheduler) and,
// once a poll makes no progress, releases every block that became complete —
// one byteps_reduce_blockq_release_range per run of consecutive blocks, on the
// release stream, behind the copies that landed the pushes, or from the host
// with BYTEPS_PROPHET_LOOP_HOST_RELEASE when the pushes are already in HBM.
// Groups that are ready together thus share one release kernel: every release
// kernel that runs beside the consumer costs it ~0.4-0.6 us,
// and a block waits at most for the host work of draining its companions.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "bpsr/prophet.h"
#include "bpsr_error.h"
#include "bpsr_internal.h"
#include "bpsr_prophet_internal.h"

struct byteps_prophet_loop {
  byteps_prophet_queue* pq = nullptr;
  byteps_reduce_blockq* bq = nullptr;
  void* rel_stream = nullptr;
  int device = 0;
  std::vector<int32_t> block_of;    // per task handle
  std::vector<int32_t> block_size;  // partitions per block
  // iteration state, guarded by mu
  std::mutex mu;
  std::condition_variable cv;       // pushes -> thread
  std::condition_variable done_cv;  // thread -> end()
  bool active = false;
  bool stop = false;
  std::atomic<uint64_t> pushes{0};
  uint64_t seen = 0;
  std::vector<int32_t> left;        // partitions not yet released, per block
  std::vector<char> released;       // block released this iteration
  int32_t blocks_released = 0;
  uint64_t release_calls = 0;       // release kernels / host releases issued, ever
  std::vector<char> got;            // task handle pushed this iteration
  int err = 0;
  bool inline_drain = false;   // BYTEPS_PROPHET_LOOP_INLINE: pushers drain
  bool host_release = false;   // BYTEPS_PROPHET_LOOP_HOST_RELEASE: release_host, no stream
  std::atomic<bool> waiting{false};  // the loop thread sleeps on cv
  std::mutex drain_mu;
  std::vector<byteps_prophet_task> drained;  // one drain's releases (under drain_mu)
  // thread mode: pushes land in an inbox the loop thread empties into the
  // scheduler itself, so pushers and the drain never contend on its lock
  std::mutex inbox_mu;
  std::vector<byteps_prophet_task> inbox, taken;
  std::thread th;

  int nblocks() const { return (int)block_size.size(); }

  // Release every complete, unreleased block, one range per run (under mu).
  int release_complete() {
    const int nb = nblocks();
    for (int b = 0; b < nb;) {
      if (released[b] || left[b] != 0) {
        ++b;
        continue;
      }
      int e = b;
      while (e < nb && !released[e] && left[e] == 0) released[e++] = 1;
      const int rc = host_release ? byteps_reduce_blockq_release_host(bq, b, e - b)
                                  : byteps_reduce_blockq_release_range(bq, b, e - b, rel_stream);
      if (rc) return rc;
      ++release_calls;
      blocks_released += e - b;
      b = e;
    }
    return 0;
  }

  // Drain the scheduler: poll until a zero poll made no progress (a zero poll
  // may still advance collection or end a block, and the next may release);
  // at each release group's end report the group's partitions finished
  // (credit back: the next poll may release more); when the scheduler can go
  // no further, release the complete blocks — the groups drained together in
  // one kernel per run of blocks.  One drainer at a time (drain_mu).
  int drain() {
    std::lock_guard<std::mutex> dg(drain_mu);
    drained.clear();
    bpsr::prophet_drain(pq, &drained);  // credit returned per group inside
    std::lock_guard<std::mutex> g(mu);
    for (const auto& t : drained)
      if (t.handle < block_of.size()) --left[block_of[t.handle]];
    const int rc = release_complete();
    if (rc && !err) err = rc;
    if (err || blocks_released == nblocks()) done_cv.notify_all();
    return rc;
  }

  void run() {
    (void)hipSetDevice(device);
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      waiting.store(true);
      cv.wait(lk, [&] { return stop || (active && pushes.load() != seen); });
      waiting.store(false);
      if (stop) return;
      seen = pushes.load();
      lk.unlock();
      {
        std::lock_guard<std::mutex> g(inbox_mu);
        taken.swap(inbox);
      }
      const int rc = bpsr::prophet_add_many(pq, taken.data(), taken.size());
      taken.clear();
      if (rc) {
        std::lock_guard<std::mutex> g(mu);
        if (!err) err = rc;
        done_cv.notify_all();
      } else {
        drain();
      }
      lk.lock();
    }
  }
};

extern "C" {

int byteps_prophet_loop_create(byteps_prophet_queue* pq, byteps_reduce_blockq* bq,
                               const int32_t* block_of, int32_t nhandles, int32_t nblocks,
                               void* release_stream, int flags, byteps_prophet_loop** out) {
  if (!pq || !bq || !block_of || !out || nhandles < 0 || nblocks < 1)
    return bpsr::fail(BYTEPS_REDUCE_EARGS, "null argument, nhandles < 0 or nblocks < 1");
  *out = nullptr;
  if (!release_stream && !(flags & BYTEPS_PROPHET_LOOP_INLINE) &&
      !(flags & BYTEPS_PROPHET_LOOP_HOST_RELEASE))
    return bpsr::fail(BYTEPS_REDUCE_EARGS,
                      "loop thread with stream releases needs a release_stream (NULL would be "
                      "the loop thread's own per-thread stream, unordered with the pushes' copies)");
  auto* l = new (std::nothrow) byteps_prophet_loop;
  if (!l) return bpsr::fail(BYTEPS_REDUCE_EARGS, "out of memory");
  l->pq = pq;
  l->bq = bq;
  l->rel_stream = release_stream;
  l->block_size.assign(nblocks, 0);
  l->block_of.assign(block_of, block_of + nhandles);
  for (int32_t h = 0; h < nhandles; ++h) {
    if (block_of[h] < 0 || block_of[h] >= nblocks) {
      delete l;
      return bpsr::fail(BYTEPS_REDUCE_EARGS, "block_of[%d] = %d outside [0, %d)", h, block_of[h],
                        nblocks);
    }
    ++l->block_size[block_of[h]];
  }
  hipError_t e = hipGetDevice(&l->device);
  if (e != hipSuccess) {
    delete l;
    return bpsr::hip_fail(e, "hipGetDevice");
  }
  l->inline_drain = (flags & BYTEPS_PROPHET_LOOP_INLINE) != 0;
  l->host_release = (flags & BYTEPS_PROPHET_LOOP_HOST_RELEASE) != 0;
  if (l->host_release) {
    const int rc = byteps_reduce_blockq_host_releases(bq, 1);
    if (rc) {
      delete l;
      return rc;
    }
  }
  if (!l->inline_drain) l->th = std::thread([l] { l->run(); });
  *out = l;
  return 0;
}

int byteps_prophet_loop_begin(byteps_prophet_loop* l, void* consumer_stream) {
  if (!l) return bpsr::fail(BYTEPS_REDUCE_EARGS, "null loop");
  std::lock_guard<std::mutex> g(l->mu);
  if (l->active) return bpsr::fail(BYTEPS_REDUCE_EARGS, "iteration already begun (end it first)");
  uint64_t pend = 0;
  byteps_prophet_pending(l->pq, &pend);
  {
    std::lock_guard<std::mutex> ig(l->inbox_mu);
    pend += l->inbox.size();
  }
  if (pend) return bpsr::fail(BYTEPS_REDUCE_EARGS, "scheduler holds %llu tasks", (unsigned long long)pend);
  int rc = byteps_prophet_reset(l->pq);
  if (rc) return rc;
  if (!consumer_stream && (rc = byteps_reduce_blockq_stream(l->bq, &consumer_stream))) return rc;
  if ((rc = byteps_reduce_blockq_launch(l->bq, consumer_stream))) return rc;
  l->left = l->block_size;
  l->released.assign(l->block_size.size(), 0);
  l->blocks_released = 0;
  l->got.assign(l->block_of.size(), 0);
  l->err = 0;
  l->active = true;
  return l->release_complete();  // blocks without partitions
}

int byteps_prophet_loop_push(byteps_prophet_loop* l, const byteps_prophet_task* t) {
  if (!l || !t) return bpsr::fail(BYTEPS_REDUCE_EARGS, "null loop or task");
  {
    std::lock_guard<std::mutex> g(l->mu);
    if (!l->active) return bpsr::fail(BYTEPS_REDUCE_EARGS, "no iteration begun");
    if (t->handle >= l->block_of.size())
      return bpsr::fail(BYTEPS_REDUCE_EARGS, "handle %llu outside the table (%zu partitions)",
                        (unsigned long long)t->handle, l->block_of.size());
    if (l->got[t->handle])
      return bpsr::fail(BYTEPS_REDUCE_EARGS, "partition %llu pushed twice in one iteration",
                        (unsigned long long)t->handle);
    l->got[t->handle] = 1;
  }
  if (l->inline_drain) {
    const int rc = byteps_prophet_add_task(l->pq, t);
    if (rc) return rc;
    return l->drain();
  }
  {
    std::lock_guard<std::mutex> g(l->inbox_mu);
    l->inbox.push_back(*t);
  }
  l->pushes.fetch_add(1);
  if (l->waiting.load()) {  // the thread sleeps: wake it (else it is polling)
    std::lock_guard<std::mutex> g(l->mu);
    l->cv.notify_one();
  }
  return 0;
}

int byteps_prophet_loop_push_many(byteps_prophet_loop* l, const byteps_prophet_task* tasks,
                                  int32_t n) {
  if (!l || (!tasks && n > 0) || n < 0)
    return bpsr::fail(BYTEPS_REDUCE_EARGS, "null loop or tasks, or n < 0");
  {
    std::lock_guard<std::mutex> g(l->mu);
    if (!l->active) return bpsr::fail(BYTEPS_REDUCE_EARGS, "no iteration begun");
    // all or nothing: a bad task leaves no partition of the call marked
    for (int32_t i = 0; i < n; ++i) {
      const uint64_t h = tasks[i].handle;
      const bool out = h >= l->block_of.size();
      if (out || l->got[h]) {
        for (int32_t k = 0; k < i; ++k) l->got[tasks[k].handle] = 0;
        if (out)
          return bpsr::fail(BYTEPS_REDUCE_EARGS, "handle %llu outside the table (%zu partitions)",
                            (unsigned long long)h, l->block_of.size());
        return bpsr::fail(BYTEPS_REDUCE_EARGS, "partition %llu pushed twice in one iteration",
                          (unsigned long long)h);
      }
      l->got[h] = 1;
    }
  }
  if (n == 0) return 0;
  if (l->inline_drain) {
    if (const int rc = bpsr::prophet_add_many(l->pq, tasks, (size_t)n)) {
      std::lock_guard<std::mutex> g(l->mu);  // refused whole: none counts as pushed
      for (int32_t i = 0; i < n; ++i) l->got[tasks[i].handle] = 0;
      return rc;
    }
    return l->drain();
  }
  {
    std::lock_guard<std::mutex> g(l->inbox_mu);
    l->inbox.insert(l->inbox.end(), tasks, tasks + n);
  }
  l->pushes.fetch_add(1);
  if (l->waiting.load()) {
    std::lock_guard<std::mutex> g(l->mu);
    l->cv.notify_one();
  }
  return 0;
}

int byteps_prophet_loop_end(byteps_prophet_loop* l, double timeout_s) {
  if (!l) return bpsr::fail(BYTEPS_REDUCE_EARGS, "null loop");
  std::unique_lock<std::mutex> lk(l->mu);
  if (!l->active) return bpsr::fail(BYTEPS_REDUCE_EARGS, "no iteration begun");
  const auto pred = [&] { return l->err != 0 || l->blocks_released == l->nblocks(); };
  bool ok = true;
  if (timeout_s > 0)
    ok = l->done_cv.wait_for(lk, std::chrono::duration<double>(timeout_s), pred);
  else
    l->done_cv.wait(lk, pred);
  if (ok) {
    // The last block can be released while its drainer is still reporting
    // the group's partitions finished (outside mu): let that drain return
    // before the next begin() resets the scheduler, so no credit of this
    // iteration lands in the next one.  drain_mu is taken before mu.
    lk.unlock();
    { std::lock_guard<std::mutex> dg(l->drain_mu); }
    lk.lock();
  }
  l->active = false;
  if (l->err) return l->err;
  if (!ok)
    return bpsr::fail(BYTEPS_REDUCE_ETIMEOUT,
                      "iteration not complete after %.3f s: %d of %d blocks released", timeout_s,
                      l->blocks_released, l->nblocks());
  return 0;
}

int byteps_prophet_loop_release_calls(byteps_prophet_loop* l, uint64_t* calls) {
  if (!l || !calls) return bpsr::fail(BYTEPS_REDUCE_EARGS, "null argument");
  std::lock_guard<std::mutex> g(l->mu);
  *calls = l->release_calls;
  return 0;
}

int byteps_prophet_loop_destroy(byteps_prophet_loop* l) {
  if (!l) return 0;
  {
    std::lock_guard<std::mutex> g(l->mu);
    l->stop = true;
    l->cv.notify_all();
  }
  if (l->th.joinable()) l->th.join();
  delete l;
  return 0;
}

}  // extern "C"
