// GPU-resident parameter-server aggregation (include/bpsr/server.h): the
// per-key state machine of byteps/server/server.cc:147-308 with the engine
// threads (server.cc:70-145) replaced by HIP stream lanes and the CpuReducer
// calls replaced by the gfx950 fold kernels.
//
// Split over bpsr_server*.cpp (see bpsr_server_state.h); this file: lanes and
// their threads, the state machine, create / destroy and the single-key calls.
#include "bpsr_server_state.h"

namespace bpsr {
inline namespace srv {

// The device a server call last bound on this thread.  Every entry point
// binds the server's device (set_device), except the two per-key calls of a
// combining server's receive thread — push_ready and pull_device_view — which
// bind once per thread (bind_cached: hipSetDevice costs ≈ 30 ns, a third of a
// keyed push_ready): what they do themselves touches only the server's own
// streams and events, their launches go through the lane issuers, and
// whatever they create or allocate binds again first (force_device), since
// the caller may have switched devices in between.
thread_local int t_bound_device = -1;

int force_device(const byteps_server* s) {
  hipError_t e = hipSetDevice(s->cfg.device);
  if (e != hipSuccess) {
    t_bound_device = -1;
    return hip_fail(e, "hipSetDevice");
  }
  t_bound_device = s->cfg.device;
  return 0;
}

int set_device(const byteps_server* s) { return force_device(s); }

int bind_cached(const byteps_server* s) {
  return s->combine && t_bound_device == s->cfg.device ? 0 : force_device(s);
}

// Make the lane's fold stream wait for the pull copies issued from the
// stores (a fold rewrites a store), unless it already waits for the latest.
hipError_t wait_pull_copies(Lane& L) {
  const uint64_t p = L.pull_seq.load();
  if (p != L.fold_pull_seen.load()) {
    const hipError_t e = hipStreamWaitEvent(L.fold, L.d2h_mark, 0);
    if (e != hipSuccess) return e;
    L.fold_pull_seen.store(p);
  }
  return hipSuccess;
}

// Make the lane's fold stream wait for its copies, unless it already waits
// for the latest copy mark (push_ready-only rounds have no copies to wait for),
// and for its pull copies.
hipError_t wait_copies(Lane& L) {
  const uint64_t c = L.copy_seq.load();
  if (c != L.fold_copy_seen.load()) {
    const hipError_t e = hipStreamWaitEvent(L.fold, L.copy_mark, 0);
    if (e != hipSuccess) return e;
    L.fold_copy_seen.store(c);
  }
  return wait_pull_copies(L);
}

// Hand a launch's completion event to the lane's completer (combining):
// returns its seq; done_seq >= seq once it has completed.
uint64_t track(Lane& L, hipEvent_t ev) {
  std::lock_guard<std::mutex> g(L.done_mu);
  const uint64_t seq = ++L.issued_seq;
  L.cq.push_back({seq, ev, 0});
  L.cq_cv.notify_one();
  return seq;
}

// A keyed consumer launch is tracked like a lane's launches, on the server's
// keyed completer (s->klane), with its epoch.
uint64_t track_keyed(Lane& L, hipEvent_t ev, uint32_t epoch) {
  std::lock_guard<std::mutex> g(L.done_mu);
  const uint64_t seq = ++L.issued_seq;
  L.cq.push_back({seq, ev, epoch});
  L.cq_cv.notify_one();
  return seq;
}

void kq_epoch_done(byteps_server* s, uint32_t epoch, uint64_t seq);

// The lane's completer thread: waits for tracked launches in issue order and
// publishes how far they have completed (a keyed consumer's epoch is settled
// first: kq_epoch_done).
void completer_main(byteps_server* s, Lane* Lp) {
  (void)hipSetDevice(s->cfg.device);
  Lane& L = *Lp;
  std::unique_lock<std::mutex> lk(L.done_mu);
  for (;;) {
    L.cq_cv.wait(lk, [&] { return L.cq_stop || !L.cq.empty(); });
    if (L.cq.empty()) return;  // stopping, drained
    const Lane::Tracked t = L.cq.front();
    const uint64_t seq = t.seq;
    lk.unlock();
    if (t.kq_epoch) {
      // a keyed consumer: every pull and view of its epoch waits for this,
      // so poll its event (no other thread makes HIP calls on the device-
      // release path) — a blocking event wait wakes tens of microseconds
      // late — with short sleeps once the wait is long.  Once a slot-written
      // round has begun the epoch, the next epoch's consumer is launched
      // behind it (kq_launch_ahead).  An epoch that no round begins within
      // kKeyedIdleUs (or at destroy) is retired (kq_retire); a begun one still
      // open kKeyedCloseMs later is closed (kq_close_epoch).
      using clk = std::chrono::steady_clock;
      const auto i0 = clk::now();
      auto b0 = i0;  // when this completer saw the epoch begun
      const auto close_after = std::chrono::microseconds(std::min<int64_t>(
          (int64_t)byteps_server::kKeyedCloseMs * 1000, (int64_t)(s->kq_timeout_s * 5e5)));
      bool begun = false, ahead = false, retired = false, closed = false;
      while (hipEventQuery(t.ev) == hipErrorNotReady) {
        const auto now = clk::now();
        if (!begun && keyq_opened(s->kq) >= t.kq_epoch) {
          begun = true;
          b0 = now;
        }
        if (begun && !ahead && !retired &&
            s->kq_slot_epoch.load(std::memory_order_acquire) >= t.kq_epoch) {
          ahead = true;
          kq_launch_ahead(s, t.kq_epoch);
          continue;
        }
        if (!begun && !retired &&
            (s->kq_stopping.load(std::memory_order_acquire) ||
             now - i0 > std::chrono::microseconds(byteps_server::kKeyedIdleUs))) {
          retired = kq_retire(s, t.kq_epoch);
          continue;
        }
        if (begun && !closed && !retired &&
            (s->kq_stopping.load(std::memory_order_acquire) || now - b0 > close_after)) {
          closed = true;
          kq_close_epoch(s, t.kq_epoch);
          continue;
        }
        if (now - (begun ? b0 : i0) > std::chrono::microseconds(100))
          std::this_thread::sleep_for(std::chrono::microseconds(begun ? 5 : 20));
        else
          for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
      }
      kq_epoch_done(s, t.kq_epoch, t.seq);
    } else {
      (void)hipEventSynchronize(t.ev);  // a failed launch failed its keys already
    }
    lk.lock();
    L.cq.pop_front();
    L.done_seq = seq;
    L.done_pub.store(seq, std::memory_order_release);
    L.done_cv.notify_all();
  }
}

// server.h:138-162 GetThreadID: least accumulated bytes, sticky per key.
int pick_lane(byteps_server* s, size_t len) {
  int best = 0;
  uint64_t best_load = std::numeric_limits<uint64_t>::max();
  for (int i = 0; i < (int)s->acc_load.size(); ++i) {
    if (s->acc_load[i] < best_load) {
      best_load = s->acc_load[i];
      best = i;
    }
  }
  s->acc_load[best] += len;
  return best;
}

size_t key_slot(uint64_t key) {
  return (size_t)((key * 0x9E3779B97F4A7C15ull) >> 50) & (byteps_server::kKeyIndex - 1);
}

KeyState* get_key(byteps_server* s, uint64_t key, bool create) {
  for (size_t i = key_slot(key), probes = 0; probes < 32; ++probes) {
    KeyState* p = s->key_index[i].load(std::memory_order_acquire);
    if (!p) break;
    if (p->key == key) return p;
    i = (i + 1) & (byteps_server::kKeyIndex - 1);
  }
  {
    std::shared_lock<std::shared_mutex> g(s->map_mu);
    auto it = s->keys.find(key);
    if (it != s->keys.end()) return it->second.get();
    if (!create) return nullptr;
  }
  std::unique_lock<std::shared_mutex> g(s->map_mu);
  auto it = s->keys.find(key);  // another caller may have added it meanwhile
  if (it != s->keys.end()) return it->second.get();
  auto ks = std::make_unique<KeyState>();
  ks->key = key;
  KeyState* p = ks.get();
  s->keys.emplace(key, std::move(ks));
  if (s->key_index_n < byteps_server::kKeyIndex / 2) {
    for (size_t i = key_slot(key), probes = 0; probes < 32; ++probes) {
      if (!s->key_index[i].load(std::memory_order_relaxed)) {
        s->key_index[i].store(p, std::memory_order_release);
        ++s->key_index_n;
        break;
      }
      i = (i + 1) & (byteps_server::kKeyIndex - 1);
    }
  }
  return p;
}

int key_error(const KeyState* ks) {
  return fail(ks->error, "key %llu: an earlier fold failed: %s", (unsigned long long)ks->key,
              ks->error_msg.c_str());
}

// Allocate slots + store for a key (caller holds ks->mu).
int allocate(byteps_server* s, KeyState* ks, size_t len, int dtype) {
  if (ks->allocated) {
    if (len != ks->len || dtype != ks->dtype)
      return fail(BYTEPS_REDUCE_EARGS, "key re-declared with len %zu dtype %d (was %zu, %d)", len,
                  dtype, ks->len, ks->dtype);
    return 0;
  }
  if (elem_size(dtype) == 0) return fail(BYTEPS_REDUCE_EDTYPE, "Unsupported data type: %d", dtype);
  if (len == 0) return fail(BYTEPS_REDUCE_EARGS, "init tensor size not larger than 0");
  const int N = s->cfg.num_workers;
  // buckets of 1 MiB and more round to 64 KiB (the skew's class must not
  // depend on len, prophet_amd/arena.py); smaller ones to 4 KiB (small keys
  // are latency-bound, and many of them should not cost 80 KiB a slot)
  const size_t align = len >= (1u << 20) ? kSlotAlign : 4096;
  ks->stride = (len + align - 1) / align * align + kSlotSkew;
  if (int rc = force_device(s)) return rc;
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, ks->stride * (size_t)(N + 1));
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(key arena)");
  ks->arena = static_cast<char*>(p);
  ks->slot.resize(N);
  for (int k = 0; k < N; ++k) ks->slot[k] = ks->arena + ks->stride * k;
  ks->store = ks->arena + ks->stride * N;
  ks->got.assign(N, 0);
  ks->order.clear();
  if ((e = hipEventCreateWithFlags(&ks->done, hipEventDisableTiming)) != hipSuccess)
    return hip_fail(e, "hipEventCreate");
  if ((e = hipEventCreateWithFlags(&ks->copied, hipEventDisableTiming)) != hipSuccess)
    return hip_fail(e, "hipEventCreate");
  if ((e = hipEventCreateWithFlags(&ks->pulled, hipEventDisableTiming)) != hipSuccess)
    return hip_fail(e, "hipEventCreate");
  ks->len = len;
  ks->dtype = dtype;
  {
    std::unique_lock<std::shared_mutex> g(s->map_mu);
    ks->lane = pick_lane(s, len);
  }
  ks->allocated = true;
  return 0;
}

// May worker w's push land in its slot now?  Not while its push of the
// current round (or its init push) is still unfolded; in async mode with
// scheduling, not while an earlier async sum of the key is still queued.
bool can_push(const byteps_server* s, const KeyState* ks, int w) {
  if (ks->error) return true;  // the caller reports it
  if (ks->got[w]) return false;
  return !(s->cfg.async_mode && ks->inited && ks->pending > 0);
}

// Bring `len` bytes into worker `w`'s slot on the lane's copy stream, after
// the last issued fold of the key has consumed the slot.
int copy_in(byteps_server* s, KeyState* ks, int w, const void* data, size_t len, int loc,
            bool wait) {
  Lane& L = *s->lanes[ks->lane];
  ks->round_copied = true;
  hipError_t e = hipSuccess;
  // a keyed fold: its key's word on the host (wait_keyed_slots)
  if (ks->has_done && !wait_keyed_slots(s, ks)) e = hipStreamWaitEvent(L.copy, ks->fold_ev, 0);
  if (e == hipSuccess)
    e = hipMemcpyAsync(ks->slot[w], data, len,
                       loc == BYTEPS_SERVER_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice,
                       L.copy);
  if (e == hipSuccess) e = hipEventRecord(ks->copied, L.copy);
  if (e == hipSuccess) e = hipEventRecord(L.copy_mark, L.copy);
  if (e == hipSuccess) L.copy_seq.fetch_add(1);
  if (e == hipSuccess && wait) e = hipEventSynchronize(ks->copied);
  return e == hipSuccess ? 0 : hip_fail(e, "push copy");
}

// Queue the D2H of the store into mirror[idx] on the lane's d2h stream,
// behind the key's last issued fold (caller holds ks->mu).  Its own stream, so
// the copy overlaps the H2D pushes of the lane's other keys (PCIe is full duplex).
int queue_mirror(byteps_server* s, KeyState* ks, size_t idx) {
  Lane& L = *s->lanes[ks->lane];
  hipError_t e = ks->has_done ? hipStreamWaitEvent(L.d2h, ks->fold_ev, 0) : hipSuccess;
  if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent");
  // The copy kernel writes the pinned mirror straight over PCIe.  A
  // hipMemcpyAsync D2H queued behind a pending event wait was handed to an SDMA
  // engine that ran at ~13 GB/s beside the H2D pushes (rocprofv3 memory-copy
  // trace); the kernel path runs at the link's rate.
  int rc = byteps_reduce_copy(ks->mirror_dev[idx], ks->store, ks->len,
                              reinterpret_cast<void*>(L.d2h));
  if (rc) return rc;
  e = hipEventRecord(ks->mirrored, L.d2h);
  return e == hipSuccess ? 0 : hip_fail(e, "store mirror copy");
}

// Next mirror of an async-mode pull: a ring, so a view stays intact for the
// next num_workers pulls of the key.
size_t next_async_mirror(KeyState* ks) { return (size_t)(ks->mirror_next++ % ks->mirror.size()); }

// Pin the key's store mirrors on first use (fixed addresses from then on, as
// server.cc:60-69 reuses its response buffer to avoid re-registering memory);
// with queue_now, also mirror the finished current round.  Caller holds ks->mu.
int ensure_mirror(byteps_server* s, KeyState* ks, bool queue_now) {
  if (!ks->mirror.empty()) return 0;
  if (int rc = force_device(s)) return rc;
  const int nm = s->cfg.async_mode ? s->cfg.num_workers + 1 : 2;
  hipError_t e;
  for (int i = 0; i < nm; ++i) {
    void* p = nullptr;
    if ((e = hipHostMalloc(&p, ks->len, hipHostMallocDefault)) != hipSuccess)
      return hip_fail(e, "hipHostMalloc(store mirror)");
    void* d = nullptr;
    if ((e = hipHostGetDevicePointer(&d, p, 0)) != hipSuccess) {
      (void)hipHostFree(p);
      return hip_fail(e, "hipHostGetDevicePointer(store mirror)");
    }
    ks->mirror.push_back(static_cast<char*>(p));
    ks->mirror_dev.push_back(d);
  }
  if ((e = hipEventCreateWithFlags(&ks->mirrored, hipEventDisableTiming)) != hipSuccess)
    return hip_fail(e, "hipEventCreate");
  return queue_now ? queue_mirror(s, ks, ks->rounds & 1) : 0;
}

void enqueue_response(byteps_server* s, const Response& r) {
  std::lock_guard<std::mutex> g(s->rq_mu);
  s->rq.push_back(r);
  s->rq_cv.notify_one();
}

// Hand a pull to the responder (caller holds ks->mu).
void respond_later(byteps_server* s, KeyState* ks, byteps_server_pull_cb cb, void* ctx,
                   const char* view, int status) {
  Response r;
  r.key = ks->key;
  r.ks = ks;
  r.cb = cb;
  r.ctx = ctx;
  r.view = view;
  r.status = status;
  if (ks->keyed && status == 0) r.kseq = ks->fold_seq;
  enqueue_response(s, r);
}

// May a pull of the key be answered now?  Sync mode: once the round's push
// is finished (server.cc:293-304).  Engine blocking mode answers every pull at
// once from the store as it stands (server.cc:284-285 SendPullResponse with
// no gating), as does async mode.
bool pull_ready(const byteps_server* s, const KeyState* ks) {
  return s->blocking || ks->push_finished || ks->error;
}

// Count one answered pull; after NumWorkers the key re-arms (server.cc:105-113).
// Caller holds ks->mu.
void count_pull(byteps_server* s, KeyState* ks) {
  if (s->cfg.async_mode || s->blocking) return;  // nothing gates on the count
  if (++ks->pull_cnt == s->cfg.num_workers) {
    ks->push_finished = false;
    ks->pull_cnt = 0;
  }
  ks->cv.notify_all();
}

// A fold of the key failed after its push calls returned: remember it, fail
// the pulls waiting for the round, wake every waiter.  Caller holds ks->mu.
void fail_key(byteps_server* s, KeyState* ks, int rc) {
  if (!ks->error) {
    ks->error = rc;
    ks->error_msg = byteps_reduce_last_error();
  }
  for (auto& wp : ks->waiting) respond_later(s, ks, wp.cb, wp.ctx, nullptr, rc);
  ks->waiting.clear();
  for (auto& wc : ks->waiting_copies) {
    if (wc.direct) wc.direct->finish(rc);
    else respond_later(s, ks, wc.cb, wc.ctx, nullptr, rc);
  }
  ks->waiting_copies.clear();
  for (auto& a : ks->init_acks) {
    a.status = rc;
    enqueue_response(s, a);
  }
  ks->init_acks.clear();
  ks->cv.notify_all();
}

// Queue pulls into callers' buffers for the lane's issuer (caller holds
// ks->mu; the key's round is published, so its fold is issued): all of them
// under one lock, so the pulls one round completion answers ride in one
// launch.  `direct` ones are blocking pulls, whose waiters hear from the issuer.
void queue_pull_copies(byteps_server* s, KeyState* ks, const KeyState::WaitingCopy* wcs, size_t n) {
  if (n == 0) return;
  Lane& L = *s->lanes[ks->lane];
  std::unique_lock<std::mutex> kg(s->kq_park_mu, std::defer_lock);
  bool park = false;
  if (ks->keyed) {  // nothing reads a keyed store before its epoch is published
    kg.lock();
    park = s->kq_done_seq.load(std::memory_order_relaxed) < ks->fold_seq;
    if (!park) kg.unlock();
  }
  std::unique_lock<std::mutex> g(L.comb_mu, std::defer_lock);
  if (!park) g.lock();
  for (size_t i = 0; i < n; ++i) {
    const KeyState::WaitingCopy& wc = wcs[i];
    PullJob j;
    j.ks = ks;
    j.dst = wc.dst;
    j.len = wc.len;
    j.direct = wc.direct;
    j.resp.key = ks->key;
    j.resp.ks = ks;
    j.resp.cb = wc.cb;
    j.resp.ctx = wc.ctx;
    j.resp.view = static_cast<const char*>(wc.view);
    j.resp.len = wc.len;
    j.kseq = park ? ks->fold_seq : 0;
    if (park) s->kq_parked.push_back(j);
    else L.pulls.push_back(j);
  }
  if (!park) L.comb_cv.notify_one();
}

// Set on the responder thread, which runs the callers' callbacks: a blocking
// call made from inside a callback takes its own direct path, since routing it
// through the responder would wait on itself.
thread_local bool t_responder = false;

void responder_main(byteps_server* s) {
  (void)hipSetDevice(s->cfg.device);
  t_responder = true;
  for (;;) {
    Response r;
    {
      std::unique_lock<std::mutex> lk(s->rq_mu);
      s->rq_cv.wait(lk, [&] { return s->rq_stop || !s->rq.empty(); });
      if (s->rq.empty()) return;  // stopping and drained
      r = s->rq.front();
      s->rq.pop_front();
    }
    if (r.push_cb) {  // the push's bytes are in HBM: the sender's buffer is free
      int status = r.status;
      if (status == 0 && r.wait_lane) {
        std::unique_lock<std::mutex> dl(r.wait_lane->done_mu);
        r.wait_lane->done_cv.wait(dl, [&] { return r.wait_lane->done_seq >= r.wait_seq; });
      } else if (status == 0) {
        hipError_t e = hipEventSynchronize(r.ks->copied);
        if (e != hipSuccess) status = hip_fail(e, "push copy sync");
      }
      r.push_cb(r.ctx, r.key, r.worker, status);
      continue;
    }
    int status = r.status;
    if (status == 0 && r.kseq) {  // a view of a keyed round: its epoch first
      Lane& K = *s->klane;
      std::unique_lock<std::mutex> dl(K.done_mu);
      K.done_cv.wait(dl, [&] { return K.done_seq >= r.kseq; });
      dl.unlock();
      std::lock_guard<std::mutex> g(r.ks->mu);
      if (r.ks->error) status = r.ks->error;
    }
    if (status == 0 && r.wait_lane) {  // a pull copied by the lane's issuer
      std::unique_lock<std::mutex> dl(r.wait_lane->done_mu);
      r.wait_lane->done_cv.wait(dl, [&] { return r.wait_lane->done_seq >= r.wait_seq; });
    } else if (status == 0) {
      // The event still names the answered round's copy: the next round
      // cannot finish before this pull is counted (it needs this worker's
      // next push, which follows the answer).
      hipError_t e = hipEventSynchronize(r.ks->mirrored);
      if (e != hipSuccess) status = hip_fail(e, "store mirror sync");
    }
    if (status == 0) {
      // Count BEFORE answering, under the key lock, as the reference counts
      // under flag_mu_ in the same step as SendPullResponse
      // (server.cc:100-113, 293-298): once the worker has its answer it may
      // push and finish the next round, and a late count would land there.
      std::lock_guard<std::mutex> g(r.ks->mu);
      count_pull(s, r.ks);
    }
    r.cb(r.ctx, r.key, status == 0 ? r.view : nullptr,
         status == 0 ? (r.len ? r.len : r.ks->len) : 0, status);
  }
}

// A round's fold is issued: publish it (caller holds ks->mu).  `mark`: also
// raise the lane's fold mark (a batched issue raises it once, before).
int finish_round(byteps_server* s, KeyState* ks, const std::vector<int>& order,
                 bool mark, hipEvent_t batch, uint64_t batch_seq,
                 bool keyed) {
  Lane& L = *s->lanes[ks->lane];
  s->n_rounds_folded.add();
  ks->keyed = keyed;  // a keyed consumer's fold, tracked by the keyed completer
  ks->fold_lane = keyed ? -1 : ks->lane;
  ks->round_copied = false;
  ks->round_mark_copy = false;
  if (mark) {  // a single fold: its own event, and the lane's mark
    hipError_t e = hipEventRecord(ks->done, L.fold);
    if (e == hipSuccess) e = hipEventRecord(L.fold_mark, L.fold);
    if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
    ks->fold_ev = ks->done;
    ks->fold_seq = s->combine ? track(L, ks->done) : 0;
  } else {     // batched: the batch's own event (or the lane mark behind it)
    ks->fold_ev = batch ? batch : L.fold_mark;
    ks->fold_seq = batch_seq;
  }
  ks->has_done = true;
  int rc = 0;
  if (!ks->mirror.empty() && (rc = queue_mirror(s, ks, (ks->rounds + 1) & 1))) return rc;
  ks->last_order = order;
  std::fill(ks->got.begin(), ks->got.end(), 0);
  ks->rounds++;
  ks->push_finished = true;
  ks->pull_cnt = 0;
  const char* view = ks->mirror.empty() ? nullptr : ks->mirror[ks->rounds & 1];
  for (auto& wp : ks->waiting) respond_later(s, ks, wp.cb, wp.ctx, view, 0);
  ks->waiting.clear();
  queue_pull_copies(s, ks, ks->waiting_copies.data(), ks->waiting_copies.size());
  ks->waiting_copies.clear();
  ks->cv.notify_all();
  return 0;
}

int injected_failure(byteps_server* s) {
  if (s->fail_after < 0 || s->issued.fetch_add(1) < s->fail_after) return 0;
  return fail(BYTEPS_REDUCE_EHIP, "injected fold failure (BPSR_SERVER_FAIL_AFTER=%ld)",
              s->fail_after);
}


// Blocking readers of a keyed round's store wait for its epoch to be
// published (caller holds no lock); then the key's error, if it failed.
void wait_published(byteps_server* s, KeyState* ks, uint64_t seq) {
  (void)ks;
  Lane& K = *s->klane;
  if (K.done_pub.load(std::memory_order_acquire) >= seq) return;
  std::unique_lock<std::mutex> dl(K.done_mu);
  K.done_cv.wait(dl, [&] { return K.done_seq >= seq; });
}

// Issue a job's kernels on the lane's fold stream and apply its state
// changes — the body of the engine thread (server.cc:70-145).  Caller holds
// ks->mu.
int execute(byteps_server* s, const FoldJob& j) {
  if (int rc = injected_failure(s)) return rc;
  KeyState* ks = j.ks;
  Lane& L = *s->lanes[ks->lane];
  void* fs = reinterpret_cast<void*>(L.fold);
  FoldJob fallback;
  if (j.kind == kKeyRelease) {  // a keyed round whose pushes were copied: behind the copies
    const int rc = key_release(s, ks, j.order, L.copy);
    if (rc <= 0) return rc;
    fallback = j;  // device releases went off meanwhile: an ordinary fused fold
    fallback.kind = kFinishFused;
    return execute(s, fallback);
  }
  // Folds run behind the slots' copies (byteps_server_push_async returns
  // before they finish; the copy stream is in order, so the lane's copy mark
  // covers every copy issued so far, batched ones included) and behind the
  // last mirror D2H of the store.
  hipError_t we = wait_copies(L);
  if (we == hipSuccess && ks->mirrored) we = hipStreamWaitEvent(L.fold, ks->mirrored, 0);
  if (we != hipSuccess) return hip_fail(we, "hipStreamWaitEvent");
  s->n_fold_launches.fetch_add(1, std::memory_order_relaxed);
  int rc = 0;
  switch (j.kind) {
    case kSumRecv:  // SUM_RECV (server.cc:117-139): merged (= first arrival's slot) += push
      return byteps_reduce_sum(ks->slot[j.acc], ks->slot[j.w], ks->len, ks->dtype, fs);
    case kAsyncSum: {  // server.cc:220-230: every push is summed straight into the store
      rc = byteps_reduce_sum(ks->store, ks->slot[j.w], ks->len, ks->dtype, fs);
      if (rc) return rc;
      s->n_rounds_folded.add();
      hipError_t e = hipEventRecord(ks->done, L.fold);
      if (e == hipSuccess) e = hipEventRecord(L.fold_mark, L.fold);
      if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
      ks->fold_ev = ks->done;
      ks->fold_seq = 0;
      ks->has_done = true;
      ks->rounds++;
      ks->cv.notify_all();
      return 0;
    }
    case kFinishIncremental:  // COPY_MERGED (server.cc:82-115)
      rc = byteps_reduce_copy(ks->store, ks->slot[j.acc], ks->len, fs);
      break;
    default: {  // one fused left fold in arrival order straight into the store
      const int N = (int)j.order.size();
      std::vector<const void*> srcs(N);
      for (int k = 0; k < N; ++k) srcs[k] = ks->slot[j.order[k]];
      rc = byteps_reduce_sum_n(ks->store, srcs.data(), N, ks->len, ks->dtype,
                               BYTEPS_REDUCE_MODE_REFERENCE, fs);
    }
  }
  if (rc) return rc;
  return finish_round(s, ks, j.order);
}

// Run a job now (reference default: the engine takes messages FIFO and this
// build issues them to the lane's stream in arrival order), or queue it for
// the lane's dispatcher (scheduling on).  Caller holds ks->mu.
int submit(byteps_server* s, KeyState* ks, FoldJob&& j) {
  if (!s->schedule) {
    // The arrival is already recorded: a fold that cannot be issued must
    // fail the key, or every other worker's push / pull of it waits forever
    // (the dispatcher and flush_folds do the same for their jobs).
    const int rc = execute(s, j);
    if (rc) fail_key(s, ks, rc);
    return rc;
  }
  ks->pending++;
  s->lanes[ks->lane]->q->push(ks->key, std::move(j));
  return 0;
}

// BYTEPS_SERVER_ENABLE_SCHEDULE: the lane's engine thread.  Pops by
// (fewest counted pushes, oldest) and, like the reference engine thread that
// runs each message to completion before the next pop (server.cc:70-145),
// waits for each job's kernels before popping again — which is what lets
// later arrivals overtake queued ones.
void dispatcher_main(byteps_server* s, int lane) {
  (void)hipSetDevice(s->cfg.device);
  Lane& L = *s->lanes[lane];
  FoldJob j;
  uint64_t key = 0;
  while (L.q->wait_pop(&j, &key)) {
    {
      std::lock_guard<std::mutex> dl(L.dbg_mu);
      if (L.log.size() < (size_t)kMaxDebugLog) L.log.push_back(key);
    }
    KeyState* ks = j.ks;
    {
      std::lock_guard<std::mutex> g(ks->mu);
      ks->pending--;
      if (!ks->error) {
        const int rc = execute(s, j);
        if (rc) fail_key(s, ks, rc);
      }
      if (hipEventRecord(L.job_done, L.fold) != hipSuccess) fail_key(s, ks, BYTEPS_REDUCE_EHIP);
      ks->cv.notify_all();
    }
    (void)hipEventSynchronize(L.job_done);
  }
}

// A push's bytes are in slot w: advance the state machine (caller holds ks->mu).
// With `defer` (a batched call, no scheduling), a round's fused fold is not
// issued here but handed back, to go out with the call's other keys in one
// batched launch per lane (flush_folds); the key counts it as pending.
// May an arrival of the current (non-init) round take position `pos`?
int check_pos(const byteps_server* s, const KeyState* ks, int pos) {
  const int N = s->cfg.num_workers;
  if (pos >= N) return fail(BYTEPS_REDUCE_EARGS, "arrival position %d outside [0, %d)", pos, N);
  const bool stamp = pos >= 0 && s->cfg.policy == BYTEPS_SERVER_FUSED;
  if (!ks->inited || s->cfg.async_mode) return 0;
  if (ks->arrived > 0 && stamp != ks->stamped)
    return fail(BYTEPS_REDUCE_EARGS, "key %llu: stamped and unstamped arrivals in one round",
                (unsigned long long)ks->key);
  if (stamp && ks->arrived > 0 && ks->order[pos] >= 0)
    return fail(BYTEPS_REDUCE_EARGS, "key %llu: arrival position %d taken twice",
                (unsigned long long)ks->key, pos);
  return 0;
}

// `pos` >= 0 (a server group's range split, fused policy): the arrival takes
// that position of the round's order, which the group stamped for the whole
// key, instead of its position here — every piece of the key then folds in the
// same order (server.cc:216-250 has one order per key).
int arrive(byteps_server* s, KeyState* ks, int w, std::vector<FoldJob>* defer,
           int pos) {
  if (ks->error) return key_error(ks);
  const int N = s->cfg.num_workers;
  Lane& L = *s->lanes[ks->lane];
  if (int rc = check_pos(s, ks, pos)) return rc;
  if (!ks->inited) {
    // Round 0: server.cc:175-199 — after all NumWorkers init pushes the store
    // is initialised by copying the LAST arrived push, in the handler itself
    // (stamped: the push at the last position).
    if (ks->got[w]) return fail(BYTEPS_REDUCE_EARGS, "worker %d sent two init pushes", w);
    ks->got[w] = 1;
    if (pos < 0 || pos == N - 1) ks->init_last = w;
    if (++ks->init_count < N) return 0;
    w = ks->init_last;
    // every init push is counted: a failure from here on fails the key (the
    // other workers' init pushes wait for `inited || error`)
    int rc = injected_failure(s);
    hipError_t we = rc ? hipSuccess : wait_copies(L);
    if (!rc && we != hipSuccess) rc = hip_fail(we, "hipStreamWaitEvent");
    if (!rc)
      rc = byteps_reduce_copy(ks->store, ks->slot[w], ks->len, reinterpret_cast<void*>(L.fold));
    if (!rc) {
      hipError_t e = hipEventRecord(ks->done, L.fold);
      if (e == hipSuccess) e = hipEventRecord(L.fold_mark, L.fold);
      if (e != hipSuccess) rc = hip_fail(e, "hipEventRecord");
    }
    if (rc) {
      fail_key(s, ks, rc);
      return rc;
    }
    ks->fold_ev = ks->done;
    ks->fold_seq = 0;
    ks->fold_lane = ks->lane;
    ks->keyed = false;
    ks->round_copied = false;
    ks->round_mark_copy = false;
    ks->has_done = true;
    ks->inited = true;
    std::fill(ks->got.begin(), ks->got.end(), 0);
    // server.cc:196-198: every held init push is answered now
    for (auto& a : ks->init_acks) enqueue_response(s, a);
    ks->init_acks.clear();
    ks->cv.notify_all();
    return 0;
  }
  EngineQueue<FoldJob>* q = s->schedule ? L.q.get() : nullptr;
  if (s->cfg.async_mode) {
    FoldJob j;
    j.ks = ks;
    j.kind = kAsyncSum;
    j.w = w;
    const int rc = submit(s, ks, std::move(j));
    if (q) q->clear_counter(ks->key);  // server.cc:277
    return rc;
  }
  if (ks->got[w]) return fail(BYTEPS_REDUCE_EARGS, "worker %d pushed twice in one round", w);
  const bool stamp = pos >= 0 && s->cfg.policy == BYTEPS_SERVER_FUSED;
  if (stamp) {
    if (ks->arrived == 0) ks->order.assign(N, -1);
    ks->order[pos] = w;
  } else {
    ks->order.push_back(w);
  }
  ks->stamped = stamp;
  ks->got[w] = 1;
  ks->arrived++;
  if (ks->arrived > 1 && s->cfg.policy == BYTEPS_SERVER_INCREMENTAL) {
    FoldJob j;  // SUM_RECV (server.cc:245-251)
    j.ks = ks;
    j.kind = kSumRecv;
    j.w = w;
    j.acc = ks->order[0];
    const int rc = submit(s, ks, std::move(j));
    if (rc) return rc;
  } else if (ks->arrived > 1 && ks->arrived < N && q) {
    q->count(ks->key);  // the SUM_RECV the reference would have queued
  }
  if (ks->arrived < N) return 0;
  if (!q && keyed_member(s, ks)) {
    // device release: no launch for this round (the order moves through a
    // scratch vector that keeps its capacity: no allocation per round)
    std::vector<int>& order = ks->order_tmp;
    order.assign(ks->order.begin(), ks->order.end());
    ks->order.clear();
    ks->arrived = 0;
    if (!ks->round_copied) {  // the pushes are in their slots already (push_ready)
      // a release from the host orders nothing on the device: the producers
      // a caller named with byteps_server_order_after are waited for here
      // (a no-op without a pending order_after)
      int rc = wait_order_gate(s);
      if (!rc) rc = key_release(s, ks, order, nullptr);
      if (rc <= 0) {
        if (rc) fail_key(s, ks, rc);
        return rc;
      }
    } else {
      // Copied pushes: the consumer passes this key at once (a SKIP word from
      // the host) and the round folds with a lane launch behind its copies,
      // which publishes it.  Releasing it behind the copies instead made the
      // consumer wait on lane-stream work — which could sit behind launches
      // the consumer's own residency kept off the chip: with non-blocking
      // device pushes from 8 threads an epoch never completed (r04s38-s48).
      const int rc = key_release(s, ks, order, nullptr, /*skip=*/true);
      if (rc < 0) {
        fail_key(s, ks, rc);
        return rc;
      }
    }
    // copied pushes, or device releases turned off meanwhile: an ordinary fold
    FoldJob j;
    j.ks = ks;
    j.kind = kFinishFused;
    j.acc = order[0];
    j.order = order;
    if (defer) {
      ks->pending++;
      defer->push_back(std::move(j));
      return 0;
    }
    return submit(s, ks, std::move(j));
  }
  FoldJob j;
  j.ks = ks;
  j.kind = s->cfg.policy == BYTEPS_SERVER_INCREMENTAL ? kFinishIncremental : kFinishFused;
  j.acc = ks->order[0];
  // the order's buffer travels with the job and comes back through
  // order_spare once the issuer has published the round (recycle_order):
  // no allocation here and no free on another thread, per round
  j.order.swap(ks->order);
  ks->order.swap(ks->order_spare);
  ks->order.clear();
  ks->arrived = 0;
  // Combining: EVERY finished round goes to the lane's issuer (a fold that
  // writes the store must queue behind the lane's queued copies into the
  // slots and pull copies out of the store, which only the issuer orders);
  // otherwise the batchable fused rounds of a batched call.
  if (defer && !q && (s->combine || (j.kind == kFinishFused && N <= kMaxSrcs))) {
    ks->pending++;
    defer->push_back(std::move(j));
    return 0;
  }
  const int rc = submit(s, ks, std::move(j));
  if (q) q->clear_counter(ks->key);  // server.cc:269-271
  return rc;
}

// A published round's order buffer goes back to its key (caller holds
// ks->mu), for the next round's arrivals (arrive).
void recycle_order(KeyState* ks, FoldJob& j) {
  if (ks->order_spare.capacity() == 0) ks->order_spare.swap(j.order);
}

// Issue deferred fused folds: per (lane, dtype) ONE batched launch whose
// buckets are the keys' rounds (dst = store, sources = slots in arrival order),
// then each key's round is published.  Returns the first error.
int issue_one(byteps_server* s, FoldJob& j);
int flush_folds(byteps_server* s, std::vector<FoldJob>& jobs) {
  if (jobs.empty()) return 0;
  int first_rc = 0;
  // rounds a batched launch cannot carry (incremental COPY_MERGED, more than
  // kMaxSrcs sources) go out one by one, in their arrival order
  {
    std::vector<FoldJob> keep;
    keep.reserve(jobs.size());
    for (auto& j : jobs) {
      if (j.kind == kFinishFused && (int)j.order.size() <= kMaxSrcs) {
        keep.push_back(std::move(j));
      } else {
        const int rc = issue_one(s, j);
        if (rc && !first_rc) first_rc = rc;
      }
    }
    jobs.swap(keep);
  }
  std::stable_sort(jobs.begin(), jobs.end(), [](const FoldJob& a, const FoldJob& b) {
    return a.ks->lane != b.ks->lane ? a.ks->lane < b.ks->lane : a.ks->dtype < b.ks->dtype;
  });
  size_t i = 0;
  while (i < jobs.size()) {
    size_t e = i + 1;
    while (e < jobs.size() && jobs[e].ks->lane == jobs[i].ks->lane &&
           jobs[e].ks->dtype == jobs[i].ks->dtype)
      ++e;
    Lane& L = *s->lanes[jobs[i].ks->lane];
    std::lock_guard<std::mutex> bg(L.batch_mu);
    std::vector<byteps_bucket_desc> d(e - i);
    // The rounds' copies: each round's own copy events when every copy of
    // every round in the batch recorded one, else every copy of the lane.
    bool lane_wide = false;
    std::vector<hipEvent_t> evs;
    for (size_t k = i; k < e && !lane_wide; ++k) {
      KeyState* ks = jobs[k].ks;
      std::lock_guard<std::mutex> g(ks->mu);
      if (ks->round_mark_copy) lane_wide = true;
      else if (ks->round_copied) evs.push_back(ks->copied);
    }
    hipError_t we0 = lane_wide ? wait_copies(L) : wait_pull_copies(L);
    for (size_t k = 0; !lane_wide && we0 == hipSuccess && k < evs.size(); ++k)
      we0 = hipStreamWaitEvent(L.fold, evs[k], 0);
    int rc = we0 == hipSuccess ? 0 : hip_fail(we0, "hipStreamWaitEvent");
    for (size_t k = i; k < e; ++k) {
      KeyState* ks = jobs[k].ks;
      std::lock_guard<std::mutex> g(ks->mu);
      if (ks->mirrored) {
        hipError_t we = hipStreamWaitEvent(L.fold, ks->mirrored, 0);
        if (we != hipSuccess && !rc) rc = hip_fail(we, "hipStreamWaitEvent");
      }
      byteps_bucket_desc& b = d[k - i];
      std::memset(&b, 0, sizeof(b));
      b.dst = ks->store;
      for (size_t m = 0; m < jobs[k].order.size(); ++m) b.srcs[m] = ks->slot[jobs[k].order[m]];
      b.len = ks->len;
      b.n = (int)jobs[k].order.size();
    }
    hipEvent_t bev = nullptr;  // the launch's own event (batched_with_ring records it)
    if (!rc)
      rc = batched_with_ring(d.data(), (int)d.size(), jobs[i].ks->dtype,
                             BYTEPS_REDUCE_MODE_REFERENCE, L.fold, L.ring, &bev);
    uint64_t bseq = 0;
    if (!rc) {  // raised before any round is published: a pull that sees one waits past it
      s->n_fold_launches.fetch_add(1, std::memory_order_relaxed);
      hipError_t me = hipEventRecord(L.fold_mark, L.fold);
      if (me != hipSuccess) rc = hip_fail(me, "hipEventRecord");
      if (!rc && bev && s->combine) bseq = track(L, bev);
    }
    for (size_t k = i; k < e; ++k) {
      KeyState* ks = jobs[k].ks;
      std::lock_guard<std::mutex> g(ks->mu);
      ks->pending--;
      const int r2 = rc ? rc : finish_round(s, ks, jobs[k].order, /*mark=*/false, bev, bseq);
      if (r2) fail_key(s, ks, r2);
      recycle_order(ks, jobs[k]);
      ks->cv.notify_all();
    }
    if (rc && !first_rc) first_rc = rc;
    i = e;
  }
  jobs.clear();
  return first_rc;
}

// Engine blocking mode (server.cc:205-262): the handler did the copy / sum
// itself before answering the push, so the push returns once the work it
// issued on the key's lane has completed.
int finish_blocking(byteps_server* s, KeyState* ks, std::unique_lock<std::mutex>& lk) {
  hipStream_t fs = s->lanes[ks->lane]->fold;
  lk.unlock();
  hipError_t e = hipStreamSynchronize(fs);
  return e == hipSuccess ? 0 : hip_fail(e, "engine blocking: fold sync");
}

// Issue one deferred round (no batching partner).
int issue_one(byteps_server* s, FoldJob& j) {
  KeyState* ks = j.ks;
  Lane& IL = *s->lanes[ks->lane];
  const char* was = IL.where.load();
  IL.where = "issue_one: key lock";
  std::lock_guard<std::mutex> g(ks->mu);
  IL.where = was;
  ks->pending--;
  const int rc = ks->error ? 0 : execute(s, j);
  if (rc) fail_key(s, ks, rc);
  recycle_order(ks, j);
  ks->cv.notify_all();
  return rc;
}

// Hand the rounds a single-key call completed (defer lists of arrive; caller
// holds no key lock) to their lanes' issuer threads.  The call returns at
// once: the round is published (pulls may go) when the issuer has issued its
// fold.  Keys arriving together — the last worker of many keys, or several
// workers' calls at once — thus share ONE batched launch per lane instead of
// one launch each, and no caller issues other callers' folds.  The reference
// engine pays a host sum per message (server.cc:70-145); here the host work
// per round is an append and a wake-up.
int issue_combined(byteps_server* s, std::vector<FoldJob>& jobs) {
  for (auto& j : jobs) {
    Lane& L = *s->lanes[j.ks->lane];
    std::lock_guard<std::mutex> g(L.comb_mu);
    L.comb.push_back(std::move(j));
    L.comb_cv.notify_one();
  }
  jobs.clear();
  return 0;
}

// The rounds a batched call (push_many / push_ready_many) completed.  When
// combining they go to the lane issuers like any other call's: another
// worker's non-blocking push may still have its copy into a slot of the same
// key queued there, or a pull its copy out of the store, and only the issuer
// issues those before the fold (issuer_main).  Otherwise this thread issues
// them as one batched launch per lane.
int issue_deferred(byteps_server* s, std::vector<FoldJob>& jobs) {
  return s->combine ? issue_combined(s, jobs) : flush_folds(s, jobs);
}

// Issue the non-blocking device pushes that piled up on a lane: ONE wait for
// the lane's folds so far (a slot is free once the fold that read it was
// issued — the caller waited for that, can_push), ONE batched copy into the
// slots, the lane's copy mark (later folds wait for it), then the pushes'
// acknowledgements, which the responder sends once the copy has completed.
void issue_copies(byteps_server* s, Lane& L, std::vector<CopyJob>& jobs) {
  int rc = 0;
  uint64_t seq = 0;
  {
    std::lock_guard<std::mutex> bg(L.batch_mu);
    hipError_t e = hipStreamWaitEvent(L.copy, L.fold_mark, 0);
    if (e != hipSuccess) rc = hip_fail(e, "hipStreamWaitEvent");
    hipEvent_t last = nullptr;
    L.where = "copies: key locks";
    for (auto& j : jobs) {  // keyed folds run on the consumer's stream
      std::lock_guard<std::mutex> g(j.ks->mu);
      if (!rc && j.ks->keyed && j.ks->has_done && !wait_keyed_slots(s, j.ks) &&
          j.ks->fold_ev != last) {
        last = j.ks->fold_ev;
        if ((e = hipStreamWaitEvent(L.copy, last, 0)) != hipSuccess) rc = hip_fail(e, "hipStreamWaitEvent");
      }
    }
    std::vector<byteps_bucket_desc> d(jobs.size());
    for (size_t k = 0; k < jobs.size(); ++k) {
      std::memset(&d[k], 0, sizeof(d[k]));
      d[k].dst = jobs[k].ks->slot[jobs[k].w];
      d[k].srcs[0] = jobs[k].src;
      d[k].len = jobs[k].len;
      d[k].n = 1;
    }
    hipEvent_t cev = nullptr;
    L.where = "copies: launch";
    if (!rc)
      rc = batched_with_ring(d.data(), (int)d.size(), BYTEPS_REDUCE_UINT8,
                             BYTEPS_REDUCE_MODE_REFERENCE, L.copy, L.ring, &cev);
    L.where = "copies: answers";
    if (!rc) {
      s->n_copy_launches.fetch_add(1, std::memory_order_relaxed);
      e = hipEventRecord(L.copy_mark, L.copy);
      if (e != hipSuccess) rc = hip_fail(e, "hipEventRecord");
      else L.copy_seq.fetch_add(1);
      if (!rc && cev) seq = track(L, cev);
    }
  }
  for (auto& j : jobs) {
    if (rc) {  // the copy never ran: fail the key (its round cannot fold)
      std::lock_guard<std::mutex> g(j.ks->mu);
      fail_key(s, j.ks, rc);
      j.ack.status = rc;
    } else {
      j.ack.wait_lane = &L;
      j.ack.wait_seq = seq;
    }
    if (j.direct) {  // a blocking push waits on the lane itself
      j.direct->lane = rc ? nullptr : &L;
      j.direct->seq = seq;
      j.direct->finish(rc);
      continue;
    }
    enqueue_response(s, j.ack);
  }
  jobs.clear();
}

// Issue the pulls into device buffers that piled up on a lane: ONE wait for
// the lane's folds so far (every pulled round was issued before its pull was
// queued), ONE batched copy from the stores on the d2h stream, the d2h mark
// (later folds of the lane wait for it before rewriting a store), then the
// answers, which the responder sends once the copy has completed.
void issue_pull_copies(byteps_server* s, Lane& L, std::vector<PullJob>& jobs) {
  int rc = 0;
  uint64_t seq = 0;
  {
    std::lock_guard<std::mutex> bg(L.batch_mu);
    hipError_t e = hipStreamWaitEvent(L.d2h, L.fold_mark, 0);
    if (e != hipSuccess) rc = hip_fail(e, "hipStreamWaitEvent");
    std::vector<byteps_bucket_desc> d(jobs.size());
    for (size_t k = 0; k < jobs.size(); ++k) {
      std::memset(&d[k], 0, sizeof(d[k]));
      d[k].dst = jobs[k].dst;
      d[k].srcs[0] = jobs[k].ks->store;
      d[k].len = jobs[k].len;
      d[k].n = 1;
    }
    hipEvent_t cev = nullptr;
    if (!rc)
      rc = batched_with_ring(d.data(), (int)d.size(), BYTEPS_REDUCE_UINT8,
                             BYTEPS_REDUCE_MODE_REFERENCE, L.d2h, L.ring, &cev);
    if (!rc) {
      s->n_pull_launches.fetch_add(1, std::memory_order_relaxed);
      e = hipEventRecord(L.d2h_mark, L.d2h);
      if (e != hipSuccess) rc = hip_fail(e, "hipEventRecord");
      else L.pull_seq.fetch_add(1);
      if (!rc && cev) seq = track(L, cev);
    }
  }
  s->n_pulls.add(jobs.size());
  for (auto& j : jobs) {
    if (j.direct) {  // a blocking pull waits on the lane itself, then counts
      j.direct->lane = &L;
      j.direct->seq = seq;
      j.direct->finish(rc);
      continue;
    }
    if (rc) {
      j.resp.status = rc;
    } else {
      j.resp.wait_lane = &L;
      j.resp.wait_seq = seq;
    }
    enqueue_response(s, j.resp);
  }
  jobs.clear();
}

// The lane's issuer thread (combining): one batch of whatever rounds piled
// up since the last issue.  Drains before it exits.
void issuer_main(byteps_server* s, int lane) {
  (void)hipSetDevice(s->cfg.device);
  // with device releases, every launch of this thread fits beside a running
  // keyed consumer (2 × 58 KiB of each CU's LDS): 4 workgroups' worth per CU
  if (s->dev_release) t_occ_floor = 4;
  t_where = &s->lanes[lane]->where;
  Lane& L = *s->lanes[lane];
  std::vector<FoldJob> folds;
  std::vector<CopyJob> copies;
  std::vector<PullJob> pulls;
  std::unique_lock<std::mutex> lk(L.comb_mu);
  for (;;) {
    L.comb_cv.wait(lk, [&] {
      return L.comb_stop || !L.comb.empty() || !L.copies.empty() || !L.pulls.empty();
    });
    if (L.comb.empty() && L.copies.empty() && L.pulls.empty()) return;  // stopping, drained
    // at most `inflight` of the lane's launches queued or running: while the
    // device works through them, the rounds completing meanwhile pile up and
    // go out together in the next launch
    lk.unlock();
    L.where = "window";
    {
      std::unique_lock<std::mutex> dl(L.done_mu);
      L.done_cv.wait(dl, [&] { return L.issued_seq - L.done_seq < byteps_server::kInflight; });
    }
    lk.lock();
    folds.swap(L.comb);
    copies.swap(L.copies);
    pulls.swap(L.pulls);
    lk.unlock();
    const auto t0 = std::chrono::steady_clock::now();
    L.where = "copies";
    if (!copies.empty()) issue_copies(s, L, copies);  // before the folds that read them
    L.where = "pulls";
    if (!pulls.empty()) issue_pull_copies(s, L, pulls);  // before folds that rewrite stores
    L.where = "folds";
    if (folds.size() == 1)
      (void)issue_one(s, folds[0]);
    else if (!folds.empty())
      (void)flush_folds(s, folds);  // a failed fold fails its keys (fail_key)
    folds.clear();
    L.where = "idle";
    lk.lock();
    if (!L.pulls.empty()) {
      // the pulls parked on the rounds just published go out now, in one
      // launch behind the folds, rather than after another wake-up
      pulls.swap(L.pulls);
      lk.unlock();
      issue_pull_copies(s, L, pulls);
      lk.lock();
    }
    s->issuer_ns.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                               std::chrono::steady_clock::now() - t0).count(),
                           std::memory_order_relaxed);
  }
}

// After a single-key call issued (or queued) its round: the key's own error,
// if its fold failed by the time the call returns.
int own_key_status(KeyState* ks) {
  std::lock_guard<std::mutex> g(ks->mu);
  return ks->error ? key_error(ks) : 0;
}

// Init pushes block until every worker's init push has arrived and the store
// is initialised: the reference answers them only then (server.cc:184-198).
int arrive_and_wait_init(byteps_server* s, KeyState* ks, int w, std::unique_lock<std::mutex>& lk,
                         std::vector<FoldJob>* defer) {
  const bool init_round = !ks->inited;
  int rc = arrive(s, ks, w, defer);
  if (rc || !init_round) return rc;
  ks->cv.wait(lk, [&] { return ks->inited || ks->error; });
  return ks->error ? key_error(ks) : 0;
}

// The pull destination as the device addresses it: device memory itself, or
// pinned host memory mapped for the device; nullptr for pageable memory.
void* device_view(void* out, int location) {
  if (location == BYTEPS_SERVER_DEVICE) return out;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, out, 0) == hipSuccess && d) return d;
  (void)hipGetLastError();  // pageable: not an error, just not addressable
  return nullptr;
}

// Copying pulls into pinned host memory: the library's copy kernel writes
// the destination through its device view, so the D2H runs beside the push
// H2D copies (SDMA) at the link's full-duplex rate — two SDMA copies, one per
// direction, share ~54 GB/s, SDMA H2D + kernel D2H move 87 GB/s together
// (tools/pcie_probe.py, r05s04).  Device destinations and pageable memory:
// hipMemcpyAsync.
void* pull_kernel_dst(void* out, int location) {
  return location == BYTEPS_SERVER_HOST ? device_view(out, location) : nullptr;
}

KeyState* key_for_pull(byteps_server* s, uint64_t key) {
  KeyState* ks = get_key(s, key, false);
  if (!ks || !ks->allocated)  // server.cc:282-283
    fail(BYTEPS_REDUCE_EARGS, "Processing pull request when the key %llu has not been inited yet",
         (unsigned long long)key);
  return ks && ks->allocated ? ks : nullptr;
}

void destroy_lanes(byteps_server* s) {
  for (auto& Lp : s->lanes)
    if (Lp && Lp->q) Lp->q->stop();
  for (auto& Lp : s->lanes)
    if (Lp && Lp->dispatcher.joinable()) Lp->dispatcher.join();
  for (auto& Lp : s->lanes) {
    if (!Lp) continue;
    std::lock_guard<std::mutex> g(Lp->comb_mu);
    Lp->comb_stop = true;
    Lp->comb_cv.notify_all();
  }
  for (auto& Lp : s->lanes)  // the issuers issue what is queued, then exit
    if (Lp && Lp->issuer.joinable()) Lp->issuer.join();
  for (auto& Lp : s->lanes) {
    if (!Lp) continue;
    std::lock_guard<std::mutex> g(Lp->done_mu);
    Lp->cq_stop = true;
    Lp->cq_cv.notify_all();
  }
  for (auto& Lp : s->lanes)  // the completers see every tracked launch finish
    if (Lp && Lp->completer.joinable()) Lp->completer.join();
}

}  // namespace srv
}  // namespace bpsr

using namespace bpsr;

extern "C" {

int byteps_server_config_from_env(byteps_server_config* cfg) {
  if (!cfg) return fail(BYTEPS_REDUCE_EARGS, "null config");
  cfg->num_workers = getenv("DMLC_NUM_WORKER") ? atoi(getenv("DMLC_NUM_WORKER")) : 1;
  cfg->engine_lanes = getenv("BYTEPS_SERVER_ENGINE_THREAD")
                          ? atoi(getenv("BYTEPS_SERVER_ENGINE_THREAD")) : 4;
  const char* a = getenv("BYTEPS_ENABLE_ASYNC");
  cfg->async_mode = (a && atoi(a) != 0) ? 1 : 0;
  const char* p = getenv("BPSR_SERVER_POLICY");
  cfg->policy = (p && std::string(p) == "incremental") ? BYTEPS_SERVER_INCREMENTAL
                                                       : BYTEPS_SERVER_FUSED;
  cfg->device = 0;
  const char* sc = getenv("BYTEPS_SERVER_ENABLE_SCHEDULE");  // server.cc:335
  cfg->enable_schedule = (sc && atoi(sc) != 0) ? 1 : 0;
  const char* eb = getenv("BYTEPS_SERVER_ENGINE_BLOCKING");  // server.cc:324
  cfg->engine_blocking = (eb && atoi(eb) != 0) ? 1 : 0;
  // the dedicated server process: nothing else waits on its GPU, and a server
  // whose rounds are copied (ps-lite's host buffers) never runs a consumer
  // (server.h)
  cfg->release = BYTEPS_SERVER_RELEASE_DEVICE;
  return BYTEPS_REDUCE_OK;
}

int byteps_server_create_sized(const byteps_server_config* cfg, size_t cfg_size,
                               byteps_server** out) {
  if (!cfg || !out) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  *out = nullptr;
  constexpr size_t kV3 = offsetof(byteps_server_config, release);  // ABI 3: no release
  if (cfg_size != kV3 && cfg_size != sizeof(byteps_server_config))
    return fail(BYTEPS_REDUCE_EARGS,
                "byteps_server_config of %zu bytes: not a known version (%zu: ABI 3, %zu: ABI 4-5)",
                cfg_size, kV3, sizeof(byteps_server_config));
  byteps_server_config c{};  // fields past the caller's version keep their defaults
  c.release = BYTEPS_SERVER_RELEASE_LAUNCH;
  std::memcpy(&c, cfg, cfg_size);
  return byteps_server_create(&c, out);
}

int byteps_server_create(const byteps_server_config* cfg, byteps_server** out) {
  if (!cfg || !out) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  *out = nullptr;
  if (cfg->num_workers < 1) return fail(BYTEPS_REDUCE_EARGS, "num_workers must be >= 1");
  if (cfg->engine_lanes < 1)  // server.cc:332 CHECK_GE(engine_thread_num_, 1)
    return fail(BYTEPS_REDUCE_EARGS, "engine_lanes must be >= 1");
  if (cfg->policy != BYTEPS_SERVER_FUSED && cfg->policy != BYTEPS_SERVER_INCREMENTAL)
    return fail(BYTEPS_REDUCE_EARGS, "unknown policy %d", cfg->policy);
  auto s = std::make_unique<byteps_server>();
  s->cfg = *cfg;
  s->schedule = cfg->enable_schedule != 0;
  s->blocking = cfg->engine_blocking != 0;
  if (const char* fa = getenv("BPSR_SERVER_FAIL_AFTER")) s->fail_after = atol(fa);
  if (const char* cb = getenv("BPSR_SERVER_COMBINE")) s->combine = atoi(cb) != 0;
  if (s->schedule || s->blocking) s->combine = false;
  if (cfg->release != BYTEPS_SERVER_RELEASE_LAUNCH && cfg->release != BYTEPS_SERVER_RELEASE_DEVICE)
    return fail(BYTEPS_REDUCE_EARGS, "unknown release %d", cfg->release);
  s->dev_release = cfg->release == BYTEPS_SERVER_RELEASE_DEVICE;
  if (const char* r = getenv("BPSR_SERVER_RELEASE")) {  // overrides the config either way
    if (std::string(r) == "device") s->dev_release = true;
    else if (std::string(r) == "launch") s->dev_release = false;
  }
  if (const char* ps = getenv("BPSR_SERVER_PULL_SERVICE")) s->pull_service = atoi(ps) != 0;
  if (const char* t = getenv("BPSR_SERVER_RELEASE_TIMEOUT_S"))
    if (atof(t) > 0) s->kq_timeout_s = atof(t);
  // device releases: the fused left fold of a sync round, through the lane
  // issuers, at most kKeyedMaxSrcs workers (the release word's arrival order)
  if (!s->combine || cfg->async_mode || cfg->policy != BYTEPS_SERVER_FUSED ||
      cfg->num_workers > kKeyedMaxSrcs)
    s->dev_release = false;
  int rc = force_device(s.get());
  if (rc) return rc;
  s->acc_load.assign(cfg->engine_lanes, 0);
  for (int i = 0; i < cfg->engine_lanes; ++i) {
    s->lanes.push_back(std::make_unique<Lane>());
    Lane& L = *s->lanes.back();
    hipError_t e = hipStreamCreateWithFlags(&L.fold, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&L.copy, hipStreamNonBlocking);
    // d2h streams (mirror copies, copying pulls): normal priority (a
    // high-priority queue of their own measured no gain)
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&L.d2h, hipStreamNonBlocking);
    if (e == hipSuccess && s->schedule)
      e = hipEventCreateWithFlags(&L.job_done, hipEventDisableTiming);
    if (e != hipSuccess) {
      byteps_server_destroy(s.release());
      return hip_fail(e, "hipStreamCreate");
    }
    if (s->schedule) L.q = std::make_unique<EngineQueue<FoldJob>>(true);
    // the lane's batches are read in place up to 4 MiB: a table copy would
    // wait on the host behind the lane's queued work
    L.ring = stage_ring_create(4u << 20);
    for (hipEvent_t* m : {&L.copy_mark, &L.fold_mark, &L.d2h_mark})
      if (e == hipSuccess) e = hipEventCreateWithFlags(m, hipEventDisableTiming);

    // recorded once on their (empty) streams: waiting on them is a no-op until
    // the lane issues work
    if (e == hipSuccess) e = hipEventRecord(L.copy_mark, L.copy);
    if (e == hipSuccess) e = hipEventRecord(L.fold_mark, L.fold);
    if (e == hipSuccess) e = hipEventRecord(L.d2h_mark, L.d2h);
    if (e != hipSuccess) {
      byteps_server_destroy(s.release());
      return hip_fail(e, "lane events");
    }
  }
  try {
    if (s->schedule)
      for (int i = 0; i < cfg->engine_lanes; ++i)
        s->lanes[i]->dispatcher = std::thread(dispatcher_main, s.get(), i);
    if (s->dev_release) {
      s->klane = std::make_unique<Lane>();
      s->klane->completer = std::thread(completer_main, s.get(), s->klane.get());
    }
    if (s->combine)
      for (int i = 0; i < cfg->engine_lanes; ++i) {
        s->lanes[i]->completer = std::thread(completer_main, s.get(), s->lanes[i].get());
        s->lanes[i]->issuer = std::thread(issuer_main, s.get(), i);
      }
    s->responder = std::thread(responder_main, s.get());
  } catch (...) {
    byteps_server_destroy(s.release());
    return fail(BYTEPS_REDUCE_EARGS, "cannot start the server's threads");
  }
  *out = s.release();
  return BYTEPS_REDUCE_OK;
}

int byteps_server_destroy(byteps_server* s) {
  if (!s) return BYTEPS_REDUCE_OK;
  (void)hipSetDevice(s->cfg.device);
  destroy_lanes(s);  // queued jobs are issued first (the dispatchers drain)
  if (s->klane) {    // the keyed consumers complete (or time out) and settle their epochs
    s->kq_stopping.store(true, std::memory_order_release);  // an idle epoch retires at once
    {
      std::lock_guard<std::mutex> g(s->klane->done_mu);
      s->klane->cq_stop = true;
      s->klane->cq_cv.notify_all();
    }
    if (s->klane->completer.joinable()) s->klane->completer.join();
    std::vector<PullJob> parked;
    {
      std::lock_guard<std::mutex> g(s->kq_park_mu);
      parked.swap(s->kq_parked);
    }
    for (PullJob& j : parked) {  // pulls of epochs that never completed: cancelled
      if (j.direct) {
        j.direct->finish(BYTEPS_REDUCE_ECANCELED);
      } else {
        j.resp.status = BYTEPS_REDUCE_ECANCELED;
        enqueue_response(s, j.resp);
      }
    }
  }
  if (s->responder.joinable()) {
    for (auto& kv : s->keys) {  // pulls whose round never finished: cancelled
      KeyState* ks = kv.second.get();
      std::lock_guard<std::mutex> g(ks->mu);
      for (auto& wp : ks->waiting)
        respond_later(s, ks, wp.cb, wp.ctx, nullptr, BYTEPS_REDUCE_ECANCELED);
      ks->waiting.clear();
      for (auto& wc : ks->waiting_copies) {
        if (wc.direct) wc.direct->finish(BYTEPS_REDUCE_ECANCELED);
        else respond_later(s, ks, wc.cb, wc.ctx, nullptr, BYTEPS_REDUCE_ECANCELED);
      }
      ks->waiting_copies.clear();
      for (auto& a : ks->init_acks) {  // init pushes whose round never completed
        a.status = BYTEPS_REDUCE_ECANCELED;
        enqueue_response(s, a);
      }
      ks->init_acks.clear();
    }
    {
      std::lock_guard<std::mutex> g(s->rq_mu);
      s->rq_stop = true;
    }
    s->rq_cv.notify_all();
    s->responder.join();
  }
  for (auto& Lp : s->lanes) {
    if (Lp->fold) (void)hipStreamSynchronize(Lp->fold);
    if (Lp->copy) (void)hipStreamSynchronize(Lp->copy);
    if (Lp->d2h) (void)hipStreamSynchronize(Lp->d2h);
  }
  for (auto& kv : s->keys) {
    KeyState* ks = kv.second.get();
    if (ks->done) (void)hipEventDestroy(ks->done);
    if (ks->copied) (void)hipEventDestroy(ks->copied);
    if (ks->pulled) (void)hipEventDestroy(ks->pulled);
    if (ks->mirrored) (void)hipEventDestroy(ks->mirrored);
    for (char* m : ks->mirror) (void)hipHostFree(m);
    if (ks->arena) (void)hipFree(ks->arena);
  }
  if (s->kq) (void)byteps_reduce_blockq_destroy(s->kq);
  copysvc_destroy(s->svc);
  for (hipEvent_t e : s->ev_pool) (void)hipEventDestroy(e);
  if (s->gate_ev) (void)hipEventDestroy(s->gate_ev);
  if (s->gate_stream) (void)hipStreamDestroy(s->gate_stream);
  for (hipEvent_t e : s->kq_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& Lp : s->lanes) {
    if (Lp->fold) (void)hipStreamDestroy(Lp->fold);
    if (Lp->copy) (void)hipStreamDestroy(Lp->copy);
    if (Lp->d2h) (void)hipStreamDestroy(Lp->d2h);
    if (Lp->job_done) (void)hipEventDestroy(Lp->job_done);
    if (Lp->ring) stage_ring_destroy(Lp->ring);
    for (hipEvent_t m : {Lp->copy_mark, Lp->fold_mark, Lp->d2h_mark})
      if (m) (void)hipEventDestroy(m);

  }
  delete s;
  return BYTEPS_REDUCE_OK;
}

int byteps_server_init_key(byteps_server* s, uint64_t key, size_t len, int dtype) {
  if (!s) return fail(BYTEPS_REDUCE_EARGS, "null server");
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = get_key(s, key, true);
  std::lock_guard<std::mutex> g(ks->mu);
  return allocate(s, ks, len, dtype);
}

}  // extern "C"

extern "C" {

int byteps_server_push(byteps_server* s, uint64_t key, int worker, const void* data, size_t len,
                       int dtype, int location) {
  if (!s || !data) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (worker < 0 || worker >= s->cfg.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker, s->cfg.num_workers);
  if (const void* src = service_src(s, data, len, location)) {
    int rc = set_device(s);
    if (rc) return rc;
    if (CopyService* svc = service_get(s)) return service_push(s, svc, key, worker, src, len, dtype);
  }
  if (location == BYTEPS_SERVER_DEVICE && s->combine && !t_responder) {
    // device data: the copy goes through the lane issuer (batched with the
    // other pushes that piled up) and the push returns once it has landed;
    // an issuer-batched copy reports here directly and this thread waits for
    // the launch to complete (no responder hop), other arrivals answer
    // through the callback as a non-blocking push would
    SyncWait w;
    int rc = push_async_impl(s, key, worker, data, len, dtype, location, sync_push_cb, &w, &w);
    if (rc) return rc;
    if ((rc = w.wait())) return sync_status(s, key, rc, "push");
    if (w.lane) wait_lane_done(*w.lane, w.seq);
    return BYTEPS_REDUCE_OK;
  }
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = get_key(s, key, true);
  std::unique_lock<std::mutex> lk(ks->mu);
  if ((rc = allocate(s, ks, len, dtype))) return rc;
  // A worker's next push may arrive while its previous one (of this round, or
  // its init push) is not folded yet: hold it until the slot is free.
  ks->cv.wait(lk, [&] { return can_push(s, ks, worker); });
  if (ks->error) return key_error(ks);
  if ((rc = copy_in(s, ks, worker, data, len, location, /*wait=*/false))) return rc;
  // The caller's buffer goes back once its copy has landed, waited for with
  // the key's lock released: the copy stream can sit behind a lane fold that
  // waits for a keyed epoch, and that epoch's close may need this lock to
  // skip the key (DESIGN.md §9.x "slot reuse after a device release").  The
  // round's fold is ordered behind the copy on the device, so the arrival
  // need not wait for it.  (A later copy of the key re-records the event on
  // the same in-order stream: waiting for it covers this one.)
  const hipEvent_t copied = ks->copied;
  auto landed = [&](int r) {
    if (lk.owns_lock()) lk.unlock();
    const hipError_t e = hipEventSynchronize(copied);
    return r ? r : (e == hipSuccess ? 0 : hip_fail(e, "push copy"));
  };
  thread_local std::vector<FoldJob> defer;  // keeps its capacity: no allocation per call
  defer.clear();
  if ((rc = arrive_and_wait_init(s, ks, worker, lk, s->combine ? &defer : nullptr))) return landed(rc);
  if (!defer.empty()) {
    lk.unlock();
    if (issue_combined(s, defer) && (rc = own_key_status(ks))) return landed(rc);
    lk.lock();
  }
  return landed(s->blocking ? finish_blocking(s, ks, lk) : 0);
}

int byteps_server_push_async(byteps_server* s, uint64_t key, int worker, const void* data,
                             size_t len, int dtype, int location, byteps_server_push_cb cb,
                             void* ctx) {
  return push_async_impl(s, key, worker, data, len, dtype, location, cb, ctx, nullptr);
}

}  // extern "C"

namespace bpsr {
inline namespace srv {
// byteps_server_push_async; with `direct`, a blocking push's issuer-batched
// copy reports to its waiter instead of the responder (cb/ctx serve the
// other paths, answered through the responder as for any non-blocking push).
int push_async_impl(byteps_server* s, uint64_t key, int worker, const void* data, size_t len,
                    int dtype, int location, byteps_server_push_cb cb, void* ctx,
                    SyncWait* direct, int pos) {
  if (!s || !data || !cb) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (worker < 0 || worker >= s->cfg.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker, s->cfg.num_workers);
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = get_key(s, key, true);
  std::unique_lock<std::mutex> lk(ks->mu);
  if ((rc = allocate(s, ks, len, dtype))) return rc;
  ks->cv.wait(lk, [&] { return can_push(s, ks, worker); });
  if (ks->error) return key_error(ks);
  if ((rc = check_pos(s, ks, pos))) return rc;  // before any copy is queued
  if (s->combine && location == BYTEPS_SERVER_DEVICE && ks->inited && !s->cfg.async_mode &&
      s->cfg.policy == BYTEPS_SERVER_FUSED && s->cfg.num_workers <= kMaxSrcs) {
    // the copy goes to the lane's issuer, batched with the other pushes that
    // piled up, ahead of the fold this arrival may complete (also the
    // issuer's, after the copies); acknowledged once the copy has completed
    CopyJob cj;
    cj.ks = ks;
    cj.w = worker;
    cj.src = data;
    cj.len = len;
    cj.ack.key = key;
    cj.ack.ks = ks;
    cj.ack.ctx = ctx;
    cj.ack.push_cb = cb;
    cj.ack.worker = worker;
    cj.direct = direct;
    ks->round_copied = true;
    ks->round_mark_copy = true;
    {
      Lane& L = *s->lanes[ks->lane];
      std::lock_guard<std::mutex> g(L.comb_mu);
      L.copies.push_back(cj);
      L.comb_cv.notify_one();
    }
    std::vector<FoldJob> defer;
    // cannot fail here: no error (checked under this lock), the slot is free
    // (can_push), and the fused policy defers the round's fold
    if ((rc = arrive(s, ks, worker, &defer, pos))) return rc;
    if (!defer.empty()) {
      lk.unlock();
      issue_combined(s, defer);
    }
    return BYTEPS_REDUCE_OK;
  }
  if ((rc = copy_in(s, ks, worker, data, len, location, /*wait=*/false))) return rc;
  const bool init_push = !ks->inited;
  std::vector<FoldJob> defer;
  if ((rc = arrive(s, ks, worker, s->combine ? &defer : nullptr, pos))) {  // arrival order = call order
    // the caller gets its buffer back on error: let the queued copy finish first
    (void)hipEventSynchronize(ks->copied);
    return rc;
  }
  Response r;
  r.key = key;
  r.ks = ks;
  r.ctx = ctx;
  r.push_cb = cb;
  r.worker = worker;
  if (init_push && !ks->inited) {
    // server.cc:184-185: an init push is answered only once all NumWorkers
    // init pushes are in (workers use it as a barrier, operations.cc:301-302)
    ks->init_acks.push_back(r);
    return BYTEPS_REDUCE_OK;
  }
  enqueue_response(s, r);
  if (!defer.empty()) {
    lk.unlock();
    if (issue_combined(s, defer)) return own_key_status(ks);
  }
  return BYTEPS_REDUCE_OK;
}
}  // namespace srv
}  // namespace bpsr

extern "C" {

int byteps_server_recv_slot(byteps_server* s, uint64_t key, int worker, void** slot) {
  if (!s || !slot) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (worker < 0 || worker >= s->cfg.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker, s->cfg.num_workers);
  KeyState* ks = get_key(s, key, false);
  if (!ks || !ks->allocated)
    return fail(BYTEPS_REDUCE_EARGS, "key %llu not initialised (byteps_server_init_key)",
                (unsigned long long)key);
  std::unique_lock<std::mutex> lk(ks->mu);
  ks->cv.wait(lk, [&] { return ks->pending == 0 || ks->error; });  // every fold issued
  if (ks->error) return key_error(ks);
  if (ks->has_done && !wait_keyed_slots(s, ks)) {  // the slot may be read by the last issued fold
    hipError_t e = hipEventSynchronize(ks->fold_ev);
    if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
  }
  *slot = ks->slot[worker];
  return BYTEPS_REDUCE_OK;
}

int byteps_server_push_ready(byteps_server* s, uint64_t key, int worker) {
  if (!s) return fail(BYTEPS_REDUCE_EARGS, "null server");
  if (worker < 0 || worker >= s->cfg.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker, s->cfg.num_workers);
  int rc = bind_cached(s);
  if (rc) return rc;
  KeyState* ks = get_key(s, key, false);
  if (!ks || !ks->allocated) return fail(BYTEPS_REDUCE_EARGS, "key not initialised");
  // the producers named with byteps_server_order_after, before the key lock:
  // a round released from the host waits for them, and that wait must not
  // hold the key's other workers and its completer (arrive()
  // then finds the gate passed)
  if ((rc = wait_order_gate(s))) return rc;
  std::unique_lock<std::mutex> lk(ks->mu);
  ks->cv.wait(lk, [&] { return can_push(s, ks, worker); });
  thread_local std::vector<FoldJob> defer;  // keeps its capacity: no allocation per call
  defer.clear();
  if ((rc = arrive_and_wait_init(s, ks, worker, lk, s->combine ? &defer : nullptr))) return rc;
  if (!defer.empty()) {
    lk.unlock();
    if (issue_combined(s, defer) && (rc = own_key_status(ks))) return rc;
    lk.lock();
  }
  return s->blocking ? finish_blocking(s, ks, lk) : 0;
}

int byteps_server_pull(byteps_server* s, uint64_t key, void* out, size_t len, int location) {
  if (!s || !out) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (location == BYTEPS_SERVER_DEVICE && s->combine && !s->cfg.async_mode && !t_responder) {
    // into device memory: one of the lane issuer's batched pull copies; this
    // thread waits for the launch to complete and counts the pull
    // (server.cc:105-113) itself — no HIP call here, no responder hop
    int rc = set_device(s);
    if (rc) return rc;
    KeyState* ks = key_for_pull(s, key);
    if (!ks) return BYTEPS_REDUCE_EARGS;
    if (CopyService* svc = service_for(s, out, len)) return service_pull(s, svc, ks, out, len);
    std::unique_lock<std::mutex> lk(ks->mu);
    if (len > ks->len) return fail(BYTEPS_REDUCE_EARGS, "pull of %zu bytes > key len %zu", len, ks->len);
    if (ks->error) return key_error(ks);
    SyncWait w;
    const KeyState::WaitingCopy wc{out, len, nullptr, nullptr, out, &w};
    if (pull_ready(s, ks))
      queue_pull_copies(s, ks, &wc, 1);
    else  // parked: queued with the round's other parked pulls when it finishes
      ks->waiting_copies.push_back(wc);
    lk.unlock();
    if ((rc = w.wait())) return sync_status(s, key, rc, "pull");
    wait_lane_done(*w.lane, w.seq);
    lk.lock();
    count_pull(s, ks);  // as the old path: after the copy has completed
    return BYTEPS_REDUCE_OK;
  }
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = key_for_pull(s, key);
  if (!ks) return BYTEPS_REDUCE_EARGS;
  std::unique_lock<std::mutex> lk(ks->mu);
  if (len > ks->len) return fail(BYTEPS_REDUCE_EARGS, "pull of %zu bytes > key len %zu", len, ks->len);
  if (!s->cfg.async_mode) ks->cv.wait(lk, [&] { return pull_ready(s, ks); });
  if (ks->error) return key_error(ks);
  if (ks->keyed) {  // its epoch published first
    const uint64_t need = ks->fold_seq;
    lk.unlock();
    wait_published(s, ks, need);
    lk.lock();
    if (ks->error) return key_error(ks);
  }
  s->n_pulls.add();
  s->n_pull_launches.fetch_add(1, std::memory_order_relaxed);
  // The copy runs on the lane's d2h stream behind the key's last issued fold,
  // queued under the key lock (the copy kernel into pinned host memory,
  // pull_kernel_dst; hipMemcpyAsync otherwise).  No per-thread
  // streams: a transport's pull threads come and go, and a stream per thread
  // (round 1) cost a stream creation per new thread and multiplied the
  // streams sharing the process's few hardware queues.
  Lane& L = *s->lanes[ks->lane];
  hipError_t e = ks->has_done ? hipStreamWaitEvent(L.d2h, ks->fold_ev, 0) : hipSuccess;
  if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent");
  void* dv = pull_kernel_dst(out, location);
  if (dv) {
    if ((rc = byteps_reduce_copy(dv, ks->store, len, L.d2h))) return rc;
  } else {
    e = hipMemcpyAsync(out, ks->store, len,
                       location == BYTEPS_SERVER_HOST ? hipMemcpyDeviceToHost
                                                      : hipMemcpyDeviceToDevice, L.d2h);
  }
  if (e == hipSuccess) e = hipEventRecord(ks->pulled, L.d2h);
  // Async mode keeps adding into the store: the lane's later folds wait for
  // this copy, so none lands mid-copy.  (Sync mode: the store cannot change
  // while the pull is outstanding — the next round needs this worker's next
  // push, which follows the pull.)
  if (e == hipSuccess && (s->cfg.async_mode || s->blocking))
    e = hipStreamWaitEvent(L.fold, ks->pulled, 0);
  if (e != hipSuccess) return hip_fail(e, "pull copy");
  hipEvent_t ev = ks->pulled;  // a later pull may re-record it: it then covers this copy too
  lk.unlock();
  e = hipEventSynchronize(ev);
  if (e != hipSuccess) return hip_fail(e, "pull copy");
  if (s->cfg.async_mode || s->blocking) return BYTEPS_REDUCE_OK;
  lk.lock();
  count_pull(s, ks);  // server.cc:105-113: after NumWorkers pulls the key re-arms
  return BYTEPS_REDUCE_OK;
}

int byteps_server_pull_host_view(byteps_server* s, uint64_t key, const void** data,
                                 size_t* len) {
  if (!s || !data) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  *data = nullptr;
  if (len) *len = 0;
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = key_for_pull(s, key);
  if (!ks) return BYTEPS_REDUCE_EARGS;
  std::unique_lock<std::mutex> lk(ks->mu);
  if (!s->cfg.async_mode) ks->cv.wait(lk, [&] { return pull_ready(s, ks); });
  if (ks->error) return key_error(ks);
  if (ks->keyed) {  // its epoch published first
    const uint64_t need = ks->fold_seq;
    lk.unlock();
    wait_published(s, ks, need);
    lk.lock();
    if (ks->error) return key_error(ks);
  }
  if ((rc = ensure_mirror(s, ks, !s->cfg.async_mode))) return rc;
  size_t idx = ks->rounds & 1;
  if (s->cfg.async_mode) {  // the store changes with every push: a fresh D2H per view
    idx = next_async_mirror(ks);
    if ((rc = queue_mirror(s, ks, idx))) return rc;
  }
  const char* view = ks->mirror[idx];
  hipEvent_t ev = ks->mirrored;
  lk.unlock();
  // The event still names this round's copy: the next round cannot finish
  // before this pull is counted below.
  hipError_t e = hipEventSynchronize(ev);
  if (e != hipSuccess) return hip_fail(e, "store mirror sync");
  lk.lock();
  count_pull(s, ks);
  *data = view;
  if (len) *len = ks->len;
  return BYTEPS_REDUCE_OK;
}

int byteps_server_pull_device_view(byteps_server* s, uint64_t key, const void** data,
                                   size_t* len) {
  if (!s || !data) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  *data = nullptr;
  if (len) *len = 0;
  if (s->cfg.async_mode)
    return fail(BYTEPS_REDUCE_EARGS, "device views need sync mode (async pushes rewrite the store)");
  int rc = bind_cached(s);
  if (rc) return rc;
  KeyState* ks = key_for_pull(s, key);
  if (!ks) return BYTEPS_REDUCE_EARGS;
  std::unique_lock<std::mutex> lk(ks->mu);
  ks->cv.wait(lk, [&] { return pull_ready(s, ks); });
  if (ks->error) return key_error(ks);
  // The round is published only after its fold (or the lane's batch mark
  // behind it) was recorded, so this event covers the store's last write.
  const bool has = ks->has_done;
  hipEvent_t ev = ks->fold_ev;
  const uint64_t need = ks->fold_seq;
  const int fl = ks->fold_lane;
  const void* view = ks->store;
  Lane* FL = need ? (fl < 0 ? s->klane.get() : s->lanes[fl].get()) : nullptr;
  const int kq_key = fl < 0 ? ks->kq_key.load() : -1;
  const uint32_t kq_epoch = ks->kq_round_epoch;
  // the fold completed already (published without a lock, or the key's own
  // completion word): answer at once
  if (!(FL && (FL->done_pub.load(std::memory_order_acquire) >= need ||
               (kq_key >= 0 && keyq_key_done(s->kq, kq_key, kq_epoch))))) {
    lk.unlock();
    if (FL) {  // tracked by a completer (the lane's, or the keyed one): no HIP call here
      wait_round_fold(s, *FL, need, kq_key, kq_epoch);
    } else if (has) {
      hipError_t e = hipEventSynchronize(ev);
      if (e != hipSuccess) return hip_fail(e, "store fold sync");
    }
    lk.lock();
  }
  if (ks->error) return key_error(ks);  // a keyed epoch that timed out
  s->n_pulls.add();
  count_pull(s, ks);  // server.cc:105-113: after NumWorkers pulls the key re-arms
  *data = view;
  if (len) *len = ks->len;
  return BYTEPS_REDUCE_OK;
}

int byteps_server_pull_async(byteps_server* s, uint64_t key, byteps_server_pull_cb cb,
                             void* ctx) {
  if (!s || !cb) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = key_for_pull(s, key);
  if (!ks) return BYTEPS_REDUCE_EARGS;
  std::lock_guard<std::mutex> g(ks->mu);
  if (ks->error) return key_error(ks);
  if (s->cfg.async_mode) {  // answered at once from a fresh copy of the store
    if ((rc = ensure_mirror(s, ks, false))) return rc;
    const size_t idx = next_async_mirror(ks);
    if ((rc = queue_mirror(s, ks, idx))) return rc;
    respond_later(s, ks, cb, ctx, ks->mirror[idx], 0);
    return BYTEPS_REDUCE_OK;
  }
  const bool now = s->blocking || ks->push_finished;
  if ((rc = ensure_mirror(s, ks, now))) return rc;
  if (now)  // server.cc:293-301: push already finished (blocking mode: always)
    respond_later(s, ks, cb, ctx, ks->mirror[ks->rounds & 1], 0);
  else                    // server.cc:303-304: queued until the round finishes
    ks->waiting.push_back({cb, ctx});
  return BYTEPS_REDUCE_OK;
}

int byteps_server_pull_into_async(byteps_server* s, uint64_t key, void* out, size_t len,
                                  int location, byteps_server_pull_cb cb, void* ctx) {
  if (!s || !out || !cb) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (s->cfg.async_mode || !s->combine)
    return fail(BYTEPS_REDUCE_EARGS, "pull_into_async needs sync mode and the default engine "
                                     "(no scheduling, no engine blocking, BPSR_SERVER_COMBINE!=0)");
  int rc = set_device(s);
  if (rc) return rc;
  // pinned host memory: the issuer's copy kernel writes it through its device
  // view (over PCIe); pageable memory is not addressable by the device
  void* dv = device_view(out, location);
  if (!dv)
    return fail(BYTEPS_REDUCE_EARGS, "pull_into_async: host destination is not pinned "
                                     "(host transports: byteps_server_pull_async views)");
  KeyState* ks = key_for_pull(s, key);
  if (!ks) return BYTEPS_REDUCE_EARGS;
  std::lock_guard<std::mutex> g(ks->mu);
  if (ks->error) return key_error(ks);
  if (len > ks->len) return fail(BYTEPS_REDUCE_EARGS, "pull of %zu bytes > key len %zu", len, ks->len);
  const KeyState::WaitingCopy wc{dv, len, cb, ctx, out, nullptr};
  if (ks->push_finished)  // server.cc:293-301: the round is finished
    queue_pull_copies(s, ks, &wc, 1);
  else                    // server.cc:303-304: answered once it finishes
    ks->waiting_copies.push_back(wc);
  return BYTEPS_REDUCE_OK;
}

int byteps_server_key_info(byteps_server* s, uint64_t key, uint64_t* rounds, int* lane,
                           int* last_order, int max_order) {
  if (!s) return fail(BYTEPS_REDUCE_EARGS, "null server");
  KeyState* ks = get_key(s, key, false);
  if (!ks) return fail(BYTEPS_REDUCE_EARGS, "unknown key");
  std::unique_lock<std::mutex> lk(ks->mu);
  ks->cv.wait(lk, [&] { return ks->pending == 0 || ks->error; });  // rounds handed to the issuer
  if (rounds) *rounds = ks->rounds;
  if (lane) *lane = ks->lane;
  if (last_order)
    for (int i = 0; i < max_order && i < (int)ks->last_order.size(); ++i)
      last_order[i] = ks->last_order[i];
  return ks->error ? key_error(ks) : BYTEPS_REDUCE_OK;
}

// ------------------------------------------------------- other calls --

int byteps_server_order_after(byteps_server* s, const uint64_t* keys, int n, void* event) {
  if (!s || !event || n < 0 || (n > 0 && !keys)) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  int rc = set_device(s);
  if (rc) return rc;
  // the lanes of the named keys (every lane when a key is not allocated yet:
  // its lane is picked at its first push)
  std::vector<char> on(s->lanes.size(), n == 0 ? 1 : 0);
  for (int i = 0; i < n; ++i) {
    KeyState* ks = get_key(s, keys[i], false);
    if (!ks || !ks->allocated) {
      std::fill(on.begin(), on.end(), 1);
      break;
    }
    on[ks->lane] = 1;
  }
  const hipEvent_t ev = static_cast<hipEvent_t>(event);
  for (size_t l = 0; l < on.size(); ++l) {
    if (!on[l]) continue;
    Lane& L = *s->lanes[l];
    // push copies (and the issuer's), pull copies and mirrors, and the folds
    // of push_ready rounds whose slots the caller wrote on its own stream
    // (device releases: the gate below, waited for before a host release)
    for (hipStream_t st : {L.copy, L.d2h, L.fold}) {
      const hipError_t e = hipStreamWaitEvent(st, ev, 0);
      if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent(caller event)");
    }
  }
  // the gate of the work no stream of ours orders: the copy service's copies
  // and device releases stored from the host
  if ((s->pull_service || s->dev_release) && s->combine && !s->cfg.async_mode) {
    std::lock_guard<std::mutex> g(s->gate_mu);
    if (!s->gate_stream && (rc = force_device(s))) return rc;
    hipError_t e = hipSuccess;
    if (!s->gate_stream) e = hipStreamCreateWithFlags(&s->gate_stream, hipStreamNonBlocking);
    if (e == hipSuccess && !s->gate_ev) e = hipEventCreateWithFlags(&s->gate_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamWaitEvent(s->gate_stream, ev, 0);
    if (e == hipSuccess) e = hipEventRecord(s->gate_ev, s->gate_stream);
    if (e != hipSuccess) return hip_fail(e, "order_after gate");
    s->gate_seq.fetch_add(1, std::memory_order_release);
  }
  return BYTEPS_REDUCE_OK;
}

int byteps_server_stats(byteps_server* s, uint64_t* out, int n) {
  if (!s || (n > 0 && !out) || n < 0) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  uint64_t svc_launches = 0;
  {
    std::lock_guard<std::mutex> g(s->svc_mu);
    svc_launches = bpsr::copysvc_launches(s->svc);
  }
  const uint64_t v[14] = {s->n_fold_launches.load(), s->n_rounds_folded.load(),
                          s->n_pull_launches.load(), s->n_pulls.load(), s->issuer_ns.load(),
                          s->n_copy_launches.load(), s->n_consumer_launches.load(),
                          s->n_key_releases.load(), s->n_service_pulls.load(), svc_launches,
                          s->n_service_pushes.load(), s->n_consumer_retired.load(),
                          s->n_epochs_closed.load(), s->n_lane_epochs.load()};
  for (int i = 0; i < n && i < 14; ++i) out[i] = v[i];
  return BYTEPS_REDUCE_OK;
}

int byteps_server_debug_lane(byteps_server* s, int lane, int pause, uint64_t* log_keys,
                             int max_log, int* n_log) {
  if (!s) return fail(BYTEPS_REDUCE_EARGS, "null server");
  if (lane < 0 || lane >= (int)s->lanes.size())
    return fail(BYTEPS_REDUCE_EARGS, "lane %d outside [0, %zu)", lane, s->lanes.size());
  Lane& L = *s->lanes[lane];
  if (pause >= 0) {
    if (!L.q) return fail(BYTEPS_REDUCE_EARGS, "lane pause needs enable_schedule (no dispatcher)");
    L.q->hold(pause > 0);
  }
  std::lock_guard<std::mutex> g(L.dbg_mu);
  if (n_log) *n_log = (int)L.log.size();
  if (log_keys)
    for (int i = 0; i < max_log && i < (int)L.log.size(); ++i) log_keys[i] = L.log[i];
  return BYTEPS_REDUCE_OK;
}

}  // extern "C"

// ------------------------------------------- server group internals --
// (bpsr_server_internal.h: not part of the C ABI)

namespace bpsr {

int server_push_async_at(byteps_server* s, uint64_t key, int worker, const void* data,
                         size_t len, int dtype, int location, byteps_server_push_cb cb, void* ctx,
                         int pos) {
  return push_async_impl(s, key, worker, data, len, dtype, location, cb, ctx, nullptr, pos);
}

int server_check_key(byteps_server* s, uint64_t key, size_t len, int dtype) {
  if (!s) return fail(BYTEPS_REDUCE_EARGS, "null server");
  if (elem_size(dtype) == 0) return fail(BYTEPS_REDUCE_EDTYPE, "Unsupported data type: %d", dtype);
  if (len == 0) return fail(BYTEPS_REDUCE_EARGS, "init tensor size not larger than 0");
  KeyState* ks = get_key(s, key, false);
  if (!ks) return 0;
  std::lock_guard<std::mutex> g(ks->mu);
  if (ks->error) return key_error(ks);
  if (ks->allocated && (len != ks->len || dtype != ks->dtype))
    return fail(BYTEPS_REDUCE_EARGS, "key %llu pushed with len %zu dtype %d (declared %zu, %d)",
                (unsigned long long)key, len, dtype, ks->len, ks->dtype);
  return 0;
}

void server_fail_key(byteps_server* s, uint64_t key, int rc) {
  KeyState* ks = get_key(s, key, true);
  std::lock_guard<std::mutex> g(ks->mu);
  fail_key(s, ks, rc);
}

bool server_pulls_async(const byteps_server* s) { return s->combine && !s->cfg.async_mode; }

bool server_key_inited(byteps_server* s, uint64_t key) {
  KeyState* ks = get_key(s, key, false);
  if (!ks) return false;
  std::lock_guard<std::mutex> g(ks->mu);
  return ks->inited;
}

}  // namespace bpsr

