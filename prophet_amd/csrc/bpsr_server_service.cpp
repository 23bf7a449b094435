// GPU-resident PS server: lane waits of blocking calls, and blocking device
// pulls and pushes through the pull copy service (bpsr_copy_service.cpp), with
// order_after's gate (bpsr_server_state.h).
#include "bpsr_server_state.h"

namespace bpsr {
inline namespace srv {
// A blocking call's wait for the lane's launch `seq` to complete.
void wait_lane_done(Lane& L, uint64_t seq) {
  std::unique_lock<std::mutex> dl(L.done_mu);
  L.done_cv.wait(dl, [&] { return L.done_seq >= seq; });
}
// Wait for a round's fold, read from the key's state under its lock (fold_seq
// / fold_lane / kq_round_epoch).  A keyed round is readable as soon as its
// key's completion word says so (the consumer may still be folding other
// keys): poll that word and the keyed completer's progress for up to
// kKeyedSpinUs, then sleep until the completer publishes the epoch (which
// also settles a consumer that gave up).
constexpr int kKeyedSpinUs = 200;
void wait_round_fold(byteps_server* s, Lane& FL, uint64_t need, int kq_key, uint32_t kq_epoch) {
  if (FL.done_pub.load(std::memory_order_acquire) >= need) return;
  if (kq_key >= 0 && kq_epoch) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      for (int i = 0; i < 32; ++i) {
        if (keyq_key_done(s->kq, kq_key, kq_epoch)) return;
        if (FL.done_pub.load(std::memory_order_acquire) >= need) return;
        __builtin_ia32_pause();
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kKeyedSpinUs)) break;
    }
  }
  wait_lane_done(FL, need);
}
// The pull copy service for a blocking pull of `len` bytes into `out`, when
// `out` is this device's memory (the service's release covers this device
// only) and the pull is small enough that a lane copy's launch cost matters.
constexpr size_t kServiceMaxPull = 16u << 20;
CopyService* service_get(byteps_server* s) {
  std::lock_guard<std::mutex> g(s->svc_mu);
  if (!s->svc && !s->svc_tried) {
    s->svc_tried = true;
    if (force_device(s) || copysvc_create(s->cfg.device, &s->svc)) s->svc = nullptr;  // lane copies then
  }
  // a service that gave up (a job not served in time) takes no more pulls:
  // they ride lane copies, as with BPSR_SERVER_PULL_SERVICE=0
  return s->svc && !copysvc_broken(s->svc) && !copysvc_wedged(s->svc) ? s->svc : nullptr;
}
bool on_this_device(const byteps_server* s, const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice && a.device == s->cfg.device;
}
CopyService* service_for(byteps_server* s, void* out, size_t len) {
  if (!s->pull_service || len == 0 || len > kServiceMaxPull) return nullptr;
  if (!on_this_device(s, out)) return nullptr;
  return service_get(s);
}
// A blocking push's source for the service's copiers: this device's memory;
// nullptr when the push takes the lane path.  Host sources stay on the lane
// path: the copiers reading pinned host memory over PCIe made config 1's
// host-resident rounds slower than the lanes' SDMA copies (r04s35: 28 vs 31.6
// GiB/s with views, 23 vs 30.6 with copying pulls).
const void* service_src(byteps_server* s, const void* data, size_t len, int location) {
  if (!s->pull_service || !s->combine || s->cfg.async_mode || t_responder || len == 0 ||
      len > kServiceMaxPull || location != BYTEPS_SERVER_DEVICE)
    return nullptr;
  return on_this_device(s, data) ? data : nullptr;
}
// A service copy that failed because the service gave up (a job not served
// in time): the same bytes through the key lane's d2h stream instead, so the
// call still completes (later calls take the lanes: service_get).
int fallback_copy(byteps_server* s, KeyState* ks, void* dst, const void* src, size_t len) {
  Lane& L = *s->lanes[ks->lane];
  hipError_t e = hipMemcpyAsync(dst, src, len, hipMemcpyDeviceToDevice, L.d2h);
  if (e == hipSuccess) e = hipStreamSynchronize(L.d2h);
  return e == hipSuccess ? 0 : hip_fail(e, "copy (after the copy service gave up)");
}
// The events given to byteps_server_order_after so far, waited for on the
// host before a service copy (the service copies on no stream of ours).
int wait_order_gate(byteps_server* s) {
  const uint64_t gseq = s->gate_seq.load(std::memory_order_acquire);
  if (gseq <= s->gate_done.load(std::memory_order_acquire)) return 0;
  hipEvent_t gev;
  {
    std::lock_guard<std::mutex> g(s->gate_mu);
    gev = s->gate_ev;
  }
  // the event's latest record covers every gate recorded up to gseq
  hipError_t e = hipEventSynchronize(gev);
  if (e != hipSuccess) return hip_fail(e, "order_after gate sync");
  uint64_t d = s->gate_done.load(std::memory_order_relaxed);
  while (d < gseq && !s->gate_done.compare_exchange_weak(d, gseq)) {
  }
  return 0;
}
// A blocking pull through the copy service: wait for the round's fold as a
// device view does (its completer's published sequence, no HIP call), then
// one service copy; count the pull after the copy, as the lane path does.
// Sync mode keeps the store still meanwhile: the next round needs this
// worker's next push, which follows this pull.
int service_pull(byteps_server* s, CopyService* svc, KeyState* ks, void* out, size_t len) {
  std::unique_lock<std::mutex> lk(ks->mu);
  if (len > ks->len) return fail(BYTEPS_REDUCE_EARGS, "pull of %zu bytes > key len %zu", len, ks->len);
  ks->cv.wait(lk, [&] { return pull_ready(s, ks); });
  if (ks->error) return key_error(ks);
  const bool has = ks->has_done;
  hipEvent_t ev = ks->fold_ev;
  const uint64_t need = ks->fold_seq;
  const int fl = ks->fold_lane;
  const void* store = ks->store;
  const int kq_key = fl < 0 ? ks->kq_key.load() : -1;
  const uint32_t kq_epoch = ks->kq_round_epoch;
  lk.unlock();
  if (need) {
    wait_round_fold(s, fl < 0 ? *s->klane : *s->lanes[fl], need, kq_key, kq_epoch);
  } else if (has) {
    hipError_t e = hipEventSynchronize(ev);
    if (e != hipSuccess) return hip_fail(e, "store fold sync");
  }
  lk.lock();
  if (ks->error) return key_error(ks);  // a keyed epoch that timed out
  lk.unlock();
  if (int rc = wait_order_gate(s)) return rc;
  int rc = copysvc_copy(svc, out, store, len);
  if (rc && copysvc_broken(svc)) rc = fallback_copy(s, ks, out, store, len);
  else if (!rc) s->n_service_pulls.fetch_add(1, std::memory_order_relaxed);
  if (rc) return rc;
  s->n_pulls.add();
  lk.lock();
  count_pull(s, ks);
  return BYTEPS_REDUCE_OK;
}
// A blocking push through the copy service: once the slot is free (the key's
// previous fold has completed — the same rule as the lane copy's stream wait),
// the service copies the data into the worker's slot with no key lock held
// and no HIP call; then the push arrives as if the transport had written the
// slot itself (a push_ready: the round needs no copy ordering, and a device
// release can be a host store).
int service_push(byteps_server* s, CopyService* svc, uint64_t key, int worker, const void* src,
                 size_t len, int dtype) {
  KeyState* ks = get_key(s, key, true);
  std::unique_lock<std::mutex> lk(ks->mu);
  int rc = allocate(s, ks, len, dtype);
  if (rc) return rc;
  ks->cv.wait(lk, [&] { return can_push(s, ks, worker); });
  if (ks->error) return key_error(ks);
  if (ks->has_done) {
    const bool keyed = ks->fold_lane < 0;
    const uint64_t need = ks->fold_seq;
    const int fl = ks->fold_lane;
    const int kq_key = keyed ? ks->kq_key.load() : -1;
    const uint32_t kq_epoch = ks->kq_round_epoch;
    hipEvent_t ev = ks->fold_ev;
    lk.unlock();
    if (need) {
      wait_round_fold(s, keyed ? *s->klane : *s->lanes[fl], need, kq_key, kq_epoch);
    } else {
      const hipError_t e = hipEventSynchronize(ev);
      if (e != hipSuccess) return hip_fail(e, "slot's last fold");
    }
    lk.lock();
    if (ks->error) return key_error(ks);
  }
  lk.unlock();
  if ((rc = wait_order_gate(s))) return rc;  // the data's producer on the caller's stream
  if ((rc = copysvc_copy(svc, ks->slot[worker], src, len)) && copysvc_broken(svc))
    rc = fallback_copy(s, ks, ks->slot[worker], src, len);
  if (rc) return rc;
  s->n_service_pushes.fetch_add(1, std::memory_order_relaxed);
  lk.lock();
  if (ks->error) return key_error(ks);
  std::vector<FoldJob> defer;
  if ((rc = arrive_and_wait_init(s, ks, worker, lk, &defer))) return rc;
  if (!defer.empty()) {
    lk.unlock();
    if (issue_combined(s, defer) && (rc = own_key_status(ks))) return rc;
    lk.lock();
  }
  return 0;
}
void sync_push_cb(void* ctx, uint64_t, int, int status) {
  static_cast<SyncWait*>(ctx)->finish(status);
}
// The caller's thread-local message for a status that came back through a callback.
int sync_status(byteps_server* s, uint64_t key, int status, const char* what) {
  if (status == 0) return 0;
  KeyState* ks = get_key(s, key, false);
  std::string msg = "?";
  if (ks) {
    std::lock_guard<std::mutex> g(ks->mu);
    msg = ks->error_msg;
  }
  return fail(status, "key %llu: %s failed: %s", (unsigned long long)key, what, msg.c_str());
}
}  // namespace srv
}  // namespace bpsr
