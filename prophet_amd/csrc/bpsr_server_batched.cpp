// GPU-resident PS server: the batched calls (push_ready_many, push_many,
// pull_many; include/bpsr/server.h) — one launch per lane for many keys
// (bpsr_server_state.h).
#include "bpsr_server_state.h"

namespace bpsr {
inline namespace srv {

// A push_many's host copies in flight at most (per call): 4 partitions of
// BytePS's 4,096,000-B bound.  The transport's calls of different workers then
// interleave on the link partition by partition, so rounds complete — and are
// folded and pulled back — while later partitions are still crossing PCIe,
// instead of one worker's whole batch landing before any other worker's.
constexpr size_t kHostPushInflight = 16u << 20;

hipEvent_t pool_take(byteps_server* s) {
  {
    std::lock_guard<std::mutex> g(s->ev_pool_mu);
    if (!s->ev_pool.empty()) {
      hipEvent_t e = s->ev_pool.back();
      s->ev_pool.pop_back();
      return e;
    }
  }
  hipEvent_t e = nullptr;
  return hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess ? e : nullptr;
}

void pool_give(byteps_server* s, hipEvent_t e) {
  std::lock_guard<std::mutex> g(s->ev_pool_mu);
  s->ev_pool.push_back(e);
}

// byteps_server_push_many from host memory, in BytePS's order (core_loops.cc:
// 492-564 issues every partition's ZPush as it comes): key by key, the H2D
// copy into the slot on the key's lane (its own `copied` event, and the lane's
// copy mark), then the arrival, whose completed round goes to the issuer at
// once — with at most kHostPushInflight bytes of this call's copies in flight.
// Every slot was found free before (the caller's step 1).  Returns once every
// copy has landed (the blocking contract).
int push_many_host(byteps_server* s, std::vector<KeyState*>& ks_of, const void* const* datas,
                   const size_t* lens, int n, int worker) {
  struct Flight {
    hipEvent_t ev;
    size_t bytes;
  };
  std::deque<Flight> flight;
  size_t in_flight = 0;
  int rc = 0;
  auto retire = [&](size_t need) -> int {
    while (!flight.empty() && (need == 0 || in_flight + need > kHostPushInflight)) {
      const hipError_t e = hipEventSynchronize(flight.front().ev);
      pool_give(s, flight.front().ev);
      in_flight -= flight.front().bytes;
      flight.pop_front();
      if (e != hipSuccess) return hip_fail(e, "push copy");
    }
    return 0;
  };
  std::vector<char> lane_ready(s->lanes.size(), 0);
  std::vector<FoldJob> defer;
  for (int i = 0; i < n && !rc; ++i) {
    KeyState* ks = ks_of[i];
    Lane& L = *s->lanes[ks->lane];
    if ((rc = retire(lens[i]))) break;
    hipEvent_t fe = pool_take(s);
    if (!fe) {
      rc = fail(BYTEPS_REDUCE_EHIP, "hipEventCreate (push window)");
      break;
    }
    {
      std::lock_guard<std::mutex> bg(L.batch_mu);
      hipError_t e = hipSuccess;
      if (!lane_ready[ks->lane]) {  // once per lane: behind the lane's folds so far
        lane_ready[ks->lane] = 1;
        e = hipStreamWaitEvent(L.copy, L.fold_mark, 0);
      }
      {
        std::lock_guard<std::mutex> g(ks->mu);
        // keyed folds run on the consumer's stream, not behind the fold mark
        if (e == hipSuccess && ks->keyed && ks->has_done && !wait_keyed_slots(s, ks))
          e = hipStreamWaitEvent(L.copy, ks->fold_ev, 0);
        if (e == hipSuccess)
          e = hipMemcpyAsync(ks->slot[worker], datas[i], lens[i], hipMemcpyHostToDevice, L.copy);
        if (e == hipSuccess) e = hipEventRecord(ks->copied, L.copy);
      }
      if (e == hipSuccess) e = hipEventRecord(L.copy_mark, L.copy);
      if (e == hipSuccess) L.copy_seq.fetch_add(1);
      if (e == hipSuccess) e = hipEventRecord(fe, L.copy);
      if (e != hipSuccess) {
        pool_give(s, fe);
        rc = hip_fail(e, "push copy");
        break;
      }
    }
    flight.push_back({fe, lens[i]});
    in_flight += lens[i];
    std::unique_lock<std::mutex> lk(ks->mu);
    ks->round_copied = true;
    const bool init_round = !ks->inited;
    if ((rc = arrive(s, ks, worker, &defer))) break;
    if (init_round && !ks->inited) {  // held until every worker's init push is in
      lk.unlock();
      if ((rc = issue_deferred(s, defer))) break;
      lk.lock();
      ks->cv.wait(lk, [&] { return ks->inited || ks->error; });
      if (ks->error) {
        rc = key_error(ks);
        break;
      }
    }
    lk.unlock();
    if (!defer.empty() && (rc = issue_deferred(s, defer))) break;
  }
  if (!defer.empty()) {
    const int r2 = issue_deferred(s, defer);
    if (!rc) rc = r2;
  }
  const int r3 = retire(0);
  return rc ? rc : r3;
}

}  // namespace srv
}  // namespace bpsr

using namespace bpsr;

extern "C" {

// ------------------------------------------------------- batched calls --

int byteps_server_push_ready_many(byteps_server* s, const uint64_t* keys, int n, int worker) {
  if (!s || (n > 0 && !keys) || n < 0) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (worker < 0 || worker >= s->cfg.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker, s->cfg.num_workers);
  int rc = set_device(s);
  if (rc) return rc;
  if ((rc = wait_order_gate(s))) return rc;  // before any key lock (push_ready)
  std::vector<FoldJob> defer;
  for (int i = 0; i < n; ++i) {
    KeyState* ks = get_key(s, keys[i], false);
    if (!ks || !ks->allocated) {
      (void)issue_deferred(s, defer);
      return fail(BYTEPS_REDUCE_EARGS, "key %llu not initialised", (unsigned long long)keys[i]);
    }
    std::unique_lock<std::mutex> lk(ks->mu);
    if (!can_push(s, ks, worker)) {
      // never block while holding deferred rounds: others may wait on them
      lk.unlock();
      if ((rc = issue_deferred(s, defer))) return rc;
      lk.lock();
      ks->cv.wait(lk, [&] { return can_push(s, ks, worker); });
    }
    if (ks->error) {
      lk.unlock();
      (void)issue_deferred(s, defer);
      return key_error(ks);
    }
    const bool init_round = !ks->inited;
    if ((rc = arrive(s, ks, worker, &defer))) {
      lk.unlock();
      (void)issue_deferred(s, defer);
      return rc;
    }
    if (init_round && !ks->inited) {
      lk.unlock();
      if ((rc = issue_deferred(s, defer))) return rc;
      lk.lock();
      ks->cv.wait(lk, [&] { return ks->inited || ks->error; });
      if (ks->error) return key_error(ks);
    }
  }
  return issue_deferred(s, defer);
}

int byteps_server_push_many(byteps_server* s, const uint64_t* keys, const void* const* datas,
                            const size_t* lens, int n, int worker, int dtype, int location) {
  if (!s || n < 0 || (n > 0 && (!keys || !datas || !lens)))
    return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (worker < 0 || worker >= s->cfg.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker, s->cfg.num_workers);
  int rc = set_device(s);
  if (rc) return rc;
  // 1. every slot free (its previous round folded), then the copies: per lane
  //    ONE wait for the lane's folds so far, then one batched copy (device
  //    sources) or a hipMemcpyAsync per key (host sources), then the lane's
  //    copy mark, which every later fold of the lane waits for
  std::vector<KeyState*> ks_of(n);
  std::vector<std::vector<int>> by_lane(s->lanes.size());
  for (int i = 0; i < n; ++i) {
    if (!datas[i]) return fail(BYTEPS_REDUCE_EARGS, "null data for key %d", i);
    KeyState* ks = get_key(s, keys[i], true);
    ks_of[i] = ks;
    std::unique_lock<std::mutex> lk(ks->mu);
    if ((rc = allocate(s, ks, lens[i], dtype))) return rc;
    ks->cv.wait(lk, [&] { return can_push(s, ks, worker); });
    if (ks->error) return key_error(ks);
    by_lane[ks->lane].push_back(i);
  }
  // host data (the default engine, sync mode): copies and arrivals key by key
  if (location == BYTEPS_SERVER_HOST && s->combine && !s->cfg.async_mode) {
    if ((rc = push_many_host(s, ks_of, datas, lens, n, worker))) return rc;
    return BYTEPS_REDUCE_OK;
  }
  for (size_t l = 0; l < by_lane.size(); ++l) {
    if (by_lane[l].empty()) continue;
    Lane& L = *s->lanes[l];
    std::lock_guard<std::mutex> bg(L.batch_mu);
    hipError_t e = hipStreamWaitEvent(L.copy, L.fold_mark, 0);
    if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent");
    {  // keyed folds run on the consumer's stream, not behind the fold mark
      std::vector<hipEvent_t> waits;
      for (int i : by_lane[l]) {
        std::lock_guard<std::mutex> g(ks_of[i]->mu);
        if (ks_of[i]->keyed && ks_of[i]->has_done && !wait_keyed_slots(s, ks_of[i]))
          waits.push_back(ks_of[i]->fold_ev);
      }
      std::sort(waits.begin(), waits.end());
      waits.erase(std::unique(waits.begin(), waits.end()), waits.end());
      for (hipEvent_t w : waits)
        if ((e = hipStreamWaitEvent(L.copy, w, 0)) != hipSuccess) return hip_fail(e, "hipStreamWaitEvent");
    }
    if (location == BYTEPS_SERVER_HOST) {
      // each key's own copy event: its round folds once ITS copies have
      // landed, while the lane's later partitions are still crossing PCIe
      for (int i : by_lane[l]) {
        e = hipMemcpyAsync(ks_of[i]->slot[worker], datas[i], lens[i], hipMemcpyHostToDevice,
                           L.copy);
        if (e == hipSuccess) {
          std::lock_guard<std::mutex> g(ks_of[i]->mu);
          e = hipEventRecord(ks_of[i]->copied, L.copy);
        }
        if (e != hipSuccess) return hip_fail(e, "push copy");
      }
    } else {
      std::vector<byteps_bucket_desc> d(by_lane[l].size());
      for (size_t k = 0; k < by_lane[l].size(); ++k) {
        const int i = by_lane[l][k];
        std::memset(&d[k], 0, sizeof(d[k]));
        d[k].dst = ks_of[i]->slot[worker];
        d[k].srcs[0] = datas[i];
        d[k].len = lens[i];
        d[k].n = 1;
      }
      if ((rc = batched_with_ring(d.data(), (int)d.size(), BYTEPS_REDUCE_UINT8,
                                  BYTEPS_REDUCE_MODE_REFERENCE, L.copy, L.ring)))
        return rc;
    }
    if ((e = hipEventRecord(L.copy_mark, L.copy)) != hipSuccess)
      return hip_fail(e, "hipEventRecord");
    L.copy_seq.fetch_add(1);
  }
  // 2. arrivals, with the rounds they complete folded per lane in one launch
  std::vector<FoldJob> defer;
  for (int i = 0; i < n; ++i) {
    KeyState* ks = ks_of[i];
    std::unique_lock<std::mutex> lk(ks->mu);
    ks->round_copied = true;
    if (location != BYTEPS_SERVER_HOST) ks->round_mark_copy = true;
    const bool init_round = !ks->inited;
    if ((rc = arrive(s, ks, worker, &defer))) {
      lk.unlock();
      (void)issue_deferred(s, defer);
      return rc;
    }
    if (init_round && !ks->inited) {
      lk.unlock();
      if ((rc = issue_deferred(s, defer))) return rc;
      lk.lock();
      ks->cv.wait(lk, [&] { return ks->inited || ks->error; });
      if (ks->error) return key_error(ks);
    }
  }
  if ((rc = issue_deferred(s, defer))) return rc;
  if (s->blocking)  // engine blocking mode: the folds issued above have completed
    for (size_t l = 0; l < by_lane.size(); ++l)
      if (!by_lane[l].empty()) {
        hipError_t e = hipStreamSynchronize(s->lanes[l]->fold);
        if (e != hipSuccess) return hip_fail(e, "engine blocking: fold sync");
      }
  // 3. blocking contract: every source may be reused once the call returns
  //    (a lane's copy mark, re-recorded since, covers this call's copies too)
  for (size_t l = 0; l < by_lane.size(); ++l) {
    if (by_lane[l].empty()) continue;
    hipError_t e = hipEventSynchronize(s->lanes[l]->copy_mark);
    if (e != hipSuccess) return hip_fail(e, "push copy");
  }
  return BYTEPS_REDUCE_OK;
}

int byteps_server_pull_many(byteps_server* s, const uint64_t* keys, void* const* outs,
                            const size_t* lens, int n, int location) {
  if (!s || n < 0 || (n > 0 && (!keys || !outs || !lens)))
    return fail(BYTEPS_REDUCE_EARGS, "null argument");
  int rc = set_device(s);
  if (rc) return rc;
  if (s->cfg.async_mode) {
    // every fold changes the store: each pull keeps the single call's
    // ordering (copy queued under the key lock, later folds wait for it)
    for (int i = 0; i < n; ++i)
      if ((rc = byteps_server_pull(s, keys[i], outs[i], lens[i], location))) return rc;
    return BYTEPS_REDUCE_OK;
  }
  std::vector<KeyState*> ks_of(n, nullptr);
  std::vector<std::vector<int>> ready(s->lanes.size());  // rounds finished, copies not issued
  std::vector<char> touched(s->lanes.size(), 0);
  size_t ready_bytes = 0;
  // Issue the copies of the keys found ready: per lane ONE wait for the lane's
  // folds so far (they include every ready key's round: a round is published
  // after its fold was issued and the mark raised), one batched copy (device
  // destinations) or a hipMemcpyAsync per key (host), then the d2h mark.
  auto flush = [&]() -> int {
    for (size_t l = 0; l < ready.size(); ++l) {
      if (ready[l].empty()) continue;
      Lane& L = *s->lanes[l];
      std::lock_guard<std::mutex> bg(L.batch_mu);
      hipError_t e = hipStreamWaitEvent(L.d2h, L.fold_mark, 0);
      if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent");
      if (location == BYTEPS_SERVER_HOST) {
        for (int i : ready[l]) {
          if (void* dv = pull_kernel_dst(outs[i], location)) {
            if (int rc = byteps_reduce_copy(dv, ks_of[i]->store, lens[i], L.d2h)) return rc;
            continue;
          }
          e = hipMemcpyAsync(outs[i], ks_of[i]->store, lens[i], hipMemcpyDeviceToHost, L.d2h);
          if (e != hipSuccess) return hip_fail(e, "pull copy");
        }
      } else {
        std::vector<byteps_bucket_desc> d(ready[l].size());
        for (size_t k = 0; k < ready[l].size(); ++k) {
          const int i = ready[l][k];
          std::memset(&d[k], 0, sizeof(d[k]));
          d[k].dst = outs[i];
          d[k].srcs[0] = ks_of[i]->store;
          d[k].len = lens[i];
          d[k].n = 1;
        }
        int r = batched_with_ring(d.data(), (int)d.size(), BYTEPS_REDUCE_UINT8,
                                  BYTEPS_REDUCE_MODE_REFERENCE, L.d2h, L.ring);
        if (r) return r;
      }
      s->n_pull_launches.fetch_add(1, std::memory_order_relaxed);
      if ((e = hipEventRecord(L.d2h_mark, L.d2h)) != hipSuccess)
        return hip_fail(e, "hipEventRecord");
      touched[l] = 1;
      ready[l].clear();
    }
    return 0;
  };
  for (int i = 0; i < n; ++i) {
    KeyState* ks = key_for_pull(s, keys[i]);
    if (!ks) {
      (void)flush();
      return BYTEPS_REDUCE_EARGS;
    }
    ks_of[i] = ks;
    std::unique_lock<std::mutex> lk(ks->mu);
    if (lens[i] > ks->len || !outs[i]) {
      lk.unlock();
      (void)flush();
      return fail(BYTEPS_REDUCE_EARGS, "pull %d: bad buffer or %zu bytes > key len %zu", i,
                  lens[i], ks->len);
    }
    if (!pull_ready(s, ks)) {
      lk.unlock();
      // let enough ready bytes go while this round finishes; fewer, larger
      // batched copies otherwise (rounds often complete together)
      if (ready_bytes >= kPullFlushBytes) {
        if ((rc = flush())) return rc;
        ready_bytes = 0;
      }
      lk.lock();
      ks->cv.wait(lk, [&] { return pull_ready(s, ks); });
    }
    if (ks->keyed && !ks->error) {  // its epoch published first
      const uint64_t need = ks->fold_seq;
      lk.unlock();
      wait_published(s, ks, need);
      lk.lock();
    }
    if (ks->error) {
      lk.unlock();
      (void)flush();
      return key_error(ks);
    }
    ready[ks->lane].push_back(i);
    ready_bytes += lens[i];
  }
  if ((rc = flush())) return rc;
  for (size_t l = 0; l < touched.size(); ++l) {  // a later record covers this call's copies too
    if (!touched[l]) continue;
    hipError_t e = hipEventSynchronize(s->lanes[l]->d2h_mark);
    if (e != hipSuccess) return hip_fail(e, "pull copy");
  }
  for (int i = 0; i < n; ++i) {
    std::lock_guard<std::mutex> g(ks_of[i]->mu);
    count_pull(s, ks_of[i]);  // server.cc:105-113
  }
  s->n_pulls.add((uint64_t)n);
  return BYTEPS_REDUCE_OK;
}
}  // extern "C"
