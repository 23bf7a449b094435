// GPU-resident PS server, device releases (include/bpsr/server.h): one keyed
// block queue folds every key of an epoch with ONE consumer launch, each key
// released by its round's last arrival (bpsr_server_state.h).
#include "bpsr_server_state.h"

namespace bpsr {
inline namespace srv {

// ------------------------------------------------------ device releases --

// The keyed queue over every allocated key of `dtype` (block order = key
// order), built once, at the first round completion after the init round
// (caller holds s->kq_mu and that key's mu).  Keys declared later, and keys
// of other dtypes, keep the lane launches.
void build_kq(byteps_server* s, int dtype) {
  std::vector<KeyState*> keys;
  {
    std::shared_lock<std::shared_mutex> g(s->map_mu);
    for (auto& kv : s->keys) {
      KeyState* k = kv.second.get();
      if (k->allocated && k->dtype == dtype) keys.push_back(k);
    }
  }
  if (keys.empty()) return;
  std::sort(keys.begin(), keys.end(),
            [](const KeyState* a, const KeyState* b) { return a->key < b->key; });
  const int N = s->cfg.num_workers;
  std::vector<byteps_bucket_desc> d(keys.size());
  for (size_t i = 0; i < keys.size(); ++i) {
    std::memset(&d[i], 0, sizeof(d[i]));
    d[i].dst = keys[i]->store;
    for (int w = 0; w < N; ++w) d[i].srcs[w] = keys[i]->slot[w];
    d[i].len = keys[i]->len;
    d[i].n = N;
  }
  if (force_device(s) || keyq_create(d.data(), (int)d.size(), dtype, s->kq_timeout_s, &s->kq)) {
    s->kq = nullptr;  // no queue: every round keeps the lane launches
    return;
  }
  s->kq_keys = keys;
  for (size_t i = 0; i < keys.size(); ++i) keys[i]->kq_key.store((int)i);
}

// Is this finished round of `ks` device-released?  Caller holds ks->mu.
// The first round finished through the slots (push_ready, or device data the
// copy service landed) builds the keyed queue; until then copied rounds (host
// data: the ps-lite shape) fold with lane launches and build nothing, so a
// server whose pushes all land in host memory never runs a consumer (config 1
// took 11.5-13.3 ms per round with one beside its lanes against 3.1, r05s55).
// Once the queue exists, each epoch's kind decides (key_release).
bool keyed_member(byteps_server* s, KeyState* ks) {
  if (!s->dev_release || s->kq_off.load()) return false;
  // decided once: no lock from then on (kq_mu is held across the consumer
  // launches, and every round's last arrival asks this)
  if (s->kq_tried.load(std::memory_order_acquire)) return ks->kq_key.load() >= 0;
  if (ks->round_copied) return false;  // no queue yet: a lane launch
  std::lock_guard<std::mutex> g(s->kq_mu);
  if (!s->kq_tried.load(std::memory_order_relaxed)) {
    build_kq(s, ks->dtype);
    s->kq_tried.store(true, std::memory_order_release);
  }
  return ks->kq_key.load() >= 0;
}

// Launch the consumers of every epoch up to `need` (caller holds kq_mu):
// each gets its ring slot's stop event and is tracked by the keyed completer.
int kq_launch_upto(byteps_server* s, uint32_t need) {
  for (uint32_t launched = keyq_launched(s->kq); launched < need;
       launched = keyq_launched(s->kq)) {
    const uint32_t next = launched + 1;
    const int slot = (int)(next % byteps_server::kKqRing);
    if (s->kq_ev_epoch[slot] != 0 && s->kq_done_seq.load() < s->kq_ev_seq[slot])
      return fail(BYTEPS_REDUCE_EARGS, "device releases: %d epochs in flight",
                  byteps_server::kKqRing);
    hipEvent_t& e = s->kq_ev[slot];
    if (!e) {
      if (int rc = force_device(s)) return rc;
      const hipError_t he = hipEventCreateWithFlags(&e, hipEventDisableTiming);
      if (he != hipSuccess) {
        e = nullptr;
        return hip_fail(he, "hipEventCreate(consumer)");
      }
    }
    uint32_t got = 0;
    hipStream_t cs = nullptr;
    if (int rc = keyq_launch(s->kq, e, &cs, &got)) return rc;
    s->kq_ev_epoch[slot] = got;
    s->kq_ev_seq[slot] = track_keyed(*s->klane, e, got);
    s->kq_pub_epoch.store(got, std::memory_order_release);
    s->kq_kind[slot] = byteps_server::kConsumerEpoch;
    s->kq_decided.store(got, std::memory_order_release);  // the fast path may use it now
  }
  return 0;
}

// The keyed completer, once epoch `epoch` has begun: launch the next epoch's
// consumer now, behind this one on the keyed queue, so that it is dispatched
// the moment this one completes and its tiles are resident, polling their
// words, before the next round's first push (DESIGN.md §9 "launched ahead").
// A launch that fails here is left to the next round's first release, which
// launches as before.
void kq_launch_ahead(byteps_server* s, uint32_t epoch) {
  std::lock_guard<std::mutex> g(s->kq_mu);
  if (s->kq_off.load() || !s->kq || keyq_failed(s->kq)) return;
  (void)kq_launch_upto(s, epoch + 1);
}

// Skip words for every key not yet released for `epoch` (each under its
// key's lock, as a release is): the epoch's consumer passes them and
// completes, and those keys' next rounds go to the next epoch.  A key may
// lag more than one epoch: lane epochs (no consumer) do not wait for every
// key, so a key whose round is late can still be short of a lane epoch
// before this one; it is skipped through those too (its late round then
// folds in the next epoch) — skipping only keys at exactly `epoch` left this
// consumer waiting for a key whose next round needed the epochs queued
// behind it (the device timeout, found by
// test_device_release_mixed_kinds_and_late_keys_stress).
static void skip_unreleased(byteps_server* s, uint32_t epoch) {
  const uint64_t skip = ((uint64_t)kKeySkip << 32) | kKeySkip;
  for (KeyState* k : s->kq_keys) {
    const int kk = k->kq_key.load();
    // a key released for this epoch is not locked at all: its lock may be
    // held by a push waiting for that key's own fold (wait_keyed_slots),
    // which can sit in an epoch behind this one
    if (kk < 0 || !epoch_reached(epoch, keyq_next_epoch(s->kq, kk))) continue;
    std::lock_guard<std::mutex> g(k->mu);
    while (epoch_reached(epoch, keyq_next_epoch(s->kq, kk)))  // next <= epoch (wrap-safe)
      (void)keyq_release(s->kq, kk, skip, nullptr);
  }
}

// Wait on the host until key `kq_key`'s fold in consumer epoch `epoch` has
// read its slots: the key's own completion word, not the epoch's event.  An
// epoch can hold for a late key until the completer closes it, and a lane
// copy stream put behind the epoch's event holds every later copy of the lane
// with it — a blocking push of another key then waited under that key's lock,
// which the close needed (the device timeout of
// test_device_release_mixed_kinds_and_late_keys_stress).  False: the queue
// failed or is not there; the caller then orders on the event as before.
bool wait_keyed_slots(byteps_server* s, int kq_key, uint32_t epoch) {
  if (kq_key < 0 || !epoch || !s->kq) return false;
  for (int i = 0;; ++i) {
    if (keyq_key_done(s->kq, kq_key, epoch)) return true;
    if (keyq_failed(s->kq)) return false;
    if (i < 4096)
      __builtin_ia32_pause();
    else
      std::this_thread::sleep_for(std::chrono::microseconds(5));
  }
}
bool wait_keyed_slots(byteps_server* s, const KeyState* ks) {
  return ks->keyed && ks->has_done && wait_keyed_slots(s, ks->kq_key.load(), ks->kq_round_epoch);
}

// Retire an epoch launched ahead that no round has begun (skip_unreleased),
// so its consumer does not hold its workgroup slots while the caller is idle.
// The epoch is closed first (keyq_close), so a round that begins it from then
// on is not counted as its first; such a round keeps its place in this epoch
// and is folded by it.  False: a round had begun the epoch, which is not
// retired.
bool kq_retire(byteps_server* s, uint32_t epoch) {
  if (!keyq_close(s->kq, epoch)) return false;  // a round began it after all
  skip_unreleased(s, epoch);
  s->n_consumer_retired.fetch_add(1, std::memory_order_relaxed);
  return true;
}

// Close a begun epoch whose keys have not all come (kKeyedCloseMs after its
// first release): the reference folds every key on its own, so a key that
// skips an iteration — or arrives late — must not hold the others' epoch, nor
// fail.  Its round, when it comes, is folded by a later epoch.
void kq_close_epoch(byteps_server* s, uint32_t epoch) {
  skip_unreleased(s, epoch);
  s->n_epochs_closed.fetch_add(1, std::memory_order_relaxed);
}

// Release a finished round of a keyed key (caller holds ks->mu).  The
// round's epoch is its key's next; its kind is decided by the epoch's first
// release (or its consumer's launch ahead): a slot-written round opening an
// epoch launches its consumer, a copied round (`skip`) opening one with no
// consumer launched makes it a lane epoch.  In a consumer epoch the arrival
// order and the release word go to the key's block — stored from the host
// when the round's data is in its slots already (push_ready), or by a
// one-lane kernel on `stream` behind the round's copies — and the round is
// published like an issued fold; a copied round passes the consumer with a
// skip word.  In a lane epoch every round gets a skip word and folds with a
// lane launch.  Returns 1 when the caller must fold the round with a launch
// (a lane epoch, or device releases turned off meanwhile).
int key_release(byteps_server* s, KeyState* ks, const std::vector<int>& order, hipStream_t stream,
                bool skip) {
  uint64_t perm = 0;  // position m's worker in bits 4m..4m+3 (16 positions)
  for (size_t m = 0; m < order.size(); ++m) perm |= (uint64_t)order[m] << (4 * m);
  if (skip) perm = ((uint64_t)kKeySkip << 32) | kKeySkip;
  bool first = false;  // the first round released for its epoch
  const int kk = ks->kq_key.load();
  const uint32_t need = keyq_next_epoch(s->kq, kk);
  const int slot = (int)(need % byteps_server::kKqRing);
  Lane& RL = *s->lanes[ks->lane];
  if (s->kq_off.load()) return 1;
  if (s->kq_decided.load(std::memory_order_acquire) < need) {
    // this release opens epoch `need` (no lock otherwise: a decided epoch's
    // kind and ring slot stay put until it completes, which needs this key)
    if (stream) RL.where = "key_release: kq_mu";
    std::lock_guard<std::mutex> g(s->kq_mu);
    if (stream) RL.where = "key_release: launch";
    if (s->kq_off.load()) return 1;
    if (s->kq_decided.load(std::memory_order_relaxed) < need) {
      if (skip && keyq_launched(s->kq) < need) {
        if (!keyq_advance(s->kq, need))
          return fail(BYTEPS_REDUCE_EARGS, "device releases: epoch %u opened out of order", need);
        s->kq_kind[slot] = byteps_server::kLaneEpoch;
        s->kq_decided.store(need, std::memory_order_release);
        s->n_lane_epochs.fetch_add(1, std::memory_order_relaxed);
      } else if (int rc = kq_launch_upto(s, need)) {
        return rc;
      }
    }
  }
  if (s->kq_kind[slot] == byteps_server::kLaneEpoch) {
    const uint64_t sk = ((uint64_t)kKeySkip << 32) | kKeySkip;
    if (int rc = keyq_release(s->kq, kk, sk, nullptr)) return rc;
    return skip ? 0 : 1;
  }
  const hipEvent_t ev = s->kq_ev[slot];
  const uint64_t seq = s->kq_ev_seq[slot];
  if (stream) {
    RL.where = "key_release: wait d2h";
    // behind the lane's pull copies too (a store is rewritten by the fold)
    const hipError_t we = hipStreamWaitEvent(stream, RL.d2h_mark, 0);
    if (we != hipSuccess) return hip_fail(we, "hipStreamWaitEvent");
    RL.where = "key_release: release kernel";
  }
  if (int rc = keyq_release(s->kq, kk, perm, stream, &first)) return rc;
  if (stream) RL.where = "key_release: publish";
  if (first) s->n_consumer_launches.fetch_add(1, std::memory_order_relaxed);
  if (skip) return 0;  // the round is folded by a lane launch, which publishes it
  uint32_t se = s->kq_slot_epoch.load(std::memory_order_relaxed);
  while (se < need && !s->kq_slot_epoch.compare_exchange_weak(se, need)) {
  }
  s->n_key_releases.add();
  ks->kq_round_epoch = need;
  return finish_round(s, ks, order, /*mark=*/false, ev, seq, /*keyed=*/true);
}

// The keyed completer saw epoch `epoch`'s consumer (lane seq `seq`) complete:
// if a consumer gave up waiting, every key released at that epoch or later
// fails (its store is not the round's fold) and device releases go off for
// good; then the epoch is published and the pulls parked on it go to their
// lanes' issuers (or fail with their key).
void kq_epoch_done(byteps_server* s, uint32_t epoch, uint64_t seq) {
  std::vector<PullJob> go, keep;
  std::vector<KeyState*> failed;
  {
    std::lock_guard<std::mutex> g(s->kq_mu);
    if (s->kq && keyq_failed(s->kq)) {
      if (getenv("BPSR_SERVER_RELEASE_DEBUG")) {
        fprintf(stderr, "bpsr server: epoch %u timed out: %s\n", epoch, keyq_debug(s->kq).c_str());
        for (size_t l = 0; l < s->lanes.size(); ++l) {
          Lane& L = *s->lanes[l];
          size_t nc = 0, ncp = 0, np = 0;
          uint64_t iss = 0;
          {
            std::lock_guard<std::mutex> dg(L.done_mu);
            iss = L.issued_seq;
          }
          {
            std::lock_guard<std::mutex> cg(L.comb_mu);
            nc = L.comb.size();
            ncp = L.copies.size();
            np = L.pulls.size();
          }
          fprintf(stderr,
                  "  lane %zu: issued %llu done %llu, queued folds %zu copies %zu pulls %zu, "
                  "issuer at %s\n",
                  l, (unsigned long long)iss, (unsigned long long)L.done_pub.load(), nc, ncp, np,
                  L.where.load());
        }
        int rounds_done = 0, pending = 0;
        for (KeyState* k : s->kq_keys) {
          if (keyq_next_epoch(s->kq, k->kq_key.load()) > epoch) ++rounds_done;
          pending += k->pending;
        }
        fprintf(stderr, "  keys released for this epoch %d of %zu, deferred jobs %d\n",
                rounds_done, s->kq_keys.size(), pending);
        fprintf(stderr, "  launched %u decided %u opened %u slot-epoch %u; kinds:",
                keyq_launched(s->kq), s->kq_decided.load(), keyq_opened(s->kq),
                s->kq_slot_epoch.load());
        for (uint32_t e = epoch > 4 ? epoch - 4 : 1; e <= s->kq_decided.load(); ++e)
          fprintf(stderr, " %u:%d", e, (int)s->kq_kind[e % byteps_server::kKqRing]);
        fprintf(stderr, "\n  next epoch per key:");
        for (KeyState* k : s->kq_keys)
          fprintf(stderr, " %llu:%u", (unsigned long long)k->key,
                  keyq_next_epoch(s->kq, k->kq_key.load()));
        fprintf(stderr, "\n");
      }
      s->kq_off.store(true);
      for (KeyState* k : s->kq_keys)
        if (keyq_next_epoch(s->kq, k->kq_key.load()) > epoch) failed.push_back(k);
    }
  }
  {
    std::lock_guard<std::mutex> g(s->kq_park_mu);
    s->kq_done_seq.store(seq);
    for (PullJob& j : s->kq_parked) (j.kseq <= seq ? go : keep).push_back(j);
    s->kq_parked.swap(keep);
  }
  for (KeyState* k : failed) {
    std::lock_guard<std::mutex> g(k->mu);
    fail(BYTEPS_REDUCE_ETIMEOUT, "device release: a key of the queue was not pushed within %.3f s "
         "(BPSR_SERVER_RELEASE_TIMEOUT_S); its epoch's folds are void", s->kq_timeout_s);
    fail_key(s, k, BYTEPS_REDUCE_ETIMEOUT);
  }
  for (PullJob& j : go) {
    int err = 0;
    {
      std::lock_guard<std::mutex> g(j.ks->mu);
      err = j.ks->error;
    }
    if (err) {
      if (j.direct) {
        j.direct->finish(err);
      } else {
        j.resp.status = err;
        enqueue_response(s, j.resp);
      }
      continue;
    }
    Lane& L = *s->lanes[j.ks->lane];
    std::lock_guard<std::mutex> g(L.comb_mu);
    L.pulls.push_back(j);
    L.comb_cv.notify_one();
  }
}

}  // namespace srv
}  // namespace bpsr
