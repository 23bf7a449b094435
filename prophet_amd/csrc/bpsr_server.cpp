// GPU-resident parameter-server aggregation (include/bpsr/server.h): the
// per-key state machine of byteps/server/server.cc:147-308 with the engine
// threads (server.cc:70-145) replaced by HIP stream lanes and the CpuReducer
// calls replaced by the gfx950 fold kernels.
#include "bpsr/server.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <limits>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "bpsr_engine_queue.h"
#include "bpsr_internal.h"

namespace bpsr {
namespace {

constexpr size_t kSlotAlign = 64 * 1024;  // bucket rounding before the skew (prophet_amd/arena.py)
constexpr size_t kSlotSkew = 16 * 1024;  // prophet_amd/arena.py: skewed slots
constexpr int kMaxDebugLog = 4096;
// pull_many issues the copies of the rounds found finished once this many
// bytes are ready and it must wait for another round (else at the end)
constexpr size_t kPullFlushBytes = 8u << 20;

struct KeyState;

// One engine message (server.h:65-75 BytePSEngineMessage): the fold work of
// one arrival (SUM_RECV), of a finished round (COPY_MERGED, or the fused
// left fold) or of an async push.
enum JobKind { kSumRecv = 0, kAsyncSum = 1, kFinishIncremental = 2, kFinishFused = 3,
               kKeyRelease = 4 };  // a device-released round whose pushes were copied
struct FoldJob {
  KeyState* ks = nullptr;
  int kind = kSumRecv;
  int w = -1;              // the arriving worker's slot
  int acc = -1;            // the accumulator slot (first arrival), incremental policy
  std::vector<int> order;  // arrival order of the finished round
};

struct Lane;
// A pull ready to be answered, or a push to acknowledge, by the responder.
struct Response {
  uint64_t key = 0;
  KeyState* ks = nullptr;
  byteps_server_pull_cb cb = nullptr;
  void* ctx = nullptr;
  const char* view = nullptr;  // mirror holding the answered round
  int status = 0;
  byteps_server_push_cb push_cb = nullptr;  // set: a push acknowledgement
  int worker = -1;
  // a push whose copy the lane's issuer batched: acknowledge once the lane's
  // completer has seen launch wait_seq complete (else sync `copied`); the
  // same for a pull copied into the caller's buffer (len: its length)
  Lane* wait_lane = nullptr;
  uint64_t wait_seq = 0;
  size_t len = 0;
  uint64_t kseq = 0;  // a view of a keyed round: answered once its epoch is published
};

// A blocking call served by the non-blocking machinery: the lane issuer
// batches the copy with whatever else piled up, the completer and responder
// finish it, and the caller waits here without making a HIP call.  (HIP
// calls serialise across threads: eight workers each making 4-5 calls per
// key paid ~8 us per call)
struct Lane;
// BPSR_SERVER_SPIN_US: how long a blocking call's waiter polls before it
// sleeps on a condition variable (0: sleep at once).  A sleeping waiter's
// wake-up is a futex round trip per hand-off.
int64_t spin_ns() {
  static const int64_t ns = [] {
    const char* v = getenv("BPSR_SERVER_SPIN_US");
    return v ? std::max(0L, atol(v)) * 1000L : 0L;
  }();
  return ns;
}
// Poll `ready` for up to spin_ns(); true once it holds.
template <class F>
bool spin_until(F ready) {
  const int64_t budget = spin_ns();
  if (budget == 0) return false;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    for (int i = 0; i < 64; ++i) {
      if (ready()) return true;
      __builtin_ia32_pause();
    }
    if (std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
            .count() > budget)
      return ready();
  }
}
struct SyncWait {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  std::atomic<bool> flag{false};  // `done`, set under mu, for a spinning waiter
  int status = 0;
  Lane* lane = nullptr;  // a direct pull or push: the launch its copy rides in
  uint64_t seq = 0;
  int wait() {
    // a waiter that saw the flag still takes mu, so it returns (and the
    // caller's frame goes) only after finish() has let go of it
    (void)spin_until([&] { return flag.load(std::memory_order_acquire); });
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done; });
    return status;
  }
  void finish(int st) {
    std::lock_guard<std::mutex> g(mu);
    status = st;
    done = true;
    flag.store(true, std::memory_order_release);
    cv.notify_all();
  }
};
// A non-blocking pull into a caller's device buffer (byteps_server_pull_into_async)
// whose copy waits for the lane's issuer.  `direct`: a blocking pull's waiter,
// told the launch's seq by the issuer and then waiting on the lane's
// completion itself (no responder hop).
struct PullJob {
  KeyState* ks = nullptr;
  void* dst = nullptr;
  size_t len = 0;
  Response resp;
  SyncWait* direct = nullptr;
  uint64_t kseq = 0;  // parked on a keyed epoch: the keyed completer's seq it waits for
};

// A non-blocking push of device data whose copy into its slot waits for the
// lane's issuer (batched with the other copies that piled up).
struct CopyJob {
  KeyState* ks = nullptr;
  int w = -1;
  const void* src = nullptr;
  size_t len = 0;
  Response ack;
  SyncWait* direct = nullptr;  // a blocking push's waiter (no responder hop)
};

struct Lane {
  hipStream_t fold = nullptr;  // folds, in round order per key
  hipStream_t copy = nullptr;  // push copies
  hipStream_t d2h = nullptr;   // store -> host mirror copies
  // BYTEPS_SERVER_ENABLE_SCHEDULE: pending jobs and the thread that issues them
  std::unique_ptr<EngineQueue<FoldJob>> q;
  std::thread dispatcher;
  hipEvent_t job_done = nullptr;
  std::mutex dbg_mu;
  std::vector<uint64_t> log;  // keys of dispatched jobs, in dispatch order
  // batched calls (push_many / push_ready_many / pull_many): one batched
  // launch per lane for many keys, staged through the lane's own ring
  std::mutex batch_mu;
  StageRing* ring = nullptr;
  // Lane-wide marks: the latest work issued on each stream (a later record on
  // an in-order stream covers every earlier one).  Folds wait for copy_mark
  // (every push copy of the lane so far); batched calls wait for fold_mark /
  // d2h_mark once per lane instead of one event per key.
  hipEvent_t copy_mark = nullptr, fold_mark = nullptr, d2h_mark = nullptr;
  // Combining (no scheduling, no engine blocking): the rounds single-key
  // calls complete go to the lane's issuer thread, which issues what piled up
  // as ONE batched fold launch while the callers go on (issuer_main).
  std::mutex comb_mu;
  std::condition_variable comb_cv;   // work for the issuer
  std::vector<FoldJob> comb;
  std::vector<CopyJob> copies;       // non-blocking device pushes, before the folds
  std::vector<PullJob> pulls;        // non-blocking pulls into device buffers
  bool comb_stop = false;
  std::thread issuer;
  // Completion of what the issuer issued, tracked on the host so waiters make
  // no HIP call (HIP calls serialise across threads: 8 threads syncing events
  // per key cost 3.5 us each, tools/launch_cost.cpp): the issuer appends
  // (seq, event) per launch, the lane's completer thread waits for them in
  // order and publishes done_seq; a key remembers the seq of its last round.
  std::mutex done_mu;
  std::condition_variable cq_cv;    // issuer -> completer
  std::condition_variable done_cv;  // completer -> waiters (and the issuer)
  struct Tracked {
    uint64_t seq;
    hipEvent_t ev;
    uint32_t kq_epoch;  // != 0: the keyed consumer launch of that epoch (lane 0 only)
  };
  std::deque<Tracked> cq;
  uint64_t issued_seq = 0, done_seq = 0;
  std::atomic<uint64_t> done_pub{0};  // done_seq, readable without done_mu (spinning waiters)
  std::atomic<const char*> where{"idle"};  // the issuer's step (BPSR_SERVER_RELEASE_DEBUG dumps)
  bool cq_stop = false;
  std::thread completer;
  // copies recorded into copy_mark so far / seen by a fold's wait on it (a
  // fold stream already waiting on the latest copy mark need not wait again)
  std::atomic<uint64_t> copy_seq{0}, fold_copy_seen{0};
  // pull copies recorded into d2h_mark / seen by a fold's wait on it (a
  // fold rewrites the store those copies read)
  std::atomic<uint64_t> pull_seq{0}, fold_pull_seen{0};
};

struct KeyState {
  uint64_t key = 0;
  std::mutex mu;
  std::condition_variable cv;
  // Set once, last, by allocate() (under mu) after the slots, store, events
  // and lane exist; those never change afterwards, so the pull and
  // receive-slot paths may test it and read them before taking mu.
  std::atomic<bool> allocated{false};
  bool inited = false;        // store initialised (round 0 done)
  size_t len = 0;
  int dtype = 0;
  int lane = 0;
  char* arena = nullptr;      // N receive slots + store
  size_t stride = 0;
  std::vector<char*> slot;
  char* store = nullptr;
  // current round
  std::vector<char> got;      // worker pushed this round (cleared when the round's fold is issued)
  std::vector<int> order;     // arrival order this round
  int arrived = 0;
  int init_count = 0;
  int init_last = -1;         // the init round's last arrival (its push initialises the store)
  bool stamped = false;       // this round's arrivals carry positions (a group's range split)
  std::vector<Response> init_acks;  // non-blocking init pushes, answered together (server.cc:184-198)
  int pending = 0;            // jobs queued on the lane, not yet issued (scheduling only)
  int error = 0;              // sticky failure of an issued fold: every later call returns it
  std::string error_msg;
  // completion / pull gating (server.cc:100-114, 280-306)
  uint64_t rounds = 0;
  bool push_finished = false;
  int pull_cnt = 0;
  std::vector<int> last_order;
  hipEvent_t done = nullptr;  // recorded on the lane's fold stream after a single fold
  // What to wait for to see the key's last issued fold complete: `done`, or —
  // after a batched issue (flush_folds), which records no per-key event — the
  // lane's fold mark (a later record of it covers this fold too).
  hipEvent_t fold_ev = nullptr;
  uint64_t fold_seq = 0;      // lane completion seq of the last issued round (0: untracked)
  int fold_lane = 0;          // the lane whose completer tracks fold_seq
  std::vector<int> order_tmp; // a keyed round's order on its way out (arrive)
  uint32_t kq_round_epoch = 0; // a keyed round: the consumer epoch that folds it
  // device releases: the key's block in the server's keyed queue (-1: none),
  // whether this round's last fold is a keyed consumer's, and whether a push
  // of the current round was copied into its slot (released behind the copy)
  std::atomic<int> kq_key{-1};
  bool keyed = false;
  bool round_copied = false;
  // a copy of this round is covered only by the lane's copy mark (a batched
  // device copy); otherwise every copy of the round recorded `copied` after
  // itself on the lane's (in-order) copy stream, so the round's fold can wait
  // for its own copies instead of every copy the lane has queued (a worker's
  // push_many of host data queues all its partitions' H2D at once)
  bool round_mark_copy = false;
  hipEvent_t copied = nullptr;
  hipEvent_t pulled = nullptr;  // recorded on the lane's d2h stream after a copying pull
  bool has_done = false;
  // pinned host mirrors of the store for zero-copy pull responses
  // (server.cc:42-70 responds from the store itself).  Sync mode: two, by
  // round parity, filled by ONE D2H per round.  Async mode: a ring of
  // num_workers + 1, one D2H per pull.
  std::vector<char*> mirror;
  std::vector<void*> mirror_dev;  // the same pages as the device sees them
  uint64_t mirror_next = 0;       // async ring position
  hipEvent_t mirrored = nullptr;  // recorded on the lane's d2h stream
  // byteps_server_pull_async requests waiting for this round to finish
  // (the reference's q_pull_reqmeta_, server.cc:304)
  struct Waiting {
    byteps_server_pull_cb cb;
    void* ctx;
  };
  std::vector<Waiting> waiting;
  // byteps_server_pull_into_async requests waiting for this round
  struct WaitingCopy {
    void* dst;           // as the device addresses it
    size_t len;
    byteps_server_pull_cb cb;
    void* ctx;
    const void* view;    // what the callback reports (the caller's pointer)
    SyncWait* direct;    // a blocking pull parked until the round finishes
  };
  std::vector<WaitingCopy> waiting_copies;
};

}  // namespace
}  // namespace bpsr

// A counter bumped by every per-key call: sharded over cache lines by
// calling thread, so receive threads do not bounce one line per call.
struct ShardedCount {
  static constexpr int kShards = 16;
  struct alignas(64) Slot {
    std::atomic<uint64_t> v{0};
  };
  Slot slot[kShards];
  static int shard() {
    static std::atomic<int> next{0};
    thread_local const int mine = next.fetch_add(1, std::memory_order_relaxed) % kShards;
    return mine;
  }
  void add(uint64_t n = 1) { slot[shard()].v.fetch_add(n, std::memory_order_relaxed); }
  uint64_t load() const {
    uint64_t t = 0;
    for (const Slot& x : slot) t += x.v.load(std::memory_order_relaxed);
    return t;
  }
};

struct byteps_server {
  byteps_server_config cfg;
  bool schedule = false;
  bool blocking = false;  // BYTEPS_SERVER_ENGINE_BLOCKING (server.cc:324)
  // lane issuer threads batch single-key calls' folds and device pulls
  // (BPSR_SERVER_COMBINE=0: each call issues its own; off with scheduling or
  // engine blocking, whose orders and completion rules are per call)
  bool combine = true;
  uint64_t inflight = 2;  // issuer: launches queued or running per lane (BPSR_SERVER_INFLIGHT)
  // telemetry (byteps_server_stats)
  std::atomic<uint64_t> n_fold_launches{0}, n_pull_launches{0}, issuer_ns{0},
      n_copy_launches{0};
  ShardedCount n_rounds_folded, n_pulls;
  std::vector<std::unique_ptr<bpsr::Lane>> lanes;
  // every call looks its key up; keys are added once: lookups share the lock
  std::shared_mutex map_mu;
  std::unordered_map<uint64_t, std::unique_ptr<bpsr::KeyState>> keys;
  // ... and first probe a lock-free index of the same keys (open addressing,
  // entries never removed before destroy; filled to half at most, later keys
  // only in the map): a shared lock is an atomic add on one line that every
  // calling thread bounces
  static constexpr size_t kKeyIndex = 1u << 14;
  std::unique_ptr<std::atomic<bpsr::KeyState*>[]> key_index{
      new std::atomic<bpsr::KeyState*>[kKeyIndex]()};
  size_t key_index_n = 0;  // under map_mu
  std::vector<uint64_t> acc_load;  // server.h:112 acc_load_
  // responder thread: SendPullResponse of queued pulls (server.cc:100-114)
  // and SendPushResponse of non-blocking pushes (server.cc:255)
  std::mutex rq_mu;
  std::condition_variable rq_cv;
  std::deque<bpsr::Response> rq;
  bool rq_stop = false;
  std::thread responder;
  // Fault injection for tests (BPSR_SERVER_FAIL_AFTER=n): the (n+1)-th fold
  // issue (init copy or engine job) and every later one fail as a failed
  // kernel launch would.  -1 = off.
  long fail_after = -1;
  std::atomic<long> issued{0};
  // Device releases (BPSR_SERVER_RELEASE=device: sync mode, fused policy, the
  // default engine, N <= 8).  At the first round completion after the init
  // round, ONE keyed block queue is built over every allocated key of that
  // dtype (bpsr::keyq_*: its slots in worker order and its store).  A round's
  // last arrival then stores the key's arrival order and release word
  // instead of issuing a launch (behind the round's copies, a one-lane
  // release kernel on the lane's copy stream), and one consumer launch per
  // epoch folds every key of the queue, each as soon as it is released.
  // Nothing reads a keyed store before lane 0's completer has seen its
  // epoch's consumer complete: pulls parked on it are handed to their lanes
  // then, views wait for it.  A consumer that times out (a key of the queue
  // not pushed within BPSR_SERVER_RELEASE_TIMEOUT_S) fails the keys released
  // in its epoch and turns device releases off for good.
  bool dev_release = false;
  double kq_timeout_s = 5.0;
  std::unique_ptr<bpsr::Lane> klane;  // its completer tracks the consumer launches (no streams)
  std::mutex kq_mu;  // guards the kq_* state below (taken after a key's mu, never before)
  byteps_reduce_blockq* kq = nullptr;
  bool kq_tried = false;
  std::atomic<bool> kq_off{false};
  std::vector<bpsr::KeyState*> kq_keys;  // block -> key
  static constexpr int kKqRing = 64;
  hipEvent_t kq_ev[kKqRing] = {};       // stop event of epoch e at e % kKqRing
  uint64_t kq_ev_seq[kKqRing] = {};     // lane-0 seq of that launch
  uint32_t kq_ev_epoch[kKqRing] = {};
  uint64_t kq_done_seq = 0;             // lane-0 seq up to which keyed epochs are published
  std::atomic<uint32_t> kq_pub_epoch{0};  // epochs launched with their kq_ev slot written
  std::vector<bpsr::PullJob> kq_parked; // pulls of keyed rounds not published yet
  std::atomic<uint64_t> n_consumer_launches{0};
  ShardedCount n_key_releases;
  // Blocking pulls into this device's memory (combine path): served by the
  // pull copy service, created on first use (BPSR_SERVER_PULL_SERVICE=0: the
  // lane issuers' batched copies instead).
  bool pull_service = true;
  std::mutex svc_mu;
  bpsr::CopyService* svc = nullptr;
  bool svc_tried = false;
  std::atomic<uint64_t> n_service_pulls{0}, n_service_pushes{0};
  // order_after's events for those pulls: the service copies on no stream of
  // ours, so a caller event is also waited for on a gate stream whose event
  // the next service pull synchronises on (a blocking call: it waits anyway)
  std::mutex gate_mu;
  hipStream_t gate_stream = nullptr;
  hipEvent_t gate_ev = nullptr;
  std::atomic<uint64_t> gate_seq{0}, gate_done{0};
  // events that bound a push_many's host copies in flight (push_many_host)
  std::mutex ev_pool_mu;
  std::vector<hipEvent_t> ev_pool;
};

namespace bpsr {
namespace {

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
      // release path) for up to 2 ms before a blocking wait — a blocking
      // event wait wakes tens of microseconds late
      const auto p0 = std::chrono::steady_clock::now();
      while (hipEventQuery(t.ev) == hipErrorNotReady) {
        if (std::chrono::steady_clock::now() - p0 > std::chrono::milliseconds(2)) {
          (void)hipEventSynchronize(t.ev);
          break;
        }
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
            bool wait = true) {
  Lane& L = *s->lanes[ks->lane];
  ks->round_copied = true;
  hipError_t e = hipSuccess;
  if (ks->has_done) e = hipStreamWaitEvent(L.copy, ks->fold_ev, 0);
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
  std::unique_lock<std::mutex> kg(s->kq_mu, std::defer_lock);
  bool park = false;
  if (ks->keyed) {  // nothing reads a keyed store before its epoch is published
    kg.lock();
    park = s->kq_done_seq < ks->fold_seq;
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
                 bool mark = true, hipEvent_t batch = nullptr, uint64_t batch_seq = 0,
                 bool keyed = false) {
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
bool keyed_member(byteps_server* s, KeyState* ks) {
  if (!s->dev_release || s->kq_off.load()) return false;
  std::lock_guard<std::mutex> g(s->kq_mu);
  if (!s->kq_tried) {
    s->kq_tried = true;
    build_kq(s, ks->dtype);
  }
  return ks->kq_key.load() >= 0;
}

// Release a finished round of a keyed key (caller holds ks->mu): the arrival
// order and the release word go to the key's block — stored from the host
// when the round's data is in its slots already (push_ready), or by a one-lane
// kernel on `stream` behind the round's copies — after the consumer of the
// block's epoch has been launched (the first release of an epoch launches
// it).  Then the round is published like an issued fold.  Returns 1 when
// device releases were turned off meanwhile (the caller folds with a launch).
int key_release(byteps_server* s, KeyState* ks, const std::vector<int>& order, hipStream_t stream,
                bool skip = false) {
  uint64_t perm = 0;  // position m's worker in bits 4m..4m+3 (16 positions)
  for (size_t m = 0; m < order.size(); ++m) perm |= (uint64_t)order[m] << (4 * m);
  if (skip) perm = ((uint64_t)kKeySkip << 32) | kKeySkip;
  hipEvent_t ev = nullptr;
  uint64_t seq = 0;
  const int kk = ks->kq_key.load();
  uint32_t need = keyq_next_epoch(s->kq, kk);
  Lane& RL = *s->lanes[ks->lane];
  if (!s->kq_off.load() && s->kq_pub_epoch.load(std::memory_order_acquire) >= need) {
    // the epoch's consumer is launched and its slot published: no lock (the
    // slot cannot be reused before this epoch completes, which needs this key)
    const int slot = (int)(need % byteps_server::kKqRing);
    ev = s->kq_ev[slot];
    seq = s->kq_ev_seq[slot];
    if (stream) {
      RL.where = "key_release: wait d2h";
      // behind the lane's pull copies too (a store is rewritten by the fold)
      const hipError_t we = hipStreamWaitEvent(stream, RL.d2h_mark, 0);
      if (we != hipSuccess) return hip_fail(we, "hipStreamWaitEvent");
      RL.where = "key_release: release kernel";
    }
    if (int rc = keyq_release(s->kq, kk, perm, stream)) return rc;
  } else {
    if (stream) RL.where = "key_release: kq_mu";
    std::lock_guard<std::mutex> g(s->kq_mu);
    if (stream) RL.where = "key_release: launch";
    if (s->kq_off.load()) return 1;
    uint32_t launched = 0;
    keyq_state(s->kq, kk, &need, &launched);
    for (; launched < need; launched = keyq_launched(s->kq)) {
      const uint32_t next = launched + 1;
      const int slot = (int)(next % byteps_server::kKqRing);
      if (s->kq_ev_epoch[slot] != 0 && s->kq_done_seq < s->kq_ev_seq[slot])
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
      s->n_consumer_launches.fetch_add(1, std::memory_order_relaxed);
      s->kq_pub_epoch.store(got, std::memory_order_release);  // the fast path may use it now
    }
    if (stream) {
      RL.where = "key_release: wait d2h";
      const hipError_t we = hipStreamWaitEvent(stream, RL.d2h_mark, 0);
      if (we != hipSuccess) return hip_fail(we, "hipStreamWaitEvent");
      RL.where = "key_release: release kernel";
    }
    if (int rc = keyq_release(s->kq, kk, perm, stream)) return rc;
    const int slot = (int)(need % byteps_server::kKqRing);
    ev = s->kq_ev[slot];
    seq = s->kq_ev_seq[slot];
  }
  if (stream) RL.where = "key_release: publish";
  if (skip) return 0;  // the round is folded by a lane launch, which publishes it
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
      }
      s->kq_off.store(true);
      for (KeyState* k : s->kq_keys)
        if (keyq_next_epoch(s->kq, k->kq_key.load()) > epoch) failed.push_back(k);
    }
    s->kq_done_seq = seq;
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
int arrive(byteps_server* s, KeyState* ks, int w, std::vector<FoldJob>* defer = nullptr,
           int pos = -1) {
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
      const int rc = key_release(s, ks, order, nullptr);
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
  j.order = ks->order;
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
      if (!rc && j.ks->keyed && j.ks->has_done && j.ks->fold_ev != last) {
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
      L.done_cv.wait(dl, [&] { return L.issued_seq - L.done_seq < s->inflight; });
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
                         std::vector<FoldJob>* defer = nullptr) {
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

}  // namespace
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
  // the dedicated server process: nothing else waits on its GPU (server.h)
  cfg->release = BYTEPS_SERVER_RELEASE_DEVICE;
  return BYTEPS_REDUCE_OK;
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
  if (const char* fl = getenv("BPSR_SERVER_INFLIGHT")) s->inflight = std::max(1L, atol(fl));
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
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  (void)prio_lo;
  const char* pv = getenv("BPSR_SERVER_D2H_PRIORITY");
  const bool d2h_high = pv && std::string(pv) == "high";
  for (int i = 0; i < cfg->engine_lanes; ++i) {
    s->lanes.push_back(std::make_unique<Lane>());
    Lane& L = *s->lanes.back();
    hipError_t e = hipStreamCreateWithFlags(&L.fold, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&L.copy, hipStreamNonBlocking);
    // d2h streams (mirror copies, copying pulls): normal priority by default;
    // BPSR_SERVER_D2H_PRIORITY=high puts them on a hardware queue of their own
    // (measured: no gain for copying pulls).
    if (e == hipSuccess)
      e = d2h_high ? hipStreamCreateWithPriority(&L.d2h, hipStreamNonBlocking, prio_hi)
                   : hipStreamCreateWithFlags(&L.d2h, hipStreamNonBlocking);
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
    {
      std::lock_guard<std::mutex> g(s->klane->done_mu);
      s->klane->cq_stop = true;
      s->klane->cq_cv.notify_all();
    }
    if (s->klane->completer.joinable()) s->klane->completer.join();
    std::vector<PullJob> parked;
    {
      std::lock_guard<std::mutex> g(s->kq_mu);
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

namespace bpsr {
namespace {
int push_async_impl(byteps_server* s, uint64_t key, int worker, const void* data, size_t len,
                    int dtype, int location, byteps_server_push_cb cb, void* ctx,
                    SyncWait* direct, int pos = -1);
// A blocking call's wait for the lane's launch `seq` to complete.
void wait_lane_done(Lane& L, uint64_t seq) {
  if (spin_until([&] { return L.done_pub.load(std::memory_order_acquire) >= seq; })) return;
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
  return s->svc && !copysvc_broken(s->svc) ? s->svc : nullptr;
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
}  // namespace
}  // namespace bpsr

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
  if ((rc = copy_in(s, ks, worker, data, len, location))) return rc;
  std::vector<FoldJob> defer;
  if ((rc = arrive_and_wait_init(s, ks, worker, lk, s->combine ? &defer : nullptr))) return rc;
  if (!defer.empty()) {
    lk.unlock();
    if (issue_combined(s, defer) && (rc = own_key_status(ks))) return rc;
    lk.lock();
  }
  return s->blocking ? finish_blocking(s, ks, lk) : 0;
}

int byteps_server_push_async(byteps_server* s, uint64_t key, int worker, const void* data,
                             size_t len, int dtype, int location, byteps_server_push_cb cb,
                             void* ctx) {
  return push_async_impl(s, key, worker, data, len, dtype, location, cb, ctx, nullptr);
}

}  // extern "C"

namespace bpsr {
namespace {
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
}  // namespace
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
  if (ks->has_done) {  // the slot may be read by the last issued fold
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
  std::unique_lock<std::mutex> lk(ks->mu);
  ks->cv.wait(lk, [&] { return can_push(s, ks, worker); });
  std::vector<FoldJob> defer;
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

// ------------------------------------------------------- batched calls --

int byteps_server_push_ready_many(byteps_server* s, const uint64_t* keys, int n, int worker) {
  if (!s || (n > 0 && !keys) || n < 0) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (worker < 0 || worker >= s->cfg.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker, s->cfg.num_workers);
  int rc = set_device(s);
  if (rc) return rc;
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
        if (e == hipSuccess && ks->keyed && ks->has_done)
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
        if (ks_of[i]->keyed && ks_of[i]->has_done) waits.push_back(ks_of[i]->fold_ev);
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
    for (hipStream_t st : {L.copy, L.d2h, L.fold}) {
      const hipError_t e = hipStreamWaitEvent(st, ev, 0);
      if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent(caller event)");
    }
  }
  if (s->pull_service && s->combine && !s->cfg.async_mode) {  // the copy service's gate
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
  const uint64_t v[11] = {s->n_fold_launches.load(), s->n_rounds_folded.load(),
                          s->n_pull_launches.load(), s->n_pulls.load(), s->issuer_ns.load(),
                          s->n_copy_launches.load(), s->n_consumer_launches.load(),
                          s->n_key_releases.load(), s->n_service_pulls.load(), svc_launches,
                          s->n_service_pushes.load()};
  for (int i = 0; i < n && i < 11; ++i) out[i] = v[i];
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
