// The GPU-resident PS server's state and helpers, shared by its sources
// (not part of the C ABI):
//   bpsr_server.cpp          lanes, issuer / completer / responder threads, the
//                            per-key state machine, the single-key C calls
//   bpsr_server_keyed.cpp    device releases (the keyed block queue)
//   bpsr_server_service.cpp  blocking calls through the pull copy service,
//                            lane waits, order_after's gate
//   bpsr_server_batched.cpp  push_ready_many / push_many / pull_many
#pragma once

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
inline namespace srv {

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
struct SyncWait {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  int status = 0;
  Lane* lane = nullptr;  // a direct pull or push: the launch its copy rides in
  uint64_t seq = 0;
  int wait() {
    // the waiter returns (and the caller's frame goes) only after finish()
    // has let go of mu
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done; });
    return status;
  }
  void finish(int st) {
    std::lock_guard<std::mutex> g(mu);
    status = st;
    done = true;
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
  std::vector<int> order_spare;  // a buffer for the next round's order (recycle_order)
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

}  // namespace srv
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
  // the issuer keeps at most this many of its lane's launches queued or
  // running (1 and 4 measured neutral against 2, profiles/r03_server_inflight.jsonl)
  static constexpr uint64_t kInflight = 2;
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
  std::atomic<bool> kq_tried{false};  // the keyed queue was built or refused (set once)
  std::atomic<bool> kq_off{false};
  std::atomic<bool> kq_stopping{false};  // destroy: retire an idle epoch at once
  std::vector<bpsr::KeyState*> kq_keys;  // block -> key
  static constexpr int kKqRing = 64;
  // an epoch launched ahead that no round begins within this is retired
  // (kq_retire): its consumer would otherwise hold two workgroup slots per CU
  // and keep device-wide waits (hipDeviceSynchronize, NULL-stream copies) open
  static constexpr int kKeyedIdleUs = 1000;
  hipEvent_t kq_ev[kKqRing] = {};       // stop event of epoch e at e % kKqRing
  uint64_t kq_ev_seq[kKqRing] = {};     // lane-0 seq of that launch
  uint32_t kq_ev_epoch[kKqRing] = {};
  // lane-0 seq up to which keyed epochs are published, and the pulls parked
  // on later ones: under kq_park_mu (never held together with kq_mu, which a
  // consumer launch holds), so a round's pulls are never queued behind a launch
  std::mutex kq_park_mu;
  std::atomic<uint64_t> kq_done_seq{0};
  std::atomic<uint32_t> kq_pub_epoch{0};  // epochs launched with their kq_ev slot written
  // Per-epoch release choice (round 6): an epoch's kind is decided in epoch
  // order, by its first release or by its consumer's launch (ahead): a
  // consumer epoch is folded by a keyed consumer launch; a lane epoch — opened
  // by a copied round while no consumer was launched for it — has none, and
  // every round in it folds with a lane launch (its keys only get skip words,
  // which keep their epochs in step).  kq_kind[e % kKqRing] is written before
  // kq_decided publishes e.
  static constexpr uint8_t kConsumerEpoch = 1, kLaneEpoch = 2;
  uint8_t kq_kind[kKqRing] = {};
  std::atomic<uint32_t> kq_decided{0};
  // the highest epoch a slot-written round was released into (a consumer
  // epoch with one launches its successor ahead; an all-copied one does not)
  std::atomic<uint32_t> kq_slot_epoch{0};
  // a consumer epoch still open this long after its first release is closed:
  // its keys not released yet get skip words and their rounds go to the next
  // epoch (kq_close_epoch) — no key has to be pushed in every epoch
  static constexpr int kKeyedCloseMs = 100;
  std::atomic<uint64_t> n_epochs_closed{0}, n_lane_epochs{0};
  std::vector<bpsr::PullJob> kq_parked; // pulls of keyed rounds not published yet (kq_park_mu)
  std::atomic<uint64_t> n_consumer_launches{0};  // epochs a round was released for
  std::atomic<uint64_t> n_consumer_retired{0};   // epochs launched ahead and retired idle
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
inline namespace srv {

int force_device(const byteps_server* s);
int set_device(const byteps_server* s);
int bind_cached(const byteps_server* s);
hipError_t wait_pull_copies(Lane& L);
hipError_t wait_copies(Lane& L);
uint64_t track(Lane& L, hipEvent_t ev);
uint64_t track_keyed(Lane& L, hipEvent_t ev, uint32_t epoch);
void completer_main(byteps_server* s, Lane* Lp);
int pick_lane(byteps_server* s, size_t len);
size_t key_slot(uint64_t key);
KeyState* get_key(byteps_server* s, uint64_t key, bool create);
int key_error(const KeyState* ks);
int allocate(byteps_server* s, KeyState* ks, size_t len, int dtype);
bool can_push(const byteps_server* s, const KeyState* ks, int w);
int copy_in(byteps_server* s, KeyState* ks, int w, const void* data, size_t len, int loc,
            bool wait = true);
int queue_mirror(byteps_server* s, KeyState* ks, size_t idx);
int ensure_mirror(byteps_server* s, KeyState* ks, bool queue_now);
void enqueue_response(byteps_server* s, const Response& r);
void respond_later(byteps_server* s, KeyState* ks, byteps_server_pull_cb cb, void* ctx,
                   const char* view, int status);
bool pull_ready(const byteps_server* s, const KeyState* ks);
void count_pull(byteps_server* s, KeyState* ks);
void fail_key(byteps_server* s, KeyState* ks, int rc);
void queue_pull_copies(byteps_server* s, KeyState* ks, const KeyState::WaitingCopy* wcs, size_t n);
void responder_main(byteps_server* s);
int finish_round(byteps_server* s, KeyState* ks, const std::vector<int>& order,
                 bool mark = true, hipEvent_t batch = nullptr, uint64_t batch_seq = 0,
                 bool keyed = false);
int injected_failure(byteps_server* s);
void build_kq(byteps_server* s, int dtype);
bool keyed_member(byteps_server* s, KeyState* ks);
bool wait_keyed_slots(byteps_server* s, int kq_key, uint32_t epoch);
bool wait_keyed_slots(byteps_server* s, const KeyState* ks);
int key_release(byteps_server* s, KeyState* ks, const std::vector<int>& order, hipStream_t stream,
                bool skip = false);
int kq_launch_upto(byteps_server* s, uint32_t need);
void kq_launch_ahead(byteps_server* s, uint32_t epoch);
bool kq_retire(byteps_server* s, uint32_t epoch);
void kq_close_epoch(byteps_server* s, uint32_t epoch);
void kq_epoch_done(byteps_server* s, uint32_t epoch, uint64_t seq);
void wait_published(byteps_server* s, KeyState* ks, uint64_t seq);
int execute(byteps_server* s, const FoldJob& j);
int submit(byteps_server* s, KeyState* ks, FoldJob&& j);
void dispatcher_main(byteps_server* s, int lane);
int check_pos(const byteps_server* s, const KeyState* ks, int pos);
int arrive(byteps_server* s, KeyState* ks, int w, std::vector<FoldJob>* defer = nullptr,
           int pos = -1);
int flush_folds(byteps_server* s, std::vector<FoldJob>& jobs);
int finish_blocking(byteps_server* s, KeyState* ks, std::unique_lock<std::mutex>& lk);
int issue_one(byteps_server* s, FoldJob& j);
void recycle_order(KeyState* ks, FoldJob& j);
int issue_combined(byteps_server* s, std::vector<FoldJob>& jobs);
int issue_deferred(byteps_server* s, std::vector<FoldJob>& jobs);
void issue_copies(byteps_server* s, Lane& L, std::vector<CopyJob>& jobs);
void issue_pull_copies(byteps_server* s, Lane& L, std::vector<PullJob>& jobs);
void issuer_main(byteps_server* s, int lane);
int own_key_status(KeyState* ks);
int arrive_and_wait_init(byteps_server* s, KeyState* ks, int w, std::unique_lock<std::mutex>& lk,
                         std::vector<FoldJob>* defer = nullptr);
void* device_view(void* out, int location);
void* pull_kernel_dst(void* out, int location);
KeyState* key_for_pull(byteps_server* s, uint64_t key);
void destroy_lanes(byteps_server* s);
void wait_lane_done(Lane& L, uint64_t seq);
void wait_round_fold(byteps_server* s, Lane& FL, uint64_t need, int kq_key, uint32_t kq_epoch);
CopyService* service_get(byteps_server* s);
bool on_this_device(const byteps_server* s, const void* p);
CopyService* service_for(byteps_server* s, void* out, size_t len);
const void* service_src(byteps_server* s, const void* data, size_t len, int location);
int fallback_copy(byteps_server* s, KeyState* ks, void* dst, const void* src, size_t len);
int wait_order_gate(byteps_server* s);
int service_pull(byteps_server* s, CopyService* svc, KeyState* ks, void* out, size_t len);
int service_push(byteps_server* s, CopyService* svc, uint64_t key, int worker, const void* src,
                 size_t len, int dtype);
void sync_push_cb(void* ctx, uint64_t, int, int status);
int sync_status(byteps_server* s, uint64_t key, int status, const char* what);
// byteps_server_push_async; with `direct`, a blocking push's issuer-batched
// copy reports to its waiter (bpsr_server.cpp)
int push_async_impl(byteps_server* s, uint64_t key, int worker, const void* data, size_t len,
                    int dtype, int location, byteps_server_push_cb cb, void* ctx,
                    SyncWait* direct, int pos = -1);
// the responder thread (its own calls copy directly)
extern thread_local bool t_responder;
// push_many from host memory, key by key (bpsr_server_batched.cpp)
int push_many_host(byteps_server* s, std::vector<KeyState*>& ks_of, const void* const* datas,
                   const size_t* lens, int n, int worker);

}  // namespace srv
}  // namespace bpsr
