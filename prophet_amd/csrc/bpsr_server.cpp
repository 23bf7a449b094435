// GPU-resident parameter-server aggregation (include/bpsr/server.h): the
// per-key state machine of byteps/server/server.cc:147-308 with the engine
// threads (server.cc:70-145) replaced by HIP stream lanes and the CpuReducer
// calls replaced by the gfx950 fold kernels.
#include "bpsr/server.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <deque>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "bpsr_internal.h"

namespace bpsr {
namespace {

constexpr size_t kSlotAlign = 4096;
constexpr size_t kSlotSkew = 16 * 1024;  // prophet_amd/arena.py: skewed slots

struct Lane {
  hipStream_t fold = nullptr;  // folds, in round order per key
  hipStream_t copy = nullptr;  // push/pull copies
  hipStream_t d2h = nullptr;   // per-round store -> host mirror copies
};

struct KeyState {
  uint64_t key = 0;
  std::mutex mu;
  std::condition_variable cv;
  bool allocated = false;
  bool inited = false;        // store initialised (round 0 done)
  size_t len = 0;
  int dtype = 0;
  int lane = 0;
  char* arena = nullptr;      // N receive slots + store
  size_t stride = 0;
  std::vector<char*> slot;
  char* store = nullptr;
  // current round
  std::vector<char> got;      // worker pushed this round
  std::vector<int> order;     // arrival order this round
  int arrived = 0;
  int init_count = 0;
  // completion / pull gating (server.cc:100-114, 280-306)
  uint64_t rounds = 0;
  bool push_finished = false;
  int pull_cnt = 0;
  std::vector<int> last_order;
  hipEvent_t done = nullptr;  // recorded on the lane's fold stream after the round
  hipEvent_t copied = nullptr;
  bool has_done = false;
  // pinned host mirror of the store for zero-copy pull responses
  // (byteps_server_pull_host_view; server.cc:42-70 responds from the store
  // itself).  Two buffers by round parity, filled by ONE D2H per round.
  char* mirror[2] = {nullptr, nullptr};
  void* mirror_dev[2] = {nullptr, nullptr};  // the same pages as the device sees them
  hipEvent_t mirrored = nullptr;  // recorded on the lane's d2h stream
  // byteps_server_pull_async requests waiting for this round to finish
  // (the reference's q_pull_reqmeta_, server.cc:304)
  struct Waiting {
    byteps_server_pull_cb cb;
    void* ctx;
  };
  std::vector<Waiting> waiting;
};

// A pull ready to be answered by the responder thread.
struct Response {
  uint64_t key;
  KeyState* ks;
  byteps_server_pull_cb cb;
  void* ctx;
  const char* view;  // mirror holding the answered round
  int status;
  byteps_server_push_cb push_cb = nullptr;  // set: a push acknowledgement
  int worker = -1;
};

}  // namespace
}  // namespace bpsr

struct byteps_server {
  byteps_server_config cfg;
  std::vector<bpsr::Lane> lanes;
  std::mutex map_mu;
  std::unordered_map<uint64_t, std::unique_ptr<bpsr::KeyState>> keys;
  std::vector<uint64_t> acc_load;  // server.h:112 acc_load_
  // responder thread for byteps_server_pull_async (the engine threads'
  // SendPullResponse of queued pulls, server.cc:100-114)
  std::mutex rq_mu;
  std::condition_variable rq_cv;
  std::deque<bpsr::Response> rq;
  bool rq_stop = false;
  std::thread responder;
};

namespace bpsr {
namespace {

int set_device(const byteps_server* s) {
  hipError_t e = hipSetDevice(s->cfg.device);
  return e == hipSuccess ? 0 : hip_fail(e, "hipSetDevice");
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

KeyState* get_key(byteps_server* s, uint64_t key, bool create) {
  std::lock_guard<std::mutex> g(s->map_mu);
  auto it = s->keys.find(key);
  if (it != s->keys.end()) return it->second.get();
  if (!create) return nullptr;
  auto ks = std::make_unique<KeyState>();
  ks->key = key;
  KeyState* p = ks.get();
  s->keys.emplace(key, std::move(ks));
  return p;
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
  ks->stride = (len + kSlotAlign - 1) / kSlotAlign * kSlotAlign + kSlotSkew;
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
  ks->len = len;
  ks->dtype = dtype;
  {
    std::lock_guard<std::mutex> g(s->map_mu);
    ks->lane = pick_lane(s, len);
  }
  ks->allocated = true;
  return 0;
}

// Bring `len` bytes into worker `w`'s slot on the lane's copy stream, after
// the previous round's fold has consumed the slot; wait for the copy.
int copy_in(byteps_server* s, KeyState* ks, int w, const void* data, size_t len, int loc,
            bool wait = true) {
  Lane& L = s->lanes[ks->lane];
  hipError_t e = hipSuccess;
  if (ks->has_done) e = hipStreamWaitEvent(L.copy, ks->done, 0);
  if (e == hipSuccess)
    e = hipMemcpyAsync(ks->slot[w], data, len,
                       loc == BYTEPS_SERVER_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice,
                       L.copy);
  if (e == hipSuccess) e = hipEventRecord(ks->copied, L.copy);
  if (e == hipSuccess && wait) e = hipEventSynchronize(ks->copied);
  return e == hipSuccess ? 0 : hip_fail(e, "push copy");
}

// Queue the D2H of the store into mirror[round & 1] on the lane's d2h stream,
// behind the round's fold (caller holds ks->mu).  Its own stream, so the copy
// overlaps the H2D pushes of the lane's other keys (PCIe is full duplex).
int queue_mirror(byteps_server* s, KeyState* ks, uint64_t round) {
  Lane& L = s->lanes[ks->lane];
  hipError_t e = ks->has_done ? hipStreamWaitEvent(L.d2h, ks->done, 0) : hipSuccess;
  if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent");
  // The copy kernel writes the pinned mirror straight over PCIe.  A
  // hipMemcpyAsync D2H queued behind a pending event wait was handed to an SDMA
  // engine that ran at ~13 GB/s beside the H2D pushes (rocprofv3 memory-copy
  // trace); the kernel path runs at the link's rate.
  int rc = byteps_reduce_copy(ks->mirror_dev[round & 1], ks->store, ks->len,
                              reinterpret_cast<void*>(L.d2h));
  if (rc) return rc;
  e = hipEventRecord(ks->mirrored, L.d2h);
  return e == hipSuccess ? 0 : hip_fail(e, "store mirror copy");
}

// Pin the key's two store mirrors on first use (fixed addresses from then on,
// as server.cc:60-69 reuses its response buffer to avoid re-registering
// memory); with queue_now, also mirror the finished current round.  Caller
// holds ks->mu.
int ensure_mirror(byteps_server* s, KeyState* ks, bool queue_now) {
  if (ks->mirror[0]) return 0;
  hipError_t e;
  for (int i = 0; i < 2; ++i) {
    void* p = nullptr;
    if ((e = hipHostMalloc(&p, ks->len, hipHostMallocDefault)) != hipSuccess)
      return hip_fail(e, "hipHostMalloc(store mirror)");
    ks->mirror[i] = static_cast<char*>(p);
    if ((e = hipHostGetDevicePointer(&ks->mirror_dev[i], p, 0)) != hipSuccess)
      return hip_fail(e, "hipHostGetDevicePointer(store mirror)");
  }
  if ((e = hipEventCreateWithFlags(&ks->mirrored, hipEventDisableTiming)) != hipSuccess)
    return hip_fail(e, "hipEventCreate");
  return queue_now ? queue_mirror(s, ks, ks->rounds) : 0;
}

// Hand a ready pull of the current round to the responder (caller holds ks->mu).
void respond_later(byteps_server* s, uint64_t key, KeyState* ks, byteps_server_pull_cb cb,
                   void* ctx, int status) {
  Response r{key, ks, cb, ctx, ks->mirror[ks->rounds & 1], status};
  std::lock_guard<std::mutex> g(s->rq_mu);
  s->rq.push_back(r);
  s->rq_cv.notify_one();
}

// Count one answered pull; after NumWorkers the key re-arms (server.cc:105-113).
// Caller holds ks->mu.
void count_pull(byteps_server* s, KeyState* ks) {
  if (s->cfg.async_mode) return;
  if (++ks->pull_cnt == s->cfg.num_workers) {
    ks->push_finished = false;
    ks->pull_cnt = 0;
  }
  ks->cv.notify_all();
}

void responder_main(byteps_server* s) {
  (void)hipSetDevice(s->cfg.device);
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
      hipError_t e = hipEventSynchronize(r.ks->copied);
      r.push_cb(r.ctx, r.key, r.worker, e == hipSuccess ? 0 : hip_fail(e, "push copy sync"));
      continue;
    }
    int status = r.status;
    if (status == 0) {
      // The event still names this round's copy: the next round cannot finish
      // before this pull is counted below.
      hipError_t e = hipEventSynchronize(r.ks->mirrored);
      if (e != hipSuccess) status = hip_fail(e, "store mirror sync");
    }
    r.cb(r.ctx, r.key, status == 0 ? r.view : nullptr, status == 0 ? r.ks->len : 0, status);
    if (r.status == 0) {
      std::lock_guard<std::mutex> g(r.ks->mu);
      count_pull(s, r.ks);
    }
  }
}

// A push's bytes are in slot w: advance the state machine (caller holds ks->mu).
int arrive(byteps_server* s, KeyState* ks, int w) {
  const int N = s->cfg.num_workers;
  Lane& L = s->lanes[ks->lane];
  void* fold_stream = reinterpret_cast<void*>(L.fold);
  int rc = 0;
  // Folds run behind the slots' H2D copies (byteps_server_push_async returns
  // before they finish; the copy stream is in order, so the last recorded copy
  // covers every earlier one) and behind the last mirror D2H of the store.
  hipError_t we = hipStreamWaitEvent(L.fold, ks->copied, 0);
  if (we == hipSuccess && ks->mirror[0]) we = hipStreamWaitEvent(L.fold, ks->mirrored, 0);
  if (we != hipSuccess) return hip_fail(we, "hipStreamWaitEvent");
  if (!ks->inited) {
    // Round 0: server.cc:175-199 — after all NumWorkers init pushes the store
    // is initialised by copying the LAST arrived push.
    if (ks->got[w]) return fail(BYTEPS_REDUCE_EARGS, "worker %d sent two init pushes", w);
    ks->got[w] = 1;
    if (++ks->init_count < N) return 0;
    rc = byteps_reduce_copy(ks->store, ks->slot[w], ks->len, fold_stream);
    if (rc) return rc;
    hipError_t e = hipEventRecord(ks->done, L.fold);
    if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
    ks->has_done = true;
    ks->inited = true;
    std::fill(ks->got.begin(), ks->got.end(), 0);
    ks->cv.notify_all();
    return 0;
  }
  if (s->cfg.async_mode) {
    // server.cc:220-230: every push is summed straight into the store.
    rc = byteps_reduce_sum(ks->store, ks->slot[w], ks->len, ks->dtype, fold_stream);
    if (rc) return rc;
    hipError_t e = hipEventRecord(ks->done, L.fold);
    if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
    ks->has_done = true;
    ks->rounds++;
    ks->cv.notify_all();
    return 0;
  }
  if (ks->got[w]) return fail(BYTEPS_REDUCE_EARGS, "worker %d pushed twice in one round", w);
  ks->got[w] = 1;
  ks->order.push_back(w);
  ks->arrived++;
  if (s->cfg.policy == BYTEPS_SERVER_INCREMENTAL && ks->arrived > 1) {
    // SUM_RECV (server.cc:117-139): merged (= first arrival's slot) += this push
    rc = byteps_reduce_sum(ks->slot[ks->order[0]], ks->slot[w], ks->len, ks->dtype, fold_stream);
    if (rc) return rc;
  }
  if (ks->arrived < N) return 0;
  if (s->cfg.policy == BYTEPS_SERVER_INCREMENTAL) {
    // COPY_MERGED (server.cc:82-115)
    rc = byteps_reduce_copy(ks->store, ks->slot[ks->order[0]], ks->len, fold_stream);
  } else {
    // one fused left fold in arrival order straight into the store
    std::vector<const void*> srcs(N);
    for (int k = 0; k < N; ++k) srcs[k] = ks->slot[ks->order[k]];
    rc = byteps_reduce_sum_n(ks->store, srcs.data(), N, ks->len, ks->dtype,
                             BYTEPS_REDUCE_MODE_REFERENCE, fold_stream);
  }
  if (rc) return rc;
  hipError_t e = hipEventRecord(ks->done, L.fold);
  if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
  ks->has_done = true;
  if (ks->mirror[0] && (rc = queue_mirror(s, ks, ks->rounds + 1))) return rc;
  ks->last_order = ks->order;
  ks->order.clear();
  ks->arrived = 0;
  std::fill(ks->got.begin(), ks->got.end(), 0);
  ks->rounds++;
  ks->push_finished = true;
  ks->pull_cnt = 0;
  for (auto& wp : ks->waiting) respond_later(s, ks->key, ks, wp.cb, wp.ctx, 0);
  ks->waiting.clear();
  ks->cv.notify_all();
  return 0;
}

// Init pushes block until every worker's init push has arrived and the store
// is initialised: the reference answers them only then (server.cc:184-198).
int arrive_and_wait_init(byteps_server* s, KeyState* ks, int w, std::unique_lock<std::mutex>& lk) {
  const bool init_round = !ks->inited;
  int rc = arrive(s, ks, w);
  if (rc || !init_round) return rc;
  ks->cv.wait(lk, [&] { return ks->inited; });
  return 0;
}

// Per-thread stream for pull copies (a pull blocks only on its own copy).
hipStream_t pull_stream(int device) {
  thread_local hipStream_t st = nullptr;
  thread_local int dev = -1;
  if (st && dev == device) return st;
  if (st) (void)hipStreamDestroy(st);
  st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) st = nullptr;
  dev = device;
  return st;
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
  int rc = set_device(s.get());
  if (rc) return rc;
  s->lanes.resize(cfg->engine_lanes);
  s->acc_load.assign(cfg->engine_lanes, 0);
  for (auto& L : s->lanes) {
    hipError_t e = hipStreamCreateWithFlags(&L.fold, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&L.copy, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&L.d2h, hipStreamNonBlocking);
    if (e != hipSuccess) {
      byteps_server_destroy(s.release());
      return hip_fail(e, "hipStreamCreate");
    }
  }
  try {
    s->responder = std::thread(responder_main, s.get());
  } catch (...) {
    byteps_server_destroy(s.release());
    return fail(BYTEPS_REDUCE_EARGS, "cannot start the pull responder thread");
  }
  *out = s.release();
  return BYTEPS_REDUCE_OK;
}

int byteps_server_destroy(byteps_server* s) {
  if (!s) return BYTEPS_REDUCE_OK;
  (void)hipSetDevice(s->cfg.device);
  if (s->responder.joinable()) {
    for (auto& kv : s->keys) {  // pulls whose round never finished: cancelled
      KeyState* ks = kv.second.get();
      std::lock_guard<std::mutex> g(ks->mu);
      for (auto& wp : ks->waiting)
        respond_later(s, kv.first, ks, wp.cb, wp.ctx, BYTEPS_REDUCE_ECANCELED);
      ks->waiting.clear();
    }
    {
      std::lock_guard<std::mutex> g(s->rq_mu);
      s->rq_stop = true;
    }
    s->rq_cv.notify_all();
    s->responder.join();
  }
  for (auto& L : s->lanes) {
    if (L.fold) (void)hipStreamSynchronize(L.fold);
    if (L.copy) (void)hipStreamSynchronize(L.copy);
    if (L.d2h) (void)hipStreamSynchronize(L.d2h);
  }
  for (auto& kv : s->keys) {
    KeyState* ks = kv.second.get();
    if (ks->done) (void)hipEventDestroy(ks->done);
    if (ks->copied) (void)hipEventDestroy(ks->copied);
    if (ks->mirrored) (void)hipEventDestroy(ks->mirrored);
    for (char* m : ks->mirror)
      if (m) (void)hipHostFree(m);
    if (ks->arena) (void)hipFree(ks->arena);
  }
  for (auto& L : s->lanes) {
    if (L.fold) (void)hipStreamDestroy(L.fold);
    if (L.copy) (void)hipStreamDestroy(L.copy);
    if (L.d2h) (void)hipStreamDestroy(L.d2h);
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

int byteps_server_push(byteps_server* s, uint64_t key, int worker, const void* data, size_t len,
                       int dtype, int location) {
  if (!s || !data) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (worker < 0 || worker >= s->cfg.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker, s->cfg.num_workers);
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = get_key(s, key, true);
  std::unique_lock<std::mutex> lk(ks->mu);
  if ((rc = allocate(s, ks, len, dtype))) return rc;
  if (s->cfg.async_mode == 0 && ks->inited && ks->got[worker]) {
    // A worker's next-round push may arrive while the key still waits for the
    // other workers' pulls of this round; hold it until the key re-arms.
    ks->cv.wait(lk, [&] { return !ks->got[worker]; });
  }
  if ((rc = copy_in(s, ks, worker, data, len, location))) return rc;
  return arrive_and_wait_init(s, ks, worker, lk);
}

int byteps_server_push_async(byteps_server* s, uint64_t key, int worker, const void* data,
                             size_t len, int dtype, int location, byteps_server_push_cb cb,
                             void* ctx) {
  if (!s || !data || !cb) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (worker < 0 || worker >= s->cfg.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker, s->cfg.num_workers);
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = get_key(s, key, true);
  std::unique_lock<std::mutex> lk(ks->mu);
  if ((rc = allocate(s, ks, len, dtype))) return rc;
  if (s->cfg.async_mode == 0 && ks->inited && ks->got[worker])
    ks->cv.wait(lk, [&] { return !ks->got[worker]; });
  if ((rc = copy_in(s, ks, worker, data, len, location, /*wait=*/false))) return rc;
  if ((rc = arrive(s, ks, worker))) {  // arrival order = call order
    // the caller gets its buffer back on error: let the queued copy finish first
    (void)hipEventSynchronize(ks->copied);
    return rc;
  }
  Response r{key, ks, nullptr, ctx, nullptr, 0, cb, worker};
  std::lock_guard<std::mutex> g(s->rq_mu);
  s->rq.push_back(r);
  s->rq_cv.notify_one();
  return BYTEPS_REDUCE_OK;
}

int byteps_server_recv_slot(byteps_server* s, uint64_t key, int worker, void** slot) {
  if (!s || !slot) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (worker < 0 || worker >= s->cfg.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker, s->cfg.num_workers);
  KeyState* ks = get_key(s, key, false);
  if (!ks || !ks->allocated)
    return fail(BYTEPS_REDUCE_EARGS, "key %llu not initialised (byteps_server_init_key)",
                (unsigned long long)key);
  std::lock_guard<std::mutex> g(ks->mu);
  if (ks->has_done) {  // the slot may be read by the last queued fold
    hipError_t e = hipEventSynchronize(ks->done);
    if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
  }
  *slot = ks->slot[worker];
  return BYTEPS_REDUCE_OK;
}

int byteps_server_push_ready(byteps_server* s, uint64_t key, int worker) {
  if (!s) return fail(BYTEPS_REDUCE_EARGS, "null server");
  if (worker < 0 || worker >= s->cfg.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker, s->cfg.num_workers);
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = get_key(s, key, false);
  if (!ks || !ks->allocated) return fail(BYTEPS_REDUCE_EARGS, "key not initialised");
  std::unique_lock<std::mutex> lk(ks->mu);
  return arrive_and_wait_init(s, ks, worker, lk);
}

int byteps_server_pull(byteps_server* s, uint64_t key, void* out, size_t len, int location) {
  if (!s || !out) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = get_key(s, key, false);
  if (!ks || !ks->allocated)  // server.cc:282-283
    return fail(BYTEPS_REDUCE_EARGS,
                "Processing pull request when the key %llu has not been inited yet",
                (unsigned long long)key);
  std::unique_lock<std::mutex> lk(ks->mu);
  if (len > ks->len) return fail(BYTEPS_REDUCE_EARGS, "pull of %zu bytes > key len %zu", len, ks->len);
  if (!s->cfg.async_mode) ks->cv.wait(lk, [&] { return ks->push_finished; });
  hipStream_t cs = pull_stream(s->cfg.device);
  if (!cs) return fail(BYTEPS_REDUCE_EHIP, "cannot create the pull stream");
  // Order the copy after the round's fold while still holding the key lock
  // (async mode keeps adding into the store); the copy itself runs unlocked.
  hipError_t e = ks->has_done ? hipStreamWaitEvent(cs, ks->done, 0) : hipSuccess;
  lk.unlock();
  // In sync mode the store cannot change while this pull is outstanding: the
  // next round needs this worker's next push, which follows the pull.
  if (e == hipSuccess)
    e = hipMemcpyAsync(out, ks->store, len,
                       location == BYTEPS_SERVER_HOST ? hipMemcpyDeviceToHost
                                                      : hipMemcpyDeviceToDevice, cs);
  if (e == hipSuccess) e = hipStreamSynchronize(cs);
  if (e != hipSuccess) return hip_fail(e, "pull copy");
  lk.lock();
  if (!s->cfg.async_mode) {
    // server.cc:105-113: after NumWorkers pulls the key re-arms
    if (++ks->pull_cnt == s->cfg.num_workers) {
      ks->push_finished = false;
      ks->pull_cnt = 0;
    }
    ks->cv.notify_all();
  }
  return BYTEPS_REDUCE_OK;
}

int byteps_server_pull_host_view(byteps_server* s, uint64_t key, const void** data,
                                 size_t* len) {
  if (!s || !data) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  *data = nullptr;
  if (len) *len = 0;
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = get_key(s, key, false);
  if (!ks || !ks->allocated)  // server.cc:282-283
    return fail(BYTEPS_REDUCE_EARGS,
                "Processing pull request when the key %llu has not been inited yet",
                (unsigned long long)key);
  std::unique_lock<std::mutex> lk(ks->mu);
  if (!s->cfg.async_mode) ks->cv.wait(lk, [&] { return ks->push_finished; });
  hipError_t e = hipSuccess;
  if ((rc = ensure_mirror(s, ks, !s->cfg.async_mode))) return rc;
  // async mode: the store changes with every push, so each view is a fresh D2H
  if (s->cfg.async_mode && (rc = queue_mirror(s, ks, ks->rounds))) return rc;
  const char* view = ks->mirror[ks->rounds & 1];
  hipEvent_t ev = ks->mirrored;
  lk.unlock();
  // The event still names this round's copy: the next round cannot finish
  // before this pull is counted below.
  if ((e = hipEventSynchronize(ev)) != hipSuccess) return hip_fail(e, "store mirror sync");
  lk.lock();
  count_pull(s, ks);
  *data = view;
  if (len) *len = ks->len;
  return BYTEPS_REDUCE_OK;
}

int byteps_server_pull_async(byteps_server* s, uint64_t key, byteps_server_pull_cb cb,
                             void* ctx) {
  if (!s || !cb) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  int rc = set_device(s);
  if (rc) return rc;
  KeyState* ks = get_key(s, key, false);
  if (!ks || !ks->allocated)  // server.cc:282-283
    return fail(BYTEPS_REDUCE_EARGS,
                "Processing pull request when the key %llu has not been inited yet",
                (unsigned long long)key);
  std::lock_guard<std::mutex> g(ks->mu);
  if (s->cfg.async_mode) {  // answered at once from a fresh copy of the store
    if ((rc = ensure_mirror(s, ks, false)) || (rc = queue_mirror(s, ks, ks->rounds))) return rc;
    respond_later(s, key, ks, cb, ctx, 0);
    return BYTEPS_REDUCE_OK;
  }
  if ((rc = ensure_mirror(s, ks, ks->push_finished))) return rc;
  if (ks->push_finished)  // server.cc:293-301: push already finished
    respond_later(s, key, ks, cb, ctx, 0);
  else                    // server.cc:303-304: queued until the round finishes
    ks->waiting.push_back({cb, ctx});
  return BYTEPS_REDUCE_OK;
}

int byteps_server_key_info(byteps_server* s, uint64_t key, uint64_t* rounds, int* lane,
                           int* last_order, int max_order) {
  if (!s) return fail(BYTEPS_REDUCE_EARGS, "null server");
  KeyState* ks = get_key(s, key, false);
  if (!ks) return fail(BYTEPS_REDUCE_EARGS, "unknown key");
  std::lock_guard<std::mutex> g(ks->mu);
  if (rounds) *rounds = ks->rounds;
  if (lane) *lane = ks->lane;
  if (last_order)
    for (int i = 0; i < max_order && i < (int)ks->last_order.size(); ++i)
      last_order[i] = ks->last_order[i];
  return BYTEPS_REDUCE_OK;
}

}  // extern "C"
