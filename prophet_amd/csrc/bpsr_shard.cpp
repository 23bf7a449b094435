// Key-space sharding across the GPUs of a node (include/bpsr/shard.h): the
// worker local reduce of byteps/common/core_loops.cc:184-263 and the scatter
// of landed buckets to their owners, as point-to-point transfers plus the
// gfx950 rank-order fold.
//
// Transfers go through one of two transports behind the same group-of-P2P
// interface: RCCL (grouped ncclSend/ncclRecv, plus ncclAllGather /
// ncclBroadcast for the return legs) or an in-process group (one process
// driving several GPUs: device copies between the ranks' buffers, ordered by
// HIP events, with a host rendezvous per transfer).  RCCL is resolved with
// dlopen at first use, so the library carries no link dependency on it and,
// inside a process that already loaded an RCCL (torch's), uses that one.
#include "bpsr/shard.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "bpsr_internal.h"

namespace bpsr {
namespace {

// ------------------------------------------------------------------ RCCL --
struct Rccl {
  bool ok = false;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommUserRank)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommCuDevice)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t,
                            hipStream_t) = nullptr;
  const char* (*ErrorString)(ncclResult_t) = nullptr;
  ncclResult_t (*GetVersion)(int*) = nullptr;  // optional (byteps_shard_rccl_version)
};

template <class F>
bool sym(void* h, const char* name, F* out) {
  *out = reinterpret_cast<F>(dlsym(h, name));
  return *out != nullptr;
}

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    // An RCCL already in the process (torch's) is found by soname first;
    // otherwise the search path (libbpsr.so's runpath: the ROCm lib dir).
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      x.err = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
      return x;
    }
    bool ok = sym(h, "ncclGetUniqueId", &x.GetUniqueId) &&
              sym(h, "ncclCommInitRank", &x.CommInitRank) &&
              sym(h, "ncclCommDestroy", &x.CommDestroy) &&
              sym(h, "ncclCommCount", &x.CommCount) &&
              sym(h, "ncclCommUserRank", &x.CommUserRank) &&
              sym(h, "ncclCommCuDevice", &x.CommCuDevice) && sym(h, "ncclSend", &x.Send) &&
              sym(h, "ncclRecv", &x.Recv) && sym(h, "ncclGroupStart", &x.GroupStart) &&
              sym(h, "ncclGroupEnd", &x.GroupEnd) && sym(h, "ncclAllGather", &x.AllGather) &&
              sym(h, "ncclBroadcast", &x.Broadcast) &&
              sym(h, "ncclGetErrorString", &x.ErrorString);
    if (!ok) {
      x.err = "librccl.so.1 lacks an entry point this library needs";
      return x;
    }
    (void)sym(h, "ncclGetVersion", &x.GetVersion);
    x.ok = true;
    return x;
  }();
  return r;
}

int rccl_loaded() {
  const Rccl& r = rccl();
  return r.ok ? 0 : fail(BYTEPS_REDUCE_ERCCL, "%s", r.err.c_str());
}

int rccl_fail(ncclResult_t e, const char* what) {
  return fail(BYTEPS_REDUCE_ERCCL, "%s: %s", what, rccl().ErrorString(e));
}

// ------------------------------------------------------ in-process group --
// One transfer posted by its sender: the receiver copies `bytes` from `buf`
// once `ready` (recorded on the sender's stream) has passed, then records
// `consumed` on its own stream; the sender's stream waits for `consumed`
// before anything later may overwrite `buf`.
struct Post {
  const void* buf = nullptr;
  size_t bytes = 0;
  hipEvent_t ready = nullptr;
  hipEvent_t consumed = nullptr;
  bool matched = false;
  int status = 0;
};

struct LocalGroup {
  int world = 0;
  std::vector<int> devices;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::deque<std::shared_ptr<Post>>> box;  // [src * world + dst], FIFO
  std::atomic<bool> broken{false};  // a rank gave up waiting: every later call fails
};

double local_timeout_s() {
  static const double t = [] {
    const char* v = getenv("BPSR_SHARD_TIMEOUT_S");
    const double x = v ? atof(v) : 120.0;
    return x > 0 ? x : 120.0;
  }();
  return t;
}

}  // namespace
}  // namespace bpsr

struct byteps_shard_comm {
  int kind = 0;  // kOwned, kWrapped, kLocal
  ncclComm_t nc = nullptr;
  int world = 1, rank = 0, device = 0;
  std::shared_ptr<bpsr::LocalGroup> group;
};

namespace bpsr {
namespace {

enum { kOwned = 0, kWrapped = 1, kLocal = 2 };

struct P2P {
  bool send;
  int peer;
  const void* sbuf;
  void* rbuf;
  size_t bytes;
};

int run_rccl(byteps_shard_comm* c, const std::vector<P2P>& ops, hipStream_t s) {
  const Rccl& r = rccl();
  ncclResult_t e = r.GroupStart();
  if (e != ncclSuccess) return rccl_fail(e, "ncclGroupStart");
  int rc = 0;
  for (const P2P& o : ops) {
    e = o.send ? r.Send(o.sbuf, o.bytes, ncclUint8, o.peer, c->nc, s)
               : r.Recv(o.rbuf, o.bytes, ncclUint8, o.peer, c->nc, s);
    if (e != ncclSuccess) {
      rc = rccl_fail(e, o.send ? "ncclSend" : "ncclRecv");
      break;
    }
  }
  e = r.GroupEnd();  // always closes the group
  if (!rc && e != ncclSuccess) rc = rccl_fail(e, "ncclGroupEnd");
  return rc;
}

int run_local(byteps_shard_comm* c, const std::vector<P2P>& ops, hipStream_t s) {
  LocalGroup& G = *c->group;
  const int W = G.world, me = c->rank;
  const auto deadline =
      std::chrono::steady_clock::now() +
      std::chrono::milliseconds((long long)(local_timeout_s() * 1000.0));
  std::vector<std::shared_ptr<Post>> mine;
  hipError_t he = hipSuccess;
  // 1. post every send (before waiting for any receive: no rank can then
  //    wait on a peer that is itself waiting)
  for (const P2P& o : ops) {
    if (!o.send) continue;
    auto p = std::make_shared<Post>();
    p->buf = o.sbuf;
    p->bytes = o.bytes;
    he = hipEventCreateWithFlags(&p->ready, hipEventDisableTiming);
    if (he == hipSuccess) he = hipEventRecord(p->ready, s);
    if (he != hipSuccess) {
      if (p->ready) (void)hipEventDestroy(p->ready);
      p->ready = nullptr;
      p->status = hip_fail(he, "shard send event");
    }
    {
      std::lock_guard<std::mutex> g(G.mu);
      G.box[(size_t)me * W + o.peer].push_back(p);
    }
    G.cv.notify_all();
    mine.push_back(p);
  }
  int rc = 0;
  for (auto& p : mine)
    if (!rc && p->status) rc = p->status;
  // 2. receives, in call order; a peer's sends to this rank arrive in its
  //    call order (collective calls are made in the same order everywhere)
  for (const P2P& o : ops) {
    if (o.send) continue;
    std::shared_ptr<Post> p;
    {
      std::unique_lock<std::mutex> lk(G.mu);
      auto& q = G.box[(size_t)o.peer * W + me];
      if (!G.cv.wait_until(lk, deadline, [&] { return G.broken || !q.empty(); })) G.broken = true;
      if (G.broken) {
        G.cv.notify_all();
        return rc ? rc : fail(BYTEPS_REDUCE_ETIMEOUT, "shard group: rank %d waited for rank %d "
                                                      "past %.0f s (group now broken)",
                              me, o.peer, local_timeout_s());
      }
      p = q.front();
      q.pop_front();
    }
    int st = p->status;
    if (!st && p->bytes != o.bytes)
      st = fail(BYTEPS_REDUCE_EARGS, "shard group: rank %d sent %zu bytes, rank %d expects %zu",
                o.peer, p->bytes, me, o.bytes);
    if (!st) {
      he = hipStreamWaitEvent(s, p->ready, 0);
      if (he == hipSuccess && o.bytes)
        he = hipMemcpyAsync(o.rbuf, p->buf, o.bytes, hipMemcpyDeviceToDevice, s);
      if (he == hipSuccess) he = hipEventCreateWithFlags(&p->consumed, hipEventDisableTiming);
      if (he == hipSuccess) he = hipEventRecord(p->consumed, s);
      if (he != hipSuccess) st = hip_fail(he, "shard group copy");
    }
    {
      std::lock_guard<std::mutex> g(G.mu);
      p->status = p->status ? p->status : st;
      p->matched = true;
    }
    G.cv.notify_all();
    if (st && !rc) rc = st;
  }
  // 3. every send consumed: this stream's later work waits for the copies
  //    that read from its buffers
  for (auto& p : mine) {
    {
      std::unique_lock<std::mutex> lk(G.mu);
      if (!G.cv.wait_until(lk, deadline, [&] { return G.broken || p->matched; })) G.broken = true;
      if (!p->matched) {
        G.cv.notify_all();
        if (!rc)
          rc = fail(BYTEPS_REDUCE_ETIMEOUT, "shard group: rank %d's send was not received "
                                            "within %.0f s (group now broken)",
                    me, local_timeout_s());
        continue;  // the post stays with the group (a peer may still read it)
      }
    }
    if (p->consumed) {
      he = hipStreamWaitEvent(s, p->consumed, 0);
      if (he != hipSuccess && !rc) rc = hip_fail(he, "shard group wait");
      (void)hipEventDestroy(p->consumed);  // released once complete
    }
    if (p->ready) (void)hipEventDestroy(p->ready);
    if (p->status && !rc) rc = p->status;
  }
  return rc;
}

int run_group(byteps_shard_comm* c, const std::vector<P2P>& ops, hipStream_t s) {
  if (ops.empty()) return 0;
  return c->kind == kLocal ? run_local(c, ops, s) : run_rccl(c, ops, s);
}

// ------------------------------------------------------------ helpers --
inline hipStream_t to_stream(void* s) {
  return s ? reinterpret_cast<hipStream_t>(s) : hipStreamPerThread;
}

struct Range {
  size_t lo, hi;
  size_t n() const { return hi - lo; }
};

Range owner(size_t elems, int world, int rank) {
  const size_t per = elems / (size_t)world;
  Range r{per * (size_t)rank, per * (size_t)(rank + 1)};
  if (rank == world - 1) r.hi = elems;  // tail to the last rank (the NCCL root)
  return r;
}

int begin_call(byteps_shard_comm* c, int dtype, int mode, bool check_mode, size_t* es) {
  if (!c) return fail(BYTEPS_REDUCE_EARGS, "null communicator");
  const int s = elem_size(dtype);
  if (!s) return fail(BYTEPS_REDUCE_EDTYPE, "Unsupported data type: %d", dtype);
  if (check_mode && mode != kModeReference && mode != kModeAccumF32)
    return fail(BYTEPS_REDUCE_EARGS, "unknown mode %d", mode);
  *es = (size_t)s;
  if (c->kind != kLocal) {
    const int rc = rccl_loaded();
    if (rc) return rc;
  } else if (c->group->broken) {
    return fail(BYTEPS_REDUCE_ETIMEOUT, "shard group broken by an earlier timeout");
  }
  return 0;
}

// After validation (so argument errors come back without touching a GPU).
int use_device(const byteps_shard_comm* c) {
  hipError_t e = hipSetDevice(c->device);
  return e == hipSuccess ? 0 : hip_fail(e, "hipSetDevice");
}

inline const char* at(const void* p, size_t off) { return static_cast<const char*>(p) + off; }
inline char* at(void* p, size_t off) { return static_cast<char*>(p) + off; }

}  // namespace
}  // namespace bpsr

using namespace bpsr;

extern "C" {

int byteps_shard_owner_range(size_t elems, int world, int rank, size_t* lo, size_t* hi) {
  if (world < 1 || rank < 0 || rank >= world || !lo || !hi)
    return fail(BYTEPS_REDUCE_EARGS, "owner_range: world %d, rank %d", world, rank);
  const Range r = owner(elems, world, rank);
  *lo = r.lo;
  *hi = r.hi;
  return BYTEPS_REDUCE_OK;
}

int byteps_shard_reduce_root_of(uint64_t key, const int* roots, int nroots) {
  if (!roots || nroots < 1) return fail(BYTEPS_REDUCE_EARGS, "no reduce roots");
  // Hash_DJB2 (global.cc:507-516) over std::to_string(key)
  const std::string str = std::to_string(key);
  uint64_t h = 5381;
  for (unsigned char ch : str) h = ((h << 5) + h) + ch;
  return roots[h % (uint64_t)nroots];
}

int byteps_shard_get_unique_id(void* id) {
  if (!id) return fail(BYTEPS_REDUCE_EARGS, "null id buffer");
  int rc = rccl_loaded();
  if (rc) return rc;
  ncclUniqueId u;
  ncclResult_t e = rccl().GetUniqueId(&u);
  if (e != ncclSuccess) return rccl_fail(e, "ncclGetUniqueId");
  static_assert(sizeof(u) == BYTEPS_SHARD_UNIQUE_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id, &u, sizeof(u));
  return BYTEPS_REDUCE_OK;
}

int byteps_shard_comm_init(const void* id, int world, int rank, int device,
                           byteps_shard_comm** out) {
  if (!out) return fail(BYTEPS_REDUCE_EARGS, "null out-pointer");
  *out = nullptr;
  if (!id || world < 1 || rank < 0 || rank >= world || device < 0)
    return fail(BYTEPS_REDUCE_EARGS, "comm_init: world %d, rank %d, device %d", world, rank,
                device);
  int rc = rccl_loaded();
  if (rc) return rc;
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) return hip_fail(he, "hipSetDevice");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  auto c = std::make_unique<byteps_shard_comm>();
  ncclResult_t e = rccl().CommInitRank(&c->nc, world, u, rank);
  if (e != ncclSuccess) return rccl_fail(e, "ncclCommInitRank");
  c->kind = kOwned;
  c->world = world;
  c->rank = rank;
  c->device = device;
  *out = c.release();
  return BYTEPS_REDUCE_OK;
}

int byteps_shard_comm_wrap(void* nccl_comm, byteps_shard_comm** out) {
  if (!out) return fail(BYTEPS_REDUCE_EARGS, "null out-pointer");
  *out = nullptr;
  if (!nccl_comm) return fail(BYTEPS_REDUCE_EARGS, "null RCCL communicator");
  int rc = rccl_loaded();
  if (rc) return rc;
  auto c = std::make_unique<byteps_shard_comm>();
  c->kind = kWrapped;
  c->nc = reinterpret_cast<ncclComm_t>(nccl_comm);
  const Rccl& r = rccl();
  ncclResult_t e = r.CommCount(c->nc, &c->world);
  if (e == ncclSuccess) e = r.CommUserRank(c->nc, &c->rank);
  if (e == ncclSuccess) e = r.CommCuDevice(c->nc, &c->device);
  if (e != ncclSuccess) return rccl_fail(e, "RCCL communicator query");
  *out = c.release();
  return BYTEPS_REDUCE_OK;
}

int byteps_shard_comm_init_local(int world, const int* devices, byteps_shard_comm** comms) {
  if (world < 1 || !devices || !comms)
    return fail(BYTEPS_REDUCE_EARGS, "comm_init_local: world %d", world);
  for (int r = 0; r < world; ++r) {
    comms[r] = nullptr;
    if (devices[r] < 0) return fail(BYTEPS_REDUCE_EARGS, "devices[%d] = %d", r, devices[r]);
  }
  auto G = std::make_shared<LocalGroup>();
  G->world = world;
  G->devices.assign(devices, devices + world);
  G->box.resize((size_t)world * world);
  // Peer access between distinct devices of the group (copies go over xGMI
  // instead of staging through host memory); already-enabled is fine.
  for (int a = 0; a < world; ++a)
    for (int b = 0; b < world; ++b) {
      if (devices[a] == devices[b]) continue;
      if (hipSetDevice(devices[a]) != hipSuccess) continue;
      (void)hipDeviceEnablePeerAccess(devices[b], 0);
      (void)hipGetLastError();
    }
  for (int r = 0; r < world; ++r) {
    comms[r] = new byteps_shard_comm();
    comms[r]->kind = kLocal;
    comms[r]->world = world;
    comms[r]->rank = r;
    comms[r]->device = devices[r];
    comms[r]->group = G;
  }
  return BYTEPS_REDUCE_OK;
}

int byteps_shard_comm_destroy(byteps_shard_comm* c) {
  if (!c) return BYTEPS_REDUCE_OK;
  int rc = BYTEPS_REDUCE_OK;
  if (c->kind == kOwned && c->nc && rccl().ok) {
    (void)hipSetDevice(c->device);
    ncclResult_t e = rccl().CommDestroy(c->nc);
    if (e != ncclSuccess) rc = rccl_fail(e, "ncclCommDestroy");
  }
  delete c;
  return rc;
}

int byteps_shard_comm_info(const byteps_shard_comm* c, int* world, int* rank, int* device) {
  if (!c) return fail(BYTEPS_REDUCE_EARGS, "null communicator");
  if (world) *world = c->world;
  if (rank) *rank = c->rank;
  if (device) *device = c->device;
  return BYTEPS_REDUCE_OK;
}

int byteps_shard_rccl_version(int* version) {
  if (!version) return fail(BYTEPS_REDUCE_EARGS, "null version");
  *version = 0;
  if (int rc = rccl_loaded()) return rc;
  const Rccl& r = rccl();
  if (!r.GetVersion) return fail(BYTEPS_REDUCE_ERCCL, "librccl.so.1 has no ncclGetVersion");
  const ncclResult_t e = r.GetVersion(version);
  return e == ncclSuccess ? BYTEPS_REDUCE_OK
                          : fail(BYTEPS_REDUCE_ERCCL, "ncclGetVersion: %s", r.ErrorString(e));
}

int byteps_shard_reduce_scatter(byteps_shard_comm* c, const void* local, void* const* recv_slots,
                                void* dst, size_t elems, int dtype, int mode, void* stream) {
  size_t es = 0;
  int rc = begin_call(c, dtype, mode, true, &es);
  if (rc) return rc;
  if (elems == 0) return BYTEPS_REDUCE_OK;
  const int W = c->world, g = c->rank;
  const Range mine = owner(elems, W, g);
  if (!local) return fail(BYTEPS_REDUCE_EARGS, "null local vector");
  if (mine.n() && !dst) return fail(BYTEPS_REDUCE_EARGS, "null dst on an owning rank");
  if (mine.n() && W > 1) {
    if (!recv_slots) return fail(BYTEPS_REDUCE_EARGS, "null recv_slots on an owning rank");
    for (int r = 0; r < W; ++r)
      if (r != g && !recv_slots[r]) return fail(BYTEPS_REDUCE_EARGS, "null recv_slots[%d]", r);
  }
  std::vector<P2P> ops;
  for (int q = 0; q < W; ++q) {  // my slice of owner q's range, to q
    const Range rq = owner(elems, W, q);
    if (q != g && rq.n()) ops.push_back({true, q, at(local, rq.lo * es), nullptr, rq.n() * es});
  }
  if (mine.n())
    for (int r = 0; r < W; ++r)
      if (r != g) ops.push_back({false, r, nullptr, recv_slots[r], mine.n() * es});
  if ((rc = use_device(c))) return rc;
  hipStream_t s = to_stream(stream);
  if ((rc = run_group(c, ops, s))) return rc;
  if (!mine.n()) return BYTEPS_REDUCE_OK;
  std::vector<const void*> srcs(W);
  for (int r = 0; r < W; ++r) srcs[r] = r == g ? at(local, mine.lo * es) : recv_slots[r];
  return fold_any_alias(dst, srcs.data(), W, mine.n() * es, dtype, mode, s);
}

int byteps_shard_allgather(byteps_shard_comm* c, const void* owned, void* full, size_t elems,
                           int dtype, void* stream) {
  size_t es = 0;
  int rc = begin_call(c, dtype, 0, false, &es);
  if (rc) return rc;
  if (elems == 0) return BYTEPS_REDUCE_OK;
  const int W = c->world, g = c->rank;
  const Range mine = owner(elems, W, g);
  if (!full || (mine.n() && !owned)) return fail(BYTEPS_REDUCE_EARGS, "null buffer");
  if ((rc = use_device(c))) return rc;
  hipStream_t s = to_stream(stream);
  const size_t per = elems / (size_t)W, tail = elems - per * (size_t)W;
  if (c->kind != kLocal) {
    const Rccl& r = rccl();
    ncclResult_t e = ncclSuccess;
    // in place when owned == full + lo (ncclAllGather's in-place rule)
    if (per) e = r.AllGather(owned, full, per * es, ncclUint8, c->nc, s);
    if (e != ncclSuccess) return rccl_fail(e, "ncclAllGather");
    if (tail) {
      const void* src = g == W - 1 ? at(owned, per * es) : at(full, per * W * es);
      e = r.Broadcast(src, at(full, per * W * es), tail * es, ncclUint8, W - 1, c->nc, s);
      if (e != ncclSuccess) return rccl_fail(e, "ncclBroadcast (tail)");
    }
    return BYTEPS_REDUCE_OK;
  }
  std::vector<P2P> ops;
  for (int q = 0; q < W; ++q) {
    if (q == g) continue;
    const Range rq = owner(elems, W, q);
    if (mine.n()) ops.push_back({true, q, owned, nullptr, mine.n() * es});
    if (rq.n()) ops.push_back({false, q, nullptr, at(full, rq.lo * es), rq.n() * es});
  }
  if ((rc = run_group(c, ops, s))) return rc;
  if (mine.n() && owned != at(full, mine.lo * es)) {
    hipError_t e = hipMemcpyAsync(at(full, mine.lo * es), owned, mine.n() * es,
                                  hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return hip_fail(e, "allgather own slice");
  }
  return BYTEPS_REDUCE_OK;
}

int byteps_shard_scatter_reduce(byteps_shard_comm* c, int root, const void* const* pushes, int n,
                                void* const* recv_slots, void* dst, size_t elems, int dtype,
                                int mode, void* stream) {
  size_t es = 0;
  int rc = begin_call(c, dtype, mode, true, &es);
  if (rc) return rc;
  const int W = c->world, g = c->rank;
  if (root < 0 || root >= W) return fail(BYTEPS_REDUCE_EARGS, "root %d outside [0, %d)", root, W);
  if (n < 1) return fail(BYTEPS_REDUCE_EARGS, "need n >= 1 pushes (n=%d)", n);
  if (elems == 0) return BYTEPS_REDUCE_OK;
  const Range mine = owner(elems, W, g);
  if (g == root) {
    if (!pushes) return fail(BYTEPS_REDUCE_EARGS, "null pushes on the root");
    for (int k = 0; k < n; ++k)
      if (!pushes[k]) return fail(BYTEPS_REDUCE_EARGS, "null pushes[%d]", k);
  }
  if (mine.n()) {
    if (!dst) return fail(BYTEPS_REDUCE_EARGS, "null dst on an owning rank");
    if (g != root) {
      if (!recv_slots) return fail(BYTEPS_REDUCE_EARGS, "null recv_slots on an owning rank");
      for (int k = 0; k < n; ++k)
        if (!recv_slots[k]) return fail(BYTEPS_REDUCE_EARGS, "null recv_slots[%d]", k);
    }
  }
  std::vector<P2P> ops;
  if (g == root) {
    for (int q = 0; q < W; ++q) {
      const Range rq = owner(elems, W, q);
      if (q == root || !rq.n()) continue;
      for (int k = 0; k < n; ++k)
        ops.push_back({true, q, at(pushes[k], rq.lo * es), nullptr, rq.n() * es});
    }
  } else if (mine.n()) {
    for (int k = 0; k < n; ++k) ops.push_back({false, root, nullptr, recv_slots[k], mine.n() * es});
  }
  if ((rc = use_device(c))) return rc;
  hipStream_t s = to_stream(stream);
  if ((rc = run_group(c, ops, s))) return rc;
  if (!mine.n()) return BYTEPS_REDUCE_OK;
  std::vector<const void*> srcs(n);
  for (int k = 0; k < n; ++k) srcs[k] = g == root ? at(pushes[k], mine.lo * es) : recv_slots[k];
  return fold_any_alias(dst, srcs.data(), n, mine.n() * es, dtype, mode, s);
}

int byteps_shard_reduce_root(byteps_shard_comm* c, int root, const void* local,
                             void* const* recv_slots, void* dst, size_t elems, int dtype, int mode,
                             void* stream) {
  size_t es = 0;
  int rc = begin_call(c, dtype, mode, true, &es);
  if (rc) return rc;
  const int W = c->world, g = c->rank;
  if (root < 0 || root >= W) return fail(BYTEPS_REDUCE_EARGS, "root %d outside [0, %d)", root, W);
  if (elems == 0) return BYTEPS_REDUCE_OK;
  if (!local) return fail(BYTEPS_REDUCE_EARGS, "null local vector");
  if (g == root) {
    if (!dst) return fail(BYTEPS_REDUCE_EARGS, "null dst on the root");
    if (W > 1 && !recv_slots) return fail(BYTEPS_REDUCE_EARGS, "null recv_slots on the root");
    for (int r = 0; r < W; ++r)
      if (r != g && !recv_slots[r]) return fail(BYTEPS_REDUCE_EARGS, "null recv_slots[%d]", r);
  }
  const size_t bytes = elems * es;
  std::vector<P2P> ops;
  if (g != root) {
    ops.push_back({true, root, local, nullptr, bytes});
  } else {
    for (int r = 0; r < W; ++r)
      if (r != g) ops.push_back({false, r, nullptr, recv_slots[r], bytes});
  }
  if ((rc = use_device(c))) return rc;
  hipStream_t s = to_stream(stream);
  if ((rc = run_group(c, ops, s))) return rc;
  if (g != root) return BYTEPS_REDUCE_OK;
  std::vector<const void*> srcs(W);
  for (int r = 0; r < W; ++r) srcs[r] = r == g ? local : recv_slots[r];
  return fold_any_alias(dst, srcs.data(), W, bytes, dtype, mode, s);
}

int byteps_shard_broadcast(byteps_shard_comm* c, int root, void* buf, size_t elems, int dtype,
                           void* stream) {
  size_t es = 0;
  int rc = begin_call(c, dtype, 0, false, &es);
  if (rc) return rc;
  const int W = c->world, g = c->rank;
  if (root < 0 || root >= W) return fail(BYTEPS_REDUCE_EARGS, "root %d outside [0, %d)", root, W);
  if (elems == 0) return BYTEPS_REDUCE_OK;
  if (!buf) return fail(BYTEPS_REDUCE_EARGS, "null buffer");
  if ((rc = use_device(c))) return rc;
  hipStream_t s = to_stream(stream);
  const size_t bytes = elems * es;
  if (c->kind != kLocal) {
    ncclResult_t e = rccl().Broadcast(buf, buf, bytes, ncclUint8, root, c->nc, s);
    return e == ncclSuccess ? 0 : rccl_fail(e, "ncclBroadcast");
  }
  std::vector<P2P> ops;
  if (g == root) {
    for (int q = 0; q < W; ++q)
      if (q != g) ops.push_back({true, q, buf, nullptr, bytes});
  } else {
    ops.push_back({false, root, nullptr, buf, bytes});
  }
  return run_group(c, ops, s);
}

}  // extern "C"
