// Key space sharded over several GPU-resident server instances
// (include/bpsr/server.h, byteps_server_group_*): the reference's key ->
// server assignment (BytePSGlobal::EncodeDefaultKey, global.cc:530-567) for a
// process that owns all of a node's GPUs, or the reduce-scatter owner ranges
// applied to each large partition.  Host-side routing only; every byte of
// data moves and folds inside the instances.
#include "bpsr/server.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "bpsr_error.h"
#include "bpsr_internal.h"
#include "bpsr_server_internal.h"

namespace bpsr {
namespace {

constexpr size_t kUnit = 128;  // piece granule: 8 elements of every dtype, 16-B aligned

struct Piece {
  int server;
  size_t off, len;
};

// What the group knows of a key: its declared length and dtype (the split is
// computed from them, so a shorter pull is cut from the same pieces), and the
// arrival stamps of its rounds.  A range-split key has ONE arrival order for
// all its pieces (server.cc:216-250: one left fold per key in arrival order):
// the group gives each push the next position of its worker's round, and every
// instance folds its piece in those positions (bpsr::server_push_async_at).
struct GroupKey {
  std::mutex mu;
  size_t len = 0;  // 0: not declared yet
  int dtype = -1;
  std::vector<uint64_t> pushes;   // per worker: pushes stamped so far (= its round)
  std::map<uint64_t, int> taken;  // round -> positions handed out (erased when full)
};

}  // namespace
}  // namespace bpsr

struct byteps_server_group {
  byteps_server_group_config cfg;
  std::vector<byteps_server*> inst;
  bool pulls_async = false;  // every instance answers pull_into_async (parallel gathers)
  std::shared_mutex mu;
  std::unordered_map<uint64_t, std::unique_ptr<bpsr::GroupKey>> keys;
};

namespace bpsr {
namespace {

void route_cfg(const byteps_server_group_config& c, uint64_t key, size_t len,
               std::vector<Piece>* out) {
  out->clear();
  const int n = c.num_servers;
  const size_t min_bytes = c.split_min_bytes ? c.split_min_bytes : kUnit * (size_t)n;
  if (c.split == BYTEPS_SERVER_SPLIT_RANGE && n > 1 && len >= min_bytes &&
      len / kUnit >= (size_t)n) {
    const size_t per = len / kUnit / (size_t)n * kUnit;  // owner ranges, in 128-B units
    for (int i = 0; i < n; ++i)
      out->push_back({i, per * (size_t)i, i == n - 1 ? len - per * (size_t)i : per});
    return;
  }
  const int srv = (int)(byteps_server_key_hash(key, c.hash_fn, c.hash_coef) % (uint64_t)n);
  out->push_back({srv, 0, len});
}

void route(const byteps_server_group* g, uint64_t key, size_t len, std::vector<Piece>* out) {
  route_cfg(g->cfg, key, len, out);
}

int check_cfg(const byteps_server_group_config* cfg) {
  if (!cfg) return fail(BYTEPS_REDUCE_EARGS, "null config");
  if (cfg->num_servers < 1 || cfg->num_servers > BYTEPS_SERVER_GROUP_MAX)
    return fail(BYTEPS_REDUCE_EARGS, "num_servers %d outside [1, %d]", cfg->num_servers,
                BYTEPS_SERVER_GROUP_MAX);
  if (cfg->split != BYTEPS_SERVER_SPLIT_HASH && cfg->split != BYTEPS_SERVER_SPLIT_RANGE)
    return fail(BYTEPS_REDUCE_EARGS, "unknown split %d", cfg->split);
  if (cfg->hash_fn < BYTEPS_KEY_HASH_DJB2 || cfg->hash_fn > BYTEPS_KEY_HASH_BUILT_IN)
    return fail(BYTEPS_REDUCE_EARGS, "unknown key hash %d", cfg->hash_fn);
  for (int i = 0; i < cfg->num_servers; ++i)
    if (cfg->devices[i] < 0) return fail(BYTEPS_REDUCE_EARGS, "devices[%d] = %d", i, cfg->devices[i]);
  return 0;
}

int write_pieces(const std::vector<Piece>& ps, int* npieces, int* server, size_t* offset,
                 size_t* plen, int cap) {
  if (!npieces) return fail(BYTEPS_REDUCE_EARGS, "null npieces");
  *npieces = (int)ps.size();
  for (int i = 0; i < (int)ps.size() && i < cap; ++i) {
    if (server) server[i] = ps[i].server;
    if (offset) offset[i] = ps[i].off;
    if (plen) plen[i] = ps[i].len;
  }
  return BYTEPS_REDUCE_OK;
}

// Countdown of a scattered push: the pieces' acknowledgements.
struct Acks {
  std::mutex mu;
  std::condition_variable cv;
  int remaining = 0;
  int status = 0;
  std::vector<size_t> inst_bytes;  // host pieces not acknowledged yet, per instance
};

// One host piece's acknowledgement: its bytes leave the instance's window.
struct PieceAck {
  Acks* a;
  size_t inst;
  size_t len;
};

void ack_cb(void* ctx, uint64_t, int, int status) {
  Acks* a = static_cast<Acks*>(ctx);
  std::lock_guard<std::mutex> g(a->mu);
  if (status && !a->status) a->status = status;
  --a->remaining;
  a->cv.notify_all();
}

int check_group(const byteps_server_group* g) {
  return g ? 0 : fail(BYTEPS_REDUCE_EARGS, "null server group");
}

void pull_ack_cb(void* ctx, uint64_t, const void*, size_t, int status) {
  ack_cb(ctx, 0, 0, status);
}

// Wait for every acknowledgement counted so far.
int wait_acks(Acks& a, int rc) {
  std::unique_lock<std::mutex> lk(a.mu);
  a.cv.wait(lk, [&] { return a.remaining == 0; });
  return rc ? rc : a.status;
}

bpsr::GroupKey* group_key(byteps_server_group* g, uint64_t key, bool create) {
  {
    std::shared_lock<std::shared_mutex> lk(g->mu);
    auto it = g->keys.find(key);
    if (it != g->keys.end()) return it->second.get();
    if (!create) return nullptr;
  }
  std::unique_lock<std::shared_mutex> lk(g->mu);
  auto& slot = g->keys[key];
  if (!slot) slot = std::make_unique<bpsr::GroupKey>();
  return slot.get();
}

// Declare (first sight) or check a key's length and dtype.
int declare(byteps_server_group* g, uint64_t key, size_t len, int dtype) {
  bpsr::GroupKey* gk = group_key(g, key, true);
  std::lock_guard<std::mutex> lk(gk->mu);
  if (gk->len == 0) {
    if (len == 0) return fail(BYTEPS_REDUCE_EARGS, "init tensor size not larger than 0");
    gk->len = len;
    gk->dtype = dtype;
    gk->pushes.assign((size_t)g->cfg.server.num_workers, 0);
    return 0;
  }
  if (len != gk->len || dtype != gk->dtype)
    return fail(BYTEPS_REDUCE_EARGS, "key %llu pushed with len %zu dtype %d (declared %zu, %d)",
                (unsigned long long)key, len, dtype, gk->len, gk->dtype);
  return 0;
}

// The key's declared length (0: never declared to the group).
size_t declared_len(byteps_server_group* g, uint64_t key) {
  bpsr::GroupKey* gk = group_key(g, key, false);
  if (!gk) return 0;
  std::lock_guard<std::mutex> lk(gk->mu);
  return gk->len;
}

// The position of worker w's next push of the key in its round's order.
int stamp(byteps_server_group* g, uint64_t key, int w) {
  if (g->cfg.server.async_mode) return -1;  // no rounds
  bpsr::GroupKey* gk = group_key(g, key, true);
  std::lock_guard<std::mutex> lk(gk->mu);
  const int N = g->cfg.server.num_workers;
  if (gk->pushes.size() != (size_t)N) gk->pushes.assign((size_t)N, 0);
  const uint64_t round = gk->pushes[(size_t)w]++;
  const int pos = gk->taken[round]++;
  if (pos + 1 == N) gk->taken.erase(round);
  return pos;
}

// The pieces of a pull of `len` bytes: the key's pieces (by its declared
// length) cut to [0, len).
int pull_pieces(byteps_server_group* g, uint64_t key, size_t len, std::vector<Piece>* ps) {
  const size_t klen = declared_len(g, key);
  if (klen == 0) {  // never declared here: the instance reports it (server.cc:282-283)
    route(g, key, len, ps);
    return 0;
  }
  if (len > klen)
    return fail(BYTEPS_REDUCE_EARGS, "pull of %zu bytes > key len %zu", len, klen);
  std::vector<Piece> all;
  route(g, key, klen, &all);
  ps->clear();
  for (const Piece& p : all)
    if (p.off < len) ps->push_back({p.server, p.off, std::min(p.len, len - p.off)});
  return 0;
}

// Can instances write `p` with their copy kernels (device memory, or pinned
// host memory through its device view)?
bool addressable(const void* p, int location) {
  if (location == BYTEPS_SERVER_DEVICE) return true;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void*>(p), 0) == hipSuccess && d) return true;
  (void)hipGetLastError();
  return false;
}

// Scatter pushes: every piece validated on its instance first (nothing is
// queued if one would be refused), then queued at once on its instance (its
// own device and lanes), a range-split key's pieces with the group's stamp;
// then wait for every acknowledgement — the data is in HBM and (init round)
// every worker's init push has arrived, as a blocking push guarantees.  A
// piece that fails once others are queued fails the key on every instance, so
// none waits for a round that cannot complete.
struct PushPiece {
  byteps_server* s;
  uint64_t key;
  const void* data;
  size_t len;
  bool split;  // one piece of a range-split key (stamped)
  int pos;
};
// A call's host pieces in flight at most per instance (one PCIe link each):
// one of BytePS's 4,096,000-B partitions (a larger piece goes alone).  Different workers' calls (transport
// threads) then interleave on the link partition by partition, so a key's
// round completes — and is folded and pulled back — while later partitions
// are still crossing, instead of after one worker's whole batch
// (core_loops.cc:492-564 sends every partition as it is ready; the network
// interleaves the workers).  Config 1's first round completes at 0.6-0.8 ms
// instead of 1.1-1.2 (16 MiB window) or 1.8-2.0 ms (none); rounds with
// copying pulls 4.2-4.4 ms instead of 5.0-5.4 (r05s12, profiles/README.md).
#ifndef BPSR_HOST_PIECE_WINDOW  // (probe builds only: tools/cfg1_round_probe.py --lib)
#define BPSR_HOST_PIECE_WINDOW (4u << 20)
#endif
constexpr size_t kHostPieceWindow = BPSR_HOST_PIECE_WINDOW;

void piece_ack_cb(void* ctx, uint64_t, int, int status) {
  PieceAck* p = static_cast<PieceAck*>(ctx);
  Acks* a = p->a;
  std::lock_guard<std::mutex> g(a->mu);
  if (status && !a->status) a->status = status;
  a->inst_bytes[p->inst] -= p->len;
  --a->remaining;
  a->cv.notify_all();
}

int scatter_pushes(byteps_server_group* g, std::vector<PushPiece>& pcs, int worker, int dtype,
                   int location) {
  for (const PushPiece& p : pcs)
    if (int rc = bpsr::server_check_key(p.s, p.key, p.len, dtype)) return rc;
  // stamped only once every piece passed (a refused push takes no position):
  // one position per split key, shared by its consecutive pieces
  for (size_t i = 0; i < pcs.size(); ++i) {
    if (!pcs[i].split) continue;
    if (i > 0 && pcs[i - 1].split && pcs[i - 1].key == pcs[i].key) {
      pcs[i].pos = pcs[i - 1].pos;
      continue;
    }
    pcs[i].pos = stamp(g, pcs[i].key, worker);
  }
  Acks acks;
  const bool windowed = location == BYTEPS_SERVER_HOST;
  acks.inst_bytes.assign(g->inst.size(), 0);
  std::vector<PieceAck> pa(pcs.size());
  int rc = 0;
  size_t queued = 0;
  for (size_t i = 0; i < pcs.size(); ++i) {
    const PushPiece& p = pcs[i];
    size_t inst = 0;
    while (inst < g->inst.size() && g->inst[inst] != p.s) ++inst;
    // init pushes are answered only once every worker's is in: outside the
    // window, or workers pushing their keys in different orders would wait
    // for each other's windows
    const bool counted = windowed && bpsr::server_key_inited(p.s, p.key);
    pa[i] = {&acks, inst, counted ? p.len : 0};
    {
      std::unique_lock<std::mutex> lk(acks.mu);
      if (counted)  // the instance's window (a piece larger than it goes alone)
        acks.cv.wait(lk, [&] {
          return acks.inst_bytes[inst] == 0 || acks.inst_bytes[inst] + p.len <= kHostPieceWindow;
        });
      ++acks.remaining;
      acks.inst_bytes[inst] += pa[i].len;
    }
    rc = bpsr::server_push_async_at(p.s, p.key, worker, p.data, p.len, dtype, location,
                                    piece_ack_cb, &pa[i], p.pos);
    if (rc) {
      std::lock_guard<std::mutex> lk(acks.mu);
      --acks.remaining;
      acks.inst_bytes[inst] -= pa[i].len;
      break;
    }
    ++queued;
  }
  if (rc) {
    const std::string msg = byteps_reduce_last_error();
    for (const PushPiece& p : pcs) bpsr::server_fail_key(p.s, p.key, rc);
    (void)wait_acks(acks, rc);  // queued pieces still read the caller's data
    return fail(rc, "%s", msg.c_str());
  }
  (void)queued;
  return wait_acks(acks, 0);
}

// Gather pulls: every piece's copy queued at once (pull_into_async: the
// instances' issuers copy their pieces in parallel, each batched with the
// pulls that piled up on its lane), then wait for all answers.
struct PullPiece {
  byteps_server* s;
  uint64_t key;
  void* out;
  size_t len;
};
int gather_pulls(const std::vector<PullPiece>& pcs, int location) {
  Acks acks;
  int rc = 0;
  for (const PullPiece& p : pcs) {
    {
      std::lock_guard<std::mutex> lk(acks.mu);
      ++acks.remaining;
    }
    rc = byteps_server_pull_into_async(p.s, p.key, p.out, p.len, location, pull_ack_cb, &acks);
    if (rc) {
      std::lock_guard<std::mutex> lk(acks.mu);
      --acks.remaining;
      break;
    }
  }
  return wait_acks(acks, rc);
}

}  // namespace
}  // namespace bpsr

using namespace bpsr;

extern "C" {

uint64_t byteps_server_key_hash(uint64_t key, int fn, uint32_t coef) {
  if (fn == BYTEPS_KEY_HASH_NAIVE) return ((key >> 16) + (key % 65536)) * 9973;  // global.cc:491-493
  const std::string str = std::to_string(key);
  if (fn == BYTEPS_KEY_HASH_BUILT_IN)  // global.cc:494-497: std::hash<std::string> x coefficient
    return (uint64_t)std::hash<std::string>()(str) * (uint64_t)coef;
  uint64_t h = fn == BYTEPS_KEY_HASH_SDBM ? 0 : 5381;
  for (unsigned char c : str) {
    if (fn == BYTEPS_KEY_HASH_SDBM)
      h = c + (h << 6) + (h << 16) - h;  // global.cc:518-523
    else
      h = ((h << 5) + h) + c;            // djb2, global.cc:499-508
  }
  return h;
}

int byteps_server_group_config_from_env(byteps_server_group_config* cfg) {
  if (!cfg) return fail(BYTEPS_REDUCE_EARGS, "null config");
  std::memset(cfg, 0, sizeof(*cfg));
  int rc = byteps_server_config_from_env(&cfg->server);
  if (rc) return rc;
  const char* v = getenv("BPSR_SERVER_GPUS");
  cfg->num_servers = v ? atoi(v) : 1;
  if (cfg->num_servers < 1 || cfg->num_servers > BYTEPS_SERVER_GROUP_MAX)
    return fail(BYTEPS_REDUCE_EARGS, "BPSR_SERVER_GPUS=%s outside [1, %d]", v ? v : "",
                BYTEPS_SERVER_GROUP_MAX);
  for (int i = 0; i < cfg->num_servers; ++i) cfg->devices[i] = i;
  v = getenv("BPSR_SERVER_SPLIT");
  cfg->split = (v && std::string(v) == "range") ? BYTEPS_SERVER_SPLIT_RANGE : BYTEPS_SERVER_SPLIT_HASH;
  v = getenv("BYTEPS_KEY_HASH_FN");  // global.cc:151-152, default djb2
  const std::string h = v ? v : "djb2";
  if (h == "djb2") cfg->hash_fn = BYTEPS_KEY_HASH_DJB2;
  else if (h == "naive") cfg->hash_fn = BYTEPS_KEY_HASH_NAIVE;
  else if (h == "sdbm") cfg->hash_fn = BYTEPS_KEY_HASH_SDBM;
  else if (h == "built_in") cfg->hash_fn = BYTEPS_KEY_HASH_BUILT_IN;
  else
    return fail(BYTEPS_REDUCE_EARGS, "Unsupported BYTEPS_KEY_HASH_FN %s, must be one of "
                                     "[naive, built_in, djb2, sdbm]", h.c_str());
  v = getenv("BYTEPS_BUILT_IN_HASH_COEF");  // global.cc:155-158, default 1
  cfg->hash_coef = v ? (uint32_t)atoi(v) : 1u;
  v = getenv("BPSR_SERVER_SPLIT_MIN_BYTES");
  cfg->split_min_bytes = v ? (size_t)atoll(v) : 0;
  return BYTEPS_REDUCE_OK;
}

int byteps_server_group_create(const byteps_server_group_config* cfg, byteps_server_group** out) {
  if (!out) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  *out = nullptr;
  int rc0 = check_cfg(cfg);
  if (rc0) return rc0;
  auto g = std::make_unique<byteps_server_group>();
  g->cfg = *cfg;
  for (int i = 0; i < cfg->num_servers; ++i) {
    byteps_server_config c = cfg->server;
    c.device = cfg->devices[i];
    byteps_server* s = nullptr;
    const int rc = byteps_server_create(&c, &s);
    if (rc) {
      byteps_server_group_destroy(g.release());
      return rc;
    }
    g->inst.push_back(s);
  }
  g->pulls_async = true;
  for (byteps_server* s : g->inst) g->pulls_async = g->pulls_async && bpsr::server_pulls_async(s);
  // Instances copy with kernels between their own HBM and buffers on the
  // other GPUs (a worker's device tensors, another instance's pieces): every
  // pair of the group's devices gets peer access where the link allows it.
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) == hipSuccess) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (int i = 0; i < cfg->num_servers; ++i)
      for (int j = 0; j < cfg->num_servers; ++j) {
        const int a = cfg->devices[i], b = cfg->devices[j];
        int can = 0;
        if (a == b || a >= ndev || b >= ndev) continue;
        if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
        if (hipSetDevice(a) == hipSuccess) {
          const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
            (void)hipSetDevice(cur);
            byteps_server_group_destroy(g.release());
            return hip_fail(e, "hipDeviceEnablePeerAccess");
          }
          (void)hipGetLastError();
        }
      }
    (void)hipSetDevice(cur);
  }
  *out = g.release();
  return BYTEPS_REDUCE_OK;
}

int byteps_server_group_destroy(byteps_server_group* g) {
  if (!g) return BYTEPS_REDUCE_OK;
  int rc = BYTEPS_REDUCE_OK;
  for (byteps_server* s : g->inst) {
    const int r = byteps_server_destroy(s);
    if (r && !rc) rc = r;
  }
  delete g;
  return rc;
}

int byteps_server_route(const byteps_server_group_config* cfg, uint64_t key, size_t len,
                        int* npieces, int* server, size_t* offset, size_t* plen, int cap) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  std::vector<Piece> ps;
  route_cfg(*cfg, key, len, &ps);
  return write_pieces(ps, npieces, server, offset, plen, cap);
}

int byteps_server_group_route(byteps_server_group* g, uint64_t key, size_t len, int* npieces,
                              int* server, size_t* offset, size_t* plen, int cap) {
  int rc = check_group(g);
  if (rc) return rc;
  std::vector<Piece> ps;
  route(g, key, len, &ps);
  return write_pieces(ps, npieces, server, offset, plen, cap);
}

int byteps_server_group_instance(byteps_server_group* g, int i, byteps_server** s) {
  int rc = check_group(g);
  if (rc) return rc;
  if (!s || i < 0 || i >= (int)g->inst.size())
    return fail(BYTEPS_REDUCE_EARGS, "instance %d outside [0, %zu)", i, g->inst.size());
  *s = g->inst[i];
  return BYTEPS_REDUCE_OK;
}

int byteps_server_group_init_key(byteps_server_group* g, uint64_t key, size_t len, int dtype) {
  int rc = check_group(g);
  if (rc) return rc;
  std::vector<Piece> ps;
  route(g, key, len, &ps);
  for (const Piece& p : ps)  // the instances refuse a bad dtype / length first
    if ((rc = byteps_server_init_key(g->inst[p.server], key, p.len, dtype))) return rc;
  return declare(g, key, len, dtype);
}

// Would every instance holding a piece of `key` accept a push of `len`
// bytes of `dtype`?  Checked before the group declares the key on first sight,
// so a refused first push leaves no declaration behind (as init_key: the
// instances first, then the group).
int check_pieces(byteps_server_group* g, uint64_t key, size_t len, int dtype) {
  std::vector<Piece> ps;
  route(g, key, len, &ps);
  for (const Piece& p : ps)
    if (int rc = bpsr::server_check_key(g->inst[p.server], key, p.len, dtype)) return rc;
  return 0;
}

int byteps_server_group_push(byteps_server_group* g, uint64_t key, int worker, const void* data,
                             size_t len, int dtype, int location) {
  int rc = check_group(g);
  if (rc) return rc;
  if (!data) return fail(BYTEPS_REDUCE_EARGS, "null data");
  if (worker < 0 || worker >= g->cfg.server.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker,
                g->cfg.server.num_workers);
  if ((rc = check_pieces(g, key, len, dtype)) || (rc = declare(g, key, len, dtype))) return rc;
  std::vector<Piece> ps;
  route(g, key, len, &ps);
  const char* d = static_cast<const char*>(data);
  if (ps.size() == 1 || g->cfg.server.engine_blocking) {
    // one instance, or the engine's blocking contract piece by piece (each
    // piece in its own instance's arrival order)
    for (const Piece& p : ps)
      if ((rc = byteps_server_push(g->inst[p.server], key, worker, d + p.off, p.len, dtype,
                                   location)))
        return rc;
    return BYTEPS_REDUCE_OK;
  }
  std::vector<PushPiece> pcs;
  for (const Piece& p : ps) pcs.push_back({g->inst[p.server], key, d + p.off, p.len, true, -1});
  return scatter_pushes(g, pcs, worker, dtype, location);
}

int byteps_server_group_pull(byteps_server_group* g, uint64_t key, void* out, size_t len,
                             int location) {
  int rc = check_group(g);
  if (rc) return rc;
  if (!out) return fail(BYTEPS_REDUCE_EARGS, "null out");
  std::vector<Piece> ps;
  if ((rc = pull_pieces(g, key, len, &ps))) return rc;
  char* o = static_cast<char*>(out);
  if (ps.size() > 1 && g->pulls_async && addressable(out, location)) {
    std::vector<PullPiece> pcs;
    for (const Piece& p : ps) pcs.push_back({g->inst[p.server], key, o + p.off, p.len});
    return gather_pulls(pcs, location);
  }
  // one piece; or pageable host memory, or an engine that answers each pull
  // by its own rules (scheduling, engine blocking, async mode): piece by piece
  for (const Piece& p : ps)
    if ((rc = byteps_server_pull(g->inst[p.server], key, o + p.off, p.len, location))) return rc;
  return BYTEPS_REDUCE_OK;
}

int byteps_server_group_pull_host_view(byteps_server_group* g, uint64_t key, const void** data,
                                       size_t* len) {
  if (!data) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  *data = nullptr;
  if (len) *len = 0;
  int rc = check_group(g);
  if (rc) return rc;
  const size_t klen = declared_len(g, key);
  std::vector<Piece> ps;
  route(g, key, klen ? klen : 1, &ps);
  if (ps.size() != 1)
    return fail(BYTEPS_REDUCE_EARGS,
                "key %llu is split over %zu instances: no single view (pull it, or view each "
                "piece through byteps_server_group_instance)", (unsigned long long)key, ps.size());
  return byteps_server_pull_host_view(g->inst[ps[0].server], key, data, len);
}

int byteps_server_group_push_many(byteps_server_group* g, const uint64_t* keys,
                                  const void* const* datas, const size_t* lens, int n, int worker,
                                  int dtype, int location) {
  int rc = check_group(g);
  if (rc) return rc;
  if (n < 0 || (n > 0 && (!keys || !datas || !lens))) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  if (worker < 0 || worker >= g->cfg.server.num_workers)
    return fail(BYTEPS_REDUCE_EARGS, "worker %d outside [0, %d)", worker,
                g->cfg.server.num_workers);
  std::vector<Piece> ps;
  for (int i = 0; i < n; ++i) {
    if (!datas[i]) return fail(BYTEPS_REDUCE_EARGS, "null data for key %d", i);
    if ((rc = check_pieces(g, keys[i], lens[i], dtype))) return rc;
  }
  for (int i = 0; i < n; ++i)
    if ((rc = declare(g, keys[i], lens[i], dtype))) return rc;
  if (g->cfg.server.engine_blocking) {
    // the engine's blocking contract: each instance's keys as one batched call
    const size_t ns = g->inst.size();
    std::vector<std::vector<uint64_t>> k(ns);
    std::vector<std::vector<const void*>> d(ns);
    std::vector<std::vector<size_t>> l(ns);
    for (int i = 0; i < n; ++i) {
      route(g, keys[i], lens[i], &ps);
      for (const Piece& p : ps) {
        k[p.server].push_back(keys[i]);
        d[p.server].push_back(static_cast<const char*>(datas[i]) + p.off);
        l[p.server].push_back(p.len);
      }
    }
    for (size_t s = 0; s < ns; ++s)
      if (!k[s].empty() &&
          (rc = byteps_server_push_many(g->inst[s], k[s].data(), d[s].data(), l[s].data(),
                                        (int)k[s].size(), worker, dtype, location)))
        return rc;
    return BYTEPS_REDUCE_OK;
  }
  // every piece of every key queued at once on its instance: the instances'
  // copies and folds run in parallel (one PCIe link / HBM per GPU), each
  // instance's lane issuers batching what piles up
  std::vector<PushPiece> pcs;
  for (int i = 0; i < n; ++i) {
    route(g, keys[i], lens[i], &ps);
    for (const Piece& p : ps)
      pcs.push_back({g->inst[p.server], keys[i], static_cast<const char*>(datas[i]) + p.off,
                     p.len, ps.size() > 1, -1});
  }
  return scatter_pushes(g, pcs, worker, dtype, location);
}

int byteps_server_group_pull_many(byteps_server_group* g, const uint64_t* keys, void* const* outs,
                                  const size_t* lens, int n, int location) {
  int rc = check_group(g);
  if (rc) return rc;
  if (n < 0 || (n > 0 && (!keys || !outs || !lens))) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  const size_t ns = g->inst.size();
  std::vector<std::vector<uint64_t>> k(ns);
  std::vector<std::vector<void*>> o(ns);
  std::vector<std::vector<size_t>> l(ns);
  std::vector<PullPiece> pcs;
  bool gather = g->pulls_async;
  std::vector<Piece> ps;
  for (int i = 0; i < n; ++i) {
    if (!outs[i]) return fail(BYTEPS_REDUCE_EARGS, "null out for key %d", i);
    if ((rc = pull_pieces(g, keys[i], lens[i], &ps))) return rc;
    gather = gather && addressable(outs[i], location);
    for (const Piece& p : ps) {
      k[p.server].push_back(keys[i]);
      o[p.server].push_back(static_cast<char*>(outs[i]) + p.off);
      l[p.server].push_back(p.len);
      pcs.push_back({g->inst[p.server], keys[i], static_cast<char*>(outs[i]) + p.off, p.len});
    }
  }
  if (gather) return gather_pulls(pcs, location);  // every instance at once
  for (size_t s = 0; s < ns; ++s)
    if (!k[s].empty() &&
        (rc = byteps_server_pull_many(g->inst[s], k[s].data(), o[s].data(), l[s].data(),
                                      (int)k[s].size(), location)))
      return rc;
  return BYTEPS_REDUCE_OK;
}

int byteps_server_group_order_after(byteps_server_group* g, const uint64_t* keys, int n,
                                    void* event) {
  int rc = check_group(g);
  if (rc) return rc;
  if (!event || n < 0 || (n > 0 && !keys)) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  const size_t ns = g->inst.size();
  std::vector<std::vector<uint64_t>> k(ns);
  std::vector<char> all(ns, n == 0 ? 1 : 0);
  std::vector<Piece> ps;
  for (int i = 0; i < n; ++i) {
    const size_t klen = declared_len(g, keys[i]);
    if (klen == 0) {  // not declared yet: wherever it may land
      std::fill(all.begin(), all.end(), 1);
      break;
    }
    route(g, keys[i], klen, &ps);
    for (const Piece& p : ps) k[p.server].push_back(keys[i]);
  }
  for (size_t s = 0; s < ns; ++s) {
    if (all[s])
      rc = byteps_server_order_after(g->inst[s], nullptr, 0, event);
    else if (!k[s].empty())
      rc = byteps_server_order_after(g->inst[s], k[s].data(), (int)k[s].size(), event);
    if (rc) return rc;
  }
  return BYTEPS_REDUCE_OK;
}

}  // extern "C"
