// Key space sharded over several GPU-resident server instances
// (include/bpsr/server.h, byteps_server_group_*): the reference's key ->
// server assignment (BytePSGlobal::EncodeDefaultKey, global.cc:530-567) for a
// process that owns all of a node's GPUs, or the reduce-scatter owner ranges
// applied to each large partition.  Host-side routing only; every byte of
// data moves and folds inside the instances.
#include "bpsr/server.h"

#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "bpsr_error.h"

namespace bpsr {
namespace {

constexpr size_t kUnit = 128;  // piece granule: 8 elements of every dtype, 16-B aligned

struct Piece {
  int server;
  size_t off, len;
};

}  // namespace
}  // namespace bpsr

struct byteps_server_group {
  byteps_server_group_config cfg;
  std::vector<byteps_server*> inst;
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
  for (const Piece& p : ps)
    if ((rc = byteps_server_init_key(g->inst[p.server], key, p.len, dtype))) return rc;
  return BYTEPS_REDUCE_OK;
}

int byteps_server_group_push(byteps_server_group* g, uint64_t key, int worker, const void* data,
                             size_t len, int dtype, int location) {
  int rc = check_group(g);
  if (rc) return rc;
  if (!data) return fail(BYTEPS_REDUCE_EARGS, "null data");
  std::vector<Piece> ps;
  route(g, key, len, &ps);
  const char* d = static_cast<const char*>(data);
  if (ps.size() == 1 || g->cfg.server.engine_blocking) {
    // one instance, or the engine's blocking contract piece by piece
    for (const Piece& p : ps)
      if ((rc = byteps_server_push(g->inst[p.server], key, worker, d + p.off, p.len, dtype,
                                   location)))
        return rc;
    return BYTEPS_REDUCE_OK;
  }
  // Scatter: every piece's copy queued at once on its instance (its own
  // device and lanes), then wait for all acknowledgements — the data is in
  // HBM and (init round) every worker's init push has arrived, as a
  // blocking push guarantees.
  Acks acks;
  for (const Piece& p : ps) {
    {
      std::lock_guard<std::mutex> lk(acks.mu);
      ++acks.remaining;
    }
    rc = byteps_server_push_async(g->inst[p.server], key, worker, d + p.off, p.len, dtype,
                                  location, ack_cb, &acks);
    if (rc) {
      std::lock_guard<std::mutex> lk(acks.mu);
      --acks.remaining;
      break;
    }
  }
  std::unique_lock<std::mutex> lk(acks.mu);
  acks.cv.wait(lk, [&] { return acks.remaining == 0; });  // queued pieces still read `data`
  return rc ? rc : acks.status;
}

int byteps_server_group_pull(byteps_server_group* g, uint64_t key, void* out, size_t len,
                             int location) {
  int rc = check_group(g);
  if (rc) return rc;
  if (!out) return fail(BYTEPS_REDUCE_EARGS, "null out");
  std::vector<Piece> ps;
  route(g, key, len, &ps);
  char* o = static_cast<char*>(out);
  for (const Piece& p : ps)
    if ((rc = byteps_server_pull(g->inst[p.server], key, o + p.off, p.len, location))) return rc;
  return BYTEPS_REDUCE_OK;
}

int byteps_server_group_push_many(byteps_server_group* g, const uint64_t* keys,
                                  const void* const* datas, const size_t* lens, int n, int worker,
                                  int dtype, int location) {
  int rc = check_group(g);
  if (rc) return rc;
  if (n < 0 || (n > 0 && (!keys || !datas || !lens))) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  const size_t ns = g->inst.size();
  std::vector<std::vector<uint64_t>> k(ns);
  std::vector<std::vector<const void*>> d(ns);
  std::vector<std::vector<size_t>> l(ns);
  std::vector<Piece> ps;
  for (int i = 0; i < n; ++i) {
    if (!datas[i]) return fail(BYTEPS_REDUCE_EARGS, "null data for key %d", i);
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

int byteps_server_group_pull_many(byteps_server_group* g, const uint64_t* keys, void* const* outs,
                                  const size_t* lens, int n, int location) {
  int rc = check_group(g);
  if (rc) return rc;
  if (n < 0 || (n > 0 && (!keys || !outs || !lens))) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  const size_t ns = g->inst.size();
  std::vector<std::vector<uint64_t>> k(ns);
  std::vector<std::vector<void*>> o(ns);
  std::vector<std::vector<size_t>> l(ns);
  std::vector<Piece> ps;
  for (int i = 0; i < n; ++i) {
    if (!outs[i]) return fail(BYTEPS_REDUCE_EARGS, "null out for key %d", i);
    route(g, keys[i], lens[i], &ps);
    for (const Piece& p : ps) {
      k[p.server].push_back(keys[i]);
      o[p.server].push_back(static_cast<char*>(outs[i]) + p.off);
      l[p.server].push_back(p.len);
    }
  }
  for (size_t s = 0; s < ns; ++s)
    if (!k[s].empty() &&
        (rc = byteps_server_pull_many(g->inst[s], k[s].data(), o[s].data(), l[s].data(),
                                      (int)k[s].size(), location)))
      return rc;
  return BYTEPS_REDUCE_OK;
}

}  // extern "C"
