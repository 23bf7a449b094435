// Native driver of config 3's keys through the PS server (not product code),
// loaded by bench.py (the line's `server_cfg3` object) through ctypes: the
// timed rounds run here, on the calling thread, with no Python in the loop.
//
// The shape is the reference server's (server.cc:147-308 behind ps-lite's ONE
// receive thread, server.cc:149): 8 workers' pushes of the 165 BytePS
// partitions of ResNet-50 fp16 already sit in the server's receive slots (an
// RDMA transport writing into HBM, byteps_server_recv_slot); per round the
// receive thread signals every arrival (byteps_server_push_ready, keys in
// Prophet block order, workers in order) and then answers every pull with a
// zero-copy device view of the store (byteps_server_pull_device_view: what a
// GPUDirect transport sends from).  A round ends when the last view is handed
// out, i.e. every key's fold has completed.  Whether the folds go out as lane
// launches or through the keyed consumer (device releases) is the server's
// BPSR_SERVER_RELEASE, read when the server is created.
//
// After the timed rounds one checking round pulls every key into every
// worker's `outs` buffer (byteps_server_pull, device copies) and the recorded
// arrival order of every key goes to `orders`, so the caller can check the
// bits against its own fold of `grads` in that order.
//
//   hipcc -O2 -std=c++17 -shared -fPIC -Iinclude tools/cfg3srv_drv.cpp \
//     -o tools/libcfg3srv.so -Lprophet_amd -lbpsr -Wl,-rpath,'$ORIGIN/../prophet_amd'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "bpsr/server.h"

namespace {

int hip_rc(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  fprintf(stderr, "cfg3srv: %s: %s\n", what, hipGetErrorString(e));
  return BYTEPS_REDUCE_EHIP;
}

}  // namespace

// np keys (key i = partition i: offs[i], lens[i] bytes into each worker's
// vector), nw workers' device vectors grads[w] and pull buffers outs[w],
// fp16.  res[0..7] = median round ms, min round ms, median push phase ms,
// fold launches / round, consumer launches / round, key releases / round,
// rounds timed, max round ms.  orders: np * nw ints.  0 or a negative
// BYTEPS_REDUCE_E* code (its message on stderr).
extern "C" int cfg3srv_run(int np, const size_t* offs, const size_t* lens, int nw,
                           void* const* grads, void* const* outs, int rounds, int lanes,
                           double* res, int* orders) {
  byteps_server_config cfg;
  std::memset(&cfg, 0, sizeof(cfg));
  cfg.num_workers = nw;
  cfg.engine_lanes = lanes;
  cfg.policy = BYTEPS_SERVER_FUSED;
  byteps_server* srv = nullptr;
  int rc = byteps_server_create(&cfg, &srv);
  if (rc) {
    fprintf(stderr, "cfg3srv: create: %s\n", byteps_reduce_last_error());
    return rc;
  }
  auto fail = [&](int r, const char* what) {
    fprintf(stderr, "cfg3srv: %s: rc=%d %s\n", what, r, byteps_reduce_last_error());
    byteps_server_destroy(srv);
    return r;
  };
  // init round: blocking device pushes, one thread per worker (each is
  // answered once every worker's is in), keys in order
  {
    std::vector<int> rcs(nw, 0);
    std::vector<std::thread> th;
    for (int w = 0; w < nw; ++w)
      th.emplace_back([&, w] {
        for (int i = 0; i < np && !rcs[w]; ++i)
          rcs[w] = byteps_server_push(srv, (uint64_t)i, w,
                                      static_cast<const char*>(grads[w]) + offs[i], lens[i],
                                      BYTEPS_REDUCE_FLOAT16, BYTEPS_SERVER_DEVICE);
      });
    for (auto& t : th) t.join();
    for (int w = 0; w < nw; ++w)
      if (rcs[w]) return fail(rcs[w], "init push");
  }
  // the transport has written every worker's push into its slot (once)
  for (int w = 0; w < nw; ++w)
    for (int i = 0; i < np; ++i) {
      void* slot = nullptr;
      if ((rc = byteps_server_recv_slot(srv, (uint64_t)i, w, &slot))) return fail(rc, "recv_slot");
      if ((rc = hip_rc(hipMemcpy(slot, static_cast<const char*>(grads[w]) + offs[i], lens[i],
                                 hipMemcpyDeviceToDevice), "slot copy")))
        return fail(rc, "slot copy");
    }
  uint64_t st0[11] = {0}, st1[11] = {0};
  const int warm = 2;
  std::vector<double> ts, push_ts;
  for (int r = 0; r < warm + rounds; ++r) {
    if (r == warm && (rc = byteps_server_stats(srv, st0, 11))) return fail(rc, "stats");
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < np; ++i)
      for (int w = 0; w < nw; ++w)
        if ((rc = byteps_server_push_ready(srv, (uint64_t)i, w))) return fail(rc, "push_ready");
    const auto t1 = std::chrono::steady_clock::now();
    for (int i = 0; i < np; ++i)
      for (int w = 0; w < nw; ++w) {
        const void* v = nullptr;
        size_t vl = 0;
        if ((rc = byteps_server_pull_device_view(srv, (uint64_t)i, &v, &vl)))
          return fail(rc, "pull_device_view");
        if (!v || vl != lens[i]) return fail(BYTEPS_REDUCE_EARGS, "view length");
      }
    const auto t2 = std::chrono::steady_clock::now();
    if (r >= warm) {
      ts.push_back(std::chrono::duration<double, std::milli>(t2 - t0).count());
      push_ts.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
    }
  }
  if ((rc = byteps_server_stats(srv, st1, 11))) return fail(rc, "stats");
  // checking round: copying pulls into every worker's buffer, then the orders
  for (int i = 0; i < np; ++i)
    for (int w = 0; w < nw; ++w)
      if ((rc = byteps_server_push_ready(srv, (uint64_t)i, w))) return fail(rc, "push_ready");
  for (int i = 0; i < np; ++i)
    for (int w = 0; w < nw; ++w)
      if ((rc = byteps_server_pull(srv, (uint64_t)i, static_cast<char*>(outs[w]) + offs[i],
                                   lens[i], BYTEPS_SERVER_DEVICE)))
        return fail(rc, "pull");
  for (int i = 0; i < np; ++i) {
    uint64_t done = 0;
    int lane = 0;
    if ((rc = byteps_server_key_info(srv, (uint64_t)i, &done, &lane, orders + (size_t)i * nw, nw)))
      return fail(rc, "key_info");
  }
  if ((rc = hip_rc(hipDeviceSynchronize(), "sync"))) return fail(rc, "sync");
  std::vector<double> s = ts, p = push_ts;
  std::sort(s.begin(), s.end());
  std::sort(p.begin(), p.end());
  const double nr = (double)rounds;
  res[0] = s[s.size() / 2];
  res[1] = s.front();
  res[2] = p[p.size() / 2];
  res[3] = (double)(st1[0] - st0[0]) / nr;  // fold launches
  res[4] = (double)(st1[6] - st0[6]) / nr;  // consumer launches
  res[5] = (double)(st1[7] - st0[7]) / nr;  // key releases
  res[6] = nr;
  res[7] = s.back();
  return byteps_server_destroy(srv);
}
