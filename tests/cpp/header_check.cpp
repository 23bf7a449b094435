// Compiled by tests/test_abi.py with the reference's own language level
// (g++ -std=c++11, setup.py:171) and linked against libbpsr.so: proves the C
// ABI and the C++ CpuReducer-shaped wrapper are usable from BytePS's build.
// Runs only host-side validation paths (no GPU needed).
#include <cstdio>
#include <cstring>

#include "bpsr/gpu_reducer.hpp"
#include "bpsr/gpu_shard.hpp"
#include "bpsr/reduce.h"
#include "bpsr/shard.h"

int main() {
  bpsr::GpuReducer r(NULL, /*blocking=*/false);  // no stream sync: no GPU here
  int fails = 0;
  // unknown dtype: -1 (the reference aborts here, cpu_reducer.cc:79-80)
  if (r.sum(reinterpret_cast<void*>(0x1000), reinterpret_cast<void*>(0x2000), 64, 9) !=
      BYTEPS_REDUCE_EDTYPE) ++fails;
  if (std::strstr(r.last_error(), "Unsupported data type") == NULL) ++fails;
  // partial overlap: -2
  if (r.sum(reinterpret_cast<void*>(0x1000), reinterpret_cast<void*>(0x1004), 64, 0) !=
      BYTEPS_REDUCE_EARGS) ++fails;
  // zero length: no-op success, like the reference's empty loop
  if (r.copy(reinterpret_cast<void*>(0x1000), reinterpret_cast<void*>(0x2000), 0) != 0) ++fails;
  if (byteps_reduce_dtype_size(BYTEPS_REDUCE_FLOAT16) != 2) ++fails;
  if (byteps_reduce_version() != BYTEPS_REDUCE_ABI_VERSION) ++fails;
  byteps_reduce_plan* p = NULL;
  if (byteps_reduce_plan_create(NULL, -1, 0, 0, &p) != BYTEPS_REDUCE_EARGS || p != NULL) ++fails;
  // shard ABI (bpsr/shard.h) and the PostNcclCalls-shaped wrapper: host-only paths
  size_t lo = 0, hi = 0;
  if (byteps_shard_owner_range(10007, 3, 2, &lo, &hi) != 0 || lo != 6670 || hi != 10007) ++fails;
  byteps_shard_comm* comms[3] = {NULL, NULL, NULL};
  const int devs[3] = {0, 0, 0};
  if (byteps_shard_comm_init_local(3, devs, comms) != 0) ++fails;
  std::vector<int> no_roots, roots(2);
  roots[0] = 1;
  roots[1] = 2;
  bpsr::GpuShard rs(comms[1], NULL, no_roots), rr(comms[1], NULL, roots);
  if (rs.world() != 3 || rs.rank() != 1 || rr.using_reduce() != true) ++fails;
  if (rs.scratch_bytes(4 * 10007, 4) != 3 * 3335 * 4) ++fails;
  if (rr.scratch_bytes(4 * 10007, 4) != 3 * 4 * 10007) ++fails;
  if (rs.reduce(1, NULL, NULL, 10, 4, 0, NULL) != BYTEPS_REDUCE_EARGS) ++fails;  // len % unit
  if (rs.reduce(1, NULL, NULL, 40, 4, 9, NULL) != BYTEPS_REDUCE_EDTYPE) ++fails;
  if (rr.broadcast(1, NULL, 40, 4, 0) != BYTEPS_REDUCE_EARGS) ++fails;       // null buffer
  const int root = byteps_shard_reduce_root_of(65536, roots.data(), 2);
  if (root != 1 && root != 2) ++fails;
  for (int i = 0; i < 3; ++i)
    if (byteps_shard_comm_destroy(comms[i]) != 0) ++fails;
  std::printf("header_check fails=%d\n", fails);
  return fails;
}
