// Compiled by tests/test_abi.py with the reference's own language level
// (g++ -std=c++11, setup.py:171) and linked against libbpsr.so: proves the C
// ABI and the C++ CpuReducer-shaped wrapper are usable from BytePS's build.
// Runs only host-side validation paths (no GPU needed).
#include <cstdio>
#include <cstring>

#include "bpsr/gpu_reducer.hpp"
#include "bpsr/reduce.h"

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
  std::printf("header_check fails=%d\n", fails);
  return fails;
}
