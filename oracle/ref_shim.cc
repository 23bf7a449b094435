// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product library.
//
// C-ABI shim around the reference's own byteps::common::CpuReducer, compiled
// straight from /root/reference/byteps/common/{cpu_reducer.cc,logging.cc} with
// the reference's server build flags (setup.py:171-172, 284-291) by
// oracle/Makefile into oracle/_ref/libbpsr_ref.so.  This file contains no
// reference code; it only instantiates the reference class and forwards.
//
// Used by: oracle/gen_golden.py (golden vectors), tests/ (pinning the clean-room
// restatement oracle/bpsr_oracle.c), bench.py cpu_baseline leg (kind
// "reference").
#include <cstddef>
#include <cstdint>

#include "cpu_reducer.h"

using byteps::common::CpuReducer;

extern "C" {

// One reducer per call site; the constructor reads BYTEPS_OMP_THREAD_PER_GPU
// (cpu_reducer.cc:40-44), so callers set the env var before creating it.
void* bpsr_ref_create(void) { return new CpuReducer(nullptr); }

void bpsr_ref_destroy(void* r) { delete static_cast<CpuReducer*>(r); }

// cpu_reducer.cc:57-83 — in place dst += src, len in bytes.
int bpsr_ref_sum(void* r, void* dst, void* src, size_t len, int dtype) {
  auto* red = static_cast<CpuReducer*>(r);
  return red->sum(dst, src, len, red->GetDataType(dtype));
}

// cpu_reducer.cc:130-162 — dst = src1 + src2 (no callers upstream).
int bpsr_ref_sum3(void* r, void* dst, void* src1, void* src2, size_t len,
                  int dtype) {
  auto* red = static_cast<CpuReducer*>(r);
  return red->sum(dst, src1, src2, len, red->GetDataType(dtype));
}

// cpu_reducer.cc:209-220 — word copy + trailing bytes.
int bpsr_ref_copy(void* r, void* dst, void* src, size_t len) {
  return static_cast<CpuReducer*>(r)->copy(dst, src, len);
}

}  // extern "C"
