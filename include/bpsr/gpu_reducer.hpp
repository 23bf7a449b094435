// bpsr/gpu_reducer.hpp — header-only C++11 drop-in for
// byteps::common::CpuReducer (byteps/common/cpu_reducer.h:41-58) on top of the
// C ABI of libbpsr.so (bpsr/reduce.h).  Same method names, argument meaning
// (len in BYTES, DataType ids of common.h:52-65) and int return convention
// (0 = ok; the reference's callers CHECK_GE(ret, 0), server.cc:127-130).
//
// Differences a caller must know:
//   * operands are device pointers (or host memory registered/allocated for
//     device access), not pageable host memory;
//   * a failing call returns a negative status instead of aborting inside the
//     reducer (cpu_reducer.cc:79-80 BPS_CHECK-aborts on an unknown dtype);
//   * with blocking = true (default) every call returns after the work is done,
//     exactly like CpuReducer; with blocking = false calls are queued on the
//     reducer's stream and sync() completes them (the server engine's
//     SUM_RECV ... COPY_MERGED sequence on one key is stream-ordered anyway).
#ifndef BPSR_GPU_REDUCER_HPP
#define BPSR_GPU_REDUCER_HPP

#include <stddef.h>

#include "bpsr/reduce.h"

namespace bpsr {

class GpuReducer {
 public:
  // `stream`: an opaque hipStream_t (NULL = the calling thread's default stream).
  explicit GpuReducer(void* stream = NULL, bool blocking = true, int mode = BYTEPS_REDUCE_MODE_REFERENCE)
      : stream_(stream), blocking_(blocking), mode_(mode) {}

  // CpuReducer::sum(void* dst, void* src, size_t len, DataType dtype)
  int sum(void* dst, void* src, size_t len, int dtype) {
    return done(byteps_reduce_sum(dst, src, len, dtype, stream_));
  }
  // CpuReducer::sum(void* dst, void* src1, void* src2, size_t len, DataType dtype)
  int sum(void* dst, void* src1, void* src2, size_t len, int dtype) {
    return done(byteps_reduce_sum3(dst, src1, src2, len, dtype, stream_));
  }
  // CpuReducer::copy(void* dst, void* src, size_t len)
  int copy(void* dst, void* src, size_t len) {
    return done(byteps_reduce_copy(dst, src, len, stream_));
  }
  // CpuReducer::GetDataType(int)
  int GetDataType(int dtype) const { return dtype; }

  // One server round of a key in one launch: dst = ((srcs[0] + srcs[1]) + ...).
  int sum_n(void* dst, const void* const* srcs, int n, size_t len, int dtype) {
    return done(byteps_reduce_sum_n(dst, srcs, n, len, dtype, mode_, stream_));
  }
  int sync() { return byteps_reduce_sync(stream_); }
  const char* last_error() const { return byteps_reduce_last_error(); }
  void* stream() const { return stream_; }

 private:
  int done(int rc) {
    if (rc != BYTEPS_REDUCE_OK || !blocking_) return rc;
    return byteps_reduce_sync(stream_);
  }
  void* stream_;
  bool blocking_;
  int mode_;
};

}  // namespace bpsr

#endif  // BPSR_GPU_REDUCER_HPP
