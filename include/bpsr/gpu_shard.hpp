// bpsr/gpu_shard.hpp — header-only C++11 replacement for the worker's
// PostNcclCalls(task, REDUCE / BROADCAST) (byteps/common/core_loops.cc:184-263)
// on top of the shard C ABI (bpsr/shard.h).  Same inputs as the reference
// call site: the partition's base pointer p (= tensor data + offset), the
// output base out_p, len in BYTES, unit_len = bytes per element, the key, and
// the DataType id; the communicator and stream are the ones NcclManager would
// hand out (GetComm / GetStream).
//
//   REDUCE     without reduce roots: this rank's owned elements
//              [lo, hi) (per = len / size / unit_len, tail to the last rank,
//              core_loops.cc:210-211) of out_p receive the rank-order fold of
//              that slice of every rank's p; with BYTEPS_REDUCE_ROOTS
//              (IsUsingReduce, core_loops.cc:212-218) the whole partition is
//              folded on GetReduceRootByKey(key) into its out_p.
//   BROADCAST  all-gather of the owned slices (plus the tail from the last
//              rank) in place in p, or a broadcast of the whole partition from
//              the key's root.
//
// Differences a caller must know: the sum is a strict rank-order left fold
// (bit-reproducible; RCCL's ring reduce is not); receive slots come from a
// caller-owned device scratch buffer (world x owned bytes, or world x len
// with reduce roots; scratch_bytes() tells); calls are asynchronous on the
// stream like the NCCL calls they replace.
#ifndef BPSR_GPU_SHARD_HPP
#define BPSR_GPU_SHARD_HPP

#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "bpsr/shard.h"

namespace bpsr {

class GpuShard {
 public:
  GpuShard(byteps_shard_comm* comm, void* stream, const std::vector<int>& reduce_roots,
           int mode = BYTEPS_REDUCE_MODE_REFERENCE)
      : comm_(comm), stream_(stream), roots_(reduce_roots), mode_(mode), world_(1), rank_(0) {
    int dev = 0;
    if (byteps_shard_comm_info(comm_, &world_, &rank_, &dev) != BYTEPS_REDUCE_OK) {
      world_ = 0;
      rank_ = 0;
    }
  }

  bool using_reduce() const { return !roots_.empty(); }  // BytePSGlobal::IsUsingReduce

  // Device scratch a REDUCE of `len` bytes needs for its receive slots.
  size_t scratch_bytes(size_t len, size_t unit_len) const {
    if (!world_ || !unit_len) return 0;
    if (using_reduce()) return (size_t)world_ * len;
    size_t lo = 0, hi = 0;
    byteps_shard_owner_range(len / unit_len, world_, rank_, &lo, &hi);
    return (size_t)world_ * (hi - lo) * unit_len;
  }

  // PostNcclCalls(task, REDUCE).  scratch: scratch_bytes(len, unit_len) of device memory.
  int reduce(uint64_t key, const void* p, void* out_p, size_t len, size_t unit_len, int dtype,
             void* scratch) {
    if (!world_ || !unit_len || len % unit_len) return BYTEPS_REDUCE_EARGS;
    const size_t elems = len / unit_len;
    std::vector<void*> slots((size_t)world_, (void*)0);
    if (using_reduce()) {
      const int root = byteps_shard_reduce_root_of(key, roots_.data(), (int)roots_.size());
      if (root < 0) return root;
      for (int r = 0; r < world_; ++r) slots[r] = static_cast<char*>(scratch) + (size_t)r * len;
      return byteps_shard_reduce_root(comm_, root, p, slots.data(), out_p, elems, dtype, mode_,
                                      stream_);
    }
    size_t lo = 0, hi = 0;
    int rc = byteps_shard_owner_range(elems, world_, rank_, &lo, &hi);
    if (rc) return rc;
    const size_t owned = (hi - lo) * unit_len;
    for (int r = 0; r < world_; ++r) slots[r] = static_cast<char*>(scratch) + (size_t)r * owned;
    return byteps_shard_reduce_scatter(comm_, p, slots.data(),
                                       static_cast<char*>(out_p) + lo * unit_len, elems, dtype,
                                       mode_, stream_);
  }

  // PostNcclCalls(task, BROADCAST), in place in p.
  int broadcast(uint64_t key, void* p, size_t len, size_t unit_len, int dtype) {
    if (!world_ || !unit_len || len % unit_len) return BYTEPS_REDUCE_EARGS;
    const size_t elems = len / unit_len;
    if (using_reduce()) {
      const int root = byteps_shard_reduce_root_of(key, roots_.data(), (int)roots_.size());
      if (root < 0) return root;
      return byteps_shard_broadcast(comm_, root, p, elems, dtype, stream_);
    }
    size_t lo = 0, hi = 0;
    int rc = byteps_shard_owner_range(elems, world_, rank_, &lo, &hi);
    if (rc) return rc;
    return byteps_shard_allgather(comm_, static_cast<char*>(p) + lo * unit_len, p, elems, dtype,
                                  stream_);
  }

  int world() const { return world_; }
  int rank() const { return rank_; }

 private:
  byteps_shard_comm* comm_;
  void* stream_;
  std::vector<int> roots_;
  int mode_;
  int world_, rank_;
};

}  // namespace bpsr

#endif  // BPSR_GPU_SHARD_HPP
