/*
 * bpsr/shard.h — key-space sharding across the GPUs of one node (C ABI of
 * libbpsr.so): the worker's intra-node local reduce and the scatter of landed
 * buckets to their owning GPU, for a C++ caller shaped like
 * byteps/common/core_loops.cc.
 *
 * Reference interfaces replaced:
 *   PostNcclCalls(task, REDUCE)     core_loops.cc:184-247  -> byteps_shard_reduce_scatter
 *       (ncclReduceScatter of per = len/size/unit_len elements per rank, then
 *        ncclReduce of the left_elem tail to the root = the LAST rank,
 *        nccl_manager.cc:62-64)
 *   PostNcclCalls(task, REDUCE) with BYTEPS_REDUCE_ROOTS / IsUsingReduce()
 *                                   core_loops.cc:212-218  -> byteps_shard_reduce_root
 *   PostNcclCalls(task, BROADCAST)  core_loops.cc:248-261  -> byteps_shard_allgather
 *       (ncclAllGather of the per-rank slices + ncclBroadcast of the tail)
 *   BROADCAST under IsUsingReduce() (whole partition from the key's root)
 *                                                          -> byteps_shard_broadcast
 *   GetReduceRootByKey              global.h:107-108       -> byteps_shard_reduce_root_of
 *   NcclManager::ConstructRings     nccl_manager.cc:74-127 -> byteps_shard_get_unique_id
 *                                                             + byteps_shard_comm_init
 *
 * Ownership (core_loops.cc:210-211): with E elements over W ranks, per = E / W;
 * rank g owns elements [g*per, (g+1)*per) and the last rank also owns the
 * E - per*W tail (it is the reference's NCCL root).
 *
 * Arithmetic: unlike ncclReduceScatter / ncclReduce, whose summation order
 * follows RCCL's ring or tree, every owner here receives its slice of every
 * rank's vector by point-to-point copies (RCCL grouped send/recv over xGMI)
 * and folds them with the gfx950 fold kernel as a strict left fold in RANK
 * order, ((v_0 + v_1) + v_2) + ... — bit-reproducible and bit-identical to the
 * CpuReducer fold of the same vectors (fp16: round after every add; mode as in
 * reduce.h).  Bytes move as untyped bytes, so every reduce.h dtype (bf16
 * included) is supported.
 *
 * Communicators: an opaque byteps_shard_comm wraps either
 *   - an RCCL communicator the library creates the way NcclManager does
 *     (rank 0 calls byteps_shard_get_unique_id, the caller carries the
 *     BYTEPS_SHARD_UNIQUE_ID_BYTES bytes to every rank out of band, every rank
 *     calls byteps_shard_comm_init), or
 *   - an RCCL communicator the caller already owns (byteps_shard_comm_wrap,
 *     e.g. NcclManager::GetComm(key, op)); it is not destroyed here, or
 *   - an in-process group for ONE process driving several GPUs (a PS server
 *     process owning all of the node's GPUs; tests on one device):
 *     byteps_shard_comm_init_local creates `world` communicators at once, one
 *     per rank, each to be used by its own host thread.  Transfers are device
 *     copies ordered by HIP events; no RCCL.
 * RCCL is loaded at first use (dlopen of librccl.so.1 — in a process that
 * already loaded one, e.g. torch's, that same library), so libbpsr.so does not
 * link it.
 *
 * Calls are collective: every rank of the communicator makes the same call,
 * with the same elems and dtype, in the same order (as RCCL requires).  They
 * are asynchronous on `stream` (NULL = the calling thread's default stream,
 * hipStreamPerThread) except that an in-process group call returns only once
 * every peer has posted its transfers.  Buffers are device memory the caller
 * owns.  Errors: 0 or a negative BYTEPS_REDUCE_E* code (BYTEPS_REDUCE_ERCCL for
 * a failed RCCL call) with byteps_reduce_last_error(); nothing aborts.
 */
#ifndef BPSR_SHARD_H
#define BPSR_SHARD_H

#include <stddef.h>
#include <stdint.h>

#include "bpsr/reduce.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Only the declarations below leave libbpsr.so: it is compiled with
 * -fvisibility=hidden and linked with the reference's export policy
 * (byteps.lds:1-8, global: *byteps*; local: *). */
#pragma GCC visibility push(default)

#define BYTEPS_SHARD_UNIQUE_ID_BYTES 128 /* sizeof(ncclUniqueId) */

typedef struct byteps_shard_comm byteps_shard_comm;

/* Element range [*lo, *hi) that `rank` of `world` owns (core_loops.cc:210-211). */
int byteps_shard_owner_range(size_t elems, int world, int rank, size_t* lo, size_t* hi);

/* GetReduceRootByKey (global.h:107-108): roots[djb2(decimal key) % nroots]. */
int byteps_shard_reduce_root_of(uint64_t key, const int* roots, int nroots);

/* ncclGetUniqueId into id[0 .. BYTEPS_SHARD_UNIQUE_ID_BYTES). */
int byteps_shard_get_unique_id(void* id);
/* ncclCommInitRank on `device` (hipSetDevice first); collective over the ranks. */
int byteps_shard_comm_init(const void* id, int world, int rank, int device,
                           byteps_shard_comm** comm);
/* Wrap a caller-owned ncclComm_t (passed as void*); world/rank/device are read
 * from it.  byteps_shard_comm_destroy frees the wrapper only. */
int byteps_shard_comm_wrap(void* nccl_comm, byteps_shard_comm** comm);
/* In-process group: comms[r] for rank r on devices[r] (devices may repeat). */
int byteps_shard_comm_init_local(int world, const int* devices, byteps_shard_comm** comms);
int byteps_shard_comm_destroy(byteps_shard_comm* comm);
int byteps_shard_comm_info(const byteps_shard_comm* comm, int* world, int* rank, int* device);
/* ncclGetVersion of the RCCL this library bound (e.g. 22703 for 2.27.3): the
 * N > 1 bench line records it with each rank's communicator view. */
int byteps_shard_rccl_version(int* version);

/* Worker local reduce, PostNcclCalls(REDUCE) without reduce roots: rank g's
 * `dst` (owned(g) elements; may be `local` + lo(g) * size, in place as the
 * reference writes out_p + rank * per) receives the rank-order left fold of
 * slice g of every rank's `local` (elems elements).  recv_slots: `world`
 * device pointers of owned(g) elements each, where slice g of rank r's vector
 * lands; recv_slots[g] is not used (the own slice is read from `local`) and may
 * be NULL; all may be NULL on a rank that owns nothing. */
int byteps_shard_reduce_scatter(byteps_shard_comm* comm, const void* local,
                                void* const* recv_slots, void* dst, size_t elems, int dtype,
                                int mode, void* stream);

/* Return leg, PostNcclCalls(BROADCAST): every rank's `full` (elems elements)
 * receives every owner's `owned` slice (rank g passes owned(g) elements;
 * `owned` may be `full` + lo(g) * size, in place).  The tail travels from the
 * last rank, as the reference's ncclBroadcast from its root. */
int byteps_shard_allgather(byteps_shard_comm* comm, const void* owned, void* full, size_t elems,
                           int dtype, void* stream);

/* Landed-bucket scatter: `root` holds n workers' full vectors
 * pushes[0..n) (elems each; ignored on other ranks); every rank g receives
 * slice g of each into recv_slots[0..n) (owned(g) elements each) and folds them
 * in worker order into `dst`.  The root copies its own slices locally. */
int byteps_shard_scatter_reduce(byteps_shard_comm* comm, int root, const void* const* pushes,
                                int n, void* const* recv_slots, void* dst, size_t elems,
                                int dtype, int mode, void* stream);

/* PostNcclCalls(REDUCE) under BYTEPS_REDUCE_ROOTS (core_loops.cc:212-218): the
 * whole vector goes to `root`, whose `dst` (elems; may be `local`, in place)
 * receives the rank-order left fold of every rank's `local`.  recv_slots on the
 * root: `world` pointers of elems elements (recv_slots[root] unused); ignored
 * elsewhere. */
int byteps_shard_reduce_root(byteps_shard_comm* comm, int root, const void* local,
                             void* const* recv_slots, void* dst, size_t elems, int dtype,
                             int mode, void* stream);

/* Whole-vector broadcast from `root` into every rank's `buf` (in place). */
int byteps_shard_broadcast(byteps_shard_comm* comm, int root, void* buf, size_t elems, int dtype,
                           void* stream);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif
#endif /* BPSR_SHARD_H */
