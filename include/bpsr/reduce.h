/*
 * bpsr/reduce.h — C ABI of libbpsr.so, the MI355X (gfx950) gradient-bucket
 * reducer that replaces the host-side CpuReducer of Prophet/BytePS.
 *
 * Every exported name matches `*byteps*`, so it survives the reference's own
 * linker version script (byteps.lds:1-8 exports only *byteps*, *PyInit*,
 * *initc_lib*).  No torch, HIP or C++ types cross this boundary: pointers are
 * device pointers (or host pointers registered/allocated for device access),
 * lengths are BYTES exactly as in the reference, streams are opaque
 * hipStream_t handles passed as void* (NULL = the calling thread's default
 * stream, hipStreamPerThread).
 *
 * Reference interfaces replaced (byteps/common/cpu_reducer.h:41-58):
 *   CpuReducer::sum(void* dst, void* src, size_t len, DataType)      -> byteps_reduce_sum
 *   CpuReducer::sum(void* dst, void* s1, void* s2, size_t, DataType) -> byteps_reduce_sum3
 *   CpuReducer::copy(void* dst, void* src, size_t len)               -> byteps_reduce_copy
 *   the server's per-key fold, byteps/server/server.cc:216-273
 *   (first arrival = accumulator, N-1 SUM_RECV jobs, COPY_MERGED)    -> byteps_reduce_sum_n
 *   one Prophet block of buckets released together
 *   (byteps/common/scheduled_queue.cc:244-296)                       -> byteps_reduce_sum_batched
 *
 * Semantics (bit-exact parity with the compiled reference):
 *   - sum: dst[i] = dst[i] + src[i] for i < len / sizeof(T); the trailing
 *     len % sizeof(T) bytes are NOT touched (cpu_reducer.cc:88).
 *   - fp16: fp32 add then round-to-nearest-even to fp16 after EVERY add
 *     (cpu_reducer.cc:101-125); NaN payload rules of the F16C body for
 *     i < floor(n/8)*8 and 0x7fff for the scalar tail (cpu_reducer.h:77-173).
 *   - integers wrap (two's complement).
 *   - copy: all len bytes (cpu_reducer.cc:209-220).
 *   - sum_n: strict left fold ((s0 + s1) + s2) + ... in the given order.
 *
 * Errors: 0 on success, a negative BYTEPS_REDUCE_E* code otherwise.  Nothing
 * aborts across this ABI (the reference BPS_CHECK-aborts on a bad dtype,
 * cpu_reducer.cc:79-80).  byteps_reduce_last_error() returns a thread-local
 * message for the last failing call on the calling thread.
 *
 * Threading: calls are thread-safe for distinct buffers (the reference calls
 * CpuReducer from BYTEPS_SERVER_ENGINE_THREAD engine threads on distinct
 * keys, server.cc:70-145).  All compute calls are asynchronous on `stream`;
 * byteps_reduce_sync(stream) completes them.
 */
#ifndef BPSR_REDUCE_H
#define BPSR_REDUCE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Only the declarations below leave libbpsr.so: it is compiled with
 * -fvisibility=hidden and linked with the reference's export policy
 * (byteps.lds:1-8, global: *byteps*; local: *). */
#pragma GCC visibility push(default)

/* 3: byteps_server_config.engine_blocking; bpsr/shard.h
 * 4: byteps_server_config.release; byteps_shard_rccl_version
 * 5: byteps_server_create_sized (a caller states its config's size) */
#define BYTEPS_REDUCE_ABI_VERSION 5

/* Data type ids: byteps/common/common.h:52-65 (mshadow order), plus bf16 as a
 * build extension (the reference has none). */
enum byteps_reduce_dtype {
  BYTEPS_REDUCE_FLOAT32 = 0,
  BYTEPS_REDUCE_FLOAT64 = 1,
  BYTEPS_REDUCE_FLOAT16 = 2,
  BYTEPS_REDUCE_UINT8 = 3,
  BYTEPS_REDUCE_INT32 = 4,
  BYTEPS_REDUCE_INT8 = 5,
  BYTEPS_REDUCE_INT64 = 6,
  BYTEPS_REDUCE_BFLOAT16 = 11
};

/* Rounding mode for the 16-bit float types (ignored for the others). */
enum byteps_reduce_mode {
  /* Round to the storage type after every pairwise add: bit-exact with the
   * reference CpuReducer fold.  Default. */
  BYTEPS_REDUCE_MODE_REFERENCE = 0,
  /* Accumulate all N inputs in fp32 and round once at the end (more accurate,
   * not bit-exact; documented tolerance <= 1 ulp of the exact sum for N <= 32). */
  BYTEPS_REDUCE_MODE_ACCUM_F32 = 1
};

enum byteps_reduce_status {
  BYTEPS_REDUCE_OK = 0,
  BYTEPS_REDUCE_EDTYPE = -1,   /* unsupported data type                      */
  BYTEPS_REDUCE_EARGS = -2,    /* bad pointer / count / overlap / mode        */
  BYTEPS_REDUCE_EHIP = -3,     /* HIP runtime error (launch, copy, event)     */
  BYTEPS_REDUCE_ERCCL = -4,    /* collective error (reserved for shard APIs)  */
  BYTEPS_REDUCE_ETIMEOUT = -5, /* a block queue launch gave up on a release   */
  BYTEPS_REDUCE_ECANCELED = -6 /* a queued server pull dropped at shutdown    */
};

/* Most sources one kernel launch folds; byteps_reduce_sum_n chains launches
 * for more (still a strict left fold). */
#define BYTEPS_REDUCE_MAX_SRCS 32

/* One bucket of a batched (Prophet block) reduction: dst = fold(srcs[0..n-1]).
 * dst may alias srcs[0]. */
typedef struct byteps_bucket_desc {
  void* dst;
  const void* srcs[BYTEPS_REDUCE_MAX_SRCS];
  size_t len;   /* bytes */
  int n;        /* 1 <= n <= BYTEPS_REDUCE_MAX_SRCS */
  int reserved;
} byteps_bucket_desc;

/* Library version (BYTEPS_REDUCE_ABI_VERSION). */
int byteps_reduce_version(void);

/* Optional eager initialisation for `device` (hipSetDevice + kernel warm-up);
 * every other call initialises lazily on the current device. */
int byteps_reduce_init(int device);
int byteps_reduce_shutdown(void);

/* CpuReducer::sum(dst, src, len, dtype), cpu_reducer.cc:57-83. */
int byteps_reduce_sum(void* dst, const void* src, size_t len, int dtype, void* stream);

/* CpuReducer::sum(dst, src1, src2, len, dtype), cpu_reducer.cc:130-162. */
int byteps_reduce_sum3(void* dst, const void* src1, const void* src2, size_t len,
                       int dtype, void* stream);

/* Fused N-way left fold: dst = ((srcs[0] + srcs[1]) + ...) + srcs[n-1].
 * dst may alias srcs[0] exactly (the server's zero-copy accumulator,
 * server.cc:216-218); partial overlaps are rejected.  Trailing bytes
 * (len % sizeof(T)) of dst are copied from srcs[0]. */
int byteps_reduce_sum_n(void* dst, const void* const* srcs, int n, size_t len,
                        int dtype, int mode, void* stream);

/* One launch for a whole block of buckets (all of one dtype). */
int byteps_reduce_sum_batched(const byteps_bucket_desc* buckets, int nbuckets,
                              int dtype, int mode, void* stream);

/* A reusable batched reduction: the bucket table of one Prophet block is
 * validated and uploaded to the device once (at plan creation, on the current
 * device); every launch is then ONE kernel with no host work, no allocation
 * and no synchronisation, so it can be captured into a hipGraph.  The reference
 * keys, partitions and server receive buffers are fixed after InitTensor
 * (operations.cc:219-316), so a block's table is fixed across iterations. */
typedef struct byteps_reduce_plan byteps_reduce_plan;
int byteps_reduce_plan_create(const byteps_bucket_desc* buckets, int nbuckets, int dtype,
                              int mode, byteps_reduce_plan** plan);
int byteps_reduce_plan_launch(byteps_reduce_plan* plan, void* stream);
int byteps_reduce_plan_destroy(byteps_reduce_plan* plan);

/* Persistent block consumer: the buckets of one training iteration, grouped
 * into Prophet blocks in release order (block i = buckets
 * [block_end[i-1], block_end[i]), block_end[nblocks-1] == nbuckets), folded by
 * ONE resident kernel per iteration instead of one launch per block.  The
 * kernel takes tiles in table order and starts a block's tiles once that block
 * and every block before it are released, so a block is folded as soon as its
 * pushes have landed — no per-block launch, no per-block drain.  It replaces
 * the per-block release loop of scheduled_queue.cc:244-296 followed by one
 * reduce call per released partition.
 *
 *   launch(q, s)           enqueue the iteration's consumer on stream s;
 *   release(q, b, s)       mark block b released once the work queued before it
 *                          on stream s (e.g. the block's H2D pushes) has
 *                          completed; b < 0 releases every block;
 *   release_range(q, f, c, s)  the same for blocks [f, f + c) in ONE kernel
 *                          (a Prophet release group spanning several blocks);
 *   status(q, s)           synchronise s and report whether a launch gave up:
 *                          a workgroup that waits longer than the timeout
 *                          (default 2 s) for a release sets a sticky error, every
 *                          workgroup then stops and status returns
 *                          BYTEPS_REDUCE_ETIMEOUT (and clears it).
 *
 * Iterations are numbered by epochs (host call order): launch k waits for the
 * k-th release of every block (its release word >= k), so nothing is re-armed
 * between iterations, a block may be released before or after its
 * iteration's launch, and later iterations can be enqueued at once (the
 * caller keeps iteration k + 1's data from landing before launch k consumed
 * the buffers).  Every block must be released once per iteration.  After
 * ETIMEOUT, status() counts the abandoned iteration's missing releases as
 * given.  A launch captured into a hipGraph replays with its epoch fixed, so a
 * capture must release every block before the launch (EARGS otherwise).  One
 * launch of a queue at a time.  Launch and release may be called from
 * different threads.  Table residency as for plans (buffers fixed after
 * InitTensor).  When
 * a block's data lands after the launch, its buffers should not share a 128-B
 * line with an earlier block's (a line read for the earlier block may be
 * cached ahead of the later block's DMA).
 *
 * Live releases need the consumer and the releasing stream on DIFFERENT
 * hardware queues: HIP multiplexes streams onto a few in-order hardware queues
 * per process (GPU_MAX_HW_QUEUES, 4 by default), and a release queued behind
 * the running consumer in a shared queue cannot run until the consumer gives
 * up (timeout, ETIMEOUT; the grid always drains).  Stream priority does not
 * guarantee separate queues (measured), so the consumer always runs on the
 * library's consumer stream for the device — an all-CU-masked stream, which
 * the runtime gives a hardware queue of its own (byteps_reduce_blockq_stream).
 * Launching on that stream costs nothing extra and orders launches and status
 * calls there (work on other streams that reads the outputs must then wait for
 * it, e.g. on an event recorded there); launching on any other stream forks
 * onto it and joins back
 * (two events — ~0.14 ms per iteration at config 3, so launch on the consumer
 * stream when iterations run back to back).  The join-back is queued on the
 * launch stream once EVERY block of the launch's epoch has been released (by
 * the release call that completes the epoch, stream or host), or at
 * byteps_reduce_blockq_join / status, whichever comes first (round 6): a wait
 * for the consumer queued at launch time would sit in the launch stream's
 * in-order hardware queue, which HIP shares with other streams, ahead of any
 * release (or the copies before it) queued later on one of them — the
 * consumer would wait for a release that waits for the consumer, until the
 * timeout (false dependencies).  So work queued on the launch
 * stream after the launch is ordered after the fold only once the epoch is
 * fully released; call join before that if it must be.  The launch stream
 * must outlive that point.  A launch inside a hipGraph
 * capture stays on the capturing stream (pre-released by rule).  Releases on
 * the launch stream itself, before the launch, are always safe.
 * The consumer queues are blocking streams (HIP gives an explicit CU mask only
 * to those), so work on the legacy NULL stream waits for a running consumer —
 * and holds back every stream sharing the NULL stream's hardware queue: do not
 * queue work on the NULL stream between a live launch and its last release
 * (torch: make the current stream a non-default one).
 * Likewise on the host: between a live launch and its last release, the
 * thread that issues the releases must not block on the device
 * (hipDeviceSynchronize, hipFree — including byteps_reduce_blockq_destroy or
 * plan_destroy of another object — or a synchronous copy): the consumer is
 * waiting for the releases that thread has not issued yet. */
typedef struct byteps_reduce_blockq byteps_reduce_blockq;
int byteps_reduce_blockq_create(const byteps_bucket_desc* buckets, int nbuckets,
                                const int* block_end, int nblocks, int dtype, int mode,
                                byteps_reduce_blockq** q);
/* Consumer shape: wg_per_cu = 0 (default) dispatch-ordered — one workgroup
 * per tile, each gated on the release words of the blocks up to its own;
 * 1..8 persistent workgroups per CU sweeping the table; < 0 keeps.  Release
 * timeout in seconds (<= 0 keeps). */
int byteps_reduce_blockq_config(byteps_reduce_blockq* q, int wg_per_cu, double timeout_s);
int byteps_reduce_blockq_launch(byteps_reduce_blockq* q, void* stream);
int byteps_reduce_blockq_release(byteps_reduce_blockq* q, int block, void* stream);
int byteps_reduce_blockq_release_range(byteps_reduce_blockq* q, int first, int count,
                                       void* stream);
int byteps_reduce_blockq_status(byteps_reduce_blockq* q, void* stream);
int byteps_reduce_blockq_destroy(byteps_reduce_blockq* q);
/* Host releases (data already visible to the device, e.g. landed by RDMA into
 * HBM or written by finished device work): after
 * byteps_reduce_blockq_host_releases(q, 1), every launch carries one helper
 * workgroup that forwards release words written by the HOST into the device
 * words, and byteps_reduce_blockq_release_host(q, f, c) releases blocks
 * [f, f + c) with a store to pinned host memory — no stream, no kernel, no
 * copy per release (a release kernel running beside the consumer costs it
 * ~0.4 us each).  The caller guarantees the blocks' data is
 * complete and visible before the call; epochs, timeout and status as above;
 * stream releases may still be mixed in.  Dispatch-ordered consumer only
 * (wg_per_cu = 0); not with a captured launch.  on = 0 turns it off for later
 * launches. */
int byteps_reduce_blockq_host_releases(byteps_reduce_blockq* q, int on);
int byteps_reduce_blockq_release_host(byteps_reduce_blockq* q, int first, int count);
/* The device's consumer stream (see above); owned by the library. */
int byteps_reduce_blockq_stream(byteps_reduce_blockq* q, void** stream);
/* The device's release stream (round 6): a hardware queue of its own, owned
 * by the library, on a different compute pipe than every consumer queue.  A
 * queue that shares a pipe with a running consumer is served ~2x slower (its
 * release kernels took 43 us median instead of 5 beside config 3's consumer,
 * DESIGN.md §4.4 "pipes"), and which pipe a caller's stream lands on is the
 * runtime's choice; the library places its own queues by their HSA ids.
 * Queue a block's pushes (e.g. its H2D copies) and its stream release here,
 * or fork here with an event.  Like the consumer queues it is a blocking
 * stream (see above: no NULL-stream work between a launch and its last
 * release). */
int byteps_reduce_blockq_release_stream(byteps_reduce_blockq* q, void** stream);
/* Diagnostics: the HSA queue ids of the device's consumer queues 0-2 (0 for one
 * not made yet) and of its release queue; returns 4 (needs cap >= 4). */
int byteps_reduce_blockq_queue_ids(byteps_reduce_blockq* q, uint64_t* ids, int cap);
/* Overlap (on = 1; dispatch-ordered consumer only, EARGS otherwise):
 * consecutive launches may run at once, so one iteration's first blocks fold
 * while the previous one's last tiles drain.  A launch goes to whichever of
 * the device's two consumer queues the device's previous block-queue launch
 * did not use, and its first workgroup is dispatched only after every
 * workgroup of that previous launch has started (so waiting workgroups never
 * hold the slots an earlier launch still needs).  The launch
 * forks from `stream` unless `stream` is a consumer queue, and does NOT order
 * `stream` after the fold: byteps_reduce_blockq_join(q, s) makes s wait, on
 * the device, for every block-queue launch of the device so far (status
 * joins first).  Read outputs, or rewrite inputs, only after a join.  on = 0
 * restores the default for later launches. */
int byteps_reduce_blockq_overlap(byteps_reduce_blockq* q, int on);
int byteps_reduce_blockq_join(byteps_reduce_blockq* q, void* stream);
/* Debug (synchronises the device): out = launch epoch, nblocks, the sticky
 * error word, the host's release epoch per block, the device release words,
 * the device block_first table (nblocks + 1), and 1 if the device tile table
 * still equals what was uploaded.  Returns the count written (needs
 * cap >= 4 + 3 * nblocks). */
int byteps_reduce_blockq_debug(byteps_reduce_blockq* q, uint32_t* out, int cap);

/* CpuReducer::copy(dst, src, len), cpu_reducer.cc:209-220 (device to device). */
int byteps_reduce_copy(void* dst, const void* src, size_t len, void* stream);

/* Block the calling thread until all work queued on `stream` has finished. */
int byteps_reduce_sync(void* stream);

/* Size in bytes of one element of `dtype` (getDataTypeLength, common.cc:126-143),
 * or BYTEPS_REDUCE_EDTYPE. */
int byteps_reduce_dtype_size(int dtype);

/* Thread-local description of the last error on this thread ("" if none). */
const char* byteps_reduce_last_error(void);

/* Launch tuning (process-wide; defaults chosen from measurements, see
 * DESIGN.md §4.1).  vpt: 16-B vectors per thread per tile (1, 2 or 4);
 * nt: non-temporal loads and stores (0/1); max_grid: grid cap in 256-thread
 * workgroups (tile-stride beyond); occ: workgroups resident per CU, enforced
 * through the dynamic LDS request (0 = hardware limit, 1..8).  A value <= 0
 * (nt, occ: < 0) keeps the current setting.  Also settable through the
 * environment: BPSR_VPT, BPSR_NT, BPSR_MAX_GRID, BPSR_OCC. */
int byteps_reduce_set_tuning(int vpt, int nt, int max_grid, int occ);
int byteps_reduce_get_tuning(int* vpt, int* nt, int* max_grid, int* occ);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif
#endif /* BPSR_REDUCE_H */
