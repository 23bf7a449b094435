/*
 * bpsr/prophet.h — Prophet's PUSH-stage scheduler (C ABI of libbpsr.so), the
 * native counterpart of BytePSScheduledQueue for the PUSH queue
 * (byteps/common/scheduled_queue.cc:94-108 addTask, :199-215 findTask,
 * :217-296 getTask, :362-371 reportFinish; constants scheduled_queue.h:77-95).
 *
 * It decides WHICH partitions reach the server together — the release groups
 * a batched fold launch or a block-queue release (bpsr/reduce.h) receives:
 *   - tasks whose tensor name matches Z_keyword ("scheduled") are collected
 *     in backward order from the last checkpoint down; when the expected
 *     gradient has a queued partition, all of its partition slots are stacked;
 *     reaching the previous checkpoint opens a byte budget
 *     backward_exec[k] * (int)(batch/64) * Z_NET_B * 125 (constructor, :26-33);
 *   - release pops the stack top (lowest gradient index first) while the budget
 *     strictly exceeds the task's length (:262); a task that does not fit ends
 *     the block and collection resumes; an empty stack ends it too;
 *   - once gradient 0 is stacked, the rest is released under the byte credit
 *     Z_CREDIT, refilled by report_finish (:362-371); the empty stack resets
 *     the iteration (:276-290);
 *   - other tasks ("unscheduled") form the FIFO (_sq), served only while no
 *     scheduled task is queued (:292-318).
 * Equal gradient indices keep insertion order (the multiset compares priority
 * only, scheduled_queue.h:58-62; findTask takes lower_bound).
 *
 * Deviations from the reference: an empty stack at release
 * simply ends the block (the reference reads _mystack.top() of an empty stack,
 * :250); a credit exactly equal to the task's length releases it once and
 * charges it (the reference returns it without erasing it, :281-285, so it
 * would be sent again); checkpoints, exec times and the gradient count are
 * parameters (the reference hard-codes a 157-gradient model and 160-entry
 * arrays); exec times are doubles (the pre-run profiler's measured values,
 * global.h's _backward_exec).  The FIFO ignores ready events and ready tables
 * (they belong to the stages around PUSH).
 *
 * Host-only: no call touches a GPU.  Every call on one queue is serialised by
 * the queue's mutex (the reference's _mutex), so transport and engine threads
 * may share it.  Errors: 0 / positive on success, a negative BYTEPS_REDUCE_E*
 * code otherwise, message in byteps_reduce_last_error().
 */
#ifndef BPSR_PROPHET_H
#define BPSR_PROPHET_H

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

typedef struct byteps_prophet_config {
  int64_t batch_size;           /* Z_BATCH_SIZE                                     */
  int64_t net_b;                /* Z_NET_B (multiplied by 125, :27)                 */
  int64_t credit;               /* Z_CREDIT, bytes                                  */
  const int32_t* checkpoints;   /* ascending, checkpoints[0] == -1; NULL = the
                                   reference's 13 (scheduled_queue.h:81-82)         */
  int32_t ncheckpoints;         /* >= 2 when checkpoints is given                   */
  const double* backward_exec;  /* ncheckpoints entries; NULL = the reference's
                                   (scheduled_queue.h:84-85)                        */
} byteps_prophet_config;

typedef struct byteps_prophet_task {
  int32_t grad;           /* declared gradient index (= -priority), 0..last checkpoint */
  int32_t part;           /* partition index inside the gradient                 */
  int64_t len;            /* bytes                                               */
  int32_t total_partnum;  /* partitions of the gradient (_tensor_part)           */
  int32_t scheduled;      /* 1: name matches Z_keyword (Prophet order); 0: FIFO  */
  uint64_t key;           /* (declared_key << 16) + part                         */
  uint64_t handle;        /* caller's cookie, returned unchanged                 */
} byteps_prophet_task;

/* Phase of a released task: the budget block it was released under (>= 0),
 * BYTEPS_PROPHET_CREDIT after gradient 0, BYTEPS_PROPHET_FIFO for the FIFO. */
enum { BYTEPS_PROPHET_CREDIT = -1, BYTEPS_PROPHET_FIFO = -2 };

typedef struct byteps_prophet_queue byteps_prophet_queue;

int byteps_prophet_create(const byteps_prophet_config* cfg, byteps_prophet_queue** out);
int byteps_prophet_destroy(byteps_prophet_queue* q);

/* addTask (scheduled_queue.cc:94-108).  EARGS for a scheduled task whose
 * gradient lies outside [0, last checkpoint] or with total_partnum < 1. */
int byteps_prophet_add_task(byteps_prophet_queue* q, const byteps_prophet_task* t);

/* One getTask() call (scheduled_queue.cc:217-296): returns 1 and fills *out
 * (and *phase if non-NULL) when a task is released, 0 when none is. */
int byteps_prophet_get_task(byteps_prophet_queue* q, byteps_prophet_task* out, int32_t* phase);

/* reportFinish(size) (scheduled_queue.cc:362-371). */
int byteps_prophet_report_finish(byteps_prophet_queue* q, int64_t size);

/* Queued tasks (scheduled + FIFO). */
int byteps_prophet_pending(byteps_prophet_queue* q, uint64_t* n);

/* The iteration state, for tests and tracing. */
typedef struct byteps_prophet_state {
  int32_t pointer;      /* _pointer: checkpoint index of the block being collected */
  int32_t expected;     /* expected_priority * -1: next gradient to collect      */
  int32_t sizepointer;  /* _sizepointer: budgets opened so far                   */
  int32_t dequeue;      /* _dequeue: releasing (1) or collecting (0)             */
  int32_t meetzero;     /* _meetzero: gradient 0 stacked                         */
  int32_t stack_depth;  /* _mystack.size()                                       */
  int64_t credit;       /* _bps_credit                                           */
  double budget_left;   /* dynamic_size                                          */
} byteps_prophet_state;
int byteps_prophet_get_state(byteps_prophet_queue* q, byteps_prophet_state* out);

/* Back to the start of an iteration (collection from the last checkpoint,
 * full credit); queued tasks stay. */
int byteps_prophet_reset(byteps_prophet_queue* q);

/* Drive the queue through one iteration (the queue must hold no task when
 * called; byteps_prophet_reset first for a fresh iteration): arrivals[i] is
 * added before the i-th getTask poll (one arrival per poll, as gradients come
 * off backward); polls continue until every arrival was added and nothing is
 * queued.
 * Releases are written to released[0..n) in order; group g is
 * released[group_start[g] .. group_start[g+1]) — a run of consecutive
 * successful polls, also split where the phase changes if split_on_phase —
 * with group_phase[g] its phase.  finish_immediately reports each released
 * task finished at once (credit refilled).  group_start needs n+1 entries,
 * group_phase n.  Returns the number of groups; EARGS (nothing added) if an
 * arrival is invalid, or if max_idle consecutive empty polls pass (no progress
 * possible, e.g. credit smaller than a task; the queue then keeps what it
 * holds — reset and drain it, or destroy it). */
int byteps_prophet_release_groups(byteps_prophet_queue* q, const byteps_prophet_task* arrivals,
                                  size_t n, int finish_immediately, int split_on_phase,
                                  uint64_t max_idle, byteps_prophet_task* released,
                                  int32_t* group_start, int32_t* group_phase);

/* Prophet's pre-run profile (scheduled_queue.cc:110-167, the Global::pre_run
 * branch of addTask_helper): from the first time each gradient reached the
 * PUSH queue in one profiled iteration (tic_us[i] for gradient i, µs, any
 * epoch), derive the block boundaries and the per-block budgets that the
 * constructor then scales (:26-33):
 *   gaps x_i = |tic[i] - tic[i-1]|, i = 1..ngrad-1; avg = 2 x their mean;
 *   checkpoints = -1, then i-1 for every i whose gap exceeds avg (ascending),
 *   then ngrad-1;
 *   backward_exec (ms) = the qualifying gaps / 1000, LAST i first, then
 *   |tic[i0-1] - tic[0]| / 1000 for the first qualifying i0 — one entry per
 *   block in the order getTask opens them — padded with a final 0 so it has
 *   one entry per checkpoint, as byteps_prophet_config wants.
 * Deviation: with no qualifying gap the reference leaves backward_exec empty
 * and getTask reads past it (:240); here the one block gets the whole span
 * |tic[ngrad-1] - tic[0]| / 1000.  Writes at most `cap` entries to each
 * array; returns the number of checkpoints (EARGS if ngrad < 1, a tic is
 * negative, or cap is too small). */
int byteps_prophet_profile(const int64_t* tic_us, int32_t ngrad, int32_t* checkpoints,
                           double* backward_exec, int32_t cap);

/* Prophet's bandwidth monitor (reportFinish(size, priority),
 * scheduled_queue.cc:373-398, same pre-run pass): the highest rate any one
 * gradient's push achieved, possible_B = size * 1000 / (finish - start) bytes
 * per ms, maximised over the pushes — returned in Z_NET_B's unit (Mb/s, the
 * constructor's x125 turns it back into bytes per ms): *net_b = max over i of
 * size[i] * 8 / (finish_us[i] - start_us[i]).  Pushes with finish <= start are
 * skipped (the reference would divide by zero); EARGS if none is left.  The
 * reference never records the push start it reads (_push_start_tic is
 * declared nowhere), so the caller supplies it. */
int byteps_prophet_estimate_net_b(const int64_t* size, const int64_t* start_us,
                                  const int64_t* finish_us, int32_t n, double* net_b);

/* The PUSH loop (core_loops.cc RunPushLoopOnce -> reportFinish, as a native
 * thread): the scheduler feeding a block queue (bpsr/reduce.h).  The queue's
 * table holds the iteration's partitions; block_of[h] is the block of the
 * partition whose task handle is h (0 <= h < nhandles).  Per iteration:
 *   byteps_prophet_loop_begin(l, consumer_stream)  resets the scheduler and
 *       launches the block queue's consumer (one launch per iteration; NULL:
 *       on the library's consumer stream, byteps_reduce_blockq_stream);
 *   byteps_prophet_loop_push(l, &task)  one per partition as its bytes land
 *       (their copies queued on release_stream, or finished), in any order —
 *       the loop thread polls getTask, reports each release group's partitions
 *       finished at the group's end (credit back, so the next group may go),
 *       and when a poll makes no progress (the scheduler waits for pushes or
 *       credit) releases every block that became complete meanwhile: ONE
 *       release_range per run of consecutive blocks, on release_stream.  So
 *       the release groups that are ready together — every group, when the
 *       pushes have all landed — go out as one kernel, and a block is held
 *       back at most by the host work of draining the groups ready with it;
 *   byteps_prophet_loop_push_many(l, tasks, n)  the same for n partitions
 *       that landed together (one drain for all of them), in array order;
 *   byteps_prophet_loop_end(l, timeout_s)  waits until every block has been
 *       released (timeout_s <= 0: no limit); with the loop thread, a task the
 *       scheduler refuses (e.g. a gradient outside the model) is reported
 *       here, since the thread adds the pushes.  ETIMEOUT leaves the scheduler
 *       holding the missing partitions' state: destroy the loop and the queue
 *       (the block queue's own status() resynchronises its epochs).
 * The loop thread makes HIP calls on the device current at create time.  With
 * flags & BYTEPS_PROPHET_LOOP_INLINE there is no thread: each push drains the
 * scheduler and issues the releases itself, in the caller's thread (no
 * wake-up latency; the pushing threads then make the HIP calls).  Inline, a
 * pushing thread must not block on the device (hipDeviceSynchronize, hipFree,
 * a synchronous copy) between begin and its last push: the consumer waits
 * for releases only that thread would issue, until its timeout.  The
 * scheduler and block queue must outlive the loop and must not be driven
 * directly while it runs.
 * With flags & BYTEPS_PROPHET_LOOP_HOST_RELEASE the complete blocks are
 * released from the host (byteps_reduce_blockq_release_host, no stream work;
 * create enables host releases on the block queue): for pushes whose bytes are
 * already visible to the device when byteps_prophet_loop_push is called
 * (RDMA into HBM, or copies the caller has waited for); release_stream is then
 * unused.  Otherwise, with the loop thread, release_stream must not be NULL
 * (EARGS): NULL would mean the LOOP thread's per-thread stream, which no copy
 * the caller queued on its own stream is ordered before.  Inline, NULL is the
 * pushing thread's per-thread stream. */
enum { BYTEPS_PROPHET_LOOP_INLINE = 1, BYTEPS_PROPHET_LOOP_HOST_RELEASE = 2 };
typedef struct byteps_prophet_loop byteps_prophet_loop;
int byteps_prophet_loop_create(byteps_prophet_queue* pq, byteps_reduce_blockq* bq,
                               const int32_t* block_of, int32_t nhandles, int32_t nblocks,
                               void* release_stream, int flags, byteps_prophet_loop** out);
int byteps_prophet_loop_begin(byteps_prophet_loop* l, void* consumer_stream);
int byteps_prophet_loop_push(byteps_prophet_loop* l, const byteps_prophet_task* t);
int byteps_prophet_loop_push_many(byteps_prophet_loop* l, const byteps_prophet_task* tasks,
                                  int32_t n);
int byteps_prophet_loop_end(byteps_prophet_loop* l, double timeout_s);
/* Release calls (release_range kernels, or host releases) the loop has issued
 * since create: telemetry for how many groups went out together. */
int byteps_prophet_loop_release_calls(byteps_prophet_loop* l, uint64_t* calls);
int byteps_prophet_loop_destroy(byteps_prophet_loop* l);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif

#endif /* BPSR_PROPHET_H */
