/*
 * bpsr/server.h — GPU-resident parameter-server aggregation (C ABI of
 * libbpsr.so), the device counterpart of byteps/server/server.cc.
 *
 * Reference behaviour reproduced (server.cc:147-308, 70-145; server.h:138-162):
 *   - round 0 (store not initialised): collect one init push per worker; the
 *     store is initialised by a copy of the LAST arriving init push
 *     (server.cc:175-199);
 *   - every later round, sync mode: the first arrival is the accumulator, the
 *     others are summed into it in ARRIVAL order, and when all NumWorkers pushes
 *     have arrived the merged result becomes the store (server.cc:200-273); a
 *     pull is answered once the round's push is finished and after NumWorkers
 *     pulls the key re-arms (server.cc:280-306, 100-114);
 *   - async mode: every push is summed straight into the store
 *     (server.cc:220-230) and pulls are answered immediately;
 *   - keys are pinned to engine lanes by least accumulated bytes, sticky per key
 *     (GetThreadID, server.h:138-162) — a lane here is a pair of HIP streams,
 *     not a CPU thread.
 *
 * Device-native differences:
 *   - receive slots, the store and (incremental policy) the accumulator live in
 *     HBM, one skewed arena per key; data reaches a slot by H2D/D2D copy
 *     (byteps_server_push) or is written there directly by a transport
 *     (byteps_server_recv_slot + byteps_server_push_ready, the analogue of
 *     ps-lite's zero-copy SArray);
 *   - policy FUSED folds all N slots into the store with ONE kernel at the last
 *     arrival ((N+1)*B HBM bytes); policy INCREMENTAL mirrors SUM_RECV /
 *     COPY_MERGED (an in-place add per arrival, then a copy).  Both give the
 *     same bits: a strict left fold in arrival order.
 */
#ifndef BPSR_SERVER_H
#define BPSR_SERVER_H

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

enum byteps_server_policy { BYTEPS_SERVER_FUSED = 0, BYTEPS_SERVER_INCREMENTAL = 1 };
enum byteps_server_release { BYTEPS_SERVER_RELEASE_LAUNCH = 0, BYTEPS_SERVER_RELEASE_DEVICE = 1 };
enum byteps_server_location { BYTEPS_SERVER_HOST = 0, BYTEPS_SERVER_DEVICE = 1 };

typedef struct byteps_server_config {
  int num_workers;     /* ps::NumWorkers() / DMLC_NUM_WORKER                 */
  int engine_lanes;    /* BYTEPS_SERVER_ENGINE_THREAD (default 4)            */
  int policy;          /* byteps_server_policy                               */
  int async_mode;      /* 1 = asynchronous training (sum into the store)     */
  int device;          /* HIP device ordinal                                 */
  int enable_schedule; /* BYTEPS_SERVER_ENABLE_SCHEDULE (server.cc:335): each
                          lane gets an engine thread that issues queued folds
                          by (fewest counted pushes on the key, oldest) —
                          queue.h:68-97 — one at a time; 0 = FIFO, issued at
                          arrival (the reference default)                    */
  int engine_blocking; /* BYTEPS_SERVER_ENGINE_BLOCKING (server.cc:324): every
                          push returns only once the work it issued (copy,
                          sum, fold) has completed, and every pull is answered
                          at once from the store as it stands — no round gating,
                          no pull counting (server.cc:284-285); a pull issued
                          before the round's last push sees the previous
                          round, as in the reference.  0 = the default engine */
  int release;         /* byteps_server_release: how a finished round is folded
                          — LAUNCH (0): the lane issuers' batched fold
                          launches; DEVICE (1): device releases (below), for
                          pushes that land in HBM.  BPSR_SERVER_RELEASE=
                          launch|device overrides either way              */
} byteps_server_config;

typedef struct byteps_server byteps_server;

/* Defaults from the environment, as init_global_env (server.cc:310-337) reads
 * them: DMLC_NUM_WORKER, BYTEPS_SERVER_ENGINE_THREAD, BYTEPS_ENABLE_ASYNC
 * (here "1" means asynchronous; the reference reads the flag inverted,
 * server.cc:315), BPSR_SERVER_POLICY (fused|incremental),
 * BYTEPS_SERVER_ENABLE_SCHEDULE, BYTEPS_SERVER_ENGINE_BLOCKING, device 0, and
 * release = DEVICE (round 6; LAUNCH before): the server process
 * byteps_server() (server.cc:339-400) starts does nothing else on its GPU,
 * and device releases now cost a server whose pushes are copied nothing —
 * ps-lite delivers into host memory (server.cc:174-218), such rounds fold
 * with launches and no consumer runs (below) — while pushes that land in HBM
 * (byteps_server_push_ready after an RDMA write into GPU memory) fold at 0.54
 * of the HBM roofline instead of 0.26-0.29 (config 3's keys from one receive
 * thread, the bench line's server_cfg3).  BPSR_SERVER_RELEASE=launch keeps
 * launches. */
int byteps_server_config_from_env(byteps_server_config* cfg);

/* Device releases (release = DEVICE or BPSR_SERVER_RELEASE=device; sync mode,
 * fused policy, the default engine, num_workers <= 16 — otherwise the server
 * folds with launches).  The first round that finishes through the slots
 * (byteps_server_push_ready, or blocking pushes of device data, which the
 * copy service lands before they arrive) builds ONE keyed block queue over
 * every declared key of that key's dtype (each key's receive slots in worker
 * order and its store); rounds of copied pushes (host data, non-blocking
 * pushes) before it fold with lane launches and build nothing.  From then on
 * rounds are grouped into epochs — a key's k-th round after the build is in
 * its k-th epoch, or later (below) — and each epoch's kind is decided once:
 *   - a consumer epoch (opened by a slot-written round, or launched ahead):
 *     ONE consumer launch folds every key of the queue, each key's tiles as
 *     soon as that key's round is released — a round's last arrival issues no
 *     launch, it stores the key's arrival order and release word from the
 *     host — in its arrival order (the same bits as the launch path).  A
 *     copied round in such an epoch folds with a lane launch behind its
 *     copies and its key passes the consumer with a skip word: the consumer
 *     never waits for lane-stream work.
 *   - a lane epoch (opened by a copied round while no consumer was launched
 *     for it): no consumer runs; every round in it folds with a lane launch.
 * Once a consumer epoch has a slot-written round, the next epoch's consumer
 * is launched behind it on the keyed queue, so it is resident and polling
 * when that epoch's first release arrives; one launched ahead that no round
 * begins within 1 ms is retired (its keys get skip words, byteps_server_stats
 * out[11]).  Each key's last tile stores the epoch into the key's completion
 * word once the key's bytes are visible device-wide, so device views and
 * blocking device pulls (the copy service) of a released round are answered
 * as soon as THAT key is folded, while the consumer still folds others; other
 * pulls wait for the epoch's consumer to complete.  No key has to be pushed
 * in every epoch: a consumer epoch still open 100 ms after its first release
 * (or half of BPSR_SERVER_RELEASE_TIMEOUT_S, if less) is closed — its keys
 * not released yet get skip words and their rounds go to a later epoch
 * (out[12]) — so a key that skips an iteration or arrives late holds nobody
 * and fails nothing, as in the reference, where every key folds on its own.
 * BPSR_SERVER_RELEASE_TIMEOUT_S (default 5 s) is now the device-side safety
 * net only: a consumer whose release never comes although the host closed the
 * epoch gives up, the keys released in it fail with BYTEPS_REDUCE_ETIMEOUT and
 * the server goes back to launches for good.  Keys declared after the queue
 * was built, and keys of another dtype, always use launches.  While an epoch
 * is open its consumer waits on the device for the releases, on a hardware
 * queue of its own: a thread that still has to push should not wait for the
 * whole device (hipDeviceSynchronize, hipFree) nor put work on the legacy
 * NULL stream (it waits for every blocking stream, the consumer's included)
 * — such a wait lasts until the epoch completes or is closed (at most
 * 100 ms), or, between rounds, until the idle consumer launched ahead retires
 * (1 ms).  Work on non-blocking streams, and stream or event syncs, are fine. */
int byteps_server_create(const byteps_server_config* cfg, byteps_server** out);
/* The same, for a caller that states the size of its config: every version of
 * byteps_server_config is a prefix of the next (fields are only appended), so
 * cfg_size picks the version — 28 bytes (ABI 3: up to engine_blocking; release
 * is LAUNCH) or sizeof(byteps_server_config) (ABI 4 on); any other size is
 * BYTEPS_REDUCE_EARGS instead of fields read past the caller's struct.
 * byteps_server_create reads the whole current struct; a binding built
 * against an older header should call this with its own sizeof. */
int byteps_server_create_sized(const byteps_server_config* cfg, size_t cfg_size,
                               byteps_server** out);
int byteps_server_destroy(byteps_server* s);

/* Optional: allocate a key's slots and store before its first push. */
int byteps_server_init_key(byteps_server* s, uint64_t key, size_t len, int dtype);

/* A worker's push of `len` bytes for `key` (round 0 = init push).  The data is
 * copied into the worker's receive slot before the call returns (the caller may
 * reuse `data`); the fold is queued on the key's engine lane.  Default engine
 * (no scheduling, no engine blocking): the round a push completes is handed
 * to the lane's issuer thread, which issues the rounds that piled up as ONE
 * batched fold launch (BPSR_SERVER_COMBINE=0: the completing call issues its
 * own fold).  A failed fold fails its key: every later call on it returns the
 * error. */
int byteps_server_push(byteps_server* s, uint64_t key, int worker, const void* data,
                       size_t len, int dtype, int location);

/* Non-blocking push: queues the copy into the worker's slot and advances the
 * state machine at once (arrival order = call order; the round's fold runs
 * behind the copies on the device), then acknowledges from the server's
 * responder thread with cb(ctx, key, worker, status) once the bytes are in HBM
 * and `data` may be reused — the point at which the reference answers a push
 * (server.cc:255 SendPushResponse).  Init pushes (round 0) are answered only
 * once every worker's init push has arrived, all together, as the reference
 * does (server.cc:184-198; workers use that answer as a barrier,
 * operations.cc:301-302).  Like byteps_server_push, a worker's push issued
 * while its previous push of the key (init push included) is not folded yet
 * waits inside the call until it is.  Default engine, fused policy, sync mode,
 * device data after the init round: the copy itself is the lane issuer's,
 * batched with the other such pushes that piled up (one copy launch), and
 * `data` must stay valid until cb. */
typedef void (*byteps_server_push_cb)(void* ctx, uint64_t key, int worker, int status);
int byteps_server_push_async(byteps_server* s, uint64_t key, int worker, const void* data,
                             size_t len, int dtype, int location, byteps_server_push_cb cb,
                             void* ctx);

/* Zero-copy transport path: where worker `worker`'s push for `key` must land,
 * then the arrival notice once the bytes are there (visible to the device).
 * recv_slot waits until the key's last issued fold (or init copy) is done — a
 * device-released round: until the key's own completion word says so, not
 * for its whole epoch — so the slot is free to be written once it returns —
 * provided the worker's
 * previous push of the key has been folded, i.e. the transport writes a
 * worker's round r + 1 only after that worker pulled round r (BytePS's
 * push-then-pull order per key; the init round is complete once the init
 * pushes have been answered). */
int byteps_server_recv_slot(byteps_server* s, uint64_t key, int worker, void** slot);
int byteps_server_push_ready(byteps_server* s, uint64_t key, int worker);

/* A worker's pull: blocks until the key's current round is finished (sync mode),
 * then copies the store (len bytes) to `out`.  Into THIS device's memory with
 * the default engine in sync mode (up to 16 MiB), the pull copy service does
 * the copy: the caller waits for the round's fold as a device view does (its
 * completer's published sequence), writes one tagged job per 64 KiB into a
 * pinned ring and spins on the jobs' done words, which a persistent service
 * kernel (fetcher + 64 copier workgroups, on a non-blocking high-priority
 * stream of its own) stores once the bytes are visible device-wide — no HIP
 * call and no thread hand-off per pull (≈5–6 µs per small pull from 1 or 8
 * threads).  The kernel exits after 0.5 ms without a job, and
 * at 1 ms of age even while busy (a waiting or posting thread relaunches it
 * at once), so a device-wide synchronisation elsewhere in the process
 * (torch.cuda.synchronize, hipDeviceSynchronize, hipFree) waits for it at
 * most ~1 ms plus one relaunch's age: measured p50 / p99 0.5 / 0.5 ms under 8
 * threads copying nonstop (profiles/r05s04_copysvc_age_sweep.jsonl; a -m gpu
 * test asserts median < 4 ms, max < 10 ms).  A job not served within 10 s is
 * given up: the service raises its stop word, waits for its launch to end
 * (no copy of it lands afterwards), turns itself off for good, and the call
 * copies on the key's lane instead.  Events given to byteps_server_order_after
 * are waited for (on the host) before such a copy.  BPSR_SERVER_PULL_SERVICE=0
 * or other destinations: the copy is one of the lane issuer's batched pull
 * copies: the issuer tells the caller which of its launches carries the copy,
 * and the caller waits for the lane's completer to see that launch complete
 * (no HIP call on the caller's thread, no responder hop), then counts the
 * pull.  Pulls parked before the round finishes are queued together when it
 * does, so the pulls one round completion answers ride in one launch.  A call
 * made from inside a callback (on the responder thread) copies directly.  The
 * same holds for blocking pushes of device data (byteps_server_push).
 * Copies into pinned host memory are made by the copy kernel through the
 * memory's device view (beside the pushes' SDMA H2D copies the link then runs
 * full duplex: 87 GB/s together instead of 55, tools/pcie_probe.py); pageable
 * memory and device destinations use hipMemcpyAsync.  Blocking pushes FROM
 * this device's memory (up to 16 MiB) take the copy service the same way:
 * once the key's previous fold has completed, the service copies the data
 * into the worker's slot with no key lock held, then the push arrives as a
 * push_ready would (config 3's keys pushed and pulled one by one by 8
 * threads: 20–21 → 3.0 ms per round).  Host sources keep the lanes' copies. */
int byteps_server_pull(byteps_server* s, uint64_t key, void* out, size_t len, int location);

/* Zero-copy pull response for a host transport (server.cc:42-70 answers a pull
 * with an SArray over the store itself).  Blocks like byteps_server_pull, then
 * sets *data to a pinned host mirror of the store holding this round's result
 * (*len = key length).  The server fills the mirror with ONE device-to-host
 * copy per round, queued behind the round's fold on its own stream, instead of
 * one copy per puller; from the first view of a key on, every later round is
 * mirrored as soon as it finishes.  Two mirrors alternate by round, each at a
 * fixed address (register them with the NIC once).  Sync mode: the view stays
 * valid until this worker's next pull of the key returns.  Async mode: each
 * call copies the current store into the next of num_workers + 1 mirrors (a
 * ring), so a view stays intact for the next num_workers pulls of the key.
 * The caller must not write through the view. */
int byteps_server_pull_host_view(byteps_server* s, uint64_t key, const void** data, size_t* len);

/* Zero-copy pull for a transport that sends straight from HBM (GPUDirect RDMA
 * into the NIC, or a device-side consumer): blocks like byteps_server_pull
 * until the key's round is finished and its fold has completed, then sets
 * *data to the key's store in DEVICE memory (*len = key length) and counts
 * the pull.  No copy at all — the device counterpart of SendPullResponse
 * answering with an SArray over the store (server.cc:42-70).  Sync mode only
 * (EARGS in async mode: every push rewrites the store).  The view stays valid
 * until this worker's next push of the key (the next round cannot finish
 * without it); the caller must not write through it. */
int byteps_server_pull_device_view(byteps_server* s, uint64_t key, const void** data,
                                   size_t* len);

/* Non-blocking pull for a transport's receive thread: the reference's default
 * non-blocking engine queues a pull that arrives before the round has finished
 * (q_pull_reqmeta_, server.cc:286-305) and the engine thread answers it once
 * COPY_MERGED is done (server.cc:100-114).  Here the call returns at once; a
 * server-owned responder thread later calls
 *   cb(ctx, key, data, len, status)
 * with data/len = the zero-copy view byteps_server_pull_host_view would give
 * (same validity), status 0.  The pull is counted toward the key's re-arm just
 * BEFORE cb runs (the reference counts it with SendPullResponse under one
 * lock, server.cc:100-113, 293-298), so cb sends (or copies) the response
 * before returning, as SendPullResponse does.  Pulls still waiting at byteps_server_destroy get
 * status BYTEPS_REDUCE_ECANCELED and data NULL.  cb must not call back into
 * the server for the same key. */
typedef void (*byteps_server_pull_cb)(void* ctx, uint64_t key, const void* data, size_t len,
                                      int status);
int byteps_server_pull_async(byteps_server* s, uint64_t key, byteps_server_pull_cb cb, void* ctx);

/* Non-blocking pull INTO a caller's device buffer (a worker GPU of the node,
 * a registered device buffer of the transport): the reference's ZPull with a
 * callback (the pull response lands in the worker's buffer).  Returns at once;
 * once the key's round is finished the lane's issuer copies the store into
 * `out` (len bytes), batched with the other pulls that piled up (one copy
 * launch), and the responder thread calls cb(ctx, key, out, len, 0) when the
 * copy has completed, counting the pull just before (as byteps_server_pull_async).
 * Later folds of the key wait for the copy before rewriting the store.  Sync
 * mode and the default engine only (EARGS otherwise); device memory, or pinned
 * host memory (written through its device view; EARGS for pageable memory).
 * Pulls still waiting at byteps_server_destroy get BYTEPS_REDUCE_ECANCELED. */
int byteps_server_pull_into_async(byteps_server* s, uint64_t key, void* out, size_t len,
                                  int location, byteps_server_pull_cb cb, void* ctx);

/* Introspection for tests/debug (BYTEPS_SERVER_DEBUG analogue): completed
 * rounds, engine lane, and the arrival order of the last completed round
 * (waits until every round the key completed has been issued). */
int byteps_server_key_info(byteps_server* s, uint64_t key, uint64_t* rounds, int* lane,
                           int* last_order, int max_order);

/* Order the server's device work after the caller's: every copy into a slot,
 * copy out of a store and fold that the lanes of keys[0..n) (n = 0: every
 * lane) issue from now on runs after `event` (a hipEvent_t the caller recorded
 * on the stream that produced a push's data or last touched a pull's
 * destination) — hipStreamWaitEvent on the lanes' streams, no host wait.  Work
 * no lane stream orders waits for the event on the host first: the copy
 * service's copies, and a device release stored from the host (a push_ready
 * round with device releases on).  The event may be re-recorded or destroyed
 * once the call returns.  Call it before the push / pull calls it orders. */
int byteps_server_order_after(byteps_server* s, const uint64_t* keys, int n, void* event);

/* Telemetry since create: out[0] fold launches (single and batched), out[1]
 * rounds folded, out[2] pull copy launches, out[3] pulls answered (copies and
 * views), out[4] ns the lane issuer threads spent issuing, out[5] batched
 * push-copy launches, out[6] keyed consumer epochs a round was released into
 * and out[7] rounds released on the device (BPSR_SERVER_RELEASE=device),
 * out[8] blocking pulls served by the pull copy service, out[9] that
 * service's kernel launches, out[10] blocking pushes it served, out[11]
 * keyed consumers launched ahead of their epoch and retired because no round
 * began it within 1 ms, out[12] consumer epochs closed with keys not pushed
 * (their rounds went to a later epoch) and out[13] lane epochs (opened by a
 * copied round: no consumer); the first n (<= 14). */
int byteps_server_stats(byteps_server* s, uint64_t* out, int n);

/* Batched calls for a transport that delivers many keys at once (co-located
 * workers, an in-process transport; ps-lite sends one key per request,
 * server.cc:153).  Each is equivalent to n single calls in array order, the
 * same worker for every key, except that the work is issued per engine lane
 * in one launch: the device copies of push_many (device sources), the folds
 * of every round the call completes (fused policy), and the device copies of
 * pull_many.  A call never blocks while holding rounds it completed: it issues
 * them first.  Host sources / destinations are copied per key.
 *   push_ready_many  byteps_server_push_ready for keys[0..n)
 *   push_many        byteps_server_push (blocking) for keys[i] with datas[i], lens[i]
 *   pull_many        byteps_server_pull into outs[i] (lens[i] bytes)           */
int byteps_server_push_ready_many(byteps_server* s, const uint64_t* keys, int n, int worker);
int byteps_server_push_many(byteps_server* s, const uint64_t* keys, const void* const* datas,
                            const size_t* lens, int n, int worker, int dtype, int location);
int byteps_server_pull_many(byteps_server* s, const uint64_t* keys, void* const* outs,
                            const size_t* lens, int n, int location);

/* Debug/test hook for scheduling (enable_schedule only): pause > 0 holds the
 * lane's engine queue (nothing is issued; pushes still queue), 0 releases it,
 * < 0 leaves it; the keys of the jobs the lane issued so far, in issue order,
 * go to log_keys (up to max_log) and their count to *n_log. */
int byteps_server_debug_lane(byteps_server* s, int lane, int pause, uint64_t* log_keys,
                             int max_log, int* n_log);

/* ------------------------------------------------------------------------
 * Key space sharded over several server instances (one per GPU of a node):
 * the counterpart of the reference's key -> server assignment
 * (BytePSGlobal::EncodeDefaultKey, global.cc:530-567) inside ONE process
 * that owns the node's GPUs.  Each instance is a byteps_server (its own
 * lanes, slots and store on its own device); the group routes every call.
 *
 * Split policies:
 *   BYTEPS_SERVER_SPLIT_HASH   whole keys, instance = hash(key) % instances
 *       with the reference's BYTEPS_KEY_HASH_FN (djb2 default; naive, sdbm,
 *       built_in x BYTEPS_BUILT_IN_HASH_COEF) — the reference's own rule, the
 *       same arithmetic (each key's round is one left fold in arrival order);
 *   BYTEPS_SERVER_SPLIT_RANGE  every key of at least split_min_bytes is cut
 *       into one contiguous piece per instance — the owner ranges of the
 *       reduce-scatter split (core_loops.cc:210-211) in 128-byte units, the
 *       tail to the last instance — so each GPU owns a contiguous slice of
 *       every large partition; smaller keys go whole by hash.  Piece starts
 *       are multiples of 128 B (of 8 elements for every dtype), so the fp16
 *       body/tail rule of cpu_reducer.cc:103,118 holds piece by piece.  A
 *       split key keeps ONE arrival order, as in the reference where one
 *       server holds it (server.cc:216-250): the group stamps every push with
 *       the next position of its worker's round and every instance folds its
 *       piece in those positions (fused policy; the init round's store comes
 *       from the push stamped last).  With the incremental policy or engine
 *       blocking, each piece follows its own instance's arrival order.
 * The group records each key's length and dtype (init_key, or its first push):
 * a push of another length is refused, and a pull of fewer bytes is cut from
 * the same pieces.  Pushes scatter the pieces (each instance copies its piece
 * into its own HBM), every piece validated before any is queued; one that
 * still fails fails the key on every instance.  Pulls gather the pieces back,
 * all instances at once (pull_into_async) into device or pinned host memory
 * with the default engine, else piece by piece.  Batched calls queue every
 * piece of every key at once.  The group enables peer access between its
 * devices.  All calls are thread-safe like the single-instance ones and block
 * like them. */
enum byteps_server_split { BYTEPS_SERVER_SPLIT_HASH = 0, BYTEPS_SERVER_SPLIT_RANGE = 1 };
/* BYTEPS_KEY_HASH_FN values (global.cc:541-554). */
enum byteps_key_hash { BYTEPS_KEY_HASH_DJB2 = 0, BYTEPS_KEY_HASH_NAIVE = 1,
                       BYTEPS_KEY_HASH_SDBM = 2, BYTEPS_KEY_HASH_BUILT_IN = 3 };

typedef struct byteps_server_group_config {
  byteps_server_config server; /* every instance's config (.device is ignored)  */
  int num_servers;             /* instances (>= 1)                              */
  int devices[16];             /* device of instance i (may repeat)             */
  int split;                   /* byteps_server_split                           */
  int hash_fn;                 /* byteps_key_hash                               */
  uint32_t hash_coef;          /* built_in multiplier (BYTEPS_BUILT_IN_HASH_COEF) */
  size_t split_min_bytes;      /* RANGE: smaller keys go whole (0 = 128 * n)    */
} byteps_server_group_config;

#define BYTEPS_SERVER_GROUP_MAX 16

/* The reference's key hash (global.cc:491-523) of `key` under `fn`. */
uint64_t byteps_server_key_hash(uint64_t key, int fn, uint32_t coef);

/* Defaults from the environment: the server config (byteps_server_config_from_env),
 * num_servers and devices 0..n-1 from BPSR_SERVER_GPUS (default 1), split from
 * BPSR_SERVER_SPLIT (hash|range), BYTEPS_KEY_HASH_FN, BYTEPS_BUILT_IN_HASH_COEF,
 * BPSR_SERVER_SPLIT_MIN_BYTES.  An unknown hash name is EARGS (the reference
 * aborts, global.cc:555-557). */
int byteps_server_group_config_from_env(byteps_server_group_config* cfg);

typedef struct byteps_server_group byteps_server_group;
int byteps_server_group_create(const byteps_server_group_config* cfg, byteps_server_group** out);
int byteps_server_group_destroy(byteps_server_group* g);
/* Pieces of a key of `len` bytes: for i < *npieces (<= cap), piece i of bytes
 * [offset[i], offset[i] + plen[i]) lives on instance server[i].  The rule is a
 * pure function of the config (byteps_server_route: what a worker-side
 * transport needs to address the instances, like EncodeDefaultKey). */
int byteps_server_route(const byteps_server_group_config* cfg, uint64_t key, size_t len,
                        int* npieces, int* server, size_t* offset, size_t* plen, int cap);
int byteps_server_group_route(byteps_server_group* g, uint64_t key, size_t len, int* npieces,
                              int* server, size_t* offset, size_t* plen, int cap);
/* Instance i (for its zero-copy / view calls on routed pieces). */
int byteps_server_group_instance(byteps_server_group* g, int i, byteps_server** s);
int byteps_server_group_init_key(byteps_server_group* g, uint64_t key, size_t len, int dtype);
/* byteps_server_push / _pull over the pieces (the pieces' copies run
 * concurrently; the call returns when all are done). */
int byteps_server_group_push(byteps_server_group* g, uint64_t key, int worker, const void* data,
                             size_t len, int dtype, int location);
int byteps_server_group_pull(byteps_server_group* g, uint64_t key, void* out, size_t len,
                             int location);
/* byteps_server_pull_host_view on the instance holding a whole (unsplit) key:
 * the zero-copy pull response of server.cc:42-70 (EARGS for a key split over
 * several instances: view each piece through byteps_server_group_instance). */
int byteps_server_group_pull_host_view(byteps_server_group* g, uint64_t key, const void** data,
                                       size_t* len);
/* byteps_server_push_many / _pull_many: keys routed, one batched call per instance. */
int byteps_server_group_push_many(byteps_server_group* g, const uint64_t* keys,
                                  const void* const* datas, const size_t* lens, int n, int worker,
                                  int dtype, int location);
int byteps_server_group_pull_many(byteps_server_group* g, const uint64_t* keys,
                                  void* const* outs, const size_t* lens, int n, int location);

/* byteps_server_order_after for the instances that hold keys[0..n) (their
 * declared lengths decide the pieces; n = 0 or an undeclared key: every
 * instance). */
int byteps_server_group_order_after(byteps_server_group* g, const uint64_t* keys, int n,
                                    void* event);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif
#endif /* BPSR_SERVER_H */
