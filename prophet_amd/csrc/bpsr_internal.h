// Internal (non-ABI) declarations shared by the kernels and the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <string>
#include <stddef.h>
#include <stdint.h>

#include "bpsr/reduce.h"
#include "bpsr_error.h"

namespace bpsr {

// dtype ids: byteps/common/common.h:52-65 + bf16 extension (include/bpsr/reduce.h)
enum : int {
  kFloat32 = 0, kFloat64 = 1, kFloat16 = 2, kUInt8 = 3,
  kInt32 = 4, kInt8 = 5, kInt64 = 6, kBFloat16 = 11
};
enum : int { kModeReference = 0, kModeAccumF32 = 1 };

constexpr int kBlock = 256;     // 4 waves of 64
constexpr int kMaxSrcs = 32;    // BYTEPS_REDUCE_MAX_SRCS
// Fewer tiles than this leave CUs idle (256 CUs, several workgroups each):
// launches that would get fewer fall back to smaller tiles.
constexpr uint64_t kMinTiles = 2048;

// Byte/element geometry of one fold, identical for every operand (the vector
// path needs all operands co-aligned mod 16).
struct FoldGeom {
  uint64_t n_elems;        // len / sizeof(T)
  uint64_t head_elems;     // elements before the 16-B vector range
  uint64_t vec_off;        // byte offset of the vector range
  uint64_t nvec;           // 16-B vectors in the vector range
  uint64_t tail_begin;     // first element after the vector range
  uint64_t tail_sem_from;  // fp16: first element with F16C-tail semantics
  uint64_t trailing_bytes; // len % sizeof(T)
  uint32_t copy_trailing;  // fold into a separate dst: trailing bytes from srcs[0]
  uint32_t pad;
};

struct FoldArgs {
  const unsigned char* srcs[kMaxSrcs];
  unsigned char* dst;
  int n;
  int aligned;  // every operand element-aligned
  FoldGeom g;
  uint64_t grid;  // launched workgroups (set by the launcher)
};

// Per-bucket geometry of a batched launch (read by element tiles only).
struct BatchEntry {
  const unsigned char* srcs[kMaxSrcs];
  unsigned char* dst;
  int n;
  int aligned;
  FoldGeom g;
};

// One record per workgroup of a batched launch, rec_stride bytes apart: a
// 32-B head followed by the n source pointers.  Vector tiles carry pointers
// already advanced to the tile's first byte, so a workgroup reaches its data
// after ONE scalar round trip (head + pointers) instead of map -> bucket ->
// data.  Element tiles (unaligned head, tail, trailing bytes) are separate
// workgroups at the front of the launch, so that latency-bound work runs
// beside the vector tiles rather than after them.
enum : uint32_t { kTileFull = 0, kTilePartial = 1, kTileElem = 2 };
struct TileHead {
  unsigned char* dst;  // vector tiles: dst + the tile's first byte
  uint32_t kind;
  uint32_t n;          // sources
  uint32_t a;          // partial: valid vectors; element: part index
  uint32_t b;          // element: bucket index into the BatchEntry table
  uint32_t c;          // element: parts of this bucket's element work
  uint32_t block;      // block queue: the release block this tile belongs to
};
constexpr uint32_t kTileHeadBytes = 32;
static_assert(sizeof(TileHead) == kTileHeadBytes, "TileHead layout");
// Record stride: room for max(8, nmax) pointers (the kernel reads 8 at entry).
inline uint32_t tile_rec_stride(int nmax) {
  return (kTileHeadBytes + 8u * (uint32_t)(nmax < 8 ? 8 : nmax) + 31u) & ~31u;
}
constexpr uint32_t kPrefetchAhead = 256;  // tile-record prefetch distance: MI355X's 256 CUs
struct BatchLaunch {
  const unsigned char* recs;    // tiles records
  const BatchEntry* entries;    // per-bucket geometry
  uint32_t rec_stride;
  uint32_t tiles;
  uint32_t pf_ahead;            // L2 prefetch of record blockIdx + pf_ahead (0 = off)
  // Host side only (the kernels ignore it): when set, the launch itself
  // completes this event (hipExtLaunchKernel's stop event) instead of a
  // separate hipEventRecord behind it — a marker packet between two kernels
  // costs 3-5 us of the stream's device time (profiles/r03_event_marker_cost.jsonl).
  hipEvent_t stop;
};

// Block consumer (byteps_reduce_blockq_*).  One launch folds the whole table;
// a workgroup starts a tile only once the tile's block and every block before
// it have been released for this launch's EPOCH.  Epochs (launch k consumes
// epoch k; the k-th release of block b carries epoch k) replace a re-arm step:
// flags[b] holds the latest epoch block b was released for, so block b is
// released for launch k iff flags[b] >= k, and nothing is ever cleared.
struct BlockqCtl {
  uint32_t err;   // sticky: a workgroup gave up waiting for a release
  uint32_t pad[3];
};
struct BlockqLaunch {
  BatchLaunch L;
  uint32_t* flags;              // one word per block: the latest epoch it was released for
  const uint32_t* block_first;  // first tile of each block, [nblocks] = tiles
  BlockqCtl* ctl;
  uint32_t nblocks;
  uint32_t grid;            // launched (persistent) workgroups
  uint64_t timeout_ticks;   // wall_clock64() ticks a workgroup waits for a release
  uint32_t epoch;           // this launch's epoch (>= 1)
  uint32_t helper;          // 1: workgroup 0 forwards host release words (hflags)
  const uint32_t* hflags;   // host-written release words (pinned, device view)
  // Keyed consumer (the PS server's device releases, bpsr_server.cpp): one
  // block per key, a tile waits for its OWN block only, and the block's word
  // (arrival order << 32 | epoch) says in which order its sources fold.
  uint32_t keyed;
  uint32_t wide;             // 9..16 sources: a second word per block, kwords[nblocks + b]
                             // (order positions 8..15), khwords likewise after the first words
  uint64_t* kwords;          // device words, one per block (helper / stream releases write them)
  const uint64_t* khwords;   // host words (device view), two per block by epoch parity
  uint32_t* herr;            // host word (device view): the helper mirrors ctl->err there
  // Per-key completion: each finished tile adds to its block's counter (device,
  // monotonic across epochs); the block's last tile of an epoch stores the
  // epoch into the block's host word, once every tile's bytes are visible
  // device-wide — a key's store can be read before the whole epoch ends.
  uint32_t* kcnt;
  uint32_t* khdone;          // host words (device view), one per block
  // Dispatch sequence: each of the launch's last
  // kSeqLast workgroups (by index) adds one to the device's started counter
  // on entry; a launch on another stream is gated on the count
  // (launch_seq_gate).  Null in a captured launch.
  unsigned long long* started;
#ifdef BPSR_KEYED_TRACE
  // Probe builds only (tools/dbg/build_keyed_trace_lib.sh): the keyed
  // consumer's wall_clock64() stamps — per tile entry, word seen, folded,
  // counted; then per key the helper's forward.
  unsigned long long* ktrace;
#endif
};
constexpr uint32_t kSeqLast = 8;  // one per XCD: workgroups are dealt round-robin over 8
inline uint32_t seq_counted(uint32_t grid) { return grid < kSeqLast ? grid : kSeqLast; }
// One wave on `s`: returns once the counter reaches target (the last
// workgroups of every launch counted so far have started), or after
// timeout_ticks of wall_clock64() (a safety net; the count is exact).
hipError_t launch_seq_gate(const unsigned long long* started, unsigned long long target,
                           uint64_t timeout_ticks, hipStream_t s);
// Arrival order of a keyed block: position m's source is worker
// (perm >> 4m) & 15 — positions 0..7 in the block's word, 8..15 in its second
// word (wide queues, 9..16 sources); kKeySkip: the round is folded
// elsewhere, the tiles only pass.
constexpr uint32_t kKeySkip = 0xffffffffu;
// A keyed queue's device words lie one per 128-B line (word b at
// kwords[b * kKeyWordStride], a wide queue's second words after the first
// ones): the tiles polling one key's word, and the helper storing the next,
// do not queue on the same few lines (round 6).
constexpr uint32_t kKeyWordStride = 16;
// ... and its tile counters one per 128-B line too (kcnt[b * kKeyCntStride]).
constexpr uint32_t kKeyCntStride = 32;
constexpr int kKeyedMaxSrcs = 16;
constexpr int kKeyedNarrowSrcs = 8;   // one word per block
inline uint64_t key_word(uint32_t perm, uint32_t epoch) {
  return ((uint64_t)perm << 32) | epoch;
}
// Released for epoch e: the block's word holds e or a later epoch (wrap-safe).
__host__ __device__ inline bool epoch_reached(uint32_t have, uint32_t e) {
  return (int32_t)(have - e) >= 0;
}

struct Tuning {
  int vpt;       // 16-B vectors per thread per tile (1, 2, 4)
  int nt;        // non-temporal loads and stores
  int max_grid;  // grid cap in workgroups (tile-stride beyond)
  int occ;       // workgroups resident per CU (0 = hardware limit), set through LDS
  int small_occ;        // residency for short fold launches (occ == 1 only)
  int small_occ_batch;  // residency for short batched launches (occ == 1 only)
  uint32_t occ_min_tiles;        // fold launches shorter than this are "short"
  uint32_t occ_min_tiles_batch;  // batched launches shorter than this are "short"
  int auto_n;    // residency/tile size by source count (bpsr_api.cpp tuning_for_n)
  int copy_occ;  // workgroups per CU of long copies (0 = hardware)
  int copy_vpt;  // copy tile: kBlock * copy_vpt 16-B vectors
  uint64_t wt_max_bytes;  // nt folds below this many bytes per source store write-through
};

// Residency cap through the dynamic LDS request: a CU has 160 KiB of LDS, so
// asking for 160 KiB / occ per workgroup admits at most `occ` workgroups per
// CU.  Fewer bytes in flight per CU stream HBM better for the 9-stream fold
// (tools/hbm_probe2.hip).
constexpr size_t kLdsPerCU = 160 * 1024;
// Dynamic LDS that caps a launch at `occ` workgroups per CU.  1 KiB short of
// the even share: the same residency (occ + 1 workgroups never fit), and room
// beside them for kernels with almost no LDS that must still get onto every
// CU — the server's copy service and release kernels.
inline size_t occ_lds_bytes(int occ) {
  return occ > 0 ? ((kLdsPerCU / (size_t)occ) - 1024) & ~(size_t)255 : 0;
}
// The 1-workgroup-per-CU cap pays on long sweeps only: below occ_min_tiles
// tiles (4096: 32 MiB per source at vpt 2) a launch is latency-bound and more
// residency wins (profiles/r01_occ_sweep.jsonl, r01_thr_fold.jsonl: 8 MiB
// 16.3 -> 14.6 us).  Batched launches (one Prophet block) likewise: the cap
// measured 9 % slower on cfg3's 13-20 MB blocks (r01_thr_batch.jsonl).
// Per calling thread: the fewest workgroups per CU a launch may be sized for
// (0 = no floor).  A PS server lane issuer with device releases sets 4: while
// a keyed consumer holds 2 × 58 KiB of every CU's LDS waiting for releases,
// a launch asking for more than the 44 KiB left would never be placed, and
// the release kernels queued behind it on the lane's stream — or on a stream
// sharing its hardware queue — would never run (bpsr_server.cpp issuer_main).
extern thread_local int t_occ_floor;
// Debug: where a server lane issuer is inside the library's launch helpers
// (its Lane::where, set by issuer_main; dumped with BPSR_SERVER_RELEASE_DEBUG).
extern thread_local std::atomic<const char*>* t_where;
inline void note_where(const char* w) {
  if (t_where) t_where->store(w, std::memory_order_relaxed);
}
inline int launch_occ(const Tuning& tu, uint64_t tiles, bool batched) {
  int o;
  if (tu.occ != 1) o = tu.occ;
  else if (tiles >= (batched ? tu.occ_min_tiles_batch : tu.occ_min_tiles)) o = 1;
  else o = batched ? tu.small_occ_batch : tu.small_occ;
  if (t_occ_floor > 0 && o > 0 && o < t_occ_floor) o = t_occ_floor;
  return o;
}
// Allow `kernel` to request up to `bytes` of dynamic LDS.  hipFuncSetAttribute
// acts on the calling thread's current device, so it is applied once PER
// DEVICE: bit d of `done` records device d (a process may drive several GPUs,
// e.g. one server or shard thread per device).
struct KernelAttr {
  std::atomic<uint64_t> done{0};
};
hipError_t allow_lds(KernelAttr& once, const void* kernel, int bytes = (int)kLdsPerCU);

int elem_size(int dtype);  // 0 if unsupported

// Staging for batched launches: a ring of pinned host + device descriptor
// tables, each reused once the kernel that read it completed.  The public
// byteps_reduce_sum_batched uses one per calling thread; the PS server owns
// one per engine lane (transport threads come and go).  Not thread-safe: one
// user at a time.
struct StageRing;
// zero_copy_max: tables up to this many bytes are read by the kernel from the
// pinned staging slot itself (0 = the library default, 256 KiB).
StageRing* stage_ring_create(size_t zero_copy_max = 0);
void stage_ring_destroy(StageRing* r);
// *done (optional): the event recorded behind the launch (the staging slot's
// guard; re-recorded only after a host wait for this launch, when the slot is
// reused), so a caller can wait for the launch without recording its own.
int batched_with_ring(const struct byteps_bucket_desc* buckets, int nbuckets, int dtype,
                      int mode, hipStream_t s, StageRing* ring, hipEvent_t* done = nullptr);

// Thread-local error reporting (byteps_reduce_last_error): fail() is in
// bpsr_error.h; hip_fail formats a HIP error the same way.
int hip_fail(hipError_t e, const char* what);

// Host-side geometry: vector range, head/tail split (fp16 body/tail rule of
// cpu_reducer.cc:103,118), co-alignment test.
void make_geom(int dtype, size_t len, const void* dst, const void* const* srcs, int n,
               bool copy_trailing, FoldGeom* g, int* aligned);

// One workgroup per tile of kBlock*vpt vectors (no cap: workgroups are
// dispatched in tile order, which keeps the HBM sweep tight); the element path
// reuses the same threads, grid-stride, when there is no vector range.
inline int fold_grid(const FoldGeom& g, const Tuning& tu, int vpt) {
  (void)tu;
  const uint64_t tile = (uint64_t)kBlock * vpt;
  uint64_t blocks = (g.nvec + tile - 1) / tile;
  const uint64_t scalar = g.head_elems + (g.n_elems - g.tail_begin) + g.trailing_bytes;
  const uint64_t sblocks = (scalar + kBlock - 1) / kBlock;
  if (blocks == 0) blocks = sblocks < 65536 ? sblocks : 65536;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

#define BPSR_DECLARE_LAUNCHERS(NAME)                                                      \
  hipError_t launch_fold_##NAME(const FoldArgs& a, const Tuning& tu, hipStream_t s);      \
  hipError_t launch_batched_##NAME(const BatchLaunch& L, int vpt, const Tuning& tu,      \
                                   hipStream_t s);                                        \
  hipError_t launch_blockq_##NAME(const BlockqLaunch& Q, int vpt, int pol, size_t lds,    \
                                  bool gated, hipStream_t s);
BPSR_DECLARE_LAUNCHERS(f32)
BPSR_DECLARE_LAUNCHERS(f64)
BPSR_DECLARE_LAUNCHERS(f16)
BPSR_DECLARE_LAUNCHERS(f16acc)
BPSR_DECLARE_LAUNCHERS(bf16)
BPSR_DECLARE_LAUNCHERS(bf16acc)
BPSR_DECLARE_LAUNCHERS(i8)
BPSR_DECLARE_LAUNCHERS(i32)
BPSR_DECLARE_LAUNCHERS(i64)

hipError_t launch_fold(const FoldArgs& a, int dtype, int mode, const Tuning& tu,
                       hipStream_t s);
hipError_t launch_batched(const BatchLaunch& L, int vpt, int dtype, int mode, const Tuning& tu,
                          hipStream_t s);
hipError_t launch_blockq(const BlockqLaunch& Q, int vpt, int pol, size_t lds, bool gated,
                         int dtype, int mode, hipStream_t s);
hipError_t launch_blockq_release(uint32_t* flags, uint32_t first, uint32_t count, uint32_t epoch,
                                 hipStream_t s);
// Stream-ordered keyed release: kwords[block] = word (system scope, release;
// block: the word's index, key * kKeyWordStride);
// a wide queue's second word first (word2_at = &kwords[nblocks + block], else
// null).
hipError_t launch_key_release(uint64_t* kwords, uint32_t block, uint64_t word,
                              uint64_t* word2_at, uint64_t word2, hipStream_t s);
// The HSA id of the hardware queue behind stream `s` (a one-wave kernel reads
// hsa_queue_t::id through its dispatch's queue pointer into `out`, pinned host
// memory); synchronises `s`.  Queue placement.
hipError_t read_queue_id(hipStream_t s, uint64_t* out);

// Tile size actually used for a single fold: the tuned vpt, halved while the
// launch would have fewer than kMinTiles tiles.
inline int fold_vpt(uint64_t nvec, int vpt) {
  auto tiles = [nvec](int v) { return (nvec + (uint64_t)kBlock * v - 1) / ((uint64_t)kBlock * v); };
  while (vpt > 1 && tiles(vpt) < kMinTiles) vpt >>= 1;
  // Mid-size launches (2048..4095 tiles of 16 KiB: 32-64 MiB per source) run
  // 4-5 % faster with the bigger tile; longer sweeps prefer 8 KiB
  // (profiles/r01_thr_fold.jsonl).
  if (vpt == 2 && tiles(4) >= kMinTiles && tiles(4) < 2 * kMinTiles) vpt = 4;
  return vpt;
}
// Cache policy of a fold's buffer instructions (the kernels' NT template
// argument): plain; nt loads and stores; or nt loads with write-through (sc1)
// stores.  Write-through leaves no dirty output lines in the XCDs' L2s for the
// end-of-kernel release to flush, which mid-size launches feel as a fixed cost
// (DESIGN.md §4.1); long sweeps stream faster with nt stores.
constexpr int kPolPlain = 0, kPolNt = 1, kPolWt = 2;
constexpr uint64_t kWtMaxBytes = 96ull << 20;  // per source (Tuning default)
// write-through folds from this size per source run 4-KiB tiles, 2 per CU
constexpr uint64_t kHalfTileMinBytes = 64ull << 20;
inline int cache_pol(const Tuning& tu, uint64_t bytes_per_src) {
  if (!tu.nt) return kPolPlain;
  return bytes_per_src < tu.wt_max_bytes ? kPolWt : kPolNt;
}
// byteps_reduce_sum_n, except that dst may also alias one srcs[k] with k > 0
// exactly (n <= kMaxSrcs: one launch, every element read before it is
// written by the same thread) — the in-place owner fold of the shard calls.
int fold_any_alias(void* dst, const void* const* srcs, int n, size_t len, int dtype, int mode,
                   hipStream_t s);

hipError_t launch_copy(void* dst, const void* src, size_t len, const Tuning& tu,
                       hipStream_t s);

// Pull copy service (bpsr_copy_service.cpp, kernel in bpsr_k_service.hip):
// a persistent kernel of a few workgroups serving copies that host threads
// post into a pinned job ring — a blocking pull's copy with no HIP call and
// no thread hand-off on the caller's side.  Job j sits in slot j % kSvcRing
// of the host ring; the launch's fetcher (workgroup 0) moves posted jobs into
// the same slot of a device ring, where copier g (workgroups 1..wgs-1) finds
// jobs start + g - 1, start + g - 1 + (wgs - 1), ...  Every descriptor word
// carries the job's 16-bit tag in its top bits (addresses and lengths fit in
// 48), so a reader that sees the tag in all three words has the whole job:
// no separate publish word, no ordering between the words' stores.
constexpr uint32_t kSvcRing = 4096;
constexpr uint32_t kDoneStride = 8;  // done words one 64-B line apart (spinning host threads)
constexpr uint64_t kSvcMask = (1ull << 48) - 1;
struct SvcJob {      // 32 B: dst, src, len, each | tag << 48; one pad word
  uint64_t w[4];
};
// 1..65535, never 0 (zeroed slots); one slot's successive jobs differ
// (4096 and 65535 are coprime)
__host__ __device__ inline uint64_t svc_tag(uint64_t job) { return job % 0xFFFFull + 1; }
constexpr uint64_t kSvcExitDone = 1, kSvcExitStop = 2;
struct SvcArgs {
  const SvcJob* ring;      // host ring (device view)
  SvcJob* dring;           // device ring
  uint64_t* done;          // host words: done[slot * kDoneStride] = job + 1 once the copy is visible
  const uint32_t* stop;    // host word: nonzero = exit now, copying nothing more
  uint32_t* exited;        // host word: the fetcher stores `gen` when it decides to exit
  uint64_t* dev;           // device words: [1] jobs completed, [2] exit flag
                           // (kSvcExitDone: copy what was fetched; kSvcExitStop: copy nothing)
  uint64_t start;          // first job index of this launch
  uint64_t check_below;    // jobs below this may be done already (a relaunch): look first
  uint64_t idle_ticks;     // exit after this long without a new job ...
  uint64_t max_ticks;      // ... or once this launch is this old (a relaunch takes over)
  uint64_t stall_ticks;    // tests only: a copier holds every job this long (0 in the product)
  uint32_t wgs;            // fetcher + copiers
  uint32_t gen;            // this launch's number (for `exited`)
  uint64_t* trace;         // probes only (null in the product): per slot, wall clock at
                           // [0] fetched, [1] picked up, [2] copied and drained
};
hipError_t launch_copy_service(const SvcArgs& a, hipStream_t s);

struct CopyService;
int copysvc_create(int device, CopyService** out);
// Blocking copy of len bytes (device memory to device memory) through the
// service; returns once the bytes are visible to later work on the device.
int copysvc_copy(CopyService* svc, void* dst, const void* src, size_t len);
void copysvc_destroy(CopyService* svc);
// Non-blocking form: post the copy (jobs [*first, *first + *n)), then test
// it; copysvc_test keeps the service serving (relaunch, timeout) like a
// blocking copy's wait.  `posted_ns` = copysvc_now_ns() taken before posting.
int copysvc_post(CopyService* svc, void* dst, const void* src, size_t len, uint64_t* first,
                 uint64_t* n);
int copysvc_test(CopyService* svc, uint64_t first, uint64_t n, int64_t posted_ns, bool* done);
int64_t copysvc_now_ns();
uint64_t copysvc_launches(CopyService* svc);  // kernel launches so far (0 for null)
// A job timed out or a launch failed: the service takes no more jobs (its
// callers use another copy path from then on).
bool copysvc_broken(const CopyService* svc);
// A give-up whose launch did not end in time: hard errors, no fallback copy.
bool copysvc_wedged(const CopyService* svc);
// Probes (tools/dbg/copysvc_probe.cpp): jobs posted so far; a device trace
// buffer (kSvcRing * 4 words) used from the next launch on.
uint64_t copysvc_posted(CopyService* svc);
void copysvc_set_trace(CopyService* svc, uint64_t* dev_trace);

// Keyed block queue (bpsr_api.cpp): the PS server's device releases.  One
// block per key (bucket k: dst = the key's store, srcs = its receive slots in
// WORKER order, n <= kKeyedMaxSrcs); launch k folds every key once, each tile
// as soon as its own key is released for epoch k, in the arrival order its
// release carries.  keyq_release with s == nullptr stores the word from the
// host (the round's data already visible to the device); with a stream, a
// one-lane kernel stores it behind that stream's earlier work.  The k-th
// release of a key carries epoch k.  keyq_failed: a launch gave up waiting
// (timeout), read from pinned host memory without a copy.
int keyq_create(const struct byteps_bucket_desc* buckets, int nkeys, int dtype, double timeout_s,
                struct byteps_reduce_blockq** out);
int keyq_launch(struct byteps_reduce_blockq* q, hipEvent_t stop, hipStream_t* stream,
                uint32_t* epoch);
uint32_t keyq_next_epoch(struct byteps_reduce_blockq* q, int key);
uint32_t keyq_launched(struct byteps_reduce_blockq* q);
// Pass epoch `epoch` without a launch (the next launch consumes epoch + 1):
// an epoch no consumer folds.  False unless `epoch` is the next one to launch.
bool keyq_advance(struct byteps_reduce_blockq* q, uint32_t epoch);
// Both of the above under one lock.
void keyq_state(byteps_reduce_blockq* q, int key, uint32_t* next_epoch, uint32_t* launched);
// `first` (optional): set when this release is the first one of its epoch
// (keyq_opened; after keyq_close, none is).
int keyq_release(struct byteps_reduce_blockq* q, int key, uint64_t perm, hipStream_t s,
                 bool* first = nullptr);
// The highest epoch a key has been released for (a round, or a skip word for
// a round folded elsewhere) or closed: an epoch at or below it has begun
// (lock-free host read).
uint32_t keyq_opened(const struct byteps_reduce_blockq* q);
// Mark `epoch` begun without a round (an epoch launched ahead is retired):
// false when a round was released for it first.  Rounds released for it
// afterwards are folded by its consumer as usual, but are not its first.
bool keyq_close(struct byteps_reduce_blockq* q, uint32_t epoch);
bool keyq_failed(struct byteps_reduce_blockq* q);
// The key's fold for `epoch` is complete and visible device-wide (its block's
// last tile stored the completion word): a lock-free host read.
bool keyq_key_done(const struct byteps_reduce_blockq* q, int key, uint32_t epoch);
std::string keyq_debug(struct byteps_reduce_blockq* q);  // state summary (synchronous copy)

}  // namespace bpsr
