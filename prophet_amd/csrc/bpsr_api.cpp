// C ABI of libbpsr.so (include/bpsr/reduce.h): argument checking, geometry,
// descriptor staging and dispatch to the gfx950 kernels.  Never aborts: every
// failure is a negative status plus a thread-local message.
#include "bpsr/reduce.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "bpsr_internal.h"

namespace bpsr {

static thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(BYTEPS_REDUCE_EHIP, "%s: %s", what, hipGetErrorString(e));
}

int elem_size(int dtype) {
  switch (dtype) {
    case kInt8: case kUInt8: return 1;
    case kFloat16: case kBFloat16: return 2;
    case kInt32: case kFloat32: return 4;
    case kInt64: case kFloat64: return 8;
    default: return 0;
  }
}

void make_geom(int dtype, size_t len, const void* dst, const void* const* srcs, int n,
               bool copy_trailing, FoldGeom* g, int* aligned) {
  const uint64_t es = (uint64_t)elem_size(dtype);
  std::memset(g, 0, sizeof(*g));
  g->n_elems = len / es;
  g->trailing_bytes = len % es;
  g->copy_trailing = (copy_trailing && g->trailing_bytes) ? 1u : 0u;
  const uintptr_t d = (uintptr_t)dst;
  bool elem_al = (d % es) == 0, co = true;
  for (int k = 0; k < n; ++k) {
    const uintptr_t s = (uintptr_t)srcs[k];
    elem_al = elem_al && (s % es) == 0;
    co = co && ((s & 15u) == (d & 15u));
  }
  *aligned = elem_al ? 1 : 0;
  // fp16: elements >= floor(n/8)*8 are the reference's scalar tail
  // (cpu_reducer.cc:103 vs :118) and must not enter the vector path.
  const uint64_t vec_end = dtype == kFloat16 ? (g->n_elems / 8) * 8 : g->n_elems;
  g->tail_sem_from = dtype == kFloat16 ? vec_end : g->n_elems;
  if (elem_al && co) {
    uint64_t head = ((16u - (d & 15u)) & 15u) / es;
    if (head > g->n_elems) head = g->n_elems;
    g->head_elems = head;
    g->vec_off = head * es;
    g->nvec = vec_end > head ? ((vec_end - head) * es) / 16 : 0;
    g->tail_begin = head + g->nvec * 16 / es;
  } else {
    g->head_elems = 0;
    g->vec_off = 0;
    g->nvec = 0;
    g->tail_begin = 0;
  }
}

// Process-wide tuning, read by every launch (engine lanes and caller threads)
// and written by byteps_reduce_set_tuning: launches take a snapshot under the
// lock, so a concurrent set_tuning never tears a launch's geometry.
static std::mutex g_tuning_mu;
thread_local int t_occ_floor = 0;
thread_local std::atomic<const char*>* t_where = nullptr;

static Tuning& tuning_storage() {
  static Tuning tu = [] {
    // tools/sweep.py, tools/occ_sweep.py, tools/cfg3_probe.py (profiles/)
    Tuning t{2, 1, 1 << 20, 1, 2, 0, 4096, 4096, 1, 4, 2, kWtMaxBytes};
    if (const char* v = getenv("BPSR_WT_MAX_MIB")) t.wt_max_bytes = (uint64_t)atoll(v) << 20;
    if (const char* v = getenv("BPSR_COPY_OCC")) t.copy_occ = atoi(v);
    if (const char* v = getenv("BPSR_COPY_VPT")) t.copy_vpt = atoi(v);
    if (t.copy_occ < 0 || t.copy_occ > 8) t.copy_occ = 4;
    if (t.copy_vpt != 1 && t.copy_vpt != 4) t.copy_vpt = 2;
    if (const char* v = getenv("BPSR_OCC_MIN_TILES")) t.occ_min_tiles = (uint32_t)atol(v);
    if (const char* v = getenv("BPSR_OCC_MIN_TILES_BATCH"))
      t.occ_min_tiles_batch = (uint32_t)atol(v);
    if (const char* v = getenv("BPSR_AUTO_N")) t.auto_n = atoi(v) != 0;
    if (const char* v = getenv("BPSR_VPT")) t.vpt = atoi(v);
    if (const char* v = getenv("BPSR_NT")) t.nt = atoi(v);
    if (const char* v = getenv("BPSR_MAX_GRID")) t.max_grid = atoi(v);
    if (const char* v = getenv("BPSR_OCC")) t.occ = atoi(v);
    if (const char* v = getenv("BPSR_SMALL_OCC")) t.small_occ = atoi(v);
    if (const char* v = getenv("BPSR_SMALL_OCC_BATCH")) t.small_occ_batch = atoi(v);
    if (t.small_occ < 0 || t.small_occ > 8) t.small_occ = 2;
    if (t.small_occ_batch < 0 || t.small_occ_batch > 8) t.small_occ_batch = 0;
    if (t.vpt != 1 && t.vpt != 4) t.vpt = 2;
    if (t.occ < 0 || t.occ > 8) t.occ = 1;
    if (t.max_grid < 1) t.max_grid = 1 << 20;
    t.nt = t.nt ? 1 : 0;
    return t;
  }();
  return tu;
}

static Tuning tuning() {
  std::lock_guard<std::mutex> g(g_tuning_mu);
  return tuning_storage();
}

// Bytes in flight per CU = residency x 256 lanes x n sources x vpt x 16 B.
// The defaults (1 workgroup per CU, vpt 2) give 64 KiB at the 8-way fold;
// with n <= 4 sources that leaves the HBM queues short, and 2 workgroups per
// CU with 16 KiB tiles measured +13-26 % (profiles/r01_nsweep.jsonl: 2-way
// 256 MiB 5.21 -> 6.56 TB/s).  Applies unless BPSR_AUTO_N=0.
static Tuning tuning_for_n(int n) {
  Tuning t = tuning();
  if (t.auto_n && n <= 4 && t.occ == 1) {
    t.occ = 2;
    t.vpt = 4;
  }
  return t;
}

static inline hipStream_t to_stream(void* s) {
  return s ? reinterpret_cast<hipStream_t>(s) : hipStreamPerThread;
}

static bool overlaps_partially(const void* a, const void* b, size_t len) {
  if (a == b || len == 0) return false;
  const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
  return x < y + len && y < x + len;
}

// One fold launch over at most kMaxSrcs sources.
static int fold_once(void* dst, const void* const* srcs, int n, size_t len, int dtype,
                     int mode, bool copy_trailing, hipStream_t s) {
  FoldArgs a;
  std::memset(&a, 0, sizeof(a));
  for (int k = 0; k < n; ++k) a.srcs[k] = static_cast<const unsigned char*>(srcs[k]);
  a.dst = static_cast<unsigned char*>(dst);
  a.n = n;
  make_geom(dtype, len, dst, srcs, n, copy_trailing, &a.g, &a.aligned);
  hipError_t e = launch_fold(a, dtype, mode, tuning_for_n(n), s);
  if (e != hipSuccess) return hip_fail(e, "fold kernel launch");
  return BYTEPS_REDUCE_OK;
}

static int check_common(int dtype, int mode) {
  if (elem_size(dtype) == 0) return fail(BYTEPS_REDUCE_EDTYPE, "Unsupported data type: %d", dtype);
  if (mode != kModeReference && mode != kModeAccumF32)
    return fail(BYTEPS_REDUCE_EARGS, "unknown mode %d", mode);
  return BYTEPS_REDUCE_OK;
}

// ------------------------------------------------ batched descriptor staging --
// Per-thread ring of pinned host + device tables.  A slot is reused only after
// the event recorded behind the kernel that read it has completed.
struct StageSlot {
  int device = -1;
  size_t cap = 0;
  void* host = nullptr;      // pinned, coherent (the device reads it uncached)
  void* host_dev = nullptr;  // the same pages as the device addresses them
  void* dev = nullptr;
  hipEvent_t done = nullptr;
  bool pending = false;
};
constexpr int kRing = 8;
// Tables up to this size are read by the kernel straight from the pinned
// staging slot (each workgroup fetches its own record over PCIe once) instead
// of being copied to HBM first: a small hipMemcpyAsync H2D waits for the
// stream's earlier work on the host (130-380 us per call behind queued folds,
// rocprofv3 HIP trace of the server's issuer threads).
constexpr size_t kZeroCopyTable = 256 * 1024;  // default; a ring may read larger ones in place

struct StageRing {
  StageSlot slots[kRing];
  int next = 0;
  size_t zero_copy_max = kZeroCopyTable;
  std::vector<char> table;  // host copy of the table being built
  // Buffers a slot outgrew: freed with the ring, never while it is in use —
  // hipFree waits for the whole device, and a server lane's issuer must not
  // wait for a running keyed consumer that waits for the releases it queues.
  std::vector<void*> retired_host, retired_dev;
  ~StageRing() {
    for (auto& s : slots) {
      if (s.pending && s.done) (void)hipEventSynchronize(s.done);
      if (s.done) (void)hipEventDestroy(s.done);
      if (s.host) (void)hipHostFree(s.host);
      if (s.dev) (void)hipFree(s.dev);
    }
    for (void* p : retired_host) (void)hipHostFree(p);
    for (void* p : retired_dev) (void)hipFree(p);
  }
};
static thread_local StageRing g_ring;

StageRing* stage_ring_create(size_t zero_copy_max) {
  auto* r = new StageRing();
  if (zero_copy_max) r->zero_copy_max = zero_copy_max;
  return r;
}
void stage_ring_destroy(StageRing* r) { delete r; }

static int stage_acquire(StageRing& ring, size_t bytes, StageSlot** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  StageSlot& s = ring.slots[ring.next];
  ring.next = (ring.next + 1) % kRing;
  if (s.pending) {
    note_where("ring: slot event sync");
    e = hipEventSynchronize(s.done);
    if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize(stage)");
    s.pending = false;
  }
  if (s.device != dev || s.cap < bytes) {
    // the outgrown buffers are retired, not freed (see StageRing)
    if (s.host) ring.retired_host.push_back(s.host);
    if (s.dev) ring.retired_dev.push_back(s.dev);
    if (s.done) (void)hipEventDestroy(s.done);
    s.host = s.host_dev = s.dev = nullptr;
    s.done = nullptr;
    note_where("ring: grow");
    // grow geometrically: freeing pinned memory synchronises the device
    const size_t cap = std::max<size_t>({bytes, 2 * s.cap, kZeroCopyTable});
    s.cap = 0;
    if ((e = hipHostMalloc(&s.host, cap, hipHostMallocMapped | hipHostMallocCoherent)) !=
        hipSuccess)
      return hip_fail(e, "hipHostMalloc(stage)");
    if ((e = hipHostGetDevicePointer(&s.host_dev, s.host, 0)) != hipSuccess)
      return hip_fail(e, "hipHostGetDevicePointer(stage)");
    if ((e = hipMalloc(&s.dev, cap)) != hipSuccess) return hip_fail(e, "hipMalloc(stage)");
    if ((e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming)) != hipSuccess)
      return hip_fail(e, "hipEventCreate(stage)");
    s.cap = cap;
    s.device = dev;
  }
  *out = &s;
  return BYTEPS_REDUCE_OK;
}

// ------------------------------------------------------- batch table build --
struct TableInfo {
  int vpt = 1;   // tile size of the batched kernel for this table
  int nmax = 1;  // most sources of any bucket (residency rule, tuning_for_n)
  int live = 0;          // buckets with len > 0
  uint32_t tiles = 0;    // workgroups (element tiles first, then vector tiles)
  uint32_t rec_stride = 0;
  size_t recs_off = 0;   // byte offset of the tile records in the table
  size_t bytes = 0;      // bytes to upload
};

// Element work of one bucket (head, tail, trailing bytes) in parts of
// kElemPart elements per workgroup.
constexpr uint64_t kElemPart = (uint64_t)kBlock * 16;

// Validate buckets and write [BatchEntry x live][pad to 256][TileRec x tiles]
// into `out` (bpsr_internal.h: TileHead).  With `block_end` (a block queue:
// block i = buckets [block_end[i-1], block_end[i])), the records are laid out
// block by block — each block's element tiles, then its vector tiles — and
// `block_first` receives every block's first record (nblocks + 1 entries).
static int build_table(const byteps_bucket_desc* buckets, int nbuckets, int dtype,
                       std::vector<char>& out, TableInfo* ti, const int* block_end = nullptr,
                       int nblocks = 0, std::vector<uint32_t>* block_first = nullptr,
                       int force_vpt = 0) {
  std::vector<BatchEntry> tab;
  std::vector<int> tab_block;  // block of each live bucket
  tab.reserve(nbuckets);
  int blk = 0;
  uint64_t vecs = 0;
  int nmax = 1;
  for (int i = 0; i < nbuckets; ++i) {
    const byteps_bucket_desc& b = buckets[i];
    if (b.n < 1 || b.n > kMaxSrcs)
      return fail(BYTEPS_REDUCE_EARGS, "bucket %d: n=%d outside [1, %d]", i, b.n, kMaxSrcs);
    while (block_end && blk < nblocks && i >= block_end[blk]) ++blk;
    if (b.len == 0) continue;
    if (!b.dst) return fail(BYTEPS_REDUCE_EARGS, "bucket %d: null dst", i);
    for (int k = 0; k < b.n; ++k) {
      if (!b.srcs[k]) return fail(BYTEPS_REDUCE_EARGS, "bucket %d: null srcs[%d]", i, k);
      if (overlaps_partially(b.dst, b.srcs[k], b.len) || (k > 0 && b.srcs[k] == b.dst))
        return fail(BYTEPS_REDUCE_EARGS, "bucket %d: dst overlaps srcs[%d]", i, k);
    }
    BatchEntry e;
    std::memset(&e, 0, sizeof(e));
    for (int k = 0; k < b.n; ++k) e.srcs[k] = static_cast<const unsigned char*>(b.srcs[k]);
    e.dst = static_cast<unsigned char*>(b.dst);
    e.n = b.n;
    make_geom(dtype, b.len, b.dst, b.srcs, b.n, b.dst != b.srcs[0], &e.g, &e.aligned);
    vecs += e.g.nvec;
    nmax = std::max(nmax, b.n);
    tab.push_back(e);
    tab_block.push_back(blk);
  }
  // Same tile-size rule as a single fold (fold_vpt): the tuned vpt, halved
  // while the launch would have fewer than kMinTiles tiles.
  const int vpt = force_vpt ? force_vpt : fold_vpt(vecs, tuning_for_n(nmax).vpt);
  const uint64_t tile_vecs = (uint64_t)kBlock * vpt;
  auto elem_parts = [](const BatchEntry& e) -> uint64_t {
    const uint64_t n_scalar = e.g.head_elems + (e.g.n_elems - e.g.tail_begin);
    const bool trailing = e.g.copy_trailing && e.g.trailing_bytes > 0;
    if (n_scalar == 0 && !trailing) return 0;
    const uint64_t p = (n_scalar + kElemPart - 1) / kElemPart;
    return std::min<uint64_t>(std::max<uint64_t>(p, 1), 65536);
  };
  uint64_t tiles = 0;
  for (auto& e : tab) tiles += elem_parts(e) + (e.g.nvec + tile_vecs - 1) / tile_vecs;
  // grid.x * 256 threads must stay below 2^32
  if (tiles >= (1ull << 32) / kBlock) return fail(BYTEPS_REDUCE_EARGS, "batch too large");
  const uint32_t stride = tile_rec_stride(nmax);
  const size_t recs_off = ((sizeof(BatchEntry) * tab.size()) + 255) & ~(size_t)255;
  out.assign(recs_off + (size_t)stride * tiles, 0);
  if (!tab.empty()) std::memcpy(out.data(), tab.data(), sizeof(BatchEntry) * tab.size());
  char* rec = out.data() + recs_off;
  uint32_t cur_block = 0;
  auto put = [&](unsigned char* dst, uint32_t kind, const BatchEntry& e, uint32_t a, uint32_t b,
                 uint32_t c, uint64_t byte0) {
    TileHead h;
    std::memset(&h, 0, sizeof(h));
    h.dst = dst + byte0;
    h.kind = kind;
    h.n = (uint32_t)e.n;
    h.a = a;
    h.b = b;
    h.c = c;
    h.block = cur_block;
    std::memcpy(rec, &h, sizeof(h));
    const unsigned char** p = reinterpret_cast<const unsigned char**>(rec + kTileHeadBytes);
    for (int k = 0; k < e.n; ++k) p[k] = e.srcs[k] + byte0;
    rec += stride;
  };
  // Records of the live buckets [b0, b1): element tiles first (they are
  // latency-bound and start with the launch), then the vector tiles.
  auto emit = [&](size_t b0, size_t b1) {
    for (size_t b = b0; b < b1; ++b) {
      const uint64_t parts = elem_parts(tab[b]);
      for (uint64_t q = 0; q < parts; ++q)
        put(tab[b].dst, kTileElem, tab[b], (uint32_t)q, (uint32_t)b, (uint32_t)parts, 0);
    }
    for (size_t b = b0; b < b1; ++b) {
      const BatchEntry& e = tab[b];
      for (uint64_t v0 = 0; v0 < e.g.nvec; v0 += tile_vecs) {
        const uint64_t left = e.g.nvec - v0;
        const bool full = left >= tile_vecs;
        put(e.dst, full ? kTileFull : kTilePartial, e, full ? 0u : (uint32_t)left, (uint32_t)b,
            0, e.g.vec_off + v0 * 16);
      }
    }
  };
  char* const rec0 = rec;
  if (!block_end) {
    emit(0, tab.size());
  } else {
    block_first->assign((size_t)nblocks + 1, 0);
    size_t b0 = 0;
    for (int k = 0; k < nblocks; ++k) {
      size_t b1 = b0;
      while (b1 < tab.size() && tab_block[b1] == k) ++b1;
      (*block_first)[k] = (uint32_t)((rec - rec0) / stride);
      cur_block = (uint32_t)k;
      emit(b0, b1);
      b0 = b1;
    }
    (*block_first)[nblocks] = (uint32_t)tiles;
  }
  ti->vpt = vpt;
  ti->nmax = nmax;
  ti->live = (int)tab.size();
  ti->tiles = (uint32_t)tiles;
  ti->rec_stride = stride;
  ti->recs_off = recs_off;
  ti->bytes = out.size();
  return BYTEPS_REDUCE_OK;
}

// `in_hbm`: the records live in device memory.  A table read zero-copy from
// pinned host staging (batched_with_ring, small tables) is not prefetched:
// host pages are not cached in L2, so the touch would only add a PCIe round
// trip that every workgroup waits for before it retires.
static BatchLaunch batch_launch(const void* dev_table, const TableInfo& ti, bool in_hbm = true) {
  BatchLaunch L;
  L.entries = static_cast<const BatchEntry*>(dev_table);
  L.recs = static_cast<const unsigned char*>(dev_table) + ti.recs_off;
  L.rec_stride = ti.rec_stride;
  L.tiles = ti.tiles;
  // record prefetch distance (bpsr_kernels_impl.h prefetch_record): one
  // resident round of the 256-CU chip; BPSR_REC_PREFETCH=0 turns it off (A/B)
  static const uint32_t ahead = [] {
    const char* v = getenv("BPSR_REC_PREFETCH");
    const long x = v ? atol(v) : (long)kPrefetchAhead;
    return x > 0 ? (uint32_t)((x + 7) & ~7L) : 0u;  // a multiple of 8: the same XCD
  }();
  L.pf_ahead = in_hbm ? ahead : 0u;
  L.stop = nullptr;
  return L;
}


int batched_with_ring(const byteps_bucket_desc* buckets, int nbuckets, int dtype, int mode,
                      hipStream_t s, StageRing* ring, hipEvent_t* done) {
  if (done) *done = nullptr;
  int rc = check_common(dtype, mode);
  if (rc) return rc;
  if (nbuckets < 0 || (nbuckets > 0 && !buckets))
    return fail(BYTEPS_REDUCE_EARGS, "bad bucket table");
  if (nbuckets == 0) return BYTEPS_REDUCE_OK;
  TableInfo ti;
  if ((rc = build_table(buckets, nbuckets, dtype, ring->table, &ti))) return rc;
  if (ti.tiles == 0) return BYTEPS_REDUCE_OK;
  StageSlot* slot = nullptr;
  if ((rc = stage_acquire(*ring, ti.bytes, &slot))) return rc;
  std::memcpy(slot->host, ring->table.data(), ti.bytes);
  hipError_t e = hipSuccess;
  const void* table = slot->host_dev;
  note_where("ring: table copy");
  if (ti.bytes > ring->zero_copy_max) {  // large: one H2D copy, the kernel reads HBM
    e = hipMemcpyAsync(slot->dev, slot->host, ti.bytes, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(batch table)");
    table = slot->dev;
  }
  // (The slot's event stays a separate record: completing it by the launch
  // itself, like the block queue's join, made the server's lane issuers see
  // completions sooner and split config 3's rounds into more, smaller
  // launches — 33-43 instead of 23-31 per round at 4 lanes, r03s57.)
  note_where("ring: kernel launch");
  e = launch_batched(batch_launch(table, ti, table == slot->dev), ti.vpt, dtype, mode,
                     tuning_for_n(ti.nmax), s);
  note_where("ring: event record");
  if (e != hipSuccess) return hip_fail(e, "batched kernel launch");
  e = hipEventRecord(slot->done, s);
  if (e != hipSuccess) return hip_fail(e, "hipEventRecord(stage)");
  slot->pending = true;
  if (done) *done = slot->done;
  return BYTEPS_REDUCE_OK;
}

int fold_any_alias(void* dst, const void* const* srcs, int n, size_t len, int dtype, int mode,
                   hipStream_t s) {
  int alias = -1;
  for (int k = 0; k < n && srcs; ++k)
    if (srcs[k] == dst) alias = k;
  if (alias <= 0) return byteps_reduce_sum_n(dst, srcs, n, len, dtype, mode, s);
  int rc = check_common(dtype, mode);
  if (rc) return rc;
  if (n > kMaxSrcs)
    return fail(BYTEPS_REDUCE_EARGS, "dst aliases srcs[%d] of a %d-way fold (> %d)", alias, n,
                kMaxSrcs);
  if (len == 0) return BYTEPS_REDUCE_OK;
  for (int k = 0; k < n; ++k) {
    if (!srcs[k]) return fail(BYTEPS_REDUCE_EARGS, "null srcs[%d]", k);
    if (overlaps_partially(dst, srcs[k], len))
      return fail(BYTEPS_REDUCE_EARGS, "dst partially overlaps srcs[%d]", k);
    if (k != alias && srcs[k] == dst)
      return fail(BYTEPS_REDUCE_EARGS, "dst aliases two sources");
  }
  return fold_once(dst, srcs, n, len, dtype, mode, /*copy_trailing=*/true, s);
}

}  // namespace bpsr

using namespace bpsr;

extern "C" {

int byteps_reduce_version(void) { return BYTEPS_REDUCE_ABI_VERSION; }

int byteps_reduce_dtype_size(int dtype) {
  const int es = elem_size(dtype);
  return es ? es : fail(BYTEPS_REDUCE_EDTYPE, "Unsupported data type: %d", dtype);
}

const char* byteps_reduce_last_error(void) { return g_last_error.c_str(); }

int byteps_reduce_set_tuning(int vpt, int nt, int max_grid, int occ) {
  // validate everything before changing anything
  if (vpt > 0 && vpt != 1 && vpt != 2 && vpt != 4)
    return fail(BYTEPS_REDUCE_EARGS, "vpt must be 1, 2 or 4");
  if (occ > 8) return fail(BYTEPS_REDUCE_EARGS, "occ must be 0..8");
  std::lock_guard<std::mutex> g(g_tuning_mu);
  Tuning& t = tuning_storage();
  if (vpt > 0) t.vpt = vpt;
  if (nt >= 0) t.nt = nt ? 1 : 0;
  if (max_grid > 0) t.max_grid = max_grid;
  if (occ >= 0) t.occ = occ;
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_get_tuning(int* vpt, int* nt, int* max_grid, int* occ) {
  const Tuning t = tuning();
  if (vpt) *vpt = t.vpt;
  if (nt) *nt = t.nt;
  if (max_grid) *max_grid = t.max_grid;
  if (occ) *occ = t.occ;
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_init(int device) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  (void)tuning();
  e = hipFree(nullptr);  // forces context creation
  if (e != hipSuccess) return hip_fail(e, "hip runtime init");
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_shutdown(void) {
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_fail(e, "hipDeviceSynchronize");
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_sum(void* dst, const void* src, size_t len, int dtype, void* stream) {
  int rc = check_common(dtype, kModeReference);
  if (rc) return rc;
  if (len == 0) return BYTEPS_REDUCE_OK;
  if (!dst || !src) return fail(BYTEPS_REDUCE_EARGS, "null pointer");
  if (overlaps_partially(dst, src, len))
    return fail(BYTEPS_REDUCE_EARGS, "dst and src partially overlap");
  const void* srcs[2] = {dst, src};
  return fold_once(dst, srcs, 2, len, dtype, kModeReference, false, to_stream(stream));
}

int byteps_reduce_sum3(void* dst, const void* src1, const void* src2, size_t len, int dtype,
                       void* stream) {
  int rc = check_common(dtype, kModeReference);
  if (rc) return rc;
  if (len == 0) return BYTEPS_REDUCE_OK;
  if (!dst || !src1 || !src2) return fail(BYTEPS_REDUCE_EARGS, "null pointer");
  if (overlaps_partially(dst, src1, len) || overlaps_partially(dst, src2, len))
    return fail(BYTEPS_REDUCE_EARGS, "dst partially overlaps a source");
  const void* srcs[2] = {src1, src2};
  return fold_once(dst, srcs, 2, len, dtype, kModeReference, false, to_stream(stream));
}

int byteps_reduce_sum_n(void* dst, const void* const* srcs, int n, size_t len, int dtype,
                        int mode, void* stream) {
  int rc = check_common(dtype, mode);
  if (rc) return rc;
  if (n < 1 || !srcs) return fail(BYTEPS_REDUCE_EARGS, "need n >= 1 sources (n=%d)", n);
  if (len == 0) return BYTEPS_REDUCE_OK;
  if (!dst) return fail(BYTEPS_REDUCE_EARGS, "null dst");
  for (int k = 0; k < n; ++k) {
    if (!srcs[k]) return fail(BYTEPS_REDUCE_EARGS, "null srcs[%d]", k);
    if (overlaps_partially(dst, srcs[k], len))
      return fail(BYTEPS_REDUCE_EARGS, "dst partially overlaps srcs[%d]", k);
    if (k > 0 && srcs[k] == dst)
      return fail(BYTEPS_REDUCE_EARGS, "dst may alias only srcs[0] (srcs[%d] == dst)", k);
  }
  hipStream_t s = to_stream(stream);
  if (n == 1) {
    if (dst == srcs[0]) return BYTEPS_REDUCE_OK;
    hipError_t e = launch_copy(dst, srcs[0], len, tuning(), s);
    return e == hipSuccess ? BYTEPS_REDUCE_OK : hip_fail(e, "copy kernel launch");
  }
  // First launch folds up to kMaxSrcs sources; each further launch folds the
  // running result (as its srcs[0]) with the next kMaxSrcs-1: still a strict
  // left fold, bit-exact in reference mode.
  int take = std::min(n, kMaxSrcs);
  rc = fold_once(dst, srcs, take, len, dtype, mode, dst != srcs[0], s);
  const void* chunk[kMaxSrcs];
  for (int k = take; rc == 0 && k < n;) {
    int m = std::min(n - k, kMaxSrcs - 1);
    chunk[0] = dst;
    for (int j = 0; j < m; ++j) chunk[1 + j] = srcs[k + j];
    rc = fold_once(dst, chunk, m + 1, len, dtype, mode, false, s);
    k += m;
  }
  return rc;
}

int byteps_reduce_sum_batched(const byteps_bucket_desc* buckets, int nbuckets, int dtype,
                              int mode, void* stream) {
  // the calling thread's staging ring (pinned table + device copy, reused
  // once the kernel that read a slot has completed)
  return batched_with_ring(buckets, nbuckets, dtype, mode, to_stream(stream), &g_ring);
}

struct byteps_reduce_plan {
  int device;
  int dtype;
  int mode;
  void* dev_table;
  TableInfo ti;
};

int byteps_reduce_plan_create(const byteps_bucket_desc* buckets, int nbuckets, int dtype,
                              int mode, byteps_reduce_plan** out) {
  if (!out) return fail(BYTEPS_REDUCE_EARGS, "null plan out-pointer");
  *out = nullptr;
  int rc = check_common(dtype, mode);
  if (rc) return rc;
  if (nbuckets < 0 || (nbuckets > 0 && !buckets))
    return fail(BYTEPS_REDUCE_EARGS, "bad bucket table");
  std::vector<char> host;
  TableInfo ti;
  if ((rc = build_table(buckets, nbuckets, dtype, host, &ti))) return rc;
  auto* p = new byteps_reduce_plan();
  p->dtype = dtype;
  p->mode = mode;
  p->ti = ti;
  p->dev_table = nullptr;
  hipError_t e = hipGetDevice(&p->device);
  if (e == hipSuccess && ti.tiles > 0) {
    e = hipMalloc(&p->dev_table, ti.bytes);
    if (e == hipSuccess)
      e = hipMemcpy(p->dev_table, host.data(), ti.bytes, hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    if (p->dev_table) (void)hipFree(p->dev_table);
    delete p;
    return hip_fail(e, "plan table upload");
  }
  *out = p;
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_plan_launch(byteps_reduce_plan* p, void* stream) {
  if (!p) return fail(BYTEPS_REDUCE_EARGS, "null plan");
  if (p->ti.tiles == 0) return BYTEPS_REDUCE_OK;
  hipError_t e = launch_batched(batch_launch(p->dev_table, p->ti), p->ti.vpt, p->dtype, p->mode,
                                tuning_for_n(p->ti.nmax), to_stream(stream));
  return e == hipSuccess ? BYTEPS_REDUCE_OK : hip_fail(e, "plan kernel launch");
}

int byteps_reduce_plan_destroy(byteps_reduce_plan* p) {
  if (!p) return BYTEPS_REDUCE_OK;
  hipError_t e = hipSuccess;
  if (p->dev_table) e = hipFree(p->dev_table);
  delete p;
  return e == hipSuccess ? BYTEPS_REDUCE_OK : hip_fail(e, "plan free");
}

// ------------------------------------------------------------ block queue --
struct byteps_reduce_blockq {
  int device = 0;
  int dtype = 0;
  int mode = 0;
  int nblocks = 0;
  int occ = 0;               // 0: dispatch-ordered; > 0: persistent workgroups per CU
  int gate_occ = 2;          // dispatch-ordered: resident workgroups per CU, at most
  int cus = 0;
  double timeout_s = 2.0;
  uint64_t clock_khz = 0;    // wall_clock64() rate
  void* dev_table = nullptr; // BatchEntry table + tile records
  uint32_t* flags = nullptr; // [nblocks] release words, then [nblocks + 1] block_first
  BlockqCtl* ctl = nullptr;
  uint32_t* host_err = nullptr;  // pinned word for blockq_status
  TableInfo ti;
  // Epochs (host call order): launch k consumes epoch k; the k-th release of
  // block b carries epoch k.  Guarded: launches and releases may come from
  // different threads (a transport's receive threads release blocks).
  std::mutex mu;
  uint32_t launch_epoch = 0;
  std::vector<uint32_t> rel_epoch;  // per block: epoch of its latest release
  std::vector<char> host_table;     // what was uploaded (byteps_reduce_blockq_debug)
  // The consumer runs on the device's consumer stream (an explicit all-CU
  // mask: the runtime gives such a stream a hardware queue of its own),
  // forked from and joined into the caller's stream unless the caller
  // launches on that stream itself.  A live release must never sit behind
  // the spinning consumer in a shared in-order hardware queue, and stream
  // priority alone does not guarantee separate queues (measured: torch's
  // pooled high- and normal-priority streams shared one for some pool
  // indices, tools/pushloop_diag.py).
  bool own_queue = true;
  // Overlap (byteps_reduce_blockq_overlap): launches
  // alternate between the device's two consumer queues and do not join back.
  bool overlap = false;
  hipEvent_t fork_ev = nullptr;
  // Deferred join-back (round 6, DESIGN.md §4.4 "false dependencies"): a
  // launch forked from the caller's stream `s` (no overlap) makes `s` wait
  // for its consumer only once every block of its epoch has been released
  // (or at join / status).  A wait queued on `s` at launch time sits in the
  // in-order hardware queue `s` shares with other streams, and a release (or
  // the copies before it) queued on one of those streams would then wait
  // behind the very consumer it releases: a stall until the timeout (r05s76,
  // measured r06s02).  Each such launch completes an event of its own.
  struct PendingJoin {
    hipStream_t s;
    hipEvent_t ev;
    uint32_t epoch;
  };
  std::vector<PendingJoin> pend_join;  // under mu
  std::vector<hipEvent_t> join_evs;    // free events (under mu)
  // Host releases (byteps_reduce_blockq_host_releases): pinned, coherent
  // words the host writes and the launch's helper workgroup forwards.
  uint32_t* hflags = nullptr;
  uint32_t* hflags_dev = nullptr;
  bool host_rel = false;
  // Keyed queue (bpsr::keyq_*, the PS server's device releases): one block
  // per key, (arrival order << 32 | epoch) words, the control word in pinned
  // host memory so the server reads a timeout without a copy.
  bool keyed = false;
  bool wide = false;                // 9..16 sources: a second word per block (positions 8..15)
  uint64_t* kwords = nullptr;       // device, one per block [+ the second words after them]
  uint64_t* khwords = nullptr;      // pinned host, two per block (epoch parity) [+ second words]
  uint64_t* khwords_dev = nullptr;
  BlockqCtl* hctl = nullptr;        // pinned host
  BlockqCtl* hctl_dev = nullptr;
  uint32_t* kcnt = nullptr;         // device, one tile counter per block
  uint32_t* khdone = nullptr;       // pinned host, one completion word per block
  uint32_t* khdone_dev = nullptr;
  uint32_t opened = 0;              // highest epoch a round was released for (keyq_opened)
#ifdef BPSR_KEYED_TRACE
  unsigned long long* ktrace = nullptr;  // probe builds: kKtraceSlots launches' stamps
  size_t ktrace_per = 0;
#endif
};
#ifdef BPSR_KEYED_TRACE
constexpr uint32_t kKtraceSlots = 64;
#endif

// Per device, created on first use, never destroyed: three consumer queues
// (all-CU-masked streams, each a hardware queue of its own; queue 0 is
// byteps_reduce_blockq_stream, where every launch without overlap runs, in
// launch order; queue 1 the overlapped launches' second queue; queue 2 the
// PS server's keyed consumers, so that a block-queue join never waits for a
// keyed epoch that waits for host releases) and the dispatch sequence every block-queue launch outside a
// capture takes part in: sequence numbers, the
// started-workgroup counter and its target, the signal word, the stream of the
// latest launch, and per stream the completion event of its latest launch
// (what byteps_reduce_blockq_join waits for).
struct ConsumerDev {
  std::mutex mu;                        // sequence order = enqueue order
  hipStream_t q[3] = {nullptr, nullptr, nullptr};
  // Placement (round 6, DESIGN.md §4.4 "pipes"): the HSA ids of the consumer
  // queues and of the release queue (byteps_reduce_blockq_release_stream),
  // and queues made while placing them that did not fit (kept, idle: a
  // destroyed queue would reshuffle the hardware's queue map).
  uint64_t qid[3] = {0, 0, 0};
  hipStream_t rq = nullptr;
  uint64_t rqid = 0;

  std::vector<std::pair<hipStream_t, uint64_t>> spare;
  uint64_t* idw = nullptr;              // pinned word read_queue_id writes (host view)
  uint64_t* idw_dev = nullptr;          // ... its device view
  unsigned long long* started = nullptr;  // started counter (device, a line of its own)
  unsigned long long target = 0;        // counted workgroups of every launch so far
  hipStream_t last = nullptr;           // stream of the latest launch
  bool any = false;                     // a launch is in the sequence
  struct Tail {
    hipStream_t stream;
    hipEvent_t ev;
    bool record;  // the latest launch there carried no stop event: join records one
  };
  std::vector<Tail> tails;
};
static std::mutex g_consumer_mu;
static ConsumerDev g_cdev[64];

// Queue placement (DESIGN.md §4.4 "pipes", round 6).  The hardware serves
// its queues through 4 compute pipes, and queue ids map to pipes as id mod 4
// in every measurement (profiles/r06s01, r06s02, r06s05, r06s07).  A queue on
// the same pipe as a running consumer answers ~2x slower (43 us median
// release kernels instead of 5: the r05s34 segment); the two overlapping
// consumer queues need pipes of their own (on one pipe, overlapped config 3
// fell from 0.80 to 0.74-0.75, r06s07); and the runtime's own normal-priority
// queues serve the server's lanes best one per pipe (the host-resident
// server ran 4.2 ms rounds instead of 3.1 when the library's queues had
// pushed two of them onto one pipe, r06s08-s09).  So the library makes its
// four queues together, one per pipe: consumer queues 0 and 1, the keyed
// consumers' queue 2 and the release queue — its releases never share a pipe
// with a block-queue consumer, and queues made later keep the runtime's
// phase.  If another thread made a queue in between (ids not consecutive),
// the set is completed queue by queue; a queue that does not fit is kept
// idle for a later placement (a destroyed one could reshuffle the hardware's
// queue map).
constexpr uint64_t kPipes = 4;

// g_consumer_mu held, device current.  A new all-CU-masked stream (a hardware
// queue of its own) and the HSA id of its queue.
static hipError_t new_cu_queue(ConsumerDev& D, int cus, hipStream_t* out, uint64_t* id) {
  std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
  for (int c = 0; c < cus; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
  hipError_t e = hipSuccess;
  if (!D.idw) {
    e = hipHostMalloc(reinterpret_cast<void**>(&D.idw), 64,
                      hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&D.idw_dev), D.idw, 0);
    if (e != hipSuccess) return e;
  }
  e = hipExtStreamCreateWithCUMask(out, (uint32_t)mask.size(), mask.data());
  if (e == hipSuccess) e = read_queue_id(*out, D.idw_dev);
  if (e == hipSuccess) *id = __atomic_load_n(D.idw, __ATOMIC_ACQUIRE);
  return e;
}

// g_consumer_mu held, device current.  A queue whose id satisfies `fits`:
// an idle spare, or a new one (at most kPipes + 1 tries; the last one made
// is taken if none fits, i.e. the id-to-pipe model did not hold).
extern "C++" template <class Fits>
static hipError_t placed_queue(ConsumerDev& D, int cus, Fits fits, hipStream_t* out, uint64_t* id) {
  for (size_t i = 0; i < D.spare.size(); ++i)
    if (fits(D.spare[i].second)) {
      *out = D.spare[i].first;
      *id = D.spare[i].second;
      D.spare.erase(D.spare.begin() + (long)i);
      return hipSuccess;
    }
  for (uint64_t t = 0;; ++t) {
    hipStream_t s = nullptr;
    uint64_t qid = 0;
    const hipError_t e = new_cu_queue(D, cus, &s, &qid);
    if (e != hipSuccess) return e;
    if (fits(qid) || t == kPipes) {
      *out = s;
      *id = qid;
      return hipSuccess;
    }
    D.spare.push_back({s, qid});
  }
}

// At process exit, before the HIP runtime's own teardown (the handler is
// registered after the runtime is up, and exit handlers run in reverse):
// the library's queues are destroyed like any other stream, not left to the
// runtime's teardown — under rocprofv3 a process holding them at exit faulted
// inside the profiler's own finalizer (profiles/r06s06_exit_fault_frames.txt).
static void destroy_queue_sets() {
  std::lock_guard<std::mutex> g(g_consumer_mu);
  for (auto& D : g_cdev) {
    for (auto& q : D.q)
      if (q) (void)hipStreamDestroy(q), q = nullptr;
    if (D.rq) (void)hipStreamDestroy(D.rq), D.rq = nullptr;
    for (auto& sp : D.spare) (void)hipStreamDestroy(sp.first);
    D.spare.clear();
  }
}

// The device's four library queues, made together on first use (above):
// slots 0-2 the consumer queues, slot 3 the release queue.
static hipError_t queue_set(int device, int cus, ConsumerDev** out) {
  if (device < 0 || device >= 64) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> g(g_consumer_mu);
  ConsumerDev& D = g_cdev[device];
  *out = &D;
  if (D.rq) return hipSuccess;
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (cur != device) (void)hipSetDevice(device);
  hipStream_t* slot[4] = {&D.q[0], &D.q[1], &D.q[2], &D.rq};
  uint64_t* sid[4] = {&D.qid[0], &D.qid[1], &D.qid[2], &D.rqid};
  hipError_t e = hipSuccess;
  for (int k = 0; k < 4 && e == hipSuccess; ++k) e = new_cu_queue(D, cus, slot[k], sid[k]);
  // any queue whose pipe an earlier one of the set has: re-placed
  for (int k = 1; k < 4 && e == hipSuccess; ++k) {
    auto taken = [&](uint64_t id) {
      for (int j = 0; j < k; ++j)
        if (*sid[j] % kPipes == id % kPipes) return true;
      return false;
    };
    if (!taken(*sid[k])) continue;
    D.spare.push_back({*slot[k], *sid[k]});
    e = placed_queue(D, cus, [&](uint64_t id) { return !taken(id); }, slot[k], sid[k]);
  }
  if (cur != device && cur >= 0) (void)hipSetDevice(cur);
  if (e != hipSuccess) {
    for (int k = 0; k < 4; ++k) *slot[k] = nullptr;
    return e;
  }
  static bool registered = false;
  if (!registered) registered = std::atexit(destroy_queue_sets) == 0;
  return hipSuccess;
}

// which: 0 (every launch without overlap), 1 (the overlapped launches'
// second queue) or 2 (keyed consumers).
static hipError_t consumer_queue(int device, int cus, int which, hipStream_t* out) {
  ConsumerDev* D = nullptr;
  const hipError_t e = queue_set(device, cus, &D);
  if (e == hipSuccess) *out = D->q[which];
  return e;
}

// The device's release queue: a hardware queue on a pipe no consumer queue
// uses.
static hipError_t release_queue(int device, int cus, hipStream_t* out) {
  ConsumerDev* D = nullptr;
  const hipError_t e = queue_set(device, cus, &D);
  if (e == hipSuccess) *out = D->rq;
  return e;
}

static hipError_t consumer_stream(int device, int cus, hipStream_t* out) {
  return consumer_queue(device, cus, 0, out);
}

// D.mu held.  The started counters, once per device.
static hipError_t seq_init(ConsumerDev& D, int device) {
  if (D.started) return hipSuccess;
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (cur != device) (void)hipSetDevice(device);
  const size_t bytes = 256;
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, bytes);
  if (e == hipSuccess) e = hipMemset(p, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (cur != device && cur >= 0) (void)hipSetDevice(cur);
  if (e != hipSuccess) {
    if (p) (void)hipFree(p);
    return e;
  }
  D.started = static_cast<unsigned long long*>(p);
  return hipSuccess;
}

// D.mu held.  The join entry of stream `s`: its event completes with the
// latest launch on `s` (the launch's stop event), or is recorded on `s` by
// the next join when that launch carried none (a stop event is an
// end-of-kernel release: ~5 µs when another kernel follows on its stream,
// ~2.4 µs of an overlapped iteration; r05s22-23).
static hipError_t seq_tail(ConsumerDev& D, hipStream_t s, ConsumerDev::Tail** out) {
  for (auto& t : D.tails)
    if (t.stream == s) {
      *out = &t;
      return hipSuccess;
    }
  // Callers' streams (launches without a queue of their own) come and go:
  // drop entries whose launch has completed and that need no record, so the
  // list stays bounded by the launches still in flight.
  if (D.tails.size() >= 16) {
    size_t k = 0;
    for (auto& t : D.tails) {
      const bool own = t.stream == D.q[0] || t.stream == D.q[1] || t.stream == D.q[2];
      if (!own && !t.record && hipEventQuery(t.ev) == hipSuccess) {
        (void)hipEventDestroy(t.ev);
        continue;
      }
      D.tails[k++] = t;
    }
    D.tails.resize(k);
  }
  hipEvent_t e = nullptr;
  const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
  if (r != hipSuccess) return r;
  D.tails.push_back({s, e, false});
  *out = &D.tails.back();
  return hipSuccess;
}

// D.mu held; before enqueueing the kernel of a launch on `ls`: put it in the
// sequence and, when the device's previous launch went to another stream,
// gate `ls` until every workgroup launched so far has started (the gate
// gives up after gate_ticks).
static hipError_t seq_prepare(ConsumerDev& D, int device, BlockqLaunch& Q, hipStream_t ls,
                              uint64_t gate_ticks) {
  hipError_t e = seq_init(D, device);
  if (e != hipSuccess) return e;
  if (D.any && D.last != ls) e = launch_seq_gate(D.started, D.target, gate_ticks, ls);
  Q.started = D.started;
  return e;
}

// D.mu held; after the kernel was enqueued.
static void seq_commit(ConsumerDev& D, const BlockqLaunch& Q, hipStream_t ls) {
  if (!Q.started) return;
  D.target += seq_counted(Q.grid);
  D.last = ls;
  D.any = true;
}

// q->mu held.  Every block released for `epoch` (host call order).
static bool epoch_released(const byteps_reduce_blockq* q, uint32_t epoch) {
  for (uint32_t r : q->rel_epoch)
    if (!epoch_reached(r, epoch)) return false;
  return true;
}

// q->mu held.  Issue the deferred join-backs whose epochs are fully released
// (all of them when `all`): the caller's stream waits for that launch.
static hipError_t flush_joins(byteps_reduce_blockq* q, bool all) {
  hipError_t e = hipSuccess;
  size_t k = 0;
  for (auto& p : q->pend_join) {
    if (e == hipSuccess && (all || epoch_released(q, p.epoch))) {
      e = hipStreamWaitEvent(p.s, p.ev, 0);
      q->join_evs.push_back(p.ev);  // the wait holds the event's state at this call
      continue;
    }
    q->pend_join[k++] = p;
  }
  q->pend_join.resize(k);
  return e;
}

#ifdef BPSR_KEYED_TRACE
// Probe builds: the keyed consumer's stamps to $BPSR_KEYED_TRACE_OUT — a
// header (launch epoch, slots, words per slot, tiles, keys, clock kHz), the
// tiles' first records (block_first), then the slots.
static void dump_ktrace(byteps_reduce_blockq* q) {
  const char* path = getenv("BPSR_KEYED_TRACE_OUT");
  if (!q->ktrace || !path) return;
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> buf(q->ktrace_per * kKtraceSlots);
  std::vector<uint32_t> bf((size_t)q->nblocks + 1);
  if (hipMemcpy(buf.data(), q->ktrace, 8 * buf.size(), hipMemcpyDeviceToHost) != hipSuccess) return;
  if (hipMemcpy(bf.data(), q->flags + q->nblocks, 4 * bf.size(), hipMemcpyDeviceToHost) != hipSuccess)
    return;
  FILE* f = fopen(path, "wb");
  if (!f) return;
  const unsigned long long hdr[6] = {q->launch_epoch, kKtraceSlots, q->ktrace_per, q->ti.tiles,
                                     (unsigned long long)q->nblocks, q->clock_khz};
  fwrite(hdr, 8, 6, f);
  fwrite(bf.data(), 4, bf.size(), f);
  fwrite(buf.data(), 8, buf.size(), f);
  fclose(f);
}
#endif

static void blockq_free(byteps_reduce_blockq* q) {
#ifdef BPSR_KEYED_TRACE
  dump_ktrace(q);
  if (q->ktrace) (void)hipFree(q->ktrace);
#endif
  // a launch still waiting for releases ends at its timeout at the latest
  for (auto& p : q->pend_join) {
    (void)hipEventSynchronize(p.ev);
    (void)hipEventDestroy(p.ev);
  }
  for (hipEvent_t ev : q->join_evs) (void)hipEventDestroy(ev);
  if (q->kwords) (void)hipFree(q->kwords);
  if (q->khwords) (void)hipHostFree(q->khwords);
  if (q->hctl) (void)hipHostFree(q->hctl);
  if (q->kcnt) (void)hipFree(q->kcnt);
  if (q->khdone) (void)hipHostFree(q->khdone);
  if (q->fork_ev) (void)hipEventDestroy(q->fork_ev);
  if (q->dev_table) (void)hipFree(q->dev_table);
  if (q->flags) (void)hipFree(q->flags);
  if (q->ctl) (void)hipFree(q->ctl);
  if (q->host_err) (void)hipHostFree(q->host_err);
  if (q->hflags) (void)hipHostFree(q->hflags);
  delete q;
}

int byteps_reduce_blockq_create(const byteps_bucket_desc* buckets, int nbuckets,
                                const int* block_end, int nblocks, int dtype, int mode,
                                byteps_reduce_blockq** out) {
  if (!out) return fail(BYTEPS_REDUCE_EARGS, "null block-queue out-pointer");
  *out = nullptr;
  int rc = check_common(dtype, mode);
  if (rc) return rc;
  if (nbuckets < 0 || (nbuckets > 0 && !buckets))
    return fail(BYTEPS_REDUCE_EARGS, "bad bucket table");
  if (nblocks < 1 || !block_end) return fail(BYTEPS_REDUCE_EARGS, "need >= 1 block");
  for (int k = 0; k < nblocks; ++k) {
    const int lo = k ? block_end[k - 1] : 0;
    if (block_end[k] < lo || block_end[k] > nbuckets)
      return fail(BYTEPS_REDUCE_EARGS, "block_end[%d]=%d not in [%d, %d]", k, block_end[k], lo,
                  nbuckets);
  }
  if (block_end[nblocks - 1] != nbuckets)
    return fail(BYTEPS_REDUCE_EARGS, "last block ends at %d, not at nbuckets=%d",
                block_end[nblocks - 1], nbuckets);
  std::vector<char> host;
  std::vector<uint32_t> first;
  TableInfo ti;
  int gate_occ = 2;
  if (const char* v = getenv("BPSR_BQ_GATE_OCC")) gate_occ = atoi(v);
  if (gate_occ < 1 || gate_occ > 8) gate_occ = 2;
  int force_vpt = 0;  // tile size override for measurements (default: the fold rule)
  if (const char* v = getenv("BPSR_BQ_VPT")) force_vpt = atoi(v);
  if (force_vpt != 1 && force_vpt != 2 && force_vpt != 4) force_vpt = 0;
  if ((rc = build_table(buckets, nbuckets, dtype, host, &ti, block_end, nblocks, &first,
                        force_vpt)))
    return rc;
  auto* q = new byteps_reduce_blockq();
  q->dtype = dtype;
  q->mode = mode;
  q->nblocks = nblocks;
  q->gate_occ = gate_occ;
  q->ti = ti;
  q->rel_epoch.assign((size_t)nblocks, 0u);
  q->host_table = host;
  if (const char* v = getenv("BPSR_BQ_OWN_QUEUE")) q->own_queue = atoi(v) != 0;
  int khz = 0;
  hipError_t e = hipGetDevice(&q->device);
  if (e == hipSuccess)
    e = hipDeviceGetAttribute(&q->cus, hipDeviceAttributeMultiprocessorCount, q->device);
  if (e == hipSuccess)
    e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, q->device);
  q->clock_khz = khz > 0 ? (uint64_t)khz : 100000;
  // The release words and the control word get allocations of their own,
  // padded to whole 256-B lines: nothing else may share their cache lines.
  const size_t flag_bytes =
      (sizeof(uint32_t) * (2 * (size_t)nblocks + 1) + 255) & ~(size_t)255;
  if (e == hipSuccess && ti.tiles > 0) e = hipMalloc(&q->dev_table, ti.bytes);
  if (e == hipSuccess && ti.tiles > 0)
    e = hipMemcpy(q->dev_table, host.data(), ti.bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&q->flags), flag_bytes);
  if (e == hipSuccess) e = hipMemset(q->flags, 0, sizeof(uint32_t) * nblocks);
  if (e == hipSuccess)
    e = hipMemcpy(q->flags + nblocks, first.data(), sizeof(uint32_t) * (nblocks + 1),
                  hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&q->ctl), 256);
  if (e == hipSuccess) e = hipMemset(q->ctl, 0, 256);
  if (e == hipSuccess) e = hipDeviceSynchronize();  // words zeroed before any stream uses them
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void**>(&q->host_err), sizeof(uint32_t));
  if (e != hipSuccess) {
    blockq_free(q);
    return hip_fail(e, "block queue setup");
  }
  *out = q;
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_blockq_config(byteps_reduce_blockq* q, int wg_per_cu, double timeout_s) {
  if (!q) return fail(BYTEPS_REDUCE_EARGS, "null block queue");
  if (q->keyed && wg_per_cu > 0)
    return fail(BYTEPS_REDUCE_EARGS, "a keyed queue has the dispatch-ordered consumer");
  if (wg_per_cu > 8) return fail(BYTEPS_REDUCE_EARGS, "wg_per_cu %d > 8", wg_per_cu);
  if (wg_per_cu > 0 && q->host_rel)
    return fail(BYTEPS_REDUCE_EARGS, "host releases need the dispatch-ordered consumer");
  if (wg_per_cu > 0 && q->overlap)
    return fail(BYTEPS_REDUCE_EARGS, "overlap needs the dispatch-ordered consumer");
  if (wg_per_cu >= 0) q->occ = wg_per_cu;
  if (timeout_s > 0) q->timeout_s = timeout_s;
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_blockq_launch(byteps_reduce_blockq* q, void* stream) {
  if (!q) return fail(BYTEPS_REDUCE_EARGS, "null block queue");
  hipStream_t s = to_stream(stream);
  std::lock_guard<std::mutex> g(q->mu);
  const uint32_t epoch = q->launch_epoch + 1;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusActive) {
    // Host releases write only the pinned words; the helper workgroup that
    // forwards them is left out of a captured launch, so such a launch would
    // wait for its timeout on every replay.
    if (q->host_rel)
      return fail(BYTEPS_REDUCE_EARGS, "captured block-queue launch with host releases on "
                                       "(byteps_reduce_blockq_host_releases(q, 0) first)");
    // A captured launch keeps this epoch in every replay: only iterations
    // whose releases are captured before it (same graph, stream order) replay
    // correctly, so that is what a capture must hold.
    for (int b = 0; b < q->nblocks; ++b)
      if (!epoch_reached(q->rel_epoch[b], epoch))
        return fail(BYTEPS_REDUCE_EARGS,
                    "captured block-queue launch: release every block before the launch "
                    "(block %d is not; epochs are fixed at capture)", b);
  }
  q->launch_epoch = epoch;
  if (q->ti.tiles == 0) return BYTEPS_REDUCE_OK;
  BlockqLaunch Q;
  Q.L = batch_launch(q->dev_table, q->ti);
  Q.flags = q->flags;
  Q.block_first = q->flags + q->nblocks;
  Q.ctl = q->ctl;
  Q.nblocks = (uint32_t)q->nblocks;
  Q.timeout_ticks = (uint64_t)(q->timeout_s * 1e3 * (double)q->clock_khz);
  Q.epoch = epoch;
  Q.helper = 0;
  Q.hflags = nullptr;
  Q.keyed = 0;
  Q.wide = 0;
  Q.kwords = nullptr;
  Q.khwords = nullptr;
  Q.kcnt = nullptr;
  Q.khdone = nullptr;
  Q.herr = nullptr;
  const Tuning tu = tuning_for_n(q->ti.nmax);
  const bool gated = q->occ == 0;
  size_t lds;
  if (gated) {
    // One workgroup per tile.  Residency is capped (LDS) so that workgroups
    // spinning on a release never take a CU's last registers: the release
    // kernels and the copies that precede them must still get onto the CU
    // (at hardware occupancy — 3 of these workgroups per CU — a live release
    // behind H2D copies on another stream never arrived).
    Q.grid = q->ti.tiles;
    if (q->host_rel && cap != hipStreamCaptureStatusActive) {
      Q.helper = 1;  // workgroup 0 forwards host releases (forward_host_releases)
      Q.hflags = q->hflags_dev;
      Q.grid += 1;
    }
    int occ = launch_occ(tu, q->ti.tiles, true);
    if (occ == 0 || occ > q->gate_occ) occ = q->gate_occ;
    lds = occ_lds_bytes(occ);
  } else {
    const uint64_t cap = (uint64_t)q->cus * (uint64_t)q->occ;
    Q.grid = (uint32_t)std::min<uint64_t>(q->ti.tiles, cap);
    // residency cap through LDS (the kernel's own static LDS included)
    lds = ((kLdsPerCU / (size_t)q->occ) - 256) & ~(size_t)255;
  }
  const int pol = cache_pol(tu, (uint64_t)q->ti.tiles * q->ti.vpt * kBlock * 16);
  Q.started = nullptr;
  if (cap == hipStreamCaptureStatusActive) {
    // pre-released by rule: runs on the capturing stream, outside the sequence
    const hipError_t e = launch_blockq(Q, q->ti.vpt, pol, lds, gated, q->dtype, q->mode, s);
    return e == hipSuccess ? BYTEPS_REDUCE_OK : hip_fail(e, "block queue kernel launch");
  }
  // The consumer runs on a consumer queue of the device (a hardware queue of
  // its own), forked from `s`; without overlap it runs on queue 0 and joins
  // back into `s`, with overlap it takes the queue the device's previous
  // launch did not and does not join (byteps_reduce_blockq_join).
  if (q->device < 0 || q->device >= 64) return fail(BYTEPS_REDUCE_EARGS, "device %d", q->device);
  ConsumerDev& D = g_cdev[q->device];
  hipStream_t c0 = nullptr, c1 = nullptr;
  hipError_t e = hipSuccess;
  if (q->own_queue) e = consumer_queue(q->device, q->cus, 0, &c0);
  if (e == hipSuccess && q->own_queue && q->overlap) e = consumer_queue(q->device, q->cus, 1, &c1);
  if (e != hipSuccess) return hip_fail(e, "consumer stream");
  std::lock_guard<std::mutex> dg(D.mu);
  hipStream_t ls = s;
  if (q->own_queue) ls = q->overlap && D.last == c0 ? c1 : c0;
  const bool fork = q->own_queue && s != ls && (!q->overlap || (s != c0 && s != c1));
  if (fork) {
    if (!q->fork_ev) e = hipEventCreateWithFlags(&q->fork_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(q->fork_ev, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(ls, q->fork_ev, 0);
  }
  // The consumer's own completion completes the join event when `s` joins
  // back at once, or when the launch stream is the caller's (a join must not
  // record on a stream the caller may have destroyed since); otherwise the
  // next byteps_reduce_blockq_join records it on the consumer queue (a stop
  // event on every overlapped launch cost 2.4 µs per config-3 iteration:
  // 0.0744 vs 0.0720 ms, r05s23).
  // A launch forked from `s` without overlap joins back into `s` once its
  // epoch is fully released (flush_joins), through a stop event of its own.
  ConsumerDev::Tail* tail = nullptr;
  if (e == hipSuccess) e = seq_tail(D, ls, &tail);
  const bool join_back = q->own_queue && !q->overlap && s != ls;
  hipEvent_t jev = nullptr;
  if (e == hipSuccess && join_back) {
    if (!q->join_evs.empty()) {
      jev = q->join_evs.back();
      q->join_evs.pop_back();
    } else {
      e = hipEventCreateWithFlags(&jev, hipEventDisableTiming);
    }
  }
  if (e == hipSuccess) {
    const bool stop = !q->own_queue;
    Q.L.stop = join_back ? jev : stop ? tail->ev : nullptr;
    tail->record = !stop;
  }
  if (e == hipSuccess) e = seq_prepare(D, q->device, Q, ls, 4 * Q.timeout_ticks);
  if (e == hipSuccess) e = launch_blockq(Q, q->ti.vpt, pol, lds, gated, q->dtype, q->mode, ls);
  if (e == hipSuccess) seq_commit(D, Q, ls);
  if (e == hipSuccess && join_back) {
    q->pend_join.push_back({s, jev, epoch});
    e = flush_joins(q, false);  // a pre-released epoch joins at once
  } else if (jev) {
    q->join_evs.push_back(jev);
  }
  return e == hipSuccess ? BYTEPS_REDUCE_OK : hip_fail(e, "block queue kernel launch");
}

int byteps_reduce_blockq_overlap(byteps_reduce_blockq* q, int on) {
  if (!q) return fail(BYTEPS_REDUCE_EARGS, "null block queue");
  std::lock_guard<std::mutex> g(q->mu);
  if (!on) {
    q->overlap = false;
    return BYTEPS_REDUCE_OK;
  }
  if (q->keyed || q->occ != 0)
    return fail(BYTEPS_REDUCE_EARGS, "overlap needs the dispatch-ordered consumer "
                                     "(byteps_reduce_blockq_config wg_per_cu = 0)");
  if (q->device < 0 || q->device >= 64) return fail(BYTEPS_REDUCE_EARGS, "device %d", q->device);
  q->overlap = true;
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_blockq_join(byteps_reduce_blockq* q, void* stream) {
  if (!q) return fail(BYTEPS_REDUCE_EARGS, "null block queue");
  if (q->device < 0 || q->device >= 64) return fail(BYTEPS_REDUCE_EARGS, "device %d", q->device);
  hipStream_t s = to_stream(stream);
  std::lock_guard<std::mutex> g(q->mu);  // (q->mu before D.mu, as in launch)
  if (const hipError_t e = flush_joins(q, true)) return hip_fail(e, "block queue join-back");
  ConsumerDev& D = g_cdev[q->device];
  std::lock_guard<std::mutex> dg(D.mu);
  for (auto& t : D.tails) {
    if (t.stream == s) continue;
    hipError_t e = hipSuccess;
    if (t.record) e = hipEventRecord(t.ev, t.stream);
    t.record = false;
    if (e == hipSuccess) e = hipStreamWaitEvent(s, t.ev, 0);
    if (e != hipSuccess) return hip_fail(e, "block queue join");
  }
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_blockq_release_range(byteps_reduce_blockq* q, int first, int count,
                                       void* stream) {
  if (!q) return fail(BYTEPS_REDUCE_EARGS, "null block queue");
  if (first < 0 || count < 0 || first > q->nblocks || count > q->nblocks - first)
    return fail(BYTEPS_REDUCE_EARGS, "blocks [%d, %d+%d) outside [0, %d)", first, first, count,
                q->nblocks);
  hipStream_t s = to_stream(stream);
  std::lock_guard<std::mutex> g(q->mu);
  // Each block's release carries its own next epoch; a range whose blocks are
  // at different epochs (a block released ahead) goes out as one kernel per
  // run of equal epochs.  A one-wave kernel raises the words at system scope:
  // a hipMemset node was not seen by the consumer's polls under graph replay,
  // and hipStreamWriteValue32, copy-engine copies, host functions and events
  // measured no better for per-block releases.
  int b = first;
  const int end = first + count;
  while (b < end) {
    const uint32_t ep = q->rel_epoch[b] + 1;
    int run = b + 1;
    while (run < end && q->rel_epoch[run] + 1 == ep) ++run;
    const hipError_t e = launch_blockq_release(q->flags, (uint32_t)b, (uint32_t)(run - b), ep, s);
    if (e != hipSuccess) return hip_fail(e, "block release");
    for (int k = b; k < run; ++k) q->rel_epoch[k] = ep;
    b = run;
  }
  if (!q->pend_join.empty()) {
    const hipError_t e = flush_joins(q, false);
    if (e != hipSuccess) return hip_fail(e, "block queue join-back");
  }
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_blockq_host_releases(byteps_reduce_blockq* q, int on) {
  if (!q) return fail(BYTEPS_REDUCE_EARGS, "null block queue");
  std::lock_guard<std::mutex> g(q->mu);
  if (!on) {
    q->host_rel = false;
    return BYTEPS_REDUCE_OK;
  }
  if (q->occ != 0)
    return fail(BYTEPS_REDUCE_EARGS, "host releases need the dispatch-ordered consumer "
                                     "(byteps_reduce_blockq_config wg_per_cu = 0)");
  if (!q->hflags) {
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, sizeof(uint32_t) * (size_t)q->nblocks,
                                 hipHostMallocCoherent | hipHostMallocMapped);
    if (e != hipSuccess) return hip_fail(e, "hipHostMalloc(host release words)");
    void* d = nullptr;
    e = hipHostGetDevicePointer(&d, p, 0);
    if (e != hipSuccess) {
      (void)hipHostFree(p);
      return hip_fail(e, "hipHostGetDevicePointer(host release words)");
    }
    q->hflags = static_cast<uint32_t*>(p);
    q->hflags_dev = static_cast<uint32_t*>(d);
    // 0 = never released from the host (the helper skips such words)
    for (int b = 0; b < q->nblocks; ++b)
      __atomic_store_n(q->hflags + b, 0u, __ATOMIC_RELEASE);
  }
  q->host_rel = true;
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_blockq_release_host(byteps_reduce_blockq* q, int first, int count) {
  if (!q) return fail(BYTEPS_REDUCE_EARGS, "null block queue");
  if (first < 0 || count < 0 || first > q->nblocks || count > q->nblocks - first)
    return fail(BYTEPS_REDUCE_EARGS, "blocks [%d, %d+%d) outside [0, %d)", first, first, count,
                q->nblocks);
  std::lock_guard<std::mutex> g(q->mu);
  if (!q->host_rel)
    return fail(BYTEPS_REDUCE_EARGS, "host releases not enabled (byteps_reduce_blockq_host_releases)");
  // Each block's word carries its own next epoch (as release_range); the
  // caller's data is complete before the call, so a release store suffices.
  for (int b = first; b < first + count; ++b) {
    const uint32_t ep = q->rel_epoch[b] + 1;
    q->rel_epoch[b] = ep;
    __atomic_store_n(q->hflags + b, ep, __ATOMIC_RELEASE);
  }
  if (!q->pend_join.empty()) {
    const hipError_t e = flush_joins(q, false);
    if (e != hipSuccess) return hip_fail(e, "block queue join-back");
  }
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_blockq_release(byteps_reduce_blockq* q, int block, void* stream) {
  if (!q) return fail(BYTEPS_REDUCE_EARGS, "null block queue");
  if (block >= q->nblocks) return fail(BYTEPS_REDUCE_EARGS, "block %d >= %d", block, q->nblocks);
  return block < 0 ? byteps_reduce_blockq_release_range(q, 0, q->nblocks, stream)
                   : byteps_reduce_blockq_release_range(q, block, 1, stream);
}

int byteps_reduce_blockq_status(byteps_reduce_blockq* q, void* stream) {
  if (!q) return fail(BYTEPS_REDUCE_EARGS, "null block queue");
  hipStream_t s = to_stream(stream);
  if (q->overlap) {  // launches do not join their stream: the status waits for all of them
    const int rc = byteps_reduce_blockq_join(q, stream);
    if (rc) return rc;
  } else {           // deferred join-backs go out now (their launch streams wait)
    std::lock_guard<std::mutex> g(q->mu);
    if (const hipError_t e = flush_joins(q, true)) return hip_fail(e, "block queue join-back");
  }
  hipError_t e = hipMemcpyAsync(q->host_err, &q->ctl->err, sizeof(uint32_t),
                                hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "block queue status");
  if (*q->host_err == 0) return BYTEPS_REDUCE_OK;
  e = hipMemsetAsync(&q->ctl->err, 0, sizeof(uint32_t), s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "block queue status reset");
  {
    // The abandoned iteration's missing releases will not come: count them as
    // given, so the next iteration's releases carry the next launch's epoch.
    std::lock_guard<std::mutex> g(q->mu);
    for (auto& r : q->rel_epoch)
      if (!epoch_reached(r, q->launch_epoch)) r = q->launch_epoch;
  }
  return fail(BYTEPS_REDUCE_ETIMEOUT,
              "block queue: a block was not released within %.3f s; the launch stopped early",
              q->timeout_s);
}

int byteps_reduce_blockq_stream(byteps_reduce_blockq* q, void** stream) {
  if (!q || !stream) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  hipStream_t s = nullptr;
  hipError_t e = consumer_stream(q->device, q->cus, &s);
  if (e != hipSuccess) return hip_fail(e, "consumer stream");
  *stream = reinterpret_cast<void*>(s);
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_blockq_release_stream(byteps_reduce_blockq* q, void** stream) {
  if (!q || !stream) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  hipStream_t s = nullptr;
  hipError_t e = release_queue(q->device, q->cus, &s);
  if (e != hipSuccess) return hip_fail(e, "release stream");
  *stream = reinterpret_cast<void*>(s);
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_blockq_queue_ids(byteps_reduce_blockq* q, uint64_t* ids, int cap) {
  if (!q || !ids || cap < 4) return fail(BYTEPS_REDUCE_EARGS, "null argument or cap < 4");
  if (q->device < 0 || q->device >= 64) return fail(BYTEPS_REDUCE_EARGS, "device %d", q->device);
  std::lock_guard<std::mutex> g(g_consumer_mu);
  const ConsumerDev& D = g_cdev[q->device];
  for (int k = 0; k < 3; ++k) ids[k] = D.q[k] ? D.qid[k] : 0;
  ids[3] = D.rq ? D.rqid : 0;
  return 4;
}

int byteps_reduce_blockq_debug(byteps_reduce_blockq* q, uint32_t* out, int cap) {
  if (!q || !out) return fail(BYTEPS_REDUCE_EARGS, "null argument");
  const int nb = q->nblocks;
  const int need = 3 + 3 * nb + 1;
  if (cap < need) return fail(BYTEPS_REDUCE_EARGS, "cap %d < %d", cap, need);
  hipError_t e = hipDeviceSynchronize();
  std::vector<uint32_t> dev(2 * (size_t)nb + 1);
  if (e == hipSuccess) e = hipMemcpy(dev.data(), q->flags, dev.size() * 4, hipMemcpyDeviceToHost);
  uint32_t err = 0;
  if (e == hipSuccess) e = hipMemcpy(&err, &q->ctl->err, 4, hipMemcpyDeviceToHost);
  std::vector<char> tab(q->host_table.size());
  if (e == hipSuccess && !tab.empty())
    e = hipMemcpy(tab.data(), q->dev_table, tab.size(), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail(e, "blockq debug");
  std::lock_guard<std::mutex> g(q->mu);
  int k = 0;
  out[k++] = q->launch_epoch;
  out[k++] = (uint32_t)nb;
  out[k++] = err;
  for (int b = 0; b < nb; ++b) out[k++] = q->rel_epoch[b];
  for (size_t i = 0; i < dev.size(); ++i) out[k++] = dev[i];   // words, then block_first
  out[k++] = tab == q->host_table ? 1u : 0u;
  return k;
}

int byteps_reduce_blockq_destroy(byteps_reduce_blockq* q) {
  if (!q) return BYTEPS_REDUCE_OK;
  blockq_free(q);
  return BYTEPS_REDUCE_OK;
}

int byteps_reduce_copy(void* dst, const void* src, size_t len, void* stream) {
  if (len == 0 || dst == src) return BYTEPS_REDUCE_OK;
  if (!dst || !src) return fail(BYTEPS_REDUCE_EARGS, "null pointer");
  if (overlaps_partially(dst, src, len))
    return fail(BYTEPS_REDUCE_EARGS, "dst and src overlap");
  hipError_t e = launch_copy(dst, src, len, tuning(), to_stream(stream));
  return e == hipSuccess ? BYTEPS_REDUCE_OK : hip_fail(e, "copy kernel launch");
}

int byteps_reduce_sync(void* stream) {
  hipError_t e = hipStreamSynchronize(to_stream(stream));
  return e == hipSuccess ? BYTEPS_REDUCE_OK : hip_fail(e, "hipStreamSynchronize");
}

}  // extern "C"

// ------------------------------------------------------- keyed queue --
// (bpsr_internal.h keyq_*: the PS server's device releases)

namespace bpsr {

int keyq_create(const byteps_bucket_desc* buckets, int nkeys, int dtype, double timeout_s,
                byteps_reduce_blockq** out) {
  if (!out || nkeys < 1 || !buckets) return fail(BYTEPS_REDUCE_EARGS, "bad keyed queue table");
  *out = nullptr;
  for (int k = 0; k < nkeys; ++k)
    if (buckets[k].n < 1 || buckets[k].n > kKeyedMaxSrcs)
      return fail(BYTEPS_REDUCE_EARGS, "keyed queue: key %d has %d sources (1..%d)", k,
                  buckets[k].n, kKeyedMaxSrcs);
  std::vector<int> block_end((size_t)nkeys);
  bool wide = false;
  for (int k = 0; k < nkeys; ++k) {
    block_end[(size_t)k] = k + 1;
    wide = wide || buckets[k].n > kKeyedNarrowSrcs;
  }
  byteps_reduce_blockq* q = nullptr;
  int rc = byteps_reduce_blockq_create(buckets, nkeys, block_end.data(), nkeys, dtype,
                                       kModeReference, &q);
  if (rc) return rc;
  q->keyed = true;
  q->wide = wide;
  if (timeout_s > 0) q->timeout_s = timeout_s;
  const size_t nw = (size_t)nkeys * (wide ? 2 : 1);  // words per copy (device / host parity)
  const size_t kbytes = sizeof(uint64_t) * nw * kKeyWordStride;  // one word per line
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&q->kwords), kbytes);
  if (e == hipSuccess) e = hipMemset(q->kwords, 0, kbytes);
  void* p = nullptr;
  void* d = nullptr;
  if (e == hipSuccess)
    e = hipHostMalloc(&p, sizeof(uint64_t) * 2 * nw, hipHostMallocCoherent | hipHostMallocMapped);
  if (e == hipSuccess) {
    q->khwords = static_cast<uint64_t*>(p);
    for (size_t i = 0; i < 2 * nw; ++i) __atomic_store_n(q->khwords + i, (uint64_t)0, __ATOMIC_RELEASE);
    e = hipHostGetDevicePointer(&d, p, 0);
    q->khwords_dev = static_cast<uint64_t*>(d);
  }
  const size_t cbytes = sizeof(uint32_t) * (size_t)nkeys * kKeyCntStride;  // one per line
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&q->kcnt), cbytes);
  if (e == hipSuccess) e = hipMemset(q->kcnt, 0, cbytes);
  if (e == hipSuccess)
    e = hipHostMalloc(&p, sizeof(uint32_t) * (size_t)nkeys, hipHostMallocCoherent | hipHostMallocMapped);
  if (e == hipSuccess) {
    q->khdone = static_cast<uint32_t*>(p);
    for (int i = 0; i < nkeys; ++i) __atomic_store_n(q->khdone + i, 0u, __ATOMIC_RELEASE);
    e = hipHostGetDevicePointer(&d, p, 0);
    q->khdone_dev = static_cast<uint32_t*>(d);
  }
  if (e == hipSuccess)
    e = hipHostMalloc(&p, 256, hipHostMallocCoherent | hipHostMallocMapped);
  if (e == hipSuccess) {
    q->hctl = static_cast<BlockqCtl*>(p);
    std::memset(p, 0, 256);
    e = hipHostGetDevicePointer(&d, p, 0);
    q->hctl_dev = static_cast<BlockqCtl*>(d);
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();  // words zeroed before any stream uses them
  if (e != hipSuccess) {
    blockq_free(q);
    return hip_fail(e, "keyed queue setup");
  }
  *out = q;
  return BYTEPS_REDUCE_OK;
}

int keyq_launch(byteps_reduce_blockq* q, hipEvent_t stop, hipStream_t* stream, uint32_t* epoch) {
  std::lock_guard<std::mutex> g(q->mu);
  hipStream_t own = nullptr;
  hipError_t e = consumer_queue(q->device, q->cus, 2, &own);
  if (e != hipSuccess) return hip_fail(e, "consumer stream");
  const uint32_t ep = q->launch_epoch + 1;
  BlockqLaunch Q;
  Q.L = batch_launch(q->dev_table, q->ti);
  Q.L.stop = stop;
  Q.flags = q->flags;
  Q.block_first = q->flags + q->nblocks;
  Q.ctl = q->ctl;                // polled on the device (agent scope)
  Q.herr = &q->hctl_dev->err;    // mirrored to the host by the helper
  Q.nblocks = (uint32_t)q->nblocks;
  Q.timeout_ticks = (uint64_t)(q->timeout_s * 1e3 * (double)q->clock_khz);
  Q.epoch = ep;
  Q.helper = 1;  // workgroup 0 forwards the host words
  Q.hflags = nullptr;
  Q.keyed = 1;
  Q.wide = q->wide ? 1 : 0;
  Q.kwords = q->kwords;
  Q.khwords = q->khwords_dev;
  Q.kcnt = q->kcnt;
  Q.khdone = q->khdone_dev;
  Q.grid = q->ti.tiles + 1;
#ifdef BPSR_KEYED_TRACE
  if (!q->ktrace) {
    q->ktrace_per = 4 * (size_t)q->ti.tiles + (size_t)q->nblocks;
    if (hipMalloc(reinterpret_cast<void**>(&q->ktrace), 8 * q->ktrace_per * kKtraceSlots) != hipSuccess)
      return fail(BYTEPS_REDUCE_EHIP, "keyed trace buffer");
    (void)hipMemset(q->ktrace, 0, 8 * q->ktrace_per * kKtraceSlots);
    (void)hipDeviceSynchronize();
  }
  Q.ktrace = q->ktrace + (size_t)(ep % kKtraceSlots) * q->ktrace_per;
#endif
  // Residency: at most 2 consumer workgroups per CU, and room left beside
  // them for the work a missing release may still need — a push copy into a
  // slot (the copy kernel asks for 40 KiB of LDS) or a release kernel: 58 KiB
  // each (two fit in 160 KiB, three do not; 44 KiB stay free).
  const Tuning tu = tuning_for_n(q->ti.nmax);
  constexpr size_t kKeyedLds = 58u * 1024u;
  Q.started = nullptr;
  ConsumerDev& D = g_cdev[q->device];
  std::lock_guard<std::mutex> dg(D.mu);  // in the device's dispatch sequence
  e = seq_prepare(D, q->device, Q, own, 4 * Q.timeout_ticks);
  if (e == hipSuccess)
    e = launch_blockq(Q, q->ti.vpt, cache_pol(tu, (uint64_t)q->ti.tiles * q->ti.vpt * kBlock * 16),
                      kKeyedLds, true, q->dtype, q->mode, own);
  if (e != hipSuccess) return hip_fail(e, "keyed queue launch");
  seq_commit(D, Q, own);
  __atomic_store_n(&q->launch_epoch, ep, __ATOMIC_RELEASE);
  if (stream) *stream = own;
  if (epoch) *epoch = ep;
  return BYTEPS_REDUCE_OK;
}

// A key's release epoch is written only by its releaser (the server
// serialises a key's rounds) and the launch epoch only by keyq_launch (under
// q->mu): both are read lock-free, so releases of different keys from many
// receive threads share no lock.
uint32_t keyq_next_epoch(byteps_reduce_blockq* q, int key) {
  return __atomic_load_n(&q->rel_epoch[(size_t)key], __ATOMIC_ACQUIRE) + 1;
}

bool keyq_advance(byteps_reduce_blockq* q, uint32_t epoch) {
  std::lock_guard<std::mutex> g(q->mu);
  if (q->launch_epoch + 1 != epoch) return false;
  __atomic_store_n(&q->launch_epoch, epoch, __ATOMIC_RELEASE);
  return true;
}

uint32_t keyq_launched(byteps_reduce_blockq* q) {
  return __atomic_load_n(&q->launch_epoch, __ATOMIC_ACQUIRE);
}

void keyq_state(byteps_reduce_blockq* q, int key, uint32_t* next_epoch, uint32_t* launched) {
  *next_epoch = keyq_next_epoch(q, key);
  *launched = keyq_launched(q);
}

int keyq_release(byteps_reduce_blockq* q, int key, uint64_t perm, hipStream_t s, bool* first) {
  const uint32_t ep = q->rel_epoch[(size_t)key] + 1;
  {  // a round (folded here, or a skip word for a lane-folded one): the epoch has begun
    uint32_t o = __atomic_load_n(&q->opened, __ATOMIC_ACQUIRE);
    while (o < ep && !__atomic_compare_exchange_n(&q->opened, &o, ep, true, __ATOMIC_ACQ_REL,
                                                  __ATOMIC_ACQUIRE)) {
    }
    if (first) *first = o < ep;
  }
  const uint64_t w = key_word((uint32_t)perm, ep);
  const uint64_t w2 = key_word((uint32_t)(perm >> 32), ep);  // wide: positions 8..15
  const size_t second = (size_t)q->nblocks + (size_t)key;
  if (s) {
    const hipError_t e =
        launch_key_release(q->kwords, (uint32_t)key * kKeyWordStride, w,
                           q->wide ? q->kwords + second * kKeyWordStride : nullptr, w2, s);
    if (e != hipSuccess) return hip_fail(e, "keyed release");
  } else {
    // the second word first: the helper forwards a block once both carry the epoch
    if (q->wide) __atomic_store_n(q->khwords + 2 * second + (ep & 1u), w2, __ATOMIC_RELEASE);
    __atomic_store_n(q->khwords + 2 * (size_t)key + (ep & 1u), w, __ATOMIC_RELEASE);
  }
  __atomic_store_n(&q->rel_epoch[(size_t)key], ep, __ATOMIC_RELEASE);
  return BYTEPS_REDUCE_OK;
}

uint32_t keyq_opened(const byteps_reduce_blockq* q) {
  return __atomic_load_n(&q->opened, __ATOMIC_ACQUIRE);
}

bool keyq_close(byteps_reduce_blockq* q, uint32_t epoch) {
  uint32_t o = __atomic_load_n(&q->opened, __ATOMIC_ACQUIRE);
  while (o < epoch)
    if (__atomic_compare_exchange_n(&q->opened, &o, epoch, true, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE))
      return true;
  return false;
}

bool keyq_key_done(const byteps_reduce_blockq* q, int key, uint32_t epoch) {
  return epoch_reached(__atomic_load_n(q->khdone + key, __ATOMIC_ACQUIRE), epoch);
}

bool keyq_failed(byteps_reduce_blockq* q) {
  return __atomic_load_n(&q->hctl->err, __ATOMIC_ACQUIRE) != 0;
}

std::string keyq_debug(byteps_reduce_blockq* q) {
  std::lock_guard<std::mutex> g(q->mu);
  std::vector<uint64_t> dev((size_t)q->nblocks);
  const hipError_t e = hipMemcpy2D(dev.data(), 8, q->kwords, 8 * kKeyWordStride, 8, dev.size(),
                                  hipMemcpyDeviceToHost);
  char buf[512];
  int dev_at = 0, rel_at = 0, host_at = 0;
  const uint32_t ep = q->launch_epoch;
  int first_missing = -1;
  for (int b = 0; b < q->nblocks; ++b) {
    if ((uint32_t)dev[(size_t)b] == ep) ++dev_at;
    else if (first_missing < 0) first_missing = b;
    if (q->rel_epoch[(size_t)b] >= ep) ++rel_at;
    const uint64_t h = __atomic_load_n(q->khwords + 2 * (size_t)b + (ep & 1u), __ATOMIC_ACQUIRE);
    if ((uint32_t)h == ep) ++host_at;
  }
  snprintf(buf, sizeof(buf),
           "keyq: launch epoch %u, %d blocks: device words at epoch %d, host releases %d, "
           "host words %d, err %u, copy %d, first missing block %d (device word %llx host %llx)",
           ep, q->nblocks, dev_at, rel_at, host_at, q->hctl->err, (int)e, first_missing,
           first_missing >= 0 ? (unsigned long long)dev[(size_t)first_missing] : 0ull,
           first_missing >= 0 ? (unsigned long long)q->khwords[2 * (size_t)first_missing + (ep & 1u)]
                              : 0ull);
  return buf;
}

}  // namespace bpsr
