// CDNA4 (gfx950) kernels of the gradient-bucket reduce path — templates.
// Instantiated per dtype in bpsr_k_*.hip (parallel compilation).
//
//   fold_kernel     dst = ((s0 + s1) + ...) + s_{n-1}, one bucket, one launch.
//                   Replaces the (N-1) CpuReducer::sum calls of one server
//                   round (server.cc:216-250, cpu_reducer.cc:86-91) with a
//                   single pass: (N+1)*B HBM bytes instead of (3N-1)*B.
//   batched_kernel  the same over a table of buckets (one Prophet block,
//                   scheduled_queue.cc:244-296) in one launch.
//
// Design (pure HBM streaming, no reuse, no LDS, no MFMA):
//   * the vector range is cut into tiles of kBlock*VPT 16-byte vectors; a
//     workgroup owns a whole tile (contiguous 4*VPT KiB of every operand), lane
//     i of a wave reads base + 16*i, so every wave-instruction moves 1 KiB;
//   * per source, the VPT loads of a thread are issued back to back, all before
//     the dependent adds; the tile's stores leave as one burst at the end
//     (measured: tiles of 8-16 vectors per thread stream 5-10 % faster than a
//     grid-stride interleave, tools/hbm_probe.hip);
//   * non-temporal loads and stores (`nt`): inputs are read once, the output is
//     not re-read by this kernel;
//   * strict left fold in registers, no reassociation (bit-exact with the
//     reference order);
//   * elements outside the 16-B vector range (unaligned head, tail, and the
//     fp16 F16C-tail region, cpu_reducer.cc:118-125) go through the element
//     path with the reference's tail semantics.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bpsr_internal.h"
#include "bpsr_ops.h"

namespace bpsr {

template <bool NT>
__device__ __forceinline__ vec16 ld16(const unsigned char* p) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  if constexpr (NT) {
    return bitcast<vec16>(__builtin_nontemporal_load(reinterpret_cast<const u4*>(p)));
  } else {
    return bitcast<vec16>(*reinterpret_cast<const u4*>(p));
  }
}

template <bool NT>
__device__ __forceinline__ void st16(unsigned char* p, const vec16& v) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  if constexpr (NT) {
    __builtin_nontemporal_store(bitcast<u4>(v), reinterpret_cast<u4*>(p));
  } else {
    *reinterpret_cast<u4*>(p) = bitcast<u4>(v);
  }
}

template <class E>
__device__ __forceinline__ E ld_e(const unsigned char* p, bool aligned) {
  if (aligned) return *reinterpret_cast<const E*>(p);
  E v;
  __builtin_memcpy(&v, p, sizeof(E));
  return v;
}

template <class E>
__device__ __forceinline__ void st_e(unsigned char* p, E v, bool aligned) {
  if (aligned) {
    *reinterpret_cast<E*>(p) = v;
  } else {
    __builtin_memcpy(p, &v, sizeof(E));
  }
}

constexpr int cmin(int a, int b) { return a < b ? a : b; }

// Exact replay of one vector's fold (NaN payload rules), re-reading memory.
// Only runs for vectors whose fast-path result holds a NaN.  The addresses go
// through an empty asm so the compiler cannot merge these loads with the fast
// path's (merging drops the loads' non-temporal hint and reorders the fast
// path's load stream around the first adds).
// XS: anything indexable as srcs[k] -> source pointer (a pointer array, or the
// keyed consumer's arrival-order view of one, PermSrcs).
using SrcPtrs = const unsigned char* const*;

template <class Op, bool NT, class XS = SrcPtrs>
__device__ __forceinline__ vec16 fold_vector_exact(const XS& srcs, int n, uint64_t off) {
  auto opaque = [](const unsigned char* p) {
    asm volatile("" : "+v"(p));
    return p;
  };
  typename Op::Acc acc = Op::init(ld16<NT>(opaque(srcs[0] + off)));
  for (int k = 1; k < n; ++k) Op::accum(acc, ld16<NT>(opaque(srcs[k] + off)));
  return Op::finish(acc);
}

// One tile: vectors [v0, v0 + kBlock*VPT) clipped to nvec, of the vector
// range starting at byte `vec_off` of every operand.  Thread `lane` handles
// v0 + j*kBlock + lane, j < VPT.
//
// The loads of G sources x VPT vectors are issued back to back (G*VPT <= 32
// 16-B loads in flight per lane), then folded with plain adds (Op::fast); a
// NaN anywhere in a chain survives to its result, so one has_nan test per
// vector decides whether the exact NaN-payload rule must be replayed
// (fold_vector_exact) — a wave-uniform branch never taken on finite data.
// GUARD: the last, partial tile (vectors past nvec are neither read nor written).
// NS > 0: exactly NS sources; NS < 0: at most -NS (<= 8) sources, n at run
// time, one load group with compile-time indices (so `srcs` may be a register
// array); NS == 0: any n.  `xsrcs` (memory) serves the exact NaN replay.
template <class Op, int VPT, int NT, int NS, bool GUARD, class XS = SrcPtrs,
          class SP = const unsigned char* const*>
__device__ __forceinline__ void fold_tile_body(const SP& srcs, const XS& xsrcs, int n,
                                               unsigned char* dst, uint64_t vec_off,
                                               uint64_t v0, uint64_t nvec, int lane) {
  constexpr int NSA = NS < 0 ? -NS : NS;
  const int ns = NS > 0 ? NS : n;
  const uint64_t off0 = vec_off + (v0 + lane) * 16;
  constexpr uint64_t kStep = (uint64_t)kBlock * 16;
  constexpr int G = NSA > 0 ? cmin(NSA, 32 / VPT) : cmin(8, 32 / VPT);
  static_assert(NS >= 0 || G == NSA, "NS < 0 needs one load group");
  bool valid[VPT];
#pragma unroll
  for (int j = 0; j < VPT; ++j) valid[j] = !GUARD || (v0 + lane + (uint64_t)j * kBlock < nvec);
  typename Op::Acc acc[VPT];
  auto group = [&](int k0) __attribute__((always_inline)) {
    vec16 x[G][VPT];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (NS > 0 || k0 + g < ns) {
        const unsigned char* base = srcs[k0 + g] + off0;
#pragma unroll
        for (int j = 0; j < VPT; ++j)
          x[g][j] = valid[j] ? ld16<(NT != 0)>(base + j * kStep) : vec16{{0, 0, 0, 0}};
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (NS > 0 || k0 + g < ns) {
#pragma unroll
        for (int j = 0; j < VPT; ++j) {
          if (k0 + g == 0) acc[j] = Op::init_fast(x[g][j]);
          else Op::fast(acc[j], x[g][j]);
        }
      }
    }
  };
  if constexpr (NSA > 0) {
#pragma unroll
    for (int k0 = 0; k0 < NSA; k0 += G) group(k0);
  } else {
    for (int k0 = 0; k0 < ns; k0 += G) group(k0);
  }
  bool bad = false;
#pragma unroll
  for (int j = 0; j < VPT; ++j) bad |= valid[j] && Op::has_nan(acc[j]);
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    vec16 out = Op::finish_fast(acc[j]);
    if (__builtin_expect(bad, 0)) {
      if (valid[j] && Op::has_nan(acc[j]))
        out = fold_vector_exact<Op, (NT != 0), XS>(xsrcs, ns, off0 + j * kStep);
    }
    if (valid[j]) st16<(NT != 0)>(dst + off0 + j * kStep, out);
  }
}

// Full tile through buffer instructions: one SGPR descriptor per operand
// based at the tile's first byte (wave-uniform: kernel arguments + blockIdx),
// 32-bit lane offsets, nt as the cache-policy operand.  Same load grouping,
// fast fold and NaN replay as fold_tile_body.
// `mid` runs once the tile's loads have all been consumed and before its
// stores issue (blockq_kernel consumes its prefetched work-queue values there,
// where they are complete, so nothing is left pending across the stores).
struct NoMid {
  __device__ __forceinline__ void operator()() const {}
};

template <class Op, int VPT, int NT, int NS, class Mid = NoMid, class XS = SrcPtrs,
          class SP = const unsigned char* const*>
__device__ __forceinline__ void fold_tile_full_buf(const SP& srcs, const XS& xsrcs, int n,
                                                   unsigned char* dst, uint64_t byte0, int lane,
                                                   const Mid& mid = Mid()) {
  constexpr int kAux = NT ? 2 : 0;               // loads: 2 = nt
  constexpr int kStAux = NT == kPolWt ? 16 : kAux;  // stores: 16 = sc1 (write-through)
  constexpr int kTileBytes = kBlock * VPT * 16;
  constexpr int NSA = NS < 0 ? -NS : NS;
  constexpr int G = NSA > 0 ? cmin(NSA, 32 / VPT) : cmin(8, 32 / VPT);
  static_assert(NS >= 0 || G == NSA, "NS < 0 needs one load group");
  const int ns = NS > 0 ? NS : n;
  const int voff = lane * 16;
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  auto rsrc = [&](const unsigned char* base) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(base) + byte0, 0,
                                             kTileBytes, 0x00020000);
  };
  typename Op::Acc acc[VPT];
  auto group = [&](int k0) __attribute__((always_inline)) {
    vec16 x[G][VPT];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (NS > 0 || k0 + g < ns) {
        const auto r = rsrc(srcs[k0 + g]);
#pragma unroll
        for (int j = 0; j < VPT; ++j)
          x[g][j] = bitcast<vec16>(__builtin_amdgcn_raw_buffer_load_b128(r, voff + j * kBlock * 16,
                                                                         0, kAux));
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (NS > 0 || k0 + g < ns) {
#pragma unroll
        for (int j = 0; j < VPT; ++j) {
          if (k0 + g == 0) acc[j] = Op::init_fast(x[g][j]);
          else Op::fast(acc[j], x[g][j]);
        }
      }
    }
  };
  if constexpr (NSA > 0) {
#pragma unroll
    for (int k0 = 0; k0 < NSA; k0 += G) group(k0);
  } else {
    for (int k0 = 0; k0 < ns; k0 += G) group(k0);
  }
  mid();
  bool bad = false;
#pragma unroll
  for (int j = 0; j < VPT; ++j) bad = bad || Op::has_nan(acc[j]);
  const auto rd = __builtin_amdgcn_make_buffer_rsrc(dst + byte0, 0, kTileBytes, 0x00020000);
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    vec16 out = Op::finish_fast(acc[j]);
    if (__builtin_expect(bad, 0)) {
      if (Op::has_nan(acc[j]))
        out = fold_vector_exact<Op, (NT != 0), XS>(xsrcs, ns, byte0 + voff + j * kBlock * 16);
    }
    __builtin_amdgcn_raw_buffer_store_b128(bitcast<u4>(out), rd, voff + j * kBlock * 16, 0, kStAux);
  }
}

template <class Op, int VPT, int NT, int NS>
__device__ __forceinline__ void fold_tile(const unsigned char* const* srcs, int n,
                                          unsigned char* dst, uint64_t vec_off, uint64_t v0,
                                          uint64_t nvec, int lane) {
  if (v0 + (uint64_t)kBlock * VPT <= nvec)
    fold_tile_full_buf<Op, VPT, NT, NS>(srcs, srcs, n, dst, vec_off + v0 * 16, lane);
  else
    fold_tile_body<Op, VPT, NT, NS, true>(srcs, srcs, n, dst, vec_off, v0, nvec, lane);
}

// Element part: elements [0, head) and [tail_begin, n_elems) plus trailing
// bytes; elements >= tail_sem_from get the F16C-tail NaN rule (fp16 only).
// Each element's N loads are issued together (groups of 8) before the fold.
template <class Op, class XS = SrcPtrs>
__device__ __forceinline__ void fold_elements(const XS& srcs, int n,
                                              unsigned char* dst, const FoldGeom& g,
                                              bool aligned, uint64_t t, uint64_t stride) {
  using E = typename Op::E;
  const uint64_t n_head = g.head_elems;
  const uint64_t n_tail = g.n_elems - g.tail_begin;
  const uint64_t n_scalar = n_head + n_tail;
  for (uint64_t s = t; s < n_scalar; s += stride) {
    const uint64_t e = s < n_head ? s : g.tail_begin + (s - n_head);
    const bool tail = e >= g.tail_sem_from;
    const uint64_t off = e * sizeof(E);
    typename Op::EAcc acc{};
    for (int k0 = 0; k0 < n; k0 += 8) {
      E x[8];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (k0 + q < n) x[q] = ld_e<E>(srcs[k0 + q] + off, aligned);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (k0 + q < n) {
          if (k0 + q == 0) acc = Op::init_e(x[q], tail);
          else Op::accum_e(acc, x[q], tail);
        }
      }
    }
    st_e<E>(dst + off, Op::finish_e(acc, tail), aligned);
  }
  // Trailing len % sizeof(T) bytes of a fold into a separate dst: the fold's
  // accumulator is the first arrival (server.cc:216-218), so they come from
  // srcs[0].
  if (g.copy_trailing) {
    const uint64_t tb = g.n_elems * sizeof(E);
    for (uint64_t b = t; b < g.trailing_bytes; b += stride) dst[tb + b] = srcs[0][tb + b];
  }
}

// Pin every kernel argument the tile loop needs in SGPRs at kernel entry (no
// instruction emitted): ONE asm statement, so all the scalar loads issue
// together behind one s_waitcnt instead of as a chain of dependent scalar
// round trips.  With one resident workgroup per CU that chain would be paid
// on every tile.
template <int NS>
__device__ __forceinline__ void pin_args(const FoldArgs& a) {
  if constexpr (NS == 8) {
    asm volatile("" ::"s"(a.srcs[0]), "s"(a.srcs[1]), "s"(a.srcs[2]), "s"(a.srcs[3]),
                 "s"(a.srcs[4]), "s"(a.srcs[5]), "s"(a.srcs[6]), "s"(a.srcs[7]), "s"(a.dst),
                 "s"(a.g.nvec), "s"(a.g.vec_off), "s"(a.grid));
  } else if constexpr (NS == 2) {
    asm volatile("" ::"s"(a.srcs[0]), "s"(a.srcs[1]), "s"(a.dst), "s"(a.g.nvec),
                 "s"(a.g.vec_off), "s"(a.grid));
  } else if constexpr (NS == 16) {
    asm volatile("" ::"s"(a.srcs[0]), "s"(a.srcs[1]), "s"(a.srcs[2]), "s"(a.srcs[3]),
                 "s"(a.srcs[4]), "s"(a.srcs[5]), "s"(a.srcs[6]), "s"(a.srcs[7]),
                 "s"(a.srcs[8]), "s"(a.srcs[9]), "s"(a.srcs[10]), "s"(a.srcs[11]),
                 "s"(a.srcs[12]), "s"(a.srcs[13]), "s"(a.srcs[14]), "s"(a.srcs[15]),
                 "s"(a.dst), "s"(a.g.nvec), "s"(a.g.vec_off), "s"(a.grid));
  } else {
    asm volatile("" ::"s"(a.dst), "s"(a.g.nvec), "s"(a.g.vec_off), "s"(a.grid));
  }
}

template <class Op, int VPT, int NT, int NS>
__global__ __launch_bounds__(kBlock) void fold_kernel(FoldArgs a) {
  pin_args<NS>(a);
  // One tile per workgroup (the launcher sizes the grid to the tile count):
  // workgroups are dispatched in tile order, so the chip sweeps every operand
  // as one tight window (a persistent tile-stride loop measured 10-20 % slower).
  // The slow pieces — the guarded partial last tile and the element work
  // (unaligned head, tail, fp16 F16C tail, trailing bytes) — go to workgroup 0,
  // first off the dispatcher, so they overlap the sweep instead of trailing it
  // (as the last workgroup they extended every unaligned launch by its latency);
  // the full tiles follow in address order.
  const uint64_t tile_vecs = (uint64_t)kBlock * VPT;
  const uint64_t full = a.g.nvec / tile_vecs;
  const bool partial = full * tile_vecs < a.g.nvec;
  const uint64_t bid = blockIdx.x;
  // decided at entry, while the arguments are in SGPRs (no reload after the loop)
  const int elem_mode = a.g.nvec == 0 ? 2 : (bid == 0 ? 1 : 0);
  const uint64_t tile = partial ? (bid == 0 ? full : bid - 1) : bid;
  if (tile < full)
    fold_tile_full_buf<Op, VPT, NT, NS>(a.srcs, a.srcs, a.n, a.dst,
                                        a.g.vec_off + tile * tile_vecs * 16, threadIdx.x);
  else if (tile * tile_vecs < a.g.nvec)
    fold_tile_body<Op, VPT, NT, NS, true>(a.srcs, a.srcs, a.n, a.dst, a.g.vec_off,
                                          tile * tile_vecs, a.g.nvec, threadIdx.x);
  if (elem_mode == 2)
    fold_elements<Op>(a.srcs, a.n, a.dst, a.g, a.aligned != 0,
                      (uint64_t)blockIdx.x * kBlock + threadIdx.x, (uint64_t)a.grid * kBlock);
  else if (elem_mode == 1)
    fold_elements<Op>(a.srcs, a.n, a.dst, a.g, a.aligned != 0, threadIdx.x, kBlock);
}

// One tile record of a batched table (TileHead, bpsr_internal.h), already in
// registers: the head, the first 8 source pointers (wave-uniform, SGPRs) and
// the record's pointer array `msrcs` (for n > 8 and the exact NaN replay).
// Vector tiles go straight to their data (pointers pre-advanced to the tile);
// element tiles fetch their bucket's geometry from the entry table and stride
// over its element work.
struct RecRegs {
  unsigned char* dst;
  uint32_t kind, n, a, b, c;
  const unsigned char* p[8];
};

template <class Op, int VPT, int NT, class Mid = NoMid>
__device__ __forceinline__ void run_record(const RecRegs& r, const unsigned char* const* msrcs,
                                           const BatchEntry* entries, const Mid& mid = Mid()) {
  if (r.kind == kTileElem) {
    const BatchEntry& e = entries[r.b];
    fold_elements<Op>(e.srcs, e.n, e.dst, e.g, e.aligned != 0,
                      (uint64_t)r.a * kBlock + threadIdx.x, (uint64_t)r.c * kBlock);
    mid();
  } else if (r.n <= 8) {
    if (r.kind == kTileFull) {
      fold_tile_full_buf<Op, VPT, NT, -8>(r.p, msrcs, (int)r.n, r.dst, 0, threadIdx.x, mid);
    } else {
      fold_tile_body<Op, VPT, NT, -8, true>(r.p, msrcs, (int)r.n, r.dst, 0, 0, r.a, threadIdx.x);
      mid();
    }
  } else {
    if (r.kind == kTileFull) {
      fold_tile_full_buf<Op, VPT, NT, 0>(msrcs, msrcs, (int)r.n, r.dst, 0, threadIdx.x, mid);
    } else {
      fold_tile_body<Op, VPT, NT, 0, true>(msrcs, msrcs, (int)r.n, r.dst, 0, 0, r.a,
                                           threadIdx.x);
      mid();
    }
  }
}

// Read a record's head + 8 pointers in C++: the compiler emits scalar loads
// when nothing in the kernel can have written the table before (batched_kernel),
// and one empty asm pins them so they issue together (one scalar round trip).
__device__ __forceinline__ RecRegs load_record(const unsigned char* rec) {
  const TileHead& h = *reinterpret_cast<const TileHead*>(rec);
  const unsigned char* const* msrcs =
      reinterpret_cast<const unsigned char* const*>(rec + kTileHeadBytes);
  RecRegs r;
  r.dst = h.dst;
  r.kind = h.kind;
  r.n = h.n;
  r.a = h.a;
  r.b = h.b;
  r.c = h.c;
#pragma unroll
  for (int k = 0; k < 8; ++k) r.p[k] = msrcs[k];
  asm volatile("" ::"s"(r.dst), "s"(r.kind), "s"(r.n), "s"(r.a), "s"(r.p[0]), "s"(r.p[1]),
               "s"(r.p[2]), "s"(r.p[3]), "s"(r.p[4]), "s"(r.p[5]), "s"(r.p[6]), "s"(r.p[7]));
  return r;
}

// A record's head + 8 pointers as 24 words staged in LDS (blockq_kernel
// prefetches the next tile's record there while the current tile streams):
// uniform LDS reads, then SGPRs.
constexpr int kRecWords = (kTileHeadBytes + 8 * 8) / 4;
__device__ __forceinline__ RecRegs regs_from_words(const uint32_t* w) {
  uint32_t v[kRecWords];
#pragma unroll
  for (int k = 0; k < kRecWords; ++k) v[k] = __builtin_amdgcn_readfirstlane(w[k]);
  auto ptr = [&](int k) {
    return reinterpret_cast<unsigned char*>(((uint64_t)v[k + 1] << 32) | v[k]);
  };
  RecRegs r;
  r.dst = ptr(0);
  r.kind = v[2];
  r.n = v[3];
  r.a = v[4];
  r.b = v[5];
  r.c = v[6];
#pragma unroll
  for (int k = 0; k < 8; ++k) r.p[k] = ptr(8 + 2 * k);
  return r;
}

// L2 prefetch of the tile record that workgroup `t` will read: the record
// fetch is a dependent round trip at the head of every workgroup (nothing
// else can issue before the pointers arrive), and at one or two resident
// workgroups per CU it is not hidden behind another workgroup's loads.  A
// workgroup touches the record of the workgroup dispatched L.pf_ahead later
// (default kPrefetchAhead) — the same XCD (workgroups go to the 8 XCDs
// round-robin, and the distance is a multiple of 8), about one resident round
// ahead — so that record is in the XCD's L2 when its workgroup starts.  Tables
// read zero-copy from host memory are not prefetched (pf_ahead 0).  Two lanes, one
// dword at each end of the record (a 96-B record may straddle two 128-B
// lines).  The values are consumed by keep_prefetch at the very end, after
// the tile's own loads and stores were issued, so no wait lands earlier.
__device__ __forceinline__ uint32_t prefetch_record(const BatchLaunch& L, uint64_t b) {
  uint32_t v = 0;
  const uint64_t t = b + L.pf_ahead;
  if (L.pf_ahead != 0 && threadIdx.x < 2 && t < L.tiles) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(L.recs + t * L.rec_stride);
    v = p[threadIdx.x == 0 ? 0 : L.rec_stride / 4 - 1];
  }
  return v;
}
__device__ __forceinline__ void keep_prefetch(uint32_t v) { asm volatile("" ::"v"(v)); }

// Batched: workgroup b runs record b of the launch.
template <class Op, int VPT, int NT>
__global__ __launch_bounds__(kBlock) void batched_kernel(BatchLaunch L) {
  const unsigned char* rec = L.recs + (uint64_t)blockIdx.x * L.rec_stride;
  const RecRegs r = load_record(rec);
  const uint32_t pf = prefetch_record(L, blockIdx.x);
  run_record<Op, VPT, NT>(r, reinterpret_cast<const unsigned char* const*>(rec + kTileHeadBytes),
                          L.entries);
  keep_prefetch(pf);
}

// Persistent block consumer (byteps_reduce_blockq_*).  Q.grid resident
// workgroups sweep the tile records of the whole table in order — workgroup w
// takes tiles w, w + grid, w + 2*grid, ... — so the chip still streams the
// table as one advancing window, across block boundaries, with no launch
// boundary between blocks.  The record of the next tile is loaded while the
// current tile streams (every thread one word, staged in LDS) and consumed
// (`mid`) right after the tile's loads, before its stores: nothing is left
// pending across the stores, so the next tile's loads issue while the stores
// drain.  (A work-queue atomic in place of the static order put a vmcnt(0)
// at the top of every iteration — the returned-atomic register's write-after-
// write guard — and so an HBM write round trip per tile.)
// Blocks are consumed in table order: a workgroup may start tile t once every
// block up to t's is released for this launch's epoch.  It keeps the first tile past the released
// prefix it last saw (`ready_tiles`), so a tile costs one compare unless it
// crosses that mark; then wave 0 scans the flags 64 at a time (one load per
// lane), sleeping between polls, and the workgroup acquires at system scope
// (the data may have landed by DMA or from another queue).  Every wave reaches
// the exit: all its tiles done, or a release that does not come within
// Q.timeout_ticks sets the sticky ctl->err, which every waiting workgroup sees
// on its next poll.  Nothing is re-armed: the next launch waits for the next
// epoch.  Every access to the flags is a system-scope atomic (releases:
// blockq_release_kernel).
__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Dispatch sequence: each of the launch's last
// kSeqLast workgroups counts itself started on entry, before any wait (one
// no-return vector atomic; every other workgroup skips it — a counted start
// costs its wave the atomic's ~1 µs of vmcnt, measured 5 µs per config-3
// launch when every workgroup counted).  Hardware deals a launch's
// workgroups round-robin over the 8 XCDs and dispatches each XCD's share in
// index order, so the last 8 started means every workgroup has.  A launch
// on another stream is gated on the count (seq_gate_kernel).
__device__ __forceinline__ void note_started(const BlockqLaunch& Q) {
  if (Q.started == nullptr || threadIdx.x != 0 || blockIdx.x + kSeqLast < gridDim.x) return;
  (void)__hip_atomic_fetch_add(Q.started, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <class Op, int VPT, int NT>
__global__ __launch_bounds__(kBlock) void blockq_kernel(BlockqLaunch Q) {
  note_started(Q);
  // record slots alternate: iteration i reads slot i&1 and stages the next
  // record into the other one, so no wave overwrites a record still being read
  __shared__ __attribute__((aligned(16))) uint32_t s_rec[2][kRecWords];
  __shared__ uint32_t s_ready, s_ready_tiles, s_abort;
  const uint32_t tid = threadIdx.x;
  const uint32_t tw = tid % (uint32_t)kRecWords;
  auto rec_at = [&](uint32_t t) { return Q.L.recs + (uint64_t)t * Q.L.rec_stride; };
  if (blockIdx.x < Q.L.tiles)
    s_rec[0][tw] = reinterpret_cast<const uint32_t*>(rec_at(blockIdx.x))[tw];
  __syncthreads();
  uint32_t ready = 0, ready_tiles = 0;  // blocks [0, ready) = tiles [0, ready_tiles) released
  uint32_t it = 0;
  for (uint32_t t = blockIdx.x; t < Q.L.tiles; t += Q.grid, ++it) {
    if (t >= ready_tiles) {
      if (tid < 64) {
        const uint32_t lane = tid;
        uint32_t r = ready, rt = ready_tiles;
        bool abort = false;
        const uint64_t t0 = wall_clock64();
        for (;;) {
          const uint32_t b = r + lane;
          const bool rel = b >= Q.nblocks || epoch_reached(ld_sys(Q.flags + b), Q.epoch);
          const uint64_t pending = __ballot(!rel);
          const uint32_t r2 = pending == 0 ? (r + 64 < Q.nblocks ? r + 64 : Q.nblocks)
                                           : r + (uint32_t)__builtin_ctzll(pending);
          if (r2 != r) {
            r = r2;
            rt = Q.block_first[r];
          }
          if (rt > t) break;
          if (pending == 0) continue;  // next chunk of flags
          if (__hip_atomic_load(&Q.ctl->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            abort = true;
            break;
          }
          if (wall_clock64() - t0 > Q.timeout_ticks) {
            if (lane == 0)
              __hip_atomic_store(&Q.ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            abort = true;
            break;
          }
          __builtin_amdgcn_s_sleep(4);
        }
        if (lane == 0) {
          s_ready = r;
          s_ready_tiles = rt;
          s_abort = abort ? 1u : 0u;
        }
      }
      __syncthreads();
      if (s_abort) break;
      ready = __builtin_amdgcn_readfirstlane(s_ready);
      ready_tiles = __builtin_amdgcn_readfirstlane(s_ready_tiles);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    const uint32_t tn = t + Q.grid;
    const uint32_t w = reinterpret_cast<const uint32_t*>(rec_at(tn < Q.L.tiles ? tn : t))[tw];
    const uint32_t nslot = (it + 1) & 1;
    auto mid = [&]() __attribute__((always_inline)) { s_rec[nslot][tw] = w; };
    run_record<Op, VPT, NT>(regs_from_words(s_rec[it & 1]),
                            reinterpret_cast<const unsigned char* const*>(rec_at(t) +
                                                                          kTileHeadBytes),
                            Q.L.entries, mid);
    __syncthreads();
  }
}

// Dispatch-ordered block consumer (the block queue's default mode): one tile
// record per workgroup, grid = tiles, like batched_kernel — hardware dispatch
// in tile order keeps the sweep as tight as one batched launch.  Each wave
// loads the release words of the first 64 blocks (one system-scope load per
// lane) together with its record's scalar loads — no extra round trip — and
// its tile may start once every block up to the tile's own holds this
// launch's epoch or a later one.  A wave whose tile is not yet released polls
// the words (`s_sleep` between polls, bounded by the timeout) and acquires
// before its loads; one whose tile is released reads data no workgroup of
// this launch has touched since the launch's own acquire (blocks do not share
// lines), so it needs none.
// Host releases (byteps_reduce_blockq_release_host): workgroup 0 of a launch
// with Q.helper forwards the host-written words into the device words the
// tiles poll, one system-scope load per block and lane, `s_sleep` between
// sweeps, until every block holds this launch's epoch (or the sticky error /
// the timeout ends the launch).  One wave works; the others return at once.
// Vector atomics only (the release words are written through the vector
// path, as blockq_release_kernel does).
__device__ __forceinline__ void forward_host_releases(const BlockqLaunch& Q) {
  if (threadIdx.x >= 64) return;
  const uint32_t lane = threadIdx.x;
  const uint64_t t0 = wall_clock64();
  for (;;) {
    bool pending = false;
    for (uint32_t base = 0; base < Q.nblocks; base += 64) {
      const uint32_t b = base + lane;
      if (b < Q.nblocks) {
        uint32_t d = ld_sys(Q.flags + b);
        const uint32_t h = ld_sys(Q.hflags + b);
        if (h != 0 && !epoch_reached(d, h)) {
          __hip_atomic_fetch_max(Q.flags + b, h, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
          d = h;
        }
        pending = pending || !epoch_reached(d, Q.epoch);
      }
    }
    if (__ballot(pending) == 0) return;
    if (__hip_atomic_load(&Q.ctl->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    if (wall_clock64() - t0 > Q.timeout_ticks) {
      if (lane == 0) __hip_atomic_store(&Q.ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

template <class Op, int VPT, int NT>
__global__ __launch_bounds__(kBlock) void blockq_gate_kernel(BlockqLaunch Q) {
  note_started(Q);
  if (Q.helper && blockIdx.x == 0) {  // dispatched first: resident for the whole launch
    forward_host_releases(Q);
    return;
  }
  const uint32_t t = blockIdx.x - Q.helper;
  const uint32_t lane = threadIdx.x & 63u;
  const unsigned char* rec = Q.L.recs + (uint64_t)t * Q.L.rec_stride;
  // the words (vector load) and the record (scalar loads) travel together
  uint32_t w = lane < Q.nblocks ? ld_sys(Q.flags + lane) : Q.epoch;
  const RecRegs r = load_record(rec);
  const uint32_t blk = reinterpret_cast<const TileHead*>(rec)->block;
  const uint32_t pf = prefetch_record(Q.L, t);
  // every block b <= blk released for this epoch (blocks past 64: rare, more loads)
  auto released = [&](uint32_t w0) __attribute__((always_inline)) {
    if (__ballot(lane <= blk && !epoch_reached(w0, Q.epoch)) != 0) return false;
    for (uint32_t base = 64; base <= blk; base += 64) {
      const uint32_t b = base + lane;
      const uint32_t wb = b <= blk ? ld_sys(Q.flags + b) : Q.epoch;
      if (__ballot(!epoch_reached(wb, Q.epoch)) != 0) return false;
    }
    return true;
  };
  if (!released(w)) {
    const uint64_t t0 = wall_clock64();
    for (;;) {
      __builtin_amdgcn_s_sleep(4);
      w = lane < Q.nblocks ? ld_sys(Q.flags + lane) : Q.epoch;
      if (released(w)) break;
      if (__hip_atomic_load(&Q.ctl->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
      if (wall_clock64() - t0 > Q.timeout_ticks) {
        __hip_atomic_store(&Q.ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  run_record<Op, VPT, NT>(r, reinterpret_cast<const unsigned char* const*>(rec + kTileHeadBytes),
                          Q.L.entries);
  keep_prefetch(pf);
}

// Keyed block consumer (the PS server's device releases): one block per key,
// dispatch-ordered like blockq_gate_kernel, but a tile waits for its OWN
// block's word only (keys complete in any order; server.cc folds each key
// when its last push arrives), and that word carries the round's arrival
// order, so the tile folds its sources as the left fold in arrival order
// (server.cc:216-250) from slots laid out by worker.
__device__ __forceinline__ uint64_t ld_sys64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The device words are written on this agent only (the helper, a stream
// release kernel): agent-scope polls are served by the L2, not HBM.
__device__ __forceinline__ uint64_t ld_agent64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_err(const BlockqLaunch& Q) {
  return __hip_atomic_load(&Q.ctl->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup 0: forward the host-written words of this launch's epoch (the
// epoch's parity slot) into the device words, until every block holds this
// epoch (or the sticky error / the timeout ends the launch).  A block
// released by a stream kernel already holds it.  Vector atomics only.  Its 4
// waves take 64-key chunks in turn (wave w: chunks w, w + 4, ...), so a sweep
// costs one chunk's dependent loads (device word, then host word over PCIe)
// rather than one per chunk: with the epoch's consumer launched ahead, its
// tiles are waiting when the first push arrives, and the sweep is the delay
// between a release and its fold.
__device__ __forceinline__ void forward_host_keys(const BlockqLaunch& Q) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t first = threadIdx.x & ~63u;  // this wave's first chunk
  if (first >= Q.nblocks) return;
  const uint32_t par = Q.epoch & 1u;
  const uint64_t t0 = wall_clock64();
  for (;;) {
    bool pending = false;
    const uint32_t err = ld_err(Q);  // with the sweep's loads, not after them
    for (uint32_t base = first; base < Q.nblocks; base += kBlock) {
      const uint32_t b = base + lane;
      if (b >= Q.nblocks) continue;
      // the device word and the host words load together (one PCIe round
      // trip per sweep, not a device load and then a dependent host load):
      // a release waits at most one sweep before its tiles see it
      const uint64_t d = ld_agent64(Q.kwords + (uint64_t)b * kKeyWordStride);
      const uint64_t h = ld_sys64(Q.khwords + 2 * (uint64_t)b + par);
      // a wide queue's second words follow the first ones (the host stores
      // the second before the first; a tile checks the second's epoch too)
      const uint64_t h2 =
          Q.wide ? ld_sys64(Q.khwords + 2 * (uint64_t)(Q.nblocks + b) + par) : 0;
      if ((uint32_t)d != Q.epoch) {
        // relaxed: the word publishes no data of this workgroup (the round's
        // data landed before the host's store), and a release at system
        // scope would write back the XCD's whole L2 — once per key, while the
        // consumer's own stores fill it (measured: the epoch's consumer took
        // 0.49 ms instead of ~0.1 for config 3's 165 keys)
        if ((uint32_t)h == Q.epoch && (!Q.wide || (uint32_t)h2 == Q.epoch)) {
          if (Q.wide)
            __hip_atomic_store(Q.kwords + (uint64_t)(Q.nblocks + b) * kKeyWordStride, h2,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(Q.kwords + (uint64_t)b * kKeyWordStride, h, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
#ifdef BPSR_KEYED_TRACE
          Q.ktrace[4 * (uint64_t)Q.L.tiles + b] = wall_clock64();
#endif
        } else {
          pending = true;
        }
      }
    }
    if (__ballot(pending) == 0) return;
    // a tile gave up, or this wave does: the host reads the mirror word
    const bool late = wall_clock64() - t0 > Q.timeout_ticks;
    if (late || err) {
      if (lane == 0) {
        __hip_atomic_store(&Q.ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(Q.herr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// A pointer array seen in arrival order: position k is worker (perm >> 4k) & 7.
struct PermSrcs {
  const unsigned char* const* m;
  uint32_t perm;
  __device__ __forceinline__ const unsigned char* operator[](int k) const {
    return m[(perm >> (4 * k)) & 7u];
  }
};

// The same for up to 16 sources (a wide keyed queue): position k is worker
// (perm >> 4k) & 15, perm from the block's two release words.
struct PermSrcs16 {
  const unsigned char* const* m;
  uint64_t perm;
  __device__ __forceinline__ const unsigned char* operator[](int k) const {
    return m[(perm >> (4 * k)) & 15u];
  }
};

// A keyed tile is done: once every wave's stores have drained (write-through
// for full tiles of a write-through launch; any other tile also writes back
// its XCD's L2 first), one lane counts the tile for its block, and the
// block's last tile of the epoch stores the epoch into the block's host word.
// (Counting per wave without waiting, with the helper publishing completion,
// measured slower: 0.130 against 0.108 ms per config-3 round, r06s33.)
template <int NT>
__device__ __forceinline__ void key_tile_done(const BlockqLaunch& Q, uint32_t blk,
                                              bool written_through) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
  __syncthreads();
  if (threadIdx.x == 0) {
    if (!written_through) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const uint32_t nt = Q.block_first[blk + 1] - Q.block_first[blk];
    const uint32_t old = __hip_atomic_fetch_add(Q.kcnt + (uint64_t)blk * kKeyCntStride, 1u,
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((old + 1) % nt == 0)
      __hip_atomic_store(Q.khdone + blk, Q.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <class Op, int VPT, int NT>
__global__ __launch_bounds__(kBlock) void blockq_key_kernel(BlockqLaunch Q) {
  note_started(Q);
  if (Q.helper && blockIdx.x == 0) {  // dispatched first: resident for the whole launch
    forward_host_keys(Q);
    return;
  }
  const uint32_t t = blockIdx.x - Q.helper;
#ifdef BPSR_KEYED_TRACE
  unsigned long long* kt = Q.ktrace + 4 * (uint64_t)t;
  if (threadIdx.x == 0) kt[0] = wall_clock64();
#endif
  const unsigned char* rec = Q.L.recs + (uint64_t)t * Q.L.rec_stride;
  const RecRegs r = load_record(rec);
  const uint32_t blk = reinterpret_cast<const TileHead*>(rec)->block;
  const uint32_t pf = prefetch_record(Q.L, t);
  const uint64_t* wp = Q.kwords + (uint64_t)blk * kKeyWordStride;
  uint64_t w = ld_agent64(wp);
  if ((uint32_t)w != Q.epoch) {
    const uint64_t t0 = wall_clock64();
    for (;;) {
      __builtin_amdgcn_s_sleep(8);
      w = ld_agent64(wp);
      if ((uint32_t)w == Q.epoch) break;
      if (ld_err(Q)) return;
      if (wall_clock64() - t0 > Q.timeout_ticks) {
        __hip_atomic_store(&Q.ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
    }
    // the word was raised after the round's data landed (a host store after
    // the last push, or a stream release behind the copies); no workgroup of
    // this launch has read those lines (keys do not share lines), so an
    // agent-scope acquire for the tile's loads suffices — a system-scope one
    // per waiting tile would invalidate the XCD's L2 each time
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
#ifdef BPSR_KEYED_TRACE
  if (threadIdx.x == 0) kt[1] = wall_clock64();
#endif
  const uint32_t perm = (uint32_t)(w >> 32);
  if (perm == kKeySkip) {
    keep_prefetch(pf);
    key_tile_done<NT>(Q, blk, true);  // nothing stored: the count stays per epoch
    return;
  }
  if (Q.wide) {
    // 9..16 workers: the order's positions 8..15 are in the block's second
    // word, released before the first (it may still be on its way here)
    const uint64_t* hp = Q.kwords + (uint64_t)(Q.nblocks + blk) * kKeyWordStride;
    uint64_t hi = ld_agent64(hp);
    const uint64_t t0 = wall_clock64();
    while ((uint32_t)hi != Q.epoch) {
      __builtin_amdgcn_s_sleep(2);
      hi = ld_agent64(hp);
      if (wall_clock64() - t0 > Q.timeout_ticks) {
        __hip_atomic_store(&Q.ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
    }
    const uint64_t perm64 = ((hi >> 32) << 32) | perm;
    const unsigned char* const* m =
        reinterpret_cast<const unsigned char* const*>(rec + kTileHeadBytes);
    const PermSrcs16 ps{m, perm64};
    if (r.kind == kTileElem) {
      const BatchEntry& e = Q.L.entries[r.b];
      fold_elements<Op, PermSrcs16>(PermSrcs16{e.srcs, perm64}, e.n, e.dst, e.g,
                                    e.aligned != 0, (uint64_t)r.a * kBlock + threadIdx.x,
                                    (uint64_t)r.c * kBlock);
    } else if (r.kind == kTileFull) {
      fold_tile_full_buf<Op, VPT, NT, 0, NoMid, PermSrcs16>(ps, ps, (int)r.n, r.dst, 0,
                                                            threadIdx.x);
    } else {
      fold_tile_body<Op, VPT, NT, 0, true, PermSrcs16>(ps, ps, (int)r.n, r.dst, 0, 0, r.a,
                                                        threadIdx.x);
    }
    keep_prefetch(pf);
    key_tile_done<NT>(Q, blk, r.kind == kTileFull && NT == kPolWt);
    return;
  }
  // fast path: the 8 pointers permuted in registers (selects); element work
  // and the NaN replay index the pointer arrays in memory through the order
  // (no per-lane array, so no scratch)
  const unsigned char* q[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const uint32_t wk = (perm >> (4 * m)) & 7u;
    const unsigned char* v = r.p[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) v = wk == (uint32_t)k ? r.p[k] : v;
    q[m] = v;
  }
  const PermSrcs xs{reinterpret_cast<const unsigned char* const*>(rec + kTileHeadBytes), perm};
  if (r.kind == kTileElem) {
    const BatchEntry& e = Q.L.entries[r.b];
    fold_elements<Op, PermSrcs>(PermSrcs{e.srcs, perm}, e.n, e.dst, e.g, e.aligned != 0,
                                (uint64_t)r.a * kBlock + threadIdx.x, (uint64_t)r.c * kBlock);
  } else if (r.kind == kTileFull) {
    fold_tile_full_buf<Op, VPT, NT, -8, NoMid, PermSrcs>(q, xs, (int)r.n, r.dst, 0,
                                                         threadIdx.x);
  } else {
    fold_tile_body<Op, VPT, NT, -8, true, PermSrcs>(q, xs, (int)r.n, r.dst, 0, 0, r.a,
                                                     threadIdx.x);
  }
  keep_prefetch(pf);
#ifdef BPSR_KEYED_TRACE
  if (threadIdx.x == 0) kt[2] = wall_clock64();
#endif
  key_tile_done<NT>(Q, blk, r.kind == kTileFull && NT == kPolWt);
#ifdef BPSR_KEYED_TRACE
  if (threadIdx.x == 0) kt[3] = wall_clock64();
#endif
}

// ------------------------------------------------------------- launchers ----

// One launch of `kernel(arg)`; with `stop`, the kernel's own completion
// signal completes the event (hipExtLaunchKernel) — no marker packet behind it.
template <class K, class A>
static hipError_t launch_with_stop(K kernel, uint32_t grid, size_t lds, hipStream_t s,
                                   hipEvent_t stop, const A& arg) {
  if (stop)
    hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), (uint32_t)lds, s, nullptr, stop, 0, arg);
  else
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), lds, s, arg);
  return hipGetLastError();
}

template <class Op, int VPT, int NT, int NS>
static hipError_t launch_fold_ns(const FoldArgs& a, const Tuning& tu, hipStream_t s) {
  static KernelAttr attr;
  const hipError_t lds_ok =
      allow_lds(attr, reinterpret_cast<const void*>(&fold_kernel<Op, VPT, NT, NS>));
  if (lds_ok != hipSuccess) return lds_ok;
  FoldArgs b = a;
  b.grid = (uint32_t)fold_grid(a.g, tu, VPT);   // the kernel strides by its own grid
  hipLaunchKernelGGL((fold_kernel<Op, VPT, NT, NS>), dim3(b.grid), dim3(kBlock),
                     occ_lds_bytes(launch_occ(tu, b.grid, false)), s, b);
  return hipGetLastError();
}

template <class Op, int VPT, int NT>
static hipError_t launch_fold_vpt(const FoldArgs& a, const Tuning& tu, hipStream_t s) {
  switch (a.n) {  // compile-time source counts for the common worker counts
    case 2: return launch_fold_ns<Op, VPT, NT, 2>(a, tu, s);
    case 8: return launch_fold_ns<Op, VPT, NT, 8>(a, tu, s);
    case 16: return launch_fold_ns<Op, VPT, NT, 16>(a, tu, s);
    default: return launch_fold_ns<Op, VPT, NT, 0>(a, tu, s);
  }
}

template <class Op, int NT>
static hipError_t launch_fold_pol(const FoldArgs& a, int vpt, const Tuning& tu, hipStream_t s) {
  switch (vpt) {
    case 1: return launch_fold_vpt<Op, 1, NT>(a, tu, s);
    case 4: return launch_fold_vpt<Op, 4, NT>(a, tu, s);
    default: return launch_fold_vpt<Op, 2, NT>(a, tu, s);
  }
}

template <class Op>
static hipError_t launch_fold_op(const FoldArgs& a, const Tuning& tu, hipStream_t s) {
  int vpt = fold_vpt(a.g.nvec, tu.vpt);
  const int pol = cache_pol(tu, a.g.nvec * 16);
  Tuning t = tu;
  if (pol == kPolWt && vpt == 2 && tu.occ == 1 && a.g.nvec * 16 >= kHalfTileMinBytes) {
    // 64-96 MiB per source: 4-KiB tiles at 2 workgroups per CU (the same
    // bytes in flight per CU, half the time per tile, so half the drain at
    // the launch's end) — 2-7 % faster there
    vpt = 1;
    t.occ = 2;
  }
  switch (pol) {
    case kPolNt: return launch_fold_pol<Op, kPolNt>(a, vpt, t, s);
    case kPolWt: return launch_fold_pol<Op, kPolWt>(a, vpt, t, s);
    default: return launch_fold_pol<Op, kPolPlain>(a, vpt, t, s);
  }
}

template <class Op, int VPT>
static hipError_t launch_batched_vpt(const BatchLaunch& L, const Tuning& tu, hipStream_t s) {
  static KernelAttr attr[3];
  const void* k[3] = {reinterpret_cast<const void*>(&batched_kernel<Op, VPT, kPolPlain>),
                      reinterpret_cast<const void*>(&batched_kernel<Op, VPT, kPolNt>),
                      reinterpret_cast<const void*>(&batched_kernel<Op, VPT, kPolWt>)};
  note_where("batched: allow_lds");
  for (int i = 0; i < 3; ++i) {
    const hipError_t ok = allow_lds(attr[i], k[i]);
    if (ok != hipSuccess) return ok;
  }
  note_where("batched: launch");
  if (L.tiles == 0) return hipSuccess;
  const size_t lds = occ_lds_bytes(launch_occ(tu, L.tiles, true));
  switch (cache_pol(tu, (uint64_t)L.tiles * VPT * kBlock * 16)) {
    case kPolNt: return launch_with_stop(batched_kernel<Op, VPT, kPolNt>, L.tiles, lds, s, L.stop, L);
    case kPolWt: return launch_with_stop(batched_kernel<Op, VPT, kPolWt>, L.tiles, lds, s, L.stop, L);
    default: return launch_with_stop(batched_kernel<Op, VPT, kPolPlain>, L.tiles, lds, s, L.stop, L);
  }
}

template <class Op>
static hipError_t launch_batched_op(const BatchLaunch& L, int vpt, const Tuning& tu,
                                    hipStream_t s) {
  switch (vpt) {
    case 1: return launch_batched_vpt<Op, 1>(L, tu, s);
    case 4: return launch_batched_vpt<Op, 4>(L, tu, s);
    default: return launch_batched_vpt<Op, 2>(L, tu, s);
  }
}

template <class Op, int VPT, int NT>
static hipError_t launch_blockq_k(const BlockqLaunch& Q, size_t lds, bool gated, hipStream_t s) {
  if (Q.keyed) {
    static KernelAttr attr_k;
    const hipError_t okk =
        allow_lds(attr_k, reinterpret_cast<const void*>(&blockq_key_kernel<Op, VPT, NT>));
    if (okk != hipSuccess) return okk;
    return launch_with_stop(blockq_key_kernel<Op, VPT, NT>, Q.grid, lds, s, Q.L.stop, Q);
  }
  if (gated) {
    static KernelAttr attr_g;
    const hipError_t okg =
        allow_lds(attr_g, reinterpret_cast<const void*>(&blockq_gate_kernel<Op, VPT, NT>));
    if (okg != hipSuccess) return okg;
    return launch_with_stop(blockq_gate_kernel<Op, VPT, NT>, Q.grid, lds, s, Q.L.stop, Q);
  }
  // the kernel's own static LDS (the record staging words) comes on top of the
  // dynamic residency request, so allow 256 B less than the CU's 160 KiB
  static KernelAttr attr_p;
  const hipError_t ok = allow_lds(attr_p, reinterpret_cast<const void*>(&blockq_kernel<Op, VPT, NT>),
                                  (int)kLdsPerCU - 256);
  if (ok != hipSuccess) return ok;
  return launch_with_stop(blockq_kernel<Op, VPT, NT>, Q.grid, lds, s, Q.L.stop, Q);
}

template <class Op, int VPT>
static hipError_t launch_blockq_vpt(const BlockqLaunch& Q, int pol, size_t lds, bool gated,
                                    hipStream_t s) {
  switch (pol) {
    case kPolNt: return launch_blockq_k<Op, VPT, kPolNt>(Q, lds, gated, s);
    case kPolWt: return launch_blockq_k<Op, VPT, kPolWt>(Q, lds, gated, s);
    default: return launch_blockq_k<Op, VPT, kPolPlain>(Q, lds, gated, s);
  }
}

template <class Op>
static hipError_t launch_blockq_op(const BlockqLaunch& Q, int vpt, int pol, size_t lds,
                                   bool gated, hipStream_t s) {
  if (Q.grid == 0) return hipSuccess;
  switch (vpt) {
    case 1: return launch_blockq_vpt<Op, 1>(Q, pol, lds, gated, s);
    case 4: return launch_blockq_vpt<Op, 4>(Q, pol, lds, gated, s);
    default: return launch_blockq_vpt<Op, 2>(Q, pol, lds, gated, s);
  }
}

}  // namespace bpsr

// One translation unit per dtype family defines its entry points with this.
#define BPSR_DEFINE_LAUNCHERS(NAME, OP)                                                   \
  namespace bpsr {                                                                        \
  hipError_t launch_fold_##NAME(const FoldArgs& a, const Tuning& tu, hipStream_t s) {     \
    return launch_fold_op<OP>(a, tu, s);                                                  \
  }                                                                                       \
  hipError_t launch_batched_##NAME(const BatchLaunch& L, int vpt, const Tuning& tu,      \
                                   hipStream_t s) {                                       \
    return launch_batched_op<OP>(L, vpt, tu, s);                                          \
  }                                                                                       \
  hipError_t launch_blockq_##NAME(const BlockqLaunch& Q, int vpt, int pol, size_t lds,    \
                                  bool gated, hipStream_t s) {                            \
    return launch_blockq_op<OP>(Q, vpt, pol, lds, gated, s);                               \
  }                                                                                       \
  }
