// Element and 16-byte-vector add operators of the reduce path, one per
// (dtype, mode).  Device-only header, included by bpsr_kernels.hip.
//
// Every operator reproduces byteps/common/cpu_reducer.cc bit for bit
// (reference mode), including the NaN payload rules the compiled reference
// shows (oracle/bpsr_oracle.c header; DESIGN.md "Parity"):
//   fp32/fp64   quiet(dst) if dst is NaN, else quiet(src), else x86 default
//               NaN (sign set) for inf + -inf                (cpu_reducer.cc:86-91)
//   fp16 body   same rule on the fp16 payload, i < floor(n/8)*8 (cpu_reducer.cc:101-116)
//   fp16 tail   any NaN -> 0x7fff                            (cpu_reducer.cc:118-125,
//                                                             cpu_reducer.h:77-173)
//   bf16        build-defined: the fp16-body rule, RNE to bf16 after every add
// Finite fp16 results: one v_pk_add_f16 (a single RNE of the exact sum) equals
// the reference's fp32 add followed by RNE to fp16, because fp32 carries
// 24 >= 2*11+2 significand bits (double rounding is innocuous); the same
// argument covers bf16 through fp32 (24 >= 2*8+2).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bpsr {

typedef _Float16 h2_t __attribute__((ext_vector_type(2)));

struct alignas(16) vec16 { uint32_t w[4]; };

template <class To, class From>
__device__ __forceinline__ To bitcast(From x) { return __builtin_bit_cast(To, x); }

// ---------------------------------------------------------------- fp32 ----
__device__ __forceinline__ bool f32_nan(uint32_t u) { return (u & 0x7fffffffu) > 0x7f800000u; }

__device__ __forceinline__ uint32_t f32_nan_fix(uint32_t a, uint32_t b) {
  return f32_nan(a) ? (a | 0x00400000u) : (f32_nan(b) ? (b | 0x00400000u) : 0xffc00000u);
}

__device__ __forceinline__ uint32_t f32_add(uint32_t a, uint32_t b) {
  float r = bitcast<float>(a) + bitcast<float>(b);
  uint32_t u = bitcast<uint32_t>(r);
  return (r != r) ? f32_nan_fix(a, b) : u;
}

struct OpF32 {
  static constexpr int kSize = 4;
  using Acc = vec16;
  using E = uint32_t;
  using EAcc = uint32_t;
  __device__ static Acc init(const vec16& v) { return v; }
  __device__ static void accum(Acc& a, const vec16& b) {
    float r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = bitcast<float>(a.w[i]) + bitcast<float>(b.w[i]);
    bool bad = (r[0] != r[0]) | (r[1] != r[1]) | (r[2] != r[2]) | (r[3] != r[3]);
    if (__builtin_expect(bad, 0)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a.w[i] = (r[i] != r[i]) ? f32_nan_fix(a.w[i], b.w[i]) : bitcast<uint32_t>(r[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) a.w[i] = bitcast<uint32_t>(r[i]);
    }
  }
  // Fast path: plain adds; a NaN anywhere in the chain leaves a NaN in the
  // result (NaN + x = NaN, inf + -inf = NaN), so checking the result once
  // decides whether the exact NaN-payload rule must be replayed (has_nan).
  __device__ static void fast(Acc& a, const vec16& b) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a.w[i] = bitcast<uint32_t>(bitcast<float>(a.w[i]) + bitcast<float>(b.w[i]));
  }
  __device__ static bool has_nan(const Acc& a) {  // one v_cmp_u_f32 per element
    const float x0 = bitcast<float>(a.w[0]), x1 = bitcast<float>(a.w[1]);
    const float x2 = bitcast<float>(a.w[2]), x3 = bitcast<float>(a.w[3]);
    return __builtin_isnan(x0) || __builtin_isnan(x1) || __builtin_isnan(x2) ||
           __builtin_isnan(x3);
  }
  __device__ static vec16 finish(const Acc& a) { return a; }
  __device__ static Acc init_fast(const vec16& v) { return v; }
  __device__ static vec16 finish_fast(const Acc& a) { return a; }
  __device__ static EAcc init_e(E v, bool) { return v; }
  __device__ static void accum_e(EAcc& a, E b, bool) { a = f32_add(a, b); }
  __device__ static E finish_e(EAcc a, bool) { return a; }
};

// ---------------------------------------------------------------- fp64 ----
__device__ __forceinline__ bool f64_nan(uint64_t u) {
  return (u & 0x7fffffffffffffffull) > 0x7ff0000000000000ull;
}
__device__ __forceinline__ uint64_t f64_add(uint64_t a, uint64_t b) {
  double r = bitcast<double>(a) + bitcast<double>(b);
  if (__builtin_expect(r != r, 0)) {
    return f64_nan(a) ? (a | 0x0008000000000000ull)
                      : (f64_nan(b) ? (b | 0x0008000000000000ull) : 0xfff8000000000000ull);
  }
  return bitcast<uint64_t>(r);
}

struct OpF64 {
  static constexpr int kSize = 8;
  using Acc = vec16;
  using E = uint64_t;
  using EAcc = uint64_t;
  __device__ static Acc init(const vec16& v) { return v; }
  __device__ static void accum(Acc& a, const vec16& b) {
    uint64_t a0 = ((uint64_t)a.w[1] << 32) | a.w[0], a1 = ((uint64_t)a.w[3] << 32) | a.w[2];
    uint64_t b0 = ((uint64_t)b.w[1] << 32) | b.w[0], b1 = ((uint64_t)b.w[3] << 32) | b.w[2];
    a0 = f64_add(a0, b0);
    a1 = f64_add(a1, b1);
    a.w[0] = (uint32_t)a0; a.w[1] = (uint32_t)(a0 >> 32);
    a.w[2] = (uint32_t)a1; a.w[3] = (uint32_t)(a1 >> 32);
  }
  __device__ static void fast(Acc& a, const vec16& b) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    a = bitcast<vec16>(bitcast<d2>(a) + bitcast<d2>(b));
  }
  __device__ static bool has_nan(const Acc& a) {
    return f64_nan(((uint64_t)a.w[1] << 32) | a.w[0]) || f64_nan(((uint64_t)a.w[3] << 32) | a.w[2]);
  }
  __device__ static vec16 finish(const Acc& a) { return a; }
  __device__ static Acc init_fast(const vec16& v) { return v; }
  __device__ static vec16 finish_fast(const Acc& a) { return a; }
  __device__ static EAcc init_e(E v, bool) { return v; }
  __device__ static void accum_e(EAcc& a, E b, bool) { a = f64_add(a, b); }
  __device__ static E finish_e(EAcc a, bool) { return a; }
};

// ---------------------------------------------------------------- fp16 ----
__device__ __forceinline__ bool f16_nan(uint32_t h) { return (h & 0x7fffu) > 0x7c00u; }

// F16C-body NaN rule on one half: quiet(dst) else quiet(src) else 0xfe00.
__device__ __forceinline__ uint32_t f16_nan_fix(uint32_t a, uint32_t b) {
  return f16_nan(a) ? (a | 0x0200u) : (f16_nan(b) ? (b | 0x0200u) : 0xfe00u);
}

// Two packed halves: one v_pk_add_f16, NaN lanes repaired.
__device__ __forceinline__ uint32_t f16x2_add_body(uint32_t a, uint32_t b) {
  uint32_t r = bitcast<uint32_t>(bitcast<h2_t>(a) + bitcast<h2_t>(b));
  // (h & 0x7fff) + 0x03ff sets bit 15 of its 16-bit lane iff h is a NaN; no
  // carry crosses into the upper lane (max 0x7fff + 0x3ff = 0x83fe).
  uint32_t t = ((r & 0x7fff7fffu) + 0x03ff03ffu) & 0x80008000u;
  if (__builtin_expect(t != 0, 0)) {
    uint32_t lo = f16_nan(r & 0xffffu) ? f16_nan_fix(a & 0xffffu, b & 0xffffu) : (r & 0xffffu);
    uint32_t hi = f16_nan(r >> 16) ? f16_nan_fix(a >> 16, b >> 16) : (r >> 16);
    r = lo | (hi << 16);
  }
  return r;
}

__device__ __forceinline__ uint32_t f16_add_elem(uint32_t a, uint32_t b, bool tail) {
  _Float16 r = bitcast<_Float16>((uint16_t)a) + bitcast<_Float16>((uint16_t)b);
  uint32_t u = bitcast<uint16_t>(r);
  if (__builtin_expect(f16_nan(u), 0)) return tail ? 0x7fffu : f16_nan_fix(a, b);
  return u;
}

struct OpF16 {
  static constexpr int kSize = 2;
  using Acc = vec16;
  using E = uint16_t;
  using EAcc = uint16_t;
  __device__ static Acc init(const vec16& v) { return v; }
  __device__ static void accum(Acc& a, const vec16& b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a.w[i] = f16x2_add_body(a.w[i], b.w[i]);
  }
  __device__ static void fast(Acc& a, const vec16& b) {  // v_pk_add_f16 x4
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a.w[i] = bitcast<uint32_t>(bitcast<h2_t>(a.w[i]) + bitcast<h2_t>(b.w[i]));
  }
  __device__ static bool has_nan(const Acc& a) {
    // (h & 0x7fff) + 0x03ff sets bit 15 of its lane iff h is a NaN
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) t |= (a.w[i] & 0x7fff7fffu) + 0x03ff03ffu;
    return (t & 0x80008000u) != 0;
  }
  __device__ static vec16 finish(const Acc& a) { return a; }
  __device__ static Acc init_fast(const vec16& v) { return v; }
  __device__ static vec16 finish_fast(const Acc& a) { return a; }
  __device__ static EAcc init_e(E v, bool) { return v; }
  __device__ static void accum_e(EAcc& a, E b, bool tail) { a = (E)f16_add_elem(a, b, tail); }
  __device__ static E finish_e(EAcc a, bool) { return a; }
};

// ---------------------------------------------------------------- bf16 ----
__device__ __forceinline__ uint32_t f32_to_bf16_rne(uint32_t x) {
  if (f32_nan(x)) return (x >> 16) | 0x0040u;
  return (x + 0x7fffu + ((x >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ uint32_t bf16_add(uint32_t a, uint32_t b) {
  return f32_to_bf16_rne(f32_add(a << 16, b << 16));
}

struct OpBF16 {
  static constexpr int kSize = 2;
  using Acc = vec16;
  using E = uint16_t;
  using EAcc = uint16_t;
  __device__ static Acc init(const vec16& v) { return v; }
  __device__ static void accum(Acc& a, const vec16& b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t lo = bf16_add(a.w[i] & 0xffffu, b.w[i] & 0xffffu);
      uint32_t hi = bf16_add(a.w[i] >> 16, b.w[i] >> 16);
      a.w[i] = lo | (hi << 16);
    }
  }
  // Fast path: widen (shift / mask), v_pk_add_f32, then gfx950's
  // v_cvt_pk_bf16_f32 (RNE, two lanes in one instruction) — 6 VALU ops per
  // pair instead of ~16 with the integer RNE sequence, which had made the bf16
  // fold VALU-bound (0.46 of the HBM roofline).  Its NaN encoding does not
  // matter: a NaN result triggers the exact replay (has_nan).
  __device__ static void fast(Acc& a, const vec16& b) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f2 x = {bitcast<float>(a.w[i] << 16), bitcast<float>(a.w[i] & 0xffff0000u)};
      const f2 y = {bitcast<float>(b.w[i] << 16), bitcast<float>(b.w[i] & 0xffff0000u)};
      a.w[i] = bitcast<uint32_t>(__builtin_convertvector(x + y, bf2));
    }
  }
  __device__ static bool has_nan(const Acc& a) {
    uint32_t t = 0;  // (h & 0x7fff) + 0x007f sets bit 15 iff h is a bf16 NaN
#pragma unroll
    for (int i = 0; i < 4; ++i) t |= (a.w[i] & 0x7fff7fffu) + 0x007f007fu;
    return (t & 0x80008000u) != 0;
  }
  __device__ static vec16 finish(const Acc& a) { return a; }
  __device__ static Acc init_fast(const vec16& v) { return v; }
  __device__ static vec16 finish_fast(const Acc& a) { return a; }
  __device__ static EAcc init_e(E v, bool) { return v; }
  __device__ static void accum_e(EAcc& a, E b, bool) { a = (E)bf16_add(a, b); }
  __device__ static E finish_e(EAcc a, bool) { return a; }
};

// ------------------------------------------- fp16 / bf16, fp32 accumulate ----
// BYTEPS_REDUCE_MODE_ACCUM_F32: convert once, fold in fp32 (same NaN rule as
// fp32), round once.  Build-defined; not a reference mode.
__device__ __forceinline__ uint32_t h2f_bits(uint32_t h) {
  return bitcast<uint32_t>((float)bitcast<_Float16>((uint16_t)h)) |
         (f16_nan(h) ? 0x00400000u : 0u);
}
__device__ __forceinline__ uint32_t f2h_bits(uint32_t x) {
  if (f32_nan(x)) return ((x >> 16) & 0x8000u) | 0x7e00u | ((x >> 13) & 0x3ffu);
  return bitcast<uint16_t>((_Float16)bitcast<float>(x));
}

template <bool BF>
struct OpAcc16 {
  static constexpr int kSize = 2;
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef _Float16 hh2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bb2 __attribute__((ext_vector_type(2)));
  struct Acc { f2 f[4]; };  // element 2i in f[i].x, 2i+1 in f[i].y
  using E = uint16_t;
  using EAcc = uint32_t;
  __device__ static uint32_t up(uint32_t h) { return BF ? (h << 16) : h2f_bits(h); }
  __device__ static uint32_t down(uint32_t x) { return BF ? f32_to_bf16_rne(x) : f2h_bits(x); }
  __device__ static uint32_t bits(float x) { return bitcast<uint32_t>(x); }
  // Exact path (NaN payload rules): element by element.
  __device__ static Acc init(const vec16& v) {
    Acc a;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a.f[i] = f2{bitcast<float>(up(v.w[i] & 0xffffu)), bitcast<float>(up(v.w[i] >> 16))};
    return a;
  }
  __device__ static void accum(Acc& a, const vec16& b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a.f[i].x = bitcast<float>(f32_add(bits(a.f[i].x), up(b.w[i] & 0xffffu)));
      a.f[i].y = bitcast<float>(f32_add(bits(a.f[i].y), up(b.w[i] >> 16)));
    }
  }
  __device__ static vec16 finish(const Acc& a) {
    vec16 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v.w[i] = down(bits(a.f[i].x)) | (down(bits(a.f[i].y)) << 16);
    return v;
  }
  // Fast path: hardware widening (v_cvt_f32_f16 / shift), v_pk_add_f32, and
  // one packed RNE narrowing per pair (v_cvt_pk_f16_f32 / v_cvt_pk_bf16_f32).
  // Any NaN reaches the result and sends the vector to the exact replay.
  __device__ static f2 widen(uint32_t w) {
    if constexpr (BF) {
      return f2{bitcast<float>(w << 16), bitcast<float>(w & 0xffff0000u)};
    } else {
      return __builtin_convertvector(bitcast<hh2>(w), f2);
    }
  }
  __device__ static Acc init_fast(const vec16& v) {
    Acc a;
#pragma unroll
    for (int i = 0; i < 4; ++i) a.f[i] = widen(v.w[i]);
    return a;
  }
  __device__ static void fast(Acc& a, const vec16& b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a.f[i] += widen(b.w[i]);
  }
  __device__ static bool has_nan(const Acc& a) {
    bool r = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) r |= __builtin_isnan(a.f[i].x) || __builtin_isnan(a.f[i].y);
    return r;
  }
  __device__ static vec16 finish_fast(const Acc& a) {
    vec16 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (BF) {
        v.w[i] = bitcast<uint32_t>(__builtin_convertvector(a.f[i], bb2));
      } else {
        v.w[i] = bitcast<uint32_t>(__builtin_convertvector(a.f[i], hh2));
      }
    }
    return v;
  }
  __device__ static EAcc init_e(E v, bool) { return up(v); }
  __device__ static void accum_e(EAcc& a, E b, bool) { a = f32_add(a, up(b)); }
  __device__ static E finish_e(EAcc a, bool) { return (E)down(a); }
};

// ------------------------------------------------------------- integers ----
struct OpI8 {  // uint8 and int8: identical two's-complement bits
  static constexpr int kSize = 1;
  using Acc = vec16;
  using E = uint8_t;
  using EAcc = uint8_t;
  __device__ static Acc init(const vec16& v) { return v; }
  __device__ static void accum(Acc& a, const vec16& b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // SWAR: 4 byte adds per dword, no cross-byte carry
      uint32_t x = a.w[i], y = b.w[i];
      a.w[i] = ((x & 0x7f7f7f7fu) + (y & 0x7f7f7f7fu)) ^ ((x ^ y) & 0x80808080u);
    }
  }
  __device__ static void fast(Acc& a, const vec16& b) { accum(a, b); }
  __device__ static bool has_nan(const Acc&) { return false; }
  __device__ static vec16 finish(const Acc& a) { return a; }
  __device__ static Acc init_fast(const vec16& v) { return v; }
  __device__ static vec16 finish_fast(const Acc& a) { return a; }
  __device__ static EAcc init_e(E v, bool) { return v; }
  __device__ static void accum_e(EAcc& a, E b, bool) { a = (E)(a + b); }
  __device__ static E finish_e(EAcc a, bool) { return a; }
};

struct OpI32 {
  static constexpr int kSize = 4;
  using Acc = vec16;
  using E = uint32_t;
  using EAcc = uint32_t;
  __device__ static Acc init(const vec16& v) { return v; }
  __device__ static void accum(Acc& a, const vec16& b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a.w[i] += b.w[i];
  }
  __device__ static void fast(Acc& a, const vec16& b) { accum(a, b); }
  __device__ static bool has_nan(const Acc&) { return false; }
  __device__ static vec16 finish(const Acc& a) { return a; }
  __device__ static Acc init_fast(const vec16& v) { return v; }
  __device__ static vec16 finish_fast(const Acc& a) { return a; }
  __device__ static EAcc init_e(E v, bool) { return v; }
  __device__ static void accum_e(EAcc& a, E b, bool) { a += b; }
  __device__ static E finish_e(EAcc a, bool) { return a; }
};

struct OpI64 {
  static constexpr int kSize = 8;
  using Acc = vec16;
  using E = uint64_t;
  using EAcc = uint64_t;
  __device__ static Acc init(const vec16& v) { return v; }
  __device__ static void accum(Acc& a, const vec16& b) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      uint64_t x = ((uint64_t)a.w[2 * i + 1] << 32) | a.w[2 * i];
      uint64_t y = ((uint64_t)b.w[2 * i + 1] << 32) | b.w[2 * i];
      x += y;
      a.w[2 * i] = (uint32_t)x; a.w[2 * i + 1] = (uint32_t)(x >> 32);
    }
  }
  __device__ static void fast(Acc& a, const vec16& b) { accum(a, b); }
  __device__ static bool has_nan(const Acc&) { return false; }
  __device__ static vec16 finish(const Acc& a) { return a; }
  __device__ static Acc init_fast(const vec16& v) { return v; }
  __device__ static vec16 finish_fast(const Acc& a) { return a; }
  __device__ static EAcc init_e(E v, bool) { return v; }
  __device__ static void accum_e(EAcc& a, E b, bool) { a += b; }
  __device__ static E finish_e(EAcc a, bool) { return a; }
};

}  // namespace bpsr
