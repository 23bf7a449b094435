/* ORACLE / TEST INFRASTRUCTURE ONLY — the checker, never the product.
 *
 * Clean-room CPU restatement of the reference reducer
 *   byteps/common/cpu_reducer.cc:57-83   sum(dst, src, len, dtype) dispatch
 *   byteps/common/cpu_reducer.cc:85-92   _sum<T>: dst[i] = dst[i] + src[i]
 *   byteps/common/cpu_reducer.cc:94-128  _sum_float16: F16C body + scalar tail
 *   byteps/common/cpu_reducer.cc:130-207 3-operand sum (no callers upstream)
 *   byteps/common/cpu_reducer.cc:209-220 copy: 4-byte words + trailing bytes
 *   byteps/common/cpu_reducer.h:77-173   HalfBits2Float / Float2HalfBits
 * and of the server fold byteps/server/server.cc:200-273 (first arrival is the
 * accumulator, later arrivals are summed into it in arrival order).
 *
 * Pinned: tests/golden/ holds vectors produced by the reference's own compiled
 * CpuReducer (oracle/gen_golden.py + oracle/_ref/libbpsr_ref.so, flags of
 * setup.py:171-172,284-291, gcc 11.4, x86-64 with AVX+F16C), and
 * tests/test_oracle.py checks this file against them bit for bit.
 *
 * NaN rules (probed on the compiled reference, see DESIGN.md "Parity"):
 *  - fp16, element i < floor(n/8)*8 (the F16C body, cpu_reducer.cc:101-116):
 *    result = quiet(dst) if dst is NaN, else quiet(src) if src is NaN, else
 *    the x86 default NaN 0xfe00 for inf + -inf.  Payloads are kept
 *    (vcvtph2ps / vcvtps2ph truncate/extend the payload by 13 bits).
 *  - fp16, tail elements (cpu_reducer.cc:118-125): every NaN becomes 0x7fff
 *    (HalfBits2Float maps NaN to 0x7fffffff, Float2HalfBits emits 0x7fff).
 *  - fp32/fp64: quiet(dst) if dst NaN, else quiet(src), else x86 default NaN
 *    (sign set) for inf + -inf.  When BOTH operands are NaN the reference's
 *    choice depends on vector-body vs scalar-remainder position inside each
 *    OpenMP chunk, so tests compare those positions by NaN class only.
 *  - bf16 (not in the reference: common.h:52-65 has no bf16; build-defined):
 *    the fp16-body rule with bf16 payload truncation, RNE after every add.
 */
#include "bpsr_oracle.h"

#include <math.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------- bits ---- */
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint64_t d2u(double f) { uint64_t u; memcpy(&u, &f, 8); return u; }
static inline double u2d(uint64_t u) { double f; memcpy(&f, &u, 8); return f; }

static inline int f32_isnan_bits(uint32_t u) { return (u & 0x7fffffffu) > 0x7f800000u; }
static inline int f64_isnan_bits(uint64_t u) {
  return (u & 0x7fffffffffffffffull) > 0x7ff0000000000000ull;
}

/* Exact fp16 -> fp32 (what vcvtph2ps does; NaN is quieted, payload << 13). */
static inline uint32_t h2f_bits(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  if (e == 0x1f) return sign | 0x7f800000u | (m << 13) | (m ? 0x00400000u : 0u);
  if (e == 0) {
    if (m == 0) return sign;
    int sh = 0;
    while (!(m & 0x400u)) { m <<= 1; ++sh; }
    return sign | ((uint32_t)(113 - sh) << 23) | ((m & 0x3ffu) << 13);
  }
  return sign | ((e + 112u) << 23) | (m << 13);
}

/* fp32 -> fp16, round to nearest even, overflow to inf, subnormals kept.
 * NaN: quiet, payload truncated by 13 bits (vcvtps2ph with imm 0). */
static inline uint16_t f2h_bits(uint32_t x) {
  uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
  uint32_t ax = x & 0x7fffffffu;
  if (ax > 0x7f800000u) return (uint16_t)(sign | 0x7e00u | ((ax >> 13) & 0x3ffu));
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  /* >= 65520 -> inf */
  if (ax < 0x38800000u) {                                   /* < 2^-14 */
    if (ax <= 0x33000000u) return sign;                     /* <= 2^-25 -> 0 */
    uint32_t e = ax >> 23, m = (ax & 0x7fffffu) | 0x800000u;
    uint32_t shift = 126u - e;                              /* 14..24 */
    uint32_t q = m >> shift, rem = m & ((1u << shift) - 1u), half = 1u << (shift - 1u);
    if (rem > half || (rem == half && (q & 1u))) ++q;
    return (uint16_t)(sign | q);
  }
  uint32_t v = ax - 0x38000000u;
  v += 0xfffu + ((v >> 13) & 1u);
  return (uint16_t)(sign | (v >> 13));
}

/* bf16 <-> fp32 (build-defined dtype). */
static inline uint32_t bf2f_bits(uint16_t h) { return (uint32_t)h << 16; }
static inline uint16_t f2bf_bits(uint32_t x) {
  if (f32_isnan_bits(x)) return (uint16_t)((x >> 16) | 0x0040u);
  x += 0x7fffu + ((x >> 16) & 1u);
  return (uint16_t)(x >> 16);
}

/* Restatement of cpu_reducer.h:77-111 HalfBits2Float: any NaN -> 0x7fffffff. */
static inline uint32_t h2f_tail_bits(uint16_t h) {
  if ((h & 0x7c00u) == 0x7c00u && (h & 0x3ffu)) return 0x7fffffffu;
  return h2f_bits(h);
}
/* Restatement of cpu_reducer.h:113-173 Float2HalfBits: NaN -> 0x7fff, else RNE. */
static inline uint16_t f2h_tail_bits(uint32_t x) {
  if (f32_isnan_bits(x)) return 0x7fffu;
  return f2h_bits(x);
}

/* x86 addition with the precedence the compiled reference shows. */
static inline uint32_t add_f32_bits(uint32_t a, uint32_t b) {
  if (f32_isnan_bits(a)) return a | 0x00400000u;
  if (f32_isnan_bits(b)) return b | 0x00400000u;
  uint32_t r = f2u(u2f(a) + u2f(b));
  return f32_isnan_bits(r) ? 0xffc00000u : r;
}
static inline uint64_t add_f64_bits(uint64_t a, uint64_t b) {
  if (f64_isnan_bits(a)) return a | 0x0008000000000000ull;
  if (f64_isnan_bits(b)) return b | 0x0008000000000000ull;
  uint64_t r = d2u(u2d(a) + u2d(b));
  return f64_isnan_bits(r) ? 0xfff8000000000000ull : r;
}

static inline uint16_t add_f16_body(uint16_t d, uint16_t s) {
  return f2h_bits(add_f32_bits(h2f_bits(d), h2f_bits(s)));
}
static inline uint16_t add_f16_tail(uint16_t d, uint16_t s) {
  return f2h_tail_bits(f2u(u2f(h2f_tail_bits(d)) + u2f(h2f_tail_bits(s))));
}
static inline uint16_t add_bf16(uint16_t d, uint16_t s) {
  return f2bf_bits(add_f32_bits(bf2f_bits(d), bf2f_bits(s)));
}

float bpsr_oracle_half_to_float(uint16_t h) { return u2f(h2f_bits(h)); }
uint16_t bpsr_oracle_float_to_half(float f) { return f2h_bits(f2u(f)); }

/* ------------------------------------------------------------- kernels ---- */
#define NT(n) ((n) > 0 ? (n) : 1)

/* out[i] = a[i] + b[i]; out may alias a (in-place 2-operand form). */
static int sum_into(void* out, const void* a, const void* b, size_t len, int dtype,
                    int nthreads) {
  long long i;
  switch (dtype) {
    case ORC_FLOAT32: {
      long long n = (long long)(len / 4);
      uint32_t* o = (uint32_t*)out; const uint32_t* x = a; const uint32_t* y = b;
#pragma omp parallel for schedule(static) num_threads(NT(nthreads))
      for (i = 0; i < n; ++i) o[i] = add_f32_bits(x[i], y[i]);
      return 0;
    }
    case ORC_FLOAT64: {
      long long n = (long long)(len / 8);
      uint64_t* o = (uint64_t*)out; const uint64_t* x = a; const uint64_t* y = b;
#pragma omp parallel for schedule(static) num_threads(NT(nthreads))
      for (i = 0; i < n; ++i) o[i] = add_f64_bits(x[i], y[i]);
      return 0;
    }
    case ORC_FLOAT16: {
      long long n = (long long)(len / 2), body = (n / 8) * 8;
      uint16_t* o = (uint16_t*)out; const uint16_t* x = a; const uint16_t* y = b;
#pragma omp parallel for schedule(static) num_threads(NT(nthreads))
      for (i = 0; i < body; ++i) o[i] = add_f16_body(x[i], y[i]);
      for (i = body; i < n; ++i) o[i] = add_f16_tail(x[i], y[i]);
      return 0;
    }
    case ORC_BFLOAT16: {
      long long n = (long long)(len / 2);
      uint16_t* o = (uint16_t*)out; const uint16_t* x = a; const uint16_t* y = b;
#pragma omp parallel for schedule(static) num_threads(NT(nthreads))
      for (i = 0; i < n; ++i) o[i] = add_bf16(x[i], y[i]);
      return 0;
    }
    case ORC_UINT8:
    case ORC_INT8: {  /* two's complement wrap: same bits for signed/unsigned */
      long long n = (long long)len;
      uint8_t* o = (uint8_t*)out; const uint8_t* x = a; const uint8_t* y = b;
#pragma omp parallel for schedule(static) num_threads(NT(nthreads))
      for (i = 0; i < n; ++i) o[i] = (uint8_t)(x[i] + y[i]);
      return 0;
    }
    case ORC_INT32: {
      long long n = (long long)(len / 4);
      uint32_t* o = (uint32_t*)out; const uint32_t* x = a; const uint32_t* y = b;
#pragma omp parallel for schedule(static) num_threads(NT(nthreads))
      for (i = 0; i < n; ++i) o[i] = x[i] + y[i];
      return 0;
    }
    case ORC_INT64: {
      long long n = (long long)(len / 8);
      uint64_t* o = (uint64_t*)out; const uint64_t* x = a; const uint64_t* y = b;
#pragma omp parallel for schedule(static) num_threads(NT(nthreads))
      for (i = 0; i < n; ++i) o[i] = x[i] + y[i];
      return 0;
    }
    default:
      return -1;  /* reference: BPS_CHECK(0) abort (cpu_reducer.cc:79-80) */
  }
}

int bpsr_oracle_sum(void* dst, const void* src, size_t len, int dtype, int nthreads) {
  return sum_into(dst, dst, src, len, dtype, nthreads);
}

int bpsr_oracle_sum3(void* dst, const void* src1, const void* src2, size_t len,
                     int dtype, int nthreads) {
  return sum_into(dst, src1, src2, len, dtype, nthreads);
}

int bpsr_oracle_copy(void* dst, const void* src, size_t len, int nthreads) {
  long long i, n = (long long)(len / 4);
  uint32_t* o = (uint32_t*)dst; const uint32_t* x = (const uint32_t*)src;
#pragma omp parallel for schedule(static) num_threads(NT(nthreads))
  for (i = 0; i < n; ++i) o[i] = x[i];
  if (len % 4) memcpy((char*)dst + 4 * n, (const char*)src + 4 * n, len % 4);
  return 0;
}

/* CPU-baseline form of sum (bench.py's cpu_baseline leg; still test
 * infrastructure): the reference's own loop shape, cpu_reducer.cc:85-92
 * `#pragma omp parallel for simd` over storage-type adds, built for AVX like
 * the reference (setup.py:171-172).  Same bits as bpsr_oracle_sum for every
 * non-NaN input (IEEE add in the storage type; integers wrap); which payload
 * a NaN+NaN keeps follows the compiler's operand order, as in the reference
 * (tests compare those by class).  fp16/bf16 are not vectorised here: -1, and
 * the caller uses bpsr_oracle_sum. */
__attribute__((target("avx")))
int bpsr_oracle_sum_simd(void* dst, const void* src, size_t len, int dtype, int nthreads) {
  long long i;
  switch (dtype) {
    case ORC_FLOAT32: {
      long long n = (long long)(len / 4);
      float* o = (float*)dst; const float* x = (const float*)src;
#pragma omp parallel for simd num_threads(NT(nthreads))
      for (i = 0; i < n; ++i) o[i] = o[i] + x[i];
      return 0;
    }
    case ORC_FLOAT64: {
      long long n = (long long)(len / 8);
      double* o = (double*)dst; const double* x = (const double*)src;
#pragma omp parallel for simd num_threads(NT(nthreads))
      for (i = 0; i < n; ++i) o[i] = o[i] + x[i];
      return 0;
    }
    case ORC_UINT8:
    case ORC_INT8: {
      long long n = (long long)len;
      uint8_t* o = (uint8_t*)dst; const uint8_t* x = (const uint8_t*)src;
#pragma omp parallel for simd num_threads(NT(nthreads))
      for (i = 0; i < n; ++i) o[i] = (uint8_t)(o[i] + x[i]);
      return 0;
    }
    case ORC_INT32: {
      long long n = (long long)(len / 4);
      uint32_t* o = (uint32_t*)dst; const uint32_t* x = (const uint32_t*)src;
#pragma omp parallel for simd num_threads(NT(nthreads))
      for (i = 0; i < n; ++i) o[i] = o[i] + x[i];
      return 0;
    }
    case ORC_INT64: {
      long long n = (long long)(len / 8);
      uint64_t* o = (uint64_t*)dst; const uint64_t* x = (const uint64_t*)src;
#pragma omp parallel for simd num_threads(NT(nthreads))
      for (i = 0; i < n; ++i) o[i] = o[i] + x[i];
      return 0;
    }
    default:
      return -1;
  }
}

int bpsr_oracle_sum_n(void* dst, const void* const* srcs, int n, size_t len, int dtype,
                      int nthreads) {
  if (n < 1 || !dst || !srcs) return -2;
  if (dtype != ORC_FLOAT32 && dtype != ORC_FLOAT64 && dtype != ORC_FLOAT16 &&
      dtype != ORC_BFLOAT16 && dtype != ORC_UINT8 && dtype != ORC_INT8 &&
      dtype != ORC_INT32 && dtype != ORC_INT64)
    return -1;
  if (dst != srcs[0]) bpsr_oracle_copy(dst, srcs[0], len, nthreads);
  for (int k = 1; k < n; ++k) {
    int rc = sum_into(dst, dst, srcs[k], len, dtype, nthreads);
    if (rc) return rc;
  }
  return 0;
}
