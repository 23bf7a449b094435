"""Deterministic synthetic gradient buckets.

Worker ``k``'s bucket is generated from its own seed (``1000 + k`` by default,
SURVEY.md §8d) with a splitmix64 stream, so the data is identical across numpy
versions, hosts and the GPU box.  Used by the golden-vector generator, the
parity tests and bench.py ("data": "synthetic").

Value classes
-------------
``normal``      N(0, 1) (Box–Muller over splitmix64), cast with RNE to the dtype;
                integers: full-range random bits (exercises two's-complement wrap).
``uniform100``  U(-100, 100) — the known-answer inputs of the reference's own test,
                tests/test_mxnet.py:86-90; integers: [-100, 100).
``bits``        random bit patterns with NaN/Inf excluded (floats) — covers
                subnormals, signed zeros and overflow to inf.
``special``     ``bits`` with ~3 % of positions forced to NaN (quiet and
                signalling, either sign), ±inf, ±0 and subnormals.
"""
from __future__ import annotations

import numpy as np

from .dtypes import DType, numpy_dtype, elem_size

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(seed: int, count: int) -> np.ndarray:
    """``count`` outputs of splitmix64 started at ``seed`` (Vigna's constants)."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, count + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z & _M64


def _uniform01(seed: int, count: int) -> np.ndarray:
    # 53 high bits -> [0, 1)
    return (splitmix64(seed, count) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def _normal(seed: int, count: int) -> np.ndarray:
    half = (count + 1) // 2
    u = _uniform01(seed, 2 * half)
    u1 = 1.0 - u[:half]            # (0, 1]
    u2 = u[half:]
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.concatenate([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)])
    return z[:count]


def f64_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """RNE fp64 -> fp32 -> bf16 bits (finite inputs)."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    u = u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))
    return (u >> np.uint64(16)).astype(np.uint16)


def _float_from(dtype: DType, x: np.ndarray) -> np.ndarray:
    if dtype == DType.BFLOAT16:
        return f64_to_bf16_bits(x)
    return x.astype(numpy_dtype(dtype))


def _bits_no_nan(dtype: DType, seed: int, count: int) -> np.ndarray:
    raw = splitmix64(seed, count)
    if dtype in (DType.FLOAT16, DType.BFLOAT16):
        v = (raw & np.uint64(0xFFFF)).astype(np.uint16)
        expmask = np.uint16(0x7C00 if dtype == DType.FLOAT16 else 0x7F80)
        bad = (v & expmask) == expmask
        v[bad] ^= np.uint16(0x4000)          # clear the top exponent bit -> finite
        return v
    if dtype == DType.FLOAT32:
        v = (raw & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        bad = (v & np.uint32(0x7F800000)) == np.uint32(0x7F800000)
        v[bad] ^= np.uint32(0x40000000)
        return v.view(np.float32)
    if dtype == DType.FLOAT64:
        v = raw.copy()
        em = np.uint64(0x7FF0000000000000)
        bad = (v & em) == em
        v[bad] ^= np.uint64(0x4000000000000000)
        return v.view(np.float64)
    nb = elem_size(dtype)
    return raw.astype(np.dtype(f"u{nb}")).view(numpy_dtype(dtype))


_SPECIALS = {
    DType.FLOAT16: [0x7E00, 0xFE00, 0x7E01, 0x7C01, 0xFD55, 0x7C00, 0xFC00, 0x0000, 0x8000,
                    0x0001, 0x83FF, 0x7BFF, 0xFBFF],
    DType.BFLOAT16: [0x7FC0, 0xFFC0, 0x7FC1, 0x7F81, 0xFFAA, 0x7F80, 0xFF80, 0x0000, 0x8000,
                     0x0001, 0x807F, 0x7F7F, 0xFF7F],
    DType.FLOAT32: [0x7FC00000, 0xFFC00000, 0x7FC00001, 0x7F800001, 0xFFA5A5A5, 0x7F800000,
                    0xFF800000, 0x00000000, 0x80000000, 0x00000001, 0x807FFFFF, 0x7F7FFFFF,
                    0xFF7FFFFF],
    DType.FLOAT64: [0x7FF8000000000000, 0xFFF8000000000000, 0x7FF8000000000001,
                    0x7FF0000000000001, 0x7FF0000000000000, 0xFFF0000000000000, 0x0,
                    0x8000000000000000, 0x1, 0x7FEFFFFFFFFFFFFF],
}


def bucket(dtype: DType, n_elems: int, worker: int, value_class: str = "normal",
           seed_base: int = 1000) -> np.ndarray:
    """Worker ``worker``'s synthetic bucket of ``n_elems`` elements.

    Returns a numpy array whose ``.view(np.uint8)`` is the bucket's bytes (bf16 is
    returned as uint16 bit patterns)."""
    dtype = DType(dtype)
    seed = seed_base + worker
    is_float = dtype in (DType.FLOAT32, DType.FLOAT64, DType.FLOAT16, DType.BFLOAT16)
    if value_class == "normal":
        if is_float:
            return _float_from(dtype, _normal(seed, n_elems))
        return _bits_no_nan(dtype, seed, n_elems)
    if value_class == "uniform100":
        u = _uniform01(seed, n_elems) * 200.0 - 100.0
        if is_float:
            return _float_from(dtype, u)
        if dtype == DType.UINT8:
            return (np.floor(u).astype(np.int64) & 0xFF).astype(np.uint8)
        return np.floor(u).astype(numpy_dtype(dtype))
    if value_class in ("bits", "special"):
        v = _bits_no_nan(dtype, seed, n_elems)
        if value_class == "special" and dtype in _SPECIALS:
            sp = np.array(_SPECIALS[dtype], dtype=np.uint64)
            pick = splitmix64(seed ^ 0x5A5A5A5A, n_elems)
            hit = (pick % np.uint64(32)) == np.uint64(0)
            which = (pick >> np.uint64(8)) % np.uint64(len(sp))
            bits_dtype = np.dtype(f"u{elem_size(dtype)}")
            vb = v.view(bits_dtype)
            vb[hit] = sp[which[hit]].astype(bits_dtype)
        return v
    raise ValueError(f"unknown value class {value_class!r}")


def buckets(dtype: DType, n_elems: int, n_workers: int, value_class: str = "normal",
            seed_base: int = 1000) -> list[np.ndarray]:
    return [bucket(dtype, n_elems, k, value_class, seed_base) for k in range(n_workers)]
