"""Loader and comparison rules for the golden vectors in tests/golden/.

Fixtures = inputs (regenerated from the manifest's parameters by
prophet_amd.synth, checked against the stored sha256) + expected output bytes
produced by the reference's own compiled CpuReducer (oracle/gen_golden.py).
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

from oracle.gen_golden import case_inputs  # deterministic input regeneration
from prophet_amd.dtypes import DType

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_cache = {}


def manifest() -> list[dict]:
    if "m" not in _cache:
        with open(os.path.join(GOLDEN, "manifest.json")) as f:
            _cache["m"] = json.load(f)["cases"]
        with open(os.path.join(GOLDEN, "outputs.bin"), "rb") as f:
            _cache["blob"] = f.read()
    return _cache["m"]


def expected(case: dict) -> np.ndarray:
    manifest()
    b = _cache["blob"][case["out_offset"]: case["out_offset"] + case["out_len"]]
    assert hashlib.sha256(b).hexdigest() == case["out_sha256"]
    return np.frombuffer(b, dtype=np.uint8).copy()


def inputs(case: dict) -> list[np.ndarray]:
    ins = case_inputs(case)
    h = hashlib.sha256()
    for x in ins:
        h.update(x.tobytes())
    assert h.hexdigest() == case["input_sha256"], "synthetic generator drifted"
    return ins


def case_id(case: dict) -> str:
    return (f"{case['id']}-{case['op']}-{DType(case['dtype']).name.lower()}-N{case['n_workers']}"
            f"-L{case['len_bytes']}-{case['value_class']}")


def _nan_mask(dtype: int, b: np.ndarray) -> np.ndarray | None:
    if dtype == DType.FLOAT32:
        u = b[: len(b) // 4 * 4].view(np.uint32)
        return (u & np.uint32(0x7FFFFFFF)) > np.uint32(0x7F800000)
    if dtype == DType.FLOAT64:
        u = b[: len(b) // 8 * 8].view(np.uint64)
        return (u & np.uint64(0x7FFFFFFFFFFFFFFF)) > np.uint64(0x7FF0000000000000)
    return None


def assert_bytes_match(dtype: int, got: np.ndarray, exp: np.ndarray, *,
                       nan_class_f32_f64: bool = True, what: str = "") -> None:
    """Bit-exact, except that for fp32/fp64 an expected-NaN element may differ
    in payload when ``nan_class_f32_f64`` (the compiled reference's NaN choice
    for NaN + NaN depends on the element's position in its OpenMP/SIMD
    schedule, see oracle/bpsr_oracle.c)."""
    got = np.asarray(got, dtype=np.uint8).ravel()
    exp = np.asarray(exp, dtype=np.uint8).ravel()
    assert got.shape == exp.shape, f"{what}: size {got.shape} != {exp.shape}"
    if np.array_equal(got, exp):
        return
    if nan_class_f32_f64:
        mg, me = _nan_mask(dtype, got), _nan_mask(dtype, exp)
        if mg is not None:
            es = 4 if dtype == DType.FLOAT32 else 8
            n = len(mg) * es
            wg = got[:n].view(np.uint32 if es == 4 else np.uint64)
            we = exp[:n].view(np.uint32 if es == 4 else np.uint64)
            bad = (wg != we) & ~(mg & me)
            if not bad.any() and np.array_equal(got[n:], exp[n:]):
                return
            idx = np.nonzero(bad)[0][:8]
            raise AssertionError(f"{what}: {int(bad.sum())} elements differ, first at {idx}: "
                                 f"got {[hex(int(wg[i])) for i in idx]} "
                                 f"exp {[hex(int(we[i])) for i in idx]}")
    idx = np.nonzero(got != exp)[0][:16]
    raise AssertionError(f"{what}: {int((got != exp).sum())} bytes differ, first at {idx}: "
                         f"got {got[idx]} exp {exp[idx]}")
