"""The C-ABI library loads here (no GPU) and exports exactly what
include/bpsr/reduce.h declares; host-only argument checks run without a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from prophet_amd import reducer
from prophet_amd.dtypes import ALL_DTYPES, elem_size

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bpsr", "reduce.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(byteps_\w+)\s*\(", text)))


def test_header_declares_expected_api():
    assert header_functions() == sorted(reducer.EXPORTS)


def test_library_exports_every_header_symbol():
    lib = reducer.load_library()
    for name in header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", reducer.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (byteps_\w+)", out))
    assert set(header_functions()) <= exported
    # every exported C-ABI name matches *byteps* (reference byteps.lds:1-8)
    assert all("byteps" in s for s in exported)


def test_version_and_dtype_sizes():
    lib = reducer.load_library()
    assert lib.byteps_reduce_version() == 1
    for dt in ALL_DTYPES:
        assert lib.byteps_reduce_dtype_size(int(dt)) == elem_size(dt)
    assert lib.byteps_reduce_dtype_size(7) == reducer.EDTYPE
    assert b"Unsupported data type" in lib.byteps_reduce_last_error()


def test_argument_errors_without_gpu():
    """Validation happens before any HIP call, so these run on a CPU host."""
    r = reducer.GpuReducer()
    with pytest.raises(reducer.ReduceError) as e:
        r.sum(0x1000, 0x2000, 64, 9)
    assert e.value.code == reducer.EDTYPE
    with pytest.raises(reducer.ReduceError) as e:
        r.sum(0x1000, 0x1004, 64, 0)          # partial overlap
    assert e.value.code == reducer.EARGS
    with pytest.raises(reducer.ReduceError) as e:
        r.sum_n(0x1000, [], 64, 0)
    assert e.value.code == reducer.EARGS
    with pytest.raises(reducer.ReduceError) as e:
        r.sum_n(0x1000, [0x1000, 0x1000], 64, 0)   # dst may alias srcs[0] only
    assert e.value.code == reducer.EARGS
    with pytest.raises(reducer.ReduceError) as e:
        r.sum_n(0x1000, [0x2000, 0x3000], 64, 0, mode=5)
    assert e.value.code == reducer.EARGS
    # zero-length calls are no-ops that succeed (reference loops run 0 times)
    r.sum(0x1000, 0x2000, 0, 0)
    r.copy(0x1000, 0x2000, 0)


def test_tuning_roundtrip():
    r = reducer.GpuReducer()
    old = r.get_tuning()
    r.set_tuning(8, 0, 512)
    assert r.get_tuning() == (8, 0, 512)
    with pytest.raises(reducer.ReduceError):
        r.set_tuning(3)
    r.set_tuning(*old)
    assert r.get_tuning() == old


def test_bucket_desc_layout_matches_header():
    # void* dst; const void* srcs[32]; size_t len; int n; int reserved;
    assert ctypes.sizeof(reducer.BucketDesc) == 8 + 32 * 8 + 8 + 4 + 4
