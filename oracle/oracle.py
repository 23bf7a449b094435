"""ORACLE / TEST INFRASTRUCTURE ONLY — ctypes front-ends of the two CPU oracles.

* :class:`PortReducer` — the clean-room C restatement ``oracle/liboracle.so``
  (oracle/bpsr_oracle.c), available everywhere (it is built on the GPU box too).
* :class:`RefReducer` — the reference's own ``CpuReducer`` compiled from
  /root/reference by oracle/Makefile into ``oracle/_ref/libbpsr_ref.so``
  (present when that build ran in the build container; .gpurunignore keeps it
  off the GPU box, where nothing loads it).

Both expose ``sum(dst, src, len, dtype)``, ``sum3``, ``copy`` and the server
fold ``sum_n`` on numpy arrays (host memory), mirroring
byteps/common/cpu_reducer.h:49-58.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PORT_LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libbpsr_ref.so")

_vp, _sz, _int = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int


def build(ref: bool = True) -> None:
    """Compile the restatement (and the reference build when sources exist)."""
    target = "all" if ref else "port"
    subprocess.run(["make", "-s", "-C", HERE, target], check=True)


def _ptr(a) -> int:
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"]
        return a.ctypes.data
    return int(a)


class PortReducer:
    kind = "port"

    def __init__(self, nthreads: int = 4, lib_path: str = PORT_LIB):
        if not os.path.exists(lib_path):
            build(ref=False)
        self.lib = ctypes.CDLL(lib_path)
        L = self.lib
        L.bpsr_oracle_sum.argtypes = [_vp, _vp, _sz, _int, _int]
        L.bpsr_oracle_sum3.argtypes = [_vp, _vp, _vp, _sz, _int, _int]
        L.bpsr_oracle_sum_simd.argtypes = [_vp, _vp, _sz, _int, _int]
        L.bpsr_oracle_copy.argtypes = [_vp, _vp, _sz, _int]
        L.bpsr_oracle_sum_n.argtypes = [_vp, ctypes.POINTER(_vp), _int, _sz, _int, _int]
        L.bpsr_oracle_half_to_float.argtypes = [ctypes.c_uint16]
        L.bpsr_oracle_half_to_float.restype = ctypes.c_float
        L.bpsr_oracle_float_to_half.argtypes = [ctypes.c_float]
        L.bpsr_oracle_float_to_half.restype = ctypes.c_uint16
        self.nthreads = nthreads

    def sum(self, dst, src, length: int, dtype: int) -> int:
        return self.lib.bpsr_oracle_sum(_ptr(dst), _ptr(src), length, int(dtype), self.nthreads)

    def sum_simd(self, dst, src, length: int, dtype: int) -> int:
        """The vectorised CPU-baseline form (fp32/fp64/ints; -1 otherwise)."""
        return self.lib.bpsr_oracle_sum_simd(_ptr(dst), _ptr(src), length, int(dtype),
                                             self.nthreads)

    def sum3(self, dst, a, b, length: int, dtype: int) -> int:
        return self.lib.bpsr_oracle_sum3(_ptr(dst), _ptr(a), _ptr(b), length, int(dtype),
                                         self.nthreads)

    def copy(self, dst, src, length: int) -> int:
        return self.lib.bpsr_oracle_copy(_ptr(dst), _ptr(src), length, self.nthreads)

    def sum_n(self, dst, srcs, length: int, dtype: int) -> int:
        arr = (_vp * len(srcs))(*[_ptr(s) for s in srcs])
        return self.lib.bpsr_oracle_sum_n(_ptr(dst), arr, len(srcs), length, int(dtype),
                                          self.nthreads)


class RefReducer:
    """The reference CpuReducer itself (cpu_reducer.cc), via oracle/ref_shim.cc."""

    kind = "reference"

    @staticmethod
    def available() -> bool:
        return os.path.exists(REF_LIB)

    def __init__(self, nthreads: int = 4, lib_path: str = REF_LIB):
        # CpuReducer reads BYTEPS_OMP_THREAD_PER_GPU in its constructor
        # (cpu_reducer.cc:40-44).
        old = os.environ.get("BYTEPS_OMP_THREAD_PER_GPU")
        os.environ["BYTEPS_OMP_THREAD_PER_GPU"] = str(nthreads)
        try:
            self.lib = ctypes.CDLL(lib_path)
            L = self.lib
            L.bpsr_ref_create.restype = _vp
            L.bpsr_ref_destroy.argtypes = [_vp]
            L.bpsr_ref_sum.argtypes = [_vp, _vp, _vp, _sz, _int]
            L.bpsr_ref_sum3.argtypes = [_vp, _vp, _vp, _vp, _sz, _int]
            L.bpsr_ref_copy.argtypes = [_vp, _vp, _vp, _sz]
            self.handle = L.bpsr_ref_create()
        finally:
            if old is None:
                os.environ.pop("BYTEPS_OMP_THREAD_PER_GPU", None)
            else:
                os.environ["BYTEPS_OMP_THREAD_PER_GPU"] = old
        self.nthreads = nthreads

    def __del__(self):
        try:
            self.lib.bpsr_ref_destroy(self.handle)
        except Exception:
            pass

    def sum(self, dst, src, length: int, dtype: int) -> int:
        return self.lib.bpsr_ref_sum(self.handle, _ptr(dst), _ptr(src), length, int(dtype))

    def sum3(self, dst, a, b, length: int, dtype: int) -> int:
        return self.lib.bpsr_ref_sum3(self.handle, _ptr(dst), _ptr(a), _ptr(b), length,
                                      int(dtype))

    def copy(self, dst, src, length: int) -> int:
        return self.lib.bpsr_ref_copy(self.handle, _ptr(dst), _ptr(src), length)

    def sum_n(self, dst, srcs, length: int, dtype: int) -> int:
        """Server fold, server.cc:216-250: merged = first arrival, then N-1 sums."""
        if _ptr(dst) != _ptr(srcs[0]):
            self.copy(dst, srcs[0], length)
        for s in srcs[1:]:
            rc = self.sum(dst, s, length, dtype)
            if rc:
                return rc
        return 0
