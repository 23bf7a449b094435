"""Host-side mirror of the reference reducer surface, over the C ABI.

:class:`GpuReducer` keeps ``CpuReducer``'s method names and argument meaning
(byteps/common/cpu_reducer.h:41-58):

=====================================  =========================================
reference                              here
=====================================  =========================================
``sum(dst, src, len, dtype)``          ``GpuReducer.sum`` -> ``byteps_reduce_sum``
``sum(dst, src1, src2, len, dtype)``   ``GpuReducer.sum3`` -> ``byteps_reduce_sum3``
``copy(dst, src, len)``                ``GpuReducer.copy`` -> ``byteps_reduce_copy``
``GetDataType(int)``                   ``GpuReducer.GetDataType``
server fold, server.cc:216-273         ``GpuReducer.sum_n`` -> ``byteps_reduce_sum_n``
one Prophet block                      ``GpuReducer.sum_batched``
=====================================  =========================================

``len`` is in BYTES as in the reference.  Operands are device pointers (ints)
or torch CUDA tensors (their ``data_ptr()``); ``stream`` defaults to torch's
current stream on the operand's device so the calls order with the caller's
torch work.  Errors raise :class:`ReduceError` carrying the negative status
(the reference aborts via BPS_CHECK instead, cpu_reducer.cc:79-80).

There is no fallback: if ``libbpsr.so`` is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes
import os
from typing import Sequence

from .dtypes import DType, elem_size

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libbpsr.so")
MAX_SRCS = 32

MODE_REFERENCE = 0
MODE_ACCUM_F32 = 1

OK, EDTYPE, EARGS, EHIP, ERCCL, ETIMEOUT, ECANCELED = 0, -1, -2, -3, -4, -5, -6

_vp, _sz, _int = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int

# Every symbol include/bpsr/reduce.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "byteps_reduce_version", "byteps_reduce_init", "byteps_reduce_shutdown",
    "byteps_reduce_sum", "byteps_reduce_sum3", "byteps_reduce_sum_n",
    "byteps_reduce_sum_batched", "byteps_reduce_copy", "byteps_reduce_sync",
    "byteps_reduce_dtype_size", "byteps_reduce_last_error",
    "byteps_reduce_set_tuning", "byteps_reduce_get_tuning",
    "byteps_reduce_plan_create", "byteps_reduce_plan_launch", "byteps_reduce_plan_destroy",
    "byteps_reduce_blockq_create", "byteps_reduce_blockq_config", "byteps_reduce_blockq_launch",
    "byteps_reduce_blockq_release", "byteps_reduce_blockq_status", "byteps_reduce_blockq_destroy",
    "byteps_reduce_blockq_debug", "byteps_reduce_blockq_stream",
    "byteps_reduce_blockq_release_range", "byteps_reduce_blockq_host_releases",
    "byteps_reduce_blockq_release_host", "byteps_reduce_blockq_overlap",
    "byteps_reduce_blockq_join", "byteps_reduce_blockq_release_stream",
    "byteps_reduce_blockq_queue_ids",
)


class BucketDesc(ctypes.Structure):
    """``byteps_bucket_desc`` (include/bpsr/reduce.h)."""
    _fields_ = [("dst", _vp), ("srcs", _vp * MAX_SRCS), ("len", _sz), ("n", _int),
                ("reserved", _int)]


class ReduceError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"byteps_reduce error {code}: {msg}")
        self.code = code


_LIB = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libbpsr.so (once).  Raises if it has not been built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build it with `make -C prophet_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(path)
    L.byteps_reduce_version.restype = _int
    L.byteps_reduce_init.argtypes = [_int]
    L.byteps_reduce_sum.argtypes = [_vp, _vp, _sz, _int, _vp]
    L.byteps_reduce_sum3.argtypes = [_vp, _vp, _vp, _sz, _int, _vp]
    L.byteps_reduce_sum_n.argtypes = [_vp, ctypes.POINTER(_vp), _int, _sz, _int, _int, _vp]
    L.byteps_reduce_sum_batched.argtypes = [ctypes.POINTER(BucketDesc), _int, _int, _int, _vp]
    L.byteps_reduce_copy.argtypes = [_vp, _vp, _sz, _vp]
    L.byteps_reduce_sync.argtypes = [_vp]
    L.byteps_reduce_dtype_size.argtypes = [_int]
    L.byteps_reduce_last_error.restype = ctypes.c_char_p
    L.byteps_reduce_set_tuning.argtypes = [_int, _int, _int, _int]
    L.byteps_reduce_get_tuning.argtypes = [ctypes.POINTER(_int)] * 4
    L.byteps_reduce_plan_create.argtypes = [ctypes.POINTER(BucketDesc), _int, _int, _int,
                                            ctypes.POINTER(_vp)]
    L.byteps_reduce_plan_launch.argtypes = [_vp, _vp]
    L.byteps_reduce_plan_destroy.argtypes = [_vp]
    L.byteps_reduce_blockq_create.argtypes = [ctypes.POINTER(BucketDesc), _int,
                                              ctypes.POINTER(_int), _int, _int, _int,
                                              ctypes.POINTER(_vp)]
    L.byteps_reduce_blockq_config.argtypes = [_vp, _int, ctypes.c_double]
    L.byteps_reduce_blockq_launch.argtypes = [_vp, _vp]
    L.byteps_reduce_blockq_release.argtypes = [_vp, _int, _vp]
    L.byteps_reduce_blockq_release_range.argtypes = [_vp, _int, _int, _vp]
    L.byteps_reduce_blockq_status.argtypes = [_vp, _vp]
    L.byteps_reduce_blockq_host_releases.argtypes = [_vp, _int]
    L.byteps_reduce_blockq_release_host.argtypes = [_vp, _int, _int]
    L.byteps_reduce_blockq_destroy.argtypes = [_vp]
    L.byteps_reduce_blockq_debug.argtypes = [_vp, ctypes.POINTER(ctypes.c_uint32), _int]
    L.byteps_reduce_blockq_stream.argtypes = [_vp, ctypes.POINTER(_vp)]
    L.byteps_reduce_blockq_overlap.argtypes = [_vp, _int]
    L.byteps_reduce_blockq_join.argtypes = [_vp, _vp]
    L.byteps_reduce_blockq_release_stream.argtypes = [_vp, ctypes.POINTER(_vp)]
    L.byteps_reduce_blockq_queue_ids.argtypes = [_vp, ctypes.POINTER(ctypes.c_uint64), _int]
    _LIB = L
    return L


def _check(rc: int) -> None:
    if rc != OK:
        msg = (_LIB.byteps_reduce_last_error() or b"").decode(errors="replace")
        raise ReduceError(rc, msg)


def _ptr(x) -> int:
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return int(x.data_ptr())
    if x is None:
        return 0
    raise TypeError(f"expected a device pointer or tensor, got {type(x)!r}")


def _fits(length: int, *xs) -> None:
    """Host-side bounds check before a launch: every tensor operand holds at
    least ``length`` bytes (raw pointers carry no size and are the caller's)."""
    for x in xs:
        if hasattr(x, "data_ptr") and hasattr(x, "element_size"):
            have = int(x.numel()) * int(x.element_size())
            if int(length) > have:
                raise ValueError(f"{int(length)}-byte operation on a {have}-byte tensor")


def _stream_of(x, stream):
    if stream is not None:
        return int(getattr(stream, "cuda_stream", stream))
    if hasattr(x, "device") and getattr(x.device, "type", "") == "cuda":
        import torch
        return int(torch.cuda.current_stream(x.device).cuda_stream)
    return 0  # library default: hipStreamPerThread


class GpuReducer:
    """Drop-in for ``byteps::common::CpuReducer`` on device memory."""

    def __init__(self, device: int | None = None):
        self.lib = load_library()
        if device is not None:
            _check(self.lib.byteps_reduce_init(int(device)))

    # cpu_reducer.h:58
    @staticmethod
    def GetDataType(dtype: int) -> DType:
        return DType(dtype)

    def sum(self, dst, src, length: int, dtype: int, stream=None) -> int:
        """In place ``dst += src`` over ``length`` bytes (cpu_reducer.cc:57-83)."""
        _fits(length, dst, src)
        _check(self.lib.byteps_reduce_sum(_ptr(dst), _ptr(src), int(length), int(dtype),
                                          _stream_of(dst, stream)))
        return 0

    def sum3(self, dst, src1, src2, length: int, dtype: int, stream=None) -> int:
        """``dst = src1 + src2`` (cpu_reducer.cc:130-162)."""
        _fits(length, dst, src1, src2)
        _check(self.lib.byteps_reduce_sum3(_ptr(dst), _ptr(src1), _ptr(src2), int(length),
                                           int(dtype), _stream_of(dst, stream)))
        return 0

    def copy(self, dst, src, length: int, stream=None) -> int:
        """``length``-byte device copy (cpu_reducer.cc:209-220)."""
        _fits(length, dst, src)
        _check(self.lib.byteps_reduce_copy(_ptr(dst), _ptr(src), int(length),
                                           _stream_of(dst, stream)))
        return 0

    def sum_n(self, dst, srcs: Sequence, length: int, dtype: int,
              mode: int = MODE_REFERENCE, stream=None) -> int:
        """Left fold ``dst = ((srcs[0] + srcs[1]) + ...)`` in the given order."""
        _fits(length, dst, *srcs)
        arr = (_vp * len(srcs))(*[_ptr(s) for s in srcs])
        _check(self.lib.byteps_reduce_sum_n(_ptr(dst), arr, len(srcs), int(length),
                                            int(dtype), int(mode), _stream_of(dst, stream)))
        return 0

    def sum_batched(self, buckets: Sequence[tuple], dtype: int, mode: int = MODE_REFERENCE,
                    stream=None) -> int:
        """One launch for a block of buckets; each item is ``(dst, srcs, length)``."""
        descs = _descs(buckets)
        first = buckets[0][0] if buckets else None
        _check(self.lib.byteps_reduce_sum_batched(descs, len(buckets), int(dtype), int(mode),
                                                  _stream_of(first, stream)))
        return 0

    def make_plan(self, buckets: Sequence[tuple], dtype: int,
                  mode: int = MODE_REFERENCE) -> "Plan":
        """Upload a block's bucket table once; ``Plan.launch`` is then one
        kernel launch (graph-capturable).  Tensors in ``buckets`` must stay
        alive (and at the same addresses) for the plan's lifetime."""
        return Plan(self.lib, buckets, dtype, mode)

    def make_blockq(self, blocks: Sequence[Sequence[tuple]], dtype: int,
                    mode: int = MODE_REFERENCE) -> "BlockQueue":
        """One iteration's Prophet blocks (in release order; each a list of
        ``(dst, srcs, length)`` buckets) folded by ONE persistent launch per
        iteration that starts each block once it is released
        (``byteps_reduce_blockq_*``)."""
        return BlockQueue(self.lib, blocks, dtype, mode)

    def sync(self, stream=None) -> None:
        _check(self.lib.byteps_reduce_sync(_stream_of(None, stream)))

    def set_tuning(self, vpt: int = 0, nt: int = -1, max_grid: int = 0, occ: int = -1) -> None:
        _check(self.lib.byteps_reduce_set_tuning(vpt, nt, max_grid, occ))

    def get_tuning(self) -> tuple[int, int, int, int]:
        a, b, c, d = _int(), _int(), _int(), _int()
        _check(self.lib.byteps_reduce_get_tuning(ctypes.byref(a), ctypes.byref(b),
                                                 ctypes.byref(c), ctypes.byref(d)))
        return a.value, b.value, c.value, d.value

    @staticmethod
    def dtype_size(dtype: int) -> int:
        return elem_size(dtype)


def _descs(buckets):
    descs = (BucketDesc * max(1, len(buckets)))()
    for i, (dst, srcs, length) in enumerate(buckets):
        if len(srcs) > MAX_SRCS:
            raise ReduceError(EARGS, f"bucket {i}: more than {MAX_SRCS} sources")
        descs[i].dst = _ptr(dst)
        for k, s in enumerate(srcs):
            descs[i].srcs[k] = _ptr(s)
        descs[i].len = int(length)
        descs[i].n = len(srcs)
    return descs


class Plan:
    """``byteps_reduce_plan``: a Prophet block's bucket table resident on the device."""

    def __init__(self, lib, buckets, dtype, mode):
        self.lib = lib
        self.handle = _vp()
        self._keep = buckets          # keep the tensors alive
        self.first = buckets[0][0] if buckets else None
        _check(lib.byteps_reduce_plan_create(_descs(buckets), len(buckets), int(dtype),
                                             int(mode), ctypes.byref(self.handle)))

    def launch(self, stream=None) -> None:
        _check(self.lib.byteps_reduce_plan_launch(self.handle, _stream_of(self.first, stream)))

    def close(self) -> None:
        if self.handle:
            self.lib.byteps_reduce_plan_destroy(self.handle)
            self.handle = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BlockQueue:
    """``byteps_reduce_blockq``: a persistent consumer over an iteration's blocks.

    Per iteration: ``launch()`` once and ``release(b)`` for every block, in
    either order (epochs pair the k-th launch with the k-th release of each
    block; a block is consumed once it and all earlier blocks are released),
    ``status()`` to learn whether the launch gave up waiting."""

    def __init__(self, lib, blocks, dtype, mode):
        self.lib = lib
        self.handle = _vp()
        buckets = [b for blk in blocks for b in blk]
        ends, acc = [], 0
        for blk in blocks:
            acc += len(blk)
            ends.append(acc)
        self.nblocks = len(blocks)
        self._keep = buckets
        self.first = buckets[0][0] if buckets else None
        arr = (_int * max(1, len(ends)))(*ends)
        _check(lib.byteps_reduce_blockq_create(_descs(buckets), len(buckets), arr, len(ends),
                                               int(dtype), int(mode),
                                               ctypes.byref(self.handle)))

    def config(self, wg_per_cu: int = -1, timeout_s: float = 0.0) -> None:
        """``wg_per_cu`` 0: dispatch-ordered consumer (default); 1..8:
        persistent workgroups per CU; < 0 keeps.  ``timeout_s`` <= 0 keeps."""
        _check(self.lib.byteps_reduce_blockq_config(self.handle, int(wg_per_cu),
                                                    float(timeout_s)))

    def launch(self, stream=None) -> None:
        _check(self.lib.byteps_reduce_blockq_launch(self.handle, _stream_of(self.first, stream)))

    def release(self, block: int = -1, stream=None) -> None:
        _check(self.lib.byteps_reduce_blockq_release(self.handle, int(block),
                                                     _stream_of(self.first, stream)))

    def release_range(self, first: int, count: int, stream=None) -> None:
        """Release blocks [first, first + count) with one kernel."""
        _check(self.lib.byteps_reduce_blockq_release_range(self.handle, int(first), int(count),
                                                           _stream_of(self.first, stream)))

    def host_releases(self, on: bool = True) -> None:
        """Later launches carry a helper workgroup that forwards host
        releases (``release_host``); dispatch-ordered consumer only."""
        _check(self.lib.byteps_reduce_blockq_host_releases(self.handle, 1 if on else 0))

    def release_host(self, first: int, count: int = 1) -> None:
        """Release blocks [first, first + count) from the host: no stream, no
        kernel.  Their data must already be complete and visible to the device."""
        _check(self.lib.byteps_reduce_blockq_release_host(self.handle, int(first), int(count)))

    def overlap(self, on: bool = True) -> None:
        """Consecutive launches may overlap (byteps_reduce_blockq_overlap):
        a launch no longer orders its stream after the fold — ``join``
        before reading the outputs or rewriting the inputs."""
        _check(self.lib.byteps_reduce_blockq_overlap(self.handle, 1 if on else 0))

    def join(self, stream=None) -> None:
        """``stream`` (default: torch's current stream) waits on the device
        for every block-queue launch of the device so far."""
        _check(self.lib.byteps_reduce_blockq_join(self.handle, _stream_of(self.first, stream)))

    def status(self, stream=None) -> None:
        _check(self.lib.byteps_reduce_blockq_status(self.handle, _stream_of(self.first, stream)))

    def stream(self):
        """The device's consumer stream (byteps_reduce_blockq_stream) as a
        torch ExternalStream: launch here to skip the fork/join onto it."""
        import torch
        p = _vp()
        _check(self.lib.byteps_reduce_blockq_stream(self.handle, ctypes.byref(p)))
        return torch.cuda.ExternalStream(p.value)

    def release_stream(self):
        """The device's release stream (byteps_reduce_blockq_release_stream) as
        a torch ExternalStream: a hardware queue on a compute pipe no consumer
        queue uses — queue pushes and stream releases here."""
        import torch
        p = _vp()
        _check(self.lib.byteps_reduce_blockq_release_stream(self.handle, ctypes.byref(p)))
        return torch.cuda.ExternalStream(p.value)

    def queue_ids(self) -> dict:
        """HSA queue ids of the device's consumer queues and release queue
        (byteps_reduce_blockq_queue_ids; 0 = not made yet)."""
        ids = (ctypes.c_uint64 * 4)()
        n = self.lib.byteps_reduce_blockq_queue_ids(self.handle, ids, 4)
        if n < 0:
            _check(n)
        return {"consumer": [ids[0], ids[1], ids[2]], "release": ids[3]}

    def debug(self) -> dict:
        """byteps_reduce_blockq_debug (synchronises the device)."""
        nb = self.nblocks
        buf = (ctypes.c_uint32 * (4 + 3 * nb + 8))()
        k = self.lib.byteps_reduce_blockq_debug(self.handle, buf, len(buf))
        if k < 0:
            _check(k)
        v = list(buf[:k])
        return {"launch_epoch": v[0], "nblocks": v[1], "err": v[2],
                "rel_epoch": v[3:3 + nb], "words": v[3 + nb:3 + 2 * nb],
                "block_first": v[3 + 2 * nb:4 + 3 * nb], "table_intact": bool(v[-1])}

    def close(self) -> None:
        if self.handle:
            self.lib.byteps_reduce_blockq_destroy(self.handle)
            self.handle = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# torch-tensor convenience: whole-tensor ops with dtype taken from the tensor
def tensor_sum_n(dst, srcs, mode: int = MODE_REFERENCE, reducer: GpuReducer | None = None):
    from .dtypes import from_torch
    r = reducer or GpuReducer()
    nbytes = dst.numel() * dst.element_size()
    for s in srcs:
        if s.numel() * s.element_size() != nbytes or s.dtype != dst.dtype:
            raise ReduceError(EARGS, "sources must match dst in dtype and size")
        if not s.is_contiguous():
            raise ReduceError(EARGS, "sources must be contiguous")
    if not dst.is_contiguous():
        raise ReduceError(EARGS, "dst must be contiguous")
    r.sum_n(dst, srcs, nbytes, from_torch(dst.dtype), mode)
    return dst
