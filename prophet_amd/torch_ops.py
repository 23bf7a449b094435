"""torch operator surface of the reduce path (``torch.ops.bpsr.*``).

What byteps/torch would call on device tensors in place of the host
``CpuReducer`` (byteps/common/cpu_reducer.h:49-58), registered with
``torch.library`` so the ops order with the caller's torch work (they run on
the current stream of the tensors' device), show up in profiles under their
own names, and trace through ``torch.compile`` (fake implementations give the
output metadata without touching data):

====================================  ===========================================
op                                    reference / C ABI
====================================  ===========================================
``bpsr::sum_(dst, src)``              ``CpuReducer::sum(dst, src, len, dtype)``,
                                      cpu_reducer.cc:57-83 -> byteps_reduce_sum
``bpsr::sum3_(dst, a, b)``            ``CpuReducer::sum(dst, a, b, len, dtype)``,
                                      cpu_reducer.cc:130-162 -> byteps_reduce_sum3
``bpsr::copy_(dst, src)``             ``CpuReducer::copy``, cpu_reducer.cc:209-220
``bpsr::sum_n(srcs, mode) -> out``    one server round, server.cc:216-273
                                      (left fold in list order) -> byteps_reduce_sum_n
``bpsr::sum_n_out(dst, srcs, mode)``  the same into ``dst`` (``dst`` may be
                                      ``srcs[0]``: the zero-copy accumulator)
====================================  ===========================================

Tensors must be contiguous, on one CUDA (HIP) device, of one dtype among the
reference's (+ bf16) and of equal size; ``len`` is the whole tensor.  There is
no CPU kernel: a CPU tensor raises (no silent fallback).
"""
from __future__ import annotations

from typing import List

import torch

from .dtypes import from_torch
from .reducer import MODE_REFERENCE, GpuReducer, ReduceError, EARGS

_RED = None


def _red() -> GpuReducer:
    global _RED
    if _RED is None:
        _RED = GpuReducer()
    return _RED


def _check_same(dst: torch.Tensor, others) -> int:
    for t in (dst, *others):
        if t.device.type != "cuda":
            raise ReduceError(EARGS, f"bpsr ops need device tensors, got {t.device}")
        if not t.is_contiguous():
            raise ReduceError(EARGS, "bpsr ops need contiguous tensors")
        if t.dtype != dst.dtype or t.numel() != dst.numel() or t.device != dst.device:
            raise ReduceError(EARGS, "bpsr ops need tensors of one dtype, size and device")
    return dst.numel() * dst.element_size()


def _stream(t: torch.Tensor) -> int:
    return int(torch.cuda.current_stream(t.device).cuda_stream)


@torch.library.custom_op("bpsr::sum_", mutates_args=("dst",), device_types="cuda")
def sum_(dst: torch.Tensor, src: torch.Tensor) -> None:
    n = _check_same(dst, [src])
    _red().sum(dst, src, n, from_torch(dst.dtype), stream=_stream(dst))


@torch.library.custom_op("bpsr::sum3_", mutates_args=("dst",), device_types="cuda")
def sum3_(dst: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> None:
    n = _check_same(dst, [a, b])
    _red().sum3(dst, a, b, n, from_torch(dst.dtype), stream=_stream(dst))


@torch.library.custom_op("bpsr::copy_", mutates_args=("dst",), device_types="cuda")
def copy_(dst: torch.Tensor, src: torch.Tensor) -> None:
    n = _check_same(dst, [src])
    _red().copy(dst, src, n, stream=_stream(dst))


@torch.library.custom_op("bpsr::sum_n_out", mutates_args=("dst",), device_types="cuda")
def sum_n_out(dst: torch.Tensor, srcs: List[torch.Tensor], mode: int = MODE_REFERENCE) -> None:
    if not srcs:
        raise ReduceError(EARGS, "sum_n needs at least one source")
    n = _check_same(dst, srcs)
    _red().sum_n(dst, list(srcs), n, from_torch(dst.dtype), mode, stream=_stream(dst))


@torch.library.custom_op("bpsr::sum_n", mutates_args=(), device_types="cuda")
def sum_n(srcs: List[torch.Tensor], mode: int = MODE_REFERENCE) -> torch.Tensor:
    if not srcs:
        raise ReduceError(EARGS, "sum_n needs at least one source")
    out = torch.empty_like(srcs[0])
    n = _check_same(out, srcs)
    _red().sum_n(out, list(srcs), n, from_torch(out.dtype), mode, stream=_stream(out))
    return out


@sum_.register_fake
def _(dst, src):
    return None


@sum3_.register_fake
def _(dst, a, b):
    return None


@copy_.register_fake
def _(dst, src):
    return None


@sum_n_out.register_fake
def _(dst, srcs, mode=MODE_REFERENCE):
    return None


@sum_n.register_fake
def _(srcs, mode=MODE_REFERENCE):
    return torch.empty_like(srcs[0])


OPS = ("sum_", "sum3_", "copy_", "sum_n_out", "sum_n")

__all__ = ["sum_", "sum3_", "copy_", "sum_n_out", "sum_n", "OPS"]
