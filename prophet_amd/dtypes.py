"""Data types of the reduce path.

Ids follow the reference's ``DataType`` enum, byteps/common/common.h:52-65
(mshadow order); element sizes follow ``getDataTypeLength``,
byteps/common/common.cc:126-143.  ``BFLOAT16`` is the build's own extension:
the reference has no bf16 (common.h:52-65; byteps/torch/adapter.cc:25-45 throws
on it; cpu_reducer.cc:79-80 aborts), so its semantics are build-defined and
pinned only to this build's CPU restatement (DESIGN.md "Parity").
"""
from __future__ import annotations

import enum

import numpy as np


class DType(enum.IntEnum):
    FLOAT32 = 0
    FLOAT64 = 1
    FLOAT16 = 2
    UINT8 = 3
    INT32 = 4
    INT8 = 5
    INT64 = 6
    BFLOAT16 = 11  # build extension, outside the reference's id range


# byteps/common/common.h:52-65 names, for callers that use the reference's spelling
BYTEPS_FLOAT32 = DType.FLOAT32
BYTEPS_FLOAT64 = DType.FLOAT64
BYTEPS_FLOAT16 = DType.FLOAT16
BYTEPS_UINT8 = DType.UINT8
BYTEPS_INT32 = DType.INT32
BYTEPS_INT8 = DType.INT8
BYTEPS_INT64 = DType.INT64
BYTEPS_BFLOAT16 = DType.BFLOAT16

_SIZES = {
    DType.INT8: 1, DType.UINT8: 1, DType.FLOAT16: 2, DType.BFLOAT16: 2,
    DType.INT32: 4, DType.FLOAT32: 4, DType.INT64: 8, DType.FLOAT64: 8,
}

_NUMPY = {
    DType.FLOAT32: np.float32, DType.FLOAT64: np.float64, DType.FLOAT16: np.float16,
    DType.UINT8: np.uint8, DType.INT32: np.int32, DType.INT8: np.int8,
    DType.INT64: np.int64, DType.BFLOAT16: np.uint16,  # bf16 carried as raw bits
}

REFERENCE_DTYPES = (DType.FLOAT32, DType.FLOAT64, DType.FLOAT16, DType.UINT8,
                    DType.INT32, DType.INT8, DType.INT64)
ALL_DTYPES = REFERENCE_DTYPES + (DType.BFLOAT16,)
FLOAT_DTYPES = (DType.FLOAT32, DType.FLOAT64, DType.FLOAT16, DType.BFLOAT16)


def elem_size(dtype: int) -> int:
    """getDataTypeLength (common.cc:126-143); raises ValueError where the
    reference would BPS_CHECK-abort."""
    try:
        return _SIZES[DType(dtype)]
    except (ValueError, KeyError):
        raise ValueError(f"Unsupported data type: {dtype}") from None


def numpy_dtype(dtype: int):
    return _NUMPY[DType(dtype)]


def from_torch(tdtype) -> DType:
    """torch dtype -> DType (mirrors byteps/torch/adapter.cc:25-45, plus bf16)."""
    import torch
    table = {
        torch.float32: DType.FLOAT32, torch.float64: DType.FLOAT64,
        torch.float16: DType.FLOAT16, torch.uint8: DType.UINT8,
        torch.int32: DType.INT32, torch.int8: DType.INT8, torch.int64: DType.INT64,
        torch.bfloat16: DType.BFLOAT16,
    }
    if tdtype not in table:
        raise ValueError(f"Unsupported data type: {tdtype}")
    return table[tdtype]


def to_torch(dtype: int):
    import torch
    return {
        DType.FLOAT32: torch.float32, DType.FLOAT64: torch.float64,
        DType.FLOAT16: torch.float16, DType.UINT8: torch.uint8,
        DType.INT32: torch.int32, DType.INT8: torch.int8, DType.INT64: torch.int64,
        DType.BFLOAT16: torch.bfloat16,
    }[DType(dtype)]
