"""prophet_amd — MI355X-native gradient-bucket reduction for Prophet/BytePS.

The hot path of the reference (byteps/common/cpu_reducer.cc, called from
byteps/server/server.cc:91,127-130 and byteps/common/core_loops.cc:479-481)
re-built as hand-written CDNA4 HIP kernels behind a C ABI
(``include/bpsr/reduce.h`` -> ``prophet_amd/libbpsr.so``).

Python surface:
  * :class:`prophet_amd.reducer.GpuReducer` — mirrors ``CpuReducer``
    (``sum``/``copy``/``GetDataType``) on device pointers, through the C ABI.
  * :mod:`prophet_amd.torch_ops` — the same ops as ``torch.ops.bpsr.*``.
  * :mod:`prophet_amd.dtypes` — the reference DataType ids.
  * :mod:`prophet_amd.synth` — deterministic synthetic buckets.
"""
from .dtypes import DType, elem_size  # noqa: F401

__all__ = ["DType", "elem_size"]
