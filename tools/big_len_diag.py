#!/usr/bin/env python3
"""Folds past 2^31 elements / 4 GiB: full-tensor and windowed comparisons
against torch's own add (diagnostic for tests/test_parity_gpu.py::
test_beyond_32bit_lengths)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from prophet_amd.dtypes import DType  # noqa: E402
from prophet_amd.reducer import GpuReducer  # noqa: E402

dev = torch.device('cuda:0')
red = GpuReducer(device=0)
for rep in range(2):
    n = (1 << 31) + 1027
    g = torch.Generator(device=dev).manual_seed(99)
    ins = [torch.randn(n, device=dev, generator=g) for _ in range(2)]
    out = torch.full((n + 64,), 7.0, device=dev)
    red.sum_n(out, ins, n * 4, DType.FLOAT32)
    torch.cuda.synchronize()
    for lo in (0, (1 << 31) - 5000, n - 9000):
        hi = min(lo + 9000, n)
        w = ins[0][lo:hi] + ins[1][lo:hi]
        bad = (out[lo:hi].view(torch.int32) != w.view(torch.int32))
        nb = int(bad.sum())
        msg = f"rep {rep} lo {lo} bad {nb}"
        if nb:
            idx = torch.nonzero(bad).flatten()
            i = int(idx[0])
            msg += (f" first {lo + i} last {lo + int(idx[-1])} out {out[lo + i].item()} "
                    f"want {w[i].item()} a {ins[0][lo + i].item()} b {ins[1][lo + i].item()}")
            full = ins[0][lo + i:lo + i + 1] + ins[1][lo + i:lo + i + 1]
            msg += f" one-elem-add {full.item()}"
        print(msg, flush=True)
    want = ins[0] + ins[1]
    print("full-tensor mismatches", int((out[:n].view(torch.int32) != want.view(torch.int32)).sum()),
          flush=True)
    del ins, out, want
    torch.cuda.empty_cache()
