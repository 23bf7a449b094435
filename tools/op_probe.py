#!/usr/bin/env python3
"""The single-call entry points of the reducer surface at one large size, each
timed over back-to-back launches (HIP events) on a skewed arena:
  sum    byteps_reduce_sum   in place dst += src    (CpuReducer::sum, cpu_reducer.cc:57-83)
  sum3   byteps_reduce_sum3  dst = s1 + s2          (cpu_reducer.cc:130-162)
  copy   byteps_reduce_copy                         (cpu_reducer.cc:209-220)
  torch_copy  torch's own device copy of the same bytes, for reference.
Algorithmic HBM bytes: sum/sum3 3B, copy 2B."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, default=256)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    B = int(a.mib * (1 << 20))
    sets = []
    for _ in range(3):
        s = BucketArena(3, B, dev).slots()
        for t in s:
            t.view(torch.float32).copy_(torch.randn(B // 4, device=dev))
        sets.append(s)
    st = torch.cuda.current_stream()
    ops = {
        "sum": (3, lambda s: red.sum(s[0], s[1], B, DType.FLOAT32, stream=st)),
        "sum3": (3, lambda s: red.sum3(s[2], s[0], s[1], B, DType.FLOAT32, stream=st)),
        "copy": (2, lambda s: red.copy(s[2], s[0], B, stream=st)),
        "torch_copy": (2, lambda s: s[2].copy_(s[0])),
    }
    for name, (k, fn) in ops.items():
        for i in range(3):
            fn(sets[i])
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(a.reps):
                fn(sets[i % 3])
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / a.reps)
        med = statistics.median(ts)
        print(json.dumps({"op": name, "bytes": B, "us": round(med * 1e3, 2),
                          "GBps": round(k * B / (med * 1e-3) / 1e9, 1),
                          "hbm_frac": round(k * B / (med * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
