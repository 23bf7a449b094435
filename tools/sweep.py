#!/usr/bin/env python3
"""Launch-tuning sweep of the fold kernel on config 2 (8 x 256 MiB fp32), plus
reference points (torch copy, torch read-only sum) for the achievable HBM rate.

Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24);
prints one JSON line per variant with median/min kernel time and GB/s of
(N+1)*B algorithmic bytes.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workers", type=int, default=8)
    p.add_argument("--bucket-mib", type=int, default=256)
    p.add_argument("--dtype", default="f32")
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--vpt", default="1,2,4")
    p.add_argument("--nt", default="0,1")
    p.add_argument("--grid", default="512,1024,2048,4096,16384,1000000")
    a = p.parse_args()

    import torch
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer

    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[a.dtype]
    did = {"f32": DType.FLOAT32, "f16": DType.FLOAT16, "bf16": DType.BFLOAT16}[a.dtype]
    es = torch.tensor([], dtype=tdt).element_size()
    B = a.bucket_mib << 20
    n = B // es
    N = a.workers
    sets = []
    for s in range(3):
        srcs = [torch.randn(n, device=dev).to(tdt) for _ in range(N)]
        sets.append((torch.empty_like(srcs[0]), srcs))
    s = torch.cuda.current_stream()

    def time_it(fn, reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn(0)
        torch.cuda.synchronize()
        e0.record(s)
        for i in range(reps):
            fn(i)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    variants = list(itertools.product([int(x) for x in a.vpt.split(",")],
                                      [int(x) for x in a.nt.split(",")],
                                      [int(x) for x in a.grid.split(",")]))
    res = {v: [] for v in variants}
    res["torch_copy"] = []
    res["torch_readsum"] = []
    big = torch.empty(N * n, dtype=tdt, device=dev)
    big2 = torch.empty_like(big)
    for r in range(a.rounds):
        for v in variants:
            red.set_tuning(*v)

            def fn(i, v=v):
                d, ss = sets[i % 3]
                red.sum_n(d, ss, B, did, stream=s)
            res[v].append(time_it(fn, a.reps))
        res["torch_copy"].append(time_it(lambda i: big2.copy_(big), 3))
        res["torch_readsum"].append(time_it(lambda i: big.sum(), 3))
    alg = (N + 1) * B
    for k, ts in res.items():
        med, mn = statistics.median(ts), min(ts)
        if k == "torch_copy":
            gbps = 2 * N * B / (med * 1e-3) / 1e9
        elif k == "torch_readsum":
            gbps = N * B / (med * 1e-3) / 1e9
        else:
            gbps = alg / (med * 1e-3) / 1e9
        print(json.dumps({"variant": k if isinstance(k, str) else
                          {"vpt": k[0], "nt": k[1], "max_grid": k[2]},
                          "median_ms": round(med, 4), "min_ms": round(mn, 4),
                          "GBps": round(gbps, 1), "frac_8TBps": round(gbps / 8000, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
