#!/usr/bin/env python3
"""Launch-tuning and HBM-layout sweep of the fold kernel on config 2
(8 x 256 MiB fp32), with torch copy as a reference point.

Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24);
prints one JSON line per (layout, variant) with median/min kernel time and
GB/s of (N+1)*B algorithmic bytes.
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
    p.add_argument("--nt", default="1")
    p.add_argument("--grid", default="1048576")
    p.add_argument("--occ", default="0,1,2")
    p.add_argument("--layouts", default="separate,skew16k")
    a = p.parse_args()

    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer

    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[a.dtype]
    did = {"f32": DType.FLOAT32, "f16": DType.FLOAT16, "bf16": DType.BFLOAT16}[a.dtype]
    B = a.bucket_mib << 20
    N = a.workers
    s = torch.cuda.current_stream()

    def make_sets(layout):
        sets = []
        for _ in range(3):
            if layout == "separate":
                bufs = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(N + 1)]
            else:
                skew = int(layout.split("@")[0][4:-1]) * 1024   # "skew<K>k[@rep]"
                bufs = BucketArena(N + 1, B, dev, skew=skew).slots()
            for b in bufs[:N]:
                b.view(tdt).normal_()
            sets.append((bufs[N], bufs[:N]))
        return sets

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
                                      [int(x) for x in a.grid.split(",")],
                                      [int(x) for x in a.occ.split(",")]))
    alg = (N + 1) * B
    for layout in a.layouts.split(","):
        sets = make_sets(layout.split("@")[0])
        res = {v: [] for v in variants}
        res["torch_copy"] = []
        for r in range(a.rounds):
            for v in variants:
                red.set_tuning(*v)

                def fn(i, v=v):
                    d, ss = sets[i % 3]
                    red.sum_n(d, ss, B, did, stream=s)
                res[v].append(time_it(fn, a.reps))
            res["torch_copy"].append(time_it(lambda i: sets[i % 3][0].copy_(sets[i % 3][1][0]), a.reps))
        for k, ts in res.items():
            med, mn = statistics.median(ts), min(ts)
            gbps = (2 * B if k == "torch_copy" else alg) / (med * 1e-3) / 1e9
            print(json.dumps({"layout": layout, "variant": k if isinstance(k, str) else
                              {"vpt": k[0], "nt": k[1], "max_grid": k[2], "occ": k[3]},
                              "median_ms": round(med, 4), "min_ms": round(mn, 4),
                              "GBps": round(gbps, 1), "frac_8TBps": round(gbps / 8000, 4)}),
                  flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
