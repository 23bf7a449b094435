#!/usr/bin/env python3
"""Small-launch latency of the batched kernel vs the single-bucket fold:
20 launches captured in one hipGraph, replayed; device time per launch.
Cases: one 256 KiB bucket (fold and plan), cfg3's last Prophet blocks as
plans, and the same bytes as one bucket."""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from prophet_amd.buckets import partition_all, prophet_blocks, resnet50_param_sizes
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    N = 8
    side = torch.cuda.Stream()

    def graph_time(launch, reps=20):
        with torch.cuda.stream(side):
            launch(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            for _ in range(reps):
                launch(side)
        ts = []
        for _ in range(7):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / reps)
        return round(statistics.median(ts), 2)

    def mk(nbytes_list, dt):
        out = []
        for nb in nbytes_list:
            srcs = [torch.randn(nb // 2, device=dev).half().view(torch.uint8)[:nb] for _ in range(N)]
            out.append((torch.empty(nb, dtype=torch.uint8, device=dev), srcs, nb))
        return out

    emit = lambda **k: print(json.dumps(k), flush=True)
    for nb in (4096, 65536, 262144, 1 << 20):
        b = mk([nb], DType.FLOAT16)
        d, s, L = b[0]
        emit(case="fold", bytes=nb, us=graph_time(lambda st: red.sum_n(d, s, L, DType.FLOAT16, stream=st)))
        p = red.make_plan(b, DType.FLOAT16)
        emit(case="plan_1bucket", bytes=nb, us=graph_time(lambda st: p.launch(st)))
    sizes = [n * 2 for n in resnet50_param_sizes()]
    parts = partition_all(sizes)
    for bi, blk in enumerate(prophet_blocks(len(sizes))):
        tset = set(blk)
        lens = [p.len for p in parts if p.tensor in tset]
        b = mk(lens, DType.FLOAT16)
        p = red.make_plan(b, DType.FLOAT16)
        tot = sum(lens)
        one = mk([tot], DType.FLOAT16)
        p1 = red.make_plan(one, DType.FLOAT16)
        d, s, L = one[0]
        emit(case="block", block=bi, buckets=len(lens), bytes=tot,
             plan_us=graph_time(lambda st: p.launch(st)),
             one_bucket_plan_us=graph_time(lambda st: p1.launch(st)),
             one_bucket_fold_us=graph_time(lambda st: red.sum_n(d, s, L, DType.FLOAT16, stream=st)))


if __name__ == "__main__":
    main()
