#!/usr/bin/env python3
"""Fixed cost of one small launch, graph-replayed back to back (no host in the
loop): the floor under cfg3's small Prophet blocks.

For each variant, K identical launches are captured into one hipGraph and the
replay is timed with HIP events; us/launch = replay time / K.  Variants:
  torch_fill     torch's own 256-element fill (the chip's launch floor)
  fold_<B>       byteps_reduce_sum_n, 8 sources of B bytes fp16
  plan_<B>x<m>   one batched plan of m buckets of B bytes each, 8 sources
Prints one JSON line per variant."""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    K = 200
    N = 8

    def graph_time(launch):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                launch(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            for _ in range(K):
                launch(side)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = None
        for _ in range(5):
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) * 1e3 / K
            best = t if best is None else min(best, t)
        return best

    x = torch.empty(256, device=dev)
    print(json.dumps({"variant": "torch_fill", "us_per_launch": round(
        graph_time(lambda s: x.fill_(1.0)), 3)}), flush=True)

    for B in (1024, 65536, 1 << 20):
        srcs = [torch.randn(B // 2, device=dev).half() for _ in range(N)]
        out = torch.empty_like(srcs[0])
        us = graph_time(lambda s: red.sum_n(out, srcs, B, DType.FLOAT16, stream=s))
        print(json.dumps({"variant": f"fold_{B}", "us_per_launch": round(us, 3),
                          "hbm_frac": round((N + 1) * B / (us * 1e-6) / 8e12, 4)}), flush=True)

    for B, m in ((1024, 1), (1024, 16), (65536, 16), (262144, 16)):
        bufs = [([torch.randn(B // 2, device=dev).half() for _ in range(N)],
                 torch.empty(B // 2, device=dev).half()) for _ in range(m)]
        plan = red.make_plan([(o, s, B) for s, o in bufs], DType.FLOAT16)
        us = graph_time(lambda s: plan.launch(s))
        print(json.dumps({"variant": f"plan_{B}x{m}", "us_per_launch": round(us, 3),
                          "hbm_frac": round((N + 1) * B * m / (us * 1e-6) / 8e12, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
