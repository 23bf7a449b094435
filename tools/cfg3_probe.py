#!/usr/bin/env python3
"""cfg3 block-boundary probe: the 12 Prophet-block plans of ResNet-50 fp16
(8-way) replayed from a hipGraph, with the blocks spread over 1, 2 or 4
streams (independent buckets need no ordering between blocks) and with the
1-workgroup-per-CU residency cap on or off.  One JSON line per variant."""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--occ", default="1,0,2")
    ap.add_argument("--streams", default="1,2,4")
    a = ap.parse_args()
    import torch
    from prophet_amd.buckets import partition_all, prophet_blocks, resnet50_param_sizes
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    N, sets = 8, 3
    sizes = [n * 2 for n in resnet50_param_sizes()]
    parts = partition_all(sizes)
    blocks = prophet_blocks(len(sizes))
    total = sum(sizes)
    toff = [0]
    for n in sizes:
        toff.append(toff[-1] + n)
    data = [([torch.randn(total // 2, device=dev).half().view(torch.uint8) for _ in range(N)],
             torch.empty(total, dtype=torch.uint8, device=dev)) for _ in range(sets)]

    def views(i, p):
        w, out = data[i]
        o = toff[p.tensor] + p.offset
        return out[o:o + p.len], [x[o:o + p.len] for x in w], p.len

    by_block = [[p for p in parts if p.tensor in set(b)] for b in blocks]
    plans = [[red.make_plan([views(i, p) for p in bp], DType.FLOAT16) for bp in by_block]
             for i in range(sets)]
    base = red.get_tuning()

    def build(i, nstreams):
        main_s = torch.cuda.Stream()
        eng = [torch.cuda.Stream() for _ in range(nstreams)]

        def body():
            if nstreams == 1:
                for pl in plans[i]:
                    pl.launch(main_s)
                return
            for e in eng:
                e.wait_stream(main_s)
            for b, pl in enumerate(plans[i]):
                pl.launch(eng[b % nstreams])
            for e in eng:
                main_s.wait_stream(e)
        main_s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(main_s):
            body()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=main_s):
            body()
        return g

    ref = data[0][1].clone()
    env = {k: v for k, v in os.environ.items() if k.startswith("BPSR_")}
    for occ in [int(x) for x in a.occ.split(",")]:
        red.set_tuning(occ=occ)
        for ns in [int(x) for x in a.streams.split(",")]:
            graphs = [build(i, ns) for i in range(sets)]
            for g in graphs:
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for r in range(5):
                e0.record()
                for k in range(30):
                    graphs[k % sets].replay()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 30)
            if ns == 1 and occ == int(a.occ.split(",")[0]):
                ref = data[0][1].clone()
            ok = bool(torch.equal(data[0][1], ref))
            med = statistics.median(ts)
            print(json.dumps({"env": env, "occ": occ, "streams": ns, "ms": round(med, 4),
                              "min_ms": round(min(ts), 4),
                              "hbm_frac": round((N + 1) * total / (med * 1e-3) / 8e12, 4),
                              "same_bits": ok}), flush=True)
    red.set_tuning(occ=base[3])


if __name__ == "__main__":
    main()
