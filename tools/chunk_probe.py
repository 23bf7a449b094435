#!/usr/bin/env python3
"""Large folds (beyond the 256 MiB headline bucket) as one launch vs a
sequence of chunk launches on the same stream (element-wise, so chunking at
16-B / 8-element boundaries gives the same bits), and by tile size.  8-way
fp32 from the 16-KiB-skewed arena, 3 rotated sets, HIP events over
back-to-back launches; exactness on windows that straddle the chunk cuts."""
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
    ap.add_argument("--sizes", default="553430176,536870912,268435456,1073741824")
    ap.add_argument("--chunks-mib", default="0,256,128,64")
    ap.add_argument("--vpts", default="2,4")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    base = red.get_tuning()
    N = 8
    st = torch.cuda.current_stream()
    for B in [int(x) for x in a.sizes.split(",")]:
        B = B // 16 * 16
        n_sets = 3 if B <= (600 << 20) else 2
        sets = []
        for s in range(n_sets):
            slots = BucketArena(N + 1, B, dev).slots()
            g = torch.Generator(device=dev)
            for k in range(N):
                g.manual_seed(100 * s + k)
                slots[k].view(torch.float32).copy_(torch.randn(B // 4, device=dev, generator=g))
            sets.append((slots[N], slots[:N]))
        torch.cuda.synchronize()
        for vpt in [int(x) for x in a.vpts.split(",")]:
            red.set_tuning(vpt=vpt)
            for cm in [int(x) for x in a.chunks_mib.split(",")]:
                C = B if cm == 0 else min(B, cm << 20)
                cuts = list(range(0, B, C))

                def step(i):
                    d, srcs = sets[i % n_sets]
                    for o in cuts:
                        ln = min(C, B - o)
                        red.sum_n(d[o:o + ln], [x[o:o + ln] for x in srcs], ln, DType.FLOAT32,
                                  stream=st)
                for i in range(n_sets):
                    step(i)
                torch.cuda.synchronize()
                ts = []
                for _ in range(3):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for i in range(a.reps):
                        step(i)
                    e1.record(st)
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) / a.reps)
                d, srcs = sets[(a.reps - 1) % n_sets]
                ok = True
                for o in [0, C, B // 2, B - (1 << 16)]:
                    o = max(0, min(o, B - (1 << 16))) // 16 * 16
                    w = slice(o // 4, o // 4 + (1 << 14))
                    ref = srcs[0].view(torch.float32)[w].clone()
                    for x in srcs[1:]:
                        ref.add_(x.view(torch.float32)[w])
                    ok = ok and bool(torch.equal(ref.view(torch.int32),
                                                 d.view(torch.float32)[w].view(torch.int32)))
                med = statistics.median(ts)
                print(json.dumps({"probe": "chunk", "bucket_bytes": B, "vpt": vpt,
                                  "chunk_mib": cm, "launches": len(cuts),
                                  "us": round(med * 1e3, 2),
                                  "frac": round((N + 1) * B / (med * 1e-3) / 8e12, 4),
                                  "exact": ok}), flush=True)
        red.set_tuning(vpt=base[0])
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
