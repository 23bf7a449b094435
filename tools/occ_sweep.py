#!/usr/bin/env python3
"""Occupancy cap x bucket size for the 8-way fold: kernel time without host
launch overhead (20 launches captured in one hipGraph, replayed), so small
buckets measure the device, not Python.  One JSON line per (bytes, occ, vpt).
With --workers <= 4 run it under BPSR_AUTO_N=0, or the library's source-count
rule (bpsr_api.cpp tuning_for_n) replaces an occ=1 request by occ 2 / vpt 4."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--dtype", default="f32")
    p.add_argument("--workers", type=int, default=8)
    p.add_argument("--mib", default="0.25,1,2,4,8,16,32,64,128,256")
    p.add_argument("--occ", default="0,1,2,4")
    p.add_argument("--vpt", default="1,2,4")
    p.add_argument("--launches", type=int, default=20)
    a = p.parse_args()
    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    tdt = {"f32": torch.float32, "f16": torch.float16}[a.dtype]
    did = {"f32": DType.FLOAT32, "f16": DType.FLOAT16}[a.dtype]
    N = a.workers
    for mib in [float(x) for x in a.mib.split(",")]:
        B = int(mib * (1 << 20)) // 16 * 16
        sets = 3
        data = []
        for _ in range(sets):
            slots = BucketArena(N + 1, B, dev).slots()
            for t in slots[:N]:
                t.view(tdt).copy_(torch.randn(B // t.view(tdt).element_size(), device=dev))
            data.append((slots[N], slots[:N]))
        for occ in [int(x) for x in a.occ.split(",")]:
            for vpt in [int(x) for x in a.vpt.split(",")]:
                red.set_tuning(vpt=vpt, occ=occ)
                side = torch.cuda.Stream()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(side):
                    for i in range(3):
                        red.sum_n(data[i][0], data[i][1], B, did, stream=side)
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=side):
                    for i in range(a.launches):
                        d, ss = data[i % sets]
                        red.sum_n(d, ss, B, did, stream=side)
                ts = []
                for _ in range(5):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) / a.launches)
                med = statistics.median(ts)
                print(json.dumps({"mib": mib, "occ": occ, "vpt": vpt, "us": round(med * 1e3, 2),
                                  "GBps": round((N + 1) * B / (med * 1e-3) / 1e9, 1)}), flush=True)
                del g
        del data
        torch.cuda.empty_cache()
    red.set_tuning(vpt=2, occ=1)


if __name__ == "__main__":
    main()
