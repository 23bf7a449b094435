#!/usr/bin/env python3
"""byteps_reduce_copy device time per launch (20 launches captured in one
hipGraph, replayed; median of 5) at a few sizes — measurement tool."""
import json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from prophet_amd.reducer import GpuReducer
dev = torch.device("cuda:0")
red = GpuReducer(device=0)
for mib in [float(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,4,16,64,256").split(",")]:
    B = int(mib * (1 << 20))
    sets = [(torch.empty(B, dtype=torch.uint8, device=dev), torch.randint(0, 255, (B,), dtype=torch.uint8, device=dev)) for _ in range(3)]
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for d, x in sets:
            red.copy(d, x, B)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(20):
            d, x = sets[i % 3]
            red.copy(d, x, B)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / 20)
    us = statistics.median(ts)
    ok = all(torch.equal(d, x) for d, x in sets)
    print(json.dumps({"mib": mib, "us": round(us, 2), "GBps": round(2 * B / (us * 1e-6) / 1e9, 1), "exact": ok}), flush=True)
