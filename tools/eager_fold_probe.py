#!/usr/bin/env python3
"""Measurement tool: an 8-way fp32 fold of the given sizes timed eagerly (HIP
events around 20 back-to-back launches on one stream, a spin kernel first,
median of 5), from skewed arenas as the bench uses."""
import json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from prophet_amd.arena import BucketArena
from prophet_amd.dtypes import DType
from prophet_amd.reducer import GpuReducer
dev = torch.device("cuda:0")
red = GpuReducer(device=0)
N, reps = 8, 20
for nbytes in [int(x) for x in sys.argv[1].split(",")]:
    data = []
    for s in range(3):
        slots = BucketArena(N + 1, nbytes, dev).slots()
        for t in slots[:N]:
            t.view(torch.float32).copy_(torch.randn(nbytes // 4, device=dev))
        data.append((slots[N], slots[:N]))
    st = torch.cuda.Stream()
    def launch(i):
        o, w = data[i % 3]
        red.sum_n(o, w, nbytes, DType.FLOAT32, stream=st)
    with torch.cuda.stream(st):
        for i in range(3):
            launch(i)
    torch.cuda.synchronize()
    eager = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            torch.cuda._sleep(2_000_000)
        e0.record(st)
        for i in range(reps):
            launch(i)
        e1.record(st)
        torch.cuda.synchronize()
        eager.append(e0.elapsed_time(e1) * 1e3 / reps)
    print(json.dumps({"bytes": nbytes, "eager_us": round(statistics.median(eager), 2)}),
          flush=True)
    del data
    torch.cuda.empty_cache()
