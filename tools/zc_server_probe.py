#!/usr/bin/env python3
"""Upper bounds for config 1's host-resident server round (2 workers x 64 MiB
fp32 in pinned host memory, aggregate back into pinned host memory) WITHOUT
the server's staging: the fold kernel reads the pushes straight from the
pinned pages (hipHostGetDevicePointer) and writes (a) the pinned result page
directly, or (b) HBM, then a copy kernel writes the pinned mirror — as one
64 MiB key, and as the 17 BytePS partitions spread over 4 streams.  Against
these, the server's measured round (staged H2D copies, fold, mirror D2H:
3.3-3.8 ms = 33-38 GiB/s) shows what a zero-copy push path could buy.
HIP events around each round (all streams joined); exactness checked."""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    from prophet_amd.stream import _Dev, _host_device_ptr
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    N, B = 2, 64 << 20
    part = 4096000
    host = [torch.randn(B // 4).pin_memory() for _ in range(N)]
    out = torch.empty(B // 4).pin_memory()
    dsrc = [_host_device_ptr(h) for h in host]
    dout = _host_device_ptr(out)
    store = torch.empty(B, dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    main_st = torch.cuda.current_stream(dev)
    want = (host[0] + host[1]).view(torch.int32)
    cuts = [(o, min(part, B - o)) for o in range(0, B, part)]

    def rnd(mode, keys):
        pieces = [(0, B)] if keys == 1 else cuts
        ev0 = torch.cuda.Event()
        ev0.record(main_st)
        for i, (o, ln) in enumerate(pieces):
            st = streams[i % len(streams)]
            st.wait_event(ev0)
            srcs = [_Dev(p + o) for p in dsrc]
            if mode == "direct":   # fold straight into the pinned result
                red.sum_n(_Dev(dout + o), srcs, ln, DType.FLOAT32, stream=st)
            else:                  # fold into HBM, then the copy kernel writes the mirror
                red.sum_n(_Dev(store.data_ptr() + o), srcs, ln, DType.FLOAT32, stream=st)
                red.copy(_Dev(dout + o), _Dev(store.data_ptr() + o), ln, stream=st)
        for st in streams[: len(pieces)]:
            e = torch.cuda.Event()
            e.record(st)
            main_st.wait_event(e)

    for mode in ("direct", "via_hbm"):
        for keys in (1, 17):
            for _ in range(2):
                rnd(mode, keys)
            torch.cuda.synchronize()
            ts = []
            for _ in range(10):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(main_st)
                rnd(mode, keys)
                e1.record(main_st)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            out.zero_()
            rnd(mode, keys)
            torch.cuda.synchronize()
            ok = bool(torch.equal(out.view(torch.int32), want))
            med = statistics.median(ts)
            print(json.dumps({"probe": "zc_server", "mode": mode, "keys": keys, "n_workers": N,
                              "bucket_bytes": B, "round_ms": round(med, 3),
                              "gibps": round(N * B / (med * 1e-3) / (1 << 30), 2), "exact": ok}),
                  flush=True)


if __name__ == "__main__":
    main()
