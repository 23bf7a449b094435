#!/usr/bin/env python3
"""Slot stride of the receive arena vs fold rate, for bucket sizes that are
not powers of two (config 4's whole VGG-16 set and its G-way shards).

A slot stride is the bucket rounded up to `align`, plus the 16 KiB skew
(prophet_amd/arena.py).  With 64 KiB rounding an odd bucket leaves the N read
streams at irregular offsets modulo the HBM interleave; rounding to a larger
power of two restores the headline's pattern (stride = 16 KiB modulo the
alignment).  8-way fp32 fold, 3 rotated arenas, HIP events over back-to-back
launches; bit-exact check against torch's left fold on a window."""
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
    ap.add_argument("--sizes", default="553430176,276715088,138357544,69178772,268435456")
    ap.add_argument("--aligns-kib", default="64,256,1024,2048,4096,8192")
    ap.add_argument("--skew", type=int, default=16 * 1024)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--pads-mib", default="0", help="extra MiB between slots (spacing test)")
    a = ap.parse_args()
    import torch
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    N = 8
    st = torch.cuda.current_stream()
    for B in [int(x) for x in a.sizes.split(",")]:
        B = B // 4 * 4
        for rnd in range(a.rounds):
            for akib, pad in [(int(x), int(y)) for x in a.aligns_kib.split(",")
                              for y in a.pads_mib.split(",")]:
                align = akib * 1024
                stride = (B + align - 1) // align * align + (pad << 20) + a.skew
                sets = []
                for s in range(3):
                    slab = torch.empty(stride * (N + 1), dtype=torch.uint8, device=dev)
                    slots = [slab[k * stride: k * stride + B] for k in range(N + 1)]
                    g = torch.Generator(device=dev)
                    for k in range(N):
                        g.manual_seed(100 * s + k)
                        slots[k].view(torch.float32).copy_(torch.randn(B // 4, device=dev,
                                                                      generator=g))
                    sets.append((slots[N], slots[:N], slab))

                def step(i):
                    d, srcs, _ = sets[i % 3]
                    red.sum_n(d, srcs, B, DType.FLOAT32, stream=st)
                for i in range(3):
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
                d, srcs, _ = sets[(a.reps - 1) % 3]
                w = slice(0, 1 << 18)
                ref = srcs[0].view(torch.float32)[w].clone()
                for x in srcs[1:]:
                    ref.add_(x.view(torch.float32)[w])
                ok = bool(torch.equal(ref.view(torch.int32), d.view(torch.float32)[w].view(torch.int32)))
                med = statistics.median(ts)
                print(json.dumps({"probe": "stride", "bucket_bytes": B, "align_kib": akib, "pad_mib": pad, "stride": stride,
                                  "stride_mod_align": stride % align if align else None,
                                  "round": rnd, "us": round(med * 1e3, 2),
                                  "frac": round((N + 1) * B / (med * 1e-3) / 8e12, 4),
                                  "exact": ok}), flush=True)
                del sets
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
