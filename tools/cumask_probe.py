#!/usr/bin/env python3
"""Headline fold (8-way fp32, 256 MiB per source, skewed arena) on streams
whose CU mask leaves only part of the chip to the kernel: does a fold with
fewer CUs (fewer concurrent DRAM streams) reach a higher HBM rate?  Also the
tile size (VPT) per mask, since bytes in flight per CU then matter more.
HIP-event time per launch on the masked stream; bit-exact check once."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def masked_stream(hip, n_words: int, keep_per_word: int):
    """Every 32-bit mask word keeps its lowest `keep_per_word` bits."""
    words = (ctypes.c_uint32 * n_words)(*([((1 << keep_per_word) - 1) & 0xFFFFFFFF] * n_words))
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), n_words, words)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
    return s.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, default=256)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--keep", default="32,30,28,24,20,16")
    ap.add_argument("--shapes", default="2:1,4:1,1:2", help="vpt:workgroups-per-CU list")
    a = ap.parse_args()
    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    hip = ctypes.CDLL("libamdhip64.so")
    props = torch.cuda.get_device_properties(dev)
    n_cu = props.multi_processor_count
    n_words = (n_cu + 31) // 32
    red = GpuReducer(device=0)
    N, B = 8, int(a.mib * (1 << 20))
    sets = []
    for _ in range(3):
        s = BucketArena(N + 1, B, dev).slots()
        for t in s[:N]:
            t.view(torch.float32).copy_(torch.randn(B // 4, device=dev))
        sets.append((s[N], s[:N]))
    torch.cuda.synchronize()
    alg = (N + 1) * B
    base = red.get_tuning()
    for keep in [int(x) for x in a.keep.split(",")]:
        sh = masked_stream(hip, n_words, keep)
        ext = torch.cuda.ExternalStream(sh, device=dev)
        for shape in a.shapes.split(","):
            vpt, occ = (int(x) for x in shape.split(":"))
            red.set_tuning(vpt=vpt, occ=occ)
            with torch.cuda.stream(ext):
                def step(i):
                    d, s = sets[i % 3]
                    red.sum_n(d, s, B, DType.FLOAT32, stream=ext)
                for i in range(3):
                    step(i)
                ext.synchronize()
                ts = []
                for _ in range(5):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(ext)
                    for i in range(a.reps):
                        step(i)
                    e1.record(ext)
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) / a.reps)
                d, s = sets[(a.reps - 1) % 3]
                chk = s[0].view(torch.float32)[: 1 << 20].clone()
                for x in s[1:]:
                    chk.add_(x.view(torch.float32)[: 1 << 20])
                ok = bool(torch.equal(chk.view(torch.uint8), d[: 4 << 20]))
            med = statistics.median(ts)
            print(json.dumps({"probe": "cumask", "cus_kept": keep * n_words, "of": n_cu,
                              "vpt": vpt, "wg_per_cu": occ, "us": round(med * 1e3, 2),
                              "frac": round(alg / (med * 1e-3) / 8e12, 4),
                              "spread": round((max(ts) - min(ts)) / med, 4), "exact": ok}),
                  flush=True)
        red.set_tuning(vpt=base[0], occ=base[3])
        hip.hipStreamDestroy(ctypes.c_void_p(sh))


if __name__ == "__main__":
    main()
