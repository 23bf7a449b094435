#!/usr/bin/env python3
"""What an event recorded between two folds costs, by its release scope.

HIP's default event record ends with a system-scope release (L2 writeback and
invalidate); hipEventReleaseToDevice makes it a device-scope release.  The
server records events behind its folds (round completion, lane marks, the
staging ring), so the scope matters wherever folds and events alternate.
Back-to-back 8-way folds of B bytes per source (fp16), with no event between
them, a default event after each, or a device-scope event after each; HIP
events (default flags) only at the ends of the timed block.  Not product code."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HIP_EVENT_DISABLE_TIMING = 0x2
HIP_EVENT_RELEASE_TO_DEVICE = 0x40000000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-kib", default="64,1024,4000,16384,65536,262144")
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    evs = {}
    for name, flags in (("default", HIP_EVENT_DISABLE_TIMING),
                        ("device", HIP_EVENT_DISABLE_TIMING | HIP_EVENT_RELEASE_TO_DEVICE)):
        e = ctypes.c_void_p()
        assert hip.hipEventCreateWithFlags(ctypes.byref(e), flags) == 0
        evs[name] = e
    N = 8
    for kib in [int(x) for x in a.sizes_kib.split(",")]:
        B = kib * 1024
        reps = max(10, min(a.reps, int(a.reps * 4096 / max(kib, 4096))))
        sets = []
        for s in range(3):
            slots = BucketArena(N + 1, B, dev).slots()
            for k in range(N):
                slots[k].view(torch.float16).copy_(torch.randn(B // 2, device=dev).half())
            sets.append((slots[N], slots[:N]))
        for rnd in range(2):
            for mode in ("none", "default", "device"):
                def step(i):
                    d, srcs = sets[i % 3]
                    red.sum_n(d, srcs, B, DType.FLOAT16, stream=st)
                    if mode != "none":
                        hip.hipEventRecord(evs[mode], sh)
                for i in range(3):
                    step(i)
                torch.cuda.synchronize()
                ts = []
                for _ in range(3):
                    torch.cuda._sleep(20_000_000)  # the host queues the block behind a spin
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for i in range(reps):
                        step(i)
                    e1.record(st)
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) / reps * 1e3)
                print(json.dumps({"probe": "event_scope", "bytes_per_source": B, "event": mode,
                                  "round": rnd, "us_per_fold": round(statistics.median(ts), 2)}),
                      flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
