#!/usr/bin/env python3
"""How the receive arena is allocated vs the fold's HBM rate.

The same skewed arena (prophet_amd/arena.py layout: slots = bucket rounded to
64 KiB + 16 KiB skew, N+1 slots per set, 3 rotated sets) allocated by
  torch       torch's caching allocator (what bench.py uses),
  hipmalloc   one hipMalloc per set,
  contiguous  hipExtMallocWithFlags(hipDeviceMallocContiguous) per set,
then the 8-way fp32 fold through the C ABI (byteps_reduce_sum_n), HIP events
over back-to-back launches.  Run each method in a fresh process (placement
depends on what the process allocated before).  Exactness on a window."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--method", default="torch", choices=["torch", "hipmalloc", "contiguous"])
    ap.add_argument("--sizes", default="268435456,553430176,1073741824")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer, load_library
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    lib = load_library()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                          ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    N = 8
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    for B in [int(x) for x in a.sizes.split(",")]:
        B = B // 16 * 16
        stride = (B + 65535) // 65536 * 65536 + 16384
        total = stride * (N + 1)
        sets, owned = [], []
        for s in range(3):
            if a.method == "torch":
                slab = torch.empty(total, dtype=torch.uint8, device=dev)
                owned.append(slab)
                base = slab.data_ptr()
            else:
                p = ctypes.c_void_p()
                rc = (hip.hipMalloc(ctypes.byref(p), total) if a.method == "hipmalloc" else
                      hip.hipExtMallocWithFlags(ctypes.byref(p), total,
                                                HIP_DEVICE_MALLOC_CONTIGUOUS))
                if rc != 0:
                    print(json.dumps({"probe": "alloc", "method": a.method, "bucket_bytes": B,
                                      "error": f"allocation rc={rc}"}), flush=True)
                    break
                base = p.value
                owned.append(p)
            g = torch.Generator(device=dev)
            for k in range(N):
                g.manual_seed(100 * s + k)
                t = torch.randn(B // 4, device=dev, generator=g)
                torch.cuda.synchronize()
                hip.hipMemcpy(ctypes.c_void_p(base + k * stride), ctypes.c_void_p(t.data_ptr()),
                              B, 3)
                del t
            sets.append((base + N * stride, [base + k * stride for k in range(N)]))
        if len(sets) < 3:
            continue
        torch.cuda.synchronize()
        arrs = [(d, (ctypes.c_void_p * N)(*srcs)) for d, srcs in sets]

        def step(i):
            d, arr = arrs[i % 3]
            rc = lib.byteps_reduce_sum_n(ctypes.c_void_p(d), arr, N, ctypes.c_size_t(B),
                                         int(DType.FLOAT32), 0, sh)
            assert rc == 0, rc
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
        # exactness: window of the last-folded set
        d, srcs = sets[(a.reps - 1) % 3]
        W = 1 << 16
        win = torch.empty(W // 4, dtype=torch.float32, device=dev)
        ref = None
        for sp in srcs:
            hip.hipMemcpy(ctypes.c_void_p(win.data_ptr()), ctypes.c_void_p(sp), W, 3)
            ref = win.clone() if ref is None else ref.add_(win)
        hip.hipMemcpy(ctypes.c_void_p(win.data_ptr()), ctypes.c_void_p(d), W, 3)
        ok = bool(torch.equal(ref.view(torch.int32), win.view(torch.int32)))
        med = statistics.median(ts)
        print(json.dumps({"probe": "alloc", "method": a.method, "bucket_bytes": B,
                          "us": round(med * 1e3, 2),
                          "frac": round((N + 1) * B / (med * 1e-3) / 8e12, 4),
                          "spread": round((max(ts) - min(ts)) / med, 4), "exact": ok}),
              flush=True)
        torch.cuda.synchronize()
        if a.method != "torch":
            for p in owned:
                hip.hipFree(p)
        del owned, sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
