#!/usr/bin/env python3
"""Receive slots interleaved in chunks vs contiguous per-worker slots.

The fold's rate depends on how far apart the N source streams are in the
address space (tools/stride_probe.py --pads-mib: 0.82 with the slots 256 MiB
apart, 0.77-0.80 with them 0.5-1.3 GiB apart; config 4's 553 MB buckets never
above 0.80).  A server owns its receive slots, so it can lay a bucket out as
chunks of C bytes, chunk c of every worker (and of the output) side by side:
the streams are then at most (N+1)·C apart whatever the bucket size.  The
fold of such an arena is one batched launch (one table entry per chunk).
8-way fp32, 3 rotated arenas, HIP events over back-to-back launches,
exactness on windows."""
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
    ap.add_argument("--sizes", default="268435456,553430176")
    ap.add_argument("--chunks-kib", default="0,256,1024,4096,16384")
    ap.add_argument("--skew", type=int, default=16 * 1024)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    N = 8
    st = torch.cuda.current_stream()
    for B in [int(x) for x in a.sizes.split(",")]:
        B = B // 16 * 16
        for rnd in range(a.rounds):
            for ck in [int(x) for x in a.chunks_kib.split(",")]:
                sets = []
                for s in range(3):
                    if ck == 0:   # contiguous slots (the default arena)
                        slots = BucketArena(N + 1, B, dev, skew=a.skew).slots()
                        buckets = [(slots[N], slots[:N], B)]
                        flat = [slots[k] for k in range(N + 1)]
                        keep = slots
                    else:
                        C = ck * 1024
                        nc = (B + C - 1) // C
                        region = C + a.skew
                        slab = torch.empty(nc * (N + 1) * region, dtype=torch.uint8, device=dev)
                        buckets = []
                        for c in range(nc):
                            ln = min(C, B - c * C)
                            base = c * (N + 1) * region
                            parts = [slab[base + k * region: base + k * region + ln]
                                     for k in range(N + 1)]
                            buckets.append((parts[N], parts[:N], ln))
                        keep = slab
                        flat = None
                    g = torch.Generator(device=dev)
                    for k in range(N):
                        g.manual_seed(100 * s + k)
                        x = torch.randn(B // 4, device=dev, generator=g).view(torch.uint8)
                        o = 0
                        for (_, srcs, ln) in buckets:
                            srcs[k].copy_(x[o:o + ln])
                            o += ln
                    plan = red.make_plan(buckets, DType.FLOAT32) if len(buckets) > 1 else None
                    sets.append((buckets, keep, plan))

                def step(i):
                    buckets, _, plan = sets[i % 3]
                    if plan is None:
                        d, srcs, ln = buckets[0]
                        red.sum_n(d, srcs, ln, DType.FLOAT32, stream=st)
                    else:
                        plan.launch(st)
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
                buckets, _, _ = sets[(a.reps - 1) % 3]
                ok = True
                for bi in sorted({0, len(buckets) // 2, len(buckets) - 1}):
                    d, srcs, ln = buckets[bi]
                    m = min(ln, 1 << 16) // 4
                    ref = srcs[0].view(torch.float32)[:m].clone()
                    for x in srcs[1:]:
                        ref.add_(x.view(torch.float32)[:m])
                    ok = ok and bool(torch.equal(ref.view(torch.int32),
                                                 d.view(torch.float32)[:m].view(torch.int32)))
                med = statistics.median(ts)
                print(json.dumps({"probe": "interleave", "bucket_bytes": B, "chunk_kib": ck,
                                  "chunks": len(buckets), "round": rnd,
                                  "us": round(med * 1e3, 2),
                                  "frac": round((N + 1) * B / (med * 1e-3) / 8e12, 4),
                                  "exact": ok}), flush=True)
                for _, _, plan in sets:
                    if plan is not None:
                        plan.close()
                del sets
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
