#!/usr/bin/env python3
"""Non-uniform slot offsets for the headline fold (8-way fp32, 256 MiB per
source): slot k at k * 256 MiB + s_k, with s_k from a few structured and
random patterns (multiples of 4 KiB below 1 MiB), against the product arena's
uniform s_k = 16 KiB * k.  Every pattern is timed in each of `--rounds`
passes (patterns interleaved, so box drift hits all alike); HIP events over
back-to-back launches on 3 rotated sets; exactness on a window."""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def patterns(n_random: int, seed: int):
    """Slot k's byte offset beyond k * 256 MiB: cumulative gaps (every gap
    >= 0, so slots never overlap); the product arena is 16 KiB gaps."""
    K = 9

    def cum(gaps):
        out, o = [0], 0
        for g in gaps:
            o += g
            out.append(o)
        return out
    pats = {"uniform16k": cum([16384] * (K - 1)),
            "uniform4k": cum([4096] * (K - 1)),
            "uniform48k": cum([49152] * (K - 1)),
            "alt8k24k": cum([8192 if k % 2 else 24576 for k in range(K - 1)]),
            "growing4k": cum([4096 * (k + 1) for k in range(K - 1)]),
            "shrinking4k": cum([4096 * (K - 1 - k) for k in range(K - 1)])}
    rng = random.Random(seed)
    for i in range(n_random):
        pats[f"rand{i}"] = cum([4096 * rng.randrange(0, 17) for _ in range(K - 1)])
    return pats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--random", type=int, default=10)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    N, B = 8, 256 << 20
    span = 256 << 20
    st = torch.cuda.current_stream()
    pats = patterns(a.random, a.seed)
    res = {name: [] for name in pats}
    for rnd in range(a.rounds):
        for name, offs in pats.items():
            sets = []
            for s in range(3):
                slab = torch.empty(N * span + offs[-1] + B, dtype=torch.uint8, device=dev)
                slots = [slab[k * span + offs[k]: k * span + offs[k] + B] for k in range(N + 1)]
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
            frac = (N + 1) * B / (med * 1e-3) / 8e12
            res[name].append(frac)
            print(json.dumps({"probe": "skew_pattern", "pattern": name, "offsets_kib":
                              [o // 1024 for o in offs], "round": rnd, "us": round(med * 1e3, 2),
                              "frac": round(frac, 4), "exact": ok}), flush=True)
            del sets
            torch.cuda.empty_cache()
    summary = sorted(((statistics.mean(v), k) for k, v in res.items()), reverse=True)
    print(json.dumps({"probe": "skew_pattern_summary",
                      "mean_frac": [[k, round(m, 4)] for m, k in summary]}), flush=True)


if __name__ == "__main__":
    main()
