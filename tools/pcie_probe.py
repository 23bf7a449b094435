"""Probe (not product code): what the host link of one MI355X moves, per
direction and both at once, by SDMA copies (hipMemcpyAsync on pinned memory)
and by the library's copy kernel reading or writing pinned host memory through
its device view (byteps_reduce_copy), alone and mixed.  One JSON line per
case: GB/s = bytes moved / median wall time of the case.
    python tools/pcie_probe.py [--mib 64] [--reps 10]"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda", 0)
    n = a.mib << 20
    red = GpuReducer(device=0)
    hs = [torch.empty(n, dtype=torch.uint8).pin_memory() for _ in range(2)]
    ds = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(2)]
    for h in hs:
        h.fill_(7)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def sdma_h2d(s):
        with torch.cuda.stream(s):
            ds[0].copy_(hs[0], non_blocking=True)

    def sdma_d2h(s):
        with torch.cuda.stream(s):
            hs[1].copy_(ds[1], non_blocking=True)

    def kern_h2d(s):
        red.copy(ds[0], hs[0], n, stream=s)

    def kern_d2h(s):
        red.copy(hs[1], ds[1], n, stream=s)

    cases = {
        "sdma_h2d": [sdma_h2d], "sdma_d2h": [sdma_d2h], "kern_h2d": [kern_h2d],
        "kern_d2h": [kern_d2h], "sdma_h2d+sdma_d2h": [sdma_h2d, sdma_d2h],
        "sdma_h2d+kern_d2h": [sdma_h2d, kern_d2h], "kern_h2d+sdma_d2h": [kern_h2d, sdma_d2h],
        "kern_h2d+kern_d2h": [kern_h2d, kern_d2h],
    }
    for name, fns in cases.items():
        ts = []
        for i in range(a.reps + 2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for fn, s in zip(fns, (s1, s2)):
                fn(s)
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(time.perf_counter() - t0)
        t = statistics.median(ts)
        print(json.dumps({"case": name, "mib_per_direction": a.mib,
                          "GBps_total": round(len(fns) * n / t / 1e9, 2),
                          "ms": round(t * 1e3, 3)}), flush=True)
    # config 1's H2D shape: 34 copies of 4,096,000 B (2 workers x 17
    # partitions) by SDMA on one stream / round-robin over 4 streams, by the
    # copy kernel on one / 4 streams, and as ONE batched copy kernel launch
    part, nparts = 4_096_000, 34
    src = torch.empty(part * nparts, dtype=torch.uint8).pin_memory()
    src.fill_(3)
    dst = torch.empty(part * nparts, dtype=torch.uint8, device=dev)
    ss = [torch.cuda.Stream(dev) for _ in range(4)]

    def many(kind, nst):
        for i in range(nparts):
            s = ss[i % nst]
            d, h = dst[i * part:(i + 1) * part], src[i * part:(i + 1) * part]
            if kind == "sdma":
                with torch.cuda.stream(s):
                    d.copy_(h, non_blocking=True)
            else:
                red.copy(d, h, part, stream=s)

    def batched():
        from prophet_amd.dtypes import DType
        red.sum_batched([(dst[i * part:(i + 1) * part], [src[i * part:(i + 1) * part]], part)
                         for i in range(nparts)], DType.UINT8, stream=ss[0])
    for name, fn in (("sdma_34x4MB_1stream", lambda: many("sdma", 1)),
                     ("sdma_34x4MB_4streams", lambda: many("sdma", 4)),
                     ("kern_34x4MB_1stream", lambda: many("kern", 1)),
                     ("kern_34x4MB_4streams", lambda: many("kern", 4)),
                     ("kern_34x4MB_batched", batched)):
        ts = []
        for i in range(a.reps + 2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(time.perf_counter() - t0)
        t = statistics.median(ts)
        print(json.dumps({"case": name, "GBps": round(part * nparts / t / 1e9, 2),
                          "ms": round(t * 1e3, 3)}), flush=True)
        assert bool((dst == 3).all()), name
        dst.zero_()
    assert bool((ds[0] == 7).all())


if __name__ == "__main__":
    main()
