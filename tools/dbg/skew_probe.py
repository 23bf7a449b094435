"""Probe (not product code), round 6: the 8-way fp32 fold of one bucket per
worker (the product's byteps_reduce_sum_n, 9 arena slots: 8 sources + the
output) by arena skew — bytes added between consecutive slots beyond the
64-KiB-rounded bucket (prophet_amd/arena.py).  Config 4's whole VGG-16 set
(553,430,176 B) folds at 0.78-0.79 with the default 16 KiB skew against
0.82 for the 256-MiB headline (DESIGN.md §5 "slot spacing"); VERDICT round 5
asks whether another skew brings it to the headline's class.  Each skew is
timed in `passes` interleaved passes (HIP events around `reps` folds, best
pass kept); one JSON line per (bucket, skew).
    python tools/dbg/skew_probe.py [--bytes 553430176,268435456] [--skews 16,64,...] (KiB)"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", default="553430176,268435456")
    ap.add_argument("--skews", default="16,32,64,128,256,512,1024,2048,2064,3072,4096,8192")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--passes", type=int, default=3)
    a = ap.parse_args()
    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(0)
    N = 8
    for nbytes in [int(x) for x in a.bytes.split(",")]:
        skews = [int(x) * 1024 for x in a.skews.split(",")]
        best = {s: float("inf") for s in skews}
        for p in range(a.passes):
            for skew in skews:
                ar = BucketArena(N + 1, nbytes, dev, skew=skew)
                slots = ar.slots()
                for k in range(N):
                    slots[k].view(torch.float32).normal_()
                out, srcs = slots[N], slots[:N]
                torch.cuda.synchronize()
                red.sum_n(out.data_ptr(), [s.data_ptr() for s in srcs], nbytes, DType.FLOAT32)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    red.sum_n(out.data_ptr(), [s.data_ptr() for s in srcs], nbytes, DType.FLOAT32)
                e1.record()
                torch.cuda.synchronize()
                best[skew] = min(best[skew], e0.elapsed_time(e1) / a.reps)
                del ar, slots, out, srcs
                torch.cuda.empty_cache()
        for skew in skews:
            ms = best[skew]
            print(json.dumps({"bucket_bytes": nbytes, "skew_kib": skew // 1024, "ms": round(ms, 4),
                              "frac_of_8TBps": round((N + 1) * nbytes / (ms * 1e-3) / 8e12, 4)}),
                  flush=True)


if __name__ == "__main__":
    main()
