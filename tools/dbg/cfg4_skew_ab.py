"""Probe (not product code), round 6: bench.scaling_leg (config 4 at G = 1:
the whole 553 MB VGG-16 set, 8-way fp32, two alternating input sets) with the
arena's skew forced to each candidate, interleaved `rounds` times in one
process.  One line per run.
    python tools/dbg/cfg4_skew_ab.py [--skews 16,2064,2080] [--rounds 3] (KiB)"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skews", default="16,2064,2080")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import bench
    from prophet_amd import arena
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(0)

    def fold_f32(dst, srcs):
        red.sum_n(dst.data_ptr(), [s.data_ptr() for s in srcs], dst.numel() * 4, DType.FLOAT32)

    for r in range(a.rounds):
        for kib in [int(x) for x in a.skews.split(",")]:
            arena.default_skew = lambda b, k=kib: k * 1024
            res = bench.scaling_leg(dev, 1, 0, 8, fold_f32)
            print(json.dumps({"round": r, "skew_kib": kib, "g1_fold_ms": res["g1_fold_ms"],
                              "frac": res["per_gpu_frac_of_roofline"]}), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
