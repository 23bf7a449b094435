"""Probe (not product code): bench.server_cfg3_leg three times, one JSON line each.
    python tools/dbg/server_cfg3_once.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import bench
    dev = torch.device("cuda:0")
    for rep in range(3):
        r = bench.server_cfg3_leg(dev, rounds=40)
        print(json.dumps({"rep": rep, **{k: (r[k]["round_ms"], r[k]["push_phase_ms"], r[k]["frac_of_roofline"],
                                             r[k]["exact_vs_torch_fold_in_recorded_order"])
                                         for k in ("launch", "device_releases")}}), flush=True)


if __name__ == "__main__":
    main()
