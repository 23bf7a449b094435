"""Probe (not product code): bench.server_cfg3_leg three times, one JSON line each.
    python tools/dbg/server_cfg3_once.py [--reps N] [--maps FILE]
--maps: copy /proc/self/maps to FILE at the end (round 6: to tell which
library an exit-time fault's addresses belong to)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--maps", default="")
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda:0")
    for rep in range(a.reps):
        r = bench.server_cfg3_leg(dev, rounds=40)
        print(json.dumps({"rep": rep, **{k: (r[k]["round_ms"], r[k]["push_phase_ms"], r[k]["frac_of_roofline"],
                                             r[k]["exact_vs_torch_fold_in_recorded_order"])
                                         for k in ("launch", "device_releases")}}), flush=True)
    if a.maps:
        with open("/proc/self/maps") as f, open(a.maps, "w") as g:
            g.write(f.read())


if __name__ == "__main__":
    main()
