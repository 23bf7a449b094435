"""Probe (not product code): bench.cfg3_leg once, one JSON line of each
variant's fraction of the roofline.  python tools/dbg/cfg3_once.py TAG"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import bench
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    r = bench.cfg3_leg(dev, GpuReducer(0))
    print(json.dumps({"tag": sys.argv[1] if len(sys.argv) > 1 else "",
                      **{k: v["frac_of_roofline"] for k, v in r.items() if isinstance(v, dict)
                         and "frac_of_roofline" in v}}), flush=True)


if __name__ == "__main__":
    main()
