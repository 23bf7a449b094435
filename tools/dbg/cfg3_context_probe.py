"""Probe (not product code): config 3's block-queue variants (bench.cfg3_leg)
measured alone and again after another bench leg ran in the same process —
`--after` picks the leg (pcie, server_cfg1, e2e, group_idle: a server group
made and closed with no rounds), or `--seq` runs a comma-separated sequence
of legs (cfg3 measures).  Prints one line per measurement."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--after", default="server_cfg1")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--seq", default="")
    ap.add_argument("--persistent", type=int, default=0,
                    help="> 0: block queues use that many persistent workgroups per CU "
                         "(no stalled dispatch; overlap requests ignored)")
    a = ap.parse_args()
    import torch
    import bench
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(0)
    if a.persistent:
        from prophet_amd import reducer as _r
        _cfg, _ov = _r.BlockQueue.config, _r.BlockQueue.overlap
        _r.BlockQueue.config = lambda q, wg_per_cu=-1, timeout_s=0.0: _cfg(q, a.persistent, timeout_s)
        _r.BlockQueue.overlap = lambda q, on=True: None
        _hr = _r.BlockQueue.host_releases

        def host_releases(q, on=True):   # host releases need the dispatch-ordered consumer
            _cfg(q, 0, 0.0)
            _hr(q, on)
        _r.BlockQueue.host_releases = host_releases

    def show(tag):
        r = bench.cfg3_leg(dev, red, iters=a.iters, reps=3)
        print(tag, {k: (v["ms_per_iter"], v["frac_of_roofline"]) for k, v in r.items()
                    if isinstance(v, dict) and "ms_per_iter" in v},
              "queues", r.get("hsa_queue_ids"), flush=True)

    if a.seq:
        link = None
        for i, leg in enumerate(a.seq.split(",")):
            if leg == "cfg3":
                show(f"{i}:cfg3")
            elif leg == "pcie":
                link = bench.pcie_leg(dev, red)
            elif leg == "server_cfg1":
                r = bench.server_group_leg(dev, 1, 0, link=link)
                print(f"{i}:server_cfg1", r["round_ms"], r.get("frac_of_link"),
                      r["copying_pulls"]["round_ms"], flush=True)
            elif leg == "e2e":
                r = bench.e2e_leg(dev, 1, 0, link=link)
                print(f"{i}:e2e", r["ms"], r.get("frac_of_link"), flush=True)
            elif leg in ("mkq", "tinyq"):
                # round 6: the block queue's library queues made (mkq: the
                # consumer and release queues only), or also one small
                # pre-released launch folded (tinyq)
                from prophet_amd.dtypes import DType
                x = [torch.ones(1 << 16, device=dev) for _ in range(3)]
                q = red.make_blockq([[(x[0], x[1:], 4 << 16)]], DType.FLOAT32)
                q.stream()
                q.release_stream()
                if leg == "tinyq":
                    q.release(-1)
                    q.launch()
                    q.status()
                torch.cuda.synchronize()
                q.close()
                print(f"{i}:{leg}", q.queue_ids() if False else "", flush=True)
            elif leg == "headline":
                bench.main_headline_for_probe(dev) if hasattr(bench, "main_headline_for_probe") else None
        return
    show("alone")
    link = bench.pcie_leg(dev, red)
    if a.after == "server_cfg1":
        bench.server_group_leg(dev, 1, 0, link=link)
    elif a.after == "e2e":
        bench.e2e_leg(dev, 1, 0, link=link)
    elif a.after == "group_idle":
        from prophet_amd.server import PSServerGroup
        g = PSServerGroup(2, devices=[0], engine_lanes=4, split="hash")
        g.close()
    show(f"after_{a.after}")


if __name__ == "__main__":
    main()
