"""Probe (not product code): where config 1's server round spends its time.
The bench's server_cfg1 round (bench.server_group_leg's shape: per worker one
push_many of the 17 partitions, a pull thread pulling views in key order),
with host timestamps: when each worker's push_many returns and when each
pull returns, relative to the round start.  Prints one JSON line per round.
    python tools/cfg1_round_probe.py [--rounds 5] [--pull view|copy] [--lanes 4]"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--pull", default="view", choices=["view", "copy", "none"])
    ap.add_argument("--lanes", type=int, default=4)
    ap.add_argument("--push", default="many", choices=["many", "single"])
    ap.add_argument("--lib", default=None, help="another build of libbpsr.so (A/B)")
    a = ap.parse_args()
    import torch
    torch.cuda.init()        # torch's HIP runtime first (as every product caller)
    if a.lib:
        from prophet_amd import reducer
        reducer.load_library(a.lib)
    from prophet_amd.buckets import partition_tensor
    from prophet_amd.dtypes import DType
    from prophet_amd.server import PSServerGroup
    N, B = 2, 64 << 20
    parts = [(p.key, p.offset, p.len) for p in partition_tensor(0, B, declared_key=0)]
    keys = [k for k, _, _ in parts]
    host = [torch.randn(B // 4).pin_memory() for _ in range(N)]
    outs = [torch.zeros(B, dtype=torch.uint8).pin_memory() for _ in range(N)]
    grp = PSServerGroup(N, devices=[0], engine_lanes=a.lanes, split="hash")
    srcs = [[host[w].view(torch.uint8)[o:o + ln] for _, o, ln in parts] for w in range(N)]
    dsts = [[outs[w][o:o + ln] for _, o, ln in parts] for w in range(N)]

    def rnd(pull):
        t0 = time.perf_counter()
        stamps = {}

        def pusher(w):
            if a.push == "many":
                grp.push_many(keys, w, srcs[w], DType.FLOAT32)
            else:
                for i, k in enumerate(keys):
                    grp.push(k, w, srcs[w][i], DType.FLOAT32)
            stamps[f"push{w}"] = round((time.perf_counter() - t0) * 1e3, 3)

        def puller(w):
            ts = []
            for i, k in enumerate(keys):
                if pull == "view":
                    grp.pull_view(k)
                else:
                    grp.pull(k, dsts[w][i])
                ts.append(round((time.perf_counter() - t0) * 1e3, 3))
            stamps[f"pull{w}"] = ts
        th = [threading.Thread(target=pusher, args=(w,)) for w in range(N)]
        if pull != "none":
            th += [threading.Thread(target=puller, args=(w,)) for w in range(N)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        stamps["round_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
        return stamps
    rnd("none")
    for r in range(a.rounds):
        print(json.dumps({"round": r, "pull": a.pull, "push": a.push, "lib": a.lib or "default",
                          **rnd(a.pull)}), flush=True)
    grp.close()


if __name__ == "__main__":
    main()
