#!/usr/bin/env python3
"""Block-queue releases inside a captured hipGraph: does a replay see the
captured release, with and without a warm (uncaptured) launch first?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from prophet_amd.dtypes import DType  # noqa: E402
from prophet_amd.reducer import GpuReducer, ReduceError  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    srcs = [torch.randn(1 << 20, device=dev) for _ in range(8)]
    dst = torch.empty_like(srcs[0])
    E = 65536
    blocks = [[(dst[i * E:(i + 1) * E], [s[i * E:(i + 1) * E] for s in srcs], E * 4)]
              for i in range(16)]
    want = srcs[0].clone()
    for s in srcs[1:]:
        want.add_(s)
    for warm in (False, True):
        for sync_first in (False, True):
            q = red.make_blockq(blocks, DType.FLOAT32)
            q.config(timeout_s=0.3)
            if warm:
                q.release(-1)
                q.launch()
                q.status()
            side = torch.cuda.Stream()
            if sync_first:
                side.wait_stream(torch.cuda.current_stream())
                torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                q.release(-1, side)
                q.launch(side)
            res = []
            for r in range(3):
                dst.zero_()
                g.replay()
                torch.cuda.synchronize()
                try:
                    q.status()
                    ok = "ok"
                except ReduceError as e:
                    ok = f"ERR{e.code}"
                res.append(f"{ok}/{'exact' if torch.equal(dst, want) else 'WRONG'}")
            print(f"warm={warm} sync_first={sync_first}: {res}", flush=True)
            q.close()


if __name__ == "__main__":
    main()
