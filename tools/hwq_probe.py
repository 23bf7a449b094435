#!/usr/bin/env python3
"""Which (consumer stream, release stream) pairs let a live block-queue
release through?  A live release queued on a stream that shares a hardware
queue with the running consumer cannot run until the consumer gives up
(include/bpsr/reduce.h).  For each of torch's pooled streams (32 per
priority, handed out round-robin), launch a small block queue's consumer on
the high-priority stream i and release its blocks 5 ms later on the normal
stream i (or a library-made lowest-priority stream); report which pairs time
out.  One JSON line per pair.  Not product code."""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer, ReduceError
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    n, N = 1 << 16, 4
    ins = [[torch.randn(n, device=dev) for _ in range(N)] for _ in range(2)]
    outs = [torch.zeros(n, device=dev) for _ in range(2)]
    bq = red.make_blockq([[(outs[b], ins[b], n * 4)] for b in range(2)], DType.FLOAT32)
    bq.config(wg_per_cu=0, timeout_s=0.5)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") \
        else (None, None)
    print(json.dumps({"torch_priority_range": [lo, hi]}), flush=True)
    for i in range(34):
        cons = torch.cuda.Stream(priority=-100)
        rel = torch.cuda.Stream()
        torch.cuda.synchronize()
        bq.launch(cons)
        time.sleep(0.005)
        bq.release(0, rel)
        bq.release(1, rel)
        torch.cuda.synchronize()
        ok = True
        try:
            bq.status(cons)
        except ReduceError:
            ok = False
        print(json.dumps({"pair": i, "cons_priority": cons.priority, "rel_priority": rel.priority,
                          "cons": hex(cons.cuda_stream), "rel": hex(rel.cuda_stream),
                          "released_through": ok}), flush=True)


if __name__ == "__main__":
    main()
