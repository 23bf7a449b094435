#!/usr/bin/env python3
"""Diagnose a PUSH-loop consumer timeout seen only after earlier block queues
(tests/test_pushloop_gpu.py): run one config-3 iteration first, then small
tables with one factor changed at a time; one JSON line per case.  Not
product code."""
from __future__ import annotations

import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


_HIP = None


def cu_mask_stream(torch):
    """A stream with an explicit all-CU mask: the runtime gives such a stream a
    hardware queue of its own (no multiplexing with other streams)."""
    import ctypes
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
    s = ctypes.c_void_p()
    mask = (ctypes.c_uint32 * 8)(*([0xFFFFFFFF] * 8))
    rc = _HIP.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


def small_case(torch, red, dt_name="f32", N=5, empty=True, fifo=True, inline=False, occ=0,
               timeout=1.0, sync_before=True, cons_kind="pool_high"):
    from prophet_amd.dtypes import DType
    from prophet_amd.prophet import ProphetPushQueue, PushLoop, PushTask
    from prophet_amd.reducer import ReduceError
    dev = torch.device("cuda:0")
    tdt = {"f32": torch.float32, "f16": torch.float16}[dt_name]
    did = {"f32": DType.FLOAT32, "f16": DType.FLOAT16}[dt_name]
    es = 4 if dt_name == "f32" else 2
    n = 70_001
    lens = [n, 3 * n, 2 * n + 7, n] + ([5 * n] if fifo else [])
    grads = [3, 2, 1, 0] + ([77] if fifo else [])
    is_fifo = [False] * 4 + ([True] if fifo else [])
    block_of = ([0, 0, 2, 2] + ([2] if fifo else [])) if empty else \
        ([0, 0, 1, 1] + ([1] if fifo else []))
    nb = 3 if empty else 2
    ins = [[torch.randn(L, device=dev).to(tdt) for L in lens] for _ in range(N)]
    outs = [torch.zeros(L, device=dev, dtype=tdt) for L in lens]
    blocks = [[] for _ in range(nb)]
    for i, L in enumerate(lens):
        blocks[block_of[i]].append((outs[i], [ins[k][i] for k in range(N)], L * es))
    bq = red.make_blockq(blocks, did)
    bq.config(wg_per_cu=occ, timeout_s=timeout)
    q = ProphetPushQueue(batch_size=64, net_b=10**6, credit=1 << 30, checkpoints=(-1, 1, 3),
                         backward_exec=(5, 5, 0))
    rel = torch.cuda.Stream()
    cons = cu_mask_stream(torch) if cons_kind == "cu_mask" else torch.cuda.Stream(priority=-100)
    loop = PushLoop(q, bq, block_of, release_stream=rel, inline=inline)
    if sync_before:
        torch.cuda.synchronize()
    res = {}
    for it in range(2):
        loop.begin(cons)
        for i in range(len(lens)):
            loop.push(PushTask(grads[i], 0, lens[i] * es, 1, grads[i] << 16,
                               scheduled=not is_fifo[i]), i)
        loop.end(timeout_s=5.0)
        torch.cuda.synchronize()
        try:
            bq.status(cons)
            ok = True
        except ReduceError:
            ok = False
        exact = True
        for i in range(len(lens)):
            ref = ins[0][i].clone()
            for k in range(1, N):
                ref.add_(ins[k][i])
            exact = exact and bool(torch.equal(outs[i], ref))
        res[f"it{it}"] = {"status_ok": ok, "exact": exact}
        if not ok:
            res[f"it{it}"]["debug"] = bq.debug()
    loop.close()
    bq.close()
    return res


def resnet_iteration(torch, red):
    import test_pushloop_gpu as T
    from prophet_amd.prophet import PushLoop
    S = T._setup()
    cons, rel = torch.cuda.Stream(priority=-100), torch.cuda.Stream()
    loop = PushLoop(S["q"], S["bq"], S["block_of"], release_stream=rel)
    loop.begin(cons)
    for t, i in S["tasks"]:
        loop.push(t, i)
    loop.end(timeout_s=10.0)
    torch.cuda.synchronize()
    S["bq"].status(cons)
    ok = bool(torch.equal(S["out"], S["ref"].view(torch.uint8)))
    loop.close()
    S["bq"].close()
    return ok


def main():
    import torch
    from prophet_amd.reducer import GpuReducer
    red = GpuReducer(device=0)
    cases = [("fresh_as_test", {})]
    print(json.dumps({"case": "fresh_as_test", **small_case(torch, red)}), flush=True)
    print(json.dumps({"case": "resnet_iteration", "exact": resnet_iteration(torch, red)}),
          flush=True)
    gc.collect()
    variants = [("after_resnet_as_test", {}), ("as_test_again", {}),
                ("no_empty_block", {"empty": False}), ("no_fifo", {"fifo": False}),
                ("fp16", {"dt_name": "f16"}), ("N8", {"N": 8}), ("inline", {"inline": True}),
                ("timeout5s", {"timeout": 5.0}), ("persistent_occ1", {"occ": 1}),
                ("as_test_last", {})]
    variants += [(f"cu_mask_consumer_{k}", {"cons_kind": "cu_mask"}) for k in range(8)]
    for name, kw in variants:
        t0 = time.perf_counter()
        r = small_case(torch, red, **kw)
        print(json.dumps({"case": name, "s": round(time.perf_counter() - t0, 2), **r}),
              flush=True)
    del cases


if __name__ == "__main__":
    main()
