"""Block-queue releases on streams that share ONE hardware queue with the
launch stream (run as a subprocess by tests/test_blockq_gpu.py with
GPU_MAX_HW_QUEUES=1: HIP then multiplexes every normal-priority stream, the
NULL stream included, onto a single in-order hardware queue; the consumer
queues are CU-masked and keep queues of their own).

This is the r05s76 stall made deterministic ("false
dependencies"): a wait for the consumer queued on the launch stream at launch
time sits in the shared hardware queue ahead of the releases (and of the
copies before them) queued on any other stream, so the consumer waits for
releases that wait for the consumer — until its timeout.  Since round 6 a
launch joins back into its stream only once its epoch is fully released.

Cases (float32, exact against torch's left fold of the same sources):
  caller_stream   launch on one torch stream, copies + one release_range on another
  null_mixed      the r05s76 test: launch on the NULL stream, copies + a stream
                  release on a side stream, host releases after an event
  push_loop       the PUSH loop launched on a caller stream, its release kernels
                  on another stream
Prints one JSON line per case, then "ok" when every case passed.
Usage: python tests/blockq_shared_hwq_case.py [library path]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from prophet_amd import reducer
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer, ReduceError
    if len(sys.argv) > 1:
        reducer.load_library(sys.argv[1])
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    gen = torch.Generator(device=dev)
    # 4 blocks of 2 buckets, 4 sources each
    sizes = [[70_001, 4099], [1 << 18, 33], [300_000, 5], [9, 1 << 16]]
    N = 4

    def table(seed):
        blocks, views = [], []
        for bi, blk in enumerate(sizes):
            out = []
            for j, n in enumerate(blk):
                srcs = [torch.zeros(n, dtype=torch.float32, device=dev) for _ in range(N)]
                stage = []
                for k in range(N):
                    gen.manual_seed(seed + 100 * bi + 10 * j + k)
                    stage.append(torch.randn(n, device=dev, generator=gen))
                dst = torch.full((n,), 7.0, device=dev)
                out.append((dst.view(torch.uint8), [s.view(torch.uint8) for s in srcs], 4 * n))
                views.append((dst, srcs, stage))
            blocks.append(out)
        return blocks, views

    def want(views):
        res = []
        for dst, srcs, stage in views:
            r = stage[0].clone()
            for x in stage[1:]:
                r.add_(x)
            res.append(r)
        return res

    def exact(views, wants):
        return all(torch.equal(d, w) for (d, _, _), w in zip(views, wants))

    results = []

    def run(name, fn):
        t0 = time.perf_counter()
        try:
            ok = fn()
            err = None
        except ReduceError as e:
            ok, err = False, str(e)
        results.append({"case": name, "ok": bool(ok), "s": round(time.perf_counter() - t0, 3),
                        "error": err})
        print(json.dumps(results[-1]), flush=True)

    def caller_stream():
        blocks, views = table(11)
        wants = want(views)
        torch.cuda.synchronize()
        q = red.make_blockq(blocks, DType.FLOAT32)
        q.config(wg_per_cu=0, timeout_s=2.0)
        ls, side = torch.cuda.Stream(), torch.cuda.Stream()
        q.launch(ls)
        with torch.cuda.stream(side):
            for _, srcs, stage in views:
                for s_, x in zip(srcs, stage):
                    s_.copy_(x)
        q.release_range(0, len(blocks), side)
        q.status(ls)
        torch.cuda.synchronize()
        ok = exact(views, wants)
        q.close()
        return ok

    def null_mixed():
        blocks, views = table(23)
        wants = want(views)
        torch.cuda.synchronize()
        q = red.make_blockq(blocks, DType.FLOAT32)
        q.config(wg_per_cu=0, timeout_s=2.0)
        q.host_releases(True)
        side = torch.cuda.Stream()
        q.launch()                      # torch's current stream: the NULL stream
        ev = torch.cuda.Event()
        with torch.cuda.stream(side):
            for _, srcs, stage in views:
                for s_, x in zip(srcs, stage):
                    s_.copy_(x)
            ev.record(side)
        q.release_range(2, 2, side)     # stream-ordered, behind the copies
        ev.synchronize()                # the host knows blocks 0-1 landed
        q.release_host(0, 2)
        q.status()
        torch.cuda.synchronize()
        ok = exact(views, wants)
        q.close()
        return ok

    def push_loop():
        from prophet_amd.prophet import ProphetPushQueue, PushLoop, PushTask
        blocks, views = table(37)
        wants = want(views)
        for _, srcs, stage in views:
            for s_, x in zip(srcs, stage):
                s_.copy_(x)
        torch.cuda.synchronize()
        q = red.make_blockq(blocks, DType.FLOAT32)
        q.config(wg_per_cu=0, timeout_s=2.0)
        block_of = [b for b, blk in enumerate(blocks) for _ in blk]
        lens = [4 * n for blk in sizes for n in blk]
        pq = ProphetPushQueue(batch_size=64, net_b=10**6, credit=1 << 30, checkpoints=(-1, 3, 7),
                              backward_exec=(5, 5, 0))
        ls, rel = torch.cuda.Stream(), torch.cuda.Stream()
        lp = PushLoop(pq, q, block_of, release_stream=rel, inline=True)
        lp.begin(ls)
        for i in reversed(range(len(block_of))):
            lp.push(PushTask(i, 0, lens[i], 1, i << 16), i)
        lp.end(timeout_s=5.0)
        q.status(ls)
        torch.cuda.synchronize()
        ok = exact(views, wants)
        lp.close()
        q.close()
        return ok

    for name, fn in (("caller_stream", caller_stream), ("null_mixed", null_mixed),
                     ("push_loop", push_loop)):
        run(name, fn)
    if all(r["ok"] for r in results):
        print("ok", flush=True)


if __name__ == "__main__":
    main()
