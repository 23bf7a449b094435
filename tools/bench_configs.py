#!/usr/bin/env python3
"""Secondary BASELINE.json configs on one MI355X (bench.py measures config 2).

  cfg1   2-worker fp32 64 MiB server rounds through the GPU-resident PS server
         (host-resident and device-resident pushes, 1 key or 17 partitions).
  cfg3   8-way fp16 over ResNet-50's 161 gradient tensors (165 BytePS partitions
         of <= 4,096,000 B), Prophet block grouping: one batched launch per
         block (12 blocks) vs one launch per partition vs one launch for all.
  sweep  8-way fp16 single-bucket sum, bucket 1 KiB .. 64 MiB and 97.49 MiB.
  cfg4   8-way fp32 over VGG-16 (553,430,176 B): whole set on one GPU, and the
         per-GPU shard of a G-way key-space split (G = 2, 4, 8) timed alone —
         the device-resident sum-only scaling of SURVEY.md §8d cfg4.
  cfg5   16-way bf16, 4 GiB of pinned host gradients, streamed H2D -> fold ->
         D2H on side streams (prophet_amd.stream.StreamingReducer), plus the
         bare H2D rate of the same bytes for reference.

Every result is checked against torch's own left fold (bit-exact) before it is
reported.  Prints one JSON line per measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


VARIANTS = "all"


def emit(**kw):
    print(json.dumps(kw), flush=True)


def timed(fn, reps, stream):
    import torch
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(0)
    torch.cuda.synchronize()
    ts = []
    for r in range(3):
        with torch.cuda.stream(stream):
            torch.cuda._sleep(2_000_000)   # the host queues ahead of the GPU (bench.py _Clock)
        e0.record(stream)
        for i in range(reps):
            fn(i)
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return statistics.median(ts), min(ts)


def torch_fold(srcs, tdt):
    acc = srcs[0].view(tdt).clone()
    for s in srcs[1:]:
        acc.add_(s.view(tdt))
    return acc.view(__import__("torch").uint8)


def cfg3(red, dev, N=8, sets=3):
    import torch
    from prophet_amd.buckets import partition_all, prophet_blocks, resnet50_param_sizes
    from prophet_amd.dtypes import DType
    sizes = [n * 2 for n in resnet50_param_sizes()]
    parts = partition_all(sizes)
    blocks = prophet_blocks(len(sizes))
    total = sum(sizes)
    s = torch.cuda.current_stream()
    # per set: each worker's whole gradient vector in one buffer (partitions are views)
    data = []
    for _ in range(sets):
        w = [torch.randn(total // 2, device=dev).half().view(torch.uint8) for _ in range(N)]
        out = torch.empty(total, dtype=torch.uint8, device=dev)
        toff = [0]
        for n in sizes:
            toff.append(toff[-1] + n)
        data.append((w, out, toff))

    def views(i, p):
        w, out, toff = data[i % sets]
        o = toff[p.tensor] + p.offset
        return out[o:o + p.len], [x[o:o + p.len] for x in w]

    by_block = []
    for blk in blocks:
        tset = set(blk)
        by_block.append([p for p in parts if p.tensor in tset])

    def per_partition(i):
        for p in parts:
            d, ss = views(i, p)
            red.sum_n(d, ss, p.len, DType.FLOAT16, stream=s)

    def per_block(i):
        for bp in by_block:
            red.sum_batched([(*views(i, p), p.len) for p in bp], DType.FLOAT16, stream=s)

    def all_in_one(i):
        red.sum_batched([(*views(i, p), p.len) for p in parts], DType.FLOAT16, stream=s)

    plans = [[red.make_plan([(*views(i, p), p.len) for p in bp], DType.FLOAT16)
              for bp in by_block] for i in range(sets)]

    def per_block_plan(i):
        for pl in plans[i % sets]:
            pl.launch(s)

    graphs = []
    for i in range(sets):
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(s)
        with torch.cuda.stream(side):
            per_block_plan(i)          # warm the capture stream
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=side):
            for pl in plans[i]:
                pl.launch(side)
        graphs.append(g)

    def per_block_graph(i):
        graphs[i % sets].replay()

    # Engine streams: independent keys/blocks run concurrently, like the
    # reference's BYTEPS_SERVER_ENGINE_THREAD engine threads (server.cc:363-370).
    eng = [torch.cuda.Stream() for _ in range(4)]

    def per_block_plans_4streams(i, cur=None):
        cur = cur or torch.cuda.current_stream()
        for e in eng:
            e.wait_stream(cur)
        for b, pl in enumerate(plans[i % sets]):
            pl.launch(eng[b % len(eng)])
        for e in eng:
            cur.wait_stream(e)

    graphs4 = []
    for i in range(sets):
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(s)
        with torch.cuda.stream(side):
            per_block_plans_4streams(i, side)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=side):
            per_block_plans_4streams(i, side)
        graphs4.append(g)

    def per_block_graph4(i):
        graphs4[i % sets].replay()

    # Release groups from the native Prophet PUSH scheduler (scheduled_queue.cc:
    # 217-296) at batch 64 and Z_NET_B = 10000 (10 Gb/s in Mb/s), credit 16 MiB:
    # one plan per group, the whole iteration captured in one graph.
    from prophet_amd.prophet import ProphetPushQueue, backward_arrivals, model_checkpoints, \
        release_groups
    q = ProphetPushQueue(batch_size=64, net_b=10000, credit=16 << 20,
                         checkpoints=model_checkpoints(len(sizes)))
    rgroups = release_groups(q, backward_arrivals(sizes))
    pmap = {(p.tensor, p.part): p for p in parts}
    rplans = [[red.make_plan([(*views(i, pmap[(t.grad, t.part)]), t.len) for t in g],
                             DType.FLOAT16) for g in rgroups] for i in range(sets)]
    rgraphs = []
    for i in range(sets):
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(s)
        with torch.cuda.stream(side):
            for pl in rplans[i]:
                pl.launch(side)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=side):
            for pl in rplans[i]:
                pl.launch(side)
        rgraphs.append(g)

    def release_group_graph(i):
        rgraphs[i % sets].replay()

    # Every partition in ONE plan (no block boundaries): the batched kernel's
    # own rate on the mixed ResNet-50 sizes, without per-block launch costs.
    splans = [red.make_plan([(*views(i, p), p.len) for p in parts], DType.FLOAT16)
              for i in range(sets)]

    def single_plan(i):
        splans[i % sets].launch(s)

    # Persistent block consumer: ONE launch per iteration over the 12 blocks,
    # each started once released (byteps_reduce_blockq_*).  Releases are
    # stream-ordered one-wave kernels writing the block words, here all before
    # the launch (data resident, as for the back-to-back plans above), or one
    # per block from a second stream while the consumer runs.
    bqs = {}
    for occ in (0, 1):
        bqs[occ] = []
        for i in range(sets):
            bq = red.make_blockq([[(*views(i, p), p.len) for p in bp] for bp in by_block],
                                 DType.FLOAT16)
            bq.config(wg_per_cu=occ, timeout_s=5.0)
            bqs[occ].append(bq)

    def blockq_fn(occ):
        def fn(i):
            bq = bqs[occ][i % sets]
            bq.release(-1, s)
            bq.launch(s)
        return fn

    def blockq_graph(occ):
        gs = []
        for i in range(sets):
            bq = bqs[occ][i]
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(s)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=side):
                bq.release(-1, side)
                bq.launch(side)
            gs.append(g)
        return lambda i: gs[i % sets].replay()

    bq_variants = []
    for occ, nm in ((0, "dispatch"), (1, "persistent")):
        bq_variants.append((f"prophet_blockq_{nm}", blockq_fn(occ)))
        bq_variants.append((f"prophet_blockq_{nm}_hipgraph", blockq_graph(occ)))

    rel_stream = torch.cuda.Stream()
    # The live consumer runs on the library's consumer stream: a hardware queue
    # of its own, so the releases on rel_stream never sit behind it in a shared
    # queue (include/bpsr/reduce.h; stream priority alone did not guarantee it).
    live_stream = bqs[0][0].stream()
    nblk = len(by_block)

    def blockq_live(i, occ=0):
        """Consumer launched on live_stream; the 12 releases follow on another
        stream (as the push path issues them behind each block's H2D).  No
        cross-stream events: launch k consumes the k-th release of each block
        (epochs), so iteration k+1 may be issued at once, as from native code
        (tools/cfg3_native.cpp)."""
        bq = bqs[occ][i % sets]
        bq.launch(live_stream)
        for b in range(nblk):
            bq.release(b, rel_stream)

    def blockq_live_ranges(i):
        """Release groups of 4 blocks, one call and one kernel each."""
        bq = bqs[0][i % sets]
        bq.launch(live_stream)
        for b in range(0, nblk, 4):
            bq.release_range(b, min(4, nblk - b), rel_stream)

    live_variants = [("prophet_blockq_dispatch_live_release", blockq_live),
                     ("prophet_blockq_persistent_live_release", lambda i: blockq_live(i, occ=1)),
                     ("prophet_blockq_dispatch_live_release_ranges4", blockq_live_ranges)]
    for name, fn in live_variants:
        ts = []
        for _ in range(30):
            fn(_)
        torch.cuda.synchronize()
        for r in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(live_stream)
            t0 = time.perf_counter()
            for i in range(200):
                fn(i)
            host_us = (time.perf_counter() - t0) / 200 * 1e6
            e1.record(live_stream)
            torch.cuda.synchronize()
            ts.append((e0.elapsed_time(e1) / 200, host_us))
        w, out, _ = data[0]
        out.zero_()
        torch.cuda.synchronize()          # the consumer runs on live_stream
        fn(0)
        fn(1)
        fn(2)
        torch.cuda.synchronize()
        ok = bool(torch.equal(out, torch_fold(w, torch.float16)))
        ms = sorted(t for t, _ in ts)
        med = ms[len(ms) // 2]
        emit(config="cfg3", variant=name, driver="python (ctypes), 200 iterations x 5, timed on "
             "the consumer stream", n_workers=N, tensors=len(sizes), partitions=len(parts),
             blocks=len(blocks), bytes_per_worker=total, ms=round(med, 4), min_ms=round(ms[0], 4),
             max_ms=round(ms[-1], 4), host_us_per_iter=round(statistics.median(h for _, h in ts), 1),
             gibps=round(N * total / (med * 1e-3) / GIB, 1),
             hbm_frac=round((N + 1) * total / (med * 1e-3) / 8e12, 4), exact=ok)

    for name, fn in bq_variants + ([] if VARIANTS == "blockq" else [("per_partition_launch", per_partition),
                     ("prophet_block_batched", per_block),
                     ("single_batched_launch", all_in_one),
                     ("prophet_block_plans", per_block_plan),
                     ("prophet_block_plans_hipgraph", per_block_graph),
                     ("prophet_block_plans_4streams", per_block_plans_4streams),
                     ("prophet_block_plans_4streams_hipgraph", per_block_graph4),
                     ("prophet_release_groups_hipgraph", release_group_graph),
                     ("single_plan_no_blocks", single_plan)]):
        med, mn = timed(fn, 10, s)
        w, out, _ = data[0]
        fn(0)
        torch.cuda.synchronize()
        ok = bool(torch.equal(out, torch_fold(w, torch.float16)))
        emit(config="cfg3", variant=name, n_workers=N, tensors=len(sizes), partitions=len(parts),
             blocks=len(blocks), bytes_per_worker=total, ms=round(med, 4), min_ms=round(mn, 4),
             gibps=round(N * total / (med * 1e-3) / GIB, 1),
             hbm_frac=round((N + 1) * total / (med * 1e-3) / 8e12, 4), exact=ok)


def graph_timed(fn, launches, sets):
    """Per-launch device time of `launches` calls captured in one hipGraph
    (no host in the loop), median of 5 replays."""
    import torch
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for i in range(sets):
            fn(i, side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        for i in range(launches):
            fn(i, side)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / launches)
    return statistics.median(ts)


def size_sweep(red, dev, N=8):
    """8-way fp16 single-bucket sum over the BASELINE "1 KiB - 98 MiB" range.
    Worker slots come from one skewed arena per set (as the server allocates
    them).  `us` = device time per launch from a hipGraph of back-to-back
    launches; `us_python` = one ctypes call per launch from Python (host-bound
    below a few MiB)."""
    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType
    s = torch.cuda.current_stream()
    sizes = [1 << k for k in range(10, 27)] + [102_228_128]
    for B in sizes:
        n = B // 2
        sets = 3 if B >= (1 << 20) else 1
        data = []
        for _ in range(sets):
            slots = BucketArena(N + 1, B, dev).slots()
            for t in slots[:N]:
                t.view(torch.float16).copy_(torch.randn(n, device=dev))
            data.append((slots[:N], slots[N]))

        def fn(i, st=s):
            w, o = data[i % sets]
            red.sum_n(o, w, B, DType.FLOAT16, stream=st)
        med_py, _ = timed(fn, 50 if B < (16 << 20) else 10, s)
        med = graph_timed(fn, 60 if B < (16 << 20) else 12, sets)
        w, o = data[0]
        fn(0)
        torch.cuda.synchronize()
        ok = bool(torch.equal(o, torch_fold(w, torch.float16)))
        emit(config="sweep_fp16", bucket_bytes=B, n_workers=N, us=round(med * 1e3, 2),
             us_python=round(med_py * 1e3, 2), gibps=round(N * B / (med * 1e-3) / GIB, 1),
             hbm_frac=round((N + 1) * B / (med * 1e-3) / 8e12, 4), exact=ok)
        del data
        torch.cuda.empty_cache()


def cfg4(red, dev, N=8):
    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.buckets import vgg16_param_sizes
    from prophet_amd.dtypes import DType
    from prophet_amd.shard import owner_ranges
    s = torch.cuda.current_stream()
    E = sum(vgg16_param_sizes())
    for G in (1, 2, 4, 8):
        lo, hi = owner_ranges(E, G)[G - 1]
        n = hi - lo
        B = n * 4
        sets = 3 if (N + 1) * B * 3 < (40 << 30) else 2
        data = []
        for _ in range(sets):
            slots = BucketArena(N + 1, B, dev).slots()
            for t in slots[:N]:
                t.view(torch.float32).copy_(torch.randn(n, device=dev))
            data.append((slots[N], slots[:N]))

        def fn(i):
            o, w = data[i % sets]
            red.sum_n(o, w, B, DType.FLOAT32, stream=s)
        med, mn = timed(fn, 10, s)
        o, w = data[0]
        fn(0)
        torch.cuda.synchronize()
        ok = bool(torch.equal(o, torch_fold(w, torch.float32)))
        emit(config="cfg4", gpus_in_split=G, shard_elems=n, ms=round(med, 4),
             per_gpu_gibps=round(N * B / (med * 1e-3) / GIB, 1),
             node_gibps_if_parallel=round(G * N * B / (med * 1e-3) / GIB, 1),
             whole_set_time_ms_if_parallel=round(med, 4),
             hbm_frac=round((N + 1) * B / (med * 1e-3) / 8e12, 4), exact=ok)
        del data
        torch.cuda.empty_cache()


def cfg5(red, dev, N=16, B=256 << 20, chunk=32 << 20):
    import torch
    from prophet_amd.dtypes import DType
    streamed(red, dev, "cfg5", N, B, torch.bfloat16, DType.BFLOAT16, chunk)


def cfg2_e2e(red, dev, N=8, B=256 << 20, chunk=32 << 20):
    """Config 2's workload (8 x 256 MiB fp32) from pinned host memory to a pinned
    host result through the streaming path: the PCIe-inclusive rate the north
    star asks DESIGN.md to record beside the device-resident headline."""
    import torch
    from prophet_amd.dtypes import DType
    streamed(red, dev, "cfg2_e2e", N, B, torch.float32, DType.FLOAT32, chunk)


def streamed(red, dev, name, N, B, tdt, dtype_id, chunk):
    import torch
    from prophet_amd.stream import StreamingReducer
    es = torch.empty(0, dtype=tdt).element_size()
    n = B // es
    t0 = time.perf_counter()
    host = [torch.empty(B, dtype=torch.uint8, pin_memory=True) for _ in range(N)]
    g = torch.Generator()
    for k, h in enumerate(host):
        g.manual_seed(1000 + k)
        h.view(tdt).copy_(torch.randn(n, generator=g))
    out = torch.empty(B, dtype=torch.uint8, pin_memory=True)
    setup_s = time.perf_counter() - t0
    sr = StreamingReducer(N, chunk_bytes=chunk, depth=3, device=dev, reducer=red)
    sr.reduce(host, out, B, dtype_id)                # warm-up
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        sr.reduce(host, out, B, dtype_id)
        ts.append(time.perf_counter() - t)
    med = statistics.median(ts)
    # check an 8 MiB window against torch's left fold on the device
    w = 8 << 20
    acc = host[0][:w].to(dev).view(tdt).clone()
    for h in host[1:]:
        acc.add_(h[:w].to(dev).view(tdt))
    ok = bool(torch.equal(acc.view(torch.uint8).cpu(), out[:w]))
    # bare H2D of the same N*B bytes into one device buffer (reference rate)
    dbuf = torch.empty(chunk, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for h in host:
        for o in range(0, B, chunk):
            dbuf.copy_(h[o:o + chunk], non_blocking=True)
    torch.cuda.synchronize()
    h2d = time.perf_counter() - t
    emit(config=name, n_workers=N, bucket_bytes=B, total_bytes=N * B, chunk_bytes=chunk,
         e2e_s=round(med, 4), e2e_gibps=round(N * B / med / GIB, 2),
         h2d_only_gibps=round(N * B / h2d / GIB, 2), e2e_over_h2d=round(h2d / med, 3),
         host_setup_s=round(setup_s, 1), exact_window=ok)


def cfg1(dev, N=2, B=64 << 20):
    """2-worker fp32 64 MiB server rounds through the GPU-resident PS server
    (prophet_amd.server, in-process transport): pushes start in pinned host
    memory (as ps-lite's receive buffers would be) or on the device; one round =
    every worker pushes, then every worker pulls the merged bucket to host.
    As one key, and as the 17 BytePS partitions of 4,096,000 B on 4 lanes."""
    import threading
    import torch
    from prophet_amd.buckets import partition_tensor
    from prophet_amd.dtypes import DType
    from prophet_amd.server import PSServer
    n = B // 4
    host = [torch.randn(n).pin_memory() for _ in range(N)]
    devd = [h.to(dev) for h in host]
    for layout in ("1key", "17keys"):
        parts = [(0, 0, B)] if layout == "1key" else \
            [(p.key, p.offset, p.len) for p in partition_tensor(0, B)]
        for src_loc, srcs in (("host", host), ("device", devd)):
            for policy in (0, 1):
                srv = PSServer(N, engine_lanes=4, policy=policy)
                out = torch.empty(B, dtype=torch.uint8).pin_memory()

                def rnd(init=False):
                    def w(k):
                        b = srcs[k].view(torch.uint8)
                        for key, off, ln in parts:
                            srv.push(key, k, b[off:off + ln], DType.FLOAT32)
                        if not init:
                            for key, off, ln in parts:
                                if k == 0:
                                    srv.pull(key, out[off:off + ln])
                                else:
                                    tmp = torch.empty(ln, dtype=torch.uint8).pin_memory() \
                                        if not hasattr(rnd, "tmp") else rnd.tmp[:ln]
                                    rnd.tmp = tmp if not hasattr(rnd, "tmp") else rnd.tmp
                                    srv.pull(key, tmp[:ln])
                    ts = [threading.Thread(target=w, args=(k,)) for k in range(N)]
                    for t in ts:
                        t.start()
                    for t in ts:
                        t.join()
                rnd.tmp = torch.empty(B, dtype=torch.uint8).pin_memory()
                rnd(init=True)
                rnd()
                ts_ = []
                for _ in range(10):
                    t0 = time.perf_counter()
                    rnd()
                    ts_.append(time.perf_counter() - t0)
                med = statistics.median(ts_)
                want = (host[0] + host[1]).view(torch.uint8)
                ok = bool(torch.equal(out, want))
                emit(config="cfg1", layout=layout, pushes_from=src_loc,
                     policy=["fused", "incremental"][policy], n_workers=N, bucket_bytes=B,
                     round_ms=round(med * 1e3, 3), gibps=round(N * B / med / GIB, 2), exact=ok)
                srv.close()
    cfg1_pipelined(host, N, B)
    cfg1_pipelined(host, N, B, view=True)
    cfg1_pipelined(host, N, B, view=True, push_async=True)


def cfg1_pipelined(host, N, B, view=False, push_async=False):
    """cfg1 with BytePS's worker loop structure: each worker has a push thread
    and a pull thread (core_loops.cc:492-528 PushLoop, 530-564 PullLoop); the
    pull of a partition is issued as soon as that partition's push returned, so
    the D2H of partition k overlaps the H2D of partition k+1.
    view=True: pulls are zero-copy responses (byteps_server_pull_host_view, the
    analogue of server.cc:42-70 answering from the store's SArray): one D2H per
    key per round into a pinned mirror that a transport would send from, instead
    of one D2H per puller.  The exactness round copies the views out.
    push_async=True: pushes are non-blocking (byteps_server_push_async): a push
    thread queues all its partitions' H2D copies back to back."""
    import threading
    import torch
    from prophet_amd.buckets import partition_tensor
    from prophet_amd.dtypes import DType
    from prophet_amd.server import PSServer
    parts = [(p.key, p.offset, p.len) for p in partition_tensor(0, B)]
    lanes = int(os.environ.get("BPSR_CFG1_LANES", "4"))
    srv = PSServer(N, engine_lanes=lanes, policy=0)
    outs = [torch.empty(B, dtype=torch.uint8).pin_memory() for _ in range(N)]

    import numpy as np

    def rnd(init=False, check=False):
        pushed = [[threading.Event() for _ in parts] for _ in range(N)]

        def pusher(k):
            b = host[k].view(torch.uint8)
            for i, (key, off, ln) in enumerate(parts):
                if push_async:
                    srv.push_async(key, k, b[off:off + ln], DType.FLOAT32)
                else:
                    srv.push(key, k, b[off:off + ln], DType.FLOAT32)
                pushed[k][i].set()

        def puller(k):
            for i, (key, off, ln) in enumerate(parts):
                pushed[k][i].wait()
                if not view:
                    srv.pull(key, outs[k][off:off + ln])
                else:
                    v = srv.pull_view(key)
                    if check:
                        outs[k][off:off + ln].numpy()[:] = np.frombuffer(v, np.uint8)
        ts = [threading.Thread(target=pusher, args=(k,)) for k in range(N)]
        if not init:
            ts += [threading.Thread(target=puller, args=(k,)) for k in range(N)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    rnd(init=True)
    rnd()
    ts_ = []
    for _ in range(10):
        t0 = time.perf_counter()
        rnd()
        ts_.append(time.perf_counter() - t0)
    med = statistics.median(ts_)
    if view:
        rnd(check=True)
    want = host[0].clone()
    for h in host[1:]:
        want += h
    ok = all(bool(torch.equal(o, want.view(torch.uint8))) for o in outs)
    emit(config="cfg1", layout="17keys_push_pull_threads" + ("_pull_view" if view else "")
         + ("_push_async" if push_async else ""),
         pushes_from="host", policy="fused", lanes=lanes,
         n_workers=N, bucket_bytes=B, round_ms=round(med * 1e3, 3),
         gibps=round(N * B / med / GIB, 2), exact=ok)
    srv.close()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--only", default="cfg1,cfg3,sweep,cfg4,cfg5,cfg2e2e")
    p.add_argument("--variants", default="all", help="cfg3: all | blockq")
    a = p.parse_args()
    global VARIANTS
    VARIANTS = a.variants
    import torch
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    todo = a.only.split(",")
    if "cfg1" in todo:
        cfg1(dev)
    if "cfg3" in todo:
        cfg3(red, dev)
    if "sweep" in todo:
        size_sweep(red, dev)
    if "cfg4" in todo:
        cfg4(red, dev)
    if "cfg5" in todo:
        cfg5(red, dev)
    if "cfg2e2e" in todo:
        cfg2_e2e(red, dev)


if __name__ == "__main__":
    main()
