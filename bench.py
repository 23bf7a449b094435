#!/usr/bin/env python3
"""Benchmark of the device-resident N-way gradient-bucket sum (BASELINE.json).

Workload (BASELINE.json configs[1]): 8-way fp32 left fold
of one 256 MiB bucket per GPU — the server round of byteps/server/server.cc:
216-273 for one key, done as ONE fused HIP kernel through the C ABI
(byteps_reduce_sum_n).  Inputs are synthetic gradients (seeded N(0,1)),
resident in HBM before the timed region; 3 input sets are rotated so every
step streams from HBM rather than the 256 MiB Infinity Cache.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process
per GPU; each GPU owns a contiguous slice of the key space and reduces its own
256 MiB bucket per step (weak scaling, no data-path collective — the sum is
element-wise).  Barrier + synchronize bracket the timed steps, the max over
ranks is taken, and value = total gradient bytes aggregated by all ranks / time.

Prints ONE JSON line (rank 0).  Metric: GiB/s = N_workers * B / t / 2^30 per
step, summed over GPUs.  ``roofline`` prices the dominant kernel at
(N_workers + 1) * B algorithmic HBM bytes per launch against 8.0 TB/s;
``cpu_baseline`` times the reference's own CpuReducer (oracle/_ref, the
reference server round: zero-copy first arrival + (N-1) sums + copy to store)
on a bounded sample on the host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GIB = float(1 << 30)
# --dtype name -> (byteps DataType id, torch dtype name); ids: common.h:52-65 (+ bf16 = 11)
DTYPES = {"f32": (0, "float32"), "f64": (1, "float64"), "f16": (2, "float16"),
          "u8": (3, "uint8"), "i32": (4, "int32"), "i8": (5, "int8"), "i64": (6, "int64"),
          "bf16": (11, "bfloat16")}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workers", type=int, default=8, help="N-way (pushing workers)")
    p.add_argument("--bucket-mib", type=float, default=256.0)
    p.add_argument("--dtype", default="f32", choices=list(DTYPES))
    p.add_argument("--mode", default="reference", choices=["reference", "accum"],
                   help="f16/bf16: round after every add (reference) or fp32 accumulate")
    p.add_argument("--sets", type=int, default=3, help="rotated input sets")
    p.add_argument("--layout", default="arena", choices=["arena", "separate"],
                   help="worker slots in one skewed HBM arena, or separate allocations")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-scatter", action="store_true",
                   help="N > 1: skip the config-4 RCCL scatter leg reported beside value")
    p.add_argument("--cpu-sample-mib", type=float, default=64.0,
                   help="bucket size of the CPU baseline sample")
    return p.parse_args()


def cpu_baseline(n_workers: int, dtype_id: int, sample_mib: float) -> dict | None:
    """Reference CpuReducer (or the restatement) on host cores, server-round pattern."""
    import numpy as np

    from oracle.oracle import PortReducer, RefReducer
    from prophet_amd import synth

    es = {0: 4, 1: 8, 2: 2, 3: 1, 4: 4, 5: 1, 6: 8, 11: 2}[dtype_id]
    if dtype_id == 11:           # reference has no bf16: time the restatement
        kinds = [("port", PortReducer)]
    else:
        kinds = [("reference", RefReducer)] if RefReducer.available() else [("port", PortReducer)]
    kind, cls = kinds[0]
    L = int(sample_mib * (1 << 20)) // es * es
    n = L // es
    ins = [np.ascontiguousarray(synth.bucket(dtype_id, n, k, "normal")).view(np.uint8)
           for k in range(n_workers)]
    store = np.empty(L, np.uint8)
    merged = np.empty(L, np.uint8)
    out = {}
    ncpu = os.cpu_count() or 1
    try:
        ncpu = len(os.sched_getaffinity(0))
    except Exception:
        pass
    for label, threads in (("default", 4), ("all", max(1, min(ncpu, 64)))):
        red = cls(nthreads=threads)

        def round_once():
            merged[:] = ins[0]           # stands in for the ps-lite receive buffer
            t0 = time.perf_counter()
            for s in ins[1:]:            # server.cc:127-130 SUM_RECV jobs
                red.sum(merged, s, L, dtype_id)
            red.copy(store, merged, L)   # server.cc:91 COPY_MERGED
            return time.perf_counter() - t0

        for _ in range(2):
            round_once()
        ts = []
        t_begin = time.perf_counter()
        budget = 10.0 if label == "default" else 4.0   # seconds of CPU work per leg
        while len(ts) < 10 or (time.perf_counter() - t_begin < budget and len(ts) < 2000):
            ts.append(round_once())
        med = statistics.median(ts)
        out[label] = dict(threads=threads, gibps=n_workers * L / med / GIB,
                          median_s=med, min_s=min(ts), reps=len(ts))
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    d = out["default"]
    return {
        "value": round(d["gibps"], 3), "unit": "GiB/s", "cores": d["threads"], "kind": kind,
        "sample": (f"{n_workers}-way server round (zero-copy first arrival, {n_workers - 1} "
                   f"CpuReducer::sum + 1 copy) of one {L / (1 << 20):.0f} MiB bucket, "
                   f"median of {d['reps']} reps (~10 s of CPU work); "
                   f"BYTEPS_OMP_THREAD_PER_GPU=4 (reference default)"),
        "all_cores": {"value": round(out["all"]["gibps"], 3), "cores": out["all"]["threads"],
                      "reps": out["all"]["reps"]},
        "cpu_model": cpu_model, "host_cpus": ncpu,
    }


def scatter_leg(dev, world: int, rank: int, n_workers: int, reps: int = 5,
                n_elems: int | None = None, fold=None) -> dict:
    """BASELINE config 4 on the node the bench runs on (N > 1 only): N workers'
    fp32 VGG-16 gradient vectors (553,430,176 B each) land on GPU 0; RCCL
    grouped P2P over xGMI moves each owner its key-space slice
    (ShardedReducer.scatter_reduce: the only data-path collective, SURVEY.md
    §8e), the owner folds; then the all-gather return leg (core_loops.cc:
    249-254).  Reported beside `value`, never as it.  Verified bit-exact on
    GPU 0 against torch's own left fold of the whole vector."""
    import torch
    import torch.distributed as dist
    from prophet_amd.buckets import vgg16_param_sizes
    from prophet_amd.shard import ShardedReducer
    E = n_elems or sum(vgg16_param_sizes())
    sr = ShardedReducer(E, fold=fold)   # fold=None: the HIP fold (tests inject a CPU one)
    root = 0
    cuda = dev.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize()
    gen = torch.Generator(device=dev)
    gen.manual_seed(4242)
    pushes = [torch.randn(E, device=dev, generator=gen) for _ in range(n_workers)] \
        if rank == root else None
    recv = [torch.empty(sr.owned, device=dev) for _ in range(n_workers)]
    owned = torch.empty(sr.owned, device=dev)
    full = torch.empty(E, device=dev)

    def timed(fn):
        fn()
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        sync()
        dist.barrier()
        t = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    t_scatter = timed(lambda: sr.scatter_reduce(root, pushes, recv, owned))
    t_gather = timed(lambda: sr.allgather(owned, full))
    ok = None
    if rank == root:
        ref = pushes[0].clone()
        for p in pushes[1:]:
            ref.add_(p)
        ok = bool(torch.equal(ref.view(torch.int32), full.view(torch.int32)))
    lo, hi = sr.ranges[root]
    egress = n_workers * (E - (hi - lo)) * 4
    return {"workload": f"{n_workers} x VGG-16-sized fp32 ({E * 4} B) landed on GPU 0, "
                        f"RCCL P2P scatter to {world} owners + owner fold, then all-gather",
            "scatter_fold_ms": round(t_scatter * 1e3, 3),
            "root_egress_GBps": round(egress / t_scatter / 1e9, 1),
            "allgather_ms": round(t_gather * 1e3, 3),
            "node_fold_GiBps": round(n_workers * E * 4 / t_scatter / GIB, 1),
            "exact_vs_torch_fold": ok}


def pmc_traffic(workload: str):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    PMC summary (tools/pmc_traffic.py -> profiles/pmc_traffic.json), if it was
    collected for this workload."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("workload") == workload:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # Bind this rank's GPU before the process group exists, so RCCL's
    # communicator (barrier, the max-over-ranks all_reduce) uses it.
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer

    dtype_id = DType(DTYPES[args.dtype][0])
    tdt = getattr(torch, DTYPES[args.dtype][1])
    es = torch.empty(0, dtype=tdt).element_size()
    mode = 1 if args.mode == "accum" else 0
    N = args.workers
    B = int(args.bucket_mib * (1 << 20)) // es * es
    n_elems = B // es
    red = GpuReducer(device=local_rank)

    # Input sets: the server's per-worker receive slots for this GPU's bucket,
    # carved from one HBM arena (prophet_amd/arena.py: skewed slots avoid the
    # channel aliasing of power-of-two-spaced buffers), plus the output slot.
    # Seeded N(0,1) gradients per (rank, set, worker), generated on device.
    torch.manual_seed(1000 + rank)
    sets = []
    for s in range(args.sets):
        if args.layout == "arena":
            slots = BucketArena(N + 1, B, dev).slots()
        else:
            slots = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(N + 1)]
        for t in slots[:N]:
            if tdt.is_floating_point:
                t.view(tdt).copy_(torch.randn(n_elems, device=dev))
            else:
                t.copy_(torch.randint(0, 256, (B,), dtype=torch.uint8, device=dev))
        sets.append((slots[N], slots[:N]))
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)

    def step(i):
        dst, srcs = sets[i % len(sets)]
        red.sum_n(dst, srcs, B, dtype_id, mode=mode, stream=stream)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(i)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps   # avg duration per launch, same stream
    t_step = wall / args.steps
    if world > 1:
        tt = torch.tensor([t_step, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_step, kern_ms = float(tt[0]), float(tt[1])

    # Correctness spot check of the last set against torch's own left fold.
    dst, srcs = sets[(args.steps + args.warmup - 1) % len(sets)]
    chk = srcs[0].view(tdt)[: 1 << 20].clone()
    for s in srcs[1:]:
        chk.add_(s.view(tdt)[: 1 << 20])
    ok = bool(torch.equal(chk.view(torch.uint8), dst[: chk.numel() * es])) if mode == 0 else None

    alg_bytes = (N + 1) * B
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    workload = f"{N}-way {args.dtype} left-fold sum of one {B / (1 << 20):.0f} MiB bucket per GPU"
    if mode:
        workload += " (fp32-accumulate mode)"
    tv, tnt, tgrid, tocc = red.get_tuning()
    line = {
        "metric": "GiB/s device-resident N-way gradient-bucket sum (fp32/fp16), 1/2/4/8 GPUs",
        "value": round(world * N * B / t_step / GIB, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (torch.randn on device, seeded per rank), resident in HBM, "
                f"{args.sets} rotated input sets, layout={args.layout}",
        "config": {"workload": workload, "n_workers": N, "bucket_bytes": B,
                   "parallelism": f"key-space shard x{world}", "kernel": "byteps_reduce_sum_n",
                   "tuning": {"vpt": tv, "nt": tnt, "max_grid": tgrid,
                                                 "wg_per_cu": tocc}},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": pmc_traffic(workload),
                     "alg_bytes_per_launch": alg_bytes, "kernel_ms": round(kern_ms, 5)},
        "check_vs_torch_fold": ok,
    }
    if world == 1:
        if rank == 0 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(N, int(dtype_id), args.cpu_sample_mib)
            except Exception as e:  # report, never hide
                line["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(line), flush=True)
        return
    # N > 1: the headline line is complete; the config-4 scatter leg runs after
    # it under a watchdog, so a stuck or failing collective can cost only the
    # extra field, never the line.
    import threading
    lock = threading.Lock()
    state = {"printed": False}

    def emit_and_maybe_exit(exit_now: bool):
        with lock:
            if rank == 0 and not state["printed"]:
                print(json.dumps(line), flush=True)
                state["printed"] = True
        if exit_now:
            os._exit(0)

    watchdog = threading.Timer(180.0, lambda: (line.setdefault(
        "scatter", {"error": "timed out after 180 s"}), emit_and_maybe_exit(True)))
    watchdog.daemon = True
    watchdog.start()
    if not args.no_scatter:
        try:
            line["scatter"] = scatter_leg(dev, world, rank, N)
        except Exception as e:  # report, never hide
            line["scatter"] = {"error": repr(e)}
    emit_and_maybe_exit(False)
    dist.destroy_process_group()
    watchdog.cancel()


if __name__ == "__main__":
    main()
