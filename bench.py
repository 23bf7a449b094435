#!/usr/bin/env python3
"""Benchmark of the device-resident N-way gradient-bucket sum (BASELINE.json).

Workload (BASELINE.json configs[1]): 8-way fp32 left fold
of one 256 MiB bucket per GPU — the server round of byteps/server/server.cc:
216-273 for one key, done as ONE fused HIP kernel through the C ABI
(byteps_reduce_sum_n).  Inputs are synthetic gradients (seeded N(0,1)),
resident in HBM before the timed region; 3 input sets are rotated so every
step streams from HBM rather than the 256 MiB Infinity Cache.

Multi-GPU: one process per GPU, either launched by the driver
(``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``:
RANK/LOCAL_RANK/WORLD_SIZE come from the environment) or by this script
itself (``python bench.py --gpus N`` with no WORLD_SIZE set: the parent starts
N rank processes BEFORE it touches the GPU, waits, and exits with their
status; rank 0 prints the line).  Each GPU owns a contiguous slice of the key
space and reduces its own 256 MiB bucket per step (weak scaling, no data-path
collective — the sum is element-wise).  Barrier + synchronize bracket the
timed steps, the max over ranks is taken, and value = total gradient bytes
aggregated by all ranks / time.

``scaling`` (every N): BASELINE config 4 — the 8-way fp32 VGG-16 gradient set
(553,430,176 B per worker) sharded over the N GPUs by the reference's
reduce-scatter ownership (core_loops.cc:208-247): per-GPU fold time of the
owned slice (max over ranks), the G=1 time of the whole set measured in the
same run, strong-scaling speedup/efficiency, and, for N > 1, the RCCL P2P
scatter from a landing GPU plus the all-gather return leg.

``local_reduce`` (N > 1): the worker's local reduce across the GPUs — every
rank's full VGG-16-sized gradient summed by rank-order P2P reduce-scatter +
HIP fold + all-gather, with RCCL's own all_reduce timed beside it.

``e2e_cfg5`` (every N, GPU runs): BASELINE config 5 from host memory — 16
workers' 256 MiB bf16 pushes in pinned host buffers, each GPU streaming its
key-space slice H2D -> fold -> D2H over its own PCIe link: the PCIe-inclusive
node rate the north star asks to record (never ``value``).

Prints ONE JSON line (rank 0).  Metric: GiB/s = N_workers * B / t / 2^30 per
step, summed over GPUs.  ``roofline`` prices the dominant kernel at
(N_workers + 1) * B algorithmic HBM bytes per launch against 8.0 TB/s;
``cpu_baseline`` times the clean-room CPU restatement of CpuReducer
(oracle/bpsr_oracle.c, proven bit-identical to the reference by the golden
vectors) running the reference server round on the headline 256 MiB bucket
on the host cores.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
LEAD_CYCLES = 2_000_000  # spin ahead of a timed block (~1 ms of GPU clock)
GIB = float(1 << 30)
WATCHDOG_EXIT = 3  # every rank's status when the N > 1 watchdog fires
RCCL_EXIT = 4      # every rank's status when the communicator is not N ranks on N GPUs
METRIC = "GiB/s device-resident N-way gradient-bucket sum (fp32/fp16), 1/2/4/8 GPUs"
# --dtype name -> (byteps DataType id, torch dtype name); ids: common.h:52-65 (+ bf16 = 11)
DTYPES = {"f32": (0, "float32"), "f64": (1, "float64"), "f16": (2, "float16"),
          "u8": (3, "uint8"), "i32": (4, "int32"), "i8": (5, "int8"), "i64": (6, "int64"),
          "bf16": (11, "bfloat16")}
# What decides the headline kernel's code and launch: the ISA signature of
# fold_kernel<OpF32,2,true,8> written by the build (prophet_amd/csrc/Makefile)
# plus the launch-geometry rules of the C ABI (tuning defaults, residency by
# source count: this span of bpsr_api.cpp).  A committed PMC traffic record is
# quoted only while this id matches (roofline.traffic_source).  Without a
# build signature, the kernel sources are hashed instead.
KERNEL_SIG = "prophet_amd/libbpsr.fold_f32_8.sig"
KERNEL_SOURCES = ("prophet_amd/csrc/bpsr_kernels_impl.h", "prophet_amd/csrc/bpsr_ops.h",
                  "prophet_amd/csrc/bpsr_internal.h", "prophet_amd/csrc/bpsr_k_f32.hip")
KERNEL_SOURCE_SPANS = (("prophet_amd/csrc/bpsr_api.cpp", "static Tuning& tuning_storage()",
                        "static inline hipStream_t to_stream"),
                       ("prophet_amd/csrc/bpsr_internal.h", "inline size_t occ_lds_bytes",
                        "// The 1-workgroup-per-CU cap pays"))


def parse(argv=None):
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
    p.add_argument("--skew", type=int, default=-1,
                   help="arena: bytes between consecutive slots beyond the 64 KiB-rounded "
                        "bucket (default: prophet_amd.arena.DEFAULT_SKEW)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-scaling", action="store_true",
                   help="skip the config-4 (VGG-16 sharded) scaling object")
    p.add_argument("--no-fp16", action="store_true",
                   help="N = 1: skip the fp16 run of the headline workload")
    p.add_argument("--no-cfg3", action="store_true",
                   help="N = 1: skip the config-3 (ResNet-50 fp16 Prophet blocks) object")
    p.add_argument("--no-e2e", action="store_true",
                   help="skip the config-5 host-resident (PCIe-inclusive) object")
    p.add_argument("--no-server", action="store_true",
                   help="skip the config-1 host-resident PS-server-group object")
    p.add_argument("--e2e-bucket-mib", type=int, default=256,
                   help="config-5 object: bucket MiB per worker (16 workers; BASELINE: 256)")
    p.add_argument("--no-scatter", action="store_true",
                   help="N > 1: skip the RCCL scatter + all-gather leg of `scaling`")
    p.add_argument("--scaling-elems", type=int, default=0,
                   help="elements per worker of the config-4 set (0: VGG-16, 138,357,544)")
    p.add_argument("--cpu-sample-mib", type=float, default=256.0,
                   help="bucket size of the CPU baseline sample (headline: 256)")
    p.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                   help="cpu: launcher/plumbing self-test over gloo with torch's CPU add "
                        "(no HIP; the line is marked and is not a measurement)")
    p.add_argument("--rehearse-one-gpu", action="store_true",
                   help="N > 1 rehearsal on a 1-GPU box: every rank on cuda:0 with the HIP "
                        "fold, gloo for the barrier / max-over-ranks (RCCL refuses two ranks "
                        "on one GPU); the scatter and local-reduce legs move CUDA tensors "
                        "through gloo; the line is marked, not a measurement")
    return p.parse_args(argv)


# --------------------------------------------------------------------------
# launcher: N rank processes, started before anything touches the GPU


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv: list[str], timeout_s: float = 1500.0) -> int:
    """Start ``n`` copies of this script as ranks 0..n-1 (one per GPU) and wait.

    The parent never initialises the GPU: it only spawns children (a child
    process, never an exec) and relays their status.  Rank 0's stdout is the
    parent's; the other ranks' stdout goes to stderr so exactly one JSON line
    reaches stdout.  If a rank fails, the others are terminated (exact PIDs)."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env, stdout=None if r == 0 else sys.stderr.fileno()))
    t_end = time.monotonic() + timeout_s
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        # the first rank to fail decides the status (others may then be
        # terminated by this loop, which must not mask it)
        bad = [c for c in codes if c not in (None, 0)]
        if bad or time.monotonic() > t_end:
            rc = bad[0] if bad else 124
            print(f"bench launcher: rank status {codes}; exiting {rc}", file=sys.stderr)
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=15)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(0.1)
    return rc


# --------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1 only): the clean-room restatement


def cpu_baseline(n_workers: int, dtype_id: int, sample_mib: float) -> dict | None:
    """CpuReducer server round on host cores: zero-copy first arrival, N-1
    ``sum`` calls (server.cc:127-130 SUM_RECV) and the ``copy`` to the store
    (server.cc:91 COPY_MERGED), timed with the clean-room restatement
    (oracle/bpsr_oracle.c, OpenMP like cpu_reducer.cc:85-92; bit-identical to
    the reference on every golden vector).  The reference's own build
    (oracle/_ref) pins the restatement in the build container's tests; it
    never travels to the GPU box (.gpurunignore)."""
    import numpy as np

    from oracle.oracle import PortReducer
    from prophet_amd import synth

    es = {0: 4, 1: 8, 2: 2, 3: 1, 4: 4, 5: 1, 6: 8, 11: 2}[dtype_id]
    L = int(sample_mib * (1 << 20)) // es * es
    n = L // es
    if dtype_id == 0:
        # numpy's generator: 256 MiB x N in a second or two (synth's splitmix
        # Box-Muller stream takes ~10x longer at this size); values N(0,1) alike
        ins = [np.random.default_rng(1000 + k).standard_normal(n, dtype=np.float32).view(np.uint8)
               for k in range(n_workers)]
    else:
        ins = [np.ascontiguousarray(synth.bucket(dtype_id, n, k, "normal")).view(np.uint8)
               for k in range(n_workers)]
    store = np.empty(L, np.uint8)
    merged = np.empty(L, np.uint8)
    ncpu = os.cpu_count() or 1
    try:
        ncpu = len(os.sched_getaffinity(0))
    except Exception:
        pass

    def round_once(red):
        merged[:] = ins[0]           # stands in for the ps-lite receive buffer
        t0 = time.perf_counter()
        for s in ins[1:]:
            assert red.sum(merged, s, L, dtype_id) == 0
        red.copy(store, merged, L)
        return time.perf_counter() - t0

    def legs(impls, slices):
        """Interleaved timing: each slice runs every implementation for its
        share of seconds in turn, so a noisy host (other jobs on the box's
        shared cores) weighs on all of them alike.  Median per implementation."""
        ts = {k: [] for k in impls}
        for red, _ in impls.values():
            for _ in range(2):
                round_once(red)
        for _ in range(slices):
            for k, (red, share) in impls.items():
                t_s = time.perf_counter()
                while time.perf_counter() - t_s < share or not ts[k]:
                    ts[k].append(round_once(red))
        return {k: dict(gibps=n_workers * L / statistics.median(v) / GIB,
                        median_s=statistics.median(v), min_s=min(v), reps=len(v))
                for k, v in ts.items()}

    class _Baseline:
        """The restatement in the reference's loop shape (bpsr_oracle_sum_simd:
        `omp parallel for simd`, AVX) where it has one; else its bit-level form."""
        def __init__(self, threads):
            self.p = PortReducer(nthreads=threads)
            self.simd = dtype_id in (0, 1, 3, 4, 5, 6)

        def sum(self, d, s, n, dt):
            return self.p.sum_simd(d, s, n, dt) if self.simd else self.p.sum(d, s, n, dt)

        def copy(self, d, s, n):
            return self.p.copy(d, s, n)

    # the host share this process may use: OMP_NUM_THREADS when the box sets it
    # (16 per GPU on the GPU pool, whose affinity mask shows every host CPU)
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        share = 0
    all_threads = max(1, min(share or ncpu, 64))
    impls = {"port": (_Baseline(4), 1.0), "all": (_Baseline(all_threads), 0.4)}
    res = legs(impls, 10)
    default, allc = res["port"], res["all"]
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(default["gibps"], 3), "unit": "GiB/s", "cores": 4,
        "kind": "port",
        "sample": (f"{n_workers}-way server round (zero-copy first arrival, {n_workers - 1} "
                   f"CpuReducer::sum + 1 copy) of one {L / (1 << 20):.0f} MiB bucket"
                   f"{' (the headline bucket)' if L == 256 << 20 else ''}, clean-room restatement oracle/bpsr_oracle.c in the "
                   f"reference's omp-simd loop shape (bpsr_oracle_sum_simd), median of "
                   f"{default['reps']} reps (~10 s of CPU work, in 10 slices interleaved "
                   f"with the other legs); 4 OpenMP threads = "
                   f"BYTEPS_OMP_THREAD_PER_GPU default (cpu_reducer.cc:40-44)"),
        "all_cores": {"value": round(allc["gibps"], 3), "cores": all_threads,
                      "reps": allc["reps"]},
        "cpu_model": cpu_model, "host_cpus": ncpu,
    }


# --------------------------------------------------------------------------
# folds and timers for the two device kinds


def _torch_fold(dst, srcs):
    """--device cpu plumbing self-test only: torch's own CPU left fold."""
    dst.copy_(srcs[0])
    for s in srcs[1:]:
        dst.add_(s)


class _Clock:
    """Average duration of a block of launches: HIP events on the launch
    stream (cuda) or wall time (cpu self-test)."""

    def __init__(self, dev):
        self.cuda = dev.type == "cuda"
        if self.cuda:
            import torch
            self.stream = torch.cuda.current_stream(dev)

    def sync(self):
        if self.cuda:
            import torch
            torch.cuda.synchronize()

    def time(self, fn, reps: int, lead: bool = False) -> float:
        """ms per call of fn(i) over reps calls (after the caller's warm-up).
        ``lead``: a short spin kernel goes first on the stream, so the host
        has queued the start event and the first launches by the time the GPU
        reaches them — the span then holds device work only, not the host's
        issue latency of the first launch (≈ 2 % of ten 0.1-ms folds).  Not
        for the headline: its timed region is also the wall-clock step time,
        and 100 launches of 0.36 ms amortise that latency anyway."""
        if self.cuda:
            import torch
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            if lead:
                with torch.cuda.stream(self.stream):
                    torch.cuda._sleep(LEAD_CYCLES)
            e0.record(self.stream)
            for i in range(reps):
                fn(i)
            e1.record(self.stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / reps
        t0 = time.perf_counter()
        for i in range(reps):
            fn(i)
        return (time.perf_counter() - t0) * 1e3 / reps

    def blocks(self, fn, n_blocks: int, per_block: int, first: int = 0) -> list[float]:
        """ms per call in each of ``n_blocks`` consecutive blocks of
        ``per_block`` back-to-back calls fn(first + i), one event at every
        block boundary (median and min over repetitions).  Not
        one event pair per launch: an event between two launches cost the
        second ≈ 27 µs on MI355X (r03s31: per-launch pairs 0.397 ms median vs
        0.370 averaged back to back, which rocprofv3's kernel durations
        confirm), so per-launch brackets would time the events."""
        if self.cuda:
            import torch
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(n_blocks + 1)]
            ev[0].record(self.stream)
            for b in range(n_blocks):
                for i in range(per_block):
                    fn(first + b * per_block + i)
                ev[b + 1].record(self.stream)
            torch.cuda.synchronize()
            return [ev[b].elapsed_time(ev[b + 1]) / per_block for b in range(n_blocks)]
        out = []
        for b in range(n_blocks):
            t0 = time.perf_counter()
            for i in range(per_block):
                fn(first + b * per_block + i)
            out.append((time.perf_counter() - t0) * 1e3 / per_block)
        return out


def _max_over_ranks(dist, dev, vals: list[float]) -> list[float]:
    import torch
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return vals
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t]


def _all_true(dist, dev, flag: bool) -> bool:
    import torch
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t[0]) == 1)


def _left_fold_equal(out, srcs) -> bool:
    """out (typed tensor) == torch's own left fold of srcs, bit for bit."""
    import torch
    ref = srcs[0].clone()
    for s in srcs[1:]:
        ref.add_(s)
    return bool(torch.equal(ref.view(torch.int32), out.view(torch.int32)))


# --------------------------------------------------------------------------
# config 4: VGG-16 set sharded over the GPUs


def scaling_leg(dev, world: int, rank: int, n_workers: int, fold, reps: int = 20,
                n_elems: int | None = None, sets: int = 2) -> dict:
    """BASELINE config 4, device-resident part: every worker's fp32 VGG-16
    gradient vector is cut by the reference's reduce-scatter ownership
    (``owner_ranges``, core_loops.cc:208-211) and each GPU folds its owned
    slice of the N pushes (already on their owner, as ``reduce_from_host``
    leaves them).  Strong scaling: total work fixed, so the per-GPU fold time
    should fall as 1/G.  The G=1 time of the whole set is measured in the same
    run on rank 0 (the other ranks wait at a barrier)."""
    import torch
    import torch.distributed as dist
    from prophet_amd.arena import BucketArena
    from prophet_amd.buckets import vgg16_param_sizes
    from prophet_amd.shard import owner_ranges

    E = n_elems or sum(vgg16_param_sizes())
    ranges = owner_ranges(E, world)
    clock = _Clock(dev)
    multi = world > 1 and dist.is_initialized()
    gen = torch.Generator(device=dev)

    def make_sets(m):
        out = []
        for s in range(sets):
            slots = [t.view(torch.float32) for t in BucketArena(n_workers + 1, 4 * m, dev).slots()]
            for k in range(n_workers):
                gen.manual_seed(7000 + 97 * rank + 13 * s + k)
                slots[k].copy_(torch.randn(m, device=dev, generator=gen))
            out.append((slots[n_workers], slots[:n_workers]))
        return out

    def time_folds(data) -> float:
        def step(i):
            dst, srcs = data[i % len(data)]
            fold(dst, srcs)
        for i in range(2):
            step(i)
        clock.sync()
        return clock.time(step, reps, lead=True)

    res: dict = {}
    # G = 1: the whole set on one GPU (rank 0), measured in this run
    t1 = None
    if rank == 0:
        whole = make_sets(E)
        t1 = time_folds(whole)
        del whole
    if multi:
        dist.barrier()
    lo, hi = ranges[rank]
    m = hi - lo
    data = make_sets(m) if m else []
    if multi:
        clock.sync()
        dist.barrier()
    t_g = time_folds(data) if m else 0.0
    ok = _left_fold_equal(data[0][0], data[0][1]) if m else True
    t_g, = _max_over_ranks(dist, dev, [t_g])
    ok = _all_true(dist, dev, ok)
    if world == 1:
        t1 = t_g
    t1s = _max_over_ranks(dist, dev, [t1 or 0.0])[0]
    alg_per_gpu = (n_workers + 1) * 4 * max(hi_ - lo_ for lo_, hi_ in ranges)
    res.update({
        "workload": (f"config 4: {n_workers}-way fp32 VGG-16 set ({E * 4} B per worker) sharded "
                     f"over {world} GPU(s) by reduce-scatter ownership (core_loops.cc:208-211); "
                     f"owned slices device-resident; strong scaling"),
        "shard_elems": [hi_ - lo_ for lo_, hi_ in ranges],
        "g1_fold_ms": round(t1s, 4),
        "per_gpu_fold_ms": round(t_g, 4),
        "speedup_vs_g1": round(t1s / t_g, 3) if t_g else None,
        "strong_efficiency": round(t1s / (world * t_g), 3) if t_g else None,
        "node_GiBps": round(n_workers * E * 4 / (t_g * 1e-3) / GIB, 1) if t_g else None,
        "per_gpu_frac_of_roofline": round(alg_per_gpu / (t_g * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
        if t_g else None,
        "exact_vs_torch_fold": ok,
        "reps": reps,
    })
    return res


def shard_comm(dev):
    """The shard C ABI's communicator (include/bpsr/shard.h) for this rank:
    torch's own ProcessGroupNCCL communicator wrapped (the caller-owned
    ncclComm_t a core_loops.cc caller passes from NcclManager::GetComm), else
    a communicator of the library's own (unique id carried over the torch
    group, NcclManager::ConstructRings).  Returns (ShardComm, how)."""
    import torch.distributed as dist
    from prophet_amd.shard import ShardComm
    try:
        ptr = dist.group.WORLD._get_backend(dev)._comm_ptr()
        if ptr:
            return ShardComm.wrap(ptr), "wrapped torch ProcessGroupNCCL communicator"
    except Exception:  # noqa: BLE001 — fall back to a communicator of our own
        pass
    return (ShardComm.from_group(device=dev.index),
            "library-owned RCCL communicator (unique id over the torch group)")


def rccl_rank_view(dev, comm, rank: int) -> dict:
    """This rank's view of the communicator the byteps_shard_* calls use
    (byteps_shard_comm_info: RCCL's own ncclCommCount / ncclCommUserRank /
    ncclCommCuDevice, read when the communicator was made or wrapped,
    nccl_manager.cc:74-127), the device torch bound, its PCI address, the RCCL
    version the library bound, and the visible device count."""
    import torch
    from prophet_amd.shard import rccl_version
    p = torch.cuda.get_device_properties(dev)
    return {"rank": rank, "comm_world": comm.world, "comm_rank": comm.rank,
            "comm_device": comm.device, "device": dev.index,
            "pci_bus_id": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "rccl_version": rccl_version(), "device_count": torch.cuda.device_count()}


def rccl_problems(views: list, world: int) -> list:
    """What makes a set of per-rank communicator views NOT 'N ranks on N
    distinct GPUs' (empty when the communicator is what the line claims)."""
    out = []
    if len(views) != world:
        out.append(f"{len(views)} rank views for WORLD_SIZE={world}")
    for v in views:
        if v["comm_world"] != world:
            out.append(f"rank {v['rank']}: communicator world {v['comm_world']} != {world}")
        if v["comm_rank"] != v["rank"]:
            out.append(f"rank {v['rank']}: communicator rank {v['comm_rank']}")
        if v["comm_device"] != v["device"]:
            out.append(f"rank {v['rank']}: communicator device {v['comm_device']} "
                       f"!= bound device {v['device']}")
    buses = [v["pci_bus_id"] for v in views]
    if len(set(buses)) != len(buses):
        out.append(f"ranks share a GPU: {buses}")
    if len({v["rccl_version"] for v in views}) > 1:
        out.append("ranks bound different RCCL versions")
    return out


def rccl_object(dev, comm, world: int, rank: int, view: dict | None = None) -> dict:
    """The line's ``rccl`` object at N > 1 on GPUs: every rank's view,
    gathered over the torch group, and the problems found (empty = the
    exchange legs' communicator had N ranks on N distinct GPUs).  ``view``
    replaces this rank's own (the CPU test of the failing path)."""
    import torch.distributed as dist
    views = [None] * world
    dist.all_gather_object(views, view if view is not None else rccl_rank_view(dev, comm, rank))
    return {"transport": "rccl", "world": world, "ranks": views,
            "problems": rccl_problems(views, world)}


def _transport(comm) -> str:
    return "rccl-shard-abi" if comm is not None else "torch-p2p"


def uses_shard_abi(world: int, cuda: bool, rehearse: bool) -> bool:
    """Do the N > 1 exchange legs run through the shard C ABI over RCCL?  On
    GPUs, one rank per GPU: yes.  Rehearsals with every rank on one GPU (RCCL
    refuses two ranks on one device) and the CPU self-test: torch P2P over gloo."""
    return world > 1 and cuda and not rehearse


def scatter_leg(dev, world: int, rank: int, n_workers: int, reps: int = 5,
                n_elems: int | None = None, fold=None, comm=None) -> dict:
    """BASELINE config 4's exchange (N > 1 only): N workers' fp32 VGG-16
    gradient vectors (553,430,176 B each) land on GPU 0; RCCL grouped P2P over
    xGMI moves each owner its key-space slice (ShardedReducer.scatter_reduce:
    the only data-path collective), the owner folds; then the
    all-gather return leg (core_loops.cc:249-254).  With ``comm`` (GPU runs:
    a :class:`ShardComm` over RCCL) every call is ONE byteps_shard_* call —
    the code a core_loops.cc caller binds in place of PostNcclCalls; without
    it (gloo rehearsals, CPU tests) torch.distributed P2P moves the slices.
    Verified bit-exact on GPU 0 against torch's own left fold of the whole
    vector."""
    import torch
    import torch.distributed as dist
    from prophet_amd.buckets import vgg16_param_sizes
    from prophet_amd.shard import ShardedReducer
    if os.environ.get("BPSR_BENCH_TEST_STALL") == "scatter":
        time.sleep(3600)                # test hook: a collective that never returns
    E = n_elems or sum(vgg16_param_sizes())
    # fold=None: the HIP fold (tests inject a CPU one); comm: the shard C ABI
    sr = ShardedReducer(E, fold=fold, comm=comm)
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
        ok = _left_fold_equal(full, pushes)
    lo, hi = sr.ranges[root]
    egress = n_workers * (E - (hi - lo)) * 4
    return {"workload": f"{n_workers} x VGG-16-sized fp32 ({E * 4} B) landed on GPU 0, "
                        f"RCCL P2P scatter to {world} owners + owner fold, then all-gather",
            "transport": _transport(comm),
            "scatter_fold_ms": round(t_scatter * 1e3, 3),
            "root_egress_GBps": round(egress / t_scatter / 1e9, 1),
            "allgather_ms": round(t_gather * 1e3, 3),
            "node_fold_GiBps": round(n_workers * E * 4 / t_scatter / GIB, 1),
            "exact_vs_torch_fold": ok}


def local_reduce_leg(dev, world: int, rank: int, reps: int = 5, n_elems: int | None = None,
                     fold=None, comm=None) -> dict:
    """The worker's local reduce (core_loops.cc:184-263),
    N > 1 only: every GPU holds its own full fp32 VGG-16 gradient vector and
    all of them are summed across the node.  ``ShardedReducer.allreduce`` =
    RCCL grouped P2P of every slice to its owner (the reduce-scatter
    ownership of core_loops.cc:208-211), the HIP fold of the slices in RANK
    order, then the all-gather return leg — bit-reproducible, unlike a ring.
    RCCL's own ``all_reduce`` on the same bytes is timed beside it for
    reference (its summation order follows the ring).  Exactness: strided
    windows of the result against torch's left fold, in rank order, of every
    rank's vector regenerated from its seed.  ``comm`` as in scatter_leg:
    byteps_shard_reduce_scatter + byteps_shard_allgather over RCCL."""
    import torch
    import torch.distributed as dist
    from prophet_amd.buckets import vgg16_param_sizes
    from prophet_amd.shard import ShardedReducer
    E = n_elems or sum(vgg16_param_sizes())
    sr = ShardedReducer(E, fold=fold, comm=comm)
    cuda = dev.type == "cuda"

    def vec(r):
        g = torch.Generator(device=dev)
        g.manual_seed(6100 + r)
        return torch.randn(E, device=dev, generator=g)
    local = vec(rank)
    out = torch.empty(E, device=dev)
    recv = [torch.empty(sr.owned, device=dev) for _ in range(world)]
    owned = torch.empty(sr.owned, device=dev)
    ring = local.clone()

    def sync():
        if cuda:
            torch.cuda.synchronize()

    def timed(fn):
        fn()
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        sync()
        dist.barrier()
        return _max_over_ranks(dist, dev, [(time.perf_counter() - t0) / reps])[0]

    t_det = timed(lambda: sr.allreduce(local, out, recv, owned))
    t_ring = timed(lambda: dist.all_reduce(ring))
    ok = True
    win = 1 << 16
    starts = sorted({0, E // 3, E // 2, max(0, E - win)})
    for w0 in starts:
        w1 = min(E, w0 + win)
        want = None
        for r in range(world):          # the left fold in rank order
            x = vec(r)[w0:w1]
            want = x.clone() if want is None else want.add_(x)
        ok = ok and bool(torch.equal(want.view(torch.int32), out[w0:w1].view(torch.int32)))
    ok = _all_true(dist, dev, ok)
    nbytes = E * 4
    return {"workload": (f"worker local reduce: {world} GPUs each holding a {nbytes} B fp32 "
                         f"(VGG-16-sized) gradient; rank-order P2P reduce-scatter + HIP fold + "
                         f"all-gather (ShardedReducer.allreduce) vs RCCL all_reduce"),
            "transport": _transport(comm),
            "allreduce_ms": round(t_det * 1e3, 3),
            "busbw_GBps": round(2 * (world - 1) / world * nbytes / t_det / 1e9, 1),
            "rccl_allreduce_ms": round(t_ring * 1e3, 3),
            "rccl_busbw_GBps": round(2 * (world - 1) / world * nbytes / t_ring / 1e9, 1),
            "exact_vs_rank_order_fold": ok, "reps": reps}


# --------------------------------------------------------------------------
# the metric's other dtype: the same bucket in fp16


def fp16_leg(dev, red, N: int, B: int, steps: int, sets: int = 3) -> dict:
    """The headline workload in fp16 (the metric names fp32/fp16): N workers'
    B-byte fp16 buckets in the same skewed arena, folded with the reference's
    fp16 rule (fp32 add, RNE to fp16 after every add — cpu_reducer.cc:94-128).
    HIP-event time per launch on the launch stream; bit-exact check against
    torch's own half-precision left fold (it rounds after every add too)."""
    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType
    stream = torch.cuda.current_stream(dev)
    gen = torch.Generator(device=dev)
    data = []
    for s in range(sets):
        slots = BucketArena(N + 1, B, dev).slots()
        for k in range(N):
            gen.manual_seed(5000 + 31 * s + k)
            slots[k].view(torch.float16).copy_(
                torch.randn(B // 2, device=dev, generator=gen).half())
        data.append((slots[N], slots[:N]))
    clock = _Clock(dev)

    def step(i):
        dst, srcs = data[i % sets]
        red.sum_n(dst, srcs, B, DType.FLOAT16, stream=stream)
    for i in range(3):
        step(i)
    clock.sync()
    ms = clock.time(step, steps)
    dst, srcs = data[(steps - 1) % sets]
    step(steps - 1)
    clock.sync()
    ref = srcs[0].view(torch.float16).clone()
    for x in srcs[1:]:
        ref.add_(x.view(torch.float16))
    ok = bool(torch.equal(ref.view(torch.uint8), dst))
    alg = (N + 1) * B
    return {"workload": f"{N}-way f16 left-fold sum of one {B / (1 << 20):.0f} MiB bucket",
            "kernel_ms": round(ms, 5), "value_GiBps": round(N * B / (ms * 1e-3) / GIB, 1),
            "frac_of_roofline": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "exact_vs_torch_fold": ok, "steps": steps}


# --------------------------------------------------------------------------
# config 5: host-resident pushes, PCIe-inclusive, sharded over the GPUs


def e2e_leg(dev, world: int, rank: int, n_workers: int = 16, bucket_bytes: int = 256 << 20,
            reps: int = 3, link: dict | None = None) -> dict:
    """BASELINE config 5 end to end, key-space sharded: 16 workers' 256 MiB
    bf16 pushes (4 GiB) start in pinned host memory, as ps-lite receive
    buffers would (server.cc:174); each GPU streams ITS slice of every push
    (owner_ranges, core_loops.cc:208-211) host -> HBM -> fold -> host through
    ``StreamingReducer`` (H2D, fold and D2H on three streams; ``reduce_from_host``
    with the aggregate pulled back), over its own PCIe link, no collective.
    Node rate = all pushed bytes / (max over ranks of the blocking call);
    ``frac_of_link`` = the link's shortest time for this GPU's H2D (its slices
    of the pushes) and D2H (the aggregate slice) over the measured time
    (link_bound_s, ``link`` measured in the same run).  PCIe-inclusive: never
    ``value``.  Exactness: strided windows of the pulled
    slice against torch's own bf16 left fold (fp32 add, RNE to bf16 per add)
    of the same windows on the device."""
    import torch
    import torch.distributed as dist
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    from prophet_amd.shard import owner_ranges
    from prophet_amd.stream import StreamingReducer
    E = bucket_bytes // 2
    lo, hi = owner_ranges(E, world)[rank]
    m = hi - lo
    nb = 2 * m
    gen = torch.Generator(device=dev)
    pushes = []
    for k in range(n_workers):
        gen.manual_seed(9000 + 16 * rank + k)
        h = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
        h.view(torch.bfloat16).copy_(torch.randn(m, device=dev, generator=gen).bfloat16())
        pushes.append(h)
    out = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    sr = StreamingReducer(n_workers, device=dev, reducer=GpuReducer(device=dev.index))
    multi = world > 1 and dist.is_initialized()
    torch.cuda.synchronize()
    sr.reduce(pushes, out, nb, DType.BFLOAT16)          # warm-up (pages, streams)
    times = []
    for _ in range(reps):
        if multi:
            dist.barrier()
        t0 = time.perf_counter()
        sr.reduce(pushes, out, nb, DType.BFLOAT16)
        times.append(time.perf_counter() - t0)
    t = _max_over_ranks(dist, dev, [statistics.median(times)])[0]
    ok = True
    win = 1 << 16
    for w0 in range(0, m, max(win, m // 8)):
        w1 = min(m, w0 + win)
        ref = pushes[0].view(torch.bfloat16)[w0:w1].to(dev)
        for h in pushes[1:]:
            ref.add_(h.view(torch.bfloat16)[w0:w1].to(dev))
        ok = ok and bool(torch.equal(ref.view(torch.int16).cpu(),
                                     out.view(torch.bfloat16)[w0:w1].view(torch.int16)))
    ok = _all_true(dist, dev, ok)
    total = n_workers * bucket_bytes
    out = {"workload": (f"config 5: {n_workers}-way bf16, {n_workers} x {bucket_bytes >> 20} MiB "
                        f"pinned host pushes ({total / GIB:.0f} GiB), key-space sharded over "
                        f"{world} GPU(s), streamed H2D + fold + D2H, aggregate back in host memory"),
           "node_e2e_GiBps": round(total / t / GIB, 1),
           "per_gpu_e2e_GiBps": round(n_workers * nb / t / GIB, 1),
           "ms": round(t * 1e3, 2), "reps": reps, "pcie_inclusive": True,
           "exact_vs_torch_fold_windows": ok}
    out.update(link_fracs(n_workers * nb, nb, t, link))    # every push in, the aggregate out
    return out


# --------------------------------------------------------------------------
# config 1 through the PS server group, host-resident, one server per GPU


def link_bound_s(h2d_bytes: float, d2h_bytes: float, link: dict) -> float:
    """Shortest time this GPU's link (``pcie_leg``'s measured rates) can move
    ``h2d_bytes`` in and ``d2h_bytes`` out: while both directions run each gets
    half the measured both-ways rate (the link shares it: 2 x ~43 GB/s, not
    2 x 54), the rest goes at its own one-way rate."""
    both = min(h2d_bytes, d2h_bytes)
    t = both / (link["bidir_GBps"] * 1e9 / 2)
    if h2d_bytes > d2h_bytes:
        t += (h2d_bytes - d2h_bytes) / (link["h2d_GBps"] * 1e9)
    else:
        t += (d2h_bytes - h2d_bytes) / (link["d2h_GBps"] * 1e9)
    return t


def link_fracs(h2d_bytes: float, d2h_bytes: float, t: float, link: dict | None) -> dict:
    """A host-resident object's use of the link: ``frac_of_link`` = the
    link's shortest time for the object's H2D + D2H bytes (link_bound_s) over
    its measured time; ``frac_of_h2d`` = its H2D rate over the link's one-way
    H2D rate (ignores the D2H the object must also move)."""
    if not link or not link.get("h2d_GBps"):
        return {}
    return {"frac_of_link": round(link_bound_s(h2d_bytes, d2h_bytes, link) / t, 4),
            "frac_of_h2d": round(h2d_bytes / t / (link["h2d_GBps"] * 1e9), 4),
            "link_bound_ms": round(link_bound_s(h2d_bytes, d2h_bytes, link) * 1e3, 3)}


def pcie_leg(dev, red=None, nbytes: int = 64 << 20, reps: int = 10) -> dict:
    """This GPU's PCIe link, measured in the same run as the host-resident
    objects (their rate "including H2D and D2H" needs the link's
    own rate beside it): pinned host <-> HBM copies of ``nbytes`` on side
    streams — H2D alone (SDMA, hipMemcpyAsync), D2H alone (SDMA), and both at
    once the way the server moves them (SDMA H2D + the copy kernel writing
    pinned host memory: two SDMA copies share one engine's ~54 GB/s, this mix
    runs full duplex, tools/pcie_probe.py); median over ``reps``."""
    import torch
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d2 = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def timed(fn):
        ts = []
        for i in range(reps + 2):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            if i >= 2:
                ts.append(time.perf_counter() - t0)
        return statistics.median(ts)

    def h2d():
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)

    def d2h_kernel():
        red.copy(h2, d2, nbytes, stream=s2)

    def both():
        h2d()
        d2h_kernel() if red is not None else d2h()

    def both_sdma():
        h2d()
        d2h()
    t_h2d, t_d2h, t_both, t_bs = timed(h2d), timed(d2h), timed(both), timed(both_sdma)
    return {"workload": f"pinned host <-> HBM copies of {nbytes >> 20} MiB on side streams "
                        f"(median of {reps}); bidir = SDMA H2D + copy-kernel D2H at once",
            "h2d_GBps": round(nbytes / t_h2d / 1e9, 2),
            "d2h_GBps": round(nbytes / t_d2h / 1e9, 2),
            "bidir_GBps": round(2 * nbytes / t_both / 1e9, 2),
            "bidir_sdma_only_GBps": round(2 * nbytes / t_bs / 1e9, 2)}


def server_group_leg(dev, world: int, rank: int, n_workers: int = 2,
                     bucket_bytes: int = 64 << 20, rounds: int = 10, lanes: int = 4,
                     link: dict | None = None) -> dict:
    """BASELINE config 1's server rounds from host memory on every GPU of the
    node: each rank's process is one PS server (a byteps_server_group_* group
    with ONE instance, on this rank's GPU, whole keys by the reference's djb2
    hash — server.cc:339-400 runs one server per process) serving one
    cfg1-shaped bucket: 2 workers' 64 MiB fp32 gradients as the 17 BytePS
    partitions of 4,096,000 B (operations.cc:99-136, declared key = rank), in
    pinned host memory as ps-lite's receive buffers would be.  A round, in
    BytePS's worker loop shape (core_loops.cc:492-564: every partition's ZPush
    is issued at once, and each partition's ZPull waits on the server for its
    round): each worker's push thread hands its 17 partitions to ONE
    byteps_server_group_push_many call (all 17 H2D copies in flight on the
    lanes' copy streams, each round folded as it completes), while its pull
    thread pulls the partitions in order, each answered as soon as that
    partition's round is folded — so D2H runs beside the H2D of later
    partitions (PCIe is full duplex).  Two pull forms, timed separately: the
    zero-copy pull response (``byteps_server_group_pull_host_view`` —
    server.cc:42-70 answers a pull with an SArray over its own buffer, which
    ps-lite then sends: ONE D2H per partition and round into the pinned
    mirror, shared by both workers; the headline form) and copying pulls into
    each worker's own pinned buffer (``byteps_server_group_pull``: one D2H per
    worker).  The threads persist across rounds (a barrier starts each).  Weak
    scaling: at N GPUs, N buckets over N PCIe links.  Node rate = all ranks'
    pushed bytes / the slowest rank's median round; ``frac_of_link`` = the
    link's shortest time for the round's H2D and D2H bytes (link_bound_s, from
    the same run's measured rates ``link``) over the round.  PCIe-inclusive; compare with ``cpu_baseline`` (the
    reference's host-core round).  Exactness: every worker's pull equals
    torch's sum of the two pushes (fp32, two operands: the left fold in either
    arrival order)."""
    import threading
    import torch
    from prophet_amd.buckets import partition_tensor
    from prophet_amd.dtypes import DType
    from prophet_amd.server import PSServerGroup
    multi = world > 1
    import torch.distributed as dist
    n = bucket_bytes // 4
    parts = [(p.key, p.offset, p.len) for p in partition_tensor(0, bucket_bytes,
                                                                 declared_key=rank)]
    keys = [k for k, _, _ in parts]
    gen = torch.Generator(device="cpu")
    host = []
    for w in range(n_workers):
        gen.manual_seed(12000 + 16 * rank + w)
        host.append(torch.randn(n, generator=gen).pin_memory())
    outs = [torch.zeros(bucket_bytes, dtype=torch.uint8).pin_memory() for _ in range(n_workers)]
    grp = PSServerGroup(n_workers, devices=[dev.index], engine_lanes=lanes, split="hash")
    srcs = [[host[w].view(torch.uint8)[o:o + ln] for _, o, ln in parts] for w in range(n_workers)]
    dsts = [[outs[w][o:o + ln] for _, o, ln in parts] for w in range(n_workers)]
    errors = []
    views = {}
    # persistent threads: a push thread and a pull thread per worker; the
    # main thread joins each round through two barriers (start, end)
    mode = {"pull": None, "quit": False}
    start = threading.Barrier(2 * n_workers + 1)
    end = threading.Barrier(2 * n_workers + 1)

    def pusher(w):
        while True:
            start.wait()
            if mode["quit"]:
                return
            try:
                grp.push_many(keys, w, srcs[w], DType.FLOAT32)
            except Exception as e:  # noqa: BLE001 — reported below
                errors.append(repr(e))
            end.wait()

    def puller(w):
        while True:
            start.wait()
            if mode["quit"]:
                return
            try:
                if mode["pull"] == "view":
                    for i, k in enumerate(keys):
                        views[(w, i)] = grp.pull_view(k)
                elif mode["pull"] == "copy":
                    for i, k in enumerate(keys):
                        grp.pull(k, dsts[w][i])
            except Exception as e:  # noqa: BLE001 — reported below
                errors.append(repr(e))
            end.wait()
    ts = [threading.Thread(target=f, args=(w,), daemon=True)
          for w in range(n_workers) for f in (pusher, puller)]
    for th in ts:
        th.start()

    def rnd(pull):
        mode["pull"] = pull
        start.wait(timeout=120)
        end.wait(timeout=120)
        if errors:
            raise RuntimeError(errors[0])
    want = host[0].clone()
    for h in host[1:]:
        want += h
    wantb = want.view(torch.uint8)

    def timed(pull):
        rnd(pull)
        times = []
        for _ in range(rounds):
            if multi:
                dist.barrier()
            t0 = time.perf_counter()
            rnd(pull)
            times.append(time.perf_counter() - t0)
        return _max_over_ranks(dist, dev, [statistics.median(times)])[0]

    try:
        rnd(None)            # init round: pushes only
        # copying pulls first: once a key has been viewed, the server mirrors
        # every later round of it (one D2H more per round)
        tc = timed("copy")   # copying pulls into every worker's own buffer
        ok = all(bool(torch.equal(o, wantb)) for o in outs)
        t = timed("view")    # zero-copy pull responses (the last round's views stay valid)
        ok = ok and all(bool(torch.equal(torch.frombuffer(views[(w, i)], dtype=torch.uint8),
                                         wantb[o:o + ln]))
                        for w in range(n_workers) for i, (_, o, ln) in enumerate(parts))
    finally:
        mode["quit"] = True
        try:
            start.wait(timeout=30)
        except threading.BrokenBarrierError:
            pass
        for th in ts:
            th.join(timeout=30)
    ok = _all_true(dist, dev, ok)
    grp.close()
    total = world * n_workers * bucket_bytes
    out = {"workload": (f"config 1 per GPU: {n_workers} workers x {bucket_bytes >> 20} MiB fp32 "
                        f"as {len(parts)} partitions in pinned host memory, one PS server "
                        f"(byteps_server_group_*, one instance, djb2 hash) per GPU; per worker "
                        f"one push_many of its partitions (all in flight) and a pull thread, "
                        f"{world} GPU(s) / PCIe links"),
           "pull": "host_view (zero-copy pull response, server.cc:42-70)",
           "node_GiBps": round(total / t / GIB, 2),
           "per_gpu_GiBps": round(n_workers * bucket_bytes / t / GIB, 2),
           "round_ms": round(t * 1e3, 3),
           "copying_pulls": {"node_GiBps": round(total / tc / GIB, 2),
                             "per_gpu_GiBps": round(n_workers * bucket_bytes / tc / GIB, 2),
                             "round_ms": round(tc * 1e3, 3)},
           "rounds": rounds, "lanes": lanes,
           "pcie_inclusive": True, "exact_vs_torch_sum": ok}
    # the link: every worker's push in; one D2H per partition (views: the
    # shared mirror) or one per worker (copying pulls) out
    out.update(link_fracs(n_workers * bucket_bytes, bucket_bytes, t, link))
    out["copying_pulls"].update(link_fracs(n_workers * bucket_bytes, n_workers * bucket_bytes,
                                           tc, link))
    return out


def server_cfg3_leg(dev, rounds: int = 20, lanes: int = 4, N: int = 8) -> dict:
    """BASELINE config 3's keys through the GPU-resident PS server on this GPU,
    in the reference server's shape (server.cc:147-308 behind ps-lite's ONE
    receive thread, server.cc:149): 8 workers' ResNet-50 fp16 gradients as the
    165 BytePS partitions (keys in Prophet block order) sit in the receive
    slots (an RDMA transport's writes into HBM); per round the receive thread
    signals every arrival (byteps_server_push_ready) and answers every pull
    with a zero-copy device view of the store
    (byteps_server_pull_device_view); the round ends with the last view, i.e.
    every key folded.  The timed loop is native (tools/cfg3srv_drv.cpp through
    ctypes: no Python per call).  Two ways: ``launch`` — the default path,
    lane issuers batching each completed round into fold launches; and
    ``device_releases`` — BPSR_SERVER_RELEASE=device, one keyed consumer
    launch per epoch releasing each key on the device when its last push
    arrives.  Median round over ``rounds``; ``frac_of_roofline`` =
    (N + 1) x 51,114,064 B / round / 8 TB/s.  Exactness: one further round
    pulls every key into every worker's buffer, checked bit for bit against
    torch's own fp16 left fold (fp32 add, RNE per add) in the arrival order
    the server recorded for each key."""
    import ctypes
    import torch
    from prophet_amd.buckets import partition_all, prophet_blocks, resnet50_param_sizes
    drv_path = os.path.join(ROOT, "tools", "libcfg3srv.so")
    if not os.path.exists(drv_path):
        raise RuntimeError(f"{drv_path} not built (make -C tools)")
    drv = ctypes.CDLL(drv_path)
    _vp, _sz, _int = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    drv.cfg3srv_run.argtypes = [_int, ctypes.POINTER(_sz), ctypes.POINTER(_sz), _int,
                                ctypes.POINTER(_vp), ctypes.POINTER(_vp), _int, _int,
                                ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_int)]
    sizes = [n * 2 for n in resnet50_param_sizes()]
    parts = partition_all(sizes)
    toff = [0]
    for n in sizes:
        toff.append(toff[-1] + n)
    total = toff[-1]
    table = [p for blk in prophet_blocks(len(sizes)) for p in parts if p.tensor in set(blk)]
    np_ = len(table)
    offs = (_sz * np_)(*[toff[p.tensor] + p.offset for p in table])
    lens = (_sz * np_)(*[p.len for p in table])
    gen = torch.Generator(device=dev)
    grads = []
    for k in range(N):
        gen.manual_seed(5000 + k)
        grads.append(torch.randn(total // 2, device=dev, generator=gen).half())
    outs = [torch.empty_like(g) for g in grads]
    torch.cuda.synchronize()
    alg = (N + 1) * total
    res_all = {}
    for name, rel in (("launch", None), ("device_releases", "device")):
        old = os.environ.pop("BPSR_SERVER_RELEASE", None)
        if rel:
            os.environ["BPSR_SERVER_RELEASE"] = rel
        res = (ctypes.c_double * 8)()
        orders = (_int * (np_ * N))()
        for o in outs:
            o.fill_(float("nan"))
        torch.cuda.synchronize()
        try:
            rc = drv.cfg3srv_run(np_, offs, lens, N, (_vp * N)(*[g.data_ptr() for g in grads]),
                                 (_vp * N)(*[o.data_ptr() for o in outs]), rounds, lanes, res,
                                 orders)
        finally:
            os.environ.pop("BPSR_SERVER_RELEASE", None)
            if old is not None:
                os.environ["BPSR_SERVER_RELEASE"] = old
        if rc:
            raise RuntimeError(f"cfg3srv_run ({name}) returned {rc}")
        ok = True
        for i, p in enumerate(table):
            lo = (toff[p.tensor] + p.offset) // 2
            n = p.len // 2
            order = [orders[i * N + w] for w in range(N)]
            ok = ok and sorted(order) == list(range(N))
            acc = grads[order[0]][lo:lo + n].clone()
            for w in order[1:]:
                acc.add_(grads[w][lo:lo + n])
            want = acc.view(torch.int16)
            ok = ok and all(bool(torch.equal(o[lo:lo + n].view(torch.int16), want)) for o in outs)
        ms = res[0]
        res_all[name] = {"round_ms": round(ms, 4), "min_ms": round(res[1], 4),
                         "max_ms": round(res[7], 4), "push_phase_ms": round(res[2], 4),
                         "frac_of_roofline": round(alg / (ms * 1e-3) / (HBM_PEAK_GBPS * 1e9), 4),
                         "fold_launches_per_round": round(res[3], 1),
                         "consumer_launches_per_round": round(res[4], 2),
                         "key_releases_per_round": round(res[5], 1),
                         "exact_vs_torch_fold_in_recorded_order": ok}
    return {"workload": (f"config 3's keys through the PS server: {N} workers' ResNet-50 fp16 "
                         f"({total} B each) as {np_} BytePS partitions in the receive slots; ONE "
                         f"receive thread per round: push_ready for every (key, worker), then a "
                         f"device view per pull (tools/cfg3srv_drv.cpp, native)"),
            "alg_bytes_per_round": alg, "rounds": rounds, "lanes": lanes, **res_all}


# --------------------------------------------------------------------------
# config 3: ResNet-50 fp16 Prophet blocks through the block queue


def cfg3_leg(dev, red, iters: int = 200, reps: int = 5, sets: int = 3, N: int = 8) -> dict:
    """BASELINE config 3 on this GPU: 8 workers' ResNet-50 fp16 gradients
    (161 tensors, 51,114,064 B) cut into the 165 BytePS partitions
    (operations.cc:99-136) and grouped into the 12 Prophet blocks
    (scheduled_queue.h:78-79, last checkpoint extended to 160), folded by the
    block queue: ONE consumer launch per iteration that starts each block once
    it is released (byteps_reduce_blockq_*).  ``live``: the
    product push path — the native PUSH loop (byteps_prophet_loop_*, inline)
    launches the consumer, the 165 partitions are pushed in backward order as
    one batch (they have all landed), Prophet's scheduler (scheduled_queue.cc
    getTask) releases them group by group and the loop releases the blocks
    those groups complete with stream-ordered release kernels on a second
    stream, the groups ready together as one kernel (``release_kernels_per_iter``);
    ``live_per_block``: the launch, then one release kernel per block from
    the second stream (the round-2 ``live``: every block as its own release
    group); ``pre_released``: every block released before the launch;
    ``live_host_releases``: the launch, then the 12 releases from the host
    (byteps_reduce_blockq_release_host — the pushes are resident, as after an
    RDMA write into HBM), no stream work per release.  Device time per iteration from HIP events on
    the consumer's stream (median of ``reps`` runs of ``iters`` back-to-back
    iterations over ``sets`` rotated input sets), host time of the issuing
    loop, exactness against torch's own left fold."""
    import torch
    from prophet_amd.buckets import partition_all, prophet_blocks, resnet50_param_sizes
    from prophet_amd.dtypes import DType
    from prophet_amd.prophet import ProphetPushQueue, PushLoop, PushTask, model_checkpoints
    sizes = [n * 2 for n in resnet50_param_sizes()]
    parts = partition_all(sizes)
    toff = [0]
    for n in sizes:
        toff.append(toff[-1] + n)
    total = toff[-1]
    by_block = []
    for blk in prophet_blocks(len(sizes)):
        tset = set(blk)
        by_block.append([p for p in parts if p.tensor in tset])
    # the PUSH loop's table: partition handle = position in block order
    table = [p for bp in by_block for p in bp]
    block_of = [b for b, bp in enumerate(by_block) for _ in bp]
    nparts = {}
    for p in parts:
        nparts[p.tensor] = nparts.get(p.tensor, 0) + 1
    arrivals = sorted(range(len(table)), key=lambda i: (-table[i].tensor, table[i].part))
    from prophet_amd.arena import BucketArena
    gen = torch.Generator(device=dev)
    data, queues, hqueues = [], [], []
    for i in range(sets):
        # the 8 workers' receive slots and the output: one skewed arena, the
        # headline's HBM layout (prophet_amd/arena.py; separate allocations
        # fold 1-1.5 % slower here, profiles/r05s23_overlap_skew.jsonl)
        *w, out = BucketArena(N + 1, total, dev).slots()
        for k in range(N):
            gen.manual_seed(3000 + 10 * i + k)
            w[k].copy_(torch.randn(total // 2, device=dev, generator=gen).half().view(torch.uint8))
        data.append((w, out))
        q = red.make_blockq([[(out[toff[p.tensor] + p.offset:][:p.len],
                               [x[toff[p.tensor] + p.offset:][:p.len] for x in w], p.len)
                              for p in bp] for bp in by_block], DType.FLOAT16)
        q.config(wg_per_cu=0, timeout_s=1.0)
        queues.append(q)
        hq = red.make_blockq([[(out[toff[p.tensor] + p.offset:][:p.len],
                                [x[toff[p.tensor] + p.offset:][:p.len] for x in w], p.len)
                               for p in bp] for bp in by_block], DType.FLOAT16)
        hq.config(wg_per_cu=0, timeout_s=1.0)
        hq.host_releases(True)
        hqueues.append(hq)
    # the library's consumer stream: a hardware queue of its own, so a release
    # never waits behind the spinning consumer (include/bpsr/reduce.h); the
    # stream releases on the library's release stream, a queue on a compute
    # pipe no consumer queue uses (DESIGN.md §4.4 "pipes": a torch stream
    # that lands on a running consumer's pipe runs its release kernels ~2x
    # slower).  BPSR_BENCH_REL_STREAM=torch: a torch stream (measurement only)
    live_s = queues[0].stream()
    if os.environ.get("BPSR_BENCH_REL_STREAM") == "torch":
        rel_s = torch.cuda.Stream(device=dev)
    else:
        rel_s = queues[0].release_stream()
    overlap_on = [False]
    nb = len(by_block)
    # one scheduler + inline PUSH loop per input set (a loop drives one queue);
    # Z_BATCH_SIZE 64, Z_NET_B 10000, Z_CREDIT 16 MiB, the reference's block
    # budgets (as tools/cfg3_native.cpp and tests/test_pushloop_gpu.py)
    loops, batches = [], []
    for q in queues:
        pq = ProphetPushQueue(batch_size=64, net_b=10000, credit=16 << 20,
                              checkpoints=model_checkpoints(len(sizes)))
        lp = PushLoop(pq, q, block_of, release_stream=rel_s, inline=True)
        loops.append(lp)
        batches.append(lp.make_batch(
            [PushTask(table[i].tensor, table[i].part, table[i].len, nparts[table[i].tensor],
                      (table[i].tensor << 16) + table[i].part) for i in arrivals], arrivals))
    import gc
    gc.collect()      # inline loop: no GC-triggered hipFree inside an iteration

    def live(i):      # the PUSH loop: launch, one batch of landed pushes, releases
        lp = loops[i % sets]
        lp.begin(live_s)
        lp.push_many(batches[i % sets])
        lp.end(timeout_s=5.0)

    def live_per_block(i):
        q = queues[i % sets]
        q.launch(live_s)
        for b in range(nb):
            q.release(b, rel_s)

    def pre_released(i):
        # released before the launch: on the launch stream itself without
        # overlap; with overlap on the release stream (a release queued on a
        # consumer queue waits there for the consumer before it)
        q = queues[i % sets]
        q.release(-1, rel_s if overlap_on[0] else live_s)
        q.launch(live_s)

    def live_host(i):   # the pushes are resident: releases straight from the host
        q = hqueues[i % sets]
        q.launch(live_s)
        for b in range(nb):
            q.release_host(b)

    # probe: one live iteration must complete before anything is timed (a
    # profiler that serialises dispatches would strand the consumer; it then
    # gives up after its 1-s timeout and status() raises, ending this leg)
    torch.cuda.synchronize()        # the inputs (torch's stream) before any consumer
    live(0)
    torch.cuda.synchronize()
    queues[0].status(live_s)
    alg = (N + 1) * total
    res = {"workload": (f"config 3: {N}-way fp16 ResNet-50 ({total} B per worker), "
                        f"{len(parts)} partitions in {nb} Prophet blocks, block queue "
                        "(one consumer launch per iteration); live = the native PUSH loop "
                        "(Prophet scheduler, stream-ordered release kernels, the release "
                        "groups ready together as one kernel); live_per_block = one "
                        "release kernel per block; receive slots in one skewed HBM arena"),
           "alg_bytes_per_iter": alg, "iters": iters, "reps": reps,
           "release_stream": ("torch" if os.environ.get("BPSR_BENCH_REL_STREAM") == "torch"
                              else "library (byteps_reduce_blockq_release_stream)")}
    res["overlap"] = ("consecutive launches overlap (byteps_reduce_blockq_overlap: the two "
                      "consumer queues alternate, a launch dispatched once every workgroup of "
                      "the previous one has started); *_no_overlap: one stream-ordered queue")
    rel_kernels = {"live_per_block": nb, "pre_released": 1, "live_host_releases": 0}

    def set_overlap(on):
        overlap_on[0] = on
        for q in queues + hqueues:
            q.overlap(on)

    variants = (("live", live, True), ("live_per_block", live_per_block, True),
                ("pre_released", pre_released, True), ("live_host_releases", live_host, True),
                ("live_no_overlap", live, False), ("pre_released_no_overlap", pre_released, False))
    for name, fn, ov in variants:
        set_overlap(ov)
        for i in range(30):
            fn(i)
        torch.cuda.synchronize()
        c0 = sum(lp.release_calls() for lp in loops)
        ts, hs = [], []
        for _ in range(reps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(live_s)
            t0 = time.perf_counter()
            for i in range(iters):
                fn(i)
            hs.append((time.perf_counter() - t0) / iters * 1e6)
            queues[0].join(live_s)      # both consumer queues' last launches
            e1.record(live_s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / iters)
        ms = statistics.median(ts)
        res[name] = {"ms_per_iter": round(ms, 5), "min_ms": round(min(ts), 5),
                     "spread": round((max(ts) - min(ts)) / ms, 4),
                     "frac_of_roofline": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "host_us_per_iter": round(statistics.median(hs), 1)}
        base = name.replace("_no_overlap", "")
        if base == "live":
            rel_kernels[name] = round((sum(lp.release_calls() for lp in loops) - c0)
                                      / (reps * iters), 2)
        res[name]["release_kernels_per_iter"] = rel_kernels.get(name, rel_kernels[base])
    set_overlap(True)
    for q in queues + hqueues:
        q.status(live_s)
    ok = True
    for fn in (live, live_per_block, live_host):
        for i, (w, out) in enumerate(data):
            out.zero_()
            torch.cuda.synchronize()
            fn(i)
            torch.cuda.synchronize()
            ref = w[0].view(torch.float16).clone()
            for x in w[1:]:
                ref.add_(x.view(torch.float16))
            ok = ok and bool(torch.equal(ref.view(torch.uint8), out))
    res["exact_vs_torch_fold"] = ok
    res["hsa_queue_ids"] = queues[0].queue_ids()   # consumer queues 0-2, release queue
    for lp in loops:
        lp.close()
    for q in queues + hqueues:
        q.close()
    return res


# --------------------------------------------------------------------------
# provenance of roofline.traffic


def kernel_build_id(root: str = ROOT) -> str:
    """Id of what decides the headline kernel's code and launch geometry."""
    h = hashlib.sha256()
    sig = os.path.join(root, KERNEL_SIG)
    if os.path.exists(sig):
        with open(sig, "rb") as f:
            h.update(b"isa\0" + f.read().strip())
    else:
        for rel in KERNEL_SOURCES:
            with open(os.path.join(root, rel), "rb") as f:
                h.update(rel.encode() + b"\0" + f.read())
    for rel, a, b in KERNEL_SOURCE_SPANS:
        with open(os.path.join(root, rel)) as f:
            text = f.read()
        i = text.index(a)
        h.update(rel.encode() + b"\0" + text[i:text.index(b, i)].encode())
    return h.hexdigest()[:16]


def pmc_traffic(workload: str):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    PMC summary (tools/pmc_traffic.py -> profiles/pmc_traffic.json) — quoted
    only when it was collected for this workload AND for the kernel sources
    now in the tree.  Returns (bytes or None, source dict)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, {"status": "no committed PMC record"}
    src = {"file": "profiles/pmc_traffic.json", "session": d.get("session"),
           "kernel_build": d.get("kernel_build")}
    if d.get("workload") != workload:
        src["status"] = "recorded for another workload: not quoted"
        return None, src
    try:
        now = kernel_build_id()
    except OSError:
        now = None
    if d.get("kernel_build") != now:
        src["status"] = f"kernel build changed since the PMC pass (now {now}): not quoted"
        return None, src
    src["status"] = "same workload, same kernel build (ISA signature + launch rules)"
    return d.get("hbm_bytes_per_launch"), src


# --------------------------------------------------------------------------


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    # RCCL and cross-process device memory on this ROCm stack need dmabuf IPC
    # (the legacy IPC path fails with `hipIpcGetMemHandle: invalid argument`):
    # keep it on for every rank, whoever launched us, before any HIP call.
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # Parent: start one process per GPU before anything touches the GPU.
        sys.exit(launch_ranks(args.gpus, argv))

    # stdout carries exactly one line, the JSON result: whatever the libraries
    # write to fd 1 (gloo's connection notes, runtime chatter) goes to stderr
    sys.stdout.flush()
    line_fd = os.dup(1)
    os.dup2(2, 1)

    def emit(obj) -> None:
        os.write(line_fd, (json.dumps(obj) + "\n").encode())

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}; using WORLD_SIZE",
              file=sys.stderr)
    cuda = args.device == "cuda"
    rehearse = cuda and args.rehearse_one_gpu and world > 1
    # Exchange legs (scatter, local reduce) rehearsed on one GPU move CUDA
    # tensors through gloo's host staging, far slower than RCCL over xGMI:
    # there they run on a 4,000,037-element vector unless --scaling-elems
    # says otherwise (the legs' code and checks are the point, not the rate).
    xchg_elems = args.scaling_elems or (4_000_037 if rehearse else None)
    gpu = 0 if rehearse else local_rank
    if cuda:
        # Bind this rank's GPU before the process group exists, so RCCL's
        # communicator (barrier, the max-over-ranks all_reduce) uses it.
        torch.cuda.set_device(gpu)
        dev = torch.device("cuda", gpu)
    else:
        dev = torch.device("cpu")
    if world > 1:
        if cuda and not rehearse:
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        world = dist.get_world_size()

    from prophet_amd.arena import BucketArena
    from prophet_amd.dtypes import DType

    dtype_id = DType(DTYPES[args.dtype][0])
    tdt = getattr(torch, DTYPES[args.dtype][1])
    es = torch.empty(0, dtype=tdt).element_size()
    mode = 1 if args.mode == "accum" else 0
    N = args.workers
    B = int(args.bucket_mib * (1 << 20)) // es * es
    n_elems = B // es
    if cuda:
        from prophet_amd.reducer import GpuReducer
        red = GpuReducer(device=gpu)
        stream = torch.cuda.current_stream(dev)

        def fold_bytes(dst, srcs):
            red.sum_n(dst, srcs, B, dtype_id, mode=mode, stream=stream)

        def fold_f32(dst, srcs):
            red.sum_n(dst, srcs, dst.numel() * 4, DType.FLOAT32, stream=stream)
    else:
        red = None
        if mode:
            raise SystemExit("--device cpu: reference mode only")

        def fold_bytes(dst, srcs):
            _torch_fold(dst.view(tdt), [s.view(tdt) for s in srcs])
        fold_f32 = _torch_fold

    # Input sets: the server's per-worker receive slots for this GPU's bucket,
    # carved from one HBM arena (prophet_amd/arena.py: skewed slots avoid the
    # channel aliasing of power-of-two-spaced buffers), plus the output slot.
    # Seeded N(0,1) gradients per (rank, set, worker), generated on device.
    torch.manual_seed(1000 + rank)
    sets = []
    for s in range(args.sets):
        if args.layout == "arena":
            slots = (BucketArena(N + 1, B, dev) if args.skew < 0 else
                     BucketArena(N + 1, B, dev, skew=args.skew)).slots()
        else:
            slots = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(N + 1)]
        for t in slots[:N]:
            if tdt.is_floating_point:
                t.view(tdt).copy_(torch.randn(n_elems, device=dev))
            else:
                t.copy_(torch.randint(0, 256, (B,), dtype=torch.uint8, device=dev))
        sets.append((slots[N], slots[:N]))
    clock = _Clock(dev)
    clock.sync()

    def step(i):
        dst, srcs = sets[i % len(sets)]
        fold_bytes(dst, srcs)

    for i in range(args.warmup):
        step(i)
    clock.sync()
    if world > 1:
        dist.barrier()
    clock.sync()
    t0 = time.perf_counter()
    kern_ms = clock.time(step, args.steps)   # avg duration per launch, launch stream
    clock.sync()
    if world > 1:
        dist.barrier()
    clock.sync()
    wall = time.perf_counter() - t0
    t_step = wall / args.steps
    t_step, kern_ms = _max_over_ranks(dist, dev, [t_step, kern_ms])
    # Spread of the per-launch time (median / min / max over blocks of
    # back-to-back launches), a separate pass after the timed region; it ends
    # on the same input set as the timed steps did.
    n_blk, per_blk = 5, max(1, min(args.steps // 5, 10))
    pl = sorted(clock.blocks(step, n_blk, per_blk,
                             first=args.steps + args.warmup - n_blk * per_blk))
    pl_med, pl_min, pl_max = _max_over_ranks(
        dist, dev, [statistics.median(pl), pl[0], pl[-1]])

    # Correctness spot check of the last set against torch's own left fold.
    dst, srcs = sets[(args.steps + args.warmup - 1) % len(sets)]
    chk = srcs[0].view(tdt)[: 1 << 20].clone()
    for s in srcs[1:]:
        chk.add_(s.view(tdt)[: 1 << 20])
    ok = bool(torch.equal(chk.view(torch.uint8), dst[: chk.numel() * es])) if mode == 0 else None
    ok = _all_true(dist, dev, ok) if ok is not None else None
    del sets

    devices = [f"{local_rank}"]
    if cuda:
        devices = [f"{gpu}:{torch.cuda.get_device_name(dev)}"]
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, devices[0])
        devices = gathered

    alg_bytes = (N + 1) * B
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    workload = f"{N}-way {args.dtype} left-fold sum of one {B / (1 << 20):.0f} MiB bucket per GPU"
    if mode:
        workload += " (fp32-accumulate mode)"
    traffic, traffic_src = pmc_traffic(workload)
    tuning = None
    if red is not None:
        tv, tnt, tgrid, tocc = red.get_tuning()
        tuning = {"vpt": tv, "nt": tnt, "max_grid": tgrid, "wg_per_cu": tocc}
    line = {
        "metric": METRIC,
        "value": round(world * N * B / t_step / GIB, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        # the headline's weak scaling has no exchange in its
        # timed region; what tests the sharded claim is named beside it
        "scaling_note": ("each rank folds its own bucket (the key space sharded over the "
                         "GPUs, no collective in the timed steps), so weak-scaling "
                         "efficiency tests the node's HBM/host headroom, not communication; "
                         "scaling_cfg4 (strong scaling of one set over the GPUs), its "
                         "RCCL scatter leg and local_reduce carry the exchanges"),
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (torch.randn on device, seeded per rank), resident in HBM, "
                f"{args.sets} rotated input sets, layout={args.layout}"
                + (f", skew={args.skew}" if args.skew >= 0 else ""),
        "config": {"workload": workload, "n_workers": N, "bucket_bytes": B,
                   "parallelism": f"key-space shard x{world}", "kernel": "byteps_reduce_sum_n",
                   "tuning": tuning, "devices": devices},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "alg_bytes_per_launch": alg_bytes, "kernel_ms": round(kern_ms, 5),
                     # per-launch average of each of n_blk blocks of per_blk
                     # back-to-back launches, a separate pass (max over ranks)
                     "kernel_ms_blocks": {"median": round(pl_med, 5), "min": round(pl_min, 5),
                                          "max": round(pl_max, 5), "blocks": n_blk,
                                          "launches_per_block": per_blk},
                     # also the read stream alone (N * B of the
                     # (N + 1) * B), against the same peak
                     "read_only_GBps": round(N * B / (kern_ms * 1e-3) / 1e9, 1),
                     "read_only_frac": round(N * B / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)},
        "check_vs_torch_fold": ok,
    }
    if not cuda:
        line["device"] = "cpu plumbing self-test (torch CPU add, gloo): NOT a measurement"
    if rehearse:
        line["device"] = (f"rehearsal: {world} ranks sharing cuda:0 over gloo (HIP fold, "
                          "no RCCL: the scatter and local-reduce legs move CUDA tensors "
                          f"through gloo, {xchg_elems} elements): NOT a measurement")

    # N > 1 on GPUs: the exchange legs go through the shard C ABI over RCCL
    # (byteps_shard_*), the path a core_loops.cc caller binds; gloo
    # rehearsals and the CPU self-test keep torch.distributed P2P
    comm = None
    if world == 1:
        pass
    elif not uses_shard_abi(world, cuda, rehearse):
        line["rccl"] = {"transport": "gloo, no RCCL", "world": world}
    elif args.no_scatter:
        line["rccl"] = {"transport": "not used (--no-scatter)", "world": world}

    def make_comm():
        """N > 1 on GPUs (under the watchdog): the shard communicator, then
        every rank's view of it; a communicator that is not N ranks on N
        distinct GPUs fails the run (RCCL_EXIT on every rank).  A
        communicator that cannot be made, or a view that cannot be gathered,
        is recorded and the run goes on (nothing was shown to be wrong)."""
        nonlocal comm
        if os.environ.get("BPSR_BENCH_TEST_RCCL") == "shared_device":
            # test hook (CPU self-test): every rank claims GPU 0 of a world-N
            # communicator, as a mis-bound launch would
            line["rccl"] = rccl_object(dev, None, world, rank, view={
                "rank": rank, "comm_world": world, "comm_rank": rank, "comm_device": 0,
                "device": 0, "pci_bus_id": "0000:05:00", "rccl_version": 0, "device_count": 1})
            return not line["rccl"]["problems"]
        try:
            comm, how = shard_comm(dev)
            line["shard_comm"] = how
        except Exception as e:  # report, never hide
            # no communicator to check: the exchange legs fall back to torch
            # P2P (their `transport` says so) and the line still stands
            line["shard_comm"] = {"error": repr(e)}
            line["rccl"] = {"transport": "rccl", "world": world, "error": repr(e)}
            comm = None
            return True
        try:
            line["rccl"] = rccl_object(dev, comm, world, rank)
        except Exception as e:  # report, never hide (a check that could not run)
            line["rccl"] = {"transport": "rccl", "world": world, "error": repr(e)}
            return True
        return not line["rccl"]["problems"]

    def extra_legs(state=None):
        def leg(name):
            if state is not None:
                state["leg"] = name
        leg("scaling_cfg4")
        if not args.no_scaling:
            try:
                line["scaling_cfg4"] = scaling_leg(dev, world, rank, N, fold_f32,
                                                   n_elems=args.scaling_elems or None)
            except Exception as e:  # report, never hide
                line["scaling_cfg4"] = {"error": repr(e)}
            if world > 1 and not args.no_scatter:
                leg("scatter")
                try:
                    line["scaling_cfg4"]["scatter"] = scatter_leg(
                        dev, world, rank, N, n_elems=xchg_elems,
                        fold=None if cuda else _torch_fold, comm=comm)
                except Exception as e:  # report, never hide
                    line["scaling_cfg4"]["scatter"] = {"error": repr(e)}
        if world > 1 and not args.no_scatter:
            leg("local_reduce")
            try:
                line["local_reduce"] = local_reduce_leg(
                    dev, world, rank, n_elems=xchg_elems,
                    fold=None if cuda else _torch_fold, comm=comm)
            except Exception as e:  # report, never hide
                line["local_reduce"] = {"error": repr(e)}
        # Config 3 before the host-resident server: the order that ran the
        # server at 0.65 of its link and config 3's per-block releases 30x
        # slower until round 6 placed the library's queues one per compute pipe
        # (DESIGN.md §4.4 "pipes"); no leg order is needed any more.
        if world == 1 and cuda and not args.no_cfg3:
            leg("cfg3_blockq")
            try:
                line["cfg3_blockq"] = cfg3_leg(dev, red)
            except Exception as e:  # report, never hide
                line["cfg3_blockq"] = {"error": repr(e)}
        link = None
        if cuda and not (args.no_server and args.no_e2e):
            leg("pcie")
            try:
                link = line["pcie"] = pcie_leg(dev, red)
            except Exception as e:  # report, never hide
                line["pcie"] = {"error": repr(e)}
        elif not cuda:
            line["pcie"] = {"skipped": "the PCIe probe needs a GPU (--device cpu)"}
        leg("server_cfg1")
        if cuda and not args.no_server:
            try:
                line["server_cfg1"] = server_group_leg(dev, world, rank, link=link)
            except Exception as e:  # report, never hide
                line["server_cfg1"] = {"error": repr(e)}
        elif not args.no_server:
            line["server_cfg1"] = {"skipped": "the PS server needs a GPU (--device cpu)"}
        if cuda and not args.no_e2e:
            leg("e2e_cfg5")
            try:
                line["e2e_cfg5"] = e2e_leg(dev, world, rank,
                                           bucket_bytes=args.e2e_bucket_mib << 20, link=link)
            except Exception as e:  # report, never hide
                line["e2e_cfg5"] = {"error": repr(e)}

    if world == 1:
        extra_legs(None)
        if cuda and args.dtype == "f32" and mode == 0 and not args.no_fp16:
            try:
                line["fp16"] = fp16_leg(dev, red, N, B, args.steps)
            except Exception as e:  # report, never hide
                line["fp16"] = {"error": repr(e)}
        if cuda and not args.no_cfg3 and not args.no_server:
            try:
                line["server_cfg3"] = server_cfg3_leg(dev)
            except Exception as e:  # report, never hide
                line["server_cfg3"] = {"error": repr(e)}
        if rank == 0 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(N, int(dtype_id), args.cpu_sample_mib)
            except Exception as e:  # report, never hide
                line["cpu_baseline"] = {"error": repr(e)}
        emit(line)
        return
    # N > 1: the headline line is complete; the config-4 legs run after it
    # under a watchdog.  A stuck or failing collective then costs only those
    # fields, never the line — but the run FAILS: the line carries "error" and
    # every rank exits non-zero, so a hang on first hardware contact cannot
    # pass for success (launch_ranks / torch.distributed.run relay the status).
    import threading
    lock = threading.Lock()
    state = {"printed": False, "leg": "start"}
    limit_s = float(os.environ.get("BPSR_BENCH_WATCHDOG_S", "240"))

    def emit_and_maybe_exit(exit_code):
        with lock:
            if rank == 0 and not state["printed"]:
                emit(line)
                state["printed"] = True
        if exit_code is not None:
            sys.stderr.flush()
            os._exit(exit_code)

    def on_timeout():
        msg = f"watchdog: leg {state['leg']!r} still running after {limit_s:.0f} s"
        line["error"] = msg
        line.setdefault("scaling_cfg4", {}).setdefault("error", msg)
        print(f"bench rank {rank}: {msg}", file=sys.stderr)
        emit_and_maybe_exit(WATCHDOG_EXIT)

    watchdog = threading.Timer(limit_s, on_timeout)
    watchdog.daemon = True
    watchdog.start()
    if (uses_shard_abi(world, cuda, rehearse) and not args.no_scatter) or \
            os.environ.get("BPSR_BENCH_TEST_RCCL") == "shared_device":
        state["leg"] = "rccl"
        if not make_comm():
            watchdog.cancel()
            line["error"] = f"rccl: {line['rccl'].get('problems') or line['rccl'].get('error')}"
            print(f"bench rank {rank}: {line['error']}", file=sys.stderr)
            emit_and_maybe_exit(RCCL_EXIT)
    extra_legs(state)
    watchdog.cancel()
    emit_and_maybe_exit(None)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
