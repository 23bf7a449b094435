"""Probe (not product code): device-release rounds from worker threads with
per-step timestamps, to see which step a worker is in when an epoch stalls."""
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["BPSR_SERVER_RELEASE"] = "device"
os.environ.setdefault("BPSR_SERVER_RELEASE_TIMEOUT_S", "2")
os.environ.setdefault("BPSR_SERVER_RELEASE_DEBUG", "1")
from prophet_amd.dtypes import DType  # noqa: E402
from prophet_amd.reducer import GpuReducer  # noqa: E402
from prophet_amd.server import PSServer  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2
mode = sys.argv[2] if len(sys.argv) > 2 else "ready"
side = len(sys.argv) > 3 and sys.argv[3] == "side"   # copies on a non-blocking torch stream
sizes = [1000, 65_539, 300_001]
keys = [40 + j for j in range(len(sizes))]
dt = DType.FLOAT32
dev = torch.device("cuda:0")
srv = PSServer(N, engine_lanes=2)
t0 = time.perf_counter()


def log(*a):
    print(f"{(time.perf_counter() - t0) * 1e3:9.2f} ms", *a, file=sys.stderr, flush=True)


src = {(w, j): torch.randn(n, device=dev) for w in range(N) for j, n in enumerate(sizes)}
side_streams = [torch.cuda.Stream(device=dev) for _ in range(N)]
torch.cuda.synchronize()


def worker(w):
    try:
        for j, k in enumerate(keys):
            srv.push(k, w, src[(w, j)], dt)
        log(f"w{w} init done")
        for r in range(1, 4):
            for j, k in enumerate(keys):
                if mode == "ready":
                    ptr = srv.recv_slot(k, w)
                    log(f"w{w} r{r} k{k} slot")
                    st = side_streams[w] if side else torch.cuda.current_stream(dev)
                    x = src[(w, j)]
                    GpuReducer().copy(ptr, x, x.numel() * 4, stream=st)
                    st.synchronize()
                    log(f"w{w} r{r} k{k} copied")
                    srv.push_ready(k, w)
                else:
                    srv.push(k, w, src[(w, j)], dt)
                log(f"w{w} r{r} k{k} pushed")
            for j, k in enumerate(keys):
                o = np.zeros(sizes[j] * 4, np.uint8)
                srv.pull(k, o)
                log(f"w{w} r{r} k{k} pulled")
    except Exception as e:  # noqa: BLE001
        log(f"w{w} FAILED {e!r}")


ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
for t in ts:
    t.start()
for t in ts:
    t.join()
log("stats", srv.stats())
srv.close()
