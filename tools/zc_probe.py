"""Probe (not product): fold with the sources read straight from pinned host
memory by the kernel (no H2D copy), vs the SDMA streaming path.  Prints JSON."""
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from prophet_amd.dtypes import DType  # noqa: E402
from prophet_amd.reducer import GpuReducer  # noqa: E402
from prophet_amd.stream import StreamingReducer  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def devptr(t):
    p = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(t.data_ptr()), 0)
    assert rc == 0, rc
    return p.value


class P:  # object with data_ptr for the reducer
    def __init__(self, v):
        self.v = v

    def data_ptr(self):
        return self.v


N = int(os.environ.get("ZC_N", "8"))
B = int(os.environ.get("ZC_MIB", "256")) << 20
dev = torch.device("cuda")
red = GpuReducer()
host = [torch.randn(B // 4).pin_memory().view(torch.uint8) for _ in range(N)]
hout = torch.empty(B, dtype=torch.uint8).pin_memory()
dout = torch.empty(B, dtype=torch.uint8, device=dev)
srcs = [P(devptr(h)) for h in host]
s = torch.cuda.current_stream()


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts)


want = host[0].view(torch.float32).to(dev).clone()
for h in host[1:]:
    want += h.view(torch.float32).to(dev)

t = timeit(lambda: red.sum_n(dout, srcs, B, DType.FLOAT32))
ok = torch.equal(dout, want.view(torch.uint8))
print(json.dumps(dict(v="zerocopy_src_to_hbm", n=N, mib=B >> 20, ms=round(t * 1e3, 2),
                      gibps=round(N * B / t / 2**30, 2), exact=bool(ok))), flush=True)
hdst = P(devptr(hout))
t = timeit(lambda: red.sum_n(hdst, srcs, B, DType.FLOAT32))
ok = torch.equal(hout.to(dev), want.view(torch.uint8))
print(json.dumps(dict(v="zerocopy_src_to_host", n=N, mib=B >> 20, ms=round(t * 1e3, 2),
                      gibps=round(N * B / t / 2**30, 2), exact=bool(ok))), flush=True)
sr = StreamingReducer(N, chunk_bytes=32 << 20, depth=3, device=dev, reducer=red)
t = timeit(lambda: sr.reduce(host, hout, B, DType.FLOAT32))
ok = torch.equal(hout.to(dev), want.view(torch.uint8))
print(json.dumps(dict(v="streamed_sdma", n=N, mib=B >> 20, ms=round(t * 1e3, 2),
                      gibps=round(N * B / t / 2**30, 2), exact=bool(ok))), flush=True)
