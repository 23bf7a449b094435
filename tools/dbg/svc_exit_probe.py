"""Probe (not product code): a process that serves blocking device pulls
through the copy service and exits at once without closing its server (the
service kernel may still be polling): it must exit cleanly."""
import threading
import torch
from prophet_amd.server import PSServer
from prophet_amd.dtypes import DType

dev = torch.device("cuda:0")
srv = PSServer(2)
x = [torch.full((1 << 16,), float(w + 1), device=dev) for w in range(2)]
torch.cuda.synchronize()
for r in range(3):
    ts = [threading.Thread(target=srv.push, args=(1, w, x[w], DType.FLOAT32)) for w in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if r:
        outs = [torch.empty(1 << 16, device=dev) for _ in range(2)]
        for o in outs:
            srv.pull(1, o)
        assert all(bool(torch.all(o == 3.0)) for o in outs)
print("stats", srv.stats()["service_pulls"], flush=True)
import os
os._exit(0) if os.environ.get("HARD_EXIT") else None
