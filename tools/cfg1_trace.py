"""One cfg1 pipelined variant (pull views; blocking or non-blocking pushes) for
a rocprofv3 copy/kernel trace: python tools/cfg1_trace.py [async]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

import bench_configs as b  # noqa: E402

N, B = 2, 64 << 20
host = [torch.randn(B // 4).pin_memory() for _ in range(N)]
b.cfg1_pipelined(host, N, B, view=True, push_async=len(sys.argv) > 1 and sys.argv[1] == "async")
