OUT=gpurun_out/${TAG:-r01_lanes}; mkdir -p $OUT
for l in 1 2 4 8; do BPSR_CFG1_LANES=$l timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'tools'); sys.path.insert(0,'.')
import torch, bench_configs as b
from prophet_amd import synth
N,B=2,64<<20
host=[torch.randn(B//4).pin_memory() for _ in range(N)]
b.cfg1_pipelined(host,N,B,view=True)
b.cfg1_pipelined(host,N,B,view=True,push_async=True)
" >> $OUT/lanes.log 2>&1 || exit 1; done
