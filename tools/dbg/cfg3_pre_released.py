"""Probe (not product code), round 6: config 3's block queue (bench.cfg3_leg's
table: ResNet-50 fp16, 8 workers, 165 partitions in 12 Prophet blocks, slots
in one skewed arena) with every iteration released before its launch —
the shape a PMC pass can run (it serialises dispatches, so a live release
could never reach a running consumer).  Launches are NOT overlapped: under a
PMC pass the next launch's dispatch-sequence gate spun beside the launch it
waits for, which the serialisation held back (r06s13: stuck after 20
iterations); the consumer kernel is the same either way (every launch counts
its last workgroups).  For tools/pmc_cfg3_r06.py.
    python tools/dbg/cfg3_pre_released.py [iters=40] [overlap=0]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    overlap = len(sys.argv) > 2 and sys.argv[2] == "1"
    import torch
    from prophet_amd.arena import BucketArena
    from prophet_amd.buckets import partition_all, prophet_blocks, resnet50_param_sizes
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(0)
    N = 8
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
    *w, out = BucketArena(N + 1, total, dev).slots()
    gen = torch.Generator(device=dev)
    for k in range(N):
        gen.manual_seed(3000 + k)
        w[k].copy_(torch.randn(total // 2, device=dev, generator=gen).half().view(torch.uint8))
    q = red.make_blockq([[(out[toff[p.tensor] + p.offset:][:p.len],
                           [x[toff[p.tensor] + p.offset:][:p.len] for x in w], p.len)
                          for p in bp] for bp in by_block], DType.FLOAT16)
    q.config(wg_per_cu=0, timeout_s=5.0)
    q.overlap(overlap)
    rel = q.release_stream()
    torch.cuda.synchronize()
    for i in range(iters):
        q.release(-1, rel)
        q.launch(q.stream())
        if i % 10 == 9:
            torch.cuda.synchronize()
            print(f"iteration {i + 1}", file=sys.stderr, flush=True)
    q.status(q.stream())
    torch.cuda.synchronize()
    ref = w[0].view(torch.float16).clone()
    for x in w[1:]:
        ref.add_(x.view(torch.float16))
    print('{"exact": %s, "iters": %d, "alg_bytes_per_iter": %d}'
          % ("true" if torch.equal(ref.view(torch.uint8), out) else "false", iters, (N + 1) * total),
          flush=True)
    q.close()


if __name__ == "__main__":
    main()
