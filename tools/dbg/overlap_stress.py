"""Stress probe (not product code) for overlapping block-queue launches
(byteps_reduce_blockq_overlap): two queues of different shapes on one device,
iterations enqueued back to back with releases that wait for the previous
iteration (the deadlock pattern of DESIGN.md §4.4), mixed with stream-ordered
and host releases and random host-side delays.  Every iteration's outputs are
checked against torch's left fold; prints one JSON line per phase and exits
non-zero on the first mismatch or timeout.
    python tools/dbg/overlap_stress.py [--iters 200] [--seed 1]"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--pipelined", action="store_true",
                    help="no host sync per iteration: keep every iteration's copies and "
                         "check them at the end (inputs flip sign each iteration, so the "
                         "expected sums alternate between r and -r exactly)")
    a = ap.parse_args()
    import torch
    from prophet_amd.buckets import prophet_blocks, resnet50_param_sizes
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(0)
    rng = random.Random(a.seed)
    sizes = resnet50_param_sizes()
    groups = prophet_blocks(len(sizes))

    def make(scale, N, dt):
        tdt = torch.float16 if dt == DType.FLOAT16 else torch.float32
        blocks, ins, outs = [], [], []
        for g in groups:
            blk = []
            for i in g:
                n = max(1, sizes[i] // scale)
                xs = [torch.randn(n, device=dev).to(tdt) for _ in range(N)]
                o = torch.empty(n, device=dev, dtype=tdt)
                blk.append((o.view(torch.uint8), [x.view(torch.uint8) for x in xs], o.numel() * o.element_size()))
                ins.append(xs)
                outs.append(o)
            blocks.append(blk)
        q = red.make_blockq(blocks, dt)
        q.config(wg_per_cu=0, timeout_s=2.0)
        q.overlap(True)
        return q, ins, outs

    qa, ia, oa = make(4, 8, DType.FLOAT16)
    qb, ib, ob = make(16, 5, DType.FLOAT32)
    side, out_s = torch.cuda.Stream(), torch.cuda.Stream()
    cons = qa.stream()

    def refs(ins):
        r = []
        for xs in ins:
            acc = xs[0].clone()
            for x in xs[1:]:
                acc.add_(x)
            r.append(acc)
        return r

    t0 = time.time()
    bad = 0
    kept = []
    ref_a0, ref_b0 = refs(ia), refs(ib)   # before any flip
    for it in range(a.iters):
        # new inputs for both queues, written on `side` after every launch so far
        qa.join(side)
        with torch.cuda.stream(side):
            for xs in ia + ib:
                for x in xs:
                    x.mul_(-1.0)          # exact, changes every value
        mode = rng.choice(["stream", "stream_late", "host"])
        if mode == "host":
            side.synchronize()            # data visible: host releases allowed
        qa.host_releases(mode == "host")  # read at the launch (its forwarding workgroup)
        qa.launch(cons)
        if rng.random() < 0.5:
            qb.launch(cons)
            qb.release(-1, side)
            did_b = True
        else:
            did_b = False
        if mode == "host":
            qa.release_host(0, qa.nblocks)
        else:
            if mode == "stream_late":
                time.sleep(rng.random() * 0.002)
            for b in rng.sample(range(qa.nblocks), qa.nblocks):
                qa.release(b, side)
        qa.join(out_s)
        with torch.cuda.stream(out_s):
            got_a = [o.clone() for o in oa]
            got_b = [o.clone() for o in ob] if did_b else None
        side.wait_stream(out_s)
        if a.pipelined:
            kept.append((it, got_a, got_b))
            continue
        out_s.synchronize()
        ok = all(torch.equal(g, r) for g, r in zip(got_a, refs(ia)))
        if did_b:
            ok = ok and all(torch.equal(g, r) for g, r in zip(got_b, refs(ib)))
        if not ok:
            bad += 1
            print(json.dumps({"iter": it, "mode": mode, "b": did_b, "exact": False}), flush=True)
            break
        if it % 50 == 0:
            print(json.dumps({"iter": it, "elapsed_s": round(time.time() - t0, 1)}), flush=True)
    torch.cuda.synchronize()
    for it, got_a, got_b in kept:
        sign = -1.0 if it % 2 == 0 else 1.0   # iteration it folds inputs flipped it+1 times
        ok = all(torch.equal(g, r * sign) for g, r in zip(got_a, ref_a0))
        if got_b is not None:
            ok = ok and all(torch.equal(g, r * sign) for g, r in zip(got_b, ref_b0))
        if not ok:
            bad += 1
            print(json.dumps({"iter": it, "exact": False}), flush=True)
            break
    qa.status(cons)
    qb.status(cons)
    print(json.dumps({"iters": a.iters, "mismatches": bad, "elapsed_s": round(time.time() - t0, 1)}),
          flush=True)
    qa.close()
    qb.close()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
