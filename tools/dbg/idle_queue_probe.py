"""Probe (not product code), round 6: does the host-resident server (config 1,
bench.server_group_leg) slow down merely because the process holds more
hardware queues — idle ones?  Round 5 measured 3.1 ms per round when the
server was made before the block queue's consumer queues existed and 4.3 ms
after (r05s42); the consumer queues are all-CU-masked streams (a hardware
queue each) that sit idle during the server leg.  Here idle streams of each
kind are created (and later destroyed) between server_cfg1 runs, with no
block queue at all.  One line per measurement.
    python tools/dbg/idle_queue_probe.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import bench
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(0)
    hip = ctypes.CDLL("libamdhip64.so")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    mask = (ctypes.c_uint32 * ((cus + 31) // 32))()
    for c in range(cus):
        mask[c // 32] |= 1 << (c % 32)
    made = []

    def make(kind, n):
        for _ in range(n):
            s = ctypes.c_void_p()
            if kind == "cumask":
                rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), len(mask), mask)
            elif kind == "high":
                rc = hip.hipStreamCreateWithPriority(ctypes.byref(s), 1, -1)
            else:
                rc = hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
            assert rc == 0, rc
            # one tiny op so the runtime binds a hardware queue to the stream
            ev = ctypes.c_void_p()
            assert hip.hipEventCreate(ctypes.byref(ev)) == 0
            assert hip.hipEventRecord(ev, s) == 0
            assert hip.hipEventSynchronize(ev) == 0
            hip.hipEventDestroy(ev)
            made.append(s)

    def destroy_all():
        for s in made:
            hip.hipStreamDestroy(s)
        made.clear()

    link = bench.pcie_leg(dev, red)

    def run(tag):
        r = bench.server_group_leg(dev, 1, 0, link=link)
        print(f"{tag}: round_ms {r['round_ms']} frac_of_link {r.get('frac_of_link')} "
              f"copying_pulls {r['copying_pulls']['round_ms']}", flush=True)

    run("fresh")
    run("again")
    make("cumask", 2)
    run("+2 idle cu-masked streams")
    make("cumask", 2)
    run("+4 idle cu-masked streams")
    destroy_all()
    run("cu-masked streams destroyed")
    make("high", 3)
    run("+3 idle high-priority streams")
    destroy_all()
    make("normal", 12)
    run("+12 idle normal streams")
    destroy_all()
    run("all destroyed")


if __name__ == "__main__":
    main()
