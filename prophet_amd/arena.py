"""HBM layout of per-worker bucket slots.

The server keeps one receive slot per pushing worker for each bucket (the
ps-lite receive buffers of byteps/server/server.cc:174,216-218, here resident
in HBM).  Slots are carved from one device slab with a small skew between
consecutive workers: with slots exactly a power of two apart (e.g. 256 MiB
buckets from separate allocations), the N concurrent read streams of the fold
alias onto the same HBM channel/bank pattern; a skew of a few KiB spreads
them (measured on MI355X: +2-5 % on the 8-way 256 MiB fold over separate
allocations, tools/sweep.py; DESIGN.md "HBM layout").
"""
from __future__ import annotations

DEFAULT_SKEW = 16 * 1024   # bytes between consecutive slots beyond the (64 KiB-rounded) bucket
# Buckets larger than the headline's 256 MiB: slots ~2 MiB further apart.
# With the 16 KiB skew the 8-way fp32 fold of such buckets ran at 0.78-0.80
# of 8 TB/s (config 4's 553 MB set 0.786-0.796, 512 MiB 0.787, 1 GiB 0.777)
# against 0.82 at 256 MiB; with 2 MiB + 16 KiB at 0.818-0.841 (553 MB 0.815-
# 0.818, 512 MiB 0.829, 1 GiB 0.841) — while 256 MiB buckets fold at 0.77 with
# it and 0.82 with 16 KiB (tools/dbg/skew_probe.py, profiles/
# r06s09_s10_arena_skew.jsonl; DESIGN.md §5 "slot spacing").  Which skew
# suits which slot distance is the DRAM address hash's business; these are
# the measured classes.
LARGE = 256 * 1024 * 1024 + 64 * 1024
LARGE_SKEW = 2 * 1024 * 1024 + 16 * 1024
# Buckets are rounded up to 64 KiB before the skew, so the skew's class
# modulo the channel interleave does not depend on the bucket size: with 4 KiB
# rounding a bucket of 8 KiB mod 16 KiB (config 4's VGG-16 shards) turned the
# 16 KiB skew into an effective 24 KiB, a skew class measured 5-6 % slower
# (DESIGN.md §5 "Arena skew"; r02s94: 99.3 vs 95.4 us for the G = 8 shard).
ALIGN = 64 * 1024
SMALL = 1 << 20      # below this, 4 KiB rounding (latency-bound, keep small slots small)


def default_skew(bucket_bytes: int) -> int:
    return LARGE_SKEW if bucket_bytes > LARGE else DEFAULT_SKEW


class BucketArena:
    """``n_slots`` buckets of ``bucket_bytes`` in one uint8 device tensor.
    ``skew`` None: the measured class of the bucket size (above)."""

    def __init__(self, n_slots: int, bucket_bytes: int, device, skew: int | None = None):
        import torch
        self.bucket_bytes = int(bucket_bytes)
        if skew is None:
            skew = default_skew(self.bucket_bytes)
        align = ALIGN if self.bucket_bytes >= SMALL else 4096
        self.stride = (self.bucket_bytes + align - 1) // align * align + int(skew)
        self.n_slots = n_slots
        self.slab = torch.empty(self.stride * n_slots, dtype=torch.uint8, device=device)

    def slot(self, k: int):
        o = k * self.stride
        return self.slab[o: o + self.bucket_bytes]

    def slots(self):
        return [self.slot(k) for k in range(self.n_slots)]
