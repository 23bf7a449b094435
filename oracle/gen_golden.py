#!/usr/bin/env python3
"""ORACLE / TEST INFRASTRUCTURE ONLY — generate tests/golden/ from the reference.

Run in the development container (needs /root/reference to build
oracle/_ref/libbpsr_ref.so):

    python oracle/gen_golden.py

For every case the inputs are regenerated deterministically by
prophet_amd.synth (seeded splitmix64), so only the expected OUTPUT bytes are
stored (tests/golden/outputs.bin) plus a manifest with the case parameters and
sha256 of inputs and outputs (tests/golden/manifest.json).

Expected outputs of reference dtypes come from the reference's own compiled
CpuReducer (``pinned_by: "reference"``), replaying the server fold
byteps/server/server.cc:216-250 (merged = first arrival via copy, then
``sum(merged, w_k, len, dtype)`` in arrival order k = 1..N-1).  bf16 has no
reference implementation; its vectors come from the clean-room restatement
(``pinned_by: "port"``).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.oracle import PortReducer, RefReducer, build  # noqa: E402
from prophet_amd import synth  # noqa: E402
from prophet_amd.dtypes import DType, REFERENCE_DTYPES, elem_size  # noqa: E402

OUT_DIR = os.path.join(ROOT, "tests", "golden")

SMALL_N = [1, 7, 8, 9, 63, 64, 65, 1003, 4099]   # spans the F16C body/tail split
WORKERS = [2, 3, 8, 16]


def case_inputs(c: dict) -> list[np.ndarray]:
    """Worker buckets of a case as uint8 arrays of exactly len_bytes."""
    es = elem_size(c["dtype"])
    n_alloc = -(-c["len_bytes"] // es) if c["len_bytes"] else 0
    outs = []
    for k in range(c["n_workers"]):
        if c["value_class"] == "identical":
            b = synth.bucket(c["dtype"], n_alloc, 0, "uniform100", c["seed_base"])
        else:
            b = synth.bucket(c["dtype"], n_alloc, k, c["value_class"], c["seed_base"])
        outs.append(np.ascontiguousarray(b).view(np.uint8)[: c["len_bytes"]].copy())
    return outs


def cases() -> list[dict]:
    cs = []

    def add(op, dtype, n_workers, len_bytes, value_class, seed_base=1000, tag=""):
        cs.append(dict(op=op, dtype=int(dtype), n_workers=n_workers, len_bytes=len_bytes,
                       value_class=value_class, seed_base=seed_base, tag=tag))

    for dt in list(REFERENCE_DTYPES) + [DType.BFLOAT16]:
        es = elem_size(dt)
        for N in WORKERS:
            for n in SMALL_N:
                add("fold", dt, N, n * es, "normal", seed_base=1000 + 17 * n)
        add("fold", dt, 8, 65536 * es, "normal", tag="large")
        add("fold", dt, 2, 0, "normal", tag="empty")
        # ragged: len not a multiple of sizeof(T): sum ignores the tail bytes,
        # the fold's accumulator keeps the first arrival's tail bytes.
        if es > 1:
            for n in (0, 1, 7, 1003):
                add("fold", dt, 3, n * es + es - 1, "normal", seed_base=3000 + n, tag="ragged")
        # 3-operand form (cpu_reducer.cc:130-207)
        for n in (7, 8, 1003):
            add("sum3", dt, 2, n * es, "normal", seed_base=5000 + n)
    for dt in (DType.FLOAT16, DType.BFLOAT16):
        for N in WORKERS:
            for n in (1003, 4099):
                add("fold", dt, N, n * 2, "bits", seed_base=7000 + n, tag="bits")
        add("fold", dt, 8, 65536 * 2, "bits", tag="large-bits")
    for dt in (DType.FLOAT16, DType.BFLOAT16, DType.FLOAT32, DType.FLOAT64):
        es = elem_size(dt)
        for N in (2, 8):
            for n in (63, 1003, 4099):
                add("fold", dt, N, n * es, "special", seed_base=9000 + n, tag="special")
    add("fold", DType.FLOAT32, 8, 65536 * 4, "uniform100", tag="large-uniform100")
    add("fold", DType.FLOAT32, 4, 4099 * 4, "bits", tag="f32-bits-denormals")
    # known-answer ladder of tests/test_mxnet.py:76-113: identical tensors on
    # every rank, shapes (17), (17,17), (17,17,17), expected tensor*size.
    for dt in (DType.FLOAT32, DType.FLOAT64, DType.INT32, DType.INT64):
        for N in (2, 3, 8, 12):
            for n in (17, 17 * 17, 17 ** 3):
                add("fold", dt, N, n * elem_size(dt), "identical", seed_base=1234, tag="ladder")
    for ln in (0, 1, 2, 3, 4, 5, 7, 1001, 4099):
        add("copy", DType.UINT8, 1, ln, "normal", seed_base=11000 + ln)
    for i, c in enumerate(cs):
        c["id"] = i
    return cs


def expected(c: dict, red) -> np.ndarray:
    ins = case_inputs(c)
    L = c["len_bytes"]
    if c["op"] == "copy":
        dst = np.full(L, 0xA5, dtype=np.uint8)
        assert red.copy(dst, ins[0], L) == 0
        return dst
    if c["op"] == "sum3":
        dst = np.full(L, 0xA5, dtype=np.uint8)
        assert red.sum3(dst, ins[0], ins[1], L, c["dtype"]) == 0
        return dst
    acc = ins[0].copy()       # the first arrival, zero-copy in server.cc:216-218
    for s in ins[1:]:
        assert red.sum(acc, s, L, c["dtype"]) == 0
    return acc


def main() -> None:
    build(ref=True)
    if not RefReducer.available():
        sys.exit("oracle/_ref/libbpsr_ref.so missing: /root/reference is required")
    ref, port = RefReducer(nthreads=4), PortReducer(nthreads=4)
    os.makedirs(OUT_DIR, exist_ok=True)
    blob = bytearray()
    manifest = []
    for c in cases():
        ins = case_inputs(c)
        h = hashlib.sha256()
        for x in ins:
            h.update(x.tobytes())
        red = port if c["dtype"] == DType.BFLOAT16 and c["op"] != "copy" else ref
        out = expected(c, red)
        c = dict(c, pinned_by=red.kind, input_sha256=h.hexdigest(),
                 out_offset=len(blob), out_len=int(out.nbytes),
                 out_sha256=hashlib.sha256(out.tobytes()).hexdigest())
        blob += out.tobytes()
        manifest.append(c)
    with open(os.path.join(OUT_DIR, "outputs.bin"), "wb") as f:
        f.write(bytes(blob))
    with open(os.path.join(OUT_DIR, "manifest.json"), "w") as f:
        json.dump({"generator": "oracle/gen_golden.py",
                   "reference": "byteps/common/cpu_reducer.cc via oracle/_ref/libbpsr_ref.so",
                   "fold": "server.cc:216-250 left fold in arrival order",
                   "cases": manifest}, f, indent=0)
    print(f"{len(manifest)} cases, {len(blob)} output bytes -> {OUT_DIR}")


if __name__ == "__main__":
    main()
