"""Key space over several server instances (byteps_server_group_*,
include/bpsr/server.h) on a CPU host: the reference's key hashes
(global.cc:491-523), the stateless routing rule in both split modes and the
environment configuration.  The GPU test (tests/test_server_group_gpu.py)
runs rounds through the instances."""
import ctypes
import os
import subprocess

import pytest

from prophet_amd import reducer, server
from prophet_amd.server import key_hash, make_group_config, route

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M64 = (1 << 64) - 1
KEYS = [0, 1, 7, 9, 10, 65535, 65536, 65537, (5 << 16) + 3, (160 << 16) + 0, (4097 << 16) + 9,
        123456789012, M64]


def _djb2(k):
    h = 5381
    for c in str(k).encode():
        h = (h * 33 + c) & M64
    return h


def _sdbm(k):
    h = 0
    for c in str(k).encode():
        h = (c + (h << 6) + (h << 16) - h) & M64
    return h


def test_key_hashes_match_the_reference_formulas():
    for k in KEYS:
        assert key_hash(k, "djb2") == _djb2(k)
        assert key_hash(k, "sdbm") == _sdbm(k)
        assert key_hash(k, "naive") == (((k >> 16) + (k % 65536)) * 9973) & M64


def test_built_in_hash_is_libstdcxx_std_hash(tmp_path):
    exe = tmp_path / "key_hash"
    subprocess.run(["g++", "-std=c++11", "-O2", os.path.join(ROOT, "tests", "cpp", "key_hash.cpp"),
                    "-o", str(exe)], check=True)
    for coef in (1, 3):
        out = subprocess.run([str(exe), str(coef)], input="\n".join(map(str, KEYS)),
                             capture_output=True, text=True, check=True).stdout.split()
        assert [key_hash(k, "built_in", coef) for k in KEYS] == [int(x) for x in out]


@pytest.mark.parametrize("fn", ["djb2", "naive", "sdbm"])
@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_hash_split_routes_whole_keys(fn, n):
    """EncodeDefaultKey (global.cc:537-560): one server per key, hash % n."""
    c = make_group_config(4, [0] * n, split="hash", hash_fn=fn)
    for k in KEYS:
        for ln in (1, 4096, 4_096_000):
            assert route(c, k, ln) == [(key_hash(k, fn) % n, 0, ln)]


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("ln", [128 * 8, 4_096_000, 4_095_999, 1_000_003, 411_041_792])
def test_range_split_owner_ranges_in_128_byte_units(n, ln):
    """Every instance owns one contiguous piece; starts are multiples of 128
    bytes (8 elements of every dtype: the fp16 body/tail rule holds per
    piece); the last instance takes the tail (core_loops.cc:210-211)."""
    c = make_group_config(4, [0] * n, split="range")
    ps = route(c, (3 << 16) + 1, ln)
    if ln // 128 < n:
        assert len(ps) == 1
        return
    assert [p[0] for p in ps] == list(range(n))
    per = ln // 128 // n * 128
    assert all(off == i * per and off % 128 == 0 for i, (_, off, _) in enumerate(ps))
    assert all(plen == per for _, _, plen in ps[:-1])
    assert ps[-1][1] + ps[-1][2] == ln and ps[-1][2] >= per


def test_range_split_small_keys_go_whole_by_hash():
    c = make_group_config(4, [0, 0, 0], split="range", split_min_bytes=1 << 20)
    for k in KEYS:
        assert route(c, k, (1 << 20) - 1) == [(key_hash(k) % 3, 0, (1 << 20) - 1)]
        assert len(route(c, k, 1 << 20)) == 3
    c = make_group_config(4, [0, 0, 0], split="range")     # default minimum: 128 * n
    assert len(route(c, 1, 383)) == 1 and len(route(c, 1, 384)) == 3


def test_route_config_errors():
    L = server._lib()
    n = ctypes.c_int()
    for bad in (dict(devices=[]), dict(devices=[0] * 17)):
        c = make_group_config(2, **bad)
        assert L.byteps_server_route(ctypes.byref(c), 1, 10, ctypes.byref(n), None, None, None,
                                     0) == reducer.EARGS
    c = make_group_config(2, [0, 0])
    c.split = 5
    assert L.byteps_server_route(ctypes.byref(c), 1, 10, ctypes.byref(n), None, None, None,
                                 0) == reducer.EARGS
    c = make_group_config(2, [0, -1])
    assert L.byteps_server_route(ctypes.byref(c), 1, 10, ctypes.byref(n), None, None, None,
                                 0) == reducer.EARGS
    h = ctypes.c_void_p()
    assert L.byteps_server_group_create(ctypes.byref(c), ctypes.byref(h)) == reducer.EARGS
    assert L.byteps_server_group_push(None, 1, 0, None, 0, 0, 0) == reducer.EARGS
    assert L.byteps_server_group_destroy(None) == reducer.OK


def test_group_config_from_env(monkeypatch):
    for k, v in {"DMLC_NUM_WORKER": "8", "BPSR_SERVER_GPUS": "4", "BPSR_SERVER_SPLIT": "range",
                 "BYTEPS_KEY_HASH_FN": "sdbm", "BPSR_SERVER_SPLIT_MIN_BYTES": "65536"}.items():
        monkeypatch.setenv(k, v)
    c = server.group_config_from_env()
    assert (c.server.num_workers, c.num_servers, list(c.devices[:4]), c.split, c.hash_fn,
            c.split_min_bytes) == (8, 4, [0, 1, 2, 3], server.SPLIT_RANGE, 2, 65536)
    monkeypatch.setenv("BYTEPS_KEY_HASH_FN", "built_in")
    monkeypatch.setenv("BYTEPS_BUILT_IN_HASH_COEF", "7")
    c = server.group_config_from_env()
    assert (c.hash_fn, c.hash_coef) == (3, 7)
    monkeypatch.delenv("BYTEPS_KEY_HASH_FN")
    monkeypatch.delenv("BPSR_SERVER_SPLIT")
    c = server.group_config_from_env()
    assert (c.hash_fn, c.split) == (0, server.SPLIT_HASH)        # djb2 default, whole keys
    monkeypatch.setenv("BYTEPS_KEY_HASH_FN", "md5")                # the reference aborts here
    with pytest.raises(reducer.ReduceError, match="BYTEPS_KEY_HASH_FN"):
        server.group_config_from_env()
    monkeypatch.setenv("BYTEPS_KEY_HASH_FN", "djb2")
    monkeypatch.setenv("BPSR_SERVER_GPUS", "17")
    with pytest.raises(reducer.ReduceError):
        server.group_config_from_env()


def test_producer_events_skip_host_buffers():
    """numpy 2 arrays carry a ``.device`` attribute too: the producer ordering
    of the calls (an event per device with pending work, for
    byteps_server_order_after) must skip host buffers (numpy and CPU tensors)
    without touching a GPU, and then order nothing."""
    import numpy as np
    import torch
    assert server._producer_events([np.zeros(4, np.uint8), torch.zeros(4), np.ones(2)]) == []
    calls = []
    server._order_after(lambda *a: calls.append(a) or 0, None, [1, 2], [np.zeros(4)])
    assert calls == []


def test_order_after_argument_errors_without_gpu():
    """byteps_server_order_after / _group_order_after refuse null handles and
    events before any HIP call."""
    import ctypes
    lib = server._lib()
    ev = ctypes.c_void_p(1)
    assert lib.byteps_server_order_after(None, None, 0, ev) == reducer.EARGS
    assert lib.byteps_server_group_order_after(None, None, 0, ev) == reducer.EARGS
