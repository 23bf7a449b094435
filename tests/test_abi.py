"""The C-ABI library loads here (no GPU) and exports exactly what
include/bpsr/{reduce,server,prophet,shard}.h declare; host-only argument checks run without a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from prophet_amd import reducer
from prophet_amd.dtypes import ALL_DTYPES, elem_size

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", "bpsr", h)
           for h in ("reduce.h", "server.h", "prophet.h", "shard.h")]


def header_functions(headers=HEADERS):
    names = set()
    for h in headers:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(byteps_\w+)\s*\(", text))
    return sorted(names)


def test_header_declares_expected_api():
    from prophet_amd.server import SERVER_EXPORTS
    assert header_functions(HEADERS[:1]) == sorted(reducer.EXPORTS)
    assert header_functions(HEADERS[1:2]) == sorted(SERVER_EXPORTS)
    from prophet_amd.prophet import PROPHET_EXPORTS
    assert header_functions(HEADERS[2:3]) == sorted(PROPHET_EXPORTS)
    from prophet_amd.shard import SHARD_EXPORTS
    assert header_functions(HEADERS[3:]) == sorted(SHARD_EXPORTS)


def test_library_exports_every_header_symbol():
    lib = reducer.load_library()
    for name in header_functions():
        assert hasattr(lib, name), name


def test_library_exports_nothing_but_the_header_api():
    """The reference's export policy (byteps.lds:1-8, global: *byteps*;
    local: *, passed by setup.py:207): EVERY defined dynamic symbol of
    libbpsr.so -- functions, data, vtables, typeinfo, template instantiations,
    kernel host stubs -- is one of the C functions include/bpsr/*.h declares.
    Nothing from bpsr:: or libstdc++ joins the global scope of a process that
    loads the library RTLD_GLOBAL (byteps/server/__init__.py:22-23)."""
    out = subprocess.run(["nm", "-D", "--defined-only", reducer.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    defined = {}
    for line in out.splitlines():
        parts = line.split()
        if len(parts) == 3:
            defined[parts[2]] = parts[1]
    assert defined, out
    assert set(defined) == set(header_functions()), sorted(set(defined) ^ set(header_functions()))
    assert all(kind == "T" for kind in defined.values()), defined
    assert all(re.fullmatch(r"byteps_\w+", s) and "byteps" in s for s in defined)


def test_library_build_applies_the_export_policy():
    """The build keeps the policy: hidden visibility by default, the version
    script on the link line, and the script's only global pattern byteps_*
    (a subset of the reference's *byteps*)."""
    mk = open(os.path.join(ROOT, "prophet_amd", "csrc", "Makefile")).read()
    assert "-fvisibility=hidden" in mk and "--version-script=$(HERE)bpsr.lds" in mk
    lds = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "prophet_amd", "csrc", "bpsr.lds")).read(),
                 flags=re.S)
    assert re.sub(r"\s+", " ", lds).strip() == "{ global: byteps_*; local: *; };"
    for h in HEADERS:
        text = open(h).read()
        assert text.count("#pragma GCC visibility push(default)") == 1, h
        assert text.count("#pragma GCC visibility pop") == 1, h


def test_version_and_dtype_sizes():
    lib = reducer.load_library()
    assert lib.byteps_reduce_version() == 5
    for dt in ALL_DTYPES:
        assert lib.byteps_reduce_dtype_size(int(dt)) == elem_size(dt)
    assert lib.byteps_reduce_dtype_size(7) == reducer.EDTYPE
    assert b"Unsupported data type" in lib.byteps_reduce_last_error()


def test_argument_errors_without_gpu():
    """Validation happens before any HIP call, so these run on a CPU host."""
    r = reducer.GpuReducer()
    with pytest.raises(reducer.ReduceError) as e:
        r.sum(0x1000, 0x2000, 64, 9)
    assert e.value.code == reducer.EDTYPE
    with pytest.raises(reducer.ReduceError) as e:
        r.sum(0x1000, 0x1004, 64, 0)          # partial overlap
    assert e.value.code == reducer.EARGS
    with pytest.raises(reducer.ReduceError) as e:
        r.sum_n(0x1000, [], 64, 0)
    assert e.value.code == reducer.EARGS
    with pytest.raises(reducer.ReduceError) as e:
        r.sum_n(0x1000, [0x1000, 0x1000], 64, 0)   # dst may alias srcs[0] only
    assert e.value.code == reducer.EARGS
    with pytest.raises(reducer.ReduceError) as e:
        r.sum_n(0x1000, [0x2000, 0x3000], 64, 0, mode=5)
    assert e.value.code == reducer.EARGS
    # zero-length calls are no-ops that succeed (reference loops run 0 times)
    r.sum(0x1000, 0x2000, 0, 0)
    r.copy(0x1000, 0x2000, 0)


def test_tuning_roundtrip():
    r = reducer.GpuReducer()
    old = r.get_tuning()
    r.set_tuning(4, 0, 512, 3)
    assert r.get_tuning() == (4, 0, 512, 3)
    with pytest.raises(reducer.ReduceError):
        r.set_tuning(3)
    with pytest.raises(reducer.ReduceError):
        r.set_tuning(occ=9)
    r.set_tuning(*old)
    assert r.get_tuning() == old


def test_bucket_desc_layout_matches_header():
    # void* dst; const void* srcs[32]; size_t len; int n; int reserved;
    assert ctypes.sizeof(reducer.BucketDesc) == 8 + 32 * 8 + 8 + 4 + 4


def test_cpp_wrapper_compiles_with_reference_flags(tmp_path):
    """include/bpsr/gpu_reducer.hpp, gpu_shard.hpp, reduce.h and shard.h under
    the reference's own compiler settings (g++ -std=c++11 -Wall, setup.py:171),
    linked to libbpsr.so."""
    exe = tmp_path / "header_check"
    src = os.path.join(ROOT, "tests", "cpp", "header_check.cpp")
    libdir = os.path.dirname(reducer.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    src, "-L", libdir, "-lbpsr", f"-Wl,-rpath,{libdir}", "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fails=0" in r.stdout


def test_server_config_and_errors_without_gpu(monkeypatch):
    from prophet_amd import server
    monkeypatch.setenv("DMLC_NUM_WORKER", "8")
    monkeypatch.setenv("BYTEPS_SERVER_ENGINE_THREAD", "3")
    monkeypatch.setenv("BYTEPS_ENABLE_ASYNC", "0")
    monkeypatch.setenv("BPSR_SERVER_POLICY", "incremental")
    monkeypatch.setenv("BYTEPS_SERVER_ENGINE_BLOCKING", "1")
    c = server.config_from_env()
    assert (c.num_workers, c.engine_lanes, c.async_mode, c.policy) == (8, 3, 0, server.INCREMENTAL)
    assert c.engine_blocking == 1
    monkeypatch.setenv("BYTEPS_SERVER_ENGINE_BLOCKING", "0")
    assert server.config_from_env().engine_blocking == 0
    # the dedicated server process: device releases (round 6, server.h — its
    # copied rounds run no consumer, its slot-written ones fold on the device)
    assert c.release == server.RELEASE_DEVICE
    monkeypatch.setenv("BPSR_SERVER_RELEASE", "launch")   # read at create, not here
    assert server.config_from_env().release == server.RELEASE_DEVICE
    lib = server._lib()
    bad = server.ServerConfig(0, 4, 0, 0, 0)
    h = ctypes.c_void_p()
    assert lib.byteps_server_create(ctypes.byref(bad), ctypes.byref(h)) == reducer.EARGS
    bad = server.ServerConfig(2, 0, 0, 0, 0)      # server.cc:332 CHECK_GE(threads, 1)
    assert lib.byteps_server_create(ctypes.byref(bad), ctypes.byref(h)) == reducer.EARGS
    bad = server.ServerConfig(2, 4, 0, 0, 0, 0, 0, 7)  # no such release
    assert lib.byteps_server_create(ctypes.byref(bad), ctypes.byref(h)) == reducer.EARGS
    # the sized entry point: a caller states its struct's size,
    # and a size that is no known version is refused before any field is read
    # past it; an ABI-3 struct (28 B, no release) is read as release = LAUNCH
    lib.byteps_server_create_sized.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    assert ctypes.sizeof(server.ServerConfig) == 32
    for size in (0, 20, 30, 36):
        assert lib.byteps_server_create_sized(ctypes.byref(bad), size, ctypes.byref(h)) == reducer.EARGS
        assert b"not a known version" in lib.byteps_reduce_last_error()
    bad = server.ServerConfig(0, 4, 0, 0, 0, 0, 0, 7)   # v3 prefix still validated
    assert lib.byteps_server_create_sized(ctypes.byref(bad), 28, ctypes.byref(h)) == reducer.EARGS
    assert b"num_workers" in lib.byteps_reduce_last_error()
    assert lib.byteps_server_pull(None, 1, None, 0, 0) == reducer.EARGS
    assert lib.byteps_server_pull_host_view(None, 1, None, None) == reducer.EARGS
    assert lib.byteps_server_pull_async(None, 1, server.PULL_CB(), None) == reducer.EARGS
    assert lib.byteps_server_push_async(None, 1, 0, None, 0, 0, 0, server.PUSH_CB(),
                                        None) == reducer.EARGS


def test_block_queue_argument_errors_without_gpu():
    """byteps_reduce_blockq_* validates the block partition and handles before
    any HIP call: bad block ends, a last block that does not end at nbuckets,
    no blocks, null handles."""
    lib = reducer.load_library()
    descs = (reducer.BucketDesc * 2)()
    for i in range(2):
        descs[i].dst = 0x10000 * (i + 1)
        descs[i].srcs[0] = 0x100000 * (i + 1)
        descs[i].len = 64
        descs[i].n = 1
    h = ctypes.c_void_p()
    for ends in ([3], [1], [2, 1], [1, 3]):
        arr = (ctypes.c_int * len(ends))(*ends)
        rc = lib.byteps_reduce_blockq_create(descs, 2, arr, len(ends), 0, 0, ctypes.byref(h))
        assert rc == reducer.EARGS, ends
        assert not h.value
    arr = (ctypes.c_int * 1)(2)
    assert lib.byteps_reduce_blockq_create(descs, 2, arr, 0, 0, 0, ctypes.byref(h)) == reducer.EARGS
    assert lib.byteps_reduce_blockq_create(descs, 2, arr, 1, 9, 0, ctypes.byref(h)) == reducer.EDTYPE
    assert lib.byteps_reduce_blockq_launch(None, None) == reducer.EARGS
    assert lib.byteps_reduce_blockq_release(None, 0, None) == reducer.EARGS
    assert lib.byteps_reduce_blockq_status(None, None) == reducer.EARGS
    assert lib.byteps_reduce_blockq_config(None, 0, 1.0) == reducer.EARGS
    assert lib.byteps_reduce_blockq_overlap(None, 1) == reducer.EARGS
    assert lib.byteps_reduce_blockq_join(None, None) == reducer.EARGS
    assert lib.byteps_reduce_blockq_destroy(None) == reducer.OK


def test_prophet_scheduler_from_c(tmp_path):
    """include/bpsr/prophet.h from plain C99 (gcc -Wall -Werror), linked to
    libbpsr.so: polls and the whole-iteration driver give the hand trace of
    tests/test_prophet.py::test_budget_releases_lowest_index_first, handles
    come back unchanged.  Host-only calls: no GPU."""
    exe = tmp_path / "prophet_drive"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "prophet_drive.c"), "-o", str(exe),
                    "-L", os.path.dirname(reducer.LIB_PATH), "-lbpsr",
                    "-Wl,-rpath," + os.path.dirname(reducer.LIB_PATH)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    assert out[0].split() == ["2:0", "3:0", "0:-1", "1:-1"]
    assert out[1].split() == ["2:0:101", "3:0:100", "|", "0:-1:103", "1:-1:102", "|"]
    assert out[2].split() == ["-1:5", "2:2", "6:0.2", "9:0"]       # profile
    assert out[3] == f"{4_096_000 * 8 / 3277:.3f}"                 # Z_NET_B, Mb/s
