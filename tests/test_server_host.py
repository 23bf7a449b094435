"""Host-side pieces of the server and the library that need no GPU.

* The engine queue's BYTEPS_SERVER_ENABLE_SCHEDULE ordering
  (byteps/server/queue.h:68-97), compiled from the library's own header with
  g++ and run (tests/cpp/engine_queue_check.cpp).
* byteps_reduce_set_tuning hammered from threads while other threads read the
  tuning and run the argument-check paths (SURVEY §8b "Threading": the C ABI
  is called concurrently from engine threads): every read sees a whole
  setting, never a torn mix, and failed sets change nothing.
* byteps_server_config_from_env reads BYTEPS_SERVER_ENABLE_SCHEDULE.
"""
import os
import subprocess
import threading

import pytest

from prophet_amd import reducer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("san", [None, "thread", "address,undefined"])
def test_engine_queue_schedule_order(tmp_path, san):
    exe = tmp_path / "engine_queue_check"
    flags = [f"-fsanitize={san}", "-g"] if san else []
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-pthread", *flags,
                    "-I", os.path.join(ROOT, "prophet_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "engine_queue_check.cpp"), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fails=0" in r.stdout
    assert "Sanitizer" not in r.stderr, r.stderr[-4000:]


def test_set_tuning_from_threads_never_tears():
    r = reducer.GpuReducer()
    old = r.get_tuning()
    settings = [(1, 0, 512, 3), (4, 1, 1024, 2)]
    allowed = set(settings)
    stop = threading.Event()
    bad = []

    def writer(k):
        i = 0
        while not stop.is_set():
            r.set_tuning(*settings[(i + k) % 2])
            try:
                r.set_tuning(1, 0, 777, 9)       # rejected: must change nothing
            except reducer.ReduceError:
                pass
            i += 1

    def reader():
        while not stop.is_set():
            t = r.get_tuning()
            if t not in allowed:
                bad.append(t)

    def checker():
        while not stop.is_set():
            with pytest.raises(reducer.ReduceError):
                r.sum(0x1000, 0x2000, 64, 9)       # bad dtype, before any HIP call
            with pytest.raises(reducer.ReduceError):
                r.sum_n(0x1000, [0x1000, 0x1000], 64, 0)

    r.set_tuning(*settings[0])
    ths = ([threading.Thread(target=writer, args=(k,)) for k in range(2)]
           + [threading.Thread(target=reader) for _ in range(2)]
           + [threading.Thread(target=checker) for _ in range(2)])
    for t in ths:
        t.start()
    threading.Event().wait(1.5)
    stop.set()
    for t in ths:
        t.join()
    r.set_tuning(*old)
    assert r.get_tuning() == old
    assert not bad, bad[:5]


def test_server_config_reads_schedule_flag(monkeypatch):
    from prophet_amd import server
    monkeypatch.setenv("BYTEPS_SERVER_ENABLE_SCHEDULE", "1")
    assert server.config_from_env().enable_schedule == 1
    monkeypatch.setenv("BYTEPS_SERVER_ENABLE_SCHEDULE", "0")
    assert server.config_from_env().enable_schedule == 0
    monkeypatch.delenv("BYTEPS_SERVER_ENABLE_SCHEDULE")
    assert server.config_from_env().enable_schedule == 0
    assert server._lib().byteps_server_debug_lane(None, 0, 1, None, 0, None) == reducer.EARGS
