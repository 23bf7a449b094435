"""The native Prophet scheduler's host source under sanitizers (no GPU, no
HIP): prophet_amd/csrc/bpsr_prophet.cpp built with g++ together with
tests/cpp/prophet_threads.cpp — transport threads adding, an engine thread
polling and reporting, a reader thread querying — once under
ThreadSanitizer and once under AddressSanitizer + UBSan.  Every task leaves
exactly once and the sanitizer reports nothing."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_prophet_queue_under_sanitizer(tmp_path, san):
    exe = tmp_path / "prophet_threads"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-Wall", "-Werror", "-pthread",
                    f"-fsanitize={san}", "-fno-omit-frame-pointer",
                    "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "prophet_amd", "csrc"),
                    os.path.join(ROOT, "prophet_amd", "csrc", "bpsr_prophet.cpp"),
                    os.path.join(ROOT, "tests", "cpp", "prophet_threads.cpp"),
                    "-o", str(exe)], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66",
               ASAN_OPTIONS="halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "fails=0" in r.stdout
    assert "Sanitizer" not in r.stderr, r.stderr[-4000:]
