"""The pull copy service's host side on CPU (prophet_amd/csrc/bpsr_copy_service.cpp,
compiled unchanged with g++): its job ring, launch / relaunch rules (idle and
age exits, the `exited` word, jobs stranded by an exit) and its give-up,
against a CPU model of the service kernel's protocol behind a fake HIP runtime
(tests/cpp/copysvc_model.cpp) — racing posters with every byte checked, never
two launches at once, and a give-up that returns only after the launch ended
with no copy after the stop, and a give-up whose launch never ends that returns
a hard error after a bounded wait (no unbounded wait under the
service lock, no fallback copy while the kernel may still write).  Once plain and once under ThreadSanitizer.
(VERDICT round 4 asked for this in place of re-running the r04s14 hang on the
GPU: profiles/README.md records that hang.)"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("san", [None, "thread"])
def test_copy_service_host_logic_against_kernel_model(tmp_path, san):
    exe = tmp_path / "copysvc_model"
    flags = ["-g", f"-fsanitize={san}"] if san else []
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-pthread", *flags,
                    "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "prophet_amd", "csrc"),
                    os.path.join(ROOT, "prophet_amd", "csrc", "bpsr_copy_service.cpp"),
                    os.path.join(ROOT, "tests", "cpp", "copysvc_model.cpp"), "-o", str(exe)],
                   check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fails=0" in r.stdout
    assert "give_up ms=" in r.stdout
    assert "wedged_give_up ms=" in r.stdout   # a launch that never ends: bounded, no fallback
