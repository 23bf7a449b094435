"""The C ABI from native C++ callers on the GPU (tools/*_native.cpp, built by
__graft_entry__.build() / `make -C tools`): config 3 through the block queue
(stream, pre- and host releases), the native Prophet scheduler and the PUSH
loop in all three modes; config 1 through the PS server on 4 lanes; config 3's
165 keys through the server.  Every driver checks its own results (block
queue against one plan over the same table, server rounds against the fold of
the pushes, server keys for agreement of every worker's pull) and prints one
JSON line per variant; short runs here, the
measurements are in DESIGN.md."""
import json
import os
import subprocess

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")


def _run(args, timeout=240):
    exe = os.path.join(TOOLS, args[0])
    if not os.path.exists(exe):
        pytest.fail(f"{args[0]} not built (make -C tools)")
    r = subprocess.run([exe] + args[1:], capture_output=True, text=True, timeout=timeout,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stdout
    return lines


def test_cfg3_native_every_variant_exact():
    lines = _run(["cfg3_native", "tools/cfg3_resnet50_table.txt", "20", "2",
                  "tools/cfg3_resnet50_tasks.txt"])
    names = {d["variant"] for d in lines}
    for v in ("blockq_live_release", "blockq_pre_released", "blockq_prophet_push_loop",
              "blockq_prophet_push_loop_inline", "blockq_prophet_push_loop_host_release"):
        assert v in names, names
    for d in lines:
        assert d["exact_vs_plan"] is True and d["status"] == 0, d


def test_cfg1_native_server_rounds_exact():
    for d in _run(["cfg1_native", "4", "3"]):
        assert d["exact"] is True, d


def test_server_cfg3_native_keys_consistent():
    """165 keys through the server from 8 worker threads: every worker pulls
    the same store (the fold itself is checked bit-exact by the server tests)."""
    for d in _run(["server_cfg3_native", "tools/cfg3_resnet50_table.txt", "3", "4"]):
        assert d["pulls_agree"] is True, d
