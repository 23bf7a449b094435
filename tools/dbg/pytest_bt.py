"""Debug aid (not product code): pytest with tools/dbg/libabrt_bt.so loaded, so
a native abort prints its C++ backtrace.  python tools/dbg/pytest_bt.py <pytest args>"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pytest  # noqa: E402

if __name__ == "__main__":  # spawned children (multiprocessing) re-import this module
    ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libabrt_bt.so"))
    sys.exit(pytest.main(sys.argv[1:] + ["-p", "no:faulthandler"]))
