"""ORACLE / TEST INFRASTRUCTURE ONLY.

Importable solely from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — as the checker, never as the thing measured or shipped.
The product library (prophet_amd/libbpsr.so) never links or calls anything
here.
"""
