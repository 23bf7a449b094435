"""The CPU oracle (oracle/bpsr_oracle.c) pinned against the reference.

* every golden vector (produced by the reference's compiled CpuReducer) is
  reproduced bit for bit by the clean-room restatement;
* when oracle/_ref/libbpsr_ref.so is present, fresh seeded inputs are
  cross-checked live against the reference itself;
* the known-answer ladder of the reference's own test (tests/test_mxnet.py:76-113).
"""
import numpy as np
import pytest

from golden_util import assert_bytes_match, case_id, expected, inputs, manifest
from oracle.oracle import PortReducer, RefReducer
from prophet_amd import synth
from prophet_amd.dtypes import DType, REFERENCE_DTYPES, elem_size

CASES = manifest()


@pytest.fixture(scope="module")
def port():
    return PortReducer(nthreads=4)


def run_case(red, case):
    ins = inputs(case)
    L = case["len_bytes"]
    if case["op"] == "copy":
        dst = np.full(L, 0xA5, dtype=np.uint8)
        assert red.copy(dst, ins[0], L) == 0
        return dst
    if case["op"] == "sum3":
        dst = np.full(L, 0xA5, dtype=np.uint8)
        assert red.sum3(dst, ins[0], ins[1], L, case["dtype"]) == 0
        return dst
    dst = np.full(L, 0x5A, dtype=np.uint8)
    assert red.sum_n(dst, ins, L, case["dtype"]) == 0
    return dst


@pytest.mark.parametrize("case", CASES, ids=case_id)
def test_port_matches_golden(port, case):
    got = run_case(port, case)
    assert_bytes_match(case["dtype"], got, expected(case), what=case_id(case))


def test_manifest_covers_reference_dtypes():
    seen = {(c["dtype"], c["pinned_by"]) for c in CASES}
    for dt in REFERENCE_DTYPES:
        assert (int(dt), "reference") in seen
    assert (int(DType.BFLOAT16), "port") in seen
    classes = {c["value_class"] for c in CASES}
    assert {"normal", "bits", "special", "uniform100", "identical"} <= classes


@pytest.mark.parametrize("case", [c for c in CASES if c["tag"] == "ladder"], ids=case_id)
def test_known_answer_ladder(case):
    """tests/test_mxnet.py:97-113: identical inputs on every rank, result vs
    tensor*size within 0 (size <= 3 or ints), 1e-4 (< 10), 5e-4 (< 15)."""
    N, dt = case["n_workers"], DType(case["dtype"])
    got = expected(case).view(np.dtype(np.float32 if dt == DType.FLOAT32 else
                                       np.float64 if dt == DType.FLOAT64 else
                                       np.int32 if dt == DType.INT32 else np.int64))
    tensor = inputs(case)[0].view(got.dtype)
    multiplied = tensor * got.dtype.type(N)
    if N <= 3 or dt in (DType.INT32, DType.INT64):
        thr = 0
    elif N < 10:
        thr = 1e-4
    else:
        thr = 5e-4
    # the reference takes max(tensor - multiplied) (signed); we bound |diff|,
    # which is stricter, and scale by magnitude (inputs are U(-100, 100)).
    diff = np.abs(got.astype(np.float64) - multiplied.astype(np.float64))
    assert diff.max() <= thr * max(1.0, np.abs(multiplied).max()) + 0.0


def test_unknown_dtype_is_an_error_not_an_abort(port):
    a = np.zeros(16, np.uint8)
    assert port.sum(a, a.copy(), 16, 7) == -1      # reference: BPS_CHECK abort
    assert port.sum_n(a, [a.copy(), a.copy()], 16, 99) == -1


def test_fp16_body_tail_nan_rules(port):
    # body (i < 8) keeps payloads with dst precedence; tail emits 0x7fff
    d = np.array([0x7E01, 0x3C00, 0x7C01, 0x7C00, 0xFE02, 0x3C00, 0, 0, 0x7E01], np.uint16)
    s = np.array([0x3C00, 0x7E01, 0x3C00, 0xFC00, 0x7E01, 0x3C00, 0, 0, 0x3C00], np.uint16)
    port.sum(d, s, d.nbytes, DType.FLOAT16)
    assert [hex(x) for x in d[:6]] == ["0x7e01", "0x7e01", "0x7e01", "0xfe00", "0xfe02", "0x4000"]
    assert d[8] == 0x7FFF


ref_only = pytest.mark.skipif(not RefReducer.available(),
                              reason="oracle/_ref not built (no /root/reference here)")


@ref_only
@pytest.mark.parametrize("dt", list(REFERENCE_DTYPES), ids=lambda d: DType(d).name)
@pytest.mark.parametrize("threads", [1, 4, 8])
def test_port_vs_reference_live(port, dt, threads):
    ref = RefReducer(nthreads=threads)
    es = elem_size(dt)
    for n_elems, cls, seed in ((40_003, "normal", 77), (8_191, "bits", 78),
                               (5_000, "special", 79), (12_345, "uniform100", 80)):
        if cls == "special" and dt not in (DType.FLOAT16, DType.FLOAT32, DType.FLOAT64):
            continue
        L = n_elems * es + (es - 1 if es > 1 else 0)
        ins = [np.ascontiguousarray(synth.bucket(dt, n_elems + 1, k, cls, seed)).view(np.uint8)[:L].copy()
               for k in range(5)]
        a = ins[0].copy()
        b = ins[0].copy()
        assert ref.sum_n(a, [a] + ins[1:], L, dt) == 0
        assert port.sum_n(b, [b] + ins[1:], L, dt) == 0
        assert_bytes_match(dt, b, a, what=f"{DType(dt).name} {cls} t={threads}")


@ref_only
def test_port_vs_reference_copy_and_sum3(port):
    ref = RefReducer(nthreads=4)
    for L in (0, 3, 4, 5, 1023, 4097):
        src = np.arange(L, dtype=np.uint64).astype(np.uint8)
        x, y = np.zeros(L, np.uint8), np.zeros(L, np.uint8)
        ref.copy(x, src, L)
        port.copy(y, src, L)
        assert np.array_equal(x, y)
    for dt in REFERENCE_DTYPES:
        es = elem_size(dt)
        L = 1001 * es + es - 1
        a = np.ascontiguousarray(synth.bucket(dt, 1002, 0, "normal", 5)).view(np.uint8)[:L].copy()
        b = np.ascontiguousarray(synth.bucket(dt, 1002, 1, "normal", 5)).view(np.uint8)[:L].copy()
        x, y = np.full(L, 7, np.uint8), np.full(L, 7, np.uint8)
        ref.sum3(x, a, b, L, dt)
        port.sum3(y, a, b, L, dt)
        assert_bytes_match(dt, y, x, what=f"sum3 {DType(dt).name}")


SIMD_DTYPES = {int(d) for d in (DType.FLOAT32, DType.FLOAT64, DType.INT32, DType.INT64,
                                DType.INT8, DType.UINT8)}


@pytest.mark.parametrize("case", [c for c in CASES if c["op"] == "fold"
                                  and c["dtype"] in SIMD_DTYPES], ids=case_id)
def test_simd_baseline_form_matches_golden(port, case):
    """bench.py's CPU baseline times bpsr_oracle_sum_simd (the reference's
    `omp parallel for simd` loop shape): same bits as the reference on every
    golden fold; NaN+NaN positions by class, as for the reference itself."""
    ins = inputs(case)
    L = case["len_bytes"]
    dst = np.full(L, 0x5A, dtype=np.uint8)
    assert port.copy(dst, ins[0], L) == 0
    for s in ins[1:]:
        assert port.sum_simd(dst, s, L, case["dtype"]) == 0
    assert_bytes_match(case["dtype"], dst, expected(case), what=case_id(case))


def test_simd_baseline_refuses_half_types(port):
    a = np.zeros(16, np.uint8)
    assert port.sum_simd(a, a.copy(), 16, DType.FLOAT16) == -1
    assert port.sum_simd(a, a.copy(), 16, DType.BFLOAT16) == -1
