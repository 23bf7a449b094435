"""GPU parity: the HIP path (through the C ABI) against the reference's golden
vectors and the CPU oracle, on a real MI355X.

Bar: bit-exact for every dtype in reference mode (fp32/fp64 NaN+NaN payloads
compared by class against the reference fixtures, whose choice is
schedule-dependent, but bit-exact against the oracle restatement); ACCUM_F32
mode within 1 ulp of the exactly rounded sum.
"""
import os

import numpy as np
import pytest

from golden_util import assert_bytes_match, case_id, expected, inputs, manifest
from oracle.oracle import PortReducer
from prophet_amd import synth
from prophet_amd.dtypes import ALL_DTYPES, DType, elem_size

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

CASES = manifest()


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def red(dev):
    from prophet_amd.reducer import GpuReducer
    return GpuReducer(device=0)


@pytest.fixture(scope="module")
def port():
    return PortReducer(nthreads=8)


def to_dev(a: np.ndarray, dev, pad: int = 0, offset: int = 0):
    """Device copy of host bytes at byte `offset` inside a larger buffer."""
    buf = torch.full((len(a) + offset + pad + 16,), 0xEE, dtype=torch.uint8, device=dev)
    if len(a):
        buf[offset: offset + len(a)] = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return buf, buf[offset: offset + len(a)] if len(a) else buf[offset:offset]


def ptr(buf, offset=0):
    return buf.data_ptr() + offset


def run_gpu(red, dev, case, ins, offset=0):
    L = case["len_bytes"]
    if case["op"] == "copy":
        dbuf, _ = to_dev(np.full(L, 0xA5, np.uint8), dev, offset=offset)
        sbuf, _ = to_dev(ins[0], dev, offset=offset)
        red.copy(ptr(dbuf, offset), ptr(sbuf, offset), L)
    elif case["op"] == "sum3":
        dbuf, _ = to_dev(np.full(L, 0xA5, np.uint8), dev, offset=offset)
        a, _ = to_dev(ins[0], dev, offset=offset)
        b, _ = to_dev(ins[1], dev, offset=offset)
        red.sum3(ptr(dbuf, offset), ptr(a, offset), ptr(b, offset), L, case["dtype"])
    else:
        bufs = [to_dev(x, dev, offset=offset)[0] for x in ins]
        dbuf, _ = to_dev(np.full(L, 0x5A, np.uint8), dev, offset=offset)
        red.sum_n(ptr(dbuf, offset), [ptr(b, offset) for b in bufs], L, case["dtype"])
    torch.cuda.synchronize()
    return dbuf[offset: offset + L].cpu().numpy()


@pytest.mark.parametrize("case", CASES, ids=case_id)
def test_golden(red, dev, port, case):
    ins = inputs(case)
    got = run_gpu(red, dev, case, ins)
    assert_bytes_match(case["dtype"], got, expected(case), what=case_id(case))


@pytest.mark.parametrize("case", [c for c in CASES if c["op"] == "fold" and
                                  c["value_class"] in ("special", "bits")], ids=case_id)
def test_golden_vs_port_bit_exact(red, dev, port, case):
    """Against the restatement the NaN rule is deterministic: every bit must match."""
    ins = inputs(case)
    got = run_gpu(red, dev, case, ins)
    L = case["len_bytes"]
    want = np.zeros(L, np.uint8)
    port.sum_n(want, ins, L, case["dtype"])
    assert_bytes_match(case["dtype"], got, want, nan_class_f32_f64=False, what=case_id(case))


@pytest.mark.parametrize("dt", list(ALL_DTYPES), ids=lambda d: DType(d).name)
@pytest.mark.parametrize("offset", [0, 2, 4, 8, 12])
def test_misaligned_coaligned(red, dev, port, dt, offset):
    """Sub-bucket views (e.g. a shard inside a partition) start anywhere."""
    es = elem_size(dt)
    if offset % es:
        pytest.skip("not element aligned")
    n = 4099 + 13
    L = n * es
    ins = [np.ascontiguousarray(synth.bucket(dt, n, k, "special" if dt in
           (DType.FLOAT16, DType.FLOAT32) else "normal", 321)).view(np.uint8) for k in range(3)]
    case = {"op": "fold", "len_bytes": L, "dtype": int(dt)}
    got = run_gpu(red, dev, case, ins, offset=offset)
    want = np.zeros(L, np.uint8)
    port.sum_n(want, ins, L, dt)
    assert_bytes_match(dt, got, want, nan_class_f32_f64=False, what=f"off={offset}")


@pytest.mark.parametrize("dt", [DType.FLOAT32, DType.FLOAT16, DType.INT64, DType.UINT8],
                         ids=lambda d: DType(d).name)
def test_not_coaligned_and_unaligned(red, dev, port, dt):
    """Operands with different (or no) element alignment take the element path."""
    es = elem_size(dt)
    n = 1000 + 7
    L = n * es
    ins = [np.ascontiguousarray(synth.bucket(dt, n, k, "normal", 55)).view(np.uint8)
           for k in range(4)]
    offs = [0, es, 3 * es, 1]  # last source not even element-aligned
    bufs = [to_dev(x, dev, offset=o)[0] for x, o in zip(ins, offs)]
    dbuf, _ = to_dev(np.zeros(L, np.uint8), dev, offset=5)
    red.sum_n(ptr(dbuf, 5), [ptr(b, o) for b, o in zip(bufs, offs)], L, dt)
    torch.cuda.synchronize()
    want = np.zeros(L, np.uint8)
    port.sum_n(want, ins, L, dt)
    assert_bytes_match(dt, dbuf[5:5 + L].cpu().numpy(), want, nan_class_f32_f64=False)


@pytest.mark.parametrize("dt", list(ALL_DTYPES), ids=lambda d: DType(d).name)
def test_engine_pattern_equals_fused(red, dev, port, dt):
    """N-1 in-place sum() calls (server.cc:127-130 engine loop) == one sum_n()
    == the oracle's fold of the same inputs."""
    es = elem_size(dt)
    n = 65536 + 5
    L = n * es
    host = [np.ascontiguousarray(synth.bucket(dt, n, k, "normal", 9)).view(np.uint8)
            for k in range(8)]
    ins = [torch.from_numpy(h).to(dev) for h in host]
    acc = ins[0].clone()
    for s in ins[1:]:
        red.sum(acc, s, L, dt)
    fused = torch.empty_like(acc)
    red.sum_n(fused, ins, L, dt)
    inplace = ins[0].clone()
    red.sum_n(inplace, [inplace] + ins[1:], L, dt)
    torch.cuda.synchronize()
    assert torch.equal(acc, fused)
    assert torch.equal(acc, inplace)
    want = np.zeros(L, np.uint8)
    port.sum_n(want, host, L, dt)
    assert_bytes_match(dt, acc.cpu().numpy(), want, nan_class_f32_f64=False)


def test_more_than_32_sources_chains_left_fold(red, dev, port):
    dt, n = DType.FLOAT16, 3001
    ins = [np.ascontiguousarray(synth.bucket(dt, n, k, "normal", 4)).view(np.uint8)
           for k in range(40)]
    bufs = [torch.from_numpy(x).to(dev) for x in ins]
    out = torch.empty_like(bufs[0])
    red.sum_n(out, bufs, n * 2, dt)
    torch.cuda.synchronize()
    want = np.zeros(n * 2, np.uint8)
    port.sum_n(want, ins, n * 2, dt)
    assert_bytes_match(dt, out.cpu().numpy(), want, nan_class_f32_f64=False)


@pytest.mark.parametrize("dt", [DType.FLOAT32, DType.FLOAT16, DType.BFLOAT16, DType.INT32],
                         ids=lambda d: DType(d).name)
def test_batched_block_matches_oracle(red, dev, port, dt):
    """One Prophet block (many buckets of ResNet-like sizes, 128 B .. 1 MiB) in one launch."""
    from prophet_amd.buckets import resnet50_param_sizes
    es = elem_size(dt)
    sizes = resnet50_param_sizes()[:40]          # ragged, many < 1 KiB
    N = 8
    buckets, wants = [], []
    keep = []
    for i, ne in enumerate(sizes):
        L = ne * es
        ins = [np.ascontiguousarray(synth.bucket(dt, ne, k, "normal", 100 + i)).view(np.uint8)
               for k in range(N)]
        srcs = [torch.from_numpy(x).to(dev) for x in ins]
        dst = srcs[0] if i % 2 == 0 else torch.empty_like(srcs[0])   # alias or not
        keep += srcs + [dst]
        buckets.append((dst, srcs, L))
        w = np.zeros(L, np.uint8)
        port.sum_n(w, ins, L, dt)
        wants.append(w)
    red.sum_batched(buckets, dt)
    torch.cuda.synchronize()
    for (dst, _, L), w in zip(buckets, wants):
        assert_bytes_match(dt, dst.cpu().numpy(), w, nan_class_f32_f64=False)


@pytest.mark.parametrize("dt", [DType.FLOAT32, DType.FLOAT16, DType.FLOAT64, DType.INT8],
                         ids=lambda d: DType(d).name)
@pytest.mark.parametrize("plan", [False, True], ids=["one_off", "plan"])
def test_batched_ragged_mixed_table(red, dev, port, dt, plan):
    """One table mixing every tile kind: source counts 1..32 (register path
    n <= 8 and memory path n > 8), co-aligned offsets (head + tail element
    tiles), operands that are not co-aligned (element tiles only, several
    parts), NaN/Inf/subnormal inputs (exact replay through the records'
    advanced pointers), trailing bytes, and empty buckets."""
    es = elem_size(dt)
    spec = [  # (n_elems, n_sources, offsets of dst + sources or None, class)
        (100_000, 8, None, "special"), (4099, 9, None, "normal"), (1, 1, None, "normal"),
        (70_001, 32, None, "bits"), (0, 8, None, "normal"), (3 * 1024 + 5, 2, [4, 4, 4], "normal"),
        (50_000, 3, [0, es, 2 * es, 1], "normal"), (257, 12, None, "special"),
        (300_000, 5, [2, 6, 10, 14, 2, 6], "normal"), (9, 8, None, "bits"),
    ]
    buckets, wants, views = [], [], []
    for i, (ne, N, offs, cls) in enumerate(spec):
        L = ne * es + (3 if i == 3 else 0)          # bucket 3: trailing bytes
        ins = [np.ascontiguousarray(synth.bucket(dt, ne, k, cls, 300 + i)).view(np.uint8)
               for k in range(N)]
        if i == 3:
            ins = [np.concatenate([x, np.array([k, 7, 9], np.uint8)]) for k, x in enumerate(ins)]
        offs = offs or [0] * (N + 1)
        offs = (offs + [offs[-1]] * (N + 1))[:N + 1]
        bufs = [to_dev(x, dev, offset=o)[0] for x, o in zip(ins, offs[1:])]
        dbuf, _ = to_dev(np.full(L, 0x5A, np.uint8), dev, offset=offs[0])
        buckets.append((ptr(dbuf, offs[0]), [ptr(b, o) for b, o in zip(bufs, offs[1:])], L))
        views.append((dbuf, offs[0], L, bufs))
        w = np.full(L, 0x5A, np.uint8)
        if L:
            port.sum_n(w, ins, L, dt)
        wants.append(w)
    if plan:
        p = red.make_plan(buckets, dt)
        p.launch()
        torch.cuda.synchronize()
        p.close()
    else:
        red.sum_batched(buckets, dt)
        torch.cuda.synchronize()
    for (dbuf, o, L, _), w in zip(views, wants):
        assert_bytes_match(dt, dbuf[o:o + L].cpu().numpy(), w, nan_class_f32_f64=False)


def test_batched_large_table_vpt4_equals_torch(red, dev):
    """A block above the small-table threshold (1024-vector tiles): 6 x 6 MiB
    fp32 buckets, 8 sources, against torch's own left fold (bit-exact for
    finite IEEE adds), ragged lengths."""
    g = torch.Generator(device=dev).manual_seed(7)
    N = 8
    buckets, checks = [], []
    for i in range(6):
        ne = (6 << 20) // 4 + 3 * i
        srcs = [torch.randn(ne, device=dev, generator=g) for _ in range(N)]
        dst = torch.empty_like(srcs[0])
        buckets.append((dst, srcs, ne * 4))
        checks.append((dst, srcs))
    red.sum_batched(buckets, DType.FLOAT32)
    torch.cuda.synchronize()
    for dst, srcs in checks:
        want = srcs[0].clone()
        for s in srcs[1:]:
            want.add_(s)
        assert torch.equal(dst.view(torch.int32), want.view(torch.int32))


_PREFETCH_SCRIPT = r"""
import hashlib, sys, torch
sys.path.insert(0, {root!r})
from prophet_amd.reducer import GpuReducer
from prophet_amd.dtypes import DType
red, dev = GpuReducer(device=0), torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(11)
buckets = []
for i in range(5):
    ne = (3 << 20) // 2 + 7 * i
    srcs = [torch.randn(ne, device=dev, generator=g).half() for _ in range(8)]
    buckets.append((torch.empty_like(srcs[0]), srcs, ne * 2))
red.sum_batched(buckets, DType.FLOAT16)
plan = red.make_plan(buckets, DType.FLOAT16)
outs = [b[0].clone() for b in buckets]
for b in buckets:
    b[0].zero_()
plan.launch()
torch.cuda.synchronize()
h = hashlib.sha256()
for o, b in zip(outs, buckets):
    assert torch.equal(o, b[0])
    h.update(o.view(torch.uint8).cpu().numpy().tobytes())
print(h.hexdigest())
"""


def test_record_prefetch_knob_changes_no_bits():
    """BPSR_REC_PREFETCH (the tile-record L2 prefetch of batched launches,
    plans and block queues) is read once per process: the same batched fold
    and plan (fp16, 5 ragged buckets, > 256 tiles so the prefetch reaches
    records) in two child processes, prefetch off and at its default, give
    the same bytes."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    digests = []
    for pf in ("0", None):
        env = dict(os.environ)
        env.pop("BPSR_REC_PREFETCH", None)
        if pf is not None:
            env["BPSR_REC_PREFETCH"] = pf
        r = subprocess.run([sys.executable, "-c", _PREFETCH_SCRIPT.format(root=root)], env=env,
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        digests.append(r.stdout.strip().splitlines()[-1])
    assert digests[0] == digests[1]


@pytest.mark.parametrize("mib", [95, 97])
@pytest.mark.parametrize("batched", [False, True], ids=["fold", "batched"])
def test_store_policy_threshold_equals_torch(red, dev, mib, batched):
    """Both sides of the write-through threshold (96 MiB per source,
    bpsr_internal.h cache_pol): below it the kernels store with sc1, above
    it with nt — same bytes either way.  3 fp32 sources, ragged lengths (a
    partial last tile and element work), single fold and a 2-bucket table."""
    g = torch.Generator(device=dev).manual_seed(mib)
    N = 3
    parts = [((mib << 20) // 4) + 5] if not batched else [((mib << 20) // 8) + 3, ((mib << 20) // 8) + 9]
    buckets, checks = [], []
    for ne in parts:
        srcs = [torch.randn(ne, device=dev, generator=g) for _ in range(N)]
        dst = torch.empty_like(srcs[0])
        buckets.append((dst, srcs, ne * 4))
        checks.append((dst, srcs))
    if batched:
        red.sum_batched(buckets, DType.FLOAT32)
    else:
        dst, srcs, nb = buckets[0]
        red.sum_n(dst, srcs, nb, DType.FLOAT32)
    torch.cuda.synchronize()
    for dst, srcs in checks:
        want = srcs[0].clone()
        for s in srcs[1:]:
            want.add_(s)
        assert torch.equal(dst.view(torch.int32), want.view(torch.int32))


@pytest.mark.parametrize("nbytes", [69_178_772, (80 << 20) + 6, 95 << 20])
def test_half_tile_band_equals_torch(red, dev, nbytes):
    """8-way folds of 64-96 MiB per source run 4-KiB tiles at 2 workgroups
    per CU (bpsr_kernels_impl.h launch_fold_op); config 4's G = 8 shard and
    ragged sizes, against torch's left fold."""
    g = torch.Generator(device=dev).manual_seed(nbytes % 1000)
    ne = nbytes // 4
    # every operand holds the call's bytes (len % 4 trailing bytes included:
    # GpuReducer refuses a length past a tensor's end)
    srcs = [torch.randn((nbytes + 3) // 4, device=dev, generator=g) for _ in range(8)]
    dst = torch.empty_like(srcs[0])
    red.sum_n(dst, srcs, nbytes, DType.FLOAT32)
    want = srcs[0].clone()
    for x in srcs[1:]:
        want.add_(x)
    torch.cuda.synchronize()
    assert torch.equal(dst.view(torch.int32)[:ne], want.view(torch.int32)[:ne])
    # the trailing bytes come from the first arrival (server.cc:216-218)
    tb = nbytes - 4 * ne
    assert torch.equal(dst.view(torch.uint8)[4 * ne:4 * ne + tb],
                       srcs[0].view(torch.uint8)[4 * ne:4 * ne + tb])


@pytest.mark.parametrize("dt", [DType.FLOAT16, DType.BFLOAT16], ids=lambda d: DType(d).name)
def test_accum_f32_mode_within_one_ulp(red, dev, dt):
    from prophet_amd.reducer import MODE_ACCUM_F32
    n, N = 200_003, 16
    ins = [torch.from_numpy(np.ascontiguousarray(synth.bucket(dt, n, k, "normal", 3))
                            .view(np.uint8)).to(dev) for k in range(N)]
    out = torch.empty_like(ins[0])
    red.sum_n(out, ins, n * 2, dt, mode=MODE_ACCUM_F32)
    td = torch.float16 if dt == DType.FLOAT16 else torch.bfloat16
    exact = sum(x.view(td).double() for x in ins)
    rounded = exact.to(td)
    got = out.view(td)
    # ulp of the correctly rounded result (10 / 7 stored mantissa bits)
    mbits, emin = (10, -14) if dt == DType.FLOAT16 else (7, -126)
    mag = rounded.double().abs().clamp_min(2.0 ** emin)
    ulp = torch.pow(2.0, torch.floor(torch.log2(mag)) - mbits)
    err = (got.double() - exact).abs()
    assert bool((err <= 1.0 * ulp + 1e-30).all())


def test_full_size_config2_properties(red, dev):
    """BASELINE config 2 at full size: 8 x 256 MiB fp32.  The fused fold must
    equal torch's own pairwise left fold bit for bit (IEEE fp32 adds, finite
    inputs), and a sampled window must match the oracle."""
    n = (256 << 20) // 4
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234)
    ins = [torch.randn(n, device=dev, generator=gen) for _ in range(8)]
    out = torch.empty_like(ins[0])
    red.sum_n(out, ins, n * 4, DType.FLOAT32)
    ref = ins[0].clone()
    for s in ins[1:]:
        ref.add_(s)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    # sampled oracle window
    port = PortReducer(nthreads=8)
    lo = 12_345_678
    win = [x[lo: lo + 1_000_003].cpu().numpy().view(np.uint8) for x in ins]
    want = np.zeros_like(win[0])
    port.sum_n(want, win, want.nbytes, DType.FLOAT32)
    assert np.array_equal(out[lo: lo + 1_000_003].cpu().numpy().view(np.uint8), want)


def test_full_size_fp16_left_fold_equals_torch(red, dev):
    """fp16 at 98 MiB: per-step RNE left fold == torch half add chain."""
    n = 51_114_064  # ResNet-50 element count
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    ins = [torch.randn(n, device=dev, generator=gen).half() for _ in range(8)]
    out = torch.empty_like(ins[0])
    red.sum_n(out, ins, n * 2, DType.FLOAT16)
    ref = ins[0].clone()
    for s in ins[1:]:
        ref.add_(s)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))


def test_stream_ordering_on_side_stream(red, dev):
    s = torch.cuda.Stream()
    n = 1 << 22
    a = torch.ones(n, device=dev)
    b = torch.full((n,), 2.0, device=dev)
    with torch.cuda.stream(s):
        a.mul_(3.0)                       # must complete before the reduce
        red.sum(a, b, n * 4, DType.FLOAT32)  # picks up torch's current stream = s
        a.add_(1.0)
    s.synchronize()
    assert bool((a == 6.0).all())


def test_bad_dtype_raises(red, dev):
    from prophet_amd.reducer import EDTYPE, ReduceError
    a = torch.zeros(64, dtype=torch.uint8, device=dev)
    with pytest.raises(ReduceError) as e:
        red.sum(a, a.clone(), 64, 10)
    assert e.value.code == EDTYPE


def test_plan_launch_and_graph_replay(red, dev, port):
    """A block plan (table uploaded once) equals the oracle, also when its
    launch is captured into a hipGraph and replayed with new data in place."""
    from prophet_amd.buckets import resnet50_param_sizes
    dt = DType.FLOAT16
    sizes = resnet50_param_sizes()[100:130]
    N = 8
    bufs, buckets = [], []
    for i, ne in enumerate(sizes):
        srcs = [torch.empty(ne * 2, dtype=torch.uint8, device=dev) for _ in range(N)]
        dst = torch.empty_like(srcs[0])
        bufs.append((dst, srcs))
        buckets.append((dst, srcs, ne * 2))
    plan = red.make_plan(buckets, dt)

    def fill(seed):
        wants = []
        for i, ((dst, srcs), ne) in enumerate(zip(bufs, sizes)):
            ins = [np.ascontiguousarray(synth.bucket(dt, ne, k, "normal", seed + i)).view(np.uint8)
                   for k in range(N)]
            for s, x in zip(srcs, ins):
                s.copy_(torch.from_numpy(x))
            w = np.zeros(ne * 2, np.uint8)
            port.sum_n(w, ins, ne * 2, dt)
            wants.append(w)
        return wants

    wants = fill(10)
    plan.launch()
    torch.cuda.synchronize()
    for (dst, _), w in zip(bufs, wants):
        assert np.array_equal(dst.cpu().numpy(), w)
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        plan.launch(side)
    wants = fill(20)
    g.replay()
    torch.cuda.synchronize()
    for (dst, _), w in zip(bufs, wants):
        assert np.array_equal(dst.cpu().numpy(), w)
    plan.close()


@pytest.mark.parametrize("L", [1, 15, 16, 17, 4095, 65_539, 3 << 20, (64 << 20) + 5])
@pytest.mark.parametrize("offs", [(0, 0), (3, 3), (5, 9)], ids=lambda o: f"d{o[0]}s{o[1]}")
def test_copy_sizes_offsets_guards(red, dev, L, offs):
    """CpuReducer::copy (cpu_reducer.cc:209-220): every byte of len, nothing
    outside it; co-aligned, misaligned and non-co-aligned operands, from the
    element path through short launches to long (residency-capped) ones."""
    doff, soff = offs
    gen = torch.Generator(device=dev)
    gen.manual_seed(L + doff)
    src = torch.randint(0, 256, (L + soff + 64,), dtype=torch.uint8, device=dev, generator=gen)
    dst = torch.full((L + doff + 64,), 0xEE, dtype=torch.uint8, device=dev)
    red.copy(dst.data_ptr() + doff, src.data_ptr() + soff, L)
    torch.cuda.synchronize()
    assert torch.equal(dst[doff:doff + L], src[soff:soff + L])
    assert bool((dst[:doff] == 0xEE).all()) and bool((dst[doff + L:] == 0xEE).all())


@pytest.mark.parametrize("n", [2, 3, 4, 5])
@pytest.mark.parametrize("mib", [1, 24, 96])
def test_small_source_counts_equal_torch(red, dev, n, mib):
    """n <= 4 sources run 2 workgroups/CU with 16 KiB tiles (bpsr_api.cpp
    tuning_for_n): fused fold, in-place 2-op sum and 3-op sum equal torch's
    own fp32 left fold bit for bit at short and long launch sizes (odd element
    count: partial last tile + element tail)."""
    ne = (mib << 20) // 4 + 7
    gen = torch.Generator(device=dev)
    gen.manual_seed(100 * n + mib)
    ins = [torch.randn(ne, device=dev, generator=gen) for _ in range(n)]
    ref = ins[0].clone()
    for s in ins[1:]:
        ref.add_(s)
    out = torch.empty_like(ins[0])
    red.sum_n(out, ins, ne * 4, DType.FLOAT32)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    if n == 2:
        acc = ins[0].clone()
        red.sum(acc, ins[1], ne * 4, DType.FLOAT32)        # dst += src, in place
        o3 = torch.empty_like(acc)
        red.sum3(o3, ins[0], ins[1], ne * 4, DType.FLOAT32)
        torch.cuda.synchronize()
        assert torch.equal(acc.view(torch.int32), ref.view(torch.int32))
        assert torch.equal(o3.view(torch.int32), ref.view(torch.int32))


@pytest.mark.parametrize("dt", [DType.BFLOAT16, DType.FLOAT16], ids=lambda d: DType(d).name)
def test_full_size_16bit_accum_mode_within_one_ulp(red, dev, dt):
    """fp32-accumulate mode at 64 MiB per source through the hardware
    conversions of the fast path: within 1 ulp of the exactly rounded sum."""
    n = 32 << 20
    tdt = torch.bfloat16 if dt == DType.BFLOAT16 else torch.float16
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(dt))
    ins = [torch.randn(n, device=dev, generator=gen).to(tdt) for _ in range(8)]
    out = torch.empty_like(ins[0])
    red.sum_n(out, ins, n * 2, dt, mode=1)
    exact = ins[0].double()
    for s in ins[1:]:
        exact += s.double()
    torch.cuda.synchronize()
    mbits = 7 if dt == DType.BFLOAT16 else 10
    mag = exact.abs().clamp_min(2.0 ** -14)
    ulp = torch.pow(2.0, torch.floor(torch.log2(mag)) - mbits)
    assert bool(((out.double() - exact).abs() <= ulp + 1e-30).all())


def test_full_size_bf16_left_fold_equals_torch(red, dev):
    """bf16 (build-defined: fp32 add, RNE to bf16 after every add) at 128 MiB
    per source through v_cvt_pk_bf16_f32 == torch's bf16 add chain (which
    also computes in fp32 and rounds to nearest-even)."""
    n = 64 << 20
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    ins = [torch.randn(n, device=dev, generator=gen).bfloat16() for _ in range(8)]
    out = torch.empty_like(ins[0])
    red.sum_n(out, ins, n * 2, DType.BFLOAT16)
    ref = ins[0].clone()
    for s in ins[1:]:
        ref.add_(s)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))


@pytest.mark.parametrize("dt,tdt", [(DType.UINT8, torch.uint8), (DType.FLOAT32, torch.float32)],
                         ids=["u8_4GiB", "f32_2G_elems"])
def test_beyond_32bit_lengths(red, dev, dt, tdt):
    """`len` is size_t in the reference (cpu_reducer.h:49): a bucket past 4 GiB
    (u8: > 2^32 elements) and one past 2^31 fp32 elements (8 GiB) fold
    correctly everywhere — the element head/tail at the far end, 64-bit tile
    offsets and the ragged last tile — checked against torch's own fold at the
    start, around the 2^31/2^32 boundaries and at the end; the bytes past
    `len` stay untouched (guard)."""
    es = elem_size(dt)
    n = ((1 << 32) + 4099) if dt == DType.UINT8 else ((1 << 31) + 1027)
    L = n * es
    g = torch.Generator(device=dev).manual_seed(99)
    if dt == DType.UINT8:
        ins = [torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev, generator=g)
               for _ in range(2)]
    else:
        ins = [torch.randn(n, device=dev, generator=g) for _ in range(2)]
    out = torch.full((n + 64,), 7, dtype=tdt, device=dev)
    red.sum_n(out, ins, L, dt)
    torch.cuda.synchronize()
    for lo in (0, (1 << 31) - 5000, min(n - 9000, (1 << 32) - 5000), n - 9000):
        hi = min(lo + 9000, n)
        want = ins[0][lo:hi] + ins[1][lo:hi]
        assert torch.equal(out[lo:hi].view(torch.uint8), want.view(torch.uint8)), lo
    assert bool((out[n:] == 7).all())
    del ins, out
    torch.cuda.empty_cache()
