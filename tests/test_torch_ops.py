"""torch operator surface (prophet_amd/torch_ops.py): registration and schema
on CPU; on the GPU every op against torch's own left fold (bit-exact for
finite IEEE adds, the reference rule of cpu_reducer.cc:86-91) and against the
C-ABI reducer, under torch.compile, and through torch.library.opcheck."""
import pytest

torch = pytest.importorskip("torch")

from prophet_amd import torch_ops  # noqa: E402,F401  (registers torch.ops.bpsr.*)


def test_ops_registered_with_schemas():
    for name in torch_ops.OPS:
        assert hasattr(torch.ops.bpsr, name), name
    s = str(torch.ops.bpsr.sum_n.default._schema)
    assert "Tensor[] srcs" in s and "-> Tensor" in s
    assert "Tensor(a0!) dst" in str(torch.ops.bpsr.sum_.default._schema)   # mutated in place


def test_cpu_tensors_fail_loudly():
    a, b = torch.ones(8), torch.ones(8)
    with pytest.raises(NotImplementedError):
        torch.ops.bpsr.sum_(a, b)
    with pytest.raises(NotImplementedError):
        torch.ops.bpsr.sum_n([a, b])


def _fold(srcs):
    acc = srcs[0].clone()
    for s in srcs[1:]:
        acc.add_(s)
    return acc


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.float16, torch.bfloat16, torch.int32,
                                torch.float64, torch.uint8])
def test_sum_n_equals_torch_fold(dt):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    n = 1_000_003
    if dt.is_floating_point:
        srcs = [torch.randn(n, generator=g, device=dev).to(dt) for _ in range(8)]
    else:
        srcs = [torch.randint(0, 100, (n,), generator=g, device=dev).to(dt) for _ in range(8)]
    out = torch.ops.bpsr.sum_n(srcs)
    assert out.dtype == dt and out.shape == srcs[0].shape
    want = _fold(srcs)
    assert torch.equal(out.view(torch.uint8), want.view(torch.uint8))
    dst = srcs[0].clone()
    torch.ops.bpsr.sum_n_out(dst, [dst] + srcs[1:])       # zero-copy accumulator
    assert torch.equal(dst.view(torch.uint8), want.view(torch.uint8))


@pytest.mark.gpu
def test_inplace_ops_and_copy():
    dev = torch.device("cuda:0")
    a = torch.randn(70_001, device=dev)
    b = torch.randn(70_001, device=dev)
    c = torch.randn(70_001, device=dev)
    d = a.clone()
    torch.ops.bpsr.sum_(d, b)
    assert torch.equal(d, a + b)
    e = torch.empty_like(a)
    torch.ops.bpsr.sum3_(e, b, c)
    assert torch.equal(e, b + c)
    f = torch.empty_like(a)
    torch.ops.bpsr.copy_(f, c)
    assert torch.equal(f, c)
    with pytest.raises(Exception):
        torch.ops.bpsr.sum_(d, b[:-1])                      # size mismatch


@pytest.mark.gpu
def test_ops_order_with_side_stream():
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream()
    x = [torch.randn(1 << 20, device=dev) for _ in range(4)]
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        y = [t * 2 for t in x]                              # produced on s
        out = torch.ops.bpsr.sum_n(y)                       # must run after them, on s
    s.synchronize()
    assert torch.equal(out, _fold([t * 2 for t in x]))


@pytest.mark.gpu
def test_torch_compile_and_opcheck():
    dev = torch.device("cuda:0")
    srcs = [torch.randn(4099, device=dev) for _ in range(8)]

    def f(xs):
        return torch.ops.bpsr.sum_n(xs) * 1.0

    got = torch.compile(f, fullgraph=True)(srcs)
    assert torch.equal(got, _fold(srcs))
    torch.library.opcheck(torch.ops.bpsr.sum_n.default, (srcs[:3], 0),
                          test_utils=("test_schema", "test_faketensor"))
