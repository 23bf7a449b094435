"""Gradient sets, BytePS partitioning and Prophet block grouping.

Shapes only — no model code.  They define the bucket streams the server
reduces in BASELINE configs 3 and 4:

* ResNet-50 (torchvision layout): 161 parameter tensors, 25,557,032 elements
  (SURVEY.md §8d cfg3).  Reference experiments used MXNet's 157-gradient
  ResNet-50; its Prophet block boundaries (scheduled_queue.h:78-79) are kept
  and the last block is extended from index 156 to 160 for the 161 tensors.
* VGG-16 (torchvision, no BN): 32 tensors, 138,357,544 elements (cfg4).

Partitioning follows byteps/common/operations.cc:99-136 (``PartitionTensor``)
with the bound of global.cc:42,128-135 (4,096,000 B, aligned DOWN to
8*local_size by ``AlignTo``, global.h:191-193); keys follow
operations.cc:237-247 (``(declared_key << 16) + i``).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

DEFAULT_PARTITION_BYTES = 4_096_000           # global.cc:42

# scheduled_queue.h:78-79, MXNet ResNet-50 gradient indices
PROPHET_CHECKPOINTS = (-1, 9, 22, 35, 50, 62, 77, 90, 103, 117, 130, 143, 156)


def resnet50_param_shapes() -> list[tuple[str, tuple[int, ...]]]:
    """torchvision.models.resnet50().named_parameters() order and shapes."""
    out = [("conv1.weight", (64, 3, 7, 7)), ("bn1.weight", (64,)), ("bn1.bias", (64,))]
    inplanes = 64
    for li, (planes, blocks) in enumerate(((64, 3), (128, 4), (256, 6), (512, 3)), start=1):
        for b in range(blocks):
            p = f"layer{li}.{b}."
            out += [(p + "conv1.weight", (planes, inplanes, 1, 1)),
                    (p + "bn1.weight", (planes,)), (p + "bn1.bias", (planes,)),
                    (p + "conv2.weight", (planes, planes, 3, 3)),
                    (p + "bn2.weight", (planes,)), (p + "bn2.bias", (planes,)),
                    (p + "conv3.weight", (planes * 4, planes, 1, 1)),
                    (p + "bn3.weight", (planes * 4,)), (p + "bn3.bias", (planes * 4,))]
            if b == 0:
                out += [(p + "downsample.0.weight", (planes * 4, inplanes, 1, 1)),
                        (p + "downsample.1.weight", (planes * 4,)),
                        (p + "downsample.1.bias", (planes * 4,))]
            inplanes = planes * 4
    out += [("fc.weight", (1000, 2048)), ("fc.bias", (1000,))]
    return out


def vgg16_param_shapes() -> list[tuple[str, tuple[int, ...]]]:
    """torchvision.models.vgg16().named_parameters() order and shapes."""
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M",
           512, 512, 512, "M"]
    out, cin, idx = [], 3, 0
    for v in cfg:
        if v == "M":
            idx += 1
            continue
        out += [(f"features.{idx}.weight", (v, cin, 3, 3)), (f"features.{idx}.bias", (v,))]
        cin = v
        idx += 2  # conv + relu
    for i, (fi, fo) in zip((0, 3, 6), ((25088, 4096), (4096, 4096), (4096, 1000))):
        out += [(f"classifier.{i}.weight", (fo, fi)), (f"classifier.{i}.bias", (fo,))]
    return out


def _numel(shape) -> int:
    n = 1
    for d in shape:
        n *= d
    return n


def resnet50_param_sizes() -> list[int]:
    return [_numel(s) for _, s in resnet50_param_shapes()]


def vgg16_param_sizes() -> list[int]:
    return [_numel(s) for _, s in vgg16_param_shapes()]


def partition_bound(partition_bytes: int = DEFAULT_PARTITION_BYTES, local_size: int = 1) -> int:
    """global.cc:128-135: AlignTo(bytes, 8*local_size) rounds down."""
    a = 8 * local_size
    return partition_bytes // a * a


def _atoi(text: str) -> int:
    """C atoi: leading whitespace, optional sign, digits; 0 if none."""
    t = text.lstrip()
    i = 1 if t[:1] in ("+", "-") else 0
    j = i
    while j < len(t) and t[j].isdigit():
        j += 1
    return int(t[:j]) if j > i else 0


def partition_bytes_from_env(env=None) -> int:
    """BYTEPS_PARTITION_BYTES as global.cc:128-130 reads it (atoi), else the
    4,096,000 default (global.cc:42)."""
    v = (os.environ if env is None else env).get("BYTEPS_PARTITION_BYTES")
    return _atoi(v) if v is not None else DEFAULT_PARTITION_BYTES


def local_size_from_env(env=None) -> int:
    """BYTEPS_LOCAL_SIZE (communicator.cc:71-77, atoi), else 1."""
    v = (os.environ if env is None else env).get("BYTEPS_LOCAL_SIZE")
    return _atoi(v) if v is not None else 1


@dataclass(frozen=True)
class Partition:
    """One key's bucket: bytes [offset, offset+len) of tensor ``tensor``."""
    tensor: int
    part: int
    key: int
    offset: int
    len: int


def partition_tensor(tensor_index: int, nbytes: int, declared_key: int | None = None,
                     bound: int = DEFAULT_PARTITION_BYTES) -> list[Partition]:
    """operations.cc:99-136 (PartitionTensor) + key list of operations.cc:237-247."""
    if nbytes <= 0:
        raise ValueError("init tensor size not larger than 0")   # operations.cc:229
    dk = tensor_index if declared_key is None else declared_key
    out, acc, i = [], 0, 0
    while acc < nbytes:
        ln = min(bound, nbytes - acc)
        out.append(Partition(tensor_index, i, (dk << 16) + i, acc, ln))
        acc += ln
        i += 1
    assert len(out) == (nbytes + bound - 1) // bound          # operations.cc:257-259
    return out


def partition_all(sizes_bytes: list[int], bound: int = DEFAULT_PARTITION_BYTES) -> list[Partition]:
    parts = []
    for t, nb in enumerate(sizes_bytes):
        parts += partition_tensor(t, nb, bound=bound)
    return parts


def prophet_blocks(n_tensors: int, checkpoints=PROPHET_CHECKPOINTS) -> list[list[int]]:
    """Gradient indices of each Prophet block (scheduled_queue.cc:217-243 pushes
    indices from a checkpoint down to the previous one).  The last checkpoint
    is extended to ``n_tensors - 1`` when the model has more gradients than the
    157 the reference hard-codes.  Blocks are listed in release order (the
    backward pass produces the highest index first)."""
    cps = list(checkpoints)
    if cps[-1] < n_tensors - 1:
        cps[-1] = n_tensors - 1
    blocks = [list(range(cps[i] + 1, cps[i + 1] + 1)) for i in range(len(cps) - 1)]
    return blocks[::-1]


def cantor_command(request_type: int, dtype: int) -> int:
    """GetCommandType, common.cc:99-102."""
    m = request_type
    return ((m + dtype) * (m + dtype + 1)) // 2 + dtype


def depair_command(cmd: int) -> tuple[int, int]:
    """DepairDataHandleType, server.h:77-88 -> (request_type, dtype)."""
    import math
    w = int(math.floor((math.sqrt(8 * cmd + 1) - 1) / 2))
    t = (w * w + w) // 2
    y = cmd - t
    x = w - y
    if x < 0 or y < 0:
        raise ValueError(f"bad command {cmd}")
    return x, y
