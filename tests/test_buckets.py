"""Host-side bucket logic: gradient sets, BytePS partitioning and keys
(operations.cc:99-136, 219-259; global.cc:42,128-135), Prophet blocks
(scheduled_queue.h:78-79, scheduled_queue.cc:217-243), Cantor command words
(common.cc:99-102, server.h:77-88)."""
import pytest

from prophet_amd.buckets import (DEFAULT_PARTITION_BYTES, PROPHET_CHECKPOINTS, cantor_command,
                                 depair_command, partition_all, partition_bound,
                                 partition_tensor, prophet_blocks, resnet50_param_shapes,
                                 resnet50_param_sizes, vgg16_param_sizes)
from prophet_amd.dtypes import REFERENCE_DTYPES


def test_gradient_sets_match_survey():
    r = resnet50_param_sizes()
    assert len(r) == 161 and sum(r) == 25_557_032
    assert max(r) * 2 == 4_718_592 and min(r) * 2 == 128
    assert sum(1 for n in r if n * 2 < 1024) == 62
    v = vgg16_param_sizes()
    assert len(v) == 32 and sum(v) == 138_357_544
    assert max(v) * 4 == 411_041_792
    names = [n for n, _ in resnet50_param_shapes()]
    assert names[0] == "conv1.weight" and names[-1] == "fc.bias"


def test_partition_bound_aligns_down():
    # global.cc:128-135 AlignTo(bytes, 8*local_size) = floor
    assert partition_bound(4_096_000, 1) == 4_096_000
    assert partition_bound(4_096_000, 3) == 4_096_000 // 24 * 24
    assert partition_bound(1000, 8) == 960


def test_partition_tensor_offsets_lengths_keys():
    parts = partition_tensor(5, 10_000_001, bound=4_096_000)
    assert [p.len for p in parts] == [4_096_000, 4_096_000, 1_808_001]
    assert [p.offset for p in parts] == [0, 4_096_000, 8_192_000]
    assert [p.key for p in parts] == [(5 << 16) + i for i in range(3)]   # operations.cc:237-247
    with pytest.raises(ValueError):
        partition_tensor(0, 0)                                          # operations.cc:229


def test_partition_counts_for_the_configs():
    assert len(partition_all([n * 2 for n in resnet50_param_sizes()])) == 165
    assert len(partition_all([n * 4 for n in vgg16_param_sizes()])) == 162
    assert DEFAULT_PARTITION_BYTES == 4_096_000


def test_prophet_blocks_reference_boundaries():
    # the reference's own 157-gradient model: 12 blocks between the checkpoints
    b157 = prophet_blocks(157)
    assert [len(b) for b in b157][::-1] == [10, 13, 13, 15, 12, 15, 13, 13, 14, 13, 13, 13]
    assert sorted(i for b in b157 for i in b) == list(range(157))
    assert b157[0][-1] == 156                   # released first: the last layers
    # 161 torchvision tensors: last block extended 156 -> 160
    b161 = prophet_blocks(161)
    assert sorted(i for b in b161 for i in b) == list(range(161))
    assert len(b161[0]) == 17 and PROPHET_CHECKPOINTS[-1] == 156


@pytest.mark.parametrize("req", [0, 1, 2])
def test_cantor_command_roundtrip(req):
    for dt in list(REFERENCE_DTYPES) + [11]:
        cmd = cantor_command(req, int(dt))
        assert depair_command(cmd) == (req, int(dt))
    assert cantor_command(0, 0) == 0 and cantor_command(0, 2) == 5   # d(d+1)/2 + d


def test_arena_skew_classes():
    """prophet_amd/arena.py: the measured skew classes (profiles/
    r06s09_s10_arena_skew.jsonl) — 16 KiB up to the headline's 256 MiB
    bucket, 2 MiB + 16 KiB beyond it — and the stride they give."""
    import torch
    from prophet_amd.arena import DEFAULT_SKEW, LARGE_SKEW, BucketArena, default_skew
    assert default_skew(256 << 20) == DEFAULT_SKEW == 16 << 10
    assert default_skew((256 << 20) + (64 << 10)) == DEFAULT_SKEW
    assert default_skew(553_430_176) == LARGE_SKEW == (2 << 20) + (16 << 10)
    assert default_skew(1 << 30) == LARGE_SKEW
    a = BucketArena(3, 5000, torch.device("cpu"))          # small: 4 KiB rounding
    assert a.stride == 8192 + DEFAULT_SKEW
    assert [s.numel() for s in a.slots()] == [5000] * 3
    assert a.slot(2).data_ptr() - a.slot(0).data_ptr() == 2 * a.stride
