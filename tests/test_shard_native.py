"""The shard C ABI (include/bpsr/shard.h) on a CPU host: ownership math,
GetReduceRootByKey, BYTEPS_REDUCE_ROOTS parsing, in-process communicator
objects and every argument check (all validated before any HIP call)."""
import ctypes

import pytest

from prophet_amd import reducer
from prophet_amd.dtypes import DType
from prophet_amd.shard import (ShardComm, ShardedReducer, _lib, owner_range_native,
                               owner_ranges, reduce_root_of, reduce_roots_from_env)


@pytest.mark.parametrize("elems", [0, 1, 2, 7, 8, 9, 10007, 138_357_544, 2**33 + 5])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8])
def test_owner_range_matches_reduce_scatter_split(elems, world):
    """core_loops.cc:210-211: per = len / size; tail to the last rank."""
    want = owner_ranges(elems, world)
    got = [owner_range_native(elems, world, r) for r in range(world)]
    assert got == want
    assert got[0][0] == 0 and got[-1][1] == elems
    assert all(a[1] == b[0] for a, b in zip(got, got[1:]))


def test_owner_range_argument_errors():
    L = _lib()
    lo, hi = ctypes.c_size_t(), ctypes.c_size_t()
    for world, rank in ((0, 0), (2, 2), (2, -1)):
        assert L.byteps_shard_owner_range(10, world, rank, ctypes.byref(lo),
                                          ctypes.byref(hi)) == reducer.EARGS
    assert L.byteps_shard_owner_range(10, 2, 0, None, ctypes.byref(hi)) == reducer.EARGS


def _djb2(key: int) -> int:
    """Hash_DJB2 (global.cc:507-516) over std::to_string(key), uint64 wrap."""
    h = 5381
    for ch in str(key).encode():
        h = ((h << 5) + h + ch) & (2**64 - 1)
    return h


@pytest.mark.parametrize("roots", [[0], [1, 3], [0, 1, 2, 3], [7, 2, 5]])
def test_reduce_root_of_key(roots):
    """GetReduceRootByKey (global.h:107-108): roots[djb2(key) % len(roots)],
    over the reference's key format (declared_key << 16) + partition."""
    keys = [0, 1, 9, 10, 65535, 65536] + [(dk << 16) + i for dk in (1, 2, 160, 4097)
                                         for i in (0, 1, 5)] + [2**63 + 12345]
    for k in keys:
        assert reduce_root_of(k, roots) == roots[_djb2(k) % len(roots)], k


def test_reduce_root_of_errors():
    assert _lib().byteps_shard_reduce_root_of(1, None, 0) == reducer.EARGS


@pytest.mark.parametrize("text,want", [
    (None, []), ("", []), ("0", [0]), ("0,1,2,3", [0, 1, 2, 3]), ("3 1", [3, 1]),
    ("0, 1", [0, 1]),      # `>> i` skips the space after the ignored ','
    ("0, 1 ,2", [0, 1]),   # ' ' then ',' : the ',' is not a number, parsing stops
    ("0,,1", [0]), ("2,x,3", [2]), ("x", []), ("-1,4", [-1, 4]),
])
def test_reduce_roots_env_parse(text, want):
    env = {} if text is None else {"BYTEPS_REDUCE_ROOTS": text}
    assert reduce_roots_from_env(env) == want


def test_local_group_info_without_gpu():
    comms = ShardComm.local_group([0, 0, 0])
    assert [(c.world, c.rank, c.device) for c in comms] == [(3, 0, 0), (3, 1, 0), (3, 2, 0)]
    sr = ShardedReducer(10007, comm=comms[2])
    assert (sr.world, sr.rank, sr.lo, sr.hi) == (3, 2, 6670, 10007)
    for c in comms:
        c.close()
    L = _lib()
    assert L.byteps_shard_comm_init_local(0, (ctypes.c_int * 1)(0),
                                          (ctypes.c_void_p * 1)()) == reducer.EARGS
    assert L.byteps_shard_comm_init_local(2, (ctypes.c_int * 2)(0, -1),
                                          (ctypes.c_void_p * 2)()) == reducer.EARGS
    assert L.byteps_shard_comm_destroy(None) == reducer.OK


def test_argument_errors_without_gpu():
    """Every call validates before it touches a device."""
    L = _lib()
    c0, c1 = ShardComm.local_group([0, 0])
    h = c0.handle
    P = ctypes.c_void_p
    slots = (P * 2)(0x10000, 0x20000)
    f32 = int(DType.FLOAT32)
    E = reducer.EARGS
    # null communicator
    assert L.byteps_shard_reduce_scatter(None, 0x1000, slots, 0x3000, 8, f32, 0, None) == E
    assert L.byteps_shard_allgather(None, 0x1000, 0x2000, 8, f32, None) == E
    assert L.byteps_shard_broadcast(None, 0, 0x1000, 8, f32, None) == E
    # dtype / mode
    assert L.byteps_shard_reduce_scatter(h, 0x1000, slots, 0x3000, 8, 9, 0, None) == \
        reducer.EDTYPE
    assert L.byteps_shard_reduce_scatter(h, 0x1000, slots, 0x3000, 8, f32, 7, None) == E
    assert L.byteps_shard_allgather(h, 0x1000, 0x2000, 8, 10, None) == reducer.EDTYPE
    # missing buffers
    assert L.byteps_shard_reduce_scatter(h, None, slots, 0x3000, 8, f32, 0, None) == E
    assert L.byteps_shard_reduce_scatter(h, 0x1000, None, 0x3000, 8, f32, 0, None) == E
    assert L.byteps_shard_reduce_scatter(h, 0x1000, (P * 2)(0, 0), 0x3000, 8, f32, 0, None) == E
    assert L.byteps_shard_reduce_scatter(h, 0x1000, slots, None, 8, f32, 0, None) == E
    assert L.byteps_shard_allgather(h, None, 0x2000, 8, f32, None) == E
    assert L.byteps_shard_allgather(h, 0x1000, None, 8, f32, None) == E
    # roots and counts
    pushes = (P * 3)(0x1000, 0x2000, 0x3000)
    assert L.byteps_shard_scatter_reduce(h, 2, pushes, 3, slots, 0x4000, 8, f32, 0, None) == E
    assert L.byteps_shard_scatter_reduce(h, 0, pushes, 0, slots, 0x4000, 8, f32, 0, None) == E
    assert L.byteps_shard_scatter_reduce(h, 0, (P * 3)(0x1000, 0, 0x3000), 3, slots, 0x4000, 8,
                                         f32, 0, None) == E
    assert L.byteps_shard_reduce_root(h, -1, 0x1000, slots, 0x3000, 8, f32, 0, None) == E
    assert L.byteps_shard_reduce_root(h, 0, 0x1000, None, 0x3000, 8, f32, 0, None) == E
    assert L.byteps_shard_broadcast(h, 5, 0x1000, 8, f32, None) == E
    assert L.byteps_shard_broadcast(h, 0, None, 8, f32, None) == E
    # zero elements: a no-op that succeeds with no device
    assert L.byteps_shard_reduce_scatter(h, None, None, None, 0, f32, 0, None) == reducer.OK
    assert L.byteps_shard_allgather(h, None, None, 0, f32, None) == reducer.OK
    assert L.byteps_shard_comm_info(None, None, None, None) == E
    # wrapping nothing
    out = P()
    assert L.byteps_shard_comm_wrap(None, ctypes.byref(out)) == E and not out.value
    assert L.byteps_shard_comm_init(None, 2, 0, 0, ctypes.byref(out)) == E
    uid = ctypes.create_string_buffer(128)
    assert L.byteps_shard_comm_init(uid, 2, 2, 0, ctypes.byref(out)) == E
    assert L.byteps_shard_get_unique_id(None) == E
    c0.close()
    c1.close()
