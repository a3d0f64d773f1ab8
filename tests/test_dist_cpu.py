"""Multi-process merge on CPU (gloo, world size 2): segments sharded over ranks, per-rank dense
accumulator tables in the library's word encoding, merged with dist.merge_tables, compared with a
single-process oracle run over all segments."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import random_segment

QUERY = "SELECT d1, COUNT(*), SUM(r_long), SUM(r_double), MIN(r_double), MAX(r_int) FROM t WHERE d0 < 4000 GROUP BY d1"
OPS = [0, 0, 1, 2, 3]  # COUNT, SUM(int64), SUM(f64), MIN, MAX (pinot_amd_result_accumulators op codes)


def _ordered(d: np.ndarray) -> np.ndarray:
    u = d.astype(np.float64).view(np.uint64)
    neg = (u >> np.uint64(63)) == 1
    return np.where(neg, ~u, u | np.uint64(1 << 63))


def _decode_ordered(u: np.ndarray) -> np.ndarray:
    top = (u >> np.uint64(63)) == 1
    return np.where(top, u & np.uint64((1 << 63) - 1), ~u).view(np.float64)


def _segments():
    rng = np.random.default_rng(99)
    return [random_segment(rng, int(rng.integers(1000, 20000)), name=f"s{i}") for i in range(6)]


def _key_space(segs):
    return sorted(set().union(*[set(s.columns["d1"].dict_values.tolist()) for s in segs]))


def _dense_table(groups, keys):
    nk = len(keys)
    idx = {k: i for i, k in enumerate(keys)}
    t = np.zeros((5, nk), dtype=np.uint64)
    t[3, :] = np.uint64(0xFFFFFFFFFFFFFFFF)  # MIN identity
    for (k,), (cnt, s_long, s_dbl, mn, mx) in groups.items():
        i = idx[k]
        t[0, i] = cnt
        t[1, i] = np.uint64(np.int64(int(s_long)).view(np.uint64))
        t[2, i] = np.array([s_dbl], dtype=np.float64).view(np.uint64)[0]
        t[3, i] = _ordered(np.array([mn]))[0]
        t[4, i] = _ordered(np.array([float(mx)]))[0]
    return t


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle
    from pinot_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    segs = _segments()
    keys = _key_space(segs)
    mine = pdist.shard(segs, rank, world)
    _, groups = oracle.execute(QUERY, mine)
    table = torch.from_numpy(_dense_table(groups, keys).view(np.int64).ravel().copy())
    pdist.merge_tables(table, OPS, len(keys))
    if rank == 0:
        out.put(table.numpy().view(np.uint64).reshape(5, -1).copy())
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_merge_matches_single_process():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    segs = _segments()
    keys = _key_space(segs)
    _, exp = oracle.execute(QUERY, segs)
    for i, k in enumerate(keys):
        if (k,) not in exp:
            assert merged[0, i] == 0
            continue
        cnt, s_long, s_dbl, mn, mx = exp[(k,)]
        assert int(merged[0, i]) == cnt
        assert int(merged[1, i].view(np.int64)) == int(s_long)
        assert np.isclose(merged[2:3, i].view(np.float64)[0], s_dbl, rtol=1e-12)
        assert _decode_ordered(merged[3:4, i])[0] == mn
        assert _decode_ordered(merged[4:5, i])[0] == mx


def test_shard_is_a_partition():
    from pinot_amd.dist import shard
    items = list(range(103))
    parts = [shard(items, r, 8) for r in range(8)]
    assert sorted(sum(parts, [])) == items
    assert max(map(len, parts)) - min(map(len, parts)) <= 1


# ------------------------------------------------------------------- exact 128-bit sums across ranks
I128_RANKS = 8
I128_KEYS = 365


def _rank_sums(rank):
    """Per-rank exact SUM(impressions)-scale partial sums (~1.3e18 per key and rank: 2.46M docs of
    values below 2^40 each), so the 8-rank total passes INT64_MAX."""
    rng = np.random.default_rng(1000 + rank)
    return [int(x) for x in rng.integers(1 << 60, (1 << 60) + (1 << 58), I128_KEYS, dtype=np.int64)] + \
           [-(1 << 62) - rank, (1 << 63) - 1 - rank]


def _to_words(vals):
    lo = np.array([v & ((1 << 64) - 1) for v in vals], dtype=np.uint64).view(np.int64)
    hi = np.array([(v >> 64) & ((1 << 64) - 1) for v in vals], dtype=np.uint64).view(np.int64)
    return lo, hi


def _from_words(lo, hi):
    out = []
    for a, b in zip(lo.view(np.uint64), hi.view(np.uint64)):
        v = (int(b) << 64) | int(a)
        out.append(v - (1 << 128) if v >> 127 else v)
    return out


def _i128_worker(rank, world, port, out):
    from pinot_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    vals = _rank_sums(rank)
    lo, hi = _to_words(vals)
    cnt = np.full(len(vals), 1000 + rank, dtype=np.int64)
    table = torch.from_numpy(np.concatenate([cnt, lo, hi]).copy())
    pdist.merge_tables(table, [pdist.OP_SUM_I64, pdist.OP_SUM_I128, pdist.OP_HI], len(vals))
    if rank == 0:
        out.put(table.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


def test_int128_sums_merge_exactly_across_8_ranks():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_i128_worker, args=(r, I128_RANKS, port, q)) for r in range(I128_RANKS)]
    for p in procs:
        p.start()
    merged = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    n = I128_KEYS + 2
    exp = [sum(_rank_sums(r)[k] for r in range(I128_RANKS)) for k in range(n)]
    assert max(exp) > (1 << 63)  # past INT64_MAX: an int64 all-reduce would wrap
    got = _from_words(merged[n:2 * n], merged[2 * n:3 * n])
    assert got == exp
    assert list(merged[:n]) == [sum(1000 + r for r in range(I128_RANKS))] * n


def test_int128_limbs_round_trip():
    from pinot_amd.dist import _from_limbs, _limbs
    vals = [0, 1, -1, (1 << 63) - 1, -(1 << 63), (1 << 100) + 12345, -(1 << 120) - 7, (1 << 126)]
    lo, hi = _to_words(vals)
    l = _limbs(torch.from_numpy(lo), torch.from_numpy(hi))
    a, b = _from_limbs(l)
    assert _from_words(a.numpy(), b.numpy()) == vals


# ------------------------------------------------ disjoint dictionaries: global key space + both merges
def _disjoint_segments():
    """Six segments whose d1 dictionaries differ segment to segment: shard r of 2 holds values the
    other shard never sees (and some it does)."""
    from pinot_amd.segment import DOUBLE, INT, LONG, build_segment
    rng = np.random.default_rng(7)
    out = []
    for i in range(6):
        n = int(rng.integers(2000, 9000))
        d1 = rng.integers(0, 30, n) * 10 + (i % 2) * 1000 + (i // 2)   # ranks 0/1 disjoint ranges
        d1[:5] = [5, 15, 25, 35, 45]                                    # + a shared set
        out.append(build_segment(f"dj{i}", {
            "d0": (rng.integers(0, 5000, n).astype(np.int32), INT, {}),
            "d1": (d1.astype(np.int32), INT, {}),
            "r_long": (rng.integers(-(1 << 40), 1 << 40, n), LONG, {"dictionary": False}),
            "r_double": (rng.normal(0, 1000, n), DOUBLE, {"dictionary": False}),
            "r_int": (rng.integers(-10 ** 6, 10 ** 6, n).astype(np.int32), INT, {"dictionary": False})}))
    return out


def _disjoint_worker(rank, world, port, gather_max_bytes, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle
    from pinot_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = pdist.shard(_disjoint_segments(), rank, world)
    own = sorted(set().union(*[set(s.columns["d1"].dict_values.tolist()) for s in mine]))
    ks = pdist.global_key_space(mine, ["d1"])
    keys = sorted(ks["d1"])
    assert set(own) < set(keys)  # this rank's own dictionaries do not cover the key space
    _, groups = oracle.execute(QUERY, mine)
    table = torch.from_numpy(_dense_table(groups, keys).view(np.int64).ravel().copy())
    pdist.merge_tables(table, OPS, len(keys), gather_max_bytes=gather_max_bytes)
    if rank == 0:
        out.put((keys, table.numpy().view(np.uint64).reshape(5, -1).copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("gather_max_bytes", [0, 1 << 20], ids=["allreduce", "allgather"])
def test_disjoint_dictionaries_global_key_space(gather_max_bytes):
    """Ranks with different dictionaries agree on the union key space (global_key_space: one
    all-gather), so their dense tables merge in place; equal to the single-process oracle group for
    group, through the per-kind all-reduces and through the single all-gather + local reduction."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_disjoint_worker, args=(r, 2, port, gather_max_bytes, q)) for r in range(2)]
    for p in procs:
        p.start()
    keys, merged = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    _, exp = oracle.execute(QUERY, _disjoint_segments())
    assert set(k for (k,) in exp) <= set(keys)
    for i, k in enumerate(keys):
        if (k,) not in exp:
            assert merged[0, i] == 0
            continue
        cnt, s_long, s_dbl, mn, mx = exp[(k,)]
        assert int(merged[0, i]) == cnt
        assert int(merged[1, i].view(np.int64)) == int(s_long)
        assert np.isclose(merged[2:3, i].view(np.float64)[0], s_dbl, rtol=1e-12)
        assert _decode_ordered(merged[3:4, i])[0] == mn
        assert _decode_ordered(merged[4:5, i])[0] == mx


def _gather_i128_worker(rank, world, port, out):
    from pinot_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    vals = _rank_sums(rank)
    lo, hi = _to_words(vals)
    cnt = np.full(len(vals), 1000 + rank, dtype=np.int64)
    table = torch.from_numpy(np.concatenate([cnt, lo, hi]).copy())
    pdist.merge_tables(table, [pdist.OP_SUM_I64, pdist.OP_SUM_I128, pdist.OP_HI], len(vals), gather_max_bytes=1 << 30)
    if rank == 0:
        out.put(table.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


def test_int128_sums_merge_exactly_through_allgather():
    """The small-table path (one all-gather, local limb reduction) is exact past INT64_MAX too."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_i128_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    merged = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    n = I128_KEYS + 2
    exp = [sum(_rank_sums(r)[k] for r in range(4)) for k in range(n)]
    assert _from_words(merged[n:2 * n], merged[2 * n:3 * n]) == exp
    assert list(merged[:n]) == [sum(1000 + r for r in range(4))] * n


class _Col:
    def __init__(self, values):
        self.has_dictionary = True
        self.dict_values = np.asarray(values, dtype=object if isinstance(values[0], str) else None)


class _Seg:
    def __init__(self, cols):
        self.columns = {k: _Col(v) for k, v in cols.items()}


def _key_space_worker(rank, world, port, out):
    import torch.distributed as dist
    from pinot_amd import dist as pdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    segs = {
        0: [_Seg({"i": [3, 1, 2 ** 40], "f": [0.5, -0.0, float("nan")], "s": ["b", "a"]})],
        1: [_Seg({"i": [1, 7], "f": [0.0, 0.5, 2.5], "s": ["c", "a"]})],
        2: [],  # a rank without segments
    }[rank]
    ks = pdist.global_key_space(segs, ["i", "f", "s"])
    out.put((rank, ks["i"], [repr(v) for v in ks["f"]], ks["s"]))
    dist.barrier()
    dist.destroy_process_group()


def test_global_key_space_numeric_tensors_and_strings():
    """global_key_space on 3 gloo ranks (one without segments): INT values and DOUBLE bit patterns
    (-0.0 distinct from 0.0, NaN kept) through int64 tensor all-gathers, STRING values through
    all_gather_object; every rank gets the same union, first occurrence in rank order."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_key_space_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == 3
    for _, i, f, s in got:
        assert i == [3, 1, 2 ** 40, 7]
        assert f == ["0.5", "-0.0", "nan", "0.0", "2.5"]
        assert s == ["b", "a", "c"]
