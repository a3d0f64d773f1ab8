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
