"""Sharded execution + cross-process merge on the device path (2 ranks sharing the box's GPU,
gloo carrying the all-reduces of the library's dense accumulator tables). The RCCL path of bench.py
uses the same pinot_amd.dist.merge_result with backend 'nccl' on 8 GPUs."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUERY = ("SELECT d1, COUNT(*), SUM(r_long), SUM(r_double), MIN(r_double), MAX(r_int), AVG(r_int) FROM t "
         "WHERE d0 < 4000 GROUP BY d1")


def _segments():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from pinot_amd.segment import DOUBLE, INT, LONG, build_segment
    rng = np.random.default_rng(1234)
    segs = []
    for i in range(5):
        n = int(rng.integers(5000, 40000))
        d0 = rng.integers(0, 5000, n)
        d1 = rng.integers(0, 64, n)
        d1[:64] = np.arange(64)  # every rank sees the same d1 dictionary -> same key space
        segs.append(build_segment(f"s{i}", {
            "d0": (d0.astype(np.int32), INT, {}),
            "d1": ((d1 * 3 + 1).astype(np.int32), INT, {}),
            "r_long": (rng.integers(-(1 << 40), 1 << 40, n), LONG, {"dictionary": False}),
            "r_double": (rng.normal(0, 1000, n), DOUBLE, {"dictionary": False}),
            "r_int": (rng.integers(-10 ** 6, 10 ** 6, n).astype(np.int32), INT, {"dictionary": False}),
        }))
    return segs


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from pinot_amd import dist as pdist, engine
    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bufs = pdist.shard(_segments(), rank, world)
    fps = [None] * world
    dist.all_gather_object(fps, pdist.key_space_fingerprint(bufs, ["d1"]))
    assert len(set(fps)) == 1, "ranks disagree on the group key space"
    segs = [engine.ImmutableSegment(b) for b in bufs]
    res = engine.ServerQueryExecutor().execute(QUERY, segs)
    pdist.merge_result(res)
    torch.cuda.synchronize()
    if rank == 0:
        q.put(res.groups())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_merge_equals_single_process():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    _, exp = oracle.execute(QUERY, _segments())
    assert set(got) == set(exp)
    for k, e in exp.items():
        g = got[k]
        assert g[0] == e[0] and g[1] == e[1] and g[3] == e[3] and g[4] == e[4], (k, g, e)
        assert np.isclose(g[2], e[2], rtol=1e-12)
        assert g[5][1] == e[5][1] and g[5][0] == e[5][0]
