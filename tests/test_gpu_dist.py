"""Sharded execution + cross-process merge on the device path (2 ranks sharing the box's GPU,
gloo carrying the collectives: the library's dense accumulator tables viewed in place, or every rank's
exported group rows for the device merge by value). Each
rank's segments have their own dictionaries: the ranks agree on the union key space first
(dist.global_key_space). The RCCL path of bench.py uses the same pinot_amd.dist functions with backend
'nccl' on 8 GPUs."""
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
        d1 = rng.integers(0, 64, n) + 100 * (i % 2)  # shards 0 / 1 see disjoint d1 dictionaries
        segs.append(build_segment(f"s{i}", {
            "d0": (d0.astype(np.int32), INT, {}),
            "d1": ((d1 * 3 + 1).astype(np.int32), INT, {}),
            "r_long": (rng.integers(-(1 << 40), 1 << 40, n), LONG, {"dictionary": False}),
            "r_double": (rng.normal(0, 1000, n), DOUBLE, {"dictionary": False}),
            "r_int": (rng.integers(-10 ** 6, 10 ** 6, n).astype(np.int32), INT, {"dictionary": False}),
        }))
    return segs


TRIM_QUERY = ("SET numGroupsLimit = 40; SELECT d1, COUNT(*), SUM(r_long), MIN(r_double), MAX(r_int) FROM t "
              "WHERE d0 < 4000 GROUP BY d1")
DC_QUERY = "SELECT d1, DISTINCTCOUNT(r_int), COUNT(*), SUM(r_long) FROM t WHERE d0 < 3000 GROUP BY d1"
# DISTINCTCOUNT without GROUP BY: its base query is aggregation-only (merged in place), the value-set query
# merges by value (round-3 advisor: export_groups refused the base part)
DC_AGG_QUERY = "SELECT DISTINCTCOUNT(d1), COUNT(*), SUM(r_long) FROM t WHERE d0 < 3000"
QUERIES = {"trim": TRIM_QUERY, "distinct": DC_QUERY, "distinct_agg": DC_AGG_QUERY}


def _worker(rank, world, port, q, plan):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from pinot_amd import dist as pdist, engine
    from pinot_amd.query import parse_sql
    torch.cuda.set_device(0)
    if plan == "hash" or (plan == "mixed" and rank == 0):
        os.environ["PINOT_AMD_GROUP_PLAN"] = "hash"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bufs = pdist.shard(_segments(), rank, world)
    fps = [None] * world
    dist.all_gather_object(fps, pdist.key_space_fingerprint(bufs, ["d1"]))
    assert len(set(fps)) == world, "shards were meant to hold different dictionaries"
    segs = [engine.ImmutableSegment(b) for b in bufs]
    query = QUERIES.get(plan, QUERY)
    ks = pdist.global_key_space(segs, pdist.key_columns(parse_sql(query)))
    res = engine.ServerQueryExecutor().execute(query, segs, stream=torch.cuda.current_stream(), key_space=ks)
    if plan == "dense":
        assert res.kernel_info().startswith("jit") and "hash" not in res.kernel_info()
    if plan == "hash" or (plan == "mixed" and rank == 0):
        assert "hash" in res.kernel_info()
    if plan == "mixed" and rank == 1:
        assert "hash" not in res.kernel_info()
    # dense tables merge in place (all-reduce / all-gather); any hash-table, trimmed or DISTINCTCOUNT
    # result makes every rank merge by value on the device (export -> all-gather -> merge_groups)
    pdist.merge_result(res, stream=torch.cuda.current_stream(), gather_max_bytes=int(os.environ["GATHER_MAX"]))
    torch.cuda.synchronize()
    groups = res.groups()
    q.put((rank, groups, res.num_groups_limit_reached()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("plan,gather_max", [("dense", 0), ("dense", 1 << 20), ("hash", 0), ("mixed", 0), ("trim", 0),
                                             ("distinct", 0), ("distinct_agg", 0)])
def test_two_rank_merge_equals_single_process(plan, gather_max, monkeypatch):
    """Every rank ends with the single-process result: dense plans through the in-place table merge;
    hash plans, a hash rank next to a dense rank (the ranks agree on the by-value merge), numGroupsLimit
    trimming (each segment admits its first 40 groups; the union survives sharding) and DISTINCTCOUNT
    (value sets unioned) through the device merge by value."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    monkeypatch.setenv("GATHER_MAX", str(gather_max))
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, plan)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    query = QUERIES.get(plan, QUERY)
    stats = {}
    _, exp = oracle.execute(query, _segments(), stats=stats)
    for rank, groups, reached in got:
        assert set(groups) == set(exp), rank
        # the broker ORs numGroupsLimitReached over servers: every rank reports the oracle's flag
        assert reached == bool(stats.get("num_groups_limit_reached", False)), (rank, reached, stats)
        if plan == "trim":
            assert stats["num_groups_limit_reached"]
            assert groups == exp, rank
            continue
        if plan in ("distinct", "distinct_agg"):
            assert groups == exp, rank
            continue
        for k, e in exp.items():
            g = groups[k]
            assert g[0] == e[0] and g[1] == e[1] and g[3] == e[3] and g[4] == e[4], (k, g, e)
            assert np.isclose(g[2], e[2], rtol=1e-12)
            assert g[5][1] == e[5][1] and g[5][0] == e[5][0]
