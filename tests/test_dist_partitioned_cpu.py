"""The key-partitioned merge by value and the STRING key-space exchange on CPU (gloo, 8 ranks).

dist.merge_result's by-value path sends every exported (key words, accumulator words) row to the rank
owning its key hash (one all-to-all), each rank merges its share, and the disjoint merged shares are
all-gathered (or gathered on one root). A stand-in result replays the library's export / merge contract
on the host (merge_groups builds the merged table from the given rows with the accumulator ops;
export_groups after a merge exports the merged table), so the exchange itself is what is checked: every
rank must end with the single-process merge of all ranks' rows (AggregationFunction.merge restated by
the oracle: oracle_reduce.merge), each group's partials meeting on exactly one rank.

global_key_space for STRING columns travels as UTF-8 lengths + bytes in int64 tensors (no pickles):
the union must equal the rank-order union of every rank's dictionary, unicode and empty strings included.
"""
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle_reduce import merge

FUNCS = ["COUNT", "SUM", "MIN", "MAX"]  # accumulator words: count, int64 sum, min, max


class RowsResult:
    """Host stand-in for a by-value result: groups = {key words tuple: [count, sum, min, max]}."""

    def __init__(self, groups):
        self.groups_ = dict(groups)
        self.merges = 0

    def has_dense_table(self):
        return False

    def num_groups_limit_reached(self):
        return False

    def export_groups(self, stream=None):
        keys = torch.tensor(sorted(self.groups_), dtype=torch.int64).reshape(-1, 2)
        acc = torch.tensor([self.groups_[tuple(k)] for k in keys.tolist()], dtype=torch.int64).reshape(-1, 4)
        return keys, acc

    def merge_groups(self, keys, acc, stream=None):
        self.merges += 1
        out = {}
        for k, a in zip(map(tuple, keys.tolist()), acc.tolist()):
            out[k] = [merge(f, x, y) for f, x, y in zip(FUNCS, out[k], a)] if k in out else a
        self.groups_ = out


def rank_groups(rank, seed=0):
    rng = np.random.default_rng(seed * 1000 + rank)
    n = [0, 1, 57, 300, 5, 1000, 0, 77][rank]
    g = {}
    for _ in range(n):
        k = (int(rng.integers(0, 40)), int(rng.integers(0, 1 << 40)) if rng.random() < 0.1 else 7)
        a = [1, int(rng.integers(-10 ** 9, 10 ** 9)), int(rng.integers(-100, 100)), int(rng.integers(-100, 100))]
        g[k] = [merge(f, x, y) for f, x, y in zip(FUNCS, g[k], a)] if k in g else a
    return g


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, mode, out):
    from pinot_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if mode in ("all", "root"):
            r = RowsResult(rank_groups(rank))
            pdist.merge_result(r, root=0 if mode == "root" else None)
            out.put((rank, r.groups_, r.merges))
        elif mode == "exchange":
            rows = torch.arange(rank * 100, rank * 100 + 10 * rank, dtype=torch.int64).reshape(-1, 1).repeat(1, 3)
            dest = pdist.key_owner(rows[:, :2], world)
            got = pdist.exchange_rows(rows, dest, None)
            mine = pdist.key_owner(got[:, :2], world)
            out.put((rank, got[:, 0].tolist(), bool((mine == rank).all())))
        else:  # strings
            vals = [[], ["a"], ["ü", "", "b"], ["a", "zz" * 20], ["日本語", "b"], [""], ["x" * 9], ["q"]][rank]
            segs = [SimpleNamespace(columns={"s": SimpleNamespace(has_dictionary=True,
                                                                  dict_values=np.array(vals, dtype=object))})]
            ks = pdist.global_key_space(segs, ["s"])
            out.put((rank, ks["s"], None))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {r: (a, b) for r, a, b in (q.get(timeout=180) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def _single_process(world):
    exp = {}
    for r in range(world):
        for k, a in rank_groups(r).items():
            exp[k] = [merge(f, x, y) for f, x, y in zip(FUNCS, exp[k], a)] if k in exp else a
    return exp


def test_partitioned_merge_8_ranks_every_rank():
    got = _run(8, "all")
    exp = _single_process(8)
    for r, (groups, merges) in got.items():
        assert groups == exp, r
        assert merges == 2, r  # its share, then the gathered merged shares


def test_partitioned_merge_8_ranks_root_only():
    got = _run(8, "root")
    exp = _single_process(8)
    assert got[0][0] == exp
    shares = [set(got[r][0]) for r in range(1, 8)]
    for r in range(1, 8):  # the other ranks hold only their disjoint share
        assert got[r][1] == 1 and set(got[r][0]) <= set(exp)
    for i in range(len(shares)):
        for j in range(i + 1, len(shares)):
            assert not shares[i] & shares[j]


def test_exchange_rows_delivers_each_row_once_to_its_owner():
    got = _run(4, "exchange")
    sent = sorted(v for r in range(4) for v in range(r * 100, r * 100 + 10 * r))
    assert sorted(v for r in range(4) for v in got[r][0]) == sent
    assert all(owner_ok for _, owner_ok in got.values())


def test_string_key_space_8_ranks_without_pickles():
    got = _run(8, "strings")
    per_rank = [[], ["a"], ["ü", "", "b"], ["a", "zz" * 20], ["日本語", "b"], [""], ["x" * 9], ["q"]]
    exp = list(dict.fromkeys(v for vals in per_rank for v in vals))
    for r, (vals, _) in got.items():
        assert vals == exp, r
