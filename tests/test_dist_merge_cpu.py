"""dist.merge_result's agreement and the by-value row exchange on CPU (gloo): ranks whose results
differ in kind (a dense table on one rank, a hash-table / trimmed plan on another) must all take the
by-value path together — one rank deciding alone would leave the others blocked in a different
collective (the round-2 advisor's hang). Fake results stand in for the device library: they record which
path ran; the rows they export are gathered exactly by dist.gather_rows (ragged counts, empty ranks)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class FakeResult:
    def __init__(self, rank, dense, nrows):
        self.rank, self.dense, self.nrows = rank, dense, nrows
        self.path, self.merged = None, None

    def has_dense_table(self):
        return self.dense

    def accumulators(self):
        self.path = "dense"
        return [], 0, []  # nothing to all-reduce

    def export_groups(self, stream=None):
        keys = torch.arange(self.nrows, dtype=torch.int64).reshape(-1, 1) + 1000 * self.rank
        acc = torch.stack([torch.ones(self.nrows, dtype=torch.int64),
                           torch.full((self.nrows,), self.rank, dtype=torch.int64)], dim=1)
        return keys, acc

    def merge_groups(self, keys, acc, stream=None):
        self.path = "by_value"
        self.merged = (keys.clone(), acc.clone())


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, dense_ranks, nrows, out):
    from pinot_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = FakeResult(rank, rank in dense_ranks, nrows[rank])
    pdist.merge_result(r)
    out.put((rank, r.path, None if r.merged is None else [t.tolist() for t in r.merged]))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, dense_ranks, nrows):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, dense_ranks, nrows, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (path, m)) for r, path, m in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world,dense_ranks,nrows", [
    (2, {1}, [3, 5]),         # rank 0 hash / trimmed, rank 1 dense
    (2, {0}, [0, 4]),         # the by-value rank exports nothing
    (3, {0, 2}, [2, 0, 7]),
])
def test_ranks_agree_on_by_value_merge(world, dense_ranks, nrows):
    got = _run(world, dense_ranks, nrows)
    exp_keys = [[k + 1000 * r] for r in range(world) for k in range(nrows[r])]
    exp_acc = [[1, r] for r in range(world) for _ in range(nrows[r])]
    for r in range(world):
        path, merged = got[r]
        assert path == "by_value", (r, path)
        assert merged[0] == exp_keys and merged[1] == exp_acc  # every rank, rank order, no padding


def test_all_dense_stays_in_place():
    got = _run(2, {0, 1}, [3, 3])
    assert all(path == "dense" for path, _ in got.values())
