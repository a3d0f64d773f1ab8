"""A rank whose execution failed the partitioned self-check must void the merged result on EVERY rank (round-5
advisor: a faulty rank's table all-reduced into its peers, whose own check words were 0, came back as their
result). gloo, world size 2 and 3, on CPU tensors standing in for the library's HBM words:

* dense merges (dist.merge_tables) carry the check word through the same collectives -- the all-gather path and
  the all-reduce path -- so every rank's word ends nonzero when one rank's was (the library then refuses every
  rank's groups with PINOT_AMD_EINVAL);
* merges by value (dist.merge_result) agree on a failure before any row moves: every rank raises, none blocks in a
  collective the failed rank never reaches."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dense_worker(rank, world, port, bad_rank, gather_max, out):
    from pinot_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nk = 64
    ops = [pdist.OP_SUM_I64, pdist.OP_SUM_I128, pdist.OP_HI, pdist.OP_SUM_F64, pdist.OP_MIN, pdist.OP_MAX]
    table = torch.zeros(len(ops) * nk, dtype=torch.int64)
    t = table.view(len(ops), nk)
    t[0] = rank + 1                    # COUNT
    t[1] = 10 * (rank + 1)             # 128-bit sum: low words
    t[3] = torch.tensor([1.5 * (rank + 1)] * nk, dtype=torch.float64).view(torch.int64)
    t[4] = -(1 << 63) + 7              # ordered MIN / MAX encodings (positive values: sign bit set)
    t[5] = -(1 << 63) + 3 + rank
    check = torch.tensor([7 if rank == bad_rank else 0], dtype=torch.int64)
    pdist.merge_tables(table, ops, nk, gather_max_bytes=gather_max, check=check)
    out.put((rank, int(check.item()), t[0].tolist()[:2], t[1].tolist()[:2]))
    dist.barrier()
    dist.destroy_process_group()


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        item = q.get(timeout=120)
        got[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world,bad_rank", [(2, 1), (2, None), (3, 0)])
@pytest.mark.parametrize("gather_max", [1 << 20, 0])  # one all-gather / the all-reduce per reduction kind
def test_dense_merge_carries_the_check_word(world, bad_rank, gather_max):
    got = _run(_dense_worker, world, bad_rank, gather_max)
    counts = sum(range(1, world + 1))
    for r in range(world):
        chk, count_row, sum_row = got[r]
        assert (chk != 0) == (bad_rank is not None), (r, chk)
        assert count_row == [counts, counts]                 # the table merged as before
        assert sum_row == [10 * counts, 10 * counts]


class _FakeByValue:
    """A result that merges by value (a hash-table plan), with a settable self-check outcome."""

    def __init__(self, rank, failed):
        self.rank, self.failed, self.exported = rank, failed, False

    def has_dense_table(self):
        return False

    def self_check_failed(self):
        return self.failed

    def export_groups(self, stream=None):
        self.exported = True
        return torch.zeros((0, 1), dtype=torch.int64), torch.zeros((0, 1), dtype=torch.int64)

    def merge_groups(self, keys, acc, stream=None):
        pass


def _by_value_worker(rank, world, port, bad_rank, out):
    from pinot_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = _FakeByValue(rank, rank == bad_rank)
    try:
        pdist.merge_result(r)
        outcome = "merged"
    except RuntimeError as e:
        outcome = "raised" if "self-check" in str(e) else f"other: {e}"
    out.put((rank, outcome, r.exported))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,bad_rank", [(2, 0), (2, 1), (3, 2), (2, None)])
def test_by_value_merge_fails_on_every_rank(world, bad_rank):
    got = _run(_by_value_worker, world, bad_rank)
    for r in range(world):
        outcome, exported = got[r]
        if bad_rank is None:
            assert outcome == "merged" and exported, (r, outcome)
        else:
            assert outcome == "raised" and not exported, (r, outcome, exported)  # nobody moved a row
