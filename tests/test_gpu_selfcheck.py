"""The partitioned plan's self-check (DevPartition::check, pinot_amd_result_check_word): every doc past the filter
becomes exactly one record that reaches the aggregation (DefaultGroupByExecutor.java:192-219 folds each doc once).

* Exact plans (count pass + scatter) and sampled plans (strided histogram + allotments + overflow slab, down to no
  allotment capacity at all) keep the word at 0 and match the oracle.
* A nonzero word voids the result: groups(), fetches and the matched count fail with PINOT_AMD_EINVAL naming the
  check, the process-wide failure count goes up by one per execution, and a re-execution that holds reads clean
  again. The word is set here through its device address (the injection the conftest's session check expects).
* No JIT module is ever unloaded: a process that loads every module from a warm on-disk cache (the round-5
  misreads' trigger) runs the partitioned plan clean (a subprocess with a fresh cache directory,
  cold then warm)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from helpers import EXPECTED_SELFCHECK_FAILURES, random_segment
from pinot_amd.query import parse_sql

pytestmark = pytest.mark.gpu

from test_gpu_parity import assert_same_groups  # noqa: E402

Q = ("SET numGroupsLimit = 2000000; SELECT d0, d1, COUNT(*), SUM(r_int), MIN(r_long), MAX(r_double) FROM t "
     "WHERE r_int < 600000 GROUP BY d0, d1")


@pytest.fixture(scope="module")
def engine():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from pinot_amd import engine as E
    return E


@pytest.fixture(scope="module")
def segs(engine):
    rng = np.random.default_rng(77)
    bufs = [random_segment(rng, n, name=f"sc{i}", bits_cards=(1000, 1000)) for i, n in enumerate([300_007, 123_457])]
    return bufs, [engine.ImmutableSegment(b) for b in bufs]


def _word(res):
    import torch
    from pinot_amd.engine import _DeviceWord
    return torch.as_tensor(_DeviceWord(res.check_word()), device="cuda")


@pytest.mark.parametrize("env", [{}, {"PINOT_AMD_SAMPLE_STRIDE": "2"},
                                 {"PINOT_AMD_SAMPLE_STRIDE": "2", "PINOT_AMD_PART_CAP_SCALE": "0.5"},
                                 {"PINOT_AMD_SAMPLE_STRIDE": "2", "PINOT_AMD_PART_CAP_SCALE": "0"},
                                 {"PINOT_AMD_SAMPLE_STRIDE": "2", "PINOT_AMD_PART_CAP_SCALE": "0.6", "PINOT_AMD_STAGE_CAP": "0"},
                                 {"PINOT_AMD_STAGE_CAP": "0"}])
def test_self_check_holds(engine, segs, monkeypatch, env):
    monkeypatch.delenv("PINOT_AMD_PARTITIONED", raising=False)
    monkeypatch.setenv("PINOT_AMD_SELECT_PARTITIONED", "0")
    monkeypatch.setenv("PINOT_AMD_ATOMIC_HANDOVER", "0")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    bufs, ss = segs
    before = engine.selfcheck_failures()
    res = engine.ServerQueryExecutor().execute(Q, ss)
    assert res.kernel_info().startswith("jit-partitioned"), res.kernel_info()
    nm, og = oracle.execute(Q, bufs)
    for it in range(2):
        if it:
            res.execute_again()
        assert int(_word(res).item()) == 0
        assert res.num_docs_matched() == nm
        assert_same_groups(res.groups(), og, set())
    assert engine.selfcheck_failures() == before


def test_nonzero_check_word_voids_the_result(engine, segs, monkeypatch):
    from pinot_amd._lib import PinotAmdError
    monkeypatch.delenv("PINOT_AMD_PARTITIONED", raising=False)
    monkeypatch.setenv("PINOT_AMD_SELECT_PARTITIONED", "0")
    monkeypatch.setenv("PINOT_AMD_ATOMIC_HANDOVER", "0")
    bufs, ss = segs
    res = engine.ServerQueryExecutor().execute(Q, ss)
    assert res.kernel_info().startswith("jit-partitioned"), res.kernel_info()
    before = engine.selfcheck_failures()
    w = _word(res)
    w.fill_(3)  # as if three partition runs ended off their counted records
    EXPECTED_SELFCHECK_FAILURES[0] += 1
    with pytest.raises(PinotAmdError, match="self-check failed"):
        res.groups()
    with pytest.raises(PinotAmdError, match="self-check failed"):
        res.num_docs_matched()
    assert engine.selfcheck_failures() == before + 1  # one failed execution, however often it is read
    res.execute_again()  # the next execution holds: the result reads clean again
    nm, og = oracle.execute(Q, bufs)
    assert res.num_docs_matched() == nm
    assert_same_groups(res.groups(), og, set())


_WARM = r'''
import os, sys
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "oracle"), os.path.join(sys.argv[1], "tests")]
import numpy as np
import oracle
from helpers import random_segment
from pinot_amd import engine as E
rng = np.random.default_rng(int(sys.argv[2]))
bufs = [random_segment(rng, n, name=f"w{i}", bits_cards=(700, 700)) for i, n in enumerate([120_000, 120_017, 120_034])]
segs = [E.ImmutableSegment(b) for b in bufs]
q = sys.argv[3]
nm, og = oracle.execute(q, bufs)
for _ in range(3):
    res = E.ServerQueryExecutor().execute(q, segs)
    assert res.kernel_info().startswith("jit-partitioned"), res.kernel_info()
    got = res.groups()
    assert res.num_docs_matched() == nm and set(got) == set(og), (len(got), len(og))
    for k in og:
        assert got[k][0] == og[k][0], k
print("ok", E.selfcheck_failures())
'''


def test_warm_jit_cache_processes(tmp_path):
    """Two processes over one fresh cache directory: the first compiles (cold), the second loads every module from
    the cache (warm) -- the configuration of every round-5 failure."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PINOT_AMD_JIT_CACHE_DIR=str(tmp_path), PINOT_AMD_SELECT_PARTITIONED="0",
               PINOT_AMD_ATOMIC_HANDOVER="0")
    q = ("SET numGroupsLimit = 1000000; SELECT d0, d1, COUNT(*), SUM(r_int), SUM(r_long) FROM t WHERE r_int < 600000 "
         "GROUP BY d0, d1")
    for run in ("cold", "warm"):
        p = subprocess.run([sys.executable, "-c", _WARM, root, "31", q], env=env, capture_output=True, text=True,
                           timeout=300)
        assert p.returncode == 0 and p.stdout.strip() == "ok 0", (run, p.stdout[-2000:], p.stderr[-4000:])
        if run == "cold":
            assert any(f.endswith(".co") for f in os.listdir(tmp_path)), "the cold process wrote no code objects"
