"""Segments without documents (a Pinot server can hold 0-doc segments, e.g. a sealed empty consuming
segment): alone and between non-empty ones, through the fused scan, the forced selection-vector plan
(whose launches pad each segment's tile range: an empty segment has no tiles), an inverted-index leaf,
the hash plan and the filter-only path, against the oracle."""
import os
import sys

import numpy as np
import pytest

from helpers import random_segment

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from test_gpu_parity import assert_same_groups  # noqa: E402

QUERIES = [
    "SELECT COUNT(*), SUM(r_long), MIN(r_double), MAX(r_int) FROM t WHERE d0 < 40",
    "SELECT d1, COUNT(*), SUM(r_int) FROM t WHERE r_int BETWEEN 0 AND 30000 AND d0 < 900 GROUP BY d1",
    "SELECT ts, COUNT(*), SUM(r_double) FROM t WHERE d1 IN (10, 17, 73) OR r_int IN (5, 77, 1000) GROUP BY ts",
    "SELECT d0, d1, COUNT(*), SUM(r_long) FROM t WHERE d2 BETWEEN 100 AND 600 GROUP BY d0, d1",
]


@pytest.fixture(scope="module")
def data():
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    rng = np.random.default_rng(77)
    sizes = [0, 257, 0, 70_001, 0]
    bufs = [random_segment(rng, n, name=f"e{i}", bits_cards=(3000, 37, 9000), inverted=("d1",), sorted_col=True,
                           float_col=True) for i, n in enumerate(sizes)]
    return E, bufs, [E.ImmutableSegment(b) for b in bufs]


@pytest.mark.parametrize("mode", ["auto", "select", "hash"])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
@pytest.mark.parametrize("which", ["empty_only", "mixed"])
def test_empty_segments_vs_oracle(data, monkeypatch, qi, mode, which):
    E, bufs, segs = data
    if which == "empty_only":
        bufs, segs = bufs[:1], segs[:1]
    if mode == "select":
        monkeypatch.setenv("PINOT_AMD_SELECT", "always")
        monkeypatch.setenv("PINOT_AMD_PARTITIONED", "0")
    elif mode == "hash":
        monkeypatch.setenv("PINOT_AMD_GROUP_PLAN", "hash")
    q = QUERIES[qi]
    res = E.ServerQueryExecutor().execute(q, segs)
    nm, og = oracle.execute(q, bufs)
    assert res.num_docs_matched() == nm
    from pinot_amd.query import parse_sql
    qc = parse_sql(q)
    fs = {i for i, a in enumerate(qc.aggregations) if a.func in ("SUM", "AVG") and a.column in ("r_double",)}
    assert_same_groups(res.groups(), og, fs)


def test_empty_segments_filter_doc_ids(data):
    E, bufs, segs = data
    q = "SELECT COUNT(*) FROM t WHERE d1 IN (10, 17, 73) OR r_int < 0"
    ids = E.ServerQueryExecutor().filter_doc_ids(q, segs)
    assert [len(x) for x in ids][0] == 0 and len(ids[2]) == 0 and len(ids[4]) == 0
    nm, _ = oracle.execute(q, bufs)
    assert sum(len(x) for x in ids) == nm
