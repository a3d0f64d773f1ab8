"""The prepared-plan cache (host.cpp plan_cache_*): a destroyed result's plan is kept under the identity it was built
for -- query, segments, device, planner overrides -- and the next execute of that identity runs it without planning
again. Every case checks the groups against the oracle: a re-used plan is a re-execution (pinot_amd_execute_again),
so it must give exactly what a fresh plan gives."""
import numpy as np
import pytest

import oracle
from helpers import random_segment

pytestmark = pytest.mark.gpu

Q = "SELECT d0, d1, COUNT(*), SUM(r_long), MAX(r_double) FROM t WHERE r_int > 0 GROUP BY d0, d1"


def _segs(E, seed, n=3):
    rng = np.random.default_rng(seed)
    bufs = [random_segment(rng, 20_000 + 500 * i, name=f"pc{seed}_{i}", bits_cards=(300, 37)) for i in range(n)]
    return bufs, [E.ImmutableSegment(b) for b in bufs]


def test_reissued_query_takes_the_prepared_plan():
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    bufs, segs = _segs(E, 1)
    _, exp = oracle.execute(Q, bufs)
    ex = E.ServerQueryExecutor()
    r1 = ex.execute(Q, segs)
    assert "plan_cache" not in r1.plan_timing()
    assert r1.groups() == exp
    r1.destroy()
    r2 = ex.execute(Q, segs)
    assert "plan_cache" in r2.plan_timing(), r2.plan_timing()
    assert r2.groups() == exp
    # a second identical query while r2 is alive plans afresh (one idle plan, now in use)
    r3 = ex.execute(Q, segs)
    assert "plan_cache" not in r3.plan_timing()
    assert r3.groups() == exp
    r2.destroy()
    r3.destroy()
    # both go back: two idle plans of one identity, each taken once
    r4, r5 = ex.execute(Q, segs), ex.execute(Q, segs)
    assert "plan_cache" in r4.plan_timing() and "plan_cache" in r5.plan_timing()
    assert r4.groups() == exp and r5.groups() == exp
    r4.execute_again()
    assert r4.groups() == exp


def test_other_identities_plan_afresh(monkeypatch):
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    bufs, segs = _segs(E, 2)
    ex = E.ServerQueryExecutor()
    ex.execute(Q, segs).destroy()
    # another literal, another segment set, another planner override: each its own plan
    q2 = Q.replace("r_int > 0", "r_int > 5")
    r = ex.execute(q2, segs)
    assert "plan_cache" not in r.plan_timing()
    assert r.groups() == oracle.execute(q2, bufs)[1]
    r.destroy()
    r = ex.execute(Q, segs[:2])
    assert "plan_cache" not in r.plan_timing()
    assert r.groups() == oracle.execute(Q, bufs[:2])[1]
    r.destroy()
    monkeypatch.setenv("PINOT_AMD_GROUP_PLAN", "hash")
    r = ex.execute(Q, segs)
    assert "plan_cache" not in r.plan_timing() and "hash" in r.kernel_info()
    assert r.groups() == oracle.execute(Q, bufs)[1]
    r.destroy()
    monkeypatch.delenv("PINOT_AMD_GROUP_PLAN")
    r = ex.execute(Q, segs)  # the dense plan of the first execute, kept
    assert "plan_cache" in r.plan_timing() and "hash" not in r.kernel_info()
    r.destroy()


def test_destroyed_segment_drops_its_plans():
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    bufs, segs = _segs(E, 3)
    ex = E.ServerQueryExecutor()
    ex.execute(Q, segs).destroy()
    segs[1].destroy()
    # the same data in new segments (new identities): a fresh plan over live buffers
    segs2 = [segs[0], E.ImmutableSegment(bufs[1]), segs[2]]
    r = ex.execute(Q, segs2)
    assert "plan_cache" not in r.plan_timing()
    assert r.groups() == oracle.execute(Q, bufs)[1]
    # a result outliving one of its segments is freed, not cached
    victim = E.ImmutableSegment(bufs[0])
    r2 = ex.execute(Q, [victim, segs2[1], segs2[2]])
    assert r2.groups() == oracle.execute(Q, bufs)[1]  # (finished before its segment goes)
    victim.destroy()
    r2.destroy()
    victim2 = E.ImmutableSegment(bufs[0])
    r3 = ex.execute(Q, [victim2, segs2[1], segs2[2]])
    assert "plan_cache" not in r3.plan_timing()
    assert r3.groups() == oracle.execute(Q, bufs)[1]


def test_ssb_plans_reused():
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    from pinot_amd import ssb
    bufs = [ssb.lineorder_flat_segment(f"pcs{i}", 100_003 + i, seed=60 + i) for i in range(2)]
    segs = [E.ImmutableSegment(b) for b in bufs]
    ex = E.ServerQueryExecutor()
    for name, sql in ssb.SSB_QUERIES:
        exp = oracle.execute(sql, bufs)[1]
        r = ex.execute(sql, segs)
        got1 = r.groups()
        r.destroy()
        r = ex.execute(sql, segs)
        assert "plan_cache" in r.plan_timing(), name
        assert r.groups() == got1, name
        assert set(r.groups()) == set(exp), name
        r.destroy()
