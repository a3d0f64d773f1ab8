"""The N-rank bench path (bench.py --gpus 2: torchrun children, per-rank segment shards, barrier-bracketed
timing, max over ranks, the cross-rank merge) rehearsed on one GPU: both ranks on device 0 with gloo
collectives (PINOT_AMD_DIST_BACKEND=gloo, PINOT_AMD_DIST_ONE_DEVICE=1), since RCCL needs a device per rank.
The 8-GPU RCCL run itself is the driver's."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("workload", ["scan", "highcard"])
def test_two_rank_bench_line(workload):
    env = dict(os.environ, PINOT_AMD_DIST_BACKEND="gloo", PINOT_AMD_DIST_ONE_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--workload", workload, "--segments", "2", "--rows", "1000000"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = lines[0]
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["scaling"] == "weak"
    # the whole job's rows: 2 ranks x 2 segments x 1M rows per step
    assert d["config"]["rows_per_gpu"] == 2_000_000
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # the merge's own share of a step and its bytes per rank (a scaling curve names its bottleneck)
    m = d["merge"]
    assert m["path"] in ("dense-gather", "dense-allreduce", "by-value")
    assert m["bytes_per_rank"] > 0 and m["ms_events"] >= 0 and m["ms_wall_synchronized"] > 0
    if workload == "highcard":  # 1M groups x 4 accumulator kinds: far above the 1 MiB gather threshold
        assert m["path"] == "dense-allreduce"
