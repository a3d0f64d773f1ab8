"""Per-query cached-plan latency of bench lines: device step, cached plan (plan + first execution + fetch +
Python conversion) and the library's plan phases. Usage: python scripts/plan_summary.py gpurun_out/x/*.json"""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        b = d.get("cached_plan_breakdown") or {}
        ph = b.get("plan_phases_ms") or {}
        host = (b.get("execute_ms") or 0) - d["ms_per_step"]
        print(f"{f.split('/')[-1]:16s} {d['config'].get('query', '')[:48]:48s} step={d['ms_per_step']:.3f} "
              f"cached_plan={d.get('cached_plan_ms', 0):.3f} exec-step={host:.3f} fetch={b.get('fetch_ms') or 0:.3f} "
              f"py={b.get('python_groups_ms') or 0:.3f} " + " ".join(f"{k}={v}" for k, v in ph.items()))
