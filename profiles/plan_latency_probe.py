# Re-issued query latency of configs[2] queries (inverted-index IN lists of 2K-18K literals), 30 x 10M-row segments:
# cold, execute_again, planned afresh while the first result lives, re-issued after it is destroyed (prepared plan),
# each host+device time around the execute. PYTHONPATH=. python profiles/plan_latency_probe.py
import time, torch, json
from pinot_amd import engine as E, datagen
segs = [E.ImmutableSegment(datagen.inverted_segment(f"iv{i}", 10_000_000, seed=i)) for i in range(30)]
ex = E.ServerQueryExecutor()
for s in (0.1, 0.5):
    q = datagen.inverted_query(s)
    def run(tag, r=None):
        torch.cuda.synchronize(); t = time.perf_counter()
        if r is None: r = ex.execute(q, segs)
        else: r.execute_again()
        torch.cuda.synchronize(); ms = (time.perf_counter() - t) * 1e3
        print(s, tag, "host+device ms %.2f" % ms, "kernel ms %.3f" % r.last_kernel_ms(), r.kernel_info(), r.plan_timing(), flush=True)
        return r
    a = run("cold"); a.groups()
    a2 = run("again", a)
    b = run("fresh"); b.groups(); b.destroy()
    c = run("reissued"); c.groups()
    c2 = run("reissued-again", c)
    a.destroy(); c.destroy()
