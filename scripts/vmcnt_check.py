"""Static check of a gfx9-family disassembly (llvm-objdump -d --mcpu=gfx950): does every instruction that reads or
writes a VGPR wait for the vector-memory load still writing it (s_waitcnt vmcnt)?

Round 6, the partitioned-plan misread investigation: a kernel whose decode read a prefetch register before its
load returned would misread a few lanes only when that load is slow -- a transient, block-local error. This
restates the waitcnt bookkeeping independently of the compiler: per basic block, the pending vector-memory
operations in issue order (loads return in order on gfx9: vmcnt counts loads and stores together); s_waitcnt
vmcnt(N) leaves the N most recent pending; at a join the union of the predecessors' pending sets (each register at
its most recent position), iterated to a fixpoint over loops. Any other instruction naming a register written by a
still-pending load is reported (RAW or WAW).

    python scripts/vmcnt_check.py build/part.s
"""
import re
import sys

ADDR = re.compile(r"//\s*([0-9A-Fa-f]{12,16}):")
TARGET = re.compile(r"<([A-Za-z0-9_]+)\+0x([0-9a-f]+)>")
REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")
VMEM = re.compile(r"^(global|buffer|flat|scratch)_")


def regs(ops):
    out = set()
    for m in REG.finditer(ops):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            k, a, b = m.group(3), int(m.group(4)), int(m.group(5))
            out.update((k, i) for i in range(a, b + 1))
    return out


def parse(path):
    kernels = {}
    cur = None
    for line in open(path):
        m = re.match(r"^([0-9a-f]+) <([A-Za-z0-9_]+)>:", line)
        if m:
            cur = m.group(2)
            kernels[cur] = {"base": int(m.group(1), 16), "ins": []}
            continue
        if cur is None or not line.startswith("\t"):
            continue
        a = ADDR.search(line)
        if not a:
            continue
        text = line.split("//")[0].strip()
        op, _, ops = text.partition(" ")
        tgt = TARGET.search(line)
        kernels[cur]["ins"].append({"addr": int(a.group(1), 16), "op": op, "ops": ops.strip(),
                                    "tgt": (kernels[cur]["base"] + int(tgt.group(2), 16)) if tgt and op.startswith("s_c") or (tgt and op == "s_branch") else None})
    return kernels


def check(name, k):
    ins = k["ins"]
    idx = {x["addr"]: i for i, x in enumerate(ins)}
    # successors
    succ = []
    for i, x in enumerate(ins):
        s = []
        if x["op"] == "s_branch":
            s.append(idx[x["tgt"]])
        elif x["op"].startswith("s_cbranch"):
            s.append(idx[x["tgt"]])
            if i + 1 < len(ins):
                s.append(i + 1)
        elif x["op"] in ("s_endpgm",):
            pass
        elif i + 1 < len(ins):
            s.append(i + 1)
        succ.append(s)
    # state before each instruction: dict reg -> position (1 = most recent pending vmem op); ops count pending
    state = [None] * len(ins)
    state[0] = ({}, 0)
    work = [0]
    problems = {}
    while work:
        i = work.pop()
        regmap, npend = state[i]
        regmap = dict(regmap)
        x = ins[i]
        op, ops = x["op"], x["ops"]
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", ops)
            if m:
                n = int(m.group(1))
                regmap = {r: p for r, p in regmap.items() if p <= n}
                npend = min(npend, n)
        else:
            named = regs(ops)
            is_vmem = bool(VMEM.match(op))
            is_load = is_vmem and ("load" in op or "atomic" in op and "_rtn" in op)
            dest = set()
            if is_load:
                first = ops.split(",")[0]
                dest = regs(first)
            hazard = {r for r in named - dest if r in regmap}
            if hazard:
                problems.setdefault(x["addr"], (op, ops, sorted((r, regmap[r]) for r in hazard)))
            if is_vmem:
                regmap = {r: p + 1 for r, p in regmap.items()}
                npend += 1
                for r in dest:
                    regmap[r] = 1
                if npend > 63:
                    npend = 63
        for j in succ[i]:
            if state[j] is None:
                state[j] = (regmap, npend)
                work.append(j)
            else:
                old, on = state[j]
                merged = dict(old)
                for r, p in regmap.items():
                    merged[r] = min(merged.get(r, 99), p)
                mn = max(on, npend)
                if merged != old or mn != on:
                    state[j] = (merged, mn)
                    work.append(j)
    return problems


def main():
    ks = parse(sys.argv[1])
    bad = 0
    for name, k in ks.items():
        probs = check(name, k)
        print(f"{name}: {len(k['ins'])} instructions, {len(probs)} with a register of a pending load")
        for a, (op, ops, regs_) in sorted(probs.items())[:20]:
            print(f"  {a:012X}: {op} {ops}   pending: {regs_}")
        bad += len(probs)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
