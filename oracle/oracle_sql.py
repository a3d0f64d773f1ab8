"""SQL front end of the CPU oracle. TEST INFRASTRUCTURE ONLY.

An independent restatement, for the oracle's own use, of the part of Pinot's query compilation the tested
queries need (CalciteSqlParser -> QueryContext; pinot-common/.../sql/parsers/CalciteSqlParser.java,
pinot-core/.../query/request/context/QueryContext.java), so that no product code sits between a test's SQL
text and the oracle's answer:

* SELECT list: group-by columns and aggregation functions COUNT(*), SUM, MIN, MAX, AVG, SUMLONG, MINMAXRANGE,
  DISTINCTCOUNT over a column or a binary transform of two columns (`a * b` = times, `a - b` = minus,
  `a + b` = plus; `CAST(x AS DOUBLE)` operands: the transforms read every argument as double), optional
  alias (`AS name` or a bare name);
* WHERE: AND / OR / NOT, parentheses, `=`, `<>` / `!=`, `<`, `<=`, `>`, `>=` (RangePredicate bounds with
  their inclusiveness), `[NOT] BETWEEN lo AND hi` (inclusive), `[NOT] IN (...)`; converted to conjunctive
  normal form with NOT pushed to the leaves (a negated leaf keeps a negate flag, as FilterOperatorUtils
  wraps a NOT filter);
* GROUP BY, ORDER BY (expressions ASC / DESC), LIMIT (Pinot's default 10);
* query options from `SET key = value;` prefixes or a trailing `OPTION(key=value, ...)`: numGroupsLimit
  (default 100000, InstancePlanMakerImplV2.DEFAULT_NUM_GROUPS_LIMIT), minServerGroupTrimSize (5000),
  groupTrimThreshold (1000000), serverReturnFinalResult (false), sortAggregateLimitThreshold (10000).
"""
from __future__ import annotations

import dataclasses
import re
from typing import List, Optional, Tuple

FUNCS = {"COUNT", "SUM", "MIN", "MAX", "AVG", "SUMLONG", "MINMAXRANGE", "DISTINCTCOUNT"}
TRANSFORM = {"*": ("MUL", "times"), "-": ("SUB", "minus"), "+": ("ADD", "plus")}


@dataclasses.dataclass(frozen=True)
class OPred:
    """One predicate: EQ / NOT_EQ / IN / NOT_IN on values, RANGE with optional bounds."""
    type: str
    column: str
    values: Tuple = ()
    lower: object = None
    upper: object = None
    lower_inclusive: bool = True
    upper_inclusive: bool = True


@dataclasses.dataclass
class OAgg:
    func: str
    column: str                      # "*", a column, or "times(a,b)" / "minus(a,b)" / "plus(a,b)"
    alias: Optional[str] = None
    expr: Optional[Tuple[str, str, str]] = None  # (MUL | SUB | ADD, column a, column b)

    @property
    def name(self) -> str:
        return self.alias or f"{self.func.lower()}({self.column})"


@dataclasses.dataclass
class OQuery:
    table: str
    aggregations: List[OAgg]
    group_by: List[str]
    where: Optional[tuple]           # ("and" | "or", [nodes]) | ("not", node) | ("pred", OPred)
    order_by: List[Tuple[str, bool]]
    limit: int
    num_groups_limit: int = 100_000
    min_server_group_trim_size: int = 5000
    min_segment_group_trim_size: int = -1
    group_trim_threshold: int = 1_000_000
    server_return_final_result: bool = False
    sort_aggregate_limit_threshold: int = 10_000

    @property
    def cnf(self) -> List[List[Tuple[OPred, bool]]]:
        return to_cnf(self.where)

    def order_by_targets(self) -> List[Tuple[int, int, bool]]:
        """ORDER BY items resolved against the select list: (0, group-by index) or (1, aggregation index)."""
        out = []
        for text, asc in self.order_by:
            t = text.replace(" ", "").lower()
            hit = None
            for j, g in enumerate(self.group_by):
                if t == g.lower():
                    hit = (0, j)
            for i, a in enumerate(self.aggregations):
                if t in (a.name.replace(" ", "").lower(), f"{a.func.lower()}({a.column})".lower()):
                    hit = (1, i)
            if hit is None:
                raise ValueError(f"ORDER BY {text} is not in the select list")
            out.append((hit[0], hit[1], asc))
        return out


def to_cnf(node) -> List[List[Tuple[OPred, bool]]]:
    """AND of OR-clauses of (predicate, negated) leaves."""
    if node is None:
        return []

    def push(n, neg):  # negation normal form
        kind = n[0]
        if kind == "pred":
            return ("leaf", (n[1], neg))
        if kind == "not":
            return push(n[1], not neg)
        op = kind if not neg else ("or" if kind == "and" else "and")
        return (op, [push(c, neg) for c in n[1]])

    def clauses(n):
        if n[0] == "leaf":
            return [[n[1]]]
        sub = [clauses(c) for c in n[1]]
        if n[0] == "and":
            return [cl for s in sub for cl in s]
        out = [[]]
        for s in sub:  # OR over ANDs: one clause per choice of one clause from each operand
            out = [a + b for a in out for b in s]
        return out

    return clauses(push(node, False))


_TOKENS = re.compile(r"""\s*(?:
    (?P<num>-?(?:\d+\.\d*|\d+)(?:[eE][-+]?\d+)?) |
    (?P<str>'(?:[^']|'')*') |
    (?P<op><>|!=|<=|>=|[=<>(),*+-]) |
    (?P<name>[A-Za-z_][A-Za-z0-9_.$]*)
)""", re.VERBOSE)


def _lex(sql: str):
    toks, i = [], 0
    while i < len(sql):
        m = _TOKENS.match(sql, i)
        if not m or m.end() == i:
            if sql[i:].strip() == "":
                break
            raise ValueError(f"cannot read SQL at {sql[i:i + 20]!r}")
        i = m.end()
        if m.group("num") is not None:
            v = m.group("num")
            toks.append(("lit", float(v) if re.search(r"[.eE]", v) else int(v)))
        elif m.group("str") is not None:
            toks.append(("lit", m.group("str")[1:-1].replace("''", "'")))
        elif m.group("op") is not None:
            toks.append(("op", m.group("op")))
        else:
            toks.append(("name", m.group("name")))
    toks.append(("end", None))
    return toks


class _Reader:
    def __init__(self, sql):
        self.toks = _lex(sql)
        self.pos = 0

    def at(self, k=0):
        return self.toks[min(self.pos + k, len(self.toks) - 1)]

    def word(self, w, k=0) -> bool:
        t = self.at(k)
        return t[0] == "name" and t[1].upper() == w

    def take(self):
        t = self.at()
        self.pos += 1
        return t

    def need_word(self, w):
        if not self.word(w):
            raise ValueError(f"expected {w}, found {self.at()}")
        self.pos += 1

    def need_op(self, o):
        if self.at() != ("op", o):
            raise ValueError(f"expected {o!r}, found {self.at()}")
        self.pos += 1

    def name(self) -> str:
        t = self.take()
        if t[0] != "name":
            raise ValueError(f"expected a name, found {t}")
        return t[1]

    def lit(self):
        t = self.take()
        if t[0] != "lit":
            raise ValueError(f"expected a literal, found {t}")
        return t[1]

    # ---- select list
    def arg(self) -> str:
        if self.word("CAST") and self.at(1) == ("op", "("):
            self.pos += 2
            col = self.name()
            self.need_word("AS")
            self.name()  # the target type: the transforms compute in double whatever it is
            self.need_op(")")
            return col
        return self.name()

    def select_item(self):
        t = self.at()
        if t[0] == "name" and t[1].upper() in FUNCS and self.at(1) == ("op", "("):
            func = t[1].upper()
            self.pos += 2
            expr = None
            if self.at() == ("op", "*"):
                self.pos += 1
                col = "*"
            else:
                col = self.arg()
                o = self.at()
                if o[0] == "op" and o[1] in TRANSFORM:
                    self.pos += 1
                    b = self.arg()
                    code, fname = TRANSFORM[o[1]]
                    expr, col = (code, col, b), f"{fname}({col},{b})"
            self.need_op(")")
            alias = None
            if self.word("AS"):
                self.pos += 1
                alias = self.name()
            elif self.at()[0] == "name" and not self.word("FROM"):
                alias = self.name()
            return OAgg(func, col, alias, expr)
        return self.name()

    # ---- filter
    def disjunction(self):
        parts = [self.conjunction()]
        while self.word("OR"):
            self.pos += 1
            parts.append(self.conjunction())
        return parts[0] if len(parts) == 1 else ("or", parts)

    def conjunction(self):
        parts = [self.negation()]
        while self.word("AND"):
            self.pos += 1
            parts.append(self.negation())
        return parts[0] if len(parts) == 1 else ("and", parts)

    def negation(self):
        if self.word("NOT"):
            self.pos += 1
            return ("not", self.negation())
        if self.at() == ("op", "("):
            self.pos += 1
            inner = self.disjunction()
            self.need_op(")")
            return inner
        return self.predicate()

    def predicate(self):
        col = self.name()
        negated = self.word("NOT") and (self.word("IN", 1) or self.word("BETWEEN", 1))
        if negated:
            self.pos += 1
        if self.word("IN"):
            self.pos += 1
            self.need_op("(")
            vals = [self.lit()]
            while self.at() == ("op", ","):
                self.pos += 1
                vals.append(self.lit())
            self.need_op(")")
            return ("pred", OPred("NOT_IN" if negated else "IN", col, tuple(vals)))
        if self.word("BETWEEN"):
            self.pos += 1
            lo = self.lit()
            self.need_word("AND")
            hi = self.lit()
            p = ("pred", OPred("RANGE", col, lower=lo, upper=hi))
            return ("not", p) if negated else p
        o = self.take()
        if o[0] != "op":
            raise ValueError(f"expected a comparison after {col}, found {o}")
        v = self.lit()
        if o[1] == "=":
            return ("pred", OPred("EQ", col, (v,)))
        if o[1] in ("<>", "!="):
            return ("pred", OPred("NOT_EQ", col, (v,)))
        if o[1] in ("<", "<="):
            return ("pred", OPred("RANGE", col, upper=v, upper_inclusive=o[1] == "<="))
        if o[1] in (">", ">="):
            return ("pred", OPred("RANGE", col, lower=v, lower_inclusive=o[1] == ">="))
        raise ValueError(f"unsupported comparison {o[1]}")

    def order_item(self):
        t = self.at()
        if t[0] == "name" and t[1].upper() in FUNCS and self.at(1) == ("op", "("):
            self.pos += 2
            inner = self.take()
            self.need_op(")")
            text = f"{t[1].lower()}({'*' if inner == ('op', '*') else inner[1]})"
        else:
            text = self.name()
        asc = True
        if self.word("DESC"):
            self.pos += 1
            asc = False
        elif self.word("ASC"):
            self.pos += 1
        return text, asc

    def query(self) -> OQuery:
        self.need_word("SELECT")
        items = [self.select_item()]
        while self.at() == ("op", ","):
            self.pos += 1
            items.append(self.select_item())
        self.need_word("FROM")
        table = self.name()
        where = None
        if self.word("WHERE"):
            self.pos += 1
            where = self.disjunction()
        group_by = []
        if self.word("GROUP") and self.word("BY", 1):
            self.pos += 2
            group_by.append(self.name())
            while self.at() == ("op", ","):
                self.pos += 1
                group_by.append(self.name())
        order_by = []
        if self.word("ORDER") and self.word("BY", 1):
            self.pos += 2
            order_by.append(self.order_item())
            while self.at() == ("op", ","):
                self.pos += 1
                order_by.append(self.order_item())
        limit = 10
        if self.word("LIMIT"):
            self.pos += 1
            limit = int(self.lit())
        if self.at()[0] != "end":
            raise ValueError(f"unexpected {self.at()} after the query")
        return OQuery(table, [i for i in items if isinstance(i, OAgg)], group_by, where, order_by, limit)


_SET = re.compile(r"\s*SET\s+(\w+)\s*=\s*'?([^;']*?)'?\s*;", re.IGNORECASE)
_OPTION = re.compile(r"\bOPTION\s*\(([^)]*)\)\s*;?\s*$", re.IGNORECASE)


def parse(sql: str) -> OQuery:
    """SQL text -> OQuery, with its query options applied."""
    opts = {}
    while True:
        m = _SET.match(sql)
        if not m:
            break
        opts[m.group(1).lower()] = m.group(2).strip()
        sql = sql[m.end():]
    m = _OPTION.search(sql)
    if m:
        for kv in m.group(1).split(","):
            if "=" in kv:
                k, v = kv.split("=", 1)
                opts[k.strip().lower()] = v.strip().strip("'")
        sql = sql[:m.start()]
    q = _Reader(sql).query()
    for k, v in opts.items():
        if k == "numgroupslimit":
            q.num_groups_limit = int(v)
        elif k == "minservergrouptrimsize":
            q.min_server_group_trim_size = int(v)
        elif k == "minsegmentgrouptrimsize":
            q.min_segment_group_trim_size = int(v)
        elif k == "grouptrimthreshold":
            q.group_trim_threshold = int(v)
        elif k == "serverreturnfinalresult":
            q.server_return_final_result = v.lower() == "true"
        elif k == "sortaggregatelimitthreshold":
            q.sort_aggregate_limit_threshold = int(v)
    return q
