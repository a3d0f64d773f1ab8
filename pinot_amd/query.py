"""QueryContext for the segment-execution path: a small SQL front end and the filter's CNF form.

Mirrors the pieces of pinot-core's request context that the hot path consumes
(pinot-common/.../request/context/predicate/*Predicate.java, FilterContext.java,
pinot-core/.../query/request/context/QueryContext.java): aggregation functions, GROUP BY
expressions, the filter tree, ORDER BY / LIMIT for the final reduce, and the numGroupsLimit
query option. Only the SQL this path executes is accepted (identifiers, numeric/string
literals, comparisons, BETWEEN, [NOT] IN, AND/OR/NOT); anything else raises ValueError.
"""
from __future__ import annotations

import collections
import dataclasses
import math
import re
import struct
from typing import List, Optional, Sequence, Tuple

import numpy as np

AGG_FUNCS = ("COUNT", "SUM", "MIN", "MAX", "AVG", "SUMLONG", "MINMAXRANGE", "DISTINCTCOUNT")
DEFAULT_GROUP_BY_LIMIT = 10          # Pinot's default LIMIT for group-by results
DEFAULT_NUM_GROUPS_LIMIT = 100_000   # InstancePlanMakerImplV2.DEFAULT_NUM_GROUPS_LIMIT


@dataclasses.dataclass(frozen=True)
class Predicate:
    """EQ / NOT_EQ / IN / NOT_IN / RANGE on one column (RangePredicate: None bound = UNBOUNDED)."""
    type: str
    column: str
    values: Tuple = ()
    lower: object = None
    upper: object = None
    lower_inclusive: bool = True
    upper_inclusive: bool = True

    def negated(self) -> "Predicate":
        flip = {"EQ": "NOT_EQ", "NOT_EQ": "EQ", "IN": "NOT_IN", "NOT_IN": "IN"}
        if self.type in flip:
            return dataclasses.replace(self, type=flip[self.type])
        raise NotImplementedError  # RANGE negation is represented with a negate flag


@dataclasses.dataclass
class FilterContext:
    type: str  # AND | OR | NOT | PREDICATE
    children: List["FilterContext"] = dataclasses.field(default_factory=list)
    predicate: Optional[Predicate] = None

    @staticmethod
    def pred(p: Predicate) -> "FilterContext":
        return FilterContext("PREDICATE", predicate=p)

    @staticmethod
    def and_(*c) -> "FilterContext":
        return FilterContext("AND", list(c))

    @staticmethod
    def or_(*c) -> "FilterContext":
        return FilterContext("OR", list(c))

    @staticmethod
    def not_(c) -> "FilterContext":
        return FilterContext("NOT", [c])


Leaf = Tuple[Predicate, bool]  # (predicate, negate)


def to_cnf(f: Optional[FilterContext]) -> List[List[Leaf]]:
    """AND of OR-clauses of (predicate, negate) leaves; NOT is pushed to the leaves (De Morgan)."""
    if f is None:
        return []

    def nnf(node: FilterContext, neg: bool):
        if node.type == "PREDICATE":
            return ("LEAF", (node.predicate, neg))
        if node.type == "NOT":
            return nnf(node.children[0], not neg)
        op = node.type
        if neg:
            op = "OR" if op == "AND" else "AND"
        return (op, [nnf(c, neg) for c in node.children])

    def cnf(n) -> List[List[Leaf]]:
        if n[0] == "LEAF":
            return [[n[1]]]
        parts = [cnf(c) for c in n[1]]
        if n[0] == "AND":
            out = []
            for p in parts:
                out.extend(p)
            return out
        # OR: distribute
        acc = [[]]
        for p in parts:
            acc = [a + b for a in acc for b in p]
        return acc

    return cnf(nnf(f, False))


EXPR_OPS = {"*": "MUL", "-": "SUB", "+": "ADD"}
EXPR_FUNC = {"MUL": "times", "SUB": "minus", "ADD": "plus"}


@dataclasses.dataclass
class Aggregation:
    """AggregationFunction over a column or a binary arithmetic transform of two columns.

    column: "*" for COUNT(*), the column name, or the expression's canonical text
    (``times(a,b)``, Pinot's FunctionContext names) for an expression argument.
    expr: None for a plain column, else (op, column_a, column_b) with op MUL / SUB / ADD
    (MultiplicationTransformFunction / SubtractionTransformFunction / AdditionTransformFunction;
    CAST(x AS DOUBLE) operands are accepted: every transform already computes in double)."""
    func: str          # COUNT SUM MIN MAX AVG SUMLONG MINMAXRANGE DISTINCTCOUNT
    column: str
    alias: Optional[str] = None
    expr: Optional[Tuple[str, str, str]] = None

    @property
    def name(self) -> str:
        return self.alias or f"{self.func.lower()}({self.column})"

    @property
    def columns(self) -> Tuple[str, ...]:
        if self.column == "*":
            return ()
        return (self.expr[1], self.expr[2]) if self.expr else (self.column,)


@dataclasses.dataclass
class QueryContext:
    table: str
    aggregations: List[Aggregation]
    group_by: List[str]
    filter: Optional[FilterContext]
    order_by: List[Tuple[str, bool]]   # (expression or alias, ascending)
    limit: int
    select_columns: List[str]           # plain columns in the SELECT list (group-by outputs)
    num_groups_limit: int = DEFAULT_NUM_GROUPS_LIMIT
    # the server combine table's trim options (QueryOptionsUtils: minServerGroupTrimSize, groupTrimThreshold)
    min_server_group_trim_size: int = 5000
    min_segment_group_trim_size: int = -1  # QueryOptions minSegmentGroupTrimSize (CommonConstants.java:1436)
    group_trim_threshold: int = 1_000_000
    # serverReturnFinalResult, sortAggregateLimitThreshold (CommonConstants: default 10000)
    server_return_final_result: bool = False
    sort_aggregate_limit_threshold: int = 10_000

    def safe_trim(self) -> bool:
        """QueryContext._isUnsafeTrim is false: the ORDER BY expressions, as a set, are the GROUP BY ones (no
        HAVING in this subset) -- QueryContext.java:746-747, isSameOrderAndGroupByColumns."""
        if not self.group_by or not self.order_by:
            return False
        t = self.order_by_targets()
        return all(k == 0 for k, _, _ in t) and {i for _, i, _ in t} == set(range(len(self.group_by)))

    def order_by_targets(self) -> List[Tuple[int, int, bool]]:
        """ORDER BY as (kind, index, ascending): kind 0 = group-by column index, 1 = aggregation index
        (matched by alias or the function text, as the broker's select list does)."""
        out = []
        for expr, asc in self.order_by:
            e = expr.lower().replace(" ", "")
            hit = None
            for j, g in enumerate(self.group_by):
                if e == g.lower():
                    hit = (0, j)
            for i, a in enumerate(self.aggregations):
                if e in (a.name.lower().replace(" ", ""), f"{a.func.lower()}({a.column})".lower().replace(" ", "")):
                    hit = (1, i)
            if hit is None:
                raise ValueError(f"ORDER BY {expr} not in select list")
            out.append((hit[0], hit[1], asc))
        return out

    @property
    def cnf(self) -> List[List[Leaf]]:
        return to_cnf(self.filter)


# ---------------------------------------------------------------------------------------- parser
_TOKEN = re.compile(r"\s*(?:(?P<num>-?\d+\.\d*(?:[eE][-+]?\d+)?|-?\d+(?:[eE][-+]?\d+)?)|(?P<str>'(?:[^']|'')*')"
                    r"|(?P<op><>|!=|<=|>=|=|<|>|\(|\)|,|\*|\+|-)|(?P<id>[A-Za-z_][A-Za-z0-9_.$]*))")


def _tokenize(sql: str):
    pos, out = 0, []
    sql = sql.strip().rstrip(";")
    while pos < len(sql):
        m = _TOKEN.match(sql, pos)
        if not m or m.end() == pos:
            if sql[pos:].strip() == "":
                break
            raise ValueError(f"cannot tokenize at: {sql[pos:pos + 20]!r}")
        pos = m.end()
        if m.group("num") is not None:
            t = m.group("num")
            out.append(("num", float(t) if any(ch in t for ch in ".eE") else int(t)))
        elif m.group("str") is not None:
            out.append(("str", m.group("str")[1:-1].replace("''", "'")))
        elif m.group("op") is not None:
            out.append(("op", m.group("op")))
        else:
            out.append(("id", m.group("id")))
    return out


class _Parser:
    def __init__(self, sql: str):
        self.t = _tokenize(sql)
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else ("eof", None)

    def kw(self, *words) -> bool:
        for k, w in enumerate(words):
            tok = self.peek(k)
            if tok[0] != "id" or tok[1].upper() != w:
                return False
        return True

    def eat_kw(self, *words):
        if not self.kw(*words):
            raise ValueError(f"expected {' '.join(words)} at token {self.peek()}")
        self.i += len(words)

    def eat_op(self, op):
        tok = self.peek()
        if tok != ("op", op):
            raise ValueError(f"expected {op!r} at token {tok}")
        self.i += 1

    def ident(self) -> str:
        tok = self.peek()
        if tok[0] != "id":
            raise ValueError(f"expected identifier at {tok}")
        self.i += 1
        return tok[1]

    def literal(self):
        tok = self.peek()
        if tok[0] not in ("num", "str"):
            raise ValueError(f"expected literal at {tok}")
        self.i += 1
        return tok[1]

    # -- grammar --
    def query(self) -> QueryContext:
        self.eat_kw("SELECT")
        aggs, cols = [], []
        while True:
            tok = self.peek()
            if tok[0] == "id" and tok[1].upper() in AGG_FUNCS and self.peek(1) == ("op", "("):
                func = tok[1].upper()
                self.i += 2
                expr = None
                if self.peek() == ("op", "*"):
                    self.i += 1
                    col = "*"
                else:
                    col = self.operand()
                    if self.peek()[0] == "op" and self.peek()[1] in EXPR_OPS:
                        op = EXPR_OPS[self.peek()[1]]
                        self.i += 1
                        col2 = self.operand()
                        expr = (op, col, col2)
                        col = f"{EXPR_FUNC[op]}({col},{col2})"
                self.eat_op(")")
                alias = None
                if self.kw("AS"):
                    self.i += 1
                    alias = self.ident()
                elif self.peek()[0] == "id" and self.peek()[1].upper() not in ("FROM",):
                    alias = self.ident()   # implicit alias: sum(x) revenue
                aggs.append(Aggregation(func, col, alias, expr))
            else:
                cols.append(self.ident())
            if self.peek() == ("op", ","):
                self.i += 1
                continue
            break
        self.eat_kw("FROM")
        table = self.ident()
        flt = None
        if self.kw("WHERE"):
            self.i += 1
            flt = self.expr()
        group_by = []
        if self.kw("GROUP", "BY"):
            self.i += 2
            group_by.append(self.ident())
            while self.peek() == ("op", ","):
                self.i += 1
                group_by.append(self.ident())
        order = []
        if self.kw("ORDER", "BY"):
            self.i += 2
            while True:
                order.append(self.order_item())
                if self.peek() != ("op", ","):
                    break
                self.i += 1
        limit = DEFAULT_GROUP_BY_LIMIT
        if self.kw("LIMIT"):
            self.i += 1
            limit = int(self.literal())
        if self.peek()[0] != "eof":
            raise ValueError(f"unexpected trailing token {self.peek()}")
        return QueryContext(table, aggs, group_by, flt, order, limit, cols)

    def operand(self) -> str:
        """A column, optionally as CAST(column AS type) (the cast does not change the value the
        arithmetic transforms compute: they read every argument as double)."""
        if self.kw("CAST") and self.peek(1) == ("op", "("):
            self.i += 2
            col = self.ident()
            self.eat_kw("AS")
            t = self.ident().upper()
            if t not in ("DOUBLE", "FLOAT", "LONG", "INT", "BIGINT", "INTEGER"):
                raise ValueError(f"unsupported CAST type {t}")
            self.eat_op(")")
            return col
        return self.ident()

    def order_item(self):
        tok = self.peek()
        if tok[0] == "id" and tok[1].upper() in AGG_FUNCS and self.peek(1) == ("op", "("):
            func = tok[1].upper()
            self.i += 2
            col = "*" if self.peek() == ("op", "*") else self.peek()[1]
            self.i += 1
            self.eat_op(")")
            expr = f"{func.lower()}({col})"
        else:
            expr = self.ident()
        asc = True
        if self.kw("DESC"):
            self.i += 1
            asc = False
        elif self.kw("ASC"):
            self.i += 1
        return (expr, asc)

    def expr(self) -> FilterContext:
        node = self.and_expr()
        children = [node]
        while self.kw("OR"):
            self.i += 1
            children.append(self.and_expr())
        return children[0] if len(children) == 1 else FilterContext.or_(*children)

    def and_expr(self) -> FilterContext:
        children = [self.not_expr()]
        while self.kw("AND"):
            self.i += 1
            children.append(self.not_expr())
        return children[0] if len(children) == 1 else FilterContext.and_(*children)

    def not_expr(self) -> FilterContext:
        if self.kw("NOT"):
            self.i += 1
            return FilterContext.not_(self.not_expr())
        if self.peek() == ("op", "("):
            self.i += 1
            e = self.expr()
            self.eat_op(")")
            return e
        return self.comparison()

    def comparison(self) -> FilterContext:
        col = self.ident()
        if self.kw("NOT", "IN") or self.kw("IN"):
            neg = self.kw("NOT")
            self.i += 2 if neg else 1
            self.eat_op("(")
            vals = [self.literal()]
            while self.peek() == ("op", ","):
                self.i += 1
                vals.append(self.literal())
            self.eat_op(")")
            return FilterContext.pred(Predicate("NOT_IN" if neg else "IN", col, tuple(vals)))
        if self.kw("NOT", "BETWEEN") or self.kw("BETWEEN"):
            neg = self.kw("NOT")
            self.i += 2 if neg else 1
            lo = self.literal()
            self.eat_kw("AND")
            hi = self.literal()
            p = FilterContext.pred(Predicate("RANGE", col, lower=lo, upper=hi))
            return FilterContext.not_(p) if neg else p
        tok = self.peek()
        if tok[0] != "op":
            raise ValueError(f"expected comparison operator at {tok}")
        self.i += 1
        v = self.literal()
        op = tok[1]
        if op == "=":
            return FilterContext.pred(Predicate("EQ", col, (v,)))
        if op in ("<>", "!="):
            return FilterContext.pred(Predicate("NOT_EQ", col, (v,)))
        if op == "<":
            return FilterContext.pred(Predicate("RANGE", col, upper=v, upper_inclusive=False))
        if op == "<=":
            return FilterContext.pred(Predicate("RANGE", col, upper=v, upper_inclusive=True))
        if op == ">":
            return FilterContext.pred(Predicate("RANGE", col, lower=v, lower_inclusive=False))
        if op == ">=":
            return FilterContext.pred(Predicate("RANGE", col, lower=v, lower_inclusive=True))
        raise ValueError(f"unsupported operator {op}")


_SET_OPTION = re.compile(r"^\s*SET\s+([A-Za-z_][A-Za-z0-9_]*)\s*=\s*'?([^;']*)'?\s*;", re.IGNORECASE)
_OPTION_CLAUSE = re.compile(r"\bOPTION\s*\(([^)]*)\)\s*;?\s*$", re.IGNORECASE)


def _query_options(sql: str):
    """Query options from ``SET key = value;`` prefixes (multi-stage style, CalciteSqlParser) and a
    trailing legacy ``OPTION(key=value, ...)`` clause; returns (remaining SQL, options)."""
    opts = {}
    while True:
        m = _SET_OPTION.match(sql)
        if not m:
            break
        opts[m.group(1)] = m.group(2).strip()
        sql = sql[m.end():]
    m = _OPTION_CLAUSE.search(sql)
    if m:
        for kv in m.group(1).split(","):
            if kv.strip():
                k, _, v = kv.partition("=")
                opts[k.strip()] = v.strip().strip("'")
        sql = sql[:m.start()]
    return sql, opts


_PARSED: "collections.OrderedDict[str, QueryContext]" = collections.OrderedDict()


def parse_sql(sql: str) -> QueryContext:
    """Compile a Pinot SQL query of the supported subset into a QueryContext. The numGroupsLimit,
    minServerGroupTrimSize, groupTrimThreshold, serverReturnFinalResult, sortAggregateLimitThreshold and
    minSegmentGroupTrimSize query options (QueryOptionsUtils) are honoured; other options are ignored.
    A re-issued query text returns the QueryContext compiled the first time (256 most recent texts; the contexts
    are never mutated after parsing -- derived queries are dataclasses.replace copies): a configs[2] IN list of
    18K literals took 30-80 ms to parse, longer than its device step."""
    qc = _PARSED.get(sql)
    if qc is not None:
        _PARSED.move_to_end(sql)
        return qc
    qc = _parse_sql(sql)
    _PARSED[sql] = qc
    if len(_PARSED) > 256:
        _PARSED.popitem(last=False)
    return qc


def _parse_sql(sql: str) -> QueryContext:
    sql, opts = _query_options(sql)
    qc = _Parser(sql).query()
    for k, v in opts.items():
        if k.lower() == "numgroupslimit":
            qc.num_groups_limit = int(v)
        elif k.lower() == "minservergrouptrimsize":
            qc.min_server_group_trim_size = int(v)
        elif k.lower() == "grouptrimthreshold":
            qc.group_trim_threshold = int(v)
        elif k.lower() == "serverreturnfinalresult":
            qc.server_return_final_result = v.strip().lower() == "true"
        elif k.lower() == "sortaggregatelimitthreshold":
            qc.sort_aggregate_limit_threshold = int(v)
        elif k.lower() == "minsegmentgrouptrimsize":
            qc.min_segment_group_trim_size = int(v)
    return qc


# ---------------------------------------------------------------------------------------- reduce
def final_value(func: str, partial):
    """AggregationFunction.extractFinalResult: AVG -> sum / count, MINMAXRANGE -> max - min
    (MinMaxRangeAggregationFunction: MinMaxRangePair(+inf, -inf) when no doc matched), others unchanged."""
    if func == "AVG":
        s, c = partial
        return s / c if c else float("-inf")
    if func == "MINMAXRANGE":
        mn, mx = partial
        return mx - mn
    if func == "DISTINCTCOUNT":
        return len(partial)
    return partial


def merge_partial(func: str, a, b):
    """AggregationFunction.merge (used by the combine and broker reduce)."""
    if func in ("COUNT", "SUM", "SUMLONG"):
        return a + b
    if func == "MIN":
        return min(a, b)
    if func == "MAX":
        return max(a, b)
    if func == "AVG":
        return (a[0] + b[0], a[1] + b[1])
    if func == "MINMAXRANGE":
        return (min(a[0], b[0]), max(a[1], b[1]))
    if func == "DISTINCTCOUNT":
        return a | b
    raise ValueError(func)


# ------------------------------------------------------------------------------- DISTINCTCOUNT
def split_distinct_count(qc: QueryContext):
    """DistinctCountAggregationFunction keeps, per group, the set of distinct values of its column
    among the matching docs (intermediate = the set, merge = union, final = its size). Planned as
    device queries: the query without its DISTINCTCOUNTs (or COUNT(*) if nothing else is left), and
    per DISTINCTCOUNT(c) the same filter grouped by (group-by columns..., c) — each distinct c of a
    group is one group of that query. Returns (base query, [(aggregation index, sub query)])."""
    rest = [a for a in qc.aggregations if a.func != "DISTINCTCOUNT"]
    base = dataclasses.replace(qc, aggregations=rest or [Aggregation("COUNT", "*")], order_by=[])
    subs = []
    for i, a in enumerate(qc.aggregations):
        if a.func == "DISTINCTCOUNT":
            if a.expr is not None or a.column == "*":
                raise ValueError("DISTINCTCOUNT takes one column")
            subs.append((i, dataclasses.replace(qc, aggregations=[Aggregation("COUNT", "*")], order_by=[],
                                                group_by=list(qc.group_by) + [a.column],
                                                num_groups_limit=max(qc.num_groups_limit, 1 << 30))))
    return base, subs


_NAN_BITS = 0x7FF8000000000000


def distinct_value(v):
    """The identity of a value in DISTINCTCOUNT's set and in a group key: FLOAT/DOUBLE values compare
    by Double.doubleToLongBits (every NaN one value, -0.0 != 0.0: the fastutil Double/Float open hash
    sets of DistinctCountAggregationFunction), so floats become their canonical 64-bit pattern; other
    values are themselves."""
    if isinstance(v, (float, np.floating)):
        f = float(v)
        return ("f", _NAN_BITS if math.isnan(f) else struct.unpack("<q", struct.pack("<d", f))[0])
    return v


class JavaDouble(float):
    """A FLOAT/DOUBLE group-key value with Java's key identity (Double.equals / doubleToLongBits, as the
    group-key maps use): every NaN equals every NaN and -0.0 != 0.0, so dicts keyed by group tuples
    keep the groups Pinot keeps apart. Arithmetic and ordering are a float's."""
    __slots__ = ()

    def __eq__(self, other):
        if isinstance(other, float):
            return distinct_value(float(self)) == distinct_value(float(other))
        return float.__eq__(self, other)

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    def __hash__(self):  # consistent with float's hash where the identities agree
        return hash(_NAN_BITS) if math.isnan(self) else float.__hash__(self)

    def __repr__(self):
        return float.__repr__(self)


def canonical_key(key) -> tuple:
    return tuple(distinct_value(v) for v in key)


def fold_distinct_count(qc: QueryContext, base_groups: dict, sub_groups: Sequence[Tuple[int, dict]]) -> dict:
    """Groups of the original query from split_distinct_count's results (same group keys as the
    base query: a group exists iff a doc matched, in every one of the queries alike). Keys and set
    elements are matched by distinct_value (bit patterns for floats), never by Python float equality."""
    sets = {i: {} for i, _ in sub_groups}
    for i, g in sub_groups:
        for key in g:
            sets[i].setdefault(canonical_key(key[:-1]), set()).add(distinct_value(key[-1]))
    rest_idx = [j for j, a in enumerate(qc.aggregations) if a.func != "DISTINCTCOUNT"]
    out = {}
    for key, parts in base_groups.items():
        full = [None] * len(qc.aggregations)
        for j, p in zip(rest_idx, parts):
            full[j] = p
        ck = canonical_key(key)
        for i in sets:
            full[i] = frozenset(sets[i].get(ck, ()))
        out[key] = full
    return out


def _dict_order(v):
    """A group-by value's position key in its (merged) dictionary's order: numbers ascending with
    Double.compare semantics for floats (-0.0 before 0.0, NaN last), strings by UTF-16 code units."""
    if isinstance(v, str):
        return (0, v.encode("utf-16-be"))
    if isinstance(v, float):
        return (1, (1, 0.0, 0) if math.isnan(v) else (0, v, int(math.copysign(1.0, v) > 0)))
    return (1, (0, v, 0))


def _double_order(x):
    x = float(x)
    return (1, 0.0, 0) if math.isnan(x) else (0, x, int(math.copysign(1.0, x) > 0))


class _Reverse:
    __slots__ = ("k",)

    def __init__(self, k):
        self.k = k

    def __lt__(self, o):
        return o.k < self.k

    def __eq__(self, o):
        return self.k == o.k


def server_table(qc: QueryContext, groups: dict) -> dict:
    """The server's combine table over combined groups, as the library applies it at compaction
    (pinot_amd_query_set_result_limit / set_server_options; GroupByUtils.java:104-149, IndexedTable.finish):
    no ORDER BY -> the first LIMIT groups in ascending key order (last group-by column compared first);
    ORDER BY -> sorted by it (ties in ascending key order) and cut to LIMIT under a safe trim below
    sortAggregateLimitThreshold or with serverReturnFinalResult, else to trimSize = max(5 * LIMIT,
    minServerGroupTrimSize) (no cut when that option is <= 0)."""
    keys = sorted(groups, key=lambda k: tuple(_dict_order(v) for v in reversed(k)))
    if not qc.order_by:
        return {k: groups[k] for k in keys[:qc.limit]}
    rank = {k: i for i, k in enumerate(keys)}
    targets = qc.order_by_targets()

    def sort_key(k):
        out = []
        for kind, idx, asc in targets:
            o = _dict_order(k[idx]) if kind == 0 else _double_order(final_value(qc.aggregations[idx].func, groups[k][idx]))
            out.append(o if asc else _Reverse(o))
        return tuple(out) + (rank[k],)
    ordered = sorted(keys, key=sort_key)
    if (qc.safe_trim() and qc.limit < qc.sort_aggregate_limit_threshold) or qc.server_return_final_result:
        keep = qc.limit
    elif qc.min_server_group_trim_size > 0:
        keep = max(5 * qc.limit, qc.min_server_group_trim_size)
    else:
        keep = len(ordered)
    return {k: groups[k] for k in ordered[:keep]}


def reduce_rows(qc: QueryContext, groups: dict) -> List[tuple]:
    """Broker reduce for group-by: final results, ORDER BY, LIMIT (default 10).

    groups: key tuple -> list of per-aggregation partials. Returns rows of
    (group values..., final aggregation values...).
    """
    rows = []
    for key, parts in groups.items():
        rows.append(tuple(key) + tuple(final_value(a.func, p) for a, p in zip(qc.aggregations, parts)))
    names = list(qc.group_by) + [a.name for a in qc.aggregations]
    exprs = list(qc.group_by) + [f"{a.func.lower()}({a.column})" for a in qc.aggregations]
    for expr, asc in reversed(qc.order_by):
        e = expr.lower()
        idx = None
        for i, (n, x) in enumerate(zip(names, exprs)):
            if e in (n.lower(), x.lower()):
                idx = i
        if idx is None:
            raise ValueError(f"ORDER BY {expr} not in select list")
        rows.sort(key=lambda r: r[idx], reverse=not asc)
    return rows[: qc.limit]
