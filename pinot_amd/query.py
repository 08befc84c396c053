"""QueryContext: the query IR the hot path consumes, built from the SQL subset Pinot's tests use.

Mirrors pinot-core's QueryContext (core/query/request/context/QueryContext.java:73-122) and the
FilterContext / Predicate types of pinot-common (request/context/FilterContext.java,
request/context/predicate/*.java).  Comparison operators are rewritten into predicates the way
RequestContextUtils does: `a > v` -> RANGE (v, *) exclusive, `a BETWEEN x AND y` -> RANGE [x, y],
`a <> v` / `a != v` -> NOT_EQ.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional, Tuple, Union

UNBOUNDED = "*"  # RangePredicate.UNBOUNDED


# ------------------------------------------------------------------------------------------ IR

@dataclass(frozen=True)
class Predicate:
    type: str                 # EQ, NOT_EQ, IN, NOT_IN, RANGE, IS_NULL, IS_NOT_NULL
    column: str
    values: Tuple[str, ...] = ()
    lower: str = UNBOUNDED
    upper: str = UNBOUNDED
    lower_inclusive: bool = False
    upper_inclusive: bool = False

    @property
    def is_exclusive(self):
        return self.type in ("NOT_EQ", "NOT_IN")


@dataclass
class FilterContext:
    type: str                                   # AND, OR, NOT, PREDICATE
    children: List["FilterContext"] = field(default_factory=list)
    predicate: Optional[Predicate] = None

    def leaves(self) -> List[Predicate]:
        if self.type == "PREDICATE":
            return [self.predicate]
        out = []
        for c in self.children:
            out.extend(c.leaves())
        return out


@dataclass(frozen=True)
class Expr:
    """Aggregation input / group-by / order-by expression: a column, a binary op of columns, or '*'."""
    op: str                       # COL, MUL, ADD, SUB, STAR
    cols: Tuple[str, ...] = ()

    def __str__(self):
        if self.op == "STAR":
            return "*"
        if self.op == "COL":
            return self.cols[0]
        sym = {"MUL": "times", "ADD": "plus", "SUB": "minus"}[self.op]
        return f"{sym}({self.cols[0]},{self.cols[1]})"


@dataclass(frozen=True)
class Aggregation:
    function: str     # COUNT, SUM, MIN, MAX, AVG, DISTINCTCOUNT, COUNTMV
    arg: Expr
    # `AGG(x) FILTER (WHERE f)`: the aggregation's own filter, ANDed with the query's (QueryContext's
    # filteredAggregationFunctions, QueryContext.java:512-560); part of equality, not of the hash
    filter: Optional[FilterContext] = field(default=None, hash=False)
    # SUMMV / MINMV / MAXMV / AVGMV / DISTINCTCOUNTMV: `function` over every value of a multi-value column (the same
    # intermediate and final types as the single-value function: SumMVAggregationFunction extends SumAggregationFunction)
    mv: bool = False

    @property
    def name(self) -> str:
        """The function's SQL name (SUMMV for SUM over MV values)."""
        return self.function + ("MV" if self.mv else "")

    def result_name(self):
        base = f"{self.name.lower()}({self.arg})"
        return base if self.filter is None else f"{base} FILTER(WHERE {filter_str(self.filter)})"


@dataclass
class SelectItem:
    kind: str                      # AGG or COL
    agg: Optional[Aggregation] = None
    column: Optional[str] = None
    alias: Optional[str] = None

    def name(self):
        if self.alias:
            return self.alias
        return self.agg.result_name() if self.kind == "AGG" else self.column


@dataclass
class OrderBy:
    kind: str                      # AGG, COL, ALIAS
    agg: Optional[Aggregation] = None
    column: Optional[str] = None
    asc: bool = True


@dataclass(frozen=True)
class HavingExpr:
    """A HAVING operand (PostAggregationHandler's value extractors, query/reduce/PostAggregationHandler.java): an
    aggregation's final result, a group-by key, a numeric literal, or + - * / of those."""
    kind: str                              # AGG, COL, LIT, ARITH
    agg: Optional[Aggregation] = None
    column: Optional[str] = None
    value: Optional[str] = None
    op: Optional[str] = None               # ARITH: + - * /
    args: Tuple["HavingExpr", ...] = ()

    def aggregations(self) -> List[Aggregation]:
        if self.kind == "AGG":
            return [self.agg]
        out = []
        for a in self.args:
            out.extend(a.aggregations())
        return out


@dataclass
class HavingFilter:
    """The HAVING clause (QueryContext._havingFilter): AND / OR / NOT of predicates whose left-hand side is a
    HavingExpr; `lhs <op> rhs` with a non-literal rhs is `lhs - rhs <op> 0`, as CalciteSqlParser rewrites it."""
    type: str                                       # AND, OR, NOT, PREDICATE
    children: List["HavingFilter"] = field(default_factory=list)
    lhs: Optional[HavingExpr] = None
    predicate: Optional[Predicate] = None           # its column is unused ("")

    def aggregations(self) -> List[Aggregation]:
        if self.type == "PREDICATE":
            return self.lhs.aggregations()
        out = []
        for c in self.children:
            out.extend(c.aggregations())
        return out


@dataclass
class QueryContext:
    table: str
    select: List[SelectItem]
    filter: Optional[FilterContext]
    group_by: List[str]
    order_by: List[OrderBy]
    limit: int
    options: dict = field(default_factory=dict)
    having: Optional[HavingFilter] = None

    @property
    def aggregations(self) -> List[Aggregation]:
        """Distinct aggregations in first-seen order: the select list, the HAVING filter, the ORDER BY
        (QueryContext.generateAggregationFunctions, QueryContext.java:514-560)."""
        out = []
        for s in self.select:
            if s.kind == "AGG" and s.agg not in out:
                out.append(s.agg)
        for a in (self.having.aggregations() if self.having is not None else []):
            if a not in out:
                out.append(a)
        for o in self.order_by:
            if o.kind == "AGG" and o.agg not in out:
                out.append(o.agg)
        return out


# ------------------------------------------------------------------------------------------ parser

_TOKEN = re.compile(r"\s*(?:(?P<num>-?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?)|(?P<str>'(?:[^']|'')*')|"
                    r"(?P<id>[A-Za-z_][A-Za-z0-9_.$]*)|(?P<op><>|!=|<=|>=|[=<>*+\-/(),]))")
_KEYWORDS = {"SELECT", "FROM", "WHERE", "GROUP", "BY", "ORDER", "LIMIT", "AND", "OR", "NOT", "IN", "BETWEEN",
             "ASC", "DESC", "AS", "OPTION", "IS", "NULL", "HAVING"}
_AGGS = {"COUNT", "SUM", "MIN", "MAX", "AVG", "DISTINCTCOUNT", "COUNTMV",
         "SUMMV", "MINMV", "MAXMV", "AVGMV", "DISTINCTCOUNTMV"}


def _tokenize(sql: str):
    pos = 0
    out = []
    sql = sql.strip().rstrip(";")
    while pos < len(sql):
        m = _TOKEN.match(sql, pos)
        if not m or m.end() == pos:
            if sql[pos:].strip() == "":
                break
            raise ValueError(f"cannot tokenize at: {sql[pos:pos + 20]!r}")
        pos = m.end()
        if m.group("num") is not None:
            out.append(("num", m.group("num")))
        elif m.group("str") is not None:
            out.append(("str", m.group("str")[1:-1].replace("''", "'")))
        elif m.group("id") is not None:
            v = m.group("id")
            out.append(("kw", v.upper()) if v.upper() in _KEYWORDS else ("id", v))
        else:
            out.append(("op", m.group("op")))
    return out


class _Parser:
    def __init__(self, sql):
        self.t = _tokenize(sql)
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def next(self):
        tok = self.peek()
        self.i += 1
        return tok

    def accept(self, kind, val=None):
        k, v = self.peek()
        if k == kind and (val is None or v == val):
            self.i += 1
            return True
        return False

    def expect(self, kind, val=None):
        k, v = self.next()
        if k != kind or (val is not None and v != val):
            raise ValueError(f"expected {val or kind}, got {v!r}")
        return v

    # expressions used inside aggregations: col | col op col | *
    def expr(self) -> Expr:
        if self.accept("op", "*"):
            return Expr("STAR")
        a = self.expect("id")
        k, v = self.peek()
        if k == "op" and v in ("*", "+", "-"):
            self.next()
            b = self.expect("id")
            return Expr({"*": "MUL", "+": "ADD", "-": "SUB"}[v], (a, b))
        return Expr("COL", (a,))

    def agg_or_col(self):
        k, v = self.peek()
        if k == "id" and v.upper() in _AGGS and self.peek(1) == ("op", "("):
            self.next()
            self.expect("op", "(")
            e = self.expr()
            self.expect("op", ")")
            fn = v.upper()
            if fn == "COUNT":
                e = Expr("STAR")
            filt = None
            if self.peek()[0] == "id" and self.peek()[1].upper() == "FILTER" and self.peek(1) == ("op", "("):
                # AGG(x) FILTER (WHERE f) -- CalciteSqlParser's FILTER clause -> FilterContext of the aggregation
                self.next()
                self.expect("op", "(")
                self.expect("kw", "WHERE")
                filt = self.or_expr()
                self.expect("op", ")")
            mv = fn.endswith("MV") and fn != "COUNTMV"
            return "AGG", Aggregation(fn[:-2] if mv else fn, e, filt, mv)
        return "COL", self.expect("id")

    def literal(self) -> str:
        k, v = self.next()
        if k in ("num", "str"):
            return v
        raise ValueError(f"expected literal, got {v!r}")

    def predicate(self) -> FilterContext:
        if self.accept("op", "("):
            f = self.or_expr()
            self.expect("op", ")")
            return f
        if self.accept("kw", "NOT"):
            return FilterContext("NOT", [self.predicate()])
        col = self.expect("id")
        if self.accept("kw", "IS"):  # IsNullPredicate / IsNotNullPredicate (request/context/predicate/)
            neg = self.accept("kw", "NOT")
            self.expect("kw", "NULL")
            return FilterContext("PREDICATE", predicate=Predicate("IS_NOT_NULL" if neg else "IS_NULL", col))
        if self.accept("kw", "BETWEEN"):
            lo = self.literal()
            self.expect("kw", "AND")
            hi = self.literal()
            return FilterContext("PREDICATE", predicate=Predicate("RANGE", col, (), lo, hi, True, True))
        neg = self.accept("kw", "NOT")
        if neg and self.accept("kw", "BETWEEN"):  # NOT BETWEEN -> NOT(RANGE) (CalciteSqlParser keeps the NOT)
            lo = self.literal()
            self.expect("kw", "AND")
            hi = self.literal()
            return FilterContext("NOT", [FilterContext("PREDICATE",
                                                       predicate=Predicate("RANGE", col, (), lo, hi, True, True))])
        if self.accept("kw", "IN"):
            self.expect("op", "(")
            vals = [self.literal()]
            while self.accept("op", ","):
                vals.append(self.literal())
            self.expect("op", ")")
            return FilterContext("PREDICATE", predicate=Predicate("NOT_IN" if neg else "IN", col, tuple(vals)))
        if neg:
            raise ValueError("NOT must be followed by IN or BETWEEN")
        op = self.expect("op")
        v = self.literal()
        if op == "=":
            p = Predicate("EQ", col, (v,))
        elif op in ("!=", "<>"):
            p = Predicate("NOT_EQ", col, (v,))
        elif op == ">":
            p = Predicate("RANGE", col, (), v, UNBOUNDED, False, False)
        elif op == ">=":
            p = Predicate("RANGE", col, (), v, UNBOUNDED, True, False)
        elif op == "<":
            p = Predicate("RANGE", col, (), UNBOUNDED, v, False, False)
        elif op == "<=":
            p = Predicate("RANGE", col, (), UNBOUNDED, v, False, True)
        else:
            raise ValueError(f"unsupported operator {op}")
        return FilterContext("PREDICATE", predicate=p)

    # ---- HAVING: predicates over post-aggregation values
    def h_atom(self) -> HavingExpr:
        if self.accept("op", "("):
            e = self.h_sum()
            self.expect("op", ")")
            return e
        k, v = self.peek()
        if k in ("num", "str"):
            self.next()
            return HavingExpr("LIT", value=v, op="STR" if k == "str" else None)
        kind, x = self.agg_or_col()
        return HavingExpr("AGG", agg=x) if kind == "AGG" else HavingExpr("COL", column=x)

    def h_product(self) -> HavingExpr:
        e = self.h_atom()
        while self.peek() in (("op", "*"), ("op", "/")):
            op = self.next()[1]
            e = HavingExpr("ARITH", op=op, args=(e, self.h_atom()))
        return e

    def h_sum(self) -> HavingExpr:
        e = self.h_product()
        while True:
            k, v = self.peek()
            if (k, v) in (("op", "+"), ("op", "-")):
                self.next()
                e = HavingExpr("ARITH", op=v, args=(e, self.h_product()))
            elif k == "num" and v.startswith("-"):  # `x -1` tokenised as x, -1: a subtraction
                self.next()
                e = HavingExpr("ARITH", op="-", args=(e, HavingExpr("LIT", value=v[1:])))
            else:
                return e

    def h_predicate(self) -> HavingFilter:
        k, v = self.peek()
        if (k, v) == ("op", "("):  # a parenthesised filter or an arithmetic operand: try the filter first
            save = self.i
            self.next()
            try:
                f = self.h_or()
                self.expect("op", ")")
                return f
            except ValueError:
                self.i = save
        if self.accept("kw", "NOT"):
            return HavingFilter("NOT", [self.h_predicate()])
        lhs = self.h_sum()
        leaf = lambda p: HavingFilter("PREDICATE", lhs=lhs, predicate=p)
        if self.accept("kw", "IS"):
            neg = self.accept("kw", "NOT")
            self.expect("kw", "NULL")
            return leaf(Predicate("IS_NOT_NULL" if neg else "IS_NULL", ""))
        neg = self.accept("kw", "NOT")
        if self.accept("kw", "BETWEEN"):
            lo = self.literal()
            self.expect("kw", "AND")
            hi = self.literal()
            f = leaf(Predicate("RANGE", "", (), lo, hi, True, True))
            return HavingFilter("NOT", [f]) if neg else f
        if self.accept("kw", "IN"):
            self.expect("op", "(")
            vals = [self.literal()]
            while self.accept("op", ","):
                vals.append(self.literal())
            self.expect("op", ")")
            return leaf(Predicate("NOT_IN" if neg else "IN", "", tuple(vals)))
        if neg:
            raise ValueError("NOT must be followed by IN or BETWEEN")
        op = self.expect("op")
        k, v = self.peek()
        rhs = self.h_sum()
        if rhs.kind != "LIT":  # CalciteSqlParser: `a <op> b` with a non-literal b -> `minus(a, b) <op> 0`
            lhs = HavingExpr("ARITH", op="-", args=(lhs, rhs))
            v = "0"
        else:
            v = rhs.value
        p = {"=": Predicate("EQ", "", (v,)), "!=": Predicate("NOT_EQ", "", (v,)), "<>": Predicate("NOT_EQ", "", (v,)),
             ">": Predicate("RANGE", "", (), v, UNBOUNDED, False, False),
             ">=": Predicate("RANGE", "", (), v, UNBOUNDED, True, False),
             "<": Predicate("RANGE", "", (), UNBOUNDED, v, False, False),
             "<=": Predicate("RANGE", "", (), UNBOUNDED, v, False, True)}.get(op)
        if p is None:
            raise ValueError(f"unsupported operator {op}")
        return HavingFilter("PREDICATE", lhs=lhs, predicate=p)

    def h_and(self) -> HavingFilter:
        parts = [self.h_predicate()]
        while self.accept("kw", "AND"):
            parts.append(self.h_predicate())
        return parts[0] if len(parts) == 1 else HavingFilter("AND", _flatten("AND", parts))

    def h_or(self) -> HavingFilter:
        parts = [self.h_and()]
        while self.accept("kw", "OR"):
            parts.append(self.h_and())
        return parts[0] if len(parts) == 1 else HavingFilter("OR", _flatten("OR", parts))

    def and_expr(self) -> FilterContext:
        parts = [self.predicate()]
        while self.accept("kw", "AND"):
            parts.append(self.predicate())
        return parts[0] if len(parts) == 1 else FilterContext("AND", _flatten("AND", parts))

    def or_expr(self) -> FilterContext:
        parts = [self.and_expr()]
        while self.accept("kw", "OR"):
            parts.append(self.and_expr())
        return parts[0] if len(parts) == 1 else FilterContext("OR", _flatten("OR", parts))


def filter_str(f: FilterContext) -> str:
    """A canonical text of a filter tree (FilterContext.toString's role: equal filters, equal text)."""
    if f.type == "PREDICATE":
        p = f.predicate
        if p.type == "RANGE":
            return (f"{p.column} {'[' if p.lower_inclusive else '('}{p.lower},{p.upper}"
                    f"{']' if p.upper_inclusive else ')'}")
        if p.type in ("IS_NULL", "IS_NOT_NULL"):
            return f"{p.column} {p.type.replace('_', ' ')}"
        return f"{p.column} {p.type} ({','.join(p.values)})"
    if f.type == "NOT":
        return f"NOT({filter_str(f.children[0])})"
    return f"{f.type}(" + ", ".join(filter_str(c) for c in f.children) + ")"


def _flatten(kind, parts):
    """FilterContext flattening of nested AND/AND and OR/OR (QueryOptimizer FlattenAndOrFilterOptimizer)."""
    out = []
    for p in parts:
        out.extend(p.children if p.type == kind else [p])
    return out


def parse(sql: str) -> QueryContext:
    p = _Parser(sql)
    p.expect("kw", "SELECT")
    select = []
    while True:
        kind, x = p.agg_or_col()
        alias = None
        if p.accept("kw", "AS"):
            alias = p.expect("id")
        select.append(SelectItem(kind, agg=x if kind == "AGG" else None, column=x if kind == "COL" else None,
                                 alias=alias))
        if not p.accept("op", ","):
            break
    p.expect("kw", "FROM")
    table = p.expect("id")
    filt = None
    if p.accept("kw", "WHERE"):
        filt = p.or_expr()
    group_by = []
    if p.accept("kw", "GROUP"):
        p.expect("kw", "BY")
        group_by.append(p.expect("id"))
        while p.accept("op", ","):
            group_by.append(p.expect("id"))
    having = None
    if p.accept("kw", "HAVING"):
        if not group_by:
            raise ValueError("HAVING without GROUP BY")
        having = _resolve_having(p.h_or(), select, group_by)
    order_by = []
    if p.accept("kw", "ORDER"):
        p.expect("kw", "BY")
        while True:
            kind, x = p.agg_or_col()
            asc = True
            if p.accept("kw", "DESC"):
                asc = False
            else:
                p.accept("kw", "ASC")
            if kind == "AGG":
                order_by.append(OrderBy("AGG", agg=x, asc=asc))
            else:
                aliases = {s.alias: s for s in select if s.alias}
                if x in aliases and aliases[x].kind == "AGG":
                    order_by.append(OrderBy("AGG", agg=aliases[x].agg, asc=asc))
                else:
                    order_by.append(OrderBy("COL", column=x, asc=asc))
            if not p.accept("op", ","):
                break
    limit = 10  # SQL default LIMIT in Pinot
    if p.accept("kw", "LIMIT"):
        limit = int(p.expect("num"))
    options = {}
    if p.accept("kw", "OPTION"):
        p.expect("op", "(")
        while True:
            k = p.expect("id")
            p.expect("op", "=")
            options[k] = p.literal()
            if not p.accept("op", ","):
                break
        p.expect("op", ")")
    if p.peek() != (None, None):
        raise ValueError(f"trailing tokens: {p.t[p.i:]}")
    if group_by and any(s.kind == "AGG" and s.agg.filter is not None for s in select):
        # QueryContext.generateAggregationFunctions (QueryContext.java:531-533)
        raise ValueError("GROUP BY with FILTER clauses is not supported")
    return QueryContext(table, select, filt, group_by, order_by, limit, options, having)


def _resolve_having(f: HavingFilter, select: List[SelectItem], group_by: List[str]) -> HavingFilter:
    """A HAVING identifier is a select alias (of an aggregation or a key) or a group-by column (the reference's
    QueryContext resolves aliases the same way before the reduce)."""
    aliases = {s.alias: s for s in select if s.alias}

    def expr(e: HavingExpr) -> HavingExpr:
        if e.kind == "COL":
            s = aliases.get(e.column)
            if s is not None:
                return HavingExpr("AGG", agg=s.agg) if s.kind == "AGG" else HavingExpr("COL", column=s.column)
            if e.column not in group_by:
                raise ValueError(f"HAVING column {e.column} is neither a group-by column nor a select alias")
            return e
        if e.kind == "ARITH":
            return HavingExpr("ARITH", op=e.op, args=tuple(expr(a) for a in e.args))
        return e

    if f.type == "PREDICATE":
        return HavingFilter("PREDICATE", lhs=expr(f.lhs), predicate=f.predicate)
    return HavingFilter(f.type, [_resolve_having(c, select, group_by) for c in f.children])
