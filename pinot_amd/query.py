"""Query model of the path: the subset of Pinot's QueryContext that reaches the per-segment group-by operator.

Mirrors (names and meaning):
  Predicate / FilterContext   pinot-core .../query/request/context/predicate/*, FilterContext (AND / OR /
                              PREDICATE; NOT is accepted too)
  QueryContext                core/query/request/context/QueryContext.java:164-317 (filter, group-by
                              expressions, aggregation functions, numGroupsLimit)
A small parser for the SQL/PQL subset the reference tests use (comparisons, BETWEEN, IN / NOT IN, AND / OR /
NOT, GROUP BY, TOP / LIMIT / ORDER BY accepted and ignored: trimming and ordering are broker-side) turns
strings such as the README AdAnalytics query into a QueryContext.  Literals stay strings: they are converted
per column type by the dictionary lookup, exactly as PredicateUtils.getStoredValue does.
"""
import ctypes
import re
import time

from . import _lib as L

EQ, NOT_EQ, IN, NOT_IN, RANGE = "EQ", "NOT_EQ", "IN", "NOT_IN", "RANGE"
UNBOUNDED = "*"  # RangePredicate.UNBOUNDED
_PRED_CODE = {EQ: L.PRED_EQ, NOT_EQ: L.PRED_NOT_EQ, IN: L.PRED_IN, NOT_IN: L.PRED_NOT_IN, RANGE: L.PRED_RANGE}
AGG_FUNCTIONS = {"COUNT": L.AGG_COUNT, "SUM": L.AGG_SUM, "MIN": L.AGG_MIN, "MAX": L.AGG_MAX, "AVG": L.AGG_AVG}
DEFAULT_NUM_GROUPS_LIMIT = 100000  # InstancePlanMakerImplV2.DEFAULT_NUM_GROUPS_LIMIT (:70)
DEFAULT_LIMIT = 10  # QueryContext default LIMIT / TOP
DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE = 5000  # InstancePlanMakerImplV2.DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE
DEFAULT_GROUP_TRIM_THRESHOLD = 1000000  # InstancePlanMakerImplV2.DEFAULT_GROUPBY_TRIM_THRESHOLD


class Predicate:
    def __init__(self, ptype, column, values, lower_inclusive=True, upper_inclusive=True):
        self.type = ptype
        self.column = column
        self.values = [str(v) for v in values]
        self.lower_inclusive = bool(lower_inclusive)
        self.upper_inclusive = bool(upper_inclusive)

    @staticmethod
    def eq(col, v):
        return Predicate(EQ, col, [v])

    @staticmethod
    def not_eq(col, v):
        return Predicate(NOT_EQ, col, [v])

    @staticmethod
    def in_(col, vals):
        return Predicate(IN, col, list(vals))

    @staticmethod
    def not_in(col, vals):
        return Predicate(NOT_IN, col, list(vals))

    @staticmethod
    def range(col, lower=UNBOUNDED, upper=UNBOUNDED, lower_inclusive=True, upper_inclusive=True):
        return Predicate(RANGE, col, [lower, upper], lower_inclusive, upper_inclusive)

    def __repr__(self):
        return "Predicate(%s %s %r)" % (self.column, self.type, self.values)


class FilterContext:
    AND, OR, NOT, PREDICATE = "AND", "OR", "NOT", "PREDICATE"

    def __init__(self, ftype, children=None, predicate=None):
        self.type = ftype
        self.children = children or []
        self.predicate = predicate

    @staticmethod
    def and_(*children):
        return FilterContext(FilterContext.AND, list(children))

    @staticmethod
    def or_(*children):
        return FilterContext(FilterContext.OR, list(children))

    @staticmethod
    def not_(child):
        return FilterContext(FilterContext.NOT, [child])

    @staticmethod
    def pred(p):
        return FilterContext(FilterContext.PREDICATE, predicate=p)

    def postfix(self, preds, ops):
        """Flattens to a postfix program (predicates numbered in left-to-right order)."""
        if self.type == FilterContext.PREDICATE:
            preds.append(self.predicate)
            ops.append((L.OP_PRED, len(preds) - 1))
        elif self.type == FilterContext.NOT:
            self.children[0].postfix(preds, ops)
            ops.append((L.OP_NOT, 0))
        else:
            for c in self.children:
                c.postfix(preds, ops)
            ops.append((L.OP_AND if self.type == FilterContext.AND else L.OP_OR, len(self.children)))


class QueryContext:
    def __init__(self, group_by, aggregations, filter=None, num_groups_limit=DEFAULT_NUM_GROUPS_LIMIT,
                 use_star_tree=True, select=None, order_by=None, limit=DEFAULT_LIMIT,
                 min_server_group_trim_size=DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE,
                 group_trim_threshold=DEFAULT_GROUP_TRIM_THRESHOLD, sql_group_by=False):
        self.filter = filter
        # queryOptions groupByMode=sql: GroupByOrderByCombineOperator (no 2 x numGroupsLimit inter-segment cap)
        self.sql_group_by = sql_group_by
        self.use_star_tree = use_star_tree  # debug option useStarTree (StarTreeUtils.java:51-59)
        self.group_by = list(group_by)
        self.aggregations = [(fn.upper(), col) for fn, col in aggregations]
        self.num_groups_limit = num_groups_limit
        # SQL-mode parts (QueryContext.getSelectExpressions / getOrderByExpressions / getLimit): the SELECT list as
        # ('col', name) / ('agg', FN, col), ORDER BY as [(expr, ascending)], LIMIT; the combine's trim options
        # (InstancePlanMakerImplV2.java:64-84)
        self.select = list(select) if select is not None else \
            [("col", c) for c in self.group_by] + [("agg", fn, col) for fn, col in self.aggregations]
        self.order_by = list(order_by or [])
        self.limit = limit
        self.min_server_group_trim_size = min_server_group_trim_size
        self.group_trim_threshold = group_trim_threshold
        # QueryContext.getEndTimeMs: absolute deadline (ms since the epoch), 0 = none (set_timeout)
        self.end_time_ms = 0
        # the executions record HIP timing events for GpuPlan.timing_us (PGPU_OPT_TIMING; off for serving)
        self.timing = False

    def set_timeout(self, timeout_ms):
        """End time = now + timeout_ms (the broker's arrival time + queryOptions timeoutMs,
        QueryContext.setEndTimeMs); None clears it.  Past it the GPU path raises QueryTimeoutError."""
        self.end_time_ms = 0 if timeout_ms is None else int(time.time() * 1000) + int(timeout_ms)
        return self

    def expr_ref(self, expr):
        """(kind, index) of a SELECT / ORDER BY expression over the result: (0, group-by position) or
        (1, aggregation position)."""
        if expr[0] == "col":
            return L.ORDER_GROUP_BY, self.group_by.index(expr[1])
        return L.ORDER_AGGREGATION, self.aggregations.index((expr[1].upper(), expr[2]))

    def sql_trim_c(self):
        """The SQL-mode combine / reduce options as pgpu_sql_trim (keepalive, struct)."""
        ob = (L.OrderByC * max(len(self.order_by), 1))()
        for i, (e, asc) in enumerate(self.order_by):
            ob[i].kind, ob[i].index = self.expr_ref(e)
            ob[i].ascending = int(asc)
        sel = (L.OrderByC * max(len(self.select), 1))()
        for i, e in enumerate(self.select):
            sel[i].kind, sel[i].index = self.expr_ref(e)
        t = L.SqlTrimC(len(self.order_by), ob, self.limit, self.min_server_group_trim_size, self.group_trim_threshold,
                       len(self.select), sel)
        return (ob, sel), t

    def columns(self):
        cols = []
        if self.filter is not None:
            preds = []
            self.filter.postfix(preds, [])
            cols += [p.column for p in preds]
        cols += self.group_by
        cols += [c for _, c in self.aggregations if c != "*"]
        out = []
        for c in cols:
            if c not in out:
                out.append(c)
        return out

    # ---- JSON form used by tests/golden/kat_sv.json
    @staticmethod
    def filter_from_json(j):
        if j is None:
            return None
        if "and" in j:
            return FilterContext.and_(*[QueryContext.filter_from_json(c) for c in j["and"]])
        if "or" in j:
            return FilterContext.or_(*[QueryContext.filter_from_json(c) for c in j["or"]])
        if "not" in j:
            return FilterContext.not_(QueryContext.filter_from_json(j["not"]))
        t = j["pred"]
        if t in (EQ, NOT_EQ):
            return FilterContext.pred(Predicate(t, j["col"], [j["value"]]))
        if t in (IN, NOT_IN):
            return FilterContext.pred(Predicate(t, j["col"], j["values"]))
        return FilterContext.pred(Predicate.range(j["col"], j["lower"], j["upper"], j.get("li", True), j.get("ui", True)))

    # ---- C ABI form
    def to_c(self, column_index):
        """Returns (QueryC, keepalive) for a table whose column name -> index map is `column_index`.  The ctypes
        form is built once per (query, table) and reused; options are refreshed on every call."""
        cache = self.__dict__.get("_c_cache")
        if cache is not None and cache[0] is column_index and cache[1] == self.num_groups_limit:
            q, keep = cache[2], cache[3]
            q.options = self._options()
            q.end_time_ms = getattr(self, "end_time_ms", 0)
            return q, keep
        q, keep = self._build_c(column_index)
        self._c_cache = (column_index, self.num_groups_limit, q, keep)
        return q, keep

    def _options(self):
        return (0 if getattr(self, "use_star_tree", True) else L.OPT_NO_STAR_TREE) | \
            (L.OPT_SQL_GROUP_BY if getattr(self, "sql_group_by", False) else 0) | \
            (L.OPT_NO_PLAN_CACHE if getattr(self, "no_plan_cache", False) else 0) | \
            (L.OPT_TIMING if getattr(self, "timing", False) else 0)

    def _build_c(self, column_index):
        keep = []
        preds, ops = [], []
        if self.filter is not None:
            self.filter.postfix(preds, ops)
        pc = (L.PredicateC * max(len(preds), 1))()
        for i, p in enumerate(preds):
            if p.column not in column_index:
                raise KeyError("unknown column %r" % p.column)
            vals = (ctypes.c_char_p * max(len(p.values), 1))(*[v.encode() for v in p.values])
            keep.append(vals)
            pc[i].type = _PRED_CODE[p.type]
            pc[i].column = column_index[p.column]
            pc[i].num_values = len(p.values)
            pc[i].values = ctypes.cast(vals, L.c_char_pp)
            pc[i].lower_inclusive = int(p.lower_inclusive)
            pc[i].upper_inclusive = int(p.upper_inclusive)
        oc = (L.FilterOpC * max(len(ops), 1))()
        for i, (o, a) in enumerate(ops):
            oc[i].op, oc[i].arg = o, a
        gb = (ctypes.c_int32 * max(len(self.group_by), 1))(*[column_index[c] for c in self.group_by])
        ac = (L.AggC * max(len(self.aggregations), 1))()
        for i, (fn, col) in enumerate(self.aggregations):
            if fn not in AGG_FUNCTIONS:
                raise L.UnsupportedQueryError(L.PGPU_ERR_UNSUPPORTED, "aggregation %s" % fn)
            ac[i].fn = AGG_FUNCTIONS[fn]
            ac[i].column = -1 if col == "*" else column_index[col]
        q = L.QueryC()
        q.num_predicates = len(preds)
        q.num_filter_ops = len(ops)
        q.predicates = pc
        q.filter = oc
        q.num_group_by = len(self.group_by)
        q.group_by = gb
        q.num_aggs = len(self.aggregations)
        q.aggs = ac
        q.num_groups_limit = self.num_groups_limit
        q.options = self._options()
        q.end_time_ms = getattr(self, "end_time_ms", 0)
        keep += [pc, oc, gb, ac]
        return q, keep


# ================================================================================ SQL / PQL subset parser
_TOKEN = re.compile(r"\s*(?:(?P<num>-?\d+(?:\.\d+)?(?:[eE][+-]?\d+)?)|(?P<str>'(?:[^']|'')*')|"
                    r"(?P<id>[A-Za-z_][A-Za-z0-9_.$]*|\"[^\"]+\")|(?P<op><=|>=|<>|!=|=|<|>|\(|\)|,|\*))")


def _tokenize(s):
    pos, out = 0, []
    s = s.strip().rstrip(";")
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            if s[pos:].strip() == "":
                break
            raise ValueError("cannot parse near %r" % s[pos:pos + 20])
        pos = m.end()
        if m.group("num") is not None:
            out.append(("lit", m.group("num")))
        elif m.group("str") is not None:
            out.append(("lit", m.group("str")[1:-1].replace("''", "'")))
        elif m.group("id") is not None:
            out.append(("id", m.group("id").strip('"')))
        else:
            out.append(("op", m.group("op")))
    return out


class _Parser:
    def __init__(self, sql):
        self.t = _tokenize(sql)
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def kw(self, *words):
        tok = self.peek()
        return tok[0] == "id" and tok[1].upper() in words

    def take(self, kind=None, value=None):
        tok = self.peek()
        if tok[0] is None or (kind and tok[0] != kind) or (value and str(tok[1]).upper() != value):
            raise ValueError("expected %s %s, got %r" % (kind, value, tok))
        self.i += 1
        return tok[1]

    def select_list_item(self):
        tok = self.peek()
        if tok[0] == "id" and self.peek(1) == ("op", "("):
            fn = self.take("id").upper()
            self.take("op", "(")
            col = "*" if self.peek() == ("op", "*") else None
            if col:
                self.take("op", "*")
            else:
                col = self.take("id")
            self.take("op", ")")
            return ("agg", fn, col)
        return ("col", self.take("id"))

    def select_list(self):
        items = []
        while True:
            items.append(self.select_list_item())
            if self.peek() == ("op", ","):
                self.take("op", ",")
                continue
            return items

    def literal(self):
        tok = self.peek()
        if tok[0] not in ("lit", "id"):
            raise ValueError("literal expected, got %r" % (tok,))
        self.i += 1
        return tok[1]

    def expr_or(self):
        kids = [self.expr_and()]
        while self.kw("OR"):
            self.take("id")
            kids.append(self.expr_and())
        return kids[0] if len(kids) == 1 else FilterContext.or_(*kids)

    def expr_and(self):
        kids = [self.expr_not()]
        while self.kw("AND"):
            self.take("id")
            kids.append(self.expr_not())
        return kids[0] if len(kids) == 1 else FilterContext.and_(*kids)

    def expr_not(self):
        if self.kw("NOT"):
            self.take("id")
            return FilterContext.not_(self.expr_not())
        if self.peek() == ("op", "("):
            self.take("op", "(")
            e = self.expr_or()
            self.take("op", ")")
            return e
        col = self.take("id")
        if self.kw("BETWEEN"):
            self.take("id")
            lo = self.literal()
            self.take("id", "AND")
            hi = self.literal()
            return FilterContext.pred(Predicate.range(col, lo, hi, True, True))
        negate = False
        if self.kw("NOT"):
            self.take("id")
            negate = True
        if self.kw("IN"):
            self.take("id")
            self.take("op", "(")
            vals = [self.literal()]
            while self.peek() == ("op", ","):
                self.take("op", ",")
                vals.append(self.literal())
            self.take("op", ")")
            return FilterContext.pred(Predicate.not_in(col, vals) if negate else Predicate.in_(col, vals))
        op = self.take("op")
        v = self.literal()
        if op == "=":
            return FilterContext.pred(Predicate.eq(col, v))
        if op in ("!=", "<>"):
            return FilterContext.pred(Predicate.not_eq(col, v))
        if op == ">":
            return FilterContext.pred(Predicate.range(col, v, UNBOUNDED, False, False))
        if op == ">=":
            return FilterContext.pred(Predicate.range(col, v, UNBOUNDED, True, False))
        if op == "<":
            return FilterContext.pred(Predicate.range(col, UNBOUNDED, v, False, False))
        if op == "<=":
            return FilterContext.pred(Predicate.range(col, UNBOUNDED, v, False, True))
        raise ValueError("unsupported operator %s" % op)


def parse_query(sql, num_groups_limit=DEFAULT_NUM_GROUPS_LIMIT):
    """Parses `SELECT cols / aggs FROM t [WHERE ...] [GROUP BY cols] [ORDER BY expr [ASC|DESC], ...]
    [TOP n | LIMIT n]`.  Aggregations that appear only in ORDER BY are computed as well (Pinot's hidden
    aggregations) but not selected."""
    p = _Parser(sql)
    p.take("id", "SELECT")
    items = p.select_list()
    p.take("id", "FROM")
    p.take("id")
    flt = None
    if p.kw("WHERE"):
        p.take("id")
        flt = p.expr_or()
    group_by = []
    if p.kw("GROUP"):
        p.take("id")
        p.take("id", "BY")
        group_by.append(p.take("id"))
        while p.peek() == ("op", ","):
            p.take("op", ",")
            group_by.append(p.take("id"))
    order_by, limit = [], DEFAULT_LIMIT
    if p.kw("ORDER"):
        p.take("id")
        p.take("id", "BY")
        while True:
            e = p.select_list_item()
            asc = True
            if p.kw("ASC", "DESC"):
                asc = p.take("id").upper() == "ASC"
            order_by.append((e if e[0] == "col" else ("agg", e[1], e[2]), asc))
            if p.peek() != ("op", ","):
                break
            p.take("op", ",")
    if p.kw("TOP", "LIMIT"):
        p.take("id")
        limit = int(p.take("lit"))
    select = [("col", it[1]) if it[0] == "col" else ("agg", it[1], it[2]) for it in items]
    aggs = []
    for e in [x for x in select if x[0] == "agg"] + [e for e, _ in order_by if e[0] == "agg"]:
        if (e[1], e[2]) not in aggs:
            aggs.append((e[1], e[2]))
    return QueryContext(group_by, aggs, flt, num_groups_limit, select=select, order_by=order_by, limit=limit)
