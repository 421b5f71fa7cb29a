"""Compile the rule SQL of a windowed GROUP BY into an ek_plan.

Host-side mirror of the pieces of the reference front-end that feed the hot path:
  * xsql parser for the window literal        internal/xsql/parser.go:926-975,1047-1153
  * un-aliased aggregate field naming          internal/xsql/parser.go:479,504-509 (name = function name)
  * planner window config (RawInterval, units) internal/topo/planner/planner.go:387-426,463-478
  * rule options isEventTime / lateTolerance   internal/pkg/def/rule.go:27-66

Supported subset (everything the BASELINE configs and the reference's window tests use):
  SELECT <key | agg(col | arithmetic over columns) | count(*) | window_start() | window_end()> [AS alias], ...
  FROM <stream> [WHERE <expr>]
  GROUP BY [<key>,] TUMBLINGWINDOW|HOPPINGWINDOW|SLIDINGWINDOW|SESSIONWINDOW|COUNTWINDOW(...)
           [FILTER (WHERE <expr>)] [OVER (WHEN <expr>)]
  [HAVING <expr>]
Expressions: comparisons, AND/OR, + - * / %, numeric literals, column refs, aggregate calls (HAVING).
GROUP BY dimensions: one dictionary-encoded key column (type "key") goes to the engine as is; any other set of
dimensions (several columns, bigint / float / string columns) is grouped through a host dictionary of the
reference's %v-concatenated key (ekgpu/keys.py, aggregate_operator.go:49-56) that fills a synthetic key column
`__group_key` (CompiledRule.device_columns / decode_keys). String columns travel as dense u32 codes and may only be
GROUP BY dimensions.
"""
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import abi as A
from .keys import GroupKeyDict, OrderedStringDict, StringDict

_TOKEN = re.compile(r"\s*(?:(\d+\.\d*|\.\d+|\d+(?:[eE][-+]?\d+)?)|([A-Za-z_][A-Za-z0-9_.]*)|(<=|>=|!=|<>|[=<>(),*+\-/%])|(\"[^\"]*\"|'[^']*'))")

WINDOW_TYPES = {
    "tumblingwindow": A.EK_WINDOW_TUMBLING,
    "hoppingwindow": A.EK_WINDOW_HOPPING,
    "slidingwindow": A.EK_WINDOW_SLIDING,
    "sessionwindow": A.EK_WINDOW_SESSION,
    "countwindow": A.EK_WINDOW_COUNT,
    "statewindow": A.EK_WINDOW_STATE,
}
_CMP = {"=": A.EK_OP_EQ, "!=": A.EK_OP_NEQ, "<>": A.EK_OP_NEQ, "<": A.EK_OP_LT, "<=": A.EK_OP_LTE,
        ">": A.EK_OP_GT, ">=": A.EK_OP_GTE}
_ADD = {"+": A.EK_OP_ADD, "-": A.EK_OP_SUB}
_MUL = {"*": A.EK_OP_MUL, "/": A.EK_OP_DIV, "%": A.EK_OP_MOD}
COLTYPES = {"bigint": A.EK_COL_I64, "float": A.EK_COL_F64, "key": A.EK_COL_U32, "string": A.EK_COL_U32,
            "boolean": A.EK_COL_BOOL}
GROUP_KEY = "__group_key"


class RuleError(ValueError):
    pass


@dataclass
class OutputField:
    name: str
    kind: str            # "key" | "agg" | "window_start" | "window_end"
    slot: int = -1


@dataclass
class CompiledRule:
    plan: A.ek_plan
    columns: List[str]
    fields: List[OutputField]
    sql: str
    options: Dict = field(default_factory=dict)

    group_dims: List[str] = field(default_factory=list)       # composite GROUP BY dimensions (host dictionary)
    key_dict: Optional[GroupKeyDict] = None
    string_dicts: Dict[str, StringDict] = field(default_factory=dict)
    schema: Dict[str, str] = field(default_factory=dict)

    def column_index(self, name: str) -> int:
        return self.columns.index(name)

    def device_columns(self, cols, validity=None):
        """Columns in the caller's schema order (string columns as python strings) -> the plan's columns: string
        columns as their dictionary codes, plus `__group_key` from the GROUP BY dimensions when composite.
        Returns (cols, validity)."""
        user = [c for c in self.columns if c != GROUP_KEY]
        if len(cols) != len(user):
            raise ValueError(f"expected {len(user)} columns ({user}), got {len(cols)}")
        validity = list(validity) if validity is not None else [None] * len(cols)
        out = []
        vout = list(validity)
        for j, (name, c) in enumerate(zip(user, cols)):
            if name not in self.string_dicts:
                out.append(c)
                continue
            # a nil string (None, or validity 0) is not a dictionary entry: placeholder code, validity 0
            nil = np.fromiter((s is None for s in c), dtype=bool, count=len(c))
            if nil.any():
                if not (self.plan.nullable_mask >> self.columns.index(name)) & 1:
                    raise ValueError(f"string column {name!r} holds nil values but is not declared nullable")
                v = np.ones(len(c), np.uint8) if validity[j] is None else np.array(validity[j], np.uint8)
                v[nil] = 0
                vout[j] = v
            out.append(self.string_dicts[name].encode(c, vout[j]))
        if self.key_dict is not None:
            idx = [user.index(d) for d in self.group_dims]
            out.append(self.key_dict.encode([cols[i] for i in idx], [validity[i] for i in idx]))
            vout.append(None)
        return out, (vout if any(v is not None for v in vout) else None)

    def decode_value(self, slot: int, values, tags) -> list:
        """Result values of aggregate slot `slot` -> python values: a first-row field over a string column is a
        dictionary code mapped back to its string; nil -> None."""
        fn, c = self.plan.aggs[slot].fn, self.plan.aggs[slot].column
        name = self.columns[c] if 0 <= c < len(self.columns) else None
        out = []
        for v, t in zip(values, tags):
            if t == A.EK_TAG_NULL:
                out.append(None)
            elif fn in (A.EK_AGG_FIRST, A.EK_AGG_MIN, A.EK_AGG_MAX) and name in self.string_dicts:
                out.append(self.string_dicts[name].values[int(v)])
            else:
                out.append(v)
        return out

    def decode_keys(self, keys) -> list:
        """Result key ids -> the GROUP BY dimension values (the group's first row), as tuples."""
        if self.key_dict is not None:
            return self.key_dict.decode(keys)
        return [(int(k),) for k in keys]


def _tokenize(sql: str) -> List[str]:
    pos, out = 0, []
    sql = sql.strip().rstrip(";")
    while pos < len(sql):
        m = _TOKEN.match(sql, pos)
        if not m or m.end() == pos:
            if sql[pos:].strip() == "":
                break
            raise RuleError(f"unexpected character at {pos}: {sql[pos:pos + 10]!r}")
        tok = next(g for g in m.groups() if g is not None)
        out.append(tok)
        pos = m.end()
    return out


class _Parser:
    def __init__(self, sql: str, schema: Dict[str, str]):
        self.toks = _tokenize(sql)
        self.i = 0
        self.schema = {k.lower(): (k, v) for k, v in schema.items()}
        self.columns = list(schema.keys())
        self.aggs: List[Tuple[int, int, float]] = []
        self.derived: List[Tuple[Tuple, str]] = []

    # token helpers
    def peek(self, k: int = 0) -> Optional[str]:
        j = self.i + k
        return self.toks[j] if j < len(self.toks) else None

    def kw(self, word: str) -> bool:
        t = self.peek()
        if t is not None and t.lower() == word:
            self.i += 1
            return True
        return False

    def expect(self, tok: str):
        t = self.peek()
        if t is None or t.lower() != tok.lower():
            raise RuleError(f"expected {tok!r} but found {t!r}")
        self.i += 1

    def col(self, name: str) -> int:
        ent = self.schema.get(name.lower().split(".")[-1])
        if ent is None:
            raise RuleError(f"unknown field {name}")
        return self.columns.index(ent[0])

    def agg_slot(self, fn: int, col: int, p: float) -> int:
        key = (fn, col, p)
        if key not in self.aggs:
            if len(self.aggs) >= A.EK_MAX_AGGS:
                raise RuleError("too many aggregate calls")
            self.aggs.append(key)
        return self.aggs.index(key)

    # aggregate call: name '(' args ')'
    def parse_agg(self, name: str) -> int:
        name = name.lower()
        self.expect("(")
        if name == "count" and self.peek() == "*":
            self.i += 1
            self.expect(")")
            return self.agg_slot(A.EK_AGG_COUNT_STAR, -1, 0.0)
        prog = self.add(False)   # the argument: a column or an arithmetic expression over columns
        c = prog[0][1] if len(prog) == 1 and prog[0][0] == A.EK_OP_COL else self.derived_col(prog)
        p = 0.0
        if self.peek() == ",":
            self.i += 1
            p = float(self.peek())
            self.i += 1
        self.expect(")")
        return self.agg_slot(A.AGG_BY_NAME[name], c, p)

    # aggregate argument expressions -> derived columns (GroupedTuples.AggregateEval, row.go:712-718)
    def derived_col(self, prog: List[Tuple]) -> int:
        types = []
        for k, ins in enumerate(prog):
            op = ins[0]
            if op == A.EK_OP_COL:
                t = self.schema[self.columns[ins[1]].lower()][1]
                if t == "boolean":
                    raise RuleError("aggregate arguments are arithmetic over numeric columns")
                types.append("float" if t == "float" else "int")
            elif op == A.EK_OP_CONST_I64:
                types.append("int")
            elif op == A.EK_OP_CONST_F64:
                types.append("float")
            elif op in (A.EK_OP_ADD, A.EK_OP_SUB, A.EK_OP_MUL, A.EK_OP_DIV, A.EK_OP_MOD):
                if op in (A.EK_OP_DIV, A.EK_OP_MOD):
                    r = prog[k - 1]
                    if r[0] not in (A.EK_OP_CONST_I64, A.EK_OP_CONST_F64) or r[1] == 0:
                        raise RuleError("an aggregate argument may divide only by a non-zero constant "
                                        "(a zero divisor is a per-row evaluation error)")
                b, a = types.pop(), types.pop()
                # valuer.go:861-1000: int64 op int64 stays int64 (integer division), a float64 operand promotes
                types.append("float" if "float" in (a, b) else "int")
            else:
                raise RuleError("aggregate arguments are arithmetic over columns and constants")
        key = (tuple(prog), types[-1])
        if key not in self.derived:
            if len(self.derived) >= A.EK_MAX_DERIVED:
                raise RuleError("too many expression arguments")
            if len(self.columns) + len(self.derived) >= A.EK_MAX_COLUMNS:
                raise RuleError("too many columns")
            self.derived.append(key)
        return len(self.columns) + self.derived.index(key)

    # expressions -> postfix program
    def expr(self, allow_agg: bool) -> List[Tuple]:
        return self.or_(allow_agg)

    def or_(self, aa):
        prog = self.and_(aa)
        while self.kw("or"):
            prog = prog + self.and_(aa) + [(A.EK_OP_OR,)]
        return prog

    def and_(self, aa):
        prog = self.cmp(aa)
        while self.kw("and"):
            prog = prog + self.cmp(aa) + [(A.EK_OP_AND,)]
        return prog

    def cmp(self, aa):
        prog = self.add(aa)
        t = self.peek()
        if t in _CMP:
            self.i += 1
            prog = prog + self.add(aa) + [(_CMP[t],)]
        return prog

    def add(self, aa):
        prog = self.mul(aa)
        while self.peek() in _ADD:
            op = _ADD[self.peek()]
            self.i += 1
            prog = prog + self.mul(aa) + [(op,)]
        return prog

    def mul(self, aa):
        prog = self.prim(aa)
        while self.peek() in _MUL:
            op = _MUL[self.peek()]
            self.i += 1
            prog = prog + self.prim(aa) + [(op,)]
        return prog

    def prim(self, aa):
        t = self.peek()
        if t is None:
            raise RuleError("unexpected end of expression")
        if t == "(":
            self.i += 1
            prog = self.expr(aa)
            self.expect(")")
            return prog
        if t == "-" and self.peek(1) and re.match(r"[\d.]", self.peek(1)):
            self.i += 1
            v = self.peek()
            self.i += 1
            return [self._num("-" + v)]
        if t == "-":        # unary minus on a column or sub-expression: x * -1 (keeps int64 int64, flips a float's sign)
            self.i += 1
            return self.prim(aa) + [(A.EK_OP_CONST_I64, -1), (A.EK_OP_MUL,)]
        if re.match(r"[\d.]", t):
            self.i += 1
            return [self._num(t)]
        if t.lower() in ("true", "false"):   # ast.BooleanLiteral
            self.i += 1
            return [(A.EK_OP_CONST_BOOL, 1 if t.lower() == "true" else 0)]
        self.i += 1
        if self.peek() == "(":
            if not aa or t.lower() not in A.AGG_BY_NAME:
                raise RuleError(f"function {t} is not supported here")
            return [(A.EK_OP_AGG, self.parse_agg(t))]
        return [(A.EK_OP_COL, self.col(t))]

    @staticmethod
    def _num(s: str):
        if re.fullmatch(r"-?\d+", s):
            return (A.EK_OP_CONST_I64, int(s))
        return (A.EK_OP_CONST_F64, float(s))


def _fill_prog(dst, prog: List[Tuple]) -> int:
    if len(prog) > A.EK_MAX_PROG:
        raise RuleError("expression too long")
    depth = top = 0   # the device evaluates with an 8-value register stack (ek_device.h EvalStack)
    for ins in prog:
        top += 1 if ins[0] in (A.EK_OP_COL, A.EK_OP_AGG, A.EK_OP_CONST_I64, A.EK_OP_CONST_F64, A.EK_OP_CONST_BOOL) else -1
        depth = max(depth, top)
    if depth > 8:
        raise RuleError("expression nests too deeply (more than 8 pending operands)")
    for k, ins in enumerate(prog):
        dst[k].op = ins[0]
        if ins[0] in (A.EK_OP_COL, A.EK_OP_AGG):
            dst[k].arg = ins[1]
        elif ins[0] in (A.EK_OP_CONST_I64, A.EK_OP_CONST_BOOL):
            dst[k].i64 = ins[1]
            dst[k].f64 = float(ins[1])
        elif ins[0] == A.EK_OP_CONST_F64:
            dst[k].f64 = ins[1]
    return len(prog)


def compile_rule(sql: str, schema: Dict[str, str], *, is_event_time: bool = True, late_tolerance_ms: int = 0,
                 timestamp: Optional[str] = "ts", num_keys: int = 0, tz_offset_s: int = 0,
                 debug_membership: bool = False, nullable=(), incremental: bool = False,
                 window_version: str = "", sliding_send_twice: bool = False, inc_unaligned: bool = False) -> CompiledRule:
    """schema: ordered {column: "bigint" | "float" | "key" | "string"}; the TIMESTAMP column must be bigint (epoch
    ms). A GROUP BY other than one key column adds the synthetic `__group_key` column (see the module docstring).
    sliding_send_twice: the rule option planOptimizeStrategy.windowOption.enableSendSlidingWindowTwice
    (def/rule.go:104-112): a delayed SLIDINGWINDOW emits its first part at the trigger and its second part when the
    delay expires (window_op.go:98,355-373, event_window_trigger.go:156-161); no effect on other windows.
    inc_unaligned: node.EnableAlignWindow = false (the reference's tests): processing-time incremental TUMBLING /
    HOPPING tick from the rule's start (window_inc_agg_op.go:369-377,693-699)."""
    rule = _compile_rule(sql, schema, is_event_time=is_event_time, late_tolerance_ms=late_tolerance_ms,
                         timestamp=timestamp, num_keys=num_keys, tz_offset_s=tz_offset_s,
                         debug_membership=debug_membership, nullable=nullable, incremental=incremental,
                         window_version=window_version)
    # window_op.go:98: the option only holds for a sliding window with a delay
    rule.plan.sliding_send_twice = 1 if (sliding_send_twice and rule.plan.window_type == A.EK_WINDOW_SLIDING and
                                         rule.plan.delay > 0) else 0
    rule.options.setdefault("planOptimizeStrategy", {}).setdefault("windowOption", {})[
        "enableSendSlidingWindowTwice"] = bool(sliding_send_twice)
    rule.plan.inc_unaligned = 1 if inc_unaligned else 0
    return rule


def _compile_rule(sql, schema, **kw) -> CompiledRule:
    num_keys = kw["num_keys"]
    try:
        return _compile(sql, dict(schema), **kw)
    except _Composite as c:
        if GROUP_KEY in schema:
            raise RuleError(f"column name {GROUP_KEY} is reserved")
        rule = _compile(sql, dict(schema, **{GROUP_KEY: "key"}), group_dims=c.dims, **kw)
        rule.key_dict = GroupKeyDict(c.dims, [schema[d] for d in c.dims], num_keys)
        return rule


class _Composite(Exception):
    def __init__(self, dims):
        self.dims = dims


def _compile(sql: str, schema: Dict[str, str], *, is_event_time: bool, late_tolerance_ms: int,
             timestamp: Optional[str], num_keys: int, tz_offset_s: int, debug_membership: bool, nullable,
             incremental: bool, window_version: str, group_dims: Optional[List[str]] = None) -> CompiledRule:
    if len(schema) > A.EK_MAX_COLUMNS:
        raise RuleError("too many columns")
    p = _Parser(sql, schema)
    plan = A.ek_plan()
    plan.abi_version = A.EKGPU_ABI_VERSION
    plan.n_columns = len(schema)
    for k, (name, t) in enumerate(schema.items()):
        if t not in COLTYPES:
            raise RuleError(f"unsupported column type {t}")
        plan.column_type[k] = COLTYPES[t]
    plan.is_event_time = 1 if is_event_time else 0
    plan.late_tolerance_ms = int(late_tolerance_ms)
    plan.tz_offset_s = int(tz_offset_s)
    plan.ts_column = p.col(timestamp) if (timestamp and is_event_time) else -1
    plan.key_column = -1
    plan.num_keys = int(num_keys)
    plan.debug_membership = 1 if debug_membership else 0
    # def.RuleOption.PlanOptimizeStrategy.EnableIncrementalWindow (def/rule.go:55-61); the engine applies the
    # planner's own eligibility test (planner.go:910-1017) and keeps the regular path when it fails
    plan.incremental = 1 if incremental else 0
    # planOptimizeStrategy.windowOption.windowVersion (def/rule.go:68-76; planner.go:416-425)
    plan.window_version = 2 if window_version == "v2" else 0
    plan.nullable_mask = 0
    for name in nullable:
        plan.nullable_mask |= 1 << p.col(name)

    p.expect("select")
    fields: List[OutputField] = []
    raw_select = []
    while True:
        start = p.i
        t = p.peek()
        if t is None:
            raise RuleError("unexpected end of select list")
        if t == "*":
            p.i += 1
            for c, name in enumerate(p.columns):
                raw_select.append(OutputField(name, "column", c))
            if p.peek() == ",":
                p.i += 1
                continue
            break
        if p.peek(1) == "(" and t.lower() in ("window_start", "window_end"):
            p.i += 3
            name, kind, slot = t.lower(), t.lower(), -1
        elif p.peek(1) == "(" and t.lower() in A.AGG_BY_NAME:
            p.i += 1
            slot = p.parse_agg(t)
            name, kind = t.lower(), "agg"
        else:
            p.i += 1
            name, kind, slot = t.split(".")[-1], "column", p.col(t)
        if p.kw("as"):
            name = p.peek()
            p.i += 1
        raw_select.append(OutputField(name, kind, slot))
        if p.peek() == ",":
            p.i += 1
            continue
        break
    p.expect("from")
    p.i += 1  # stream name
    where = []
    if p.kw("where"):
        where = p.expr(False)
    key_col = -1
    dims: List[str] = []
    trigger = []
    wfilter = []
    begin, emit = [], []
    wtype = A.EK_WINDOW_NONE
    if p.kw("group"):
        p.expect("by")
        while True:
            t = p.peek()
            if t is not None and t.lower() in WINDOW_TYPES:
                wtype = WINDOW_TYPES[t.lower()]
                p.i += 1
                p.expect("(")
                nums = []
                if wtype == A.EK_WINDOW_STATE:
                    # STATEWINDOW(<begin condition>, <emit condition>) (parser.go:1047-1053,1119-1124)
                    begin = p.expr(False)
                    p.expect(",")
                    emit = p.expr(False)
                    p.expect(")")
                    if p.kw("filter"):   # the window's FILTER (WHERE <cond>) clause, as for the time windows below
                        p.expect("(")
                        p.expect("where")
                        wfilter = p.expr(False)
                        p.expect(")")
                    if p.peek() == ",":
                        p.i += 1
                        continue
                    break
                if wtype != A.EK_WINDOW_COUNT:
                    unit = p.peek().lower()
                    if unit not in A.UNIT_BY_NAME:
                        raise RuleError(f"invalid time unit {unit}")
                    plan.time_unit = A.UNIT_BY_NAME[unit]
                    p.i += 1
                while p.peek() == ",":
                    p.i += 1
                    nums.append(int(p.peek()))
                    p.i += 1
                if wtype == A.EK_WINDOW_COUNT and not nums:
                    nums.append(int(p.peek()))
                    p.i += 1
                    while p.peek() == ",":
                        p.i += 1
                        nums.append(int(p.peek()))
                        p.i += 1
                p.expect(")")
                if p.kw("filter"):
                    # the window's FILTER (WHERE <cond>) clause (parser.go: WindowPlan.condition, planner.go:388-392)
                    p.expect("(")
                    p.expect("where")
                    wfilter = p.expr(False)
                    p.expect(")")
                plan.length = nums[0] if nums else 0
                if wtype in (A.EK_WINDOW_HOPPING, A.EK_WINDOW_SESSION, A.EK_WINDOW_COUNT):
                    plan.interval = nums[1] if len(nums) > 1 else 0
                elif wtype == A.EK_WINDOW_SLIDING:
                    plan.delay = nums[1] if len(nums) > 1 else 0
                if p.kw("over"):
                    p.expect("(")
                    p.expect("when")
                    trigger = p.expr(False)
                    p.expect(")")
            else:
                dims.append(p.columns[p.col(t)])
                p.i += 1
            if p.peek() == ",":
                p.i += 1
                continue
            break
    if group_dims is not None:
        key_col = p.columns.index(GROUP_KEY)
    elif len(dims) == 1 and schema[dims[0]] == "key" and dims[0] not in nullable:
        key_col = p.columns.index(dims[0])
    # (a nullable key column goes through the group-key dictionary too: a nil dimension is the reference's own group
    # "<nil>," — aggregate_operator.go:49-55 — an id of its own, so the engine's key column never holds a nil)
    elif dims:
        raise _Composite(dims)
    having = []
    if p.kw("having"):
        having = p.expr(True)
    if p.peek() is not None:
        raise RuleError(f"unexpected token {p.peek()!r}")
    plan.window_type = wtype
    plan.key_column = key_col
    if not is_event_time and timestamp and wtype in (A.EK_WINDOW_TUMBLING, A.EK_WINDOW_HOPPING, A.EK_WINDOW_SLIDING,
                                                     A.EK_WINDOW_SESSION):
        # processing-time time windows: the TIMESTAMP column carries each row's arrival time (the timestamp the
        # reference stamps at ingest); the engine's clock reaches it before the row is delivered (ek_advance_time)
        plan.ts_column = p.col(timestamp)
    if wtype == A.EK_WINDOW_NONE:
        # window-less rule: FilterOp + projection of every column (SELECT *, the C1 shape)
        if p.aggs or key_col >= 0 or having:
            raise RuleError("aggregates and GROUP BY need a window (the GPU engine's hot path)")
        if [f.slot for f in raw_select] != list(range(len(p.columns))):
            raise RuleError("window-less rules project every column (SELECT *)")
        plan.n_where = _fill_prog(plan.where_prog, where)
        plan.is_event_time = 0
        plan.ts_column = -1
        fields = [OutputField(f.name, "column", f.slot) for f in raw_select]
        return CompiledRule(plan=plan, columns=list(schema.keys()), fields=fields, sql=sql,
                            options=dict(isEventTime=False, lateTolerance=0))
    for f in raw_select:
        if f.kind == "column":
            cname = p.columns[f.slot]
            if group_dims is not None and cname in group_dims:
                fields.append(OutputField(f.name, "dim", group_dims.index(cname)))
                continue
            if f.slot != key_col:
                # a non-aggregate, non-dimension field: the column's value in the group's first row (row.go:720-726);
                # lowered to the engine's EK_AGG_FIRST (range mode)
                if len(p.aggs) >= A.EK_MAX_AGGS:
                    raise RuleError("too many aggregate calls")
                p.aggs.append((A.EK_AGG_FIRST, f.slot, 0.0))
                fields.append(OutputField(f.name, "agg", len(p.aggs) - 1))
                continue
            fields.append(OutputField(f.name, "key"))
        else:
            fields.append(f)
    strings = {c for c, t in schema.items() if t == "string"}
    # string columns aggregated by min / max (common_array_funcs.go:49,86): order-preserving int64 codes
    # (OrderedStringDict), so the engine's integer min / max is the lexicographic one; first-row fields and count()
    # over a string column need only its codes / validity
    ordered = {p.columns[c] for (fn, c, _) in p.aggs
               if fn in (A.EK_AGG_MIN, A.EK_AGG_MAX) and 0 <= c < len(p.columns) and p.columns[c] in strings}
    for c in ordered:
        plan.column_type[p.columns.index(c)] = A.EK_COL_I64
    if strings:
        free = (A.EK_AGG_FIRST, A.EK_AGG_COUNT, A.EK_AGG_MIN, A.EK_AGG_MAX)
        used = {p.columns[c] for (fn, c, _) in p.aggs if c >= 0 and c < len(p.columns) and fn not in free}
        for prog in [where, having, trigger, wfilter, begin, emit] + [list(pr) for pr, _ in p.derived]:
            used |= {p.columns[ins[1]] for ins in prog if ins[0] == A.EK_OP_COL and ins[1] < len(p.columns)}
        if used & strings:
            raise RuleError(f"string column(s) {sorted(used & strings)} may only be GROUP BY dimensions, min / max / count arguments or first-row fields")
    plan.n_aggs = len(p.aggs)
    for k, (fn, c, prm) in enumerate(p.aggs):
        plan.aggs[k].fn = fn
        plan.aggs[k].column = c
        plan.aggs[k].param = prm if fn in (A.EK_AGG_PERCENTILE_CONT, A.EK_AGG_PERCENTILE_DISC) else 0.0
    plan.n_derived = len(p.derived)
    for d, (prog, t) in enumerate(p.derived):
        plan.derived_type[d] = A.EK_COL_F64 if t == "float" else A.EK_COL_I64
        plan.n_derived_prog[d] = _fill_prog(plan.derived_prog[d], list(prog))
    plan.n_where = _fill_prog(plan.where_prog, where)
    plan.n_having = _fill_prog(plan.having_prog, having)
    plan.n_trigger = _fill_prog(plan.trigger_prog, trigger)
    plan.n_filter = _fill_prog(plan.filter_prog, wfilter)
    plan.n_begin = _fill_prog(plan.begin_prog, begin)
    plan.n_emit = _fill_prog(plan.emit_prog, emit)
    if key_col >= 0 and num_keys <= 0:
        raise RuleError("num_keys (dictionary size of the GROUP BY key) is required")
    return CompiledRule(plan=plan, columns=list(schema.keys()), fields=fields, sql=sql,
                        group_dims=list(group_dims or []), schema=dict(schema),
                        string_dicts={c: (OrderedStringDict() if c in ordered else StringDict()) for c in strings},
                        options=dict(isEventTime=is_event_time, lateTolerance=late_tolerance_ms,
                                     planOptimizeStrategy=dict(enableIncrementalWindow=bool(incremental),
                                                               windowOption=dict(windowVersion=window_version))))
