"""Incremental-aggregation windows (planOptimizeStrategy.enableIncrementalWindow): the CPU oracle pinned by the
reference's own tests (tests/golden/kat_incremental.json) and by the semantics of window_inc_agg_event_op.go /
funcs_inc_agg.go that the KATs do not reach (last-row nil, float sums, the window-creation rule)."""
import json
import os

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat_incremental.json")))
SCHEMA = {"ts": "bigint", "a": "bigint"}


def _kat_cols(case):
    z = KAT["zero_ms"]
    ts = [z + t for t in case["rows_ms"]] + [z + case["sentinel_ms"]]
    a = case["a"] + [-1]
    return [np.array(ts, np.int64), np.array(a, np.int64)]


@pytest.mark.parametrize("case", KAT["event_windows"], ids=lambda c: c["name"])
def test_event_window_kat(oracle, case):
    rule = compile_rule(case["sql"], SCHEMA, late_tolerance_ms=KAT["late_tolerance_ms"], incremental=True)
    run = oracle.run(rule.plan, _kat_cols(case))
    z = KAT["zero_ms"]
    assert len(run.windows) == len(case["expect"])
    for w, members, exp in zip(run.windows, run.members, case["expect"]):
        assert w.start - z == exp["start_ms"]
        if exp["end_ms"] is not None:   # null: the reference test's own WatermarkTuple timing is not reproduced
            assert w.end - z == exp["end_ms"]
        assert w.value(0, 0) == exp["count"]
        assert _kat_cols(case)[1][members[-1]] == exp["last_a"]   # the LastRow the reference reports


@pytest.mark.parametrize("case", KAT["functions"], ids=lambda c: c["fn"])
def test_inc_function_kat(oracle, case):
    sql = f"SELECT {case['fn']}(a) FROM demo GROUP BY TUMBLINGWINDOW(ss, 10)"
    rule = compile_rule(sql, SCHEMA, late_tolerance_ms=0, incremental=True)
    ts = np.array([1541152481000, 1541152482000, 1541152499000], np.int64)
    a = np.array(case["args"] + [0], np.int64)
    run = oracle.run(rule.plan, [ts, a])
    w = run.windows[0]
    t, v = case["expect"]
    got = w.value(0, 0)
    assert isinstance(got, int if t == "i64" else float) and got == v


def test_regular_path_when_an_aggregate_is_not_incremental(oracle):
    # rewriteIfIncAggStmt (planner.go:931-934): one non-incremental aggregate keeps the regular chain
    ts = np.array([1541152481000, 1541152482000, 1541152499000], np.int64)
    a = np.array([1, 4, 0], np.int64)
    sql = "SELECT sum(a), stddev(a) FROM demo GROUP BY TUMBLINGWINDOW(ss, 10)"
    inc = oracle.run(compile_rule(sql, SCHEMA, incremental=True).plan, [ts, a])
    reg = oracle.run(compile_rule(sql, SCHEMA).plan, [ts, a])
    assert inc.windows[0].rows() == reg.windows[0].rows()
    assert inc.windows[0].value(0, 0) == 5      # int64 sum (regular), not the float64 inc_sum


def test_last_row_nil_makes_the_field_nil(oracle):
    # incAggCal overwrites Fields per row; check=returnNilIfHasAnyNil yields nil at a nil row (function.go:155-170)
    schema = {"ts": "bigint", "k": "key", "a": "bigint"}
    sql = "SELECT k, count(a), sum(a), avg(a), max(a), count(*) FROM demo GROUP BY k, TUMBLINGWINDOW(ss, 10)"
    rule = compile_rule(sql, schema, num_keys=2, nullable=("a",), incremental=True)
    ts = np.array([1541152481000, 1541152482000, 1541152483000, 1541152484000, 1541152499000], np.int64)
    k = np.array([0, 0, 1, 1, 0], np.uint32)
    a = np.array([5, 0, 0, 7, 0], np.int64)
    va = np.array([1, 0, 0, 1, 1], np.uint8)
    run = oracle.run(rule.plan, [ts, k, a], [None, None, va])
    rows = run.windows[0].rows()
    assert rows[0] == (None, None, None, None, 2)          # key 0: last row nil
    assert rows[1] == (1, 7.0, 7.0, 7, 2)                   # key 1: nil row skipped, last row valid


def test_tumbling_row_at_the_trigger_time_is_dropped(oracle):
    # triggerWindow (window_inc_agg_event_op.go:130-137) opens a window only for ts > NextTriggerWindowTime:
    # a row exactly at the previous window's end joins no window
    sql = "SELECT count(*) FROM demo GROUP BY TUMBLINGWINDOW(ss, 10)"
    rule = compile_rule(sql, SCHEMA, incremental=True)
    base = 1541152440000                       # a minute boundary
    ts = np.array([base + 21000, base + 25000, base + 30000, base + 30000, base + 31000, base + 45000, base + 99000],
                  np.int64)
    run = oracle.run(rule.plan, [ts, np.zeros(len(ts), np.int64)])
    got = [(w.start - base, w.end - base, w.value(0, 0)) for w in run.windows]
    assert got == [(20000, 30000, 2), (30000, 40000, 1), (40000, 50000, 1)]
    reg = oracle.run(compile_rule(sql, SCHEMA).plan, [ts, np.zeros(len(ts), np.int64)])
    assert [w.value(0, 0) for w in reg.windows if len(w.keys)] == [2, 3, 1]   # the regular path keeps them


def test_misaligned_second_of_the_minute(oracle):
    # getAlignedWindowEndTime (window_op.go:194-227) maps second == interval to the interval's own end, so rows
    # in (M+10 s, M+11 s) open windows ending before them: with TUMBLINGWINDOW(ss,10) they join no window
    sql = "SELECT count(*) FROM demo GROUP BY TUMBLINGWINDOW(ss, 10)"
    rule = compile_rule(sql, SCHEMA, incremental=True)
    base = 1541152440000
    ts = np.array([base + 1000, base + 10500, base + 10900, base + 12000, base + 19000, base + 99000], np.int64)
    run = oracle.run(rule.plan, [ts, np.zeros(len(ts), np.int64)])
    got = [(w.start - base, w.end - base, w.value(0, 0)) for w in run.windows]
    assert got == [(0, 10000, 1), (10000, 20000, 2)]


def test_hopping_windows_open_at_rows(oracle):
    # a hop with no row opens no window; each window holds the rows processed after it opened
    sql = "SELECT count(*) FROM demo GROUP BY HOPPINGWINDOW(ss, 20, 5)"
    rule = compile_rule(sql, SCHEMA, incremental=True)
    base = 1541152440000
    ts = np.array([base + 21000, base + 26000, base + 27000, base + 41000, base + 99000], np.int64)
    run = oracle.run(rule.plan, [ts, np.zeros(len(ts), np.int64)])
    got = [(w.start - base, w.end - base, w.value(0, 0)) for w in run.windows]
    assert got == [(20000, 40000, 3), (25000, 45000, 3), (40000, 60000, 1)]


def test_count_window_blocks(oracle):
    # CountWindowIncAggOp (window_inc_agg_op.go:239-314): consecutive blocks of n rows, inc_* values
    schema = {"k": "key", "a": "bigint"}
    sql = "SELECT k, sum(a), avg(a) FROM demo GROUP BY k, COUNTWINDOW(3)"
    rule = compile_rule(sql, schema, is_event_time=False, timestamp=None, num_keys=2, incremental=True)
    k = np.array([0, 1, 0, 1, 1, 1, 0], np.uint32)
    a = np.array([1, 2, 4, 3, 5, 8, 9], np.int64)
    run = oracle.run(rule.plan, [k, a])
    assert [w.rows() for w in run.windows] == [{0: (5.0, 2.5), 1: (2.0, 2.0)}, {1: (16.0, 16.0 / 3)}]


def test_unsupported_incremental_shapes(oracle):
    ts = np.array([1541152481000], np.int64)
    for sql in ("SELECT count(*) FROM demo GROUP BY SLIDINGWINDOW(ss, 10, 2)",):
        with pytest.raises(RuntimeError, match="restated"):
            oracle.run(compile_rule(sql, SCHEMA, incremental=True).plan, [ts, np.zeros(1, np.int64)])


def test_where_filters_the_emitted_last_rows(oracle):
    """WHERE stays above the incremental window (FilterPlan over IncWindowPlan, planner.go:702-708; IncWindowPlan keeps
    the predicate, incAggPlan.go:76-78): FilterOp runs over the emitted collection (filter_operator.go:59-90), whose
    rows are each group's LAST row with the inc_* fields set (window_inc_agg_op.go:443-457). So a group is kept or
    dropped by its last row alone, and its aggregates still count every row of the window. Hand-derived: two 10 s
    windows, rows a = 5, 0, 3 (last 3 > 1: count 3, not 2) and a = 5, 3, 0 (last 0: no row); a last row that errors
    (a / 0) replaces the window with "run Where error: divided by zero"."""
    t0 = 1541152480000
    ts = np.array([t0, t0 + 1, t0 + 2, t0 + 10_000, t0 + 10_001, t0 + 10_002, t0 + 30_000], np.int64)
    a = np.array([5, 0, 3, 5, 3, 0, 0], np.int64)
    rule = compile_rule("SELECT count(*), sum(a) FROM demo WHERE a > 1 GROUP BY TUMBLINGWINDOW(ss, 10)", SCHEMA,
                        incremental=True)
    run = oracle.run(rule.plan, [ts, a])
    assert [len(w.keys) for w in run.windows[:2]] == [1, 0]
    assert run.windows[0].value(0, 0) == 3 and run.windows[0].value(1, 0) == 8.0
    rule = compile_rule("SELECT count(*) FROM demo WHERE 10 / a > 1 GROUP BY TUMBLINGWINDOW(ss, 10)", SCHEMA,
                        incremental=True)
    run = oracle.run(rule.plan, [ts, a])
    assert run.windows[0].status == A.EK_WIN_OK and len(run.windows[0].keys) == 1   # last a = 3: 10 / 3 = 3 > 1
    assert run.windows[1].status == A.EK_WIN_WHERE_ERROR
    assert run.errors[1] == "run Where error: divided by zero"


def test_inc_sliding_clones_the_oldest_open_window(oracle):
    """SlidingWindowIncAggEventOp emits a clone of CurrWindowList[0] (the OLDEST open window), not the window the
    trigger row opened (window_inc_agg_event_op.go:257-272): with Length 1 s and rows at +0, +0.6, +1.2 s (all
    triggers), the +1.2 s row is released before the watermark that would drop the +0 window, so its clone is the
    +0 window: rows +0 and +0.6 only (the +1.2 row is outside [+0, +1 s)). Counts 1, 2, 2; sums 1, 3, 3."""
    t0 = 1541152480000
    ts = np.array([t0, t0 + 600, t0 + 1200, t0 + 9000], np.int64)
    a = np.array([1, 2, 3, 0], np.int64)
    run = oracle.run(compile_rule("SELECT count(*), sum(a) FROM demo GROUP BY SLIDINGWINDOW(ss, 1)", SCHEMA,
                                  incremental=True).plan, [ts, a])
    assert [w.value(0, 0) for w in run.windows[:3]] == [1, 2, 2]
    assert [w.value(1, 0) for w in run.windows[:3]] == [1.0, 3.0, 3.0]    # inc_sum is float64
    assert [w.start for w in run.windows[:3]] == [t0, t0 + 600, t0 + 1200]
