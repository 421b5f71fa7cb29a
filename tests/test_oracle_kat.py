"""Pin the CPU oracle against the reference's own known-answer tests (tests/golden/*.json)."""
import json
import os

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule

GOLD = os.path.join(os.path.dirname(__file__), "golden")
FN = {"avg": A.EK_AGG_AVG, "max": A.EK_AGG_MAX, "min": A.EK_AGG_MIN, "stddev": A.EK_AGG_STDDEV,
      "stddevs": A.EK_AGG_STDDEVS, "var": A.EK_AGG_VAR, "vars": A.EK_AGG_VARS, "sum": A.EK_AGG_SUM,
      "count": A.EK_AGG_COUNT, "count_star": A.EK_AGG_COUNT_STAR,
      "percentile_cont": A.EK_AGG_PERCENTILE_CONT, "percentile_disc": A.EK_AGG_PERCENTILE_DISC}
TYPES = {"i64": A.EK_COL_I64, "f64": A.EK_COL_F64}


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def _check(got, exp):
    if exp is None:
        assert got is None
        return
    t, v = exp
    if t == "i64":
        assert isinstance(got, int) and got == v
    else:
        assert isinstance(got, float) and got == v  # bit-exact: same IEEE ops as Go


@pytest.mark.parametrize("case", _load("kat_functions.json")["agg_exec"], ids=lambda c: c["case"])
def test_agg_exec_kat(oracle, case):
    for fname, exp in case["expect"].items():
        got = oracle.agg_exec(FN[fname], TYPES[case["type"]], case["values"], case["valid"])
        _check(got, exp)


@pytest.mark.parametrize("case", _load("kat_functions.json")["percentile"], ids=lambda c: c["case"])
def test_percentile_kat(oracle, case):
    for fname, exp in case["expect"].items():
        got = oracle.agg_exec(FN[fname], TYPES[case["type"]], case["values"], case["valid"], case["p"])
        _check(got, exp)


@pytest.mark.parametrize("case", _load("kat_functions.json")["median"], ids=lambda c: c["case"])
def test_median_kat(oracle, case):
    got = oracle.agg_exec(A.EK_AGG_MEDIAN, TYPES[case["type"]], case["values"])
    _check(got, case["expect"])


@pytest.mark.parametrize("case", _load("kat_functions.json")["project_agg"], ids=lambda c: c["case"])
def test_project_agg_kat(oracle, case):
    for fname, exp in case["expect"].items():
        got = oracle.agg_exec(FN[fname], TYPES[case["type"]], case["values"], case["valid"])
        _check(got, exp)


def test_percentile_bounds_errors(oracle):
    # stats v0.7.1 BoundsErr surfaced with the reference's messages (funcs_agg.go:326,362)
    with pytest.raises(ValueError, match="percentile exec with error: Input is outside of range."):
        oracle.agg_exec(A.EK_AGG_PERCENTILE_CONT, A.EK_COL_F64, [1.0, 2.0], None, 1.5)
    with pytest.raises(ValueError, match="Input is outside of range."):
        oracle.agg_exec(A.EK_AGG_PERCENTILE_DISC, A.EK_COL_F64, [1.0, 2.0], None, -0.1)
    # n == 1 returns the element before the bounds check (stats.Percentile)
    assert oracle.agg_exec(A.EK_AGG_PERCENTILE_CONT, A.EK_COL_F64, [7.0], None, 5.0) == 7.0


def test_alignment_kat(oracle):
    g = _load("kat_alignment.json")
    for c in g["cases"]:
        got = oracle.aligned_window_end(g["ts"], c["interval"], A.UNIT_BY_NAME[c["unit"]], g["tz_offset_s"])
        assert got == c["end"], c


def _stream_cols(s):
    rows = np.array(s["rows"], dtype=object)
    return [np.array(rows[:, 0], dtype=np.int64), np.array(rows[:, 1], dtype=np.int64),
            np.array(rows[:, 2], dtype=np.uint32), np.array(rows[:, 3], dtype=np.float64)]


SCHEMA = {"ts": "bigint", "size": "bigint", "color": "key", "temp": "float"}


@pytest.mark.parametrize("case", _load("kat_window_rules.json")["tests"], ids=lambda c: c["name"])
def test_window_rule_kat(oracle, case):
    g = _load("kat_window_rules.json")
    cols = _stream_cols(g["streams"][case["stream"]])
    rule = compile_rule(case["sql"], SCHEMA, is_event_time=case.get("event_time", True), late_tolerance_ms=1000, num_keys=4)
    run = oracle.run(rule.plan, cols)
    assert len(run.windows) == case["windows_out"]
    assert run.records_late == case["late"]
    outs = [(w, run.members[i]) for i, w in enumerate(run.windows) if len(w.keys) > 0]
    assert len(outs) == len(case["outputs"])
    where_sizes = cols[1]
    for (w, members), exp in zip(outs, case["outputs"]):
        kept = [int(m) for m in members]
        if "WHERE size > 2" in case["sql"]:
            kept = [m for m in kept if where_sizes[m] > 2]
        assert sorted(kept) == sorted(exp["members"])
        assert w.value(0, 0) == len(exp["members"])  # count(*)
        if "first_color" in exp:                     # collect(*)[0]->color
            assert cols[2][kept[0]] == exp["first_color"]
        if "window_start" in exp:
            assert w.start == exp["window_start"] and w.end == exp["window_end"]


# ------------------------------------------------------------------ processing time (mock clock)
@pytest.mark.parametrize("case", _load("kat_window_proc.json")["tests"], ids=lambda c: c["name"])
def test_processing_window_kat(oracle, case):
    """window_rule_test.go TestWindow (processing time) under the reference's mock clock: the rule opens at the first
    row's second, rows arrive at their timestamps, the run ends at the last row (eko_run_proc)."""
    g = _load("kat_window_proc.json")
    cols = _stream_cols(g["streams"][case["stream"]])
    rule = compile_rule(case["sql"], SCHEMA, is_event_time=False, num_keys=4, **case.get("options", {}))
    start = case.get("start_ms", int(cols[0][0]) // 1000 * 1000)
    run = oracle.run_proc(rule.plan, cols, start, case.get("end_ms", int(cols[0][-1])))
    assert len(run.windows) == case["windows_out"]
    for w, members, exp in zip(run.windows, run.members, case["windows"]):
        assert sorted(int(m) for m in members) == exp["members"]
        assert w.end == exp["window_end"]
        if "window_start" in exp:
            assert w.start == exp["window_start"]
        if "count" in exp:
            assert (w.value(0, 0) if len(w.keys) else None) == exp["count"]


# ------------------------------------------------------------------ STATEWINDOW (WindowV2Operator)
def test_state_window_kat(oracle):
    """window_v2_op_test.go:40-91 TestStateWindow: rows a = 1, 2, 6 under statewindow(a > 1, a > 5)."""
    g = _load("kat_state_window.json")
    for case in g["tests"]:
        a = np.array([r["a"] for r in case["rows"]], np.int64)
        rule = compile_rule(case["sql"].replace("stream", "demo"), {"a": "bigint"}, is_event_time=False)
        assert rule.plan.window_type == A.EK_WINDOW_STATE
        run = oracle.run(rule.plan, [a])
        assert len(run.windows) == len(case["windows"])
        for w, m, exp in zip(run.windows, run.members, case["windows"]):
            assert [int(a[i]) for i in m] == [r["a"] for r in exp["content"]]
            assert w.value(0, 0) == len(exp["content"])          # count(*)
            assert (w.start, w.end) == (A.EK_STATE_WINDOW_START_MS, A.EK_STATE_WINDOW_END_MS)


def test_state_window_reopen_chain(oracle):
    """A row that both opens and closes a window re-opens one at the next row (window_v2_op.go:122-144:
    `if canBegin && !s.onBegin`); a row closing a window it did not open does not. Expected content derived
    by reading StateWindowOp.exec (no reference fixture covers the chain)."""
    a = np.array([0, 7, 3, 9, 2, 6, 1], np.int64)
    rule = compile_rule("SELECT count(*), sum(a) FROM demo GROUP BY STATEWINDOW(a > 1, a > 5)", {"a": "bigint"},
                        is_event_time=False)
    run = oracle.run(rule.plan, [a])
    assert [list(map(int, m)) for m in run.members] == [[1], [2, 3], [4, 5]]
    assert [w.value(1, 0) for w in run.windows] == [7, 12, 8]


def test_state_window_processing_time_where_pushdown(oracle):
    """Processing time: WHERE is pushed below the STATEWINDOW (windowPlan.go:82-99, round 6): a row it drops never reaches
    the begin / emit conditions. The rule over the whole stream equals the WHERE-less rule over the rows WHERE keeps
    (members mapped back to input rows); a = 20 satisfies the emit condition but fails WHERE, so the window it would
    have closed stays open (the post-window filter would give two windows, 1 and 2 rows)."""
    a = np.array([3, 20, 4, 7, 0, 9, 20, 2, 6, 1], np.int64)
    rule = compile_rule("SELECT count(*) FROM demo WHERE a != 20 GROUP BY STATEWINDOW(a > 1, a > 5)", {"a": "bigint"},
                        is_event_time=False)
    bare = compile_rule("SELECT count(*) FROM demo GROUP BY STATEWINDOW(a > 1, a > 5)", {"a": "bigint"},
                        is_event_time=False)
    keep = np.nonzero(a != 20)[0]
    got = oracle.run(rule.plan, [a])
    exp = oracle.run(bare.plan, [a[keep]])
    assert [sorted(int(i) for i in m) for m in got.members] == [sorted(int(keep[i]) for i in m) for m in exp.members]
    assert [w.value(0, 0) for w in got.windows] == [w.value(0, 0) for w in exp.windows]
    assert [list(map(int, m)) for m in got.members][0] == [0, 2, 3]   # 3, 4, 7: the 20 between them is gone


# ------------------------------------------------------------------ v2 event-time sliding windows
def _v2_cols(case, t0=1541152480000):
    a = np.array([r["a"] for r in case["rows"]], np.int64)
    ts = np.array([t0 + r["dt_ms"] for r in case["rows"]], np.int64)
    return a, ts


@pytest.mark.parametrize("case", _load("kat_window_v2.json")["tests"], ids=lambda c: c["name"])
def test_window_v2_sliding_kat(oracle, case):
    """window_v2_event_op_test.go: the first emitted window holds exactly the reference's rows."""
    a, ts = _v2_cols(case)
    rule = compile_rule(case["sql"].replace("eventStream", "demo"), {"a": "bigint", "ts": "bigint"}, window_version="v2",
                        late_tolerance_ms=case.get("late_tolerance_ms", 0))
    run = oracle.run(rule.plan, [a, ts])
    assert len(run.windows) >= 1
    assert [int(a[i]) for i in run.members[0]] == [r["a"] for r in case["content"]]
    assert run.windows[0].value(0, 0) == len(case["content"])
    if "window" in case:
        t0 = 1541152480000
        assert (run.windows[0].start - t0, run.windows[0].end - t0) == (case["window"]["start_dt_ms"], case["window"]["end_dt_ms"])


def test_window_v2_delayed_reemission(oracle):
    """EventSlidingWindowOp drops the emitted delay prefix only when a later delay is still pending
    (window_v2_event_op.go:56-76: newIndex stays -1 when every queued delay is due), so a due delay is emitted again at
    every later watermark, its WindowRange ending at that watermark, until a newer trigger is queued. Hand-derived:
    SLIDINGWINDOW(ss, 1, 1) OVER (WHEN a = 1), lateTolerance 0, rows (ts s, a): (0, 1) (0.5, 0) (2.5, 0) (3, 0) (3.5, 1)
    (4, 0) (6, 0): the trigger at 0 is due at 1 s; watermarks 2.5, 3 and 3.5 re-emit it (window (-1 s, wm] over the
    scanner, which gc(wm - 2 s) has cut to ts > 0.5 s after watermark 2.5); the trigger at 3.5 (due 4.5) is queued at
    3.5, so that watermark drops the first entry, watermark 4 emits nothing and watermark 6 emits the second over
    (2.5 s, 6 s]."""
    t0 = 1541152480000
    rows = [(0, 1), (500, 0), (2500, 0), (3000, 0), (3500, 1), (4000, 0), (6000, 0)]
    a = np.array([r[1] for r in rows], np.int64)
    ts = np.array([t0 + r[0] for r in rows], np.int64)
    rule = compile_rule("SELECT count(*) FROM demo GROUP BY SLIDINGWINDOW(ss, 1, 1) OVER (WHEN a = 1)",
                        {"a": "bigint", "ts": "bigint"}, window_version="v2")
    run = oracle.run(rule.plan, [a, ts])
    got = [((w.start - t0), (w.end - t0), sorted(int(i) for i in m)) for w, m in zip(run.windows, run.members)]
    assert got == [(-1000, 2500, [0, 1, 2]), (-1000, 3000, [2, 3]), (-1000, 3500, [2, 3, 4]), (2500, 6000, [3, 4, 5, 6])]


def test_window_v2_sliding_left_open_and_arrival_cut(oracle):
    """v2 windows are (t - L, t] over the rows added so far: a row exactly L before the trigger is out, and so is a
    row with the trigger's ts released in the same watermark step after it; v1 keeps both (window_op.go:605-655)."""
    ts = np.array([0, 1000, 4000, 4000, 5000], np.int64) + 1541152480000
    a = np.array([1, 2, 3, 4, 5], np.int64)
    sql = "SELECT count(*), sum(a) FROM demo GROUP BY SLIDINGWINDOW(ss, 4) OVER (WHEN a = 3)"
    sch = {"a": "bigint", "ts": "bigint"}
    v2 = oracle.run(compile_rule(sql, sch, late_tolerance_ms=1000, window_version="v2").plan, [a, ts])
    v1 = oracle.run(compile_rule(sql, sch, late_tolerance_ms=1000).plan, [a, ts])
    assert [list(map(int, m)) for m in v2.members] == [[1, 2]]
    assert v2.windows[0].value(1, 0) == 5 and (v2.windows[0].start, v2.windows[0].end) == (ts[2] - 4000, ts[2])
    assert [list(map(int, m)) for m in v1.members] == [[0, 1, 2, 3]]


# ------------------------------------------------------------------ processing-time incremental windows (mock clock)
@pytest.mark.parametrize("case", _load("kat_inc_proc.json")["tests"], ids=lambda c: c["name"])
def test_inc_processing_window_kat(oracle, case):
    """window_inc_agg_op_test.go: TumblingWindowIncAggOp / SlidingWindowIncAggOp (OVER, delay) / HoppingWindowIncAggOp
    under the mock clock (eko_run_proc): windows, members, count(*) and the emitted last row."""
    rows = case["rows"]
    a = np.array([r[1] for r in rows], np.int64)
    ts = np.array([r[0] for r in rows], np.int64)
    rule = compile_rule(case["sql"].replace("stream", "demo"), {"a": "bigint", "ts": "bigint"}, is_event_time=False,
                        incremental=True, inc_unaligned=case.get("inc_unaligned", False))
    assert rule.plan.incremental == 1
    run = oracle.run_proc(rule.plan, [a, ts], 0, case["end_ms"])
    assert len(run.windows) == len(case["windows"])
    for w, members, exp in zip(run.windows, run.members, case["windows"]):
        m = sorted(int(x) for x in members)
        assert m == exp["members"]
        assert int(a[m[-1]]) == exp["last_a"]
        assert (w.start, w.end) == (exp["window_start"], exp["window_end"])
        assert w.value(0, 0) == exp["count"]


@pytest.mark.parametrize("case", _load("kat_v2_proc.json")["tests"], ids=lambda c: c["name"])
def test_v2_processing_sliding_kat(oracle, case):
    """window_v2_op_test.go: WindowV2Operator SlidingWindowOp (OVER, delay) under the clock (eko_run_proc)."""
    t0 = 1541152480000
    a = np.array([r[1] for r in case["rows"]], np.int64)
    ts = np.array([t0 + r[0] for r in case["rows"]], np.int64)
    rule = compile_rule(case["sql"].replace("stream", "demo"), {"a": "bigint", "ts": "bigint"}, is_event_time=False,
                        window_version="v2")
    assert rule.plan.window_version == 2
    run = oracle.run_proc(rule.plan, [a, ts], t0, t0 + case["end_ms"])
    assert len(run.windows) >= 1
    w, m, exp = run.windows[0], run.members[0], case["first_window"]
    assert [int(a[i]) for i in m] == exp["content_a"]
    assert (w.start - t0, w.end - t0) == (exp["window_start"], exp["window_end"])
    assert w.value(0, 0) == len(exp["content_a"])
