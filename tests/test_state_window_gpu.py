"""GPU parity of the WindowV2Operator windows against the CPU oracle: STATEWINDOW(begin, emit) (StateWindowOp,
window_v2_op.go:94-148) and the event-time v2 sliding window (EventSlidingWindowOp, window_v2_event_op.go:78-96).
STATEWINDOW: the reference KAT (window_v2_op_test.go:40-91), the re-open chain, randomized processing-time and
event-time streams (out of order, late tolerance, WHERE above the window, HAVING, order statistics), split batches."""
import json
import os

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401  (fixture + helper)
from test_range_gpu import TRIG_SCHEMA, _iot, _with_trig

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_state_window_kat_engine(oracle, engine_mod):
    g = json.load(open(os.path.join(GOLD, "kat_state_window.json")))
    for case in g["tests"]:
        a = np.array([r["a"] for r in case["rows"]], np.int64)
        rule = compile_rule(case["sql"].replace("stream", "demo"), {"a": "bigint"}, is_event_time=False,
                            debug_membership=True)
        for batches in (1, len(a)):
            got, exp, _ = run_both(oracle, engine_mod, rule, [a], batches=batches)
            assert len(got) == len(case["windows"])
            assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
            assert got[0].value(0, 0) == len(case["windows"][0]["content"])


def test_state_window_reopen_chain_engine(oracle, engine_mod):
    a = np.array([0, 7, 3, 9, 2, 6, 1, 8, 8, 0, 2, 2, 7], np.int64)
    rule = compile_rule("SELECT count(*), sum(a), min(a) FROM demo GROUP BY STATEWINDOW(a > 1, a > 5)", {"a": "bigint"},
                        is_event_time=False, debug_membership=True)
    for batches in (1, 4, len(a)):
        got, exp, _ = run_both(oracle, engine_mod, rule, [a], batches=batches)
        assert len(got) == len(exp.windows) == 6
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("batches", [1, 13])
def test_state_window_processing_time(oracle, engine_mod, batches):
    sql = ("SELECT deviceId, count(*), sum(temperature), min(humidity), max(temperature), stddev(temperature) FROM demo "
           "GROUP BY deviceId, STATEWINDOW(trig = 1, humidity > 99)")
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=500, is_event_time=False, debug_membership=True)
    cols = _with_trig(_iot(200_000, 500, seed=91, epm=10), 400)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert len(got) > 100
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_state_window_order_statistics(oracle, engine_mod):
    sql = ("SELECT deviceId, median(temperature), percentile_disc(humidity, 0.25), count(*) FROM demo "
           "GROUP BY deviceId, STATEWINDOW(trig = 1, temperature > 99.8)")
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=300, is_event_time=False, debug_membership=True)
    cols = _with_trig(_iot(100_000, 300, seed=92, epm=10), 250)
    for batches in (1, 7):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert len(got) > 20
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("batches", [1, 9])
def test_state_window_event_time_out_of_order(oracle, engine_mod, batches):
    """Event time: rows reach the state window in WatermarkOp release order; WHERE stays above the window
    (windowPlan.go:82-99), HAVING after the aggregate."""
    sql = ("SELECT deviceId, count(*), avg(temperature), max(humidity) FROM demo WHERE temperature > 5 "
           "GROUP BY deviceId, STATEWINDOW(trig = 1, humidity > 98) HAVING count(*) > 1")
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=200, late_tolerance_ms=300, debug_membership=True)
    cols = _with_trig(_iot(60_000, 200, seed=93, epm=4), 200)
    rng = np.random.default_rng(11)
    cols[1] = (cols[1] + rng.integers(-500, 500, len(cols[1]))).astype(np.int64)
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert exp.records_late > 0 and st.records_late == exp.records_late
    assert len(got) > 20
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("batches", [1, 11])
@pytest.mark.parametrize("where", ["temperature > 20", "temperature / (humidity - 50) > 0.1"])
def test_state_window_processing_time_where_pushdown(oracle, engine_mod, batches, where):
    """Processing time: WHERE is pushed below the window (windowPlan.PushDownPredicate, windowPlan.go:82-99) and
    combined with the window FILTER into the FilterOp in front of it (planner.go:388-392): only the rows it keeps reach
    the begin / emit conditions (a row with humidity 50 makes the second WHERE fail: dropped and counted)."""
    sql = (f"SELECT deviceId, count(*), avg(temperature), max(humidity) FROM demo WHERE {where} "
           "GROUP BY deviceId, STATEWINDOW(trig = 1, humidity > 98) FILTER (WHERE humidity > 3) HAVING count(*) > 1")
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=300, is_event_time=False, debug_membership=True)
    cols = _with_trig(_iot(120_000, 300, seed=94, epm=10), 300)
    cols[3][::97] = 50.0   # humidity 50: the division WHERE fails on these rows
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert len(got) > 20
    assert st.records_filter_error == exp.records_filter_error
    if "/" in where:
        assert exp.records_filter_error > 0
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_state_window_rejections(engine_mod):
    r2 = compile_rule("SELECT deviceId, count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)", TRIG_SCHEMA,
                      num_keys=10, window_version="v2")
    with pytest.raises(engine_mod.EngineError) as e:
        engine_mod.Engine(r2.plan)
    assert e.value.code == A.EK_ERR_UNSUPPORTED


# ------------------------------------------------------------------ v2 event-time sliding windows
@pytest.mark.parametrize("case", json.load(open(os.path.join(GOLD, "kat_window_v2.json")))["tests"], ids=lambda c: c["name"])
def test_window_v2_sliding_kat_engine(oracle, engine_mod, case):
    a = np.array([r["a"] for r in case["rows"]], np.int64)
    ts = np.array([1541152480000 + r["dt_ms"] for r in case["rows"]], np.int64)
    rule = compile_rule(case["sql"].replace("eventStream", "demo"), {"a": "bigint", "ts": "bigint"}, window_version="v2",
                        debug_membership=True, late_tolerance_ms=case.get("late_tolerance_ms", 0))
    got, exp, _ = run_both(oracle, engine_mod, rule, [a, ts], batches=len(a))
    assert got[0].value(0, 0) == len(case["content"])
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("batches", [1, 7])
def test_window_v2_sliding_out_of_order(oracle, engine_mod, batches):
    sql = ("SELECT deviceId, count(*), sum(temperature), min(humidity), stddev(temperature) FROM demo "
           "GROUP BY deviceId, SLIDINGWINDOW(ms, 300) OVER (WHEN trig = 1) HAVING count(*) > 1")
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=60, late_tolerance_ms=100, debug_membership=True, window_version="v2")
    cols = _with_trig(_iot(40_000, 60, seed=94, epm=3), 80)
    rng = np.random.default_rng(12)
    cols[1] = (cols[1] + rng.integers(-150, 150, len(cols[1]))).astype(np.int64)
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert exp.records_late > 0 and st.records_late == exp.records_late
    assert len(got) > 100
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_window_v2_sliding_every_row_with_ties(oracle, engine_mod):
    """No OVER: a window per released row; rows sharing a ts see only the tied rows released before them."""
    sql = "SELECT deviceId, count(*), max(humidity) FROM demo GROUP BY deviceId, SLIDINGWINDOW(ms, 20)"
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=10, debug_membership=True, window_version="v2")
    cols = _with_trig(_iot(4000, 10, seed=95, epm=4), 10)
    for batches in (1, 5):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert len(got) == len(exp.windows) > 3900
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("batches", [1, 6])
def test_window_v2_sliding_delayed_event(oracle, engine_mod, batches):
    """EventSlidingWindowOp with a delay (window_v2_event_op.go:56-76): each due delay emits at every WatermarkTuple
    (WindowRange ending at it) until a newer trigger is pending; the scanner is cut by gc(W - L - D) at each tuple.
    Sparse triggers over a dense out-of-order stream exercise the re-emission; dense ones the prefix drop."""
    for every, n in ((400, 6000), (25, 6000)):
        sql = ("SELECT deviceId, count(*), sum(temperature), max(humidity) FROM demo "
               "GROUP BY deviceId, SLIDINGWINDOW(ms, 200, 150) OVER (WHEN trig = 1)")
        rule = compile_rule(sql, TRIG_SCHEMA, num_keys=20, late_tolerance_ms=40, debug_membership=True, window_version="v2")
        cols = _with_trig(_iot(n, 20, seed=every, epm=2), every)
        rng = np.random.default_rng(every)
        cols[1] = (cols[1] + rng.integers(-30, 30, len(cols[1]))).astype(np.int64)
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert len(exp.windows) > 20
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    small = [c[:400] for c in cols]
    got, exp, _ = run_both(oracle, engine_mod, rule, small, batches=400)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


PROC_SCHEMA = {"k": "key", "ts": "bigint", "x": "float", "y": "float"}


@pytest.mark.parametrize("case", json.load(open(os.path.join(GOLD, "kat_v2_proc.json")))["tests"], ids=lambda c: c["name"])
def test_window_v2_proc_kat_engine(oracle, engine_mod, case):
    from test_processing_gpu import run_engine
    t0 = 1541152480000
    a = np.array([r[1] for r in case["rows"]], np.int64)
    ts = np.array([t0 + r[0] for r in case["rows"]], np.int64)
    rule = compile_rule(case["sql"].replace("stream", "demo"), {"a": "bigint", "ts": "bigint"}, is_event_time=False,
                        window_version="v2", debug_membership=True)
    exp = oracle.run_proc(rule.plan, [a, ts], t0, t0 + case["end_ms"])
    for cuts in ([0, len(a)], list(range(len(a) + 1))):
        got = run_engine(engine_mod, rule, [a, ts], t0, t0 + case["end_ms"], cuts)
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
        assert (got[0].start - t0, got[0].end - t0) == (case["first_window"]["window_start"], case["first_window"]["window_end"])


V2_PROC = [
    ("over", "SELECT k, count(*), avg(x) FROM s GROUP BY k, SLIDINGWINDOW(ms, 400) OVER (WHEN x > 97)"),
    ("delay", "SELECT k, count(*), max(y), min(x) FROM s GROUP BY k, SLIDINGWINDOW(ms, 300, 500) OVER (WHEN x > 98)"),
    ("every_row_where", "SELECT k, count(*), sum(y) FROM s WHERE y > 30 GROUP BY k, SLIDINGWINDOW(ms, 60)"),
    ("delay_filter", "SELECT k, count(*) FROM s GROUP BY k, SLIDINGWINDOW(ms, 300, 200) FILTER (WHERE y < 70) OVER (WHEN x > 97)"),
]


@pytest.mark.parametrize("name,sql", V2_PROC, ids=[c[0] for c in V2_PROC])
def test_window_v2_proc_parity(oracle, engine_mod, name, sql):
    """SlidingWindowOp (window_v2_op.go:160-215) under the caller's clock: left-open windows over the scanner, a delayed
    window over the rows the later rows' gc(ts - length) left."""
    from test_processing_gpu import run_engine
    rng = np.random.default_rng(sum(map(ord, name)))
    n = 4000 if name == "every_row_where" else 20_000
    ts = (1541152480000 + 999 + np.cumsum(rng.integers(0, 9, n))).astype(np.int64)
    cols = [rng.integers(0, 17, n).astype(np.uint32), ts, rng.uniform(0, 100, n), rng.uniform(0, 100, n)]
    rule = compile_rule(sql, PROC_SCHEMA, is_event_time=False, num_keys=17, debug_membership=True, window_version="v2")
    start, end = int(ts[0]) - 300, int(ts[-1]) + 2000
    exp = oracle.run_proc(rule.plan, cols, start, end)
    assert len(exp.windows) > 10
    for cuts in ([0, n], [0, 1, 999, n // 2, n - 1, n]):
        got = run_engine(engine_mod, rule, cols, start, end, cuts)
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("batches", [1, 5])
def test_state_window_event_time_year1_rows(oracle, engine_mod, batches):
    """scanWindow keeps rows whose timestamp is After(time.Time{}) (window_v2_op.go:254-263): rows stamped exactly
    0001-01-01T00:00:00Z (the earliest the watermark accepts) join the state machine but no window's content."""
    sql = "SELECT deviceId, count(*), sum(temperature) FROM demo GROUP BY deviceId, STATEWINDOW(trig = 1, humidity > 97)"
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=50, debug_membership=True)
    cols = _with_trig(_iot(20_000, 50, seed=95, epm=4), 40)
    cols[1] = cols[1].astype(np.int64).copy()
    cols[1][:300] = -62135596800000   # Go's time.Time{} in Unix ms
    cols[-1][:300] = 1                # the first window opens on a year-1 row
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert st.records_late == exp.records_late
    assert len(got) > 5
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
