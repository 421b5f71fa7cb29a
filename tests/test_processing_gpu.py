"""Processing-time TUMBLING / HOPPING / SLIDING / SESSION windows (execProcessingWindow, window_op.go:235-470) on
the GPU under the caller's clock (ek_advance_time), against the oracle's clock replay (eko_run_proc): the
reference's processing-time KATs (window_rule_test.go TestWindow, mock clock) and seeded streams in pane and range
mode, pushed whole, in batches with clock advances between them, and one row per push."""
import json
import os

import numpy as np
import pytest

from ekgpu.rule import compile_rule
from parity import assert_windows_equal
from test_engine_gpu import engine_mod  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
KAT_SCHEMA = {"ts": "bigint", "size": "bigint", "color": "key", "temp": "float"}
SCHEMA = {"k": "key", "ts": "bigint", "x": "float", "y": "float"}


def run_engine(engine_mod, rule, cols, start, end, cuts, advance_between=True):
    """advance_time(start); push the rows in the given cuts (an advance to the next batch's first arrival between
    batches); advance_time(end); poll."""
    eng = engine_mod.Engine(rule.plan)
    eng.advance_time(start)
    ts = np.asarray(cols[rule.plan.ts_column])
    for a, b in zip(cuts[:-1], cuts[1:]):
        if b <= a:
            continue
        if advance_between:
            eng.advance_time(int(ts[a]))
        eng.push_host([c[a:b] for c in cols])
    eng.advance_time(end)
    got = eng.poll()
    eng.close()
    return got


def _kat_cases():
    return json.load(open(os.path.join(GOLD, "kat_window_proc.json")))["tests"]


@pytest.mark.parametrize("case", _kat_cases(), ids=lambda c: c["name"])
def test_processing_kat_engine(oracle, engine_mod, case):
    g = json.load(open(os.path.join(GOLD, "kat_window_proc.json")))
    rows = np.array(g["streams"][case["stream"]]["rows"], dtype=object)
    cols = [np.array(rows[:, 0], np.int64), np.array(rows[:, 1], np.int64), np.array(rows[:, 2], np.uint32),
            np.array(rows[:, 3], np.float64)]
    rule = compile_rule(case["sql"], KAT_SCHEMA, is_event_time=False, num_keys=4, debug_membership=True,
                        **case.get("options", {}))
    start = case.get("start_ms", int(cols[0][0]) // 1000 * 1000)
    end = case.get("end_ms", int(cols[0][-1]))
    exp = oracle.run_proc(rule.plan, cols, start, end)
    assert len(exp.windows) == case["windows_out"]
    n = len(cols[0])
    for cuts in ([0, n], list(range(n + 1))):
        got = run_engine(engine_mod, rule, cols, start, end, cuts)
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def _stream(n, keys, seed, gap_ms=7, burst=False):
    rng = np.random.default_rng(seed)
    steps = rng.integers(0, gap_ms, n)
    if burst:   # idle stretches: session timeouts and empty ticks
        steps[rng.random(n) < 0.002] += rng.integers(2000, 9000)
    ts = 1541152480000 + 3_456 + np.cumsum(steps)
    return [rng.integers(0, keys, n).astype(np.uint32), ts.astype(np.int64), rng.uniform(0, 100, n),
            rng.uniform(0, 100, n)]


CASES = [
    ("tumbling", "SELECT k, avg(x), max(y), count(*) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 2)"),
    ("tumbling_where", "SELECT k, sum(x), min(y), count(*) FROM s WHERE y > 30 GROUP BY k, TUMBLINGWINDOW(ss, 1)"),
    ("hopping", "SELECT k, sum(x), min(x), max(y) FROM s GROUP BY k, HOPPINGWINDOW(ss, 3, 1)"),
    ("hopping_median", "SELECT k, median(x), count(*) FROM s GROUP BY k, HOPPINGWINDOW(ss, 2, 1)"),
    ("sliding_over", "SELECT k, stddev(x), count(*) FROM s GROUP BY k, SLIDINGWINDOW(ss, 2) OVER (WHEN x > 99)"),
    ("sliding_where", "SELECT k, count(*), max(y) FROM s WHERE y > 50 GROUP BY k, SLIDINGWINDOW(ms, 300) OVER (WHEN x > 98)"),
    ("session", "SELECT k, count(*), avg(x) FROM s GROUP BY k, SESSIONWINDOW(ss, 5, 1)"),
    ("session_where", "SELECT k, count(*), sum(y) FROM s WHERE x < 60 GROUP BY k, SESSIONWINDOW(ss, 4, 1)"),
    ("ungrouped_tumbling", "SELECT count(*), avg(x) FROM s GROUP BY TUMBLINGWINDOW(ss, 1)"),
    # the window FILTER (WHERE ...) op (planner.go:388-392): combined with WHERE below tumbling / hopping / session,
    # alone before sliding windows
    ("tumbling_filter", "SELECT k, sum(x), count(*) FROM s WHERE y > 20 GROUP BY k, TUMBLINGWINDOW(ss, 1) FILTER (WHERE x < 70)"),
    ("hopping_filter", "SELECT k, max(x), count(*) FROM s GROUP BY k, HOPPINGWINDOW(ss, 2, 1) FILTER (WHERE y > 40)"),
    ("session_filter", "SELECT k, count(*), avg(y) FROM s GROUP BY k, SESSIONWINDOW(ss, 4, 1) FILTER (WHERE x > 10)"),
    ("sliding_filter", "SELECT k, count(*), min(x) FROM s WHERE y < 80 GROUP BY k, SLIDINGWINDOW(ms, 400) FILTER (WHERE x > 30) OVER (WHEN x > 97)"),
    # delayed sliding windows (window_op.go:355-373): a timer per trigger, the window [t - length, t + delay)
    ("sliding_delay", "SELECT k, count(*), stddev(x) FROM s GROUP BY k, SLIDINGWINDOW(ms, 500, 300) OVER (WHEN x > 98)"),
    ("sliding_delay_where", "SELECT k, count(*), sum(y) FROM s WHERE y > 25 GROUP BY k, SLIDINGWINDOW(ss, 1, 2) OVER (WHEN x > 99)"),
]
# enableSlidingWindowSendTwice (window_op.go:98): first part at the trigger, second part when the delay expires
SEND_TWICE = [
    ("send_twice", "SELECT k, count(*), max(x) FROM s GROUP BY k, SLIDINGWINDOW(ms, 500, 300) OVER (WHEN x > 98)"),
    ("send_twice_long_delay", "SELECT count(*), avg(y) FROM s GROUP BY SLIDINGWINDOW(ms, 200, 2000) OVER (WHEN x > 99)"),
]


@pytest.mark.parametrize("name,sql", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("batches", [1, 7])
def test_processing_windows_parity(oracle, engine_mod, name, sql, batches):
    keys = 40
    cols = _stream(60_000, keys, seed=len(name) * 31 + batches, gap_ms=6, burst=name.startswith("session") or batches == 7)
    rule = compile_rule(sql, SCHEMA, is_event_time=False, num_keys=keys, debug_membership=True)
    start = int(cols[1][0]) - 1234
    end = int(cols[1][-1]) + 12_000
    exp = oracle.run_proc(rule.plan, cols, start, end)
    assert len(exp.windows) >= 3
    cuts = np.linspace(0, len(cols[0]), batches + 1).astype(np.int64).tolist()
    got = run_engine(engine_mod, rule, cols, start, end, cuts)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("name,sql", SEND_TWICE, ids=[c[0] for c in SEND_TWICE])
@pytest.mark.parametrize("batches", [1, 7])
def test_processing_send_twice_parity(oracle, engine_mod, name, sql, batches):
    keys = 40
    cols = _stream(30_000, keys, seed=len(name) * 17 + batches, gap_ms=6, burst=batches == 7)
    rule = compile_rule(sql, SCHEMA, is_event_time=False, num_keys=keys, debug_membership=True, sliding_send_twice=True)
    assert rule.plan.sliding_send_twice == 1
    start = int(cols[1][0]) - 500
    end = int(cols[1][-1]) + 5_000
    exp = oracle.run_proc(rule.plan, cols, start, end)
    assert len(exp.windows) >= 3
    cuts = np.linspace(0, len(cols[0]), batches + 1).astype(np.int64).tolist()
    got = run_engine(engine_mod, rule, cols, start, end, cuts)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_processing_sliding_gc_edge(oracle, engine_mod):
    """A non-matching row with the trigger's timestamp, delivered before it, drops the rows exactly `length` older
    (gcInputs, window_op.go:657-673); a trigger without such a row keeps them."""
    ts = np.array([1000, 1000, 1500, 2000, 2000, 2000, 3000, 3000], np.int64) + 1541152480000
    x = np.array([0, 0, 0, 0, 99.5, 99.5, 99.5, 0], np.float64)      # triggers: x > 99
    cols = [np.zeros(len(ts), np.uint32), ts, x, np.zeros(len(ts))]
    rule = compile_rule("SELECT count(*) FROM s GROUP BY SLIDINGWINDOW(ms, 1000) OVER (WHEN x > 99)", SCHEMA,
                        is_event_time=False, num_keys=1, debug_membership=True)
    exp = oracle.run_proc(rule.plan, cols, int(ts[0]), int(ts[-1]))
    # the non-matching row at 2000 drops the rows at 1000 before the first trigger at 2000: [1500, 2000, 2000]
    assert [sorted(int(i) for i in m) for m in exp.members] == [[2, 3, 4], [2, 3, 4, 5], [3, 4, 5, 6]]
    for cuts in ([0, len(ts)], list(range(len(ts) + 1))):
        got = run_engine(engine_mod, rule, cols, int(ts[0]), int(ts[-1]), cuts)
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_processing_c2_shape_pane_mode(oracle, engine_mod):
    """The C2 rule in processing time (pane mode, direct emission): 2e6 rows, 64 Ki keys, tumbling 10 s."""
    from ekgpu.synth import IOT_SCHEMA, iot_stream
    sql = "SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)"
    rule = compile_rule(sql, IOT_SCHEMA, is_event_time=False, num_keys=65536, debug_membership=True)
    cols = list(iot_stream(2_000_000, 65536, events_per_ms=40))
    start = int(cols[1][0]) - 2500
    end = int(cols[1][-1]) + 20_000
    exp = oracle.run_proc(rule.plan, cols, start, end)
    assert len(exp.windows) >= 5
    got = run_engine(engine_mod, rule, cols, start, end, [0, 700_000, 2_000_000])
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_processing_clock_errors(engine_mod):
    rule = compile_rule("SELECT k, count(*) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1)", SCHEMA, is_event_time=False,
                        num_keys=4)
    eng = engine_mod.Engine(rule.plan)
    eng.advance_time(5_000)
    with pytest.raises(engine_mod.EngineError):
        eng.advance_time(4_000)                       # the clock never moves back
    with pytest.raises(engine_mod.EngineError):     # a row older than the clock
        eng.push_host([np.zeros(1, np.uint32), np.array([4_999], np.int64), np.zeros(1), np.zeros(1)])
    eng.close()
