"""Processing-time incremental windows (TumblingWindowIncAggOp / HoppingWindowIncAggOp / SlidingWindowIncAggOp,
window_inc_agg_op.go:316-790) on the GPU under the caller's clock, against the oracle's clock replay (eko_run_proc):
the reference's own KATs (window_inc_agg_op_test.go, tests/golden/kat_inc_proc.json), seeded streams pushed whole, in
batches with clock advances between them and one row per push (idle stretches: windows no row joined are broadcast
empty), the window FILTER in front of the op, a checkpoint split, and the event-time incremental windows with FILTER."""
import json
import os

import numpy as np
import pytest

from ekgpu.rule import compile_rule
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401  (fixture + helper)
from test_processing_gpu import run_engine

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
SCHEMA = {"k": "key", "ts": "bigint", "x": "float", "y": "float"}


@pytest.mark.parametrize("case", json.load(open(os.path.join(GOLD, "kat_inc_proc.json")))["tests"], ids=lambda c: c["name"])
def test_inc_proc_kat_engine(oracle, engine_mod, case):
    rows = case["rows"]
    a = np.array([r[1] for r in rows], np.int64)
    ts = np.array([r[0] for r in rows], np.int64)
    rule = compile_rule(case["sql"].replace("stream", "demo"), {"a": "bigint", "ts": "bigint"}, is_event_time=False,
                        incremental=True, inc_unaligned=case.get("inc_unaligned", False), debug_membership=True)
    exp = oracle.run_proc(rule.plan, [a, ts], 0, case["end_ms"])
    assert len(exp.windows) == len(case["windows"])
    n = len(a)
    for cuts in ([0, n], list(range(n + 1))):
        got = run_engine(engine_mod, rule, [a, ts], 0, case["end_ms"], cuts)
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
        assert [w.end for w in got] == [w["window_end"] for w in case["windows"]]


def _stream(n, keys, seed, gap_ms=7, idle=True):
    rng = np.random.default_rng(seed)
    steps = rng.integers(0, gap_ms, n)
    if idle:   # idle stretches: ticks and timers with no row (empty windows)
        steps[rng.random(n) < 0.002] += rng.integers(2000, 9000)
    ts = 1541152480000 + 3_456 + np.cumsum(steps)
    return [rng.integers(0, keys, n).astype(np.uint32), ts.astype(np.int64), rng.uniform(0, 100, n),
            rng.uniform(0, 100, n)]


CASES = [
    ("tumbling", "SELECT k, avg(x), max(y), count(*) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 2)", {}),
    ("tumbling_unaligned", "SELECT k, sum(x), min(y) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1)", dict(inc_unaligned=True)),
    ("hopping", "SELECT k, sum(x), min(x), max(y) FROM s GROUP BY k, HOPPINGWINDOW(ss, 3, 1)", {}),
    ("hopping_unaligned", "SELECT k, count(*), avg(y) FROM s GROUP BY k, HOPPINGWINDOW(ss, 2, 1)", dict(inc_unaligned=True)),
    ("hopping_gap", "SELECT k, count(*), max(x) FROM s GROUP BY k, HOPPINGWINDOW(ms, 500, 1500)", {}),
    ("sliding", "SELECT k, count(*), sum(y) FROM s GROUP BY k, SLIDINGWINDOW(ms, 400) OVER (WHEN x > 98)", {}),
    ("sliding_delay", "SELECT k, count(*), max(y), avg(x) FROM s GROUP BY k, SLIDINGWINDOW(ms, 300, 500) OVER (WHEN x > 98)", {}),
    ("sliding_every_row", "SELECT k, count(*), min(x) FROM s GROUP BY k, SLIDINGWINDOW(ms, 50)", {}),
    ("tumbling_filter", "SELECT k, sum(x), count(*) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1) FILTER (WHERE y > 40)", {}),
    ("sliding_filter", "SELECT k, count(*), max(x) FROM s GROUP BY k, SLIDINGWINDOW(ms, 400) FILTER (WHERE y < 60) OVER (WHEN x > 97)", {}),
    ("ungrouped_hopping", "SELECT count(*), avg(x) FROM s GROUP BY HOPPINGWINDOW(ss, 2, 1)", {}),
    ("having", "SELECT k, count(*), avg(x) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1) HAVING count(*) > 3", {}),
]


@pytest.mark.parametrize("name,sql,kw", CASES, ids=[c[0] for c in CASES])
def test_inc_proc_parity(oracle, engine_mod, name, sql, kw):
    keys = 37
    cols = _stream(30_000, keys, seed=sum(map(ord, name)))
    if name == "sliding_every_row":
        cols = [c[:4000] for c in cols]
    rule = compile_rule(sql, SCHEMA, is_event_time=False, num_keys=keys, debug_membership=True, incremental=True, **kw)
    assert rule.plan.incremental == 1
    ts = cols[1]
    start, end = int(ts[0]) - 1234, int(ts[-1]) + 7000
    exp = oracle.run_proc(rule.plan, cols, start, end)
    assert len(exp.windows) > 3
    n = len(ts)
    for cuts in ([0, n], sorted({0, 1, 777, min(5000, n - 5), n // 2, n - 3, n})):
        got = run_engine(engine_mod, rule, cols, start, end, cuts)
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    if name in ("tumbling", "hopping", "sliding_delay"):   # one row per push
        small = [c[:300] for c in cols]
        e2 = oracle.run_proc(rule.plan, small, start, int(small[1][-1]) + 3000)
        got = run_engine(engine_mod, rule, small, start, int(small[1][-1]) + 3000, list(range(301)))
        assert_windows_equal(rule.plan, got, e2.windows, check_members=True)


@pytest.mark.parametrize("name,sql,kw", [CASES[0], CASES[2], CASES[6]], ids=["tumbling", "hopping", "sliding_delay"])
def test_inc_proc_checkpoint_split(oracle, engine_mod, name, sql, kw):
    """export at a clock between two rows, import into a fresh handle, resume: the same windows as one run (the
    open windows, the ticker and the delay timers travel in the state blob, v5)."""
    keys = 29
    cols = _stream(20_000, keys, seed=7, idle=True)
    rule = compile_rule(sql, SCHEMA, is_event_time=False, num_keys=keys, debug_membership=True, incremental=True, **kw)
    ts = cols[1]
    start, end = int(ts[0]) - 500, int(ts[-1]) + 6000
    exp = oracle.run_proc(rule.plan, cols, start, end)
    cut = 11_111
    a = engine_mod.Engine(rule.plan)
    a.advance_time(start)
    a.push_host([c[:cut] for c in cols])
    a.advance_time(int(ts[cut]) - 1 if ts[cut] > ts[cut - 1] else int(ts[cut]))
    got = a.poll()
    blob = a.export_state()
    a.close()
    b = engine_mod.Engine(rule.plan)
    b.import_state(blob)
    b.push_host([c[cut:] for c in cols])
    b.advance_time(end)
    got = list(got) + list(b.poll())
    b.close()
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


EVENT_CASES = [
    ("tumbling_filter", "SELECT k, sum(x), count(*) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1) FILTER (WHERE y > 40)"),
    ("hopping_filter", "SELECT k, max(x), count(*) FROM s GROUP BY k, HOPPINGWINDOW(ss, 2, 1) FILTER (WHERE y < 70)"),
    ("sliding_filter", "SELECT k, count(*), min(y) FROM s GROUP BY k, SLIDINGWINDOW(ms, 300) FILTER (WHERE x > 20) OVER (WHEN y > 97)"),
]


@pytest.mark.parametrize("name,sql", EVENT_CASES, ids=[c[0] for c in EVENT_CASES])
def test_inc_event_time_filter(oracle, engine_mod, name, sql):
    """The window FILTER op in front of the event-time incremental window (planner.go:360-365): rows it drops still
    move the watermark but never reach the op."""
    keys = 31
    cols = _stream(25_000, keys, seed=3, idle=False)
    rule = compile_rule(sql, SCHEMA, num_keys=keys, debug_membership=True, incremental=True, late_tolerance_ms=0)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=4)
    assert len(exp.windows) > 3
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


# ------------------------------------------------------------------ WHERE above the incremental window
WSCHEMA = {"k": "key", "ts": "bigint", "x": "float", "z": "bigint"}


def _wstream(n, keys, seed, zmax=6):
    rng = np.random.default_rng(seed)
    ts = 1541152480000 + 3_456 + np.cumsum(rng.integers(0, 7, n))
    return [rng.integers(0, keys, n).astype(np.uint32), ts.astype(np.int64), rng.uniform(0, 100, n),
            rng.integers(0, zmax, n).astype(np.int64)]


WHERE_CASES = [
    ("event_tumbling", "SELECT k, count(*), avg(x) FROM s WHERE z > 2 GROUP BY k, TUMBLINGWINDOW(ss, 1)", True),
    ("event_hopping", "SELECT k, sum(x), max(z) FROM s WHERE x > 30 GROUP BY k, HOPPINGWINDOW(ss, 2, 1)", True),
    ("event_sliding", "SELECT k, count(*), min(x) FROM s WHERE z < 4 GROUP BY k, SLIDINGWINDOW(ms, 300) OVER (WHEN x > 98)", True),
    ("event_having", "SELECT k, count(*), sum(z) FROM s WHERE x > 20 GROUP BY k, TUMBLINGWINDOW(ss, 1) HAVING count(*) > 2", True),
    ("proc_tumbling", "SELECT k, count(*), avg(x) FROM s WHERE z > 2 GROUP BY k, TUMBLINGWINDOW(ss, 1)", False),
    ("proc_sliding_delay", "SELECT k, count(*), max(x) FROM s WHERE z <> 1 GROUP BY k, SLIDINGWINDOW(ms, 300, 200) OVER (WHEN x > 98)", False),
    ("proc_count", "SELECT k, sum(x), count(*) FROM s WHERE x < 50 GROUP BY k, COUNTWINDOW(500)", False),
]


@pytest.mark.parametrize("name,sql,event", WHERE_CASES, ids=[c[0] for c in WHERE_CASES])
def test_inc_where_last_rows(oracle, engine_mod, name, sql, event):
    """FilterPlan above IncWindowPlan: a group is kept or dropped by its LAST row's WHERE, its aggregates count every
    row (k_inc_where over the hidden last-row slot), then HAVING."""
    keys = 23
    cols = _wstream(20_000, keys, seed=sum(map(ord, name)))
    rule = compile_rule(sql, WSCHEMA, is_event_time=event, num_keys=keys, debug_membership=True, incremental=True)
    if event or "COUNTWINDOW" in sql:
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=3)
    else:
        ts = cols[1]
        start, end = int(ts[0]) - 100, int(ts[-1]) + 3000
        exp = oracle.run_proc(rule.plan, cols, start, end)
        got = run_engine(engine_mod, rule, cols, start, end, [0, 7000, 20_000])
    assert sum(len(w.keys) for w in exp.windows) > 0
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_inc_where_error_texts(oracle, engine_mod):
    """A last row whose WHERE errors (10 / z with z = 0) replaces the window with "run Where error: divided by zero";
    the windows whose last rows all evaluate keep their filtered rows."""
    keys = 5
    cols = _wstream(3000, keys, seed=11, zmax=40)
    rule = compile_rule("SELECT k, count(*) FROM s WHERE 10 / z > 0 GROUP BY k, TUMBLINGWINDOW(ms, 200)", WSCHEMA,
                        num_keys=keys, debug_membership=True, incremental=True)
    exp = oracle.run(rule.plan, cols)
    bad = [i for i, w in enumerate(exp.windows) if w.status != 0]
    assert bad and len(bad) < len(exp.windows)
    eng = engine_mod.Engine(rule.plan)
    eng.push_host(cols)
    got = eng.poll()
    texts = [eng.window_error(i) for i in range(len(got))]
    eng.close()
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    for i in bad:
        assert texts[i] == exp.errors[i] == "run Where error: divided by zero"
