"""GPU parity tests of RANGE mode (device event buffer, windows as index ranges): sliding, session and
count windows, plus tumbling/hopping forced through range mode, against the CPU oracle."""
import json
import os

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401  (fixture + helper)

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _kat_all():
    g = json.load(open(os.path.join(GOLD, "kat_window_rules.json")))
    return g["tests"]


@pytest.fixture
def force_range():
    os.environ["EKGPU_FORCE_RANGE"] = "1"
    yield
    del os.environ["EKGPU_FORCE_RANGE"]


def _kat_cols(case):
    g = json.load(open(os.path.join(GOLD, "kat_window_rules.json")))
    rows = np.array(g["streams"][case["stream"]]["rows"], dtype=object)
    return [np.array(rows[:, 0], np.int64), np.array(rows[:, 1], np.int64), np.array(rows[:, 2], np.uint32),
            np.array(rows[:, 3], np.float64)]


KAT_SCHEMA = {"ts": "bigint", "size": "bigint", "color": "key", "temp": "float"}


@pytest.mark.parametrize("case", _kat_all(), ids=lambda c: c["name"])
def test_window_rule_kat_range(oracle, engine_mod, case, force_range):
    """Every reference window KAT (window_rule_test.go) through range mode, whole stream and one event per push."""
    cols = _kat_cols(case)
    rule = compile_rule(case["sql"], KAT_SCHEMA, late_tolerance_ms=1000, num_keys=4, debug_membership=True,
                        is_event_time=case.get("event_time", True))
    got, exp, st = run_both(oracle, engine_mod, rule, cols)
    assert len(got) == case["windows_out"]
    assert st.records_late == case["late"]
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    got1, _, _ = run_both(oracle, engine_mod, rule, cols, batches=len(cols[0]))
    assert_windows_equal(rule.plan, got1, exp.windows, check_members=True)


def _iot(n, keys, seed, epm):
    key, ts, temp, hum = iot_stream(n, keys, seed=seed, events_per_ms=epm)
    return [key, ts, temp, hum]


TRIG_SCHEMA = {"deviceId": "key", "ts": "bigint", "temperature": "float", "humidity": "float", "trig": "bigint"}


def _with_trig(cols, every, seed=9):
    rng = np.random.default_rng(seed)
    trig = (rng.integers(0, every, len(cols[0])) == 0).astype(np.int64)
    return cols + [trig]


@pytest.mark.parametrize("batches", [1, 5])
def test_sliding_over_when_c4a_shape(oracle, engine_mod, batches):
    """C4a shape (reduced): SLIDINGWINDOW(ss, 3) OVER (WHEN trig = 1), stddev/var + HAVING."""
    sql = ("SELECT deviceId, stddev(temperature), var(temperature), count(*) FROM demo "
           "GROUP BY deviceId, SLIDINGWINDOW(ss, 3) OVER (WHEN trig = 1) HAVING count(*) > 1")
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=3000, debug_membership=True)
    cols = _with_trig(_iot(200_000, 3000, seed=61, epm=10), 500)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert len(got) > 100
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_sliding_every_event(oracle, engine_mod):
    """No OVER: one window per event (event_window_trigger.go:190-192), ties of ts inside the run."""
    sql = "SELECT deviceId, count(*), sum(temperature), max(humidity) FROM demo GROUP BY deviceId, SLIDINGWINDOW(ms, 40)"
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=20, debug_membership=True)
    cols = _iot(3000, 20, seed=62, epm=3)
    for batches in (1, 7):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert len(got) == len(exp.windows) > 2900   # the last ts run stays unreleased
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_sliding_late_tolerance_out_of_order(oracle, engine_mod):
    sql = ("SELECT deviceId, count(*), min(temperature), avg(humidity) FROM demo "
           "GROUP BY deviceId, SLIDINGWINDOW(ms, 300) OVER (WHEN trig = 1)")
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=40, late_tolerance_ms=200, debug_membership=True)
    cols = _with_trig(_iot(20_000, 40, seed=63, epm=2), 50)
    rng = np.random.default_rng(5)
    cols[1] = (cols[1] + rng.integers(-400, 400, len(cols[1]))).astype(np.int64)
    for batches in (1, 9):
        got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert exp.records_late > 0 and st.records_late == exp.records_late
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_sliding_with_delay(oracle, engine_mod):
    sql = ("SELECT deviceId, count(*), sum(temperature) FROM demo "
           "GROUP BY deviceId, SLIDINGWINDOW(ms, 200, 100) OVER (WHEN trig = 1)")
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=30, debug_membership=True)
    cols = _with_trig(_iot(30_000, 30, seed=64, epm=3), 300)
    for batches in (1, 6):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert len(got) > 10
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("late", [0, 150])
def test_sliding_send_twice_event_time(oracle, engine_mod, late):
    """enableSlidingWindowSendTwice in event time (event_window_trigger.go:129-135,156-161): the first part
    (t - L, t] when the watermark passes the trigger, the last part (t, t + D] when it passes t + D, each scan keeping
    only the expired prefix of the inputs (handleInputsForSlidingWindow, window_op.go:576-603) and the triggers gated
    by getNextWindow over what is left. No reference KAT covers this path: parity is against the oracle's restatement
    (oracle/ekoracle.c win_on_watermark / scan), in order and out of order within lateTolerance."""
    sql = ("SELECT deviceId, count(*), sum(temperature), max(humidity) FROM demo "
           "GROUP BY deviceId, SLIDINGWINDOW(ms, 200, 100) OVER (WHEN trig = 1)")
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=30, late_tolerance_ms=late, debug_membership=True,
                        sliding_send_twice=True)
    assert rule.plan.sliding_send_twice == 1
    cols = _with_trig(_iot(30_000, 30, seed=66, epm=3), 300)
    if late:
        rng = np.random.default_rng(7)
        cols[1] = (cols[1] + rng.integers(-200, 200, len(cols[1]))).astype(np.int64)
    for batches in (1, 6, 97):
        got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert len(exp.windows) > 10
        assert st.records_late == exp.records_late
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_sliding_send_twice_event_time_small(oracle, engine_mod):
    """A hand-sized stream, one row per push: sparse triggers with idle gaps longer than length + delay (every
    input expires: none kept) and dense ones (some expire: only those are kept, the live inputs are lost)."""
    sql = "SELECT count(*), sum(temperature) FROM demo GROUP BY SLIDINGWINDOW(ms, 50, 30) OVER (WHEN trig = 1)"
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=1, debug_membership=True, sliding_send_twice=True)
    t0 = 1541152480000
    ts = np.array([0, 10, 20, 25, 40, 60, 61, 90, 200, 210, 215, 230, 260, 300, 305, 500, 520, 540, 545, 600], np.int64)
    trig = np.array([0, 1, 0, 1, 0, 1, 0, 0, 1, 0, 1, 1, 0, 0, 1, 1, 0, 1, 0, 0], np.int64)
    n = len(ts)
    cols = [np.zeros(n, np.uint32), ts + t0, np.arange(n, dtype=np.float64), np.zeros(n), trig]
    for batches in (1, 3, n):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert len(exp.windows) >= 6
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("n,m", [(1000, 0), (500, 200), (300, 700)])
def test_count_window(oracle, engine_mod, n, m):
    """COUNTWINDOW(n[, m]) in processing time (C4b shape, reduced) with stddev/var + HAVING."""
    cw = f"COUNTWINDOW({n})" if m == 0 else f"COUNTWINDOW({n}, {m})"
    sql = (f"SELECT deviceId, stddev(temperature), var(temperature), count(*) FROM demo "
           f"GROUP BY deviceId, {cw} HAVING count(*) > 1")
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=100, is_event_time=False, debug_membership=True)
    cols = _iot(50_000, 100, seed=65, epm=10)
    for batches in (1, 11):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert len(got) == len(exp.windows) > 10
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_count_window_direct_uneven_batches(oracle, engine_mod):
    """COUNTWINDOW(1000): batches holding whole windows are aggregated straight from the batch (the window spanning
    the carried rows and the batch head goes through the event buffer); small batches (< 2 windows) take the
    buffered path; mostly one-row groups over a large key space, HAVING count(*) > 1 decided from the row count."""
    sql = ("SELECT deviceId, stddev(temperature), var(temperature) FROM demo "
           "GROUP BY deviceId, COUNTWINDOW(1000) HAVING count(*) > 1")
    cols = _iot(60_500, 20_000, seed=67, epm=10)
    cuts = [0, 700, 5_300, 6_100, 9_999, 10_000, 31_234, 32_000, 33_500, 60_500]
    for members in (True, False):   # without the fingerprint the direct windows launch with arithmetic ranges
        rule = compile_rule(sql, IOT_SCHEMA, num_keys=20_000, is_event_time=False, debug_membership=members)
        exp = oracle.run(rule.plan, cols)
        eng = engine_mod.Engine(rule.plan)
        for lo, hi in zip(cuts, cuts[1:]):
            eng.push_host([c[lo:hi] for c in cols])
        got = eng.poll()
        eng.close()
        assert len(got) == len(exp.windows) == 60
        assert_windows_equal(rule.plan, got, exp.windows, check_members=members)


def test_count_window_rejected_in_event_time(engine_mod):
    rule = compile_rule("SELECT count(*) FROM demo GROUP BY COUNTWINDOW(10)", IOT_SCHEMA)
    with pytest.raises(engine_mod.EngineError) as e:
        engine_mod.Engine(rule.plan)
    assert e.value.code == A.EK_ERR_UNSUPPORTED


def test_session_window(oracle, engine_mod):
    sql = "SELECT deviceId, count(*), max(temperature) FROM demo GROUP BY deviceId, SESSIONWINDOW(ss, 10, 2)"
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=50, debug_membership=True)
    key, ts, temp, hum = iot_stream(20_000, 50, seed=66, events_per_ms=1)
    # bursts separated by gaps longer than the 2 s timeout
    ts = ts + (np.arange(len(ts)) // 3000) * 3500
    cols = [key, ts.astype(np.int64), temp, hum]
    for batches in (1, 8):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert len(got) >= 3
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_tumbling_hopping_through_range_mode(oracle, engine_mod, force_range):
    for sql, keys, epm in [
        ("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)", 4000, 5),
        ("SELECT deviceId, sum(temperature), min(temperature), max(temperature) FROM demo "
         "GROUP BY deviceId, HOPPINGWINDOW(ss, 6, 2)", 2000, 2),
    ]:
        rule = compile_rule(sql, IOT_SCHEMA, num_keys=keys, debug_membership=True)
        cols = _iot(300_000, keys, seed=67, epm=epm)
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=3)
        assert len(got) >= 2
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_range_out_of_order_tumbling(oracle, engine_mod, force_range):
    sql = "SELECT deviceId, count(*), sum(temperature), max(humidity) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 2)"
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=50, late_tolerance_ms=700, debug_membership=True)
    key, ts, temp, hum = iot_stream(20_000, 50, seed=47, events_per_ms=2)
    rng = np.random.default_rng(7)
    ts = ts + rng.integers(-1500, 1500, size=len(ts))
    cols = [key, ts.astype(np.int64), temp, hum]
    for batches in (1, 13):
        got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert st.records_late == exp.records_late
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


# ------------------------------------------------------------------ order statistics (median, percentile_*)
MED_SQL = ("SELECT deviceId, median(temperature), percentile_cont(temperature, 0.9), percentile_disc(humidity, 0.5), "
           "count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)")


@pytest.mark.parametrize("keys", [4000, 3])
def test_median_percentile_tumbling(oracle, engine_mod, keys):
    """Short groups (one thread selects) and long groups (whole-workgroup radix select)."""
    rule = compile_rule(MED_SQL, IOT_SCHEMA, num_keys=keys, debug_membership=True)
    cols = _iot(300_000, keys, seed=71, epm=5)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=2)
    assert len(got) >= 4
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_median_percentile_int_columns_nulls(oracle, engine_mod):
    schema = {"k": "key", "ts": "bigint", "a": "bigint", "b": "bigint"}
    sql = ("SELECT k, median(a), percentile_cont(b, 0.5), percentile_disc(b, 0.25), percentile_cont(a, 1), count(b) "
           "FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1) HAVING count(*) > 1")
    rule = compile_rule(sql, schema, num_keys=37, nullable=("b",), debug_membership=True)
    n = 40_000
    rng = np.random.default_rng(4)
    k = rng.integers(0, 37, n).astype(np.uint32)
    ts = (1541152480000 + np.arange(n) // 4).astype(np.int64)
    a = rng.integers(-50, 50, n).astype(np.int64)          # many ties
    b = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    vb = (rng.random(n) > 0.4).astype(np.uint8)
    got, exp, _ = run_both(oracle, engine_mod, rule, [k, ts, a, b], batches=3, validity=[None, None, None, vb])
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_percentile_out_of_range_is_window_error(oracle, engine_mod):
    """stats.Percentile: index < 1 and not integral -> "Input is outside of range" -> the window errors."""
    sql = "SELECT deviceId, percentile_cont(temperature, 0.05), count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)"
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=500, debug_membership=True)
    cols = _iot(40_000, 500, seed=72, epm=5)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols)
    assert any(w.status == A.EK_WIN_AGG_ERROR for w in exp.windows)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_c5_shape_high_cardinality_median(oracle, engine_mod):
    """C5 shape (reduced): ~10 events per key over many keys in one 60 s tumbling window + a sentinel."""
    keys = 200_000
    sql = ("SELECT deviceId, median(temperature), percentile_cont(temperature, 0.9) FROM demo "
           "GROUP BY deviceId, TUMBLINGWINDOW(ss, 60)")
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=keys)
    n = 2_000_000
    key, ts, temp, hum = iot_stream(n, keys, seed=73, events_per_ms=40)
    t_min = 1541152440000                      # a minute boundary: the first 60 s window is [t_min, t_min + 60 s)
    ts = np.minimum(ts - 40_000, t_min + 59_000)
    ts[-1] = t_min + 60_000                    # sentinel: closes the window
    got, exp, _ = run_both(oracle, engine_mod, rule, [key, ts, temp, hum], batches=2)
    assert len(got) == 1 and len(got[0].keys) > 0.99 * keys
    assert_windows_equal(rule.plan, got, exp.windows)


def test_sliding_median(oracle, engine_mod):
    sql = ("SELECT deviceId, median(temperature), percentile_disc(temperature, 0.75) FROM demo "
           "GROUP BY deviceId, SLIDINGWINDOW(ss, 2) OVER (WHEN trig = 1)")
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=64, debug_membership=True)
    cols = _with_trig(_iot(60_000, 64, seed=74, epm=5), 400)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=4)
    assert len(got) > 50
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
