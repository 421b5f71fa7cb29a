"""GPU parity of the incremental-aggregation windows (planOptimizeStrategy.enableIncrementalWindow)
against the CPU oracle: event-time TUMBLING / HOPPING (window_inc_agg_event_op.go) and processing-time
COUNTWINDOW (window_inc_agg_op.go:206-314), inc_* typing (funcs_inc_agg.go), the window-opening rule at the
aligned boundaries, split micro-batches, out-of-order input and checkpoint / restore."""
import json
import os

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401  (fixture + helper)
from test_state_gpu import run_split

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat_incremental.json")))
MIN0 = 1541152440000   # a minute boundary


@pytest.mark.parametrize("case", KAT["event_windows"], ids=lambda c: c["name"])
def test_inc_kat_engine(oracle, engine_mod, case):
    z = KAT["zero_ms"]
    cols = [np.array([z + t for t in case["rows_ms"]] + [z + case["sentinel_ms"]], np.int64),
            np.array(case["a"] + [-1], np.int64)]
    rule = compile_rule(case["sql"], {"ts": "bigint", "a": "bigint"}, late_tolerance_ms=KAT["late_tolerance_ms"],
                        incremental=True, debug_membership=True)
    for batches in (1, len(cols[0])):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert [(w.start - z, w.value(0, 0)) for w in got] == [(e["start_ms"], e["count"]) for e in case["expect"]]
        assert all(e["end_ms"] is None or w.end - z == e["end_ms"] for w, e in zip(got, case["expect"]))
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


C2_INC = ("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
          "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)")


@pytest.mark.parametrize("batches", [1, 7])
def test_inc_tumbling_c2_shape(oracle, engine_mod, batches):
    """C2 query under the incremental planner: 200 s at 10 ev/ms from a minute boundary, so every window edge has
    rows exactly at the trigger time and every minute has the misaligned second (M+10 s, M+11 s)."""
    key, ts, temp, hum = iot_stream(2_000_000, 3000, seed=71, events_per_ms=10, t0=MIN0)
    rule = compile_rule(C2_INC, IOT_SCHEMA, num_keys=3000, incremental=True, debug_membership=True)
    got, exp, _ = run_both(oracle, engine_mod, rule, [key, ts, temp, hum], batches=batches)
    assert len(got) >= 15
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    reg = compile_rule(C2_INC, IOT_SCHEMA, num_keys=3000)
    assert oracle.run(reg.plan, [key, ts, temp, hum]).windows[3].member_count != exp.windows[3].member_count


INT_SCHEMA = {"deviceId": "key", "ts": "bigint", "size": "bigint", "temperature": "float"}


def _int_cols(n, keys, seed, epm, t0=MIN0):
    key, ts, temp, _ = iot_stream(n, keys, seed=seed, events_per_ms=epm, t0=t0)
    size = (np.arange(n, dtype=np.int64) * 7919 + seed) % 2001 - 1000
    return [key, ts, size, temp]


@pytest.mark.parametrize("batches", [1, 4])
def test_inc_bigint_aggregates_are_float(oracle, engine_mod, batches):
    """inc_sum / inc_avg over a BIGINT column are float64 (funcs_inc_agg.go:56-117); min / max / count stay int64."""
    sql = ("SELECT deviceId, sum(size), avg(size), min(size), max(size), count(size), min(temperature) FROM demo "
           "GROUP BY deviceId, TUMBLINGWINDOW(ss, 5) HAVING count(*) > 2")
    rule = compile_rule(sql, INT_SCHEMA, num_keys=500, incremental=True, debug_membership=True)
    cols = _int_cols(300_000, 500, seed=72, epm=5)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    w = next(w for w in got if len(w.keys))
    assert isinstance(w.value(0, 0), float) and isinstance(w.value(1, 0), float) and isinstance(w.value(2, 0), int)


@pytest.mark.parametrize("epm_inv,batches", [(37, 1), (37, 5), (3, 3)])
def test_inc_hopping(oracle, engine_mod, epm_inv, batches):
    """HOPPINGWINDOW(ss, 20, 5): windows open at the first row of each hop; in the second after M+5 s every row
    opens its own window (a row every epm_inv ms: 27 or 333 of them per minute)."""
    n = 200_000 // epm_inv
    key = (np.arange(n) * 2654435761 % 64).astype(np.uint32)
    ts = MIN0 + 3 + np.arange(n, dtype=np.int64) * epm_inv
    temp = (np.arange(n) % 97).astype(np.float64) * 0.5
    sql = ("SELECT deviceId, sum(temperature), min(temperature), max(temperature), count(*) FROM demo "
           "GROUP BY deviceId, HOPPINGWINDOW(ss, 20, 5)")
    schema = {"deviceId": "key", "ts": "bigint", "temperature": "float"}
    rule = compile_rule(sql, schema, num_keys=64, incremental=True, debug_membership=True)
    got, exp, _ = run_both(oracle, engine_mod, rule, [key, ts, temp], batches=batches)
    assert len(got) > 40
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_inc_out_of_order_late_tolerance(oracle, engine_mod):
    key, ts, temp, hum = iot_stream(400_000, 1000, seed=73, events_per_ms=4, t0=MIN0)
    rng = np.random.default_rng(5)
    ts = ts + rng.integers(-800, 800, len(ts))          # out of order by up to 1.6 s
    rule = compile_rule(C2_INC, IOT_SCHEMA, num_keys=1000, incremental=True, late_tolerance_ms=500,
                        debug_membership=True)
    got, exp, st = run_both(oracle, engine_mod, rule, [key, ts, temp, hum], batches=6)
    assert st.records_late == exp.records_late and exp.records_late > 0
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("batches", [1, 9])
def test_inc_count_window(oracle, engine_mod, batches):
    sql = "SELECT deviceId, sum(size), avg(size), max(temperature), count(*) FROM demo GROUP BY deviceId, COUNTWINDOW(1000)"
    schema = {"deviceId": "key", "size": "bigint", "temperature": "float"}
    cols = _int_cols(123_457, 2000, seed=74, epm=10)
    cols = [cols[0], cols[2], cols[3]]
    rule = compile_rule(sql, schema, num_keys=2000, is_event_time=False, timestamp=None, incremental=True,
                        debug_membership=True)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert len(got) == 123
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("sql", [C2_INC, "SELECT deviceId, sum(temperature), count(*) FROM demo "
                                          "GROUP BY deviceId, HOPPINGWINDOW(ss, 20, 5)"])
def test_inc_checkpoint_restore(oracle, engine_mod, sql):
    key, ts, temp, hum = iot_stream(600_000, 800, seed=75, events_per_ms=3, t0=MIN0)
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=800, incremental=True, late_tolerance_ms=200, debug_membership=True)
    got, exp, st, _ = run_split(oracle, engine_mod, rule, [key, ts, temp, hum], cut=277_777, twice=True)
    assert st.records_late == exp.records_late
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_inc_unsupported_shapes_rejected(engine_mod):
    for sql, kw in (("SELECT count(*) FROM demo GROUP BY SLIDINGWINDOW(ss, 10, 2)", {}),
                    ("SELECT sum(temperature) FROM demo GROUP BY TUMBLINGWINDOW(ss, 10)", {"nullable": ("temperature",)})):
        rule = compile_rule(sql, IOT_SCHEMA, incremental=True, **kw)
        with pytest.raises(engine_mod.EngineError, match="not built"):
            engine_mod.Engine(rule.plan)
    # a non-incremental aggregate keeps the regular chain (rewriteIfIncAggStmt), as in the reference planner
    rule = compile_rule("SELECT stddev(temperature), sum(temperature) FROM demo GROUP BY SLIDINGWINDOW(ss, 10)",
                        IOT_SCHEMA, incremental=True)
    engine_mod.Engine(rule.plan).close()


# ------------------------------------------------------------------ incremental sliding / event-time count windows
from test_range_gpu import TRIG_SCHEMA, _iot, _with_trig   # noqa: E402


@pytest.mark.parametrize("batches", [1, 7])
def test_inc_sliding_over_when_out_of_order(oracle, engine_mod, batches):
    """SlidingWindowIncAggEventOp: each trigger emits a clone of the OLDEST open window (window_inc_agg_event_op.go:257-272)."""
    sql = ("SELECT deviceId, count(*), sum(temperature), min(humidity), max(temperature), avg(humidity) FROM demo "
           "GROUP BY deviceId, SLIDINGWINDOW(ms, 400) OVER (WHEN trig = 1)")
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=80, late_tolerance_ms=100, incremental=True, debug_membership=True)
    cols = _with_trig(_iot(60_000, 80, seed=96, epm=3), 120)
    rng = np.random.default_rng(13)
    cols[1] = (cols[1] + rng.integers(-150, 150, len(cols[1]))).astype(np.int64)
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert exp.records_late > 0 and st.records_late == exp.records_late
    assert len(got) > 100
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_inc_sliding_every_row(oracle, engine_mod):
    sql = "SELECT deviceId, count(*), sum(humidity) FROM demo GROUP BY deviceId, SLIDINGWINDOW(ms, 25)"
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=12, incremental=True, debug_membership=True)
    cols = _with_trig(_iot(5000, 12, seed=97, epm=4), 10)
    for batches in (1, 6):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert len(got) == len(exp.windows) > 4900
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("batches", [1, 9])
def test_inc_event_time_count_window(oracle, engine_mod, batches):
    """CountWindowIncAggEventOp: blocks of n released rows, emitted at the next watermark (window_inc_agg_event_op.go:351-408)."""
    sql = "SELECT deviceId, count(*), sum(temperature), max(humidity) FROM demo GROUP BY deviceId, COUNTWINDOW(700)"
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=300, late_tolerance_ms=200, incremental=True, debug_membership=True)
    cols = _with_trig(_iot(90_000, 300, seed=98, epm=5), 10)
    rng = np.random.default_rng(14)
    cols[1] = (cols[1] + rng.integers(-300, 300, len(cols[1]))).astype(np.int64)
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert st.records_late == exp.records_late
    assert len(got) > 30
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("sql", ["SELECT deviceId, count(*), sum(temperature) FROM demo "
                                 "GROUP BY deviceId, SLIDINGWINDOW(ms, 300) OVER (WHEN trig = 1)",
                                 "SELECT deviceId, count(*), min(temperature) FROM demo GROUP BY deviceId, COUNTWINDOW(500)"])
def test_inc_sliding_count_checkpoint_restore(oracle, engine_mod, sql):
    rule = compile_rule(sql, TRIG_SCHEMA, num_keys=100, incremental=True, late_tolerance_ms=100, debug_membership=True)
    cols = _with_trig(_iot(50_000, 100, seed=99, epm=4), 100)
    got, exp, st, _ = run_split(oracle, engine_mod, rule, cols, cut=23_456, twice=True)
    assert st.records_late == exp.records_late
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
