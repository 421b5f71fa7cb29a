"""GPU tests of ek_export_state / ek_import_state (checkpoint + restore).

The reference checkpoints the window chain through ctx.PutState (watermark_op.go:204-211, window_op.go:283-340) and a
restarted rule resumes from ctx.GetState (watermark_op.go:72-101, window_op.go:131-168). Here a stream is cut at an
arbitrary event, the first part is pushed into one handle, its state is exported, the handle is DESTROYED, a fresh
handle imports the blob and receives the rest: the windows of both handles together must equal the oracle's
windows of the uncut stream (values, membership, lateness counters)."""
import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod  # noqa: F401  (fixture)
from test_range_gpu import TRIG_SCHEMA, _iot, _with_trig

pytestmark = pytest.mark.gpu


def _push(eng, cols, lo, hi, batches, validity=None):
    cuts = np.linspace(lo, hi, batches + 1).astype(np.int64)
    for b in range(batches):
        a, e = cuts[b], cuts[b + 1]
        if e > a:
            eng.push_host([c[a:e] for c in cols], None if validity is None else
                          [None if v is None else v[a:e] for v in validity])


def run_split(oracle, engine_mod, rule, cols, cut, batches=(3, 4), validity=None, twice=False):
    exp = oracle.run(rule.plan, cols, validity)
    n = len(cols[0])
    a = engine_mod.Engine(rule.plan)
    _push(a, cols, 0, cut, batches[0], validity)
    got = list(a.poll())
    blob = a.export_state()
    a.close()
    b = engine_mod.Engine(rule.plan)
    b.import_state(blob)
    if twice:   # checkpoint again mid-way through the second part, restore into a third handle
        mid = (cut + n) // 2
        _push(b, cols, cut, mid, 2, validity)
        got += list(b.poll())
        blob2 = b.export_state()
        b.close()
        b = engine_mod.Engine(rule.plan)
        b.import_state(blob2)
        cut = mid
    _push(b, cols, cut, n, batches[1], validity)
    got += list(b.poll())
    st = b.stats()
    b.close()
    return got, exp, st, blob


CASES = [
    # (id, sql, schema, compile kwargs, stream builder, cut fraction)
    ("tumbling_pane", "SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
     "GROUP BY deviceId, TUMBLINGWINDOW(ss, 2)", IOT_SCHEMA, dict(num_keys=500),
     lambda: _iot(100_000, 500, seed=81, epm=5), 0.37),
    ("hopping_pane", "SELECT deviceId, sum(temperature), min(temperature), max(humidity), stddev(humidity) FROM demo "
     "GROUP BY deviceId, HOPPINGWINDOW(ss, 6, 2)", IOT_SCHEMA, dict(num_keys=300),
     lambda: _iot(120_000, 300, seed=82, epm=4), 0.55),
    ("tumbling_pending", "SELECT deviceId, count(*), sum(humidity) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)",
     IOT_SCHEMA, dict(num_keys=50, late_tolerance_ms=1000), lambda: _iot(20_000, 50, seed=83, epm=5), 0.002),
    ("sliding_over_when", "SELECT deviceId, stddev(temperature), var(temperature), count(*) FROM demo "
     "GROUP BY deviceId, SLIDINGWINDOW(ss, 3) OVER (WHEN trig = 1) HAVING count(*) > 1", TRIG_SCHEMA,
     dict(num_keys=400), lambda: _with_trig(_iot(80_000, 400, seed=84, epm=10), 300), 0.61),
    ("sliding_delay", "SELECT deviceId, count(*), sum(temperature) FROM demo "
     "GROUP BY deviceId, SLIDINGWINDOW(ms, 200, 100) OVER (WHEN trig = 1)", TRIG_SCHEMA, dict(num_keys=30),
     lambda: _with_trig(_iot(30_000, 30, seed=85, epm=3), 300), 0.5),
    # event-time send-twice: the expired inputs kept, the queued triggers / timers and prevWindowEndTs travel (v7)
    ("sliding_send_twice_event", "SELECT deviceId, count(*), max(temperature) FROM demo "
     "GROUP BY deviceId, SLIDINGWINDOW(ms, 200, 100) OVER (WHEN trig = 1)", TRIG_SCHEMA,
     dict(num_keys=30, sliding_send_twice=True), lambda: _with_trig(_iot(30_000, 30, seed=90, epm=3), 300), 0.45),
    ("count_window", "SELECT deviceId, avg(temperature), count(*) FROM demo GROUP BY deviceId, COUNTWINDOW(700, 300)",
     IOT_SCHEMA, dict(num_keys=60, is_event_time=False), lambda: _iot(20_000, 60, seed=86, epm=10), 0.43),
    ("state_window_proc", "SELECT deviceId, count(*), sum(temperature), max(humidity) FROM demo "
     "GROUP BY deviceId, STATEWINDOW(trig = 1, humidity > 99)", TRIG_SCHEMA,
     dict(num_keys=100, is_event_time=False), lambda: _with_trig(_iot(40_000, 100, seed=88, epm=10), 300), 0.52),
    ("state_window_event", "SELECT deviceId, count(*), min(temperature) FROM demo "
     "GROUP BY deviceId, STATEWINDOW(trig = 1, humidity > 98)", TRIG_SCHEMA,
     dict(num_keys=100, late_tolerance_ms=200), lambda: _with_trig(_iot(40_000, 100, seed=89, epm=5), 200), 0.47),
    ("median_range", "SELECT deviceId, median(temperature), percentile_disc(humidity, 0.5), count(*) FROM demo "
     "GROUP BY deviceId, TUMBLINGWINDOW(ss, 2)", IOT_SCHEMA, dict(num_keys=200),
     lambda: _iot(60_000, 200, seed=87, epm=5), 0.71),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c[0])
def test_checkpoint_restore_matches_uncut_stream(oracle, engine_mod, case):
    _, sql, schema, kw, build, frac = case
    rule = compile_rule(sql, schema, debug_membership=True, **kw)
    cols = build()
    cut = max(1, int(len(cols[0]) * frac))
    got, exp, st, blob = run_split(oracle, engine_mod, rule, cols, cut)
    assert len(blob) > 0
    assert st.records_late == exp.records_late
    assert st.records_in == len(cols[0])
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_checkpoint_twice_out_of_order(oracle, engine_mod):
    """Pane mode with late drops and unsorted batches, checkpointed twice."""
    sql = "SELECT deviceId, count(*), sum(temperature), max(humidity) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 2)"
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=50, late_tolerance_ms=700, debug_membership=True)
    key, ts, temp, hum = iot_stream(30_000, 50, seed=88, events_per_ms=2)
    rng = np.random.default_rng(8)
    ts = (ts + rng.integers(-1500, 1500, size=len(ts))).astype(np.int64)
    cols = [key, ts, temp, hum]
    got, exp, st, _ = run_split(oracle, engine_mod, rule, cols, 9_001, batches=(4, 5), twice=True)
    assert exp.records_late > 0 and st.records_late == exp.records_late
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_checkpoint_session_twice(oracle, engine_mod):
    sql = "SELECT deviceId, count(*), max(temperature) FROM demo GROUP BY deviceId, SESSIONWINDOW(ss, 10, 2)"
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=50, debug_membership=True)
    key, ts, temp, hum = iot_stream(20_000, 50, seed=89, events_per_ms=1)
    ts = ts + (np.arange(len(ts)) // 3000) * 3500
    cols = [key, ts.astype(np.int64), temp, hum]
    got, exp, _, _ = run_split(oracle, engine_mod, rule, cols, 7_777, twice=True)
    assert len(exp.windows) >= 3
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_checkpoint_nullable_range_mode(oracle, engine_mod):
    schema = {"k": "key", "ts": "bigint", "a": "bigint", "b": "bigint"}
    sql = ("SELECT k, median(a), percentile_cont(b, 0.5), count(b), sum(b) FROM s "
           "GROUP BY k, TUMBLINGWINDOW(ss, 1) HAVING count(*) > 1")
    rule = compile_rule(sql, schema, num_keys=37, nullable=("b",), debug_membership=True)
    n = 30_000
    rng = np.random.default_rng(10)
    k = rng.integers(0, 37, n).astype(np.uint32)
    ts = (1541152480000 + np.arange(n) // 4).astype(np.int64)
    a = rng.integers(-50, 50, n).astype(np.int64)
    b = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    vb = (rng.random(n) > 0.4).astype(np.uint8)
    got, exp, _, _ = run_split(oracle, engine_mod, rule, [k, ts, a, b], 12_345, validity=[None, None, None, vb])
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_export_requires_polled_results_and_matching_plan(engine_mod):
    sql = "SELECT deviceId, count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)"
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=20)
    cols = _iot(10_000, 20, seed=90, epm=2)
    eng = engine_mod.Engine(rule.plan)
    eng.push_host(cols)
    with pytest.raises(engine_mod.EngineError) as e:
        eng.export_state()                       # windows emitted but not polled
    assert e.value.code == A.EK_ERR_STATE
    eng.poll()
    blob = eng.export_state()
    other = engine_mod.Engine(compile_rule(sql.replace("ss, 1", "ss, 2"), IOT_SCHEMA, num_keys=20).plan)
    with pytest.raises(engine_mod.EngineError) as e:
        other.import_state(blob)                 # a different rule
    assert e.value.code == A.EK_ERR_INVALID
    other.close()
    # the plan hash covers the window FILTER clause and send-twice: a blob of another FILTER is another plan
    fsql = "SELECT deviceId, count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 1) FILTER (WHERE temperature > 20)"
    fa = engine_mod.Engine(compile_rule(fsql, IOT_SCHEMA, num_keys=20).plan)
    fa.push_host(cols)
    fa.poll()
    fblob = fa.export_state()
    fa.close()
    for osql in (fsql.replace("> 20", "> 30"), sql):
        fo = engine_mod.Engine(compile_rule(osql, IOT_SCHEMA, num_keys=20).plan)
        with pytest.raises(engine_mod.EngineError) as e:
            fo.import_state(fblob)
        assert e.value.code == A.EK_ERR_INVALID
        fo.close()
    fresh = engine_mod.Engine(rule.plan)
    with pytest.raises(engine_mod.EngineError) as e:
        fresh.import_state(blob[: len(blob) - 9])   # truncated
    assert e.value.code == A.EK_ERR_INVALID
    fresh.import_state(blob)                     # the handle stays usable after a refused blob
    more = _iot(4_000, 20, seed=91, epm=2)
    more[1] = more[1] + (int(cols[1][-1]) - int(more[1][0]) + 1)
    fresh.push_host(more)
    assert len(fresh.poll()) >= 1
    fresh.close()
    eng.close()


# ------------------------------------------------------------------ processing time (the caller's clock)
PROC_CASES = [
    ("proc_tumbling", "SELECT k, avg(x), count(*) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1)", {}),
    ("proc_hopping_filter", "SELECT k, max(x), count(*) FROM s GROUP BY k, HOPPINGWINDOW(ss, 2, 1) FILTER (WHERE y > 30)", {}),
    ("proc_sliding", "SELECT k, count(*), min(y) FROM s GROUP BY k, SLIDINGWINDOW(ms, 400) OVER (WHEN x > 97)", {}),
    ("proc_sliding_delay", "SELECT k, count(*), sum(y) FROM s GROUP BY k, SLIDINGWINDOW(ms, 300, 500) OVER (WHEN x > 98)", {}),
    ("proc_send_twice", "SELECT k, count(*), max(y) FROM s GROUP BY k, SLIDINGWINDOW(ms, 300, 500) OVER (WHEN x > 98)",
     dict(sliding_send_twice=True)),
    ("proc_session", "SELECT k, count(*), avg(x) FROM s WHERE y < 70 GROUP BY k, SESSIONWINDOW(ss, 3, 1)", {}),
]


@pytest.mark.parametrize("name,sql,kw", PROC_CASES, ids=[c[0] for c in PROC_CASES])
def test_state_processing_time_split(oracle, engine_mod, name, sql, kw):
    """Processing-time rules checkpointed mid-stream: the clock, the next tick, an armed session timeout, pending
    delay timers and the send-twice inputs state travel in the blob (state version 3), so the restored handle goes on
    exactly where the exported one stopped (the same windows as the uncut run under the same clock)."""
    from test_processing_gpu import SCHEMA as PSCHEMA, _stream
    cols = _stream(40_000, 30, seed=len(name) * 7 + 3, gap_ms=6, burst=True)
    rule = compile_rule(sql, PSCHEMA, is_event_time=False, num_keys=30, debug_membership=True, **kw)
    start, end = int(cols[1][0]) - 777, int(cols[1][-1]) + 6_000
    exp = oracle.run_proc(rule.plan, cols, start, end)
    n = len(cols[0])
    cut = int(n * 0.47)
    clock = int(cols[1][cut - 1]) + 3       # the clock when the checkpoint is taken (no row at or after it yet)
    a = engine_mod.Engine(rule.plan)
    a.advance_time(start)
    for lo, hi in ((0, cut // 2), (cut // 2, cut)):
        a.advance_time(int(cols[1][lo]))
        a.push_host([c[lo:hi] for c in cols])
    if clock <= int(cols[1][cut]):
        a.advance_time(clock)
    got = list(a.poll())
    blob = a.export_state()
    a.close()
    b = engine_mod.Engine(rule.plan)
    b.import_state(blob)
    for lo, hi in ((cut, (cut + n) // 2), ((cut + n) // 2, n)):
        b.advance_time(int(cols[1][lo]))
        b.push_host([c[lo:hi] for c in cols])
    b.advance_time(end)
    got += list(b.poll())
    b.close()
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_state_processing_idle_gap(oracle, engine_mod):
    """A clock jump over thousands of empty tumbling windows (pane mode): they are reported empty without pane slots
    or result rows (an idle day of 1 s windows used to allocate 86,400 x keys partials)."""
    from test_processing_gpu import SCHEMA as PSCHEMA
    rule = compile_rule("SELECT k, count(*), sum(x) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1)", PSCHEMA, is_event_time=False,
                        num_keys=65536, debug_membership=True)
    t0 = 1541152480000
    ts = np.array([t0 + 10, t0 + 20, t0 + 20 + 86_400_000, t0 + 86_400_500], np.int64)
    cols = [np.array([1, 2, 3, 1], np.uint32), ts, np.array([1.0, 2.0, 3.0, 4.0]), np.zeros(4)]
    exp = oracle.run_proc(rule.plan, cols, t0, int(ts[-1]) + 3_000)
    assert len(exp.windows) > 86_000
    eng = engine_mod.Engine(rule.plan)
    eng.advance_time(t0)
    eng.push_host([c[:2] for c in cols])
    eng.advance_time(int(ts[2]))
    eng.push_host([c[2:] for c in cols])
    eng.advance_time(int(ts[-1]) + 3_000)
    got = eng.poll()
    eng.close()
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
