"""Hopping windows across event-time gaps: the empty-window discard of WindowOperator.handleInputs.

window_op.go:605-655: when a triggered hopping window holds no input (nextleft < 0), handleInputs returns
inputs[:0] and every buffered input is dropped. With lateTolerance 0 that is the event whose watermark step
triggered the empty window (k_hop_drop in ek_kernels.h). The CPU test pins the oracle on a hand-derived case;
the GPU tests compare the engine (pane mode and range mode, sorted / out-of-order / split batches) with it.
"""
import numpy as np
import pytest

from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal

SQL = ("SELECT deviceId, count(*), sum(temperature), min(humidity), avg(temperature) FROM demo "
       "GROUP BY deviceId, HOPPINGWINDOW(ss, 10, 5)")


def test_oracle_hopping_gap_kat(oracle):
    """Hand-derived from window_op.go:605-655 + event_window_trigger.go:124-180 (lateTolerance 0).

    ts 1000, 2000 -> E1 = 5000. ts 60000 raises the watermark to 60000: windows ending 5000 and 10000 hold
    {0, 1}; the window ending 15000 is empty, so inputs[:0] drops event 2 (ts 60000). ts 61000 -> no window.
    ts 80000: windows ending 65000 and 70000 hold {3} only; the one ending 75000 is empty and drops event 4.
    """
    rule = compile_rule(SQL, IOT_SCHEMA, num_keys=1, debug_membership=True)
    ts = np.array([1000, 2000, 60000, 61000, 80000], np.int64)
    cols = [np.zeros(5, np.uint32), ts, np.arange(5, dtype=np.float64), np.ones(5)]
    run = oracle.run(rule.plan, cols)
    got = [(w.end, sorted(int(x) for x in m)) for w, m in zip(run.windows, run.members) if len(m)]
    assert got == [(5000, [0, 1]), (10000, [0, 1]), (65000, [3]), (70000, [3])]


def _gap_stream(n, keys, seed, jitter=0):
    key, ts, temp, hum = iot_stream(n, keys, seed=seed, events_per_ms=2)
    rng = np.random.default_rng(seed)
    # event-time gaps of 3-40 s at random points: some exceed the 10 s window, some do not
    cuts = np.sort(rng.choice(np.arange(1, n), size=24, replace=False))
    shift = np.zeros(n, np.int64)
    for c in cuts:
        shift[c:] += int(rng.integers(3_000, 40_000))
    ts = ts + shift
    if jitter:
        ts = ts + rng.integers(-jitter, jitter + 1, size=n)
    return [key, ts.astype(np.int64), temp, hum]


@pytest.fixture(scope="module")
def engine_mod():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:
        pass
    from ekgpu import engine
    if engine.lib().ek_device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")
    return engine


def _run(engine_mod, rule, cols, batches):
    eng = engine_mod.Engine(rule.plan)
    n = len(cols[0])
    cuts = np.linspace(0, n, batches + 1).astype(np.int64)
    for b in range(batches):
        eng.push_host([c[cuts[b]:cuts[b + 1]] for c in cols])
    got = eng.poll()
    st = eng.stats()
    eng.close()
    return got, st


@pytest.mark.gpu
@pytest.mark.parametrize("jitter", [0, 300], ids=["sorted", "out_of_order"])
@pytest.mark.parametrize("batches", [1, 7, 200])
def test_hopping_gap_engine(oracle, engine_mod, jitter, batches):
    rule = compile_rule(SQL, IOT_SCHEMA, num_keys=64, debug_membership=True)
    cols = _gap_stream(60_000, 64, seed=71 + jitter, jitter=jitter)
    exp = oracle.run(rule.plan, cols)
    got, st = _run(engine_mod, rule, cols, batches)
    assert st.records_late == exp.records_late
    n_members = sum(len(m) for m in exp.members)
    assert n_members > 0
    assert st.records_discarded > 0
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.gpu
@pytest.mark.parametrize("batches", [1, 9])
def test_hopping_gap_engine_range_mode(oracle, engine_mod, batches):
    # median keeps the rule in range mode (device event buffer, windows as index ranges)
    sql = ("SELECT deviceId, count(*), median(temperature), max(humidity) FROM demo "
           "GROUP BY deviceId, HOPPINGWINDOW(ss, 10, 5)")
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=32, debug_membership=True)
    cols = _gap_stream(30_000, 32, seed=83)
    exp = oracle.run(rule.plan, cols)
    got, st = _run(engine_mod, rule, cols, batches)
    assert st.records_discarded > 0
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.gpu
@pytest.mark.parametrize("median", [False, True], ids=["pane", "range"])
def test_hopping_gap_checkpoint(oracle, engine_mod, median):
    # the discard check reads the carried stream max and E1: both must survive ek_export_state / ek_import_state
    from test_state_gpu import run_split
    sql = SQL if not median else ("SELECT deviceId, count(*), median(temperature) FROM demo "
                                  "GROUP BY deviceId, HOPPINGWINDOW(ss, 10, 5)")
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=16, debug_membership=True)
    cols = _gap_stream(20_000, 16, seed=97)
    for cut in (5_000, 13_333):
        got, exp, st, _ = run_split(oracle, engine_mod, rule, cols, cut, batches=(3, 5), twice=True)
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.gpu
@pytest.mark.parametrize("median", [False, True], ids=["pane", "range"])
def test_hopping_gap_one_event_per_push(oracle, engine_mod, median):
    # a push whose only event is discarded still advances the watermark and closes the windows below it
    sql = SQL if not median else ("SELECT deviceId, count(*), median(temperature) FROM demo "
                                  "GROUP BY deviceId, HOPPINGWINDOW(ss, 10, 5)")
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=4, debug_membership=True)
    ts = np.array([1000, 2000, 60000, 61000, 80000, 80500, 200000, 200001, 260000], np.int64)
    n = len(ts)
    cols = [(np.arange(n) % 4).astype(np.uint32), ts, np.arange(n, dtype=np.float64) * 1.5, np.ones(n)]
    exp = oracle.run(rule.plan, cols)
    got, st = _run(engine_mod, rule, cols, n)
    assert st.records_discarded == 4
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
