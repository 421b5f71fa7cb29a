"""The two lateTolerance > 0 paths where releasing events later than they arrive changes the reference's output:

* HOPPINGWINDOW: a triggered window with no member drops EVERY input present at the WatermarkTuple that fired it
  (handleInputs returns inputs[:0], window_op.go:605-655) - with lateTolerance > 0 those inputs include events
  released by the same tuple that belong to later windows;
* SESSIONWINDOW: getNextSessionWindow (event_window_trigger.go:77-110) runs at every WatermarkTuple; with
  lateTolerance > 0 a tuple can close a session by the trailing check (now - last input > timeout) before the event
  that would cut it at a tick boundary is released.

Engine vs oracle (per-event restatement) at 1, 7 and 200 pushes, on bursty out-of-order streams, plus a
hand-built session case traced through event_window_trigger.go."""
import numpy as np
import pytest

from ekgpu.rule import compile_rule
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401

pytestmark = pytest.mark.gpu
SCHEMA = {"deviceId": "key", "ts": "bigint", "temperature": "float"}
T0M = 1541152440000   # a minute boundary


def bursty(n, seed, burst=400, gap_ms=(500, 9000), jitter=600):
    rng = np.random.default_rng(seed)
    ts, t = [], T0M
    while len(ts) < n:
        k = int(rng.integers(1, burst))
        ts.extend(t + np.sort(rng.integers(0, 1500, k)))
        t += 1500 + int(rng.integers(*gap_ms))
    ts = np.array(ts[:n], dtype=np.int64)
    ts = ts - rng.integers(0, jitter, n) * (rng.random(n) < 0.2)   # out of order, some late
    return [rng.integers(0, 8, n).astype(np.uint32), ts, rng.integers(0, 800, n) / 8.0]


@pytest.mark.parametrize("pushes", [1, 7, 200])
@pytest.mark.parametrize("tol", [300, 1500])
def test_hopping_discard_late_tolerance(oracle, engine_mod, pushes, tol):
    sql = "SELECT deviceId, count(*), sum(temperature), max(temperature) FROM demo GROUP BY deviceId, HOPPINGWINDOW(ss, 3, 1)"
    rule = compile_rule(sql, SCHEMA, num_keys=8, late_tolerance_ms=tol, debug_membership=True)
    cols = bursty(6000, seed=tol + pushes)
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=pushes)
    assert len(exp.windows) > 20
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("pushes", [1, 7, 200])
@pytest.mark.parametrize("tol", [700, 2500])
def test_session_late_tolerance(oracle, engine_mod, pushes, tol):
    sql = "SELECT deviceId, count(*), avg(temperature) FROM demo GROUP BY deviceId, SESSIONWINDOW(ss, 10, 3)"
    rule = compile_rule(sql, SCHEMA, num_keys=8, late_tolerance_ms=tol, debug_membership=True)
    cols = bursty(6000, seed=tol * 3 + pushes, gap_ms=(200, 6000))
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=pushes)
    assert len(exp.windows) > 5
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_session_trailing_close_before_tick(oracle, engine_mod):
    """SESSIONWINDOW(ss, 10, 3), lateTolerance 2 s. Inputs from -12 s to p = -1 s (one per second) pass the tick at
    -10 s without a cut (the session began after tick - 10 s), so the next tick is 0. X = 4.5 s raises the
    watermark to 2.5 s: the tuple releases p and, with no later input, closes the session by the trailing check
    at p + 3 s = 2 s. q = 2.6 s arrives next (accepted: >= 2.5 s) and is released by Y = 7 s; a single evaluation
    at the final watermark would see q > tick and cut the session at the tick (0 s) instead."""
    ts = [T0M + s * 1000 for s in range(-12, 0)] + [T0M + 4500, T0M + 2600, T0M + 7000, T0M + 30000]
    n = len(ts)
    cols = [np.zeros(n, np.uint32), np.array(ts, np.int64), np.arange(n, dtype=np.float64)]
    sql = "SELECT deviceId, count(*), avg(temperature) FROM demo GROUP BY deviceId, SESSIONWINDOW(ss, 10, 3)"
    rule = compile_rule(sql, SCHEMA, num_keys=1, late_tolerance_ms=2000, debug_membership=True)
    exp = oracle.run(rule.plan, cols)
    assert exp.windows[0].end == T0M + 2000, [w.end - T0M for w in exp.windows]
    for pushes in (1, 3, n):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=pushes)
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
