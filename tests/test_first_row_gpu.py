"""GPU parity of first-row select fields (EK_AGG_FIRST, row.go:720-726): the engine folds a hidden event-buffer
position column with MIN on every aggregation path (window-major, small windows, key-major) and k_first_fetch swaps in
the source column's value. Against the oracle: the reference's project_test.go #11 / #12 KAT, and tumbling / hopping /
sliding / count / session windows with WHERE, nulls, out-of-order input, several pushes, un-grouped rules and forced
key-major launches."""
import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401
from test_first_row import SCHEMA, SQL, kat_columns

pytestmark = pytest.mark.gpu

SCH = dict(IOT_SCHEMA, v="bigint")


def _stream(n, keys, seed, epm=10, ooo=False):
    key, ts, temp, hum = iot_stream(n, keys, seed=seed, events_per_ms=epm)
    rng = np.random.default_rng(seed)
    if ooo:
        ts = ts - rng.integers(0, 40, n) * (rng.random(n) < 0.2)
    v = rng.integers(-50, 50, n).astype(np.int64)
    return [key, ts.astype(np.int64), temp, hum, v]


@pytest.mark.parametrize("case12", [False, True])
def test_first_row_project_kat(oracle, engine_mod, case12):
    cols, valid = kat_columns(case12)
    rule = compile_rule(SQL, SCHEMA, num_keys=2, nullable=("id1",), debug_membership=True)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, validity=valid)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    rows = {int(k): (int(t), int(v)) for k, t, v in zip(got[0].keys, got[0].tags[0], got[0].values[0])}
    assert rows[0] == (A.EK_TAG_I64, 1)
    assert rows[1] == ((A.EK_TAG_NULL, 0) if case12 else (A.EK_TAG_I64, 2))


@pytest.mark.parametrize("sql,batches,ooo", [
    ("SELECT deviceId, temperature, v, avg(humidity), count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 2)", 3, True),
    ("SELECT deviceId, humidity, max(temperature) FROM demo WHERE v > 0 GROUP BY deviceId, HOPPINGWINDOW(ss, 4, 2)", 2, False),
    ("SELECT deviceId, v, stddev(temperature) FROM demo GROUP BY deviceId, SLIDINGWINDOW(ss, 2) OVER (WHEN v = 49) "
     "HAVING count(*) > 1", 4, True),
    ("SELECT deviceId, temperature, median(humidity) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 3)", 2, False),
    ("SELECT temperature, v, count(*), sum(v) FROM demo GROUP BY TUMBLINGWINDOW(ss, 1)", 3, True),
])
def test_first_row_window_kinds(oracle, engine_mod, sql, batches, ooo):
    rule = compile_rule(sql, SCH, num_keys=500, late_tolerance_ms=50 if ooo else 0, debug_membership=True)
    cols = _stream(120_000, 500, seed=5, ooo=ooo)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert len(exp.windows) >= 3
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_first_row_count_and_session_with_nulls(oracle, engine_mod):
    rng = np.random.default_rng(8)
    cols = _stream(60_000, 300, seed=9)
    cols[1] = cols[1] + 1500 * (np.arange(60_000) // 12_000)   # 1.5 s gaps: the 1 s session timeout closes sessions
    valid = [None, None, (rng.random(60_000) > 0.3).astype(np.uint8), None, (rng.random(60_000) > 0.5).astype(np.uint8)]
    for sql, iet in (("SELECT deviceId, temperature, v, count(*) FROM demo GROUP BY deviceId, COUNTWINDOW(500)", False),
                     ("SELECT deviceId, v, temperature, avg(humidity) FROM demo GROUP BY deviceId, SESSIONWINDOW(ss, 5, 1)", True)):
        rule = compile_rule(sql, SCH, num_keys=300, is_event_time=iet, nullable=("temperature", "v"), debug_membership=True)
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, validity=valid, batches=3)
        assert len(exp.windows) >= 3
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("km", ["0", "1"])
def test_first_row_key_major_and_window_major(oracle, engine_mod, km, monkeypatch):
    """Overlapping sliding windows over many keys: key-major (position column sorted by key; the first member of a
    key's run is its first row) and window-major (MIN over staged positions) give the same first rows."""
    monkeypatch.setenv("EKGPU_KEYMAJOR", km)
    monkeypatch.setenv("EKGPU_SMALL_WIN", "0")
    sql = ("SELECT deviceId, temperature, v, count(*) FROM demo GROUP BY deviceId, SLIDINGWINDOW(ss, 3) "
           "OVER (WHEN v = 7)")
    rule = compile_rule(sql, SCH, num_keys=4000, debug_membership=True)
    cols = _stream(200_000, 4000, seed=13, epm=20)
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=2)
    assert len(exp.windows) > 50
    assert (st.windows_keymajor > 0) == (km == "1")
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_first_row_string_field(oracle, engine_mod):
    """A first-row field over a string column: the engine returns the dictionary code of the first row's string."""
    schema = {"deviceId": "key", "ts": "bigint", "name": "string", "x": "float"}
    n = 40_000
    rng = np.random.default_rng(21)
    words = np.array(["alpha", "beta", "gamma", "delta", "eps"])
    raw = [rng.integers(0, 200, n).astype(np.uint32), (1541152480000 + np.arange(n) // 10).astype(np.int64),
           list(words[rng.integers(0, 5, n)]), rng.uniform(0, 1, n)]
    rule = compile_rule("SELECT deviceId, name, max(x) FROM s GROUP BY deviceId, TUMBLINGWINDOW(ms, 700)", schema,
                        num_keys=200, debug_membership=True)
    cols, _ = rule.device_columns(raw)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=2)
    assert len(exp.windows) >= 3
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    w = got[0]
    first = {}
    for i in range(n):   # the oracle-independent check of one window: the first row of each key in [start, end)
        if w.start <= raw[1][i] < w.end and int(raw[0][i]) not in first:
            first[int(raw[0][i])] = raw[2][i]
    assert dict(zip(map(int, w.keys), rule.decode_value(1, w.values[1], w.tags[1]))) == first
