"""GPU parity of the key-major range path (ek_keymajor.h): the fired windows' span sorted once by key, one thread per
key walking the windows. EKGPU_KEYMAJOR=1 takes it whenever the windows are eligible (the default cost rule takes it
only for big key spaces), so the range-mode cases of test_range_gpu.py run through it here against the oracle; the
cases it must decline (WHERE errors in the span, order statistics over long per-key runs) fall back to the
window-major path and stay green."""
import os

import numpy as np
import pytest

import test_range_gpu as R
from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401  (fixture + helper)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def keymajor_forced():
    os.environ["EKGPU_KEYMAJOR"] = "1"
    yield
    del os.environ["EKGPU_KEYMAJOR"]


def _force_range():
    os.environ["EKGPU_FORCE_RANGE"] = "1"


def _unforce_range():
    os.environ.pop("EKGPU_FORCE_RANGE", None)


@pytest.mark.parametrize("batches", [1, 5])
def test_km_sliding_over_when_c4a_shape(oracle, engine_mod, batches):
    sql = ("SELECT deviceId, stddev(temperature), var(temperature), count(*) FROM demo "
           "GROUP BY deviceId, SLIDINGWINDOW(ss, 3) OVER (WHEN trig = 1) HAVING count(*) > 1")
    rule = compile_rule(sql, R.TRIG_SCHEMA, num_keys=3000, debug_membership=True)
    cols = R._with_trig(R._iot(200_000, 3000, seed=61, epm=10), 500)
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert len(got) > 100
    assert st.windows_keymajor > 0
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_km_sliding_every_event(oracle, engine_mod):
    R.test_sliding_every_event(oracle, engine_mod)


def test_km_sliding_late_tolerance_out_of_order(oracle, engine_mod):
    R.test_sliding_late_tolerance_out_of_order(oracle, engine_mod)


def test_km_sliding_with_delay(oracle, engine_mod):
    R.test_sliding_with_delay(oracle, engine_mod)


@pytest.mark.parametrize("n,m", [(1000, 0), (500, 200), (300, 700)])
def test_km_count_window(oracle, engine_mod, n, m):
    os.environ["EKGPU_SMALL_WIN"] = "0"   # the 1000-row windows would otherwise take k_small_win
    try:
        R.test_count_window(oracle, engine_mod, n, m)
    finally:
        del os.environ["EKGPU_SMALL_WIN"]


def test_km_session_window(oracle, engine_mod):
    R.test_session_window(oracle, engine_mod)


def test_km_tumbling_hopping_range(oracle, engine_mod):
    _force_range()
    try:
        R.test_tumbling_hopping_through_range_mode(oracle, engine_mod, None)
        R.test_range_out_of_order_tumbling(oracle, engine_mod, None)
    finally:
        _unforce_range()


@pytest.mark.parametrize("keys", [4000, 100, 3])
def test_km_median_percentile(oracle, engine_mod, keys):
    """4000 keys: short per-key runs, sorted in the thread's LDS lane (and walked by the E / X merge); 100 keys: ~50
    values per (key, window), more than kKmSegMax: the count pass flags them and the window-major radix select takes
    over (the in-memory rank counting that once served them faulted on MI355X); 3 keys: the same."""
    rule = compile_rule(R.MED_SQL, IOT_SCHEMA, num_keys=keys, debug_membership=True)
    cols = R._iot(300_000, keys, seed=71, epm=5)
    if keys > 3:   # 1 s windows
        rule = compile_rule(R.MED_SQL.replace("TUMBLINGWINDOW(ss, 10)", "TUMBLINGWINDOW(ss, 1)"), IOT_SCHEMA,
                            num_keys=keys, debug_membership=True)
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=2)
    assert len(got) >= 4
    assert (st.windows_keymajor > 0) == (keys > 100)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_km_median_int_nulls(oracle, engine_mod):
    R.test_median_percentile_int_columns_nulls(oracle, engine_mod)


def test_km_percentile_window_error(oracle, engine_mod):
    R.test_percentile_out_of_range_is_window_error(oracle, engine_mod)


def test_km_c5_shape(oracle, engine_mod):
    R.test_c5_shape_high_cardinality_median(oracle, engine_mod)


def test_km_sliding_median(oracle, engine_mod):
    R.test_sliding_median(oracle, engine_mod)


def test_km_where_having_errors(oracle, engine_mod):
    """A WHERE that errors on some rows (int / 0) makes its span ineligible (window-major fallback attributes the error
    per window); HAVING errors (int / 0 on aggregates) are raised by the key-major write pass. Some windows of each
    stream error, the others keep their rows."""
    schema = {"k": "key", "ts": "bigint", "a": "bigint", "b": "bigint", "trig": "bigint"}
    n = 30_000
    rng = np.random.default_rng(12)
    ts = (1541152480000 + np.arange(n) // 3).astype(np.int64)
    a = rng.integers(-20, 20, n).astype(np.int64)
    b = rng.integers(0, 5000, n).astype(np.int64)
    trig = (rng.integers(0, 300, n) == 0).astype(np.int64)
    for sql, keys in (
            ("SELECT k, count(*), sum(a) FROM s WHERE a / b >= 0 GROUP BY k, SLIDINGWINDOW(ms, 800) OVER (WHEN trig = 1)", 40),
            ("SELECT k, count(*), sum(a) FROM s WHERE a > 0 GROUP BY k, SLIDINGWINDOW(ms, 800) OVER (WHEN trig = 1) "
             "HAVING sum(a) / (count(*) - 300) > 1", 4)):
        k = np.random.default_rng(13).integers(0, keys, n).astype(np.uint32)
        rule = compile_rule(sql, schema, num_keys=keys, debug_membership=True)
        got, exp, _ = run_both(oracle, engine_mod, rule, [k, ts, a, b, trig], batches=3)
        st = [w.status for w in exp.windows]
        assert len(got) > 10 and 0 < sum(s != 0 for s in st) < len(st)
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_km_auto_rule_picks_big_key_spaces(oracle, engine_mod):
    """Default cost rule (EKGPU_KEYMAJOR unset): a heavily overlapping sliding window over 100 k keys goes key-major."""
    del os.environ["EKGPU_KEYMAJOR"]
    try:
        sql = ("SELECT deviceId, stddev(temperature), var(temperature) FROM demo "
               "GROUP BY deviceId, SLIDINGWINDOW(ss, 5) OVER (WHEN trig = 1) HAVING count(*) > 1")
        rule = compile_rule(sql, R.TRIG_SCHEMA, num_keys=100_000)
        key, ts, temp, hum = iot_stream(1_000_000, 100_000, seed=81, events_per_ms=20)
        cols = R._with_trig([key, ts, temp, hum], 2000)
        got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=2)
        assert len(got) > 100 and st.windows_keymajor > 0
        assert_windows_equal(rule.plan, got, exp.windows)
    finally:
        os.environ["EKGPU_KEYMAJOR"] = "1"


def _push_per_window(oracle, engine_mod, rule, cols, window_ms, validity=None):
    """One push per tumbling window's events: every push (but the first) fires exactly one window, so the
    key-major launch holds ONE window (single pass: no positions, block-compacted rows)."""
    exp = oracle.run(rule.plan, cols, validity)
    ts = cols[1]
    ends = np.arange((ts[0] // window_ms + 1) * window_ms, ts[-1] + 1, window_ms)
    cuts = np.concatenate([[0], np.searchsorted(ts, ends), [len(ts)]]).astype(np.int64)
    eng = engine_mod.Engine(rule.plan)
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        if hi > lo:
            eng.push_host([c[lo:hi] for c in cols], None if validity is None else
                          [None if v is None else v[lo:hi] for v in validity])
    got = eng.poll()
    st = eng.stats()
    eng.close()
    return got, exp, st


@pytest.mark.parametrize("sql", [
    # one value column, no validity: the column itself is sorted by key (no gather)
    "SELECT deviceId, median(temperature), percentile_cont(temperature, 0.9), count(*) FROM demo "
    "GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)",
    # two value columns: positions sorted + gathered, still one pass
    "SELECT deviceId, median(temperature), percentile_disc(humidity, 0.5), avg(humidity), stddev(temperature) "
    "FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 1) HAVING count(*) > 2",
])
def test_km_one_window_per_push(oracle, engine_mod, sql):
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=20_000, debug_membership=True)
    cols = R._iot(400_000, 20_000, seed=91, epm=50)
    got, exp, st = _push_per_window(oracle, engine_mod, rule, cols, 1000)
    assert len(exp.windows) >= 5 and st.windows_keymajor >= len(exp.windows)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_km_one_window_nulls_and_long_runs(oracle, engine_mod):
    """Nullable value column (validity staged, positions path) and a key space small enough that a key's run exceeds
    kKmSegMax: the one-window launch is declined before anything is written and the window-major path answers."""
    schema = {"deviceId": "key", "ts": "bigint", "v": "bigint", "w": "float"}
    rng = np.random.default_rng(17)
    n = 120_000
    ts = (1541152480000 + np.arange(n) // 40).astype(np.int64)
    for keys in (20_000, 40):
        k = rng.integers(0, keys, n).astype(np.uint32)
        cols = [k, ts, rng.integers(-100, 100, n).astype(np.int64), rng.uniform(0, 1, n)]
        valid = [None, None, None, (rng.random(n) > 0.2).astype(np.uint8)]
        sql = ("SELECT deviceId, median(v), percentile_cont(w, 0.5), count(w), max(w) FROM s "
               "GROUP BY deviceId, TUMBLINGWINDOW(ms, 500)")
        rule = compile_rule(sql, schema, num_keys=keys, nullable=("w",), debug_membership=True)
        got, exp, st = _push_per_window(oracle, engine_mod, rule, cols, 500, validity=valid)
        assert len(exp.windows) >= 4
        assert (st.windows_keymajor > 0) == (keys > 40)
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_km_write_pass_many_aggregates(oracle, engine_mod):
    """The multi-window write pass (cursor per (window, block) starting at the block's offset) with many aggregates
    over heavily overlapping sliding windows."""
    sql = ("SELECT deviceId, count(*), sum(temperature), avg(humidity), min(temperature), max(humidity), "
           "stddev(temperature), vars(humidity), count(humidity) FROM demo "
           "GROUP BY deviceId, SLIDINGWINDOW(ss, 4) OVER (WHEN trig = 1) HAVING count(*) > 1")
    rule = compile_rule(sql, R.TRIG_SCHEMA, num_keys=5000, debug_membership=True)
    cols = R._with_trig(R._iot(400_000, 5000, seed=37, epm=20), 3000)
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=2)
    assert len(got) > 100 and st.windows_keymajor > 0
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("grp", ["0", "1"])
@pytest.mark.parametrize("sql,col", [
    ("SELECT deviceId, median(temperature), percentile_cont(temperature, 0.9), count(*) FROM demo "
     "GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)", "float"),
    ("SELECT deviceId, median(v), percentile_disc(v, 0.25), avg(v), stddev(v) FROM demo "
     "GROUP BY deviceId, TUMBLINGWINDOW(ss, 1) HAVING count(*) > 2", "int"),
    # no order statistic, HAVING over count(*) alone: decided in the grouped walk after its fold
    ("SELECT deviceId, avg(temperature), max(temperature) FROM demo "
     "GROUP BY deviceId, TUMBLINGWINDOW(ss, 1) HAVING count(*) > 2", "float"),
])
def test_km_one_window_grouped_huge_keys(oracle, engine_mod, grp, sql, col, monkeypatch):
    """K > 2^16, one window per push, one value column: EKGPU_GRP=1 (default) takes the MSD-partitioned grouping
    (k_grp_*: two 8-bit digit passes, then LDS grouping per sub-bucket); =0 the radix-sorted key-major walk."""
    monkeypatch.setenv("EKGPU_GRP", grp)
    if "median" not in sql:   # no order statistic: range mode must be forced (the rule would run in pane mode)
        monkeypatch.setenv("EKGPU_FORCE_RANGE", "1")
    keys = 150_000
    cols = R._iot(1_200_000, keys, seed=57, epm=300)
    schema = dict(IOT_SCHEMA)
    if col == "int":
        cols = cols[:4] + [np.random.default_rng(2).integers(-1000, 1000, len(cols[0])).astype(np.int64)]
        schema["v"] = "bigint"
    rule = compile_rule(sql, schema, num_keys=keys, debug_membership=True)
    got, exp, st = _push_per_window(oracle, engine_mod, rule, cols, 1000)
    assert len(exp.windows) >= 3 and st.windows_keymajor >= len(exp.windows)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_km_one_window_grouped_skewed_falls_back(oracle, engine_mod):
    """A hot key puts more than kGrpCap rows into one sub-bucket: the grouped path declines before writing anything
    and the radix-sorted walk answers."""
    keys = 100_000
    cols = R._iot(600_000, keys, seed=58, epm=200)
    cols[0][::7] = 12345                       # ~86 k rows of one key
    rule = compile_rule("SELECT deviceId, max(temperature), count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)",
                        IOT_SCHEMA, num_keys=keys, debug_membership=True)
    os.environ["EKGPU_KEYMAJOR"] = "1"
    got, exp, st = _push_per_window(oracle, engine_mod, rule, cols, 1000)
    assert len(exp.windows) >= 2
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("msd", ["1", "0"])
@pytest.mark.parametrize("sql", [
    "SELECT deviceId, stddev(temperature), var(temperature), count(*) FROM demo "
    "GROUP BY deviceId, SLIDINGWINDOW(ss, 3) OVER (WHEN trig = 1) HAVING count(*) > 1",
    "SELECT deviceId, median(temperature), count(*) FROM demo GROUP BY deviceId, SLIDINGWINDOW(ss, 3) OVER (WHEN trig = 1)",
])
def test_km_msd_span_sort(oracle, engine_mod, monkeypatch, msd, sql):
    """The key-major span sort by MSD partition (km_msd: two k_grp_scatter<true> passes carrying value and position,
    k_kmsd_fix sorting each 2^s2-key sub-bucket by (key, position)) against the radix sort + gather (EKGPU_KM_MSD=0):
    both equal the oracle, over 80 000 keys (>= 65 536: the MSD path's range) and several pushes."""
    monkeypatch.setenv("EKGPU_KM_MSD", msd)
    rule = compile_rule(sql, R.TRIG_SCHEMA, num_keys=80_000, debug_membership=True)
    cols = R._with_trig(R._iot(300_000, 80_000, seed=67, epm=10), 400)
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=3)
    assert st.windows_keymajor > 0
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_km_msd_skewed_sub_bucket_falls_back(oracle, engine_mod, monkeypatch):
    """A sub-bucket above kGrpCap rows (half the rows on one key) sends km_msd back to the radix sort: same results."""
    monkeypatch.setenv("EKGPU_KM_MSD", "1")
    sql = ("SELECT deviceId, stddev(temperature), count(*) FROM demo "
           "GROUP BY deviceId, SLIDINGWINDOW(ss, 3) OVER (WHEN trig = 1)")
    rule = compile_rule(sql, R.TRIG_SCHEMA, num_keys=70_000, debug_membership=True)
    cols = R._with_trig(R._iot(200_000, 70_000, seed=71, epm=10), 400)
    cols[0][::2] = 12_345
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=2)
    assert st.windows_keymajor > 0
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
