"""median over a nullable FLOAT column (funcs_agg.go:29-55): the group's values in window order are arg0; a nil first
value is not a number ("<nil> should be number", the window's output replaced by "run Select error: ..."), the other
nils are ignored (cast.ToFloat64Slice IGNORE_NIL). The engine keeps the group's first row in a hidden first-row slot
and checks it on the emitted rows (k_first_fetch). Parity with the oracle's restatement (oracle/ekoracle.c agg_eval
EK_AGG_MEDIAN): results, statuses and error texts, on the range-mode window-major path, the key-major path and one row
per push. A BIGINT column (a nil anywhere fails, the text names the whole group) and HAVING stay refused."""
import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401  (fixture + helper)
from test_window_error_gpu import _assert_errors

pytestmark = pytest.mark.gpu
SCHEMA = {"k": "key", "ts": "bigint", "x": "float", "y": "bigint"}


def _stream(n, keys, seed, p_nil, per_ms=4):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, keys, n).astype(np.uint32)
    ts = (1541152480000 + np.arange(n) // per_ms).astype(np.int64)
    x = np.round(rng.uniform(-50, 50, n), 3)
    y = rng.integers(-100, 100, n).astype(np.int64)
    vx = (rng.random(n) >= p_nil).astype(np.uint8)
    return [k, ts, x, y], [None, None, vx, None]


def _run(oracle, engine_mod, rule, cols, valid, batches):
    exp = oracle.run(rule.plan, cols, valid)
    eng = engine_mod.Engine(rule.plan)
    cuts = np.linspace(0, len(cols[0]), batches + 1).astype(np.int64)
    for b in range(batches):
        lo, hi = cuts[b], cuts[b + 1]
        eng.push_host([c[lo:hi] for c in cols], [None if v is None else v[lo:hi] for v in valid])
    got = eng.poll()
    eng.close()
    return got, exp


@pytest.mark.parametrize("keys,p_nil", [(37, 0.004), (3000, 0.0003)])
@pytest.mark.parametrize("batches", [1, 7])
def test_nullable_median_parity(oracle, engine_mod, keys, p_nil, batches):
    sql = "SELECT k, median(x), percentile_cont(x, 0.5), count(x), count(*) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1)"
    rule = compile_rule(sql, SCHEMA, num_keys=keys, nullable=("x",), debug_membership=True)
    cols, valid = _stream(60_000, keys, seed=keys + batches, p_nil=p_nil)
    got, exp = _run(oracle, engine_mod, rule, cols, valid, batches)
    bad = [w for w in exp.windows if w.status != 0]
    assert 0 < len(bad) < len(exp.windows), "the stream must hold windows with and without a nil-first group"
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    _assert_errors(got, exp)
    assert all(t == "run Select error: <nil> should be number" for w, t in zip(exp.windows, exp.errors) if w.status)


def test_nullable_median_sliding_keymajor(oracle, engine_mod):
    """Many overlapping windows over a large key space (the key-major path), one row per push on a small stream."""
    sql = "SELECT k, median(x), count(*) FROM s GROUP BY k, SLIDINGWINDOW(ms, 400) OVER (WHEN y > 97)"
    rule = compile_rule(sql, SCHEMA, num_keys=20_000, nullable=("x",), debug_membership=True)
    cols, valid = _stream(40_000, 20_000, seed=5, p_nil=0.0002, per_ms=8)
    got, exp = _run(oracle, engine_mod, rule, cols, valid, 1)
    assert 0 < sum(1 for w in exp.windows if w.status) < len(exp.windows) and len(exp.windows) > 50
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    _assert_errors(got, exp)
    small = compile_rule(sql, SCHEMA, num_keys=50, nullable=("x",), debug_membership=True)
    cols, valid = _stream(600, 50, seed=6, p_nil=0.02, per_ms=2)
    got, exp = _run(oracle, engine_mod, small, cols, valid, 600)
    assert_windows_equal(small.plan, got, exp.windows, check_members=True)
    _assert_errors(got, exp)


def test_nullable_median_refusals(engine_mod):
    for sql, nul in (("SELECT k, median(y) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1)", ("y",)),
                     ("SELECT k, median(x) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1) HAVING count(*) > 1", ("x",))):
        rule = compile_rule(sql, SCHEMA, num_keys=4, nullable=nul)
        with pytest.raises(engine_mod.EngineError) as ei:
            engine_mod.Engine(rule.plan)
        assert ei.value.code == A.EK_ERR_UNSUPPORTED
