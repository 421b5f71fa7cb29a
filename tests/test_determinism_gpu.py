"""Small-window fold order: k_small_win groups a window's rows by key through LDS atomics, which place a
group's rows in no fixed order; the fold must still add a group's f64 values in the window's row order, as the
reference's sequential sum does (common_array_funcs.go: sliceFloatTotal). With few keys every group is long, so any
reordering shows up in the low bits: the result must equal the oracle's sequential sum bit for bit, and two runs
must agree bit for bit."""
import numpy as np
import pytest

from ekgpu.rule import compile_rule
from test_engine_gpu import engine_mod, run_both  # noqa: F401  (fixture + helper)

pytestmark = pytest.mark.gpu
SCHEMA = {"k": "key", "ts": "bigint", "x": "float"}


def _cols(n, keys, seed):
    rng = np.random.default_rng(seed)
    # values spanning many binades: a reordered f64 sum differs in the last bits
    x = rng.standard_normal(n) * np.exp(rng.uniform(-20, 20, n))
    return [rng.integers(0, keys, n).astype(np.uint32), (1541152480000 + np.arange(n)).astype(np.int64), x]


def _bits(windows):
    return [{int(k): (int(v0), int(v1)) for k, v0, v1 in zip(w.keys, w.values[0], w.values[1])} for w in windows]


@pytest.mark.parametrize("keys", [1, 3, 40])
def test_small_window_float_sum_is_sequential(oracle, engine_mod, keys):
    rule = compile_rule("SELECT k, sum(x), avg(x) FROM s GROUP BY k, COUNTWINDOW(2000)", SCHEMA, num_keys=keys,
                        is_event_time=False)
    cols = _cols(40_000, keys, 11 + keys)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols)
    got2, _, _ = run_both(oracle, engine_mod, rule, cols)
    assert len(got) == len(exp.windows) == 20
    assert _bits(got) == _bits(got2)                     # run to run
    assert _bits(got) == _bits(exp.windows)              # and the reference's sequential order, bit for bit
