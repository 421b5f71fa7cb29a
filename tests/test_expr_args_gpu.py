"""Aggregate arguments that are arithmetic expressions over columns (row.go:712-718: GroupedTuples.AggregateEval
evaluates the argument per row before the aggregate function folds it). Lowered to derived columns that k_derive
computes once per staged batch; parity with the oracle (which evaluates the same program per row, ekoracle.c
col_val) on the pane path, the range path (median / percentile), nullable inputs and several pushes."""
import numpy as np
import pytest

from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401

pytestmark = pytest.mark.gpu

CASES = [
    "SELECT deviceId, avg(temperature * 1.8 + 32), sum(humidity - temperature), max(temperature / 2), count(*) "
    "FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)",
    "SELECT deviceId, stddev(temperature * humidity), min(-temperature), sum((humidity + 1) * (temperature - 3)) "
    "FROM demo GROUP BY deviceId, HOPPINGWINDOW(ss, 6, 2) HAVING avg(temperature * 2) > 40",
    "SELECT deviceId, median(temperature * 2), percentile_cont(humidity - temperature, 0.9), avg(humidity * 0.5) "
    "FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 5)",
    "SELECT avg(temperature + humidity), count(temperature * 3) FROM demo GROUP BY TUMBLINGWINDOW(ss, 4)",
]


@pytest.mark.parametrize("sql", CASES)
@pytest.mark.parametrize("batches", [1, 3])
def test_expression_argument_parity(oracle, engine_mod, sql, batches):
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=50, debug_membership=True)
    assert rule.plan.n_derived >= 1
    cols = list(iot_stream(200_000, 50, events_per_ms=5))
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert len(exp.windows) >= 3
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_expression_argument_int_and_nulls(oracle, engine_mod):
    """int64 arithmetic stays int64 (integer division truncates, % is Go's remainder); a NULL operand makes the
    argument NULL, which the aggregate skips (count(expr) counts non-nil values only)."""
    schema = {"k": "key", "ts": "bigint", "a": "bigint", "x": "float"}
    sqls = ["SELECT k, sum(a * 3 + 1), max(a / 4), min(a % 7), count(a - a) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1)",
            "SELECT k, avg(a * x), sum(x / 2.5), max(-a), count(*) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1)"]
    n = 30_000
    rng = np.random.default_rng(11)
    k = rng.integers(0, 17, n).astype(np.uint32)
    ts = (1541152480000 + np.arange(n) // 5).astype(np.int64)
    a = rng.integers(-1000, 1000, n).astype(np.int64)
    x = rng.normal(size=n)
    va = (rng.random(n) > 0.3).astype(np.uint8)
    vx = (rng.random(n) > 0.5).astype(np.uint8)
    for sql in sqls:
        rule = compile_rule(sql, schema, num_keys=17, nullable=("a", "x"), debug_membership=True)
        got, exp, _ = run_both(oracle, engine_mod, rule, [k, ts, a, x], batches=2, validity=[None, None, va, vx])
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
