"""Un-grouped window aggregates (no GROUP BY key: one group per window, aggregate_operator.go:34-82 with an empty
dimension list) on the pane path: rows spread over partial slots by row index and merged per window by
k_finalize_merge. Parity with the oracle for tumbling / hopping, var / stddev, WHERE, HAVING, int columns,
several pushes and out-of-order input."""
import numpy as np
import pytest

from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401

pytestmark = pytest.mark.gpu

CASES = [
    "SELECT count(*), avg(temperature), max(humidity) FROM demo GROUP BY TUMBLINGWINDOW(ss, 10)",
    "SELECT count(*), sum(temperature), min(temperature), stddev(humidity), var(temperature) FROM demo "
    "GROUP BY HOPPINGWINDOW(ss, 6, 2)",
    "SELECT count(*), avg(humidity) FROM demo WHERE temperature > 20 GROUP BY TUMBLINGWINDOW(ss, 2) HAVING count(*) > 10",
    # count(*) alone over sorted batches: k_ung_tile reads no column at all
    "SELECT count(*) FROM demo GROUP BY TUMBLINGWINDOW(ss, 10)",
    "SELECT count(*) FROM demo GROUP BY HOPPINGWINDOW(ss, 4, 2) HAVING count(*) > 100",
]


@pytest.mark.parametrize("sql", CASES)
@pytest.mark.parametrize("batches", [1, 4])
def test_ungrouped_parity(oracle, engine_mod, sql, batches):
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=0, debug_membership=True)
    cols = list(iot_stream(300_000, 1000, events_per_ms=5))
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert len(exp.windows) >= 3
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_ungrouped_int_columns_out_of_order(oracle, engine_mod):
    schema = {"deviceId": "key", "ts": "bigint", "v": "bigint", "w": "float"}
    rng = np.random.default_rng(5)
    n = 200_000
    ts = 1541152480000 + np.arange(n) // 20 - rng.integers(0, 50, n) * (rng.random(n) < 0.1)
    cols = [rng.integers(0, 100, n).astype(np.uint32), ts.astype(np.int64), rng.integers(-1000, 1000, n),
            rng.uniform(-5, 5, n)]
    sql = "SELECT count(*), sum(v), avg(v), min(v), max(w), vars(v) FROM demo GROUP BY TUMBLINGWINDOW(ss, 1)"
    rule = compile_rule(sql, schema, num_keys=0, late_tolerance_ms=20, debug_membership=True)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=3)
    assert len(exp.windows) >= 3
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("ung", ["0", "1"])
def test_ungrouped_tile_path_vs_partition_path(oracle, engine_mod, ung, monkeypatch):
    """EKGPU_UNG=1 (default): sorted groups of an un-grouped rule fold tiles straight into the partial slots;
    EKGPU_UNG=0: the k_part + k_agg route. Both equal the oracle, incl. a batch split inside a pane and many panes
    per push."""
    monkeypatch.setenv("EKGPU_UNG", ung)
    sql = ("SELECT count(*), sum(temperature), min(humidity), max(humidity), var(temperature) FROM demo "
           "WHERE humidity > 5 GROUP BY TUMBLINGWINDOW(ms, 500)")
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=0, debug_membership=True)
    cols = list(iot_stream(500_000, 1000, events_per_ms=40))
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=7)
    assert len(exp.windows) >= 20
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_ungrouped_hopping_gap_discard(oracle, engine_mod):
    """Hopping discard mask (k_hop_drop) on a sorted un-grouped batch: the tile path skips the masked rows."""
    n = 60_000
    ts = 1541152480000 + np.arange(n, dtype=np.int64) // 10
    ts[n // 2:] += 9_000            # a gap wider than the window: an empty hopping window discards the inputs
    rng = np.random.default_rng(3)
    cols = [rng.integers(0, 50, n).astype(np.uint32), ts, rng.uniform(0, 100, n), rng.uniform(0, 100, n)]
    sql = "SELECT count(*), avg(temperature) FROM demo GROUP BY HOPPINGWINDOW(ss, 2, 1)"
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=0, debug_membership=True)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=1)
    assert len(exp.windows) >= 5
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
