"""The fused sorted pass (k_part MODE 3): a pane-mode batch of at least 65 536 rows is partitioned
straight from its first and last timestamps, and the partition pass itself checks that the batch is ts-sorted (then
no row is late and the running max is each row's own ts, watermark_op.go:144-155), writes the pane bounds and, for a
hopping window with lateTolerance 0, finds the widest arrival gap. A batch that fails the check is discarded before
any engine state changes and redone on the general path (k_stats, k_accept, k_pane_bounds, k_hop_drop).

Every case is checked against the oracle, windows with their membership fingerprints, and asserts which path ran
(ek_stats.fused_batches / fused_discarded). The pass is enabled by EKGPU_FUSED=1 (off by default: DESIGN.md §5.1)."""
import numpy as np
import pytest

from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401

pytestmark = pytest.mark.gpu
C2_SQL = ("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
          "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)")
C3_SQL = ("SELECT deviceId, sum(temperature), min(temperature), max(temperature), count(*) FROM demo "
          "GROUP BY deviceId, HOPPINGWINDOW(ss, 6, 2)")


@pytest.fixture(autouse=True)
def _fused_on(monkeypatch):
    """The pass is off by default (no gain measured); EKGPU_FUSED=1 is read at ek_create."""
    monkeypatch.setenv("EKGPU_FUSED", "1")


def _cols(n, keys, epm, seed=44):
    return list(iot_stream(n, keys, seed=seed, events_per_ms=epm))


def _check(oracle, engine_mod, rule, cols, batches, validity=None):
    got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches, validity=validity)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    return st


@pytest.mark.parametrize("batches", [1, 3, 7])
def test_fused_tumbling_sorted(oracle, engine_mod, batches):
    """C2's rule over a sorted stream: every batch takes the fused pass (panes spanning batches merge in the ring)."""
    rule = compile_rule(C2_SQL, IOT_SCHEMA, num_keys=4096, debug_membership=True)
    cols = _cols(700_000, 4096, epm=20)
    st = _check(oracle, engine_mod, rule, cols, batches)
    assert st.fused_batches == batches and st.fused_discarded == 0


@pytest.mark.parametrize("batches", [1, 4])
def test_fused_hopping_sorted(oracle, engine_mod, batches):
    rule = compile_rule(C3_SQL, IOT_SCHEMA, num_keys=8192, debug_membership=True)
    cols = _cols(600_000, 8192, epm=25)
    st = _check(oracle, engine_mod, rule, cols, batches)
    assert st.fused_batches == batches and st.fused_discarded == 0


def test_fused_hopping_gap_discards(oracle, engine_mod):
    """A hopping window with lateTolerance 0 and an arrival gap wider than the window: the pass measures the gap and is
    discarded, so the general path runs the empty-window discard (k_hop_drop, window_op.go:605-655)."""
    rule = compile_rule(C3_SQL, IOT_SCHEMA, num_keys=8192, debug_membership=True)
    cols = _cols(300_000, 8192, epm=25)
    cols[1] = cols[1].copy()
    cols[1][150_000:] += 20_000   # a 20 s gap > the 6 s window
    st = _check(oracle, engine_mod, rule, cols, 1)
    assert st.fused_batches == 0 and st.fused_discarded == 1
    assert st.records_discarded > 0


def test_fused_unsorted_discards(oracle, engine_mod):
    """First ts <= last ts but one inversion inside: only the pass's own order check can see it."""
    rule = compile_rule(C2_SQL, IOT_SCHEMA, num_keys=4096, late_tolerance_ms=1000, debug_membership=True)
    cols = _cols(400_000, 4096, epm=20)
    cols[1] = cols[1].copy()
    cols[1][200_001], cols[1][200_002] = cols[1][200_002] + 3, cols[1][200_001]
    assert cols[1][0] <= cols[1][-1] and not np.all(np.diff(cols[1]) >= 0)
    st = _check(oracle, engine_mod, rule, cols, 1)
    assert st.fused_batches == 0 and st.fused_discarded == 1


def test_fused_sparse_panes_discards(oracle, engine_mod):
    """A dense burst then a sparse tail: the mean rows per pane under-estimates how many panes a sparse chunk spans,
    the pass flags the overflow and the batch runs the general path."""
    rule = compile_rule(C2_SQL, IOT_SCHEMA, num_keys=1024, debug_membership=True)
    dense, sparse = 100_000, 50_000
    cols = _cols(dense + sparse, 1024, epm=1)
    cols[1] = np.concatenate([np.full(dense, cols[1][0]), cols[1][0] + 1 + 100 * np.arange(sparse)]).astype(np.int64)
    st = _check(oracle, engine_mod, rule, cols, 1)
    assert st.fused_batches == 0 and st.fused_discarded == 1


def test_fused_late_prefix_general_path(oracle, engine_mod):
    """A batch starting below the watermark (a late prefix) goes to the general path before any pass runs."""
    rule = compile_rule(C2_SQL, IOT_SCHEMA, num_keys=4096, debug_membership=True)
    a = _cols(200_000, 4096, epm=20)
    b = _cols(200_000, 4096, epm=20, seed=45)
    b[1] = b[1] + 5_000   # starts 5 s after the stream start: 5 s below the first batch's max (10 s)
    cols = [np.concatenate([x, y]) for x, y in zip(a, b)]
    st = _check(oracle, engine_mod, rule, cols, 2)
    assert st.fused_batches == 1 and st.fused_discarded == 0
    assert st.records_late > 0


def test_fused_nullable(oracle, engine_mod):
    """A nullable value column takes the fused pass (validity staged beside the values)."""
    sql = ("SELECT deviceId, avg(temperature), max(humidity), count(humidity) FROM demo "
           "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)")
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=2048, debug_membership=True, nullable=("humidity",))
    cols = _cols(500_000, 2048, epm=20)
    rng = np.random.default_rng(7)
    valid = [None, None, None, (rng.random(500_000) > 0.1).astype(np.uint8)]
    st = _check(oracle, engine_mod, rule, cols, 2, validity=valid)
    assert st.fused_batches == 2 and st.fused_discarded == 0


def test_fused_where_takes_general_path(oracle, engine_mod):
    """A rule with WHERE keeps the general path, with the same results."""
    sql = ("SELECT deviceId, avg(temperature), max(humidity), count(humidity) FROM demo WHERE temperature > 20 "
           "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)")
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=2048, debug_membership=True, nullable=("humidity",))
    cols = _cols(500_000, 2048, epm=20)
    rng = np.random.default_rng(7)
    valid = [None, None, None, (rng.random(500_000) > 0.1).astype(np.uint8)]
    st = _check(oracle, engine_mod, rule, cols, 2, validity=valid)
    assert st.fused_batches == 0


def test_fused_off_matches(oracle, engine_mod, monkeypatch):
    """EKGPU_FUSED=0 (read at ek_create): the general path on the same stream gives the same windows."""
    monkeypatch.setenv("EKGPU_FUSED", "0")
    rule = compile_rule(C2_SQL, IOT_SCHEMA, num_keys=4096, debug_membership=True)
    cols = _cols(300_000, 4096, epm=20)
    st = _check(oracle, engine_mod, rule, cols, 1)
    assert st.fused_batches == 0
