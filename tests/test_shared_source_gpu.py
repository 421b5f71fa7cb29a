"""Shared-source timestamp statistics (ABI v10, ek_batch_ts_stats + ek_batch.ts_stats): eKuiper fans one source out to
every rule subscribed to it (internal/topo/subtopo.go) and each rule's WatermarkOp scans the same timestamps
(watermark_op.go:118-155); here the scan runs once and every rule's push takes its result. A rule pushed with the
shared statistics must produce exactly what it produces without them (and what the oracle produces), for every
statistics consumer: the event-time push (sorted, out-of-order with late drops, hopping's empty-window gap check seeded
with the carried stream maximum), processing time and range mode."""
import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu

CASES = [
    ("tumbling", "SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
                 "GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)", {}),
    ("hopping_gap", "SELECT deviceId, sum(temperature), count(*) FROM demo GROUP BY deviceId, HOPPINGWINDOW(ss, 2, 1)", {}),
    ("late_drop", "SELECT deviceId, count(*), sum(temperature) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)",
     dict(late_tolerance_ms=300)),
    ("sliding", "SELECT deviceId, count(*), max(temperature) FROM demo GROUP BY deviceId, SLIDINGWINDOW(ms, 200)", {}),
    ("proc_tumbling", "SELECT deviceId, count(*), avg(temperature) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)",
     dict(is_event_time=False)),
]


def _stream(name, n=60_000, keys=97):
    key, ts, temp, hum = iot_stream(n, keys, seed=11, events_per_ms=20)
    ts = ts.copy()
    if name == "hopping_gap":
        ts[n // 3:] += 7_000            # a gap wider than the window: the empty windows' inputs are discarded
        ts[2 * n // 3:] += 5_000
    if name == "late_drop":
        rng = np.random.default_rng(3)
        ts = ts + rng.integers(-600, 600, n)
    return [key, ts.astype(np.int64), temp, hum]


def _push_all(engine_mod, rule, dcols, cuts, share_from=None, clock=None):
    """Push the batches [cuts[b], cuts[b+1]); with share_from (another rule's handle), each batch carries the
    statistics that handle computed for it. clock = (start, end, ts): processing time, the clock advanced to start,
    to each batch's first arrival and to end (tests/test_processing_gpu.py::run_engine)."""
    eng = engine_mod.Engine(rule.plan)
    if clock:
        eng.advance_time(clock[0])
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        ptrs = [c[lo:hi].data_ptr() for c in dcols]
        st = share_from.batch_ts_stats(int(hi - lo), ptrs) if share_from is not None else None
        if clock:
            eng.advance_time(int(clock[2][lo]))
        eng.push_device(int(hi - lo), ptrs, ts_stats=st)
    if clock:
        eng.advance_time(clock[1])
    got = eng.poll()
    s = eng.stats()
    eng.close()
    return got, s


@pytest.mark.parametrize("name,sql,kw", CASES, ids=[c[0] for c in CASES])
def test_shared_ts_stats_parity(oracle, engine_mod, name, sql, kw):
    import torch
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=97, debug_membership=True, **kw)
    # the statistics come from ANOTHER rule over the same source (its own ts column is the same column 1)
    other = compile_rule("SELECT count(*) FROM demo GROUP BY TUMBLINGWINDOW(ss, 60)", IOT_SCHEMA, num_keys=1,
                         is_event_time=kw.get("is_event_time", True))
    cols = _stream(name)
    dcols = [torch.from_numpy(c).cuda() for c in cols]
    clock = None
    if kw.get("is_event_time", True):
        exp = oracle.run(rule.plan, cols)
    else:
        clock = (int(cols[1][0]) - 1234, int(cols[1][-1]) + 5_000, cols[1])
        exp = oracle.run_proc(rule.plan, cols, clock[0], clock[1])
    cuts = np.linspace(0, len(cols[0]), 5).astype(np.int64)
    sharer = engine_mod.Engine(other.plan)
    got_plain, st_plain = _push_all(engine_mod, rule, dcols, cuts, clock=clock)
    got_shared, st_shared = _push_all(engine_mod, rule, dcols, cuts, share_from=sharer, clock=clock)
    sharer.close()
    assert_windows_equal(rule.plan, got_plain, exp.windows, check_members=True)
    assert_windows_equal(rule.plan, got_shared, exp.windows, check_members=True)
    assert (st_shared.records_late, st_shared.records_discarded) == (st_plain.records_late, st_plain.records_discarded)
    if name == "late_drop":
        assert st_shared.records_late > 0
    if name == "hopping_gap":
        assert st_shared.records_discarded > 0


def test_ts_stats_values_and_mismatch(oracle, engine_mod):
    """The device statistics equal numpy's; a host batch gets the same; statistics of another batch length are
    ignored by the push (it runs its own pass)."""
    import ctypes as C
    import torch
    from ekgpu.engine import lib
    rule = compile_rule(CASES[2][1], IOT_SCHEMA, num_keys=97, late_tolerance_ms=300, debug_membership=True)
    cols = _stream("late_drop", n=10_001)
    ts = cols[1]
    dcols = [torch.from_numpy(c).cuda() for c in cols]
    ptrs = [c.data_ptr() for c in dcols]
    eng = engine_mod.Engine(rule.plan)
    st = eng.batch_ts_stats(len(ts), ptrs)
    d = np.diff(ts)
    assert (st.n_rows, st.ts_column) == (len(ts), 1)
    assert (st.ts_min, st.ts_max, st.ts_first) == (ts.min(), ts.max(), ts[0])
    assert (st.unsorted, st.max_step) == (int((d < 0).any()), d.max())
    b, _keep = eng._host_batch(cols)
    h = A.ek_ts_stats()
    assert lib().ek_batch_ts_stats(eng.h, C.byref(b), C.byref(h)) == 0
    fields = [f for f, _ in A.ek_ts_stats._fields_ if f != "ts_data"]
    assert [getattr(h, f) for f in fields] == [getattr(st, f) for f in fields]
    assert (st.ts_data, h.ts_data) == (ptrs[1], b.columns[1])   # bound to the column they were computed over
    one = eng.batch_ts_stats(1, ptrs)
    assert (one.ts_min, one.ts_max, one.unsorted, one.max_step) == (ts[0], ts[0], 0, np.iinfo(np.int64).min)
    # a hint describing a different row count is ignored: the push still finds the late rows itself
    eng.push_device(len(ts), ptrs, ts_stats=one)
    got = eng.poll()
    late = eng.stats().records_late
    eng.close()
    exp = oracle.run(rule.plan, cols)
    assert late == exp.records_late > 0
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_ts_stats_of_another_column_ignored(oracle, engine_mod):
    """Statistics left over from the previous micro-batch of the same size (same n_rows, same ts column id) describe
    another column pointer (ABI v11 ts_data) and are ignored: the push runs its own pass and finds this batch's late
    rows (a sorted, late-free previous batch would otherwise take the sorted fast path with the wrong bounds)."""
    import torch
    rule = compile_rule(CASES[2][1], IOT_SCHEMA, num_keys=97, late_tolerance_ms=300, debug_membership=True)
    cols = _stream("late_drop", n=10_001)
    prev = [c.copy() for c in cols]
    prev[1] = np.sort(prev[1])                           # a sorted batch of the same size
    dprev = [torch.from_numpy(c).cuda() for c in prev]
    dcols = [torch.from_numpy(c).cuda() for c in cols]
    eng = engine_mod.Engine(rule.plan)
    stale = eng.batch_ts_stats(len(cols[1]), [c.data_ptr() for c in dprev])
    assert stale.unsorted == 0
    eng.push_device(len(cols[1]), [c.data_ptr() for c in dcols], ts_stats=stale)
    got = eng.poll()
    late = eng.stats().records_late
    eng.close()
    exp = oracle.run(rule.plan, cols)
    assert late == exp.records_late > 0
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
