"""Full-size oracle parity: every BASELINE.json GPU config at its full per-GPU size, engine vs the CPU oracle
(oracle/ekoracle.c, the per-event restatement of the reference) on the same stream, every window compared
with membership (count + Σ mix64(arrival)) and every row (tests/parity.py rule, vectorised).

  C2  TUMBLINGWINDOW(ss,10) avg/max/count, 1e8 events / 64 Ki keys (the bench stream, seed 44); and 2e7 events
      out of order by up to 50 ms with lateTolerance 50 ms (`bench.py --disorder 50`)
  C3  HOPPINGWINDOW(ss,60,5) sum/min/max/count, one of 8 shards: 2.5e7 events / 131 072 keys
  C4a SLIDINGWINDOW(ss,30) OVER (WHEN trig = 1) stddev/var/count HAVING count(*) > 1, 1e7 events / 1 M keys
  C4b COUNTWINDOW(1000) stddev/var/count HAVING count(*) > 1 (processing time), 1e8 events / 1 M keys
  C5  median + percentile_cont over one 60 s tumbling window, one of 8 shards: 1.25e8 events / 12.5 M keys

The stream is generated in HBM (bench.make_device_stream) and copied to the host for the oracle.
"""
import time

import numpy as np
import pytest

from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA
from oracle import ekoracle
from parity import assert_windows_equal_np
from test_engine_gpu import engine_mod  # noqa: F401

pytestmark = pytest.mark.gpu
T0 = 1541152480000


def _stream(n, keys, epm, seed, t0=T0):
    import torch
    from bench import make_device_stream
    cols = make_device_stream(n, keys, torch.device("cuda:0"), seed=seed, events_per_ms=epm, t0=t0)
    torch.cuda.synchronize()
    return cols


def _host(cols):
    return [c.cpu().numpy() for c in cols]


def _run_both(engine_mod, rule, dcols, pushes=1, oracle_cols=None):
    n = dcols[0].numel()
    t = time.perf_counter()
    exp = ekoracle.run(rule.plan, oracle_cols if oracle_cols is not None else _host(dcols))
    t_or = time.perf_counter() - t
    eng = engine_mod.Engine(rule.plan)
    bounds = np.linspace(0, n, pushes + 1).astype(np.int64)
    t = time.perf_counter()
    for a, b in zip(bounds[:-1], bounds[1:]):
        eng.push_device(int(b - a), [c.data_ptr() + int(a) * c.element_size() for c in dcols])
    eng.sync()
    t_gpu = time.perf_counter() - t
    got = eng.poll()
    eng.close()
    return got, exp, t_or, t_gpu


def _report(name, n, got, t_or, t_gpu):
    rows = sum(len(w.keys) for w in got)
    print(f"\n{name}: {n} events, {len(got)} windows, {rows} rows; oracle {t_or:.1f} s, engine {t_gpu * 1e3:.1f} ms "
          f"(first push, cold buffers)")


@pytest.mark.parametrize("pushes", [1, 7])
def test_c2_full_parity(engine_mod, pushes):
    sql = ("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
           "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)")
    n, keys = 100_000_000, 65536
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=keys, debug_membership=True)
    d = _stream(n, keys, 100, seed=44)
    got, exp, t_or, t_gpu = _run_both(engine_mod, rule, d, pushes=pushes)
    _report(f"C2 x{pushes}", n, got, t_or, t_gpu)
    assert len(exp.windows) == 99
    assert_windows_equal_np(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.parametrize("pushes", [1, 5])
def test_c2_disordered_parity(engine_mod, pushes):
    """`bench.py --disorder 50`: the C2 stream (2e7 events) with every ts moved back by up to 50 ms, lateTolerance
    50 ms — the engine's unsorted path (watermark release, multi-tile partition) against the oracle's per-event
    WatermarkOp (watermark_op.go:144-225)."""
    from bench import disorder_ts
    sql = ("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
           "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)")
    n, keys = 20_000_000, 65536
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=keys, late_tolerance_ms=50, debug_membership=True)
    d = _stream(n, keys, 100, seed=44)
    d[1] = disorder_ts(d[1], 44, 50)
    assert bool((d[1][1:] < d[1][:-1]).any())
    got, exp, t_or, t_gpu = _run_both(engine_mod, rule, d, pushes=pushes)
    _report(f"C2 disordered x{pushes}", n, got, t_or, t_gpu)
    assert len(exp.windows) >= 19
    assert_windows_equal_np(rule.plan, got, exp.windows, check_members=True)


def test_c3_shard_full_parity(engine_mod):
    sql = ("SELECT deviceId, sum(temperature), min(temperature), max(temperature), count(*) FROM demo "
           "GROUP BY deviceId, HOPPINGWINDOW(ss, 60, 5)")
    n, keys = 25_000_000, 131072
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=keys, debug_membership=True)
    d = _stream(n, keys, 42, seed=91)
    got, exp, t_or, t_gpu = _run_both(engine_mod, rule, d, pushes=3)
    _report("C3 shard", n, got, t_or, t_gpu)
    assert len(exp.windows) >= 100
    assert_windows_equal_np(rule.plan, got, exp.windows, check_members=True)


@pytest.mark.timeout(600)   # the per-event oracle re-aggregates 1 002 windows of 3e5 rows: ~2 min on one core
def test_c4a_sliding_full_parity(engine_mod):
    import torch
    sql = ("SELECT deviceId, stddev(temperature), var(temperature), count(*) FROM demo "
           "GROUP BY deviceId, SLIDINGWINDOW(ss, 30) OVER (WHEN trig = 1) HAVING count(*) > 1")
    n, keys = 10_000_000, 1_000_000
    schema = dict(IOT_SCHEMA, trig="bigint")
    rule = compile_rule(sql, schema, num_keys=keys, debug_membership=True)
    d = _stream(n, keys, 10, seed=92)
    i = torch.arange(n, device="cuda:0", dtype=torch.int64)
    d.append((((i * 0x9E3779B1) >> 7) % 10_000 == 0).to(torch.int64))
    got, exp, t_or, t_gpu = _run_both(engine_mod, rule, d, pushes=2)
    _report("C4a", n, got, t_or, t_gpu)
    assert len(exp.windows) > 900
    assert_windows_equal_np(rule.plan, got, exp.windows, check_members=True)


def test_c4b_count_full_parity(engine_mod):
    sql = ("SELECT deviceId, stddev(temperature), var(temperature), count(*) FROM demo "
           "GROUP BY deviceId, COUNTWINDOW(1000) HAVING count(*) > 1")
    n, keys = 100_000_000, 1_000_000
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=keys, is_event_time=False, debug_membership=True)
    d = _stream(n, keys, 100, seed=93)
    got, exp, t_or, t_gpu = _run_both(engine_mod, rule, d, pushes=3)
    _report("C4b", n, got, t_or, t_gpu)
    assert len(exp.windows) == n // 1000
    assert_windows_equal_np(rule.plan, got, exp.windows, check_members=True)


def test_c5_shard_full_parity(engine_mod):
    import torch
    sql = ("SELECT deviceId, median(temperature), percentile_cont(temperature, 0.9) FROM demo "
           "GROUP BY deviceId, TUMBLINGWINDOW(ss, 60)")
    n, keys = 125_000_000, 12_500_000
    t_min = 1541152440000                      # a minute boundary: one 60 s tumbling window
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=keys, debug_membership=True)
    d = _stream(n, keys, 2084, seed=94, t0=t_min)
    # the sentinel event at the window end closes the window (its own key 0 is in the next window)
    sent = [torch.tensor([0], dtype=torch.int32, device="cuda:0"),
            torch.tensor([t_min + 60_000], dtype=torch.int64, device="cuda:0"),
            torch.tensor([50.0], dtype=torch.float64, device="cuda:0"),
            torch.tensor([50.0], dtype=torch.float64, device="cuda:0")]
    d = [torch.cat([a, b]) for a, b in zip(d, sent)]
    got, exp, t_or, t_gpu = _run_both(engine_mod, rule, d, pushes=2)
    _report("C5 shard", n, got, t_or, t_gpu)
    assert len(exp.windows) == 1 and len(exp.windows[0].keys) > 0.99 * keys
    assert_windows_equal_np(rule.plan, got, exp.windows, check_members=True)
