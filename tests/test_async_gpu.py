"""Asynchronous pushes (ek_set_async): pushes return with their work queued, ek_reset queues behind them, and the
results / stats read back after the queued work match the oracle and the synchronous mode exactly."""
import numpy as np
import pytest

from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu

SQL = "SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)"


@pytest.mark.parametrize("device_batches", [False, True])
def test_async_pushes_match_oracle(oracle, engine_mod, device_batches):
    import torch
    key, ts, temp, hum = iot_stream(300_000, 2000, seed=31, events_per_ms=10)
    rule = compile_rule(SQL, IOT_SCHEMA, num_keys=2000, debug_membership=True)
    exp = oracle.run(rule.plan, [key, ts, temp, hum]).windows
    eng = engine_mod.Engine(rule.plan)
    eng.set_async(True)
    keep = []
    for rep in range(2):   # the second pass after an asynchronous reset
        eng.reset()
        for lo in range(0, len(ts), 60_000):
            part = [key[lo:lo + 60_000], ts[lo:lo + 60_000], temp[lo:lo + 60_000], hum[lo:lo + 60_000]]
            if device_batches:
                d = [torch.from_numpy(np.ascontiguousarray(c)).cuda() for c in part]
                torch.cuda.synchronize()
                keep.append(d)   # a device batch stays borrowed until the queued work completes
                eng.push_device(len(part[0]), [x.data_ptr() for x in d])
            else:
                eng.push_host(part)
        got = eng.poll()
        assert_windows_equal(rule.plan, got, exp, check_members=True)
    st = eng.stats()
    assert st.pushes_timed >= len(range(0, len(ts), 60_000))
    assert st.device_ms_total > 0 and st.phase_launches_total[1] > 0
    eng.set_async(False)
    eng.close()


def test_async_pinned_host_batches_are_not_borrowed(oracle, engine_mod):
    """a host batch in pinned memory makes the push's H2D copies truly asynchronous. An asynchronous push
    waits for its own copies before it returns, so the caller may refill the same pinned buffers at once."""
    import torch
    key, ts, temp, hum = iot_stream(300_000, 2000, seed=33, events_per_ms=10)
    rule = compile_rule(SQL, IOT_SCHEMA, num_keys=2000, debug_membership=True)
    exp = oracle.run(rule.plan, [key, ts, temp, hum]).windows
    eng = engine_mod.Engine(rule.plan)
    eng.set_async(True)
    step = 50_000
    bufs = [torch.empty(step, dtype=dt).pin_memory().numpy() for dt in (torch.int32, torch.int64, torch.float64, torch.float64)]
    bufs[0] = bufs[0].view(np.uint32)
    for lo in range(0, len(ts), step):
        for b, c in zip(bufs, (key, ts, temp, hum)):
            b[:] = c[lo:lo + step]
        eng.push_host(bufs)
        for b in bufs:   # the caller reuses its buffers as soon as the push returns
            b[:] = 0
    got = eng.poll()
    assert_windows_equal(rule.plan, got, exp, check_members=True)
    eng.set_async(False)
    eng.close()


def test_async_error_surfaces_at_stats(engine_mod):
    """fold_time reports a failed queued push: here none failed, so stats after asynchronous pushes return 0."""
    key, ts, temp, hum = iot_stream(70_000, 100, seed=34, events_per_ms=10)
    rule = compile_rule(SQL, IOT_SCHEMA, num_keys=100)
    eng = engine_mod.Engine(rule.plan)
    eng.set_async(True)
    eng.push_host([key, ts, temp, hum])
    st = eng.stats()   # raises on a non-zero code
    assert st.pushes_timed >= 1
    eng.set_async(False)
    eng.close()
