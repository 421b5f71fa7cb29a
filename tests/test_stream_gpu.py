"""The XCD-resident streaming path (ek_stream.h, EKGPU_STREAM=1; off by default) against the oracle: pane mode,
sorted batches, tumbling (direct emission) and hopping (pane-state merge) shapes, one and several pushes,
WHERE, and the C2 shape at 64 Ki keys."""
import os

import pytest

from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture
def stream_on():
    os.environ["EKGPU_STREAM"] = "1"
    yield
    os.environ.pop("EKGPU_STREAM", None)


@pytest.mark.parametrize("sql,n,keys,epm,batches", [
    ("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)",
     4_000_000, 65536, 100, 1),
    ("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)",
     800_000, 1000, 20, 5),
    ("SELECT deviceId, sum(temperature), min(temperature), max(humidity), count(*) FROM demo "
     "GROUP BY deviceId, HOPPINGWINDOW(ss, 6, 2)", 300_000, 5000, 20, 3),
    ("SELECT deviceId, avg(temperature), count(*) FROM demo WHERE humidity > 30 GROUP BY deviceId, TUMBLINGWINDOW(ss, 2)",
     200_000, 300, 20, 2),
])
def test_stream_path_parity(oracle, engine_mod, stream_on, sql, n, keys, epm, batches):
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=keys, debug_membership=True)
    cols = list(iot_stream(n, keys, events_per_ms=epm))
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert len(exp.windows) >= 3
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
