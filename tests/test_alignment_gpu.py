"""Window-end alignment through the ENGINE: the reference's alignment KAT (window_op_test.go:58-128, TestTime:
getAlignedWindowEndTime with time.Local = Asia/Shanghai) replayed as tumbling / hopping rules whose first event
is the KAT's timestamp. The first triggered window must end at the KAT's value, and every window must match the
oracle (pane mode, and range mode through a median aggregate)."""
import json
import os

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat_alignment.json")))
UNIT_MS = {"ms": 1, "ss": 1000, "mi": 60_000, "hh": 3_600_000, "dd": 86_400_000}
SCHEMA = {"deviceId": "key", "ts": "bigint", "temperature": "float"}


def _stream(ts0, step, n, seed):
    rng = np.random.default_rng(seed)
    ts = ts0 + np.arange(n, dtype=np.int64) * step
    return [rng.integers(0, 4, n).astype(np.uint32), ts, rng.uniform(0, 100, n)]


@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: f"{c['interval']}{c['unit']}")
@pytest.mark.parametrize("shape", ["tumbling", "hopping", "tumbling_median"])
def test_alignment_kat_engine(oracle, engine_mod, case, shape):
    iv, unit = case["interval"], case["unit"]
    L = iv * UNIT_MS[unit]
    if shape == "hopping":
        win, aggs = f"HOPPINGWINDOW({unit}, {2 * iv}, {iv})", "avg(temperature), max(temperature), count(*)"
    elif shape == "tumbling":
        win, aggs = f"TUMBLINGWINDOW({unit}, {iv})", "avg(temperature), max(temperature), count(*)"
    else:
        win, aggs = f"TUMBLINGWINDOW({unit}, {iv})", "median(temperature), count(*)"
    sql = f"SELECT deviceId, {aggs} FROM demo GROUP BY deviceId, {win}"
    rule = compile_rule(sql, SCHEMA, num_keys=4, tz_offset_s=GOLD["tz_offset_s"], debug_membership=True)
    # events from the KAT timestamp over ~5 window lengths past the first aligned end
    span = (case["end"] - GOLD["ts"]) + 5 * L
    step = max(1, span // 400)
    cols = _stream(GOLD["ts"], step, span // step + 1, seed=iv)
    for batches in (1, 5):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert len(exp.windows) >= 3
        assert exp.windows[0].end == case["end"], (exp.windows[0].end, case)
        assert got[0].end == case["end"], (got[0].end, case)
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
