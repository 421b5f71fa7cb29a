"""COUNTWINDOW rules shard by window blocks (bench.py block_stream): window k of COUNTWINDOW(n) is the
global arrivals [k n, (k + 1) n) (window_op.go:390-418), so a rank that takes the contiguous arrivals [r N, (r + 1) N)
with N a multiple of n produces exactly the global windows r N / n ... (r + 1) N / n - 1. Checked on the oracle: the
blocks' windows, concatenated in rank order, are the single stream's windows."""
import numpy as np

from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal


def test_window_blocks_equal_single_stream(oracle):
    sql = ("SELECT deviceId, stddev(temperature), var(temperature) FROM demo "
           "GROUP BY deviceId, COUNTWINDOW(1000) HAVING count(*) > 1")
    world, n_per = 4, 25_000
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=2000, is_event_time=False, debug_membership=False)
    cols = list(iot_stream(world * n_per, 2000, seed=71, events_per_ms=10))
    single = oracle.run(rule.plan, cols).windows
    union = []
    for r in range(world):
        union += oracle.run(rule.plan, [c[r * n_per:(r + 1) * n_per] for c in cols]).windows
    assert len(single) == len(union) == world * n_per // 1000
    assert_windows_equal(rule.plan, union, single, check_members=False)
