"""Global (un-grouped) aggregates across key-hash shards (C5's global count(*)).

CPU: gloo world_size 2 — each rank runs the partial plan of ekgpu.dist on its key-hash shard (through the
oracle, standing in for the rank's engine), one all_gather exchanges the partial windows, and the merge
must equal the single-stream result of the original rule. The GPU variant runs two engine handles.
"""
import math
import os
import socket

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.dist import GlobalAggError, make_partial_plan, merge_partials, pack_windows, global_windows
from ekgpu.rule import compile_rule
from ekgpu.shard import shard_of
from ekgpu.synth import IOT_SCHEMA, iot_stream

SQL = ("SELECT count(*), avg(temperature), sum(humidity), min(temperature), max(humidity), stddev(temperature), "
       "vars(humidity) FROM demo WHERE humidity > 5 GROUP BY TUMBLINGWINDOW(ss, 2) HAVING count(*) > 10")
N, KEYS = 100_000, 500


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _close(a, b, rel=1e-6):
    if a is None or b is None:
        return a is b
    if isinstance(b, int):
        return isinstance(a, int) and a == b
    return abs(a - b) <= rel * max(abs(a), abs(b), 1e-300)


def check_against_reference(merged, ref_windows, closed_end):
    ref = {w.end: w for w in ref_windows if w.end <= closed_end}
    got = {w.end: w for w in merged if w.end <= closed_end}
    assert set(got) == set(ref) and len(ref) >= 3
    for end, r in ref.items():
        g = got[end]
        assert g.status == r.status
        if len(r.keys) == 0:
            assert g.values is None
            continue
        ev = r.rows()[int(r.keys[0])]
        assert g.values is not None and len(g.values) == len(ev)
        for a, (x, y) in enumerate(zip(g.values, ev)):
            assert _close(x, y), (end, a, x, y)


def _shard_cols(cols, world, rank):
    own = np.nonzero(shard_of(cols[0], world) == rank)[0]
    return [c[own] for c in cols]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from oracle import ekoracle
        rule = compile_rule(SQL, IOT_SCHEMA)
        pp = make_partial_plan(rule)
        cols = list(iot_stream(N, KEYS, seed=81, events_per_ms=10))
        local = _shard_cols(cols, world, rank)
        wins = ekoracle.run(pp.plan, local).windows
        merged = global_windows(pp, wins)
        last = [None] * world
        dist.all_gather_object(last, max(w.end for w in wins))
        q.put((rank, [(w.start, w.end, w.status, w.values) for w in merged], min(last)))
    finally:
        dist.destroy_process_group()


def test_global_aggregate_gloo_world2(oracle):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    from ekgpu.dist import GlobalWindow
    merged = {r: [GlobalWindow(*t) for t in m] for r, m, _ in res}
    assert [(w.end, w.values) for w in merged[0]] == [(w.end, w.values) for w in merged[1]]   # every rank agrees
    closed = res[0][2]
    rule = compile_rule(SQL, IOT_SCHEMA)
    ref = oracle.run(rule.plan, list(iot_stream(N, KEYS, seed=81, events_per_ms=10))).windows
    check_against_reference(merged[0], ref, closed)


def test_partial_plan_rejects_non_decomposable():
    with pytest.raises(GlobalAggError):
        make_partial_plan(compile_rule("SELECT median(temperature) FROM demo GROUP BY TUMBLINGWINDOW(ss, 1)", IOT_SCHEMA))
    with pytest.raises(GlobalAggError):
        make_partial_plan(compile_rule("SELECT deviceId, count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)",
                                       IOT_SCHEMA, num_keys=4))


def test_merge_local_shards_oracle(oracle):
    """Merge without a collective (per-rank packed arrays given directly): 4 shards."""
    rule = compile_rule(SQL, IOT_SCHEMA)
    pp = make_partial_plan(rule)
    cols = list(iot_stream(N, KEYS, seed=82, events_per_ms=10))
    per, last = [], []
    for r in range(4):
        wins = oracle.run(pp.plan, _shard_cols(cols, 4, r)).windows
        per.append(pack_windows(wins, pp.plan.n_aggs))
        last.append(max(w.end for w in wins))
    check_against_reference(merge_partials(pp, per), oracle.run(rule.plan, cols).windows, min(last))


@pytest.mark.gpu
def test_global_aggregate_two_engine_shards(oracle):
    """C5's global count(*) shape on the device: two engine handles as two shards, merged partials."""
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    from ekgpu.engine import Engine
    sql = "SELECT count(*), avg(temperature), max(humidity) FROM demo GROUP BY TUMBLINGWINDOW(ss, 2)"
    rule = compile_rule(sql, IOT_SCHEMA)
    pp = make_partial_plan(rule)
    cols = list(iot_stream(400_000, 100_000, seed=83, events_per_ms=40))
    per, last = [], []
    for r in range(2):
        local = _shard_cols(cols, 2, r)
        eng = Engine(pp.plan)
        for lo in range(0, len(local[0]), 70_000):
            eng.push_host([c[lo:lo + 70_000] for c in local])
        wins = eng.poll()
        eng.close()
        per.append(pack_windows(wins, pp.plan.n_aggs))
        last.append(max(w.end for w in wins))
    check_against_reference(merge_partials(pp, per), oracle.run(rule.plan, cols).windows, min(last))
