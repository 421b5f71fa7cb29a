"""Multi-rank path on the CPU (gloo, world_size 2): key-hash sharding preserves the rule's result.

Each rank shards the same seeded stream (ekgpu.shard), runs the oracle on its shard with a dense local
dictionary, and the shards' rows are gathered to rank 0, where their union must equal the single-process
result row for row (bit-exact: per-key arrival order is preserved, so even f64 sums agree). Windows are
compared up to the last end every shard has closed (each shard's watermark follows its own events).
"""
import os
import socket

import numpy as np
import pytest

from ekgpu.rule import compile_rule
from ekgpu.shard import ShardDictionary, shard_batch, shard_of
from ekgpu.synth import IOT_SCHEMA, iot_stream

SQL = ("SELECT deviceId, avg(temperature), max(humidity), count(*), stddev(temperature) FROM demo "
       "GROUP BY deviceId, TUMBLINGWINDOW(ss, 2)")
N, KEYS = 60_000, 500


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows_by_window(windows, decode=None):
    out = {}
    for w in windows:
        rows = w.rows()
        if decode is not None:
            g = decode(np.fromiter(rows.keys(), dtype=np.int64, count=len(rows)))
            rows = {int(k): v for k, v in zip(g, rows.values())}
        out[w.end] = rows
    return out


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from oracle import ekoracle
        cols = list(iot_stream(N, KEYS, seed=51, events_per_ms=10))
        d = ShardDictionary()
        local, own = shard_batch(cols, 0, world, rank, d)
        rule = compile_rule(SQL, IOT_SCHEMA, num_keys=len(d.global_of))
        run = ekoracle.run(rule.plan, local)
        mine = {"rows": _rows_by_window(run.windows, d.decode), "max_ts": int(local[1].max()), "n": len(own)}
        got = [None] * world
        dist.all_gather_object(got, mine)
        if rank == 0:
            q.put(got)
    finally:
        dist.destroy_process_group()


def test_shard_of_balanced():
    keys = np.arange(65536, dtype=np.uint32)
    for world in (2, 4, 8):
        counts = np.bincount(shard_of(keys, world), minlength=world)
        assert counts.sum() == 65536 and counts.min() > 0.9 * 65536 / world


def test_key_sharded_union_equals_single_rank(oracle):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    shards = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(s["n"] for s in shards) == N

    cols = list(iot_stream(N, KEYS, seed=51, events_per_ms=10))
    rule = compile_rule(SQL, IOT_SCHEMA, num_keys=KEYS)
    ref = _rows_by_window(oracle.run(rule.plan, cols).windows)
    closed = min(s["max_ts"] for s in shards)
    ends = [e for e in ref if e <= closed]
    assert len(ends) >= 2
    for e in ends:
        union = {}
        for s in shards:
            part = s["rows"].get(e, {})
            assert not (set(part) & set(union)), "a key was emitted by two shards"
            union.update(part)
        assert union == ref[e], f"window end {e}: sharded union differs from the single-rank result"
