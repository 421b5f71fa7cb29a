"""The distributed router (ekgpu.shard.device_watermark: the global WatermarkOp computed by the ranks from their own
rows — one all_reduce MIN over the ts range, or the ranks' distinct timestamps all-gathered when the range is wider
than dense_limit) against the host router ekgpu.shard.GlobalWatermark.track over the whole
stream (watermark_op.go:144-225): the same WatermarkTuples, all_accepted and first-window anchor, on gloo with
world 2 and 4, for a sorted stream, an out-of-order stream inside the tolerance and one with late events."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream(kind, n=20_000):
    rng = np.random.default_rng(7)
    ts = 1_541_152_480_000 + np.arange(n, dtype=np.int64) // 7
    if kind == "disorder":
        ts = ts - rng.integers(0, 30, n)          # back by up to 29 ms, tolerance 30: nothing late
    elif kind == "late":
        ts = ts - rng.integers(0, 200, n) * (rng.random(n) < 0.05)   # some rows far behind: late at tolerance 20
    key = rng.integers(0, 1000, n).astype(np.uint32)
    if kind == "empty":                           # a watermark-only step: no rank holds a row
        return key[:0], ts[:0]
    return key, ts


TOL = {"sorted": 0, "disorder": 30, "late": 20, "empty": 0}


def _worker(rank, world, port, kind, q, dense_limit):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    from ekgpu.shard import device_watermark, shard_of
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        key, ts = _stream(kind)
        own = np.nonzero(shard_of(key, world) == rank)[0]
        tup = device_watermark(torch.from_numpy(ts[own].copy()), torch.from_numpy(own.astype(np.int64)), TOL[kind],
                               dist, want_list=True, dense_limit=dense_limit)
        if rank == 0:
            q.put({k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in tup.items()})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dense_limit", [1 << 24, 0], ids=["dense", "sparse"])
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("kind", ["sorted", "disorder", "late"])
def test_device_router_matches_global_watermark(kind, world, dense_limit):
    import torch.multiprocessing as mp
    from ekgpu.shard import GlobalWatermark
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, q, dense_limit)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, ts = _stream(kind)
    exp = GlobalWatermark(TOL[kind]).track(ts)
    assert got["wm_arrival"] == exp["wm_arrival"].tolist()
    assert got["wm_ts"] == exp["wm_ts"].tolist()
    assert got["all_accepted"] == exp["all_accepted"]
    assert got["all_accepted"] == (kind != "late")
    if got["origin_known"]:
        assert exp["origin_known"]
        assert (got["origin_ts"], got["origin_arrival"]) == (exp["origin_ts"], exp["origin_arrival"])
    assert got["origin_known"] == exp["origin_known"] or not got["all_accepted"]


def test_device_router_empty_step():
    """Every rank's batch empty: no tuple, nothing late, on both ranks (gloo world 2)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, "empty", q, 1 << 24)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got["wm_arrival"] == [] and got["wm_ts"] == []
    assert got["all_accepted"] is True and got["origin_known"] is False
