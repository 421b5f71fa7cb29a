"""The router's exchange (ekgpu.route.route_exchange) on gloo, world 2 and 4: every rank ingests a contiguous slice of
the global stream, splits it by owner (here the numpy restatement of ek_route_partition: a stable partition by
ek_mix64(key) & (2^62 - 1) mod world, tests/test_route_gpu.py pins the kernel to it), and after one all_to_all per column
holds exactly the rows of the keys it owns, in global arrival order (what ek_push_batch_global requires)."""
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


def _owner(key, world):
    from ekgpu.synth import mix64
    return ((mix64(key.astype(np.uint64)) & np.uint64((1 << 62) - 1)) % np.uint64(world)).astype(np.int64)


def _global(n=30_000):
    rng = np.random.default_rng(11)
    return rng.integers(0, 5000, n).astype(np.uint32), (1541152480000 + np.arange(n) // 9).astype(np.int64)


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    from ekgpu.route import route_exchange
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        key, ts = _global()
        cuts = np.linspace(0, len(key), world + 1).astype(np.int64)
        lo, hi = cuts[rank], cuts[rank + 1]
        k, t = key[lo:hi], ts[lo:hi]
        own = _owner(k, world)
        order = np.argsort(own, kind="stable")
        counts = np.bincount(own, minlength=world).tolist()
        cols = [torch.from_numpy(k[order].view(np.int32).copy()), torch.from_numpy(t[order].copy()),
                torch.from_numpy((lo + order).astype(np.int64))]
        got = route_exchange(cols, counts, dist)
        q.put((rank, got[0].numpy().view(np.uint32).tolist(), got[1].numpy().tolist(), got[2].numpy().tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_route_exchange_delivers_owned_rows_in_arrival_order(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    key, ts = _global()
    own = _owner(key, world)
    for rank, k, t, a in res:
        exp = np.nonzero(own == rank)[0]
        assert a == exp.tolist()                       # every owned row, strictly in global arrival order
        assert k == key[exp].tolist() and t == ts[exp].tolist()
