"""The key-hash router (ek_route_partition): one rank's ingest slice split into owner segments —
stable (each segment keeps arrival order), keys renamed through the shard dictionary, global arrivals attached — against
a numpy restatement of the same partition (owner = ek_mix64(key) & (2^62 - 1) mod G)."""
import numpy as np
import pytest

from test_engine_gpu import engine_mod  # noqa: F401  (fixture: torch opens the device first)

pytestmark = pytest.mark.gpu


def _mix64(x):
    from ekgpu.synth import mix64
    return mix64(np.asarray(x, dtype=np.uint64))


@pytest.mark.parametrize("n,keys,world", [(0, 10, 2), (1, 10, 2), (5000, 100, 3), (1_000_003, 65536, 8),
                                          (300_000, 1 << 20, 64), (70_000, 7, 1)])
def test_route_partition_matches_numpy(engine_mod, n, keys, world):
    import torch
    from ekgpu.route import key_owner, owned_key_map, route_partition
    rng = np.random.default_rng(n + world)
    key = rng.integers(0, keys, n).astype(np.uint32)
    ts = (1541152480000 + np.arange(n) // 7).astype(np.int64)
    val = rng.standard_normal(n)
    dev = torch.device("cuda", 0)
    cols = [torch.from_numpy(key.view(np.int32)).to(dev), torch.from_numpy(ts).to(dev), torch.from_numpy(val).to(dev)]
    lut, owned = owned_key_map(keys, world, dev)
    base = 12345
    outs, arr, cnt = route_partition(cols, [3, 1, 2], 0, world, lut, base, 0)
    # numpy restatement
    own = (_mix64(key) & np.uint64((1 << 62) - 1)) % np.uint64(world)
    assert np.array_equal(own.astype(np.int64), key_owner(torch.from_numpy(key.astype(np.int64)), world).numpy())
    order = np.argsort(own, kind="stable")
    lut_h = lut.cpu().numpy()
    assert sum(owned) == keys and cnt == np.bincount(own.astype(np.int64), minlength=world).tolist()
    assert np.array_equal(outs[0].cpu().numpy().view(np.uint32), lut_h[key[order]].astype(np.uint32))
    assert np.array_equal(outs[1].cpu().numpy(), ts[order])
    assert np.array_equal(outs[2].cpu().numpy().view(np.int64), val[order].view(np.int64))
    assert np.array_equal(arr.cpu().numpy(), base + order.astype(np.int64))
    # every owner's local ids are dense over its keys
    for r in range(world):
        ids = lut_h[(_mix64(np.arange(keys)) & np.uint64((1 << 62) - 1)) % np.uint64(world) == r]
        assert np.array_equal(np.sort(ids), np.arange(owned[r]))
