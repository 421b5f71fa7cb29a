"""Key-hash routing (ekgpu.shard): balance of the owner hash and the dense per-shard dictionaries. The
multi-rank protocol itself (global watermark, trigger exchange, union == single stream on every window) is
tested by test_sharding_global.py (gloo, CPU) and test_sharding_gpu.py (engine handles)."""
import numpy as np

from ekgpu.shard import ShardDictionary, shard_batch, shard_of


def test_shard_of_balanced():
    keys = np.arange(65536, dtype=np.uint32)
    for world in (2, 4, 8):
        counts = np.bincount(shard_of(keys, world), minlength=world)
        assert counts.sum() == 65536 and counts.min() > 0.9 * 65536 / world


def test_shard_batch_dense_dictionary():
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 1000, 5000).astype(np.uint32)
    cols = [keys, np.arange(5000, dtype=np.int64)]
    seen = []
    for r in range(4):
        d = ShardDictionary()
        local, own = shard_batch(cols, 0, 4, r, d)
        assert (shard_of(keys[own], 4) == r).all()
        assert local[0].max() + 1 == len(d.global_of)                  # dense ids
        assert np.array_equal(d.decode(local[0]), keys[own].astype(np.int64))
        assert np.array_equal(local[1], own)                            # arrival order kept
        seen.append(own)
    assert np.array_equal(np.sort(np.concatenate(seen)), np.arange(5000))
