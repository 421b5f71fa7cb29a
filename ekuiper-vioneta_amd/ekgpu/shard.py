"""Key-hash sharding of a columnar micro-batch across GPUs.

GROUP BY groups are independent and window boundaries depend only on event time, so a rule's
window/aggregate node shards by key: rank r owns every key with ``mix64(key) % world == r`` and
dictionary-encodes its keys densely (0..K_r-1) so its engine runs the same plan with
``num_keys = K_r``. Results of the shards are disjoint by key; their union is the rule's result.

This is host-side ingest logic (the reference's equivalent is the per-row group-key build in
``aggregate_operator.go:58-66``); the per-event compute stays on the GPUs.
"""
from typing import List, Tuple

import numpy as np

from .synth import mix64


def shard_of(keys: np.ndarray, world: int) -> np.ndarray:
    """Owning rank of every key (splitmix64 hash, so dense ids spread evenly)."""
    return (mix64(keys.astype(np.uint64)) % np.uint64(world)).astype(np.int64)


class ShardDictionary:
    """Dense local ids of the keys one rank owns; stable across batches (append-only)."""

    def __init__(self):
        self.local_of = {}
        self.global_of: List[int] = []

    def encode(self, keys: np.ndarray) -> np.ndarray:
        uniq, inv = np.unique(keys, return_inverse=True)
        ids = np.empty(len(uniq), dtype=np.uint32)
        for i, k in enumerate(uniq.tolist()):
            lid = self.local_of.get(k)
            if lid is None:
                lid = len(self.global_of)
                self.local_of[k] = lid
                self.global_of.append(k)
            ids[i] = lid
        return ids[inv]

    def decode(self, local_ids: np.ndarray) -> np.ndarray:
        g = np.asarray(self.global_of, dtype=np.int64)
        return g[local_ids.astype(np.int64)]


def shard_batch(cols: List[np.ndarray], key_col: int, world: int, rank: int,
                dictionary: ShardDictionary) -> Tuple[List[np.ndarray], np.ndarray]:
    """Rows of `cols` owned by `rank` (arrival order kept), key column re-encoded to local ids.
    Returns (local columns, global arrival index of every kept row)."""
    own = np.nonzero(shard_of(cols[key_col], world) == rank)[0]
    out = [c[own] for c in cols]
    out[key_col] = dictionary.encode(out[key_col])
    return out, own
