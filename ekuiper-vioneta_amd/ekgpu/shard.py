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


ZERO_MS = -62135596800000          # Go time.Time{} (0001-01-01T00:00:00Z) in Unix ms


class GlobalWatermark:
    """The rule's WatermarkOp tracking over the WHOLE stream (watermark_op.go:144-225), run by the host that
    assigns the global arrival order (the router of a key-hash-sharded rule). Per global micro-batch it yields
    the WatermarkTuples every shard receives (ek_global_ctx: wm_arrival / wm_ts), and once the first event has
    been released, the first window's anchor (origin_ts: getEarliestEventTs at that tuple,
    event_window_trigger.go:57-75,211-219).

    Restated vectorised: the stream mark starts at time.Time{} + lateTol (watermark_op.go:55-58) and moves to
    ts when ts is after it (track, :144-155); the watermark is mark - lateTol (computeWatermarkTs, :217-225) and
    a tuple is emitted whenever it advances (addAndTrigger, :157-214). An event is accepted iff ts is not before
    the last emitted watermark; the first release happens at the first tuple whose watermark reaches the
    smallest accepted ts so far."""

    def __init__(self, late_tolerance_ms: int = 0):
        self.T = int(late_tolerance_ms)
        self.arrivals = 0
        self.mark = ZERO_MS + self.T
        self.origin_known = False
        self.origin_ts = 0
        self.origin_arrival = 0
        self._acc_min = None          # smallest accepted ts before the first release

    def track(self, ts: np.ndarray) -> dict:
        ts = np.asarray(ts, dtype=np.int64)
        n = len(ts)
        base = self.arrivals
        m = np.maximum.accumulate(np.concatenate([[self.mark], ts]))
        prev = m[:-1]                     # mark before each event
        adv = np.nonzero(m[1:] > prev)[0]
        wm_arrival = (base + adv).astype(np.int64)
        wm_ts = (m[1:][adv] - self.T).astype(np.int64)
        accepted = ts >= prev - self.T    # last emitted watermark before the event = mark - lateTol
        if not self.origin_known and len(adv):
            acc_ts = np.where(accepted, ts, np.iinfo(np.int64).max)
            cm = np.minimum.accumulate(acc_ts)
            if self._acc_min is not None:
                cm = np.minimum(cm, self._acc_min)
            hit = np.nonzero(cm[adv] <= wm_ts)[0]
            if len(hit):
                k = hit[0]
                self.origin_known = True
                self.origin_ts = int(cm[adv[k]])
                self.origin_arrival = int(wm_arrival[k])
            else:
                self._acc_min = int(cm[-1]) if n else self._acc_min
        elif not self.origin_known and n:
            acc_ts = ts[accepted]
            if len(acc_ts):
                mn = int(acc_ts.min())
                self._acc_min = mn if self._acc_min is None else min(self._acc_min, mn)
        prev_w = self.mark - self.T
        steps = np.diff(np.concatenate([[prev_w], wm_ts])) if len(wm_ts) else np.zeros(0, np.int64)
        self.mark = int(m[-1])
        self.arrivals += n
        return {"wm_arrival": wm_arrival, "wm_ts": wm_ts, "arrivals_end": self.arrivals, "accepted": accepted,
                "all_accepted": bool(accepted.all()), "max_wm_step": int(steps.max()) if len(steps) else 0,
                "origin_known": self.origin_known, "origin_ts": self.origin_ts, "origin_arrival": self.origin_arrival}


def make_ctx(wm: dict, row_arrival: np.ndarray, trig_arrival=None, trig_ts=None):
    """An ek_global_ctx over host arrays (the arrays are attached to the struct to keep them alive)."""
    from . import abi as A
    ra = np.ascontiguousarray(row_arrival, dtype=np.int64)
    wa = np.ascontiguousarray(wm["wm_arrival"], dtype=np.int64)
    wt = np.ascontiguousarray(wm["wm_ts"], dtype=np.int64)
    ta = np.ascontiguousarray(trig_arrival if trig_arrival is not None else np.zeros(0), dtype=np.int64)
    tt = np.ascontiguousarray(trig_ts if trig_ts is not None else np.zeros(0), dtype=np.int64)
    g = A.ek_global_ctx()
    g.row_arrival = ra.ctypes.data if len(ra) else None
    g.arrivals_end = int(wm["arrivals_end"])
    g.wm_arrival = wa.ctypes.data if len(wa) else None
    g.wm_ts = wt.ctypes.data if len(wt) else None
    g.n_wm = len(wa)
    g.origin_known = 1 if wm["origin_known"] else 0
    g.all_accepted = 1 if wm.get("all_accepted") else 0
    g.max_wm_step = int(wm.get("max_wm_step", 0))
    g.origin_ts = int(wm["origin_ts"])
    g.origin_arrival = int(wm["origin_arrival"])
    g.trig_arrival = ta.ctypes.data if len(ta) else None
    g.trig_ts = tt.ctypes.data if len(tt) else None
    g.n_trig = len(ta)
    g.memory = A.EK_MEM_HOST
    g._keep = (ra, wa, wt, ta, tt)
    return g


def merge_triggers(parts):
    """Global trigger list from every shard's (arrival, ts) lists (after the all-gather): arrival order."""
    if not parts:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    a = np.concatenate([np.asarray(p[0], np.int64) for p in parts])
    t = np.concatenate([np.asarray(p[1], np.int64) for p in parts])
    o = np.argsort(a, kind="stable")
    return a[o], t[o]
