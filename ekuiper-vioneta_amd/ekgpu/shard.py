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


_UNIT_MS = {1: 86_400_000, 2: 3_600_000, 3: 60_000, 4: 1000, 5: 1}   # EK_UNIT_DD .. EK_UNIT_MS


def _aligned_end(ts: int, interval: int, unit: int, tz_s: int) -> int:
    """getAlignedWindowEndTime (window_op.go:194-227): the end of the window holding ts on the unit's grid."""
    off = tz_s * 1000
    local = ts + off
    day0 = (local // 86_400_000) * 86_400_000
    if unit == 1:                                    # dd
        return day0 + interval * 86_400_000 - off
    # hh: hours of the day; mi: minutes of the hour; ss: seconds of the minute; ms: millis of the second
    b0 = {2: day0, 3: (local // 3_600_000) * 3_600_000, 4: (local // 60_000) * 60_000,
          5: (local // 1000) * 1000}[unit]
    step = _UNIT_MS[unit]
    part = (local - b0) // step
    gap = interval * (part // interval + 1) if part > interval else interval
    return b0 + gap * step - off


class GlobalSession:
    """A SESSIONWINDOW(unit, length, timeout) rule's window boundaries over the WHOLE stream, run by the router
    beside GlobalWatermark: the WatermarkOp release (watermark_op.go:157-204: at each WatermarkTuple the buffered
    accepted events with ts <= watermark, in (ts, arrival) order), then the window node's EventRow and
    WatermarkTuple branches for a session (event_window_trigger.go:77-110 getNextSessionWindow, :124-196), on
    timestamps only. Every session it closes is (start, end, watermark of the closing tuple); a key-hash shard
    fires each over its own rows with ts < end (window_op.go:605-655 handleInputs: a session window is not
    overlapping, its content is the remaining inputs before the end), so the shards' union is the stream's
    windows. Host restatement of the same loop as oracle/ekoracle.c next_session / win_on_watermark."""

    def __init__(self, plan):
        u = _UNIT_MS[int(plan.time_unit)]
        self.L = int(plan.length) * u
        self.timeout = int(plan.interval) * u
        self.raw = int(plan.length)
        self.unit = int(plan.time_unit)
        self.tz = int(plan.tz_offset_s)
        self.pending = []            # heap of (ts, arrival): accepted, not released
        self.inputs = []             # released ts not yet consumed by a session (release order = ts order)
        self.has_trigger = False
        self.trigger_time = 0
        self.last_ticked = False

    def _next(self, now):
        inp = self.inputs
        if inp:
            et = inp[0]
            tick = _aligned_end(et, self.raw, self.unit, self.tz)
            p = None
            for t in inp:
                r = None
                if p is not None and t - p > self.timeout:
                    r = p + self.timeout
                if t > tick:
                    if tick - self.L > et and (r is None or tick < r):
                        return tick, True
                    tick += self.L
                if r is not None:
                    return r, False
                p = t
            if p is not None and now - p > self.timeout:
                return p + self.timeout, False
        return None, False

    def step(self, ts: np.ndarray, wm: dict) -> dict:
        """One global micro-batch (ts in arrival order, wm = GlobalWatermark.track's result for it): adds the
        sessions its tuples closed to wm as sess_start / sess_end / sess_wm."""
        import heapq
        ts = np.asarray(ts, dtype=np.int64)
        base = int(wm["arrivals_end"]) - len(ts)
        acc = np.asarray(wm["accepted"], bool)
        ev_a = (base + np.nonzero(acc)[0]).tolist()
        ev_t = ts[acc].tolist()
        out_s, out_e, out_w = [], [], []
        j = 0
        for a_k, w in zip(np.asarray(wm["wm_arrival"]).tolist(), np.asarray(wm["wm_ts"]).tolist()):
            while j < len(ev_a) and ev_a[j] <= a_k:
                heapq.heappush(self.pending, (ev_t[j], ev_a[j]))
                j += 1
            while self.pending and self.pending[0][0] <= w:
                t, _ = heapq.heappop(self.pending)
                if not self.has_trigger:
                    self.has_trigger, self.trigger_time = True, t
                self.inputs.append(t)
            we, ticked = self._next(w)
            while we is not None and we <= w:
                if not self.last_ticked and self.inputs:
                    self.has_trigger, self.trigger_time = True, self.inputs[0]
                ws = self.trigger_time if self.has_trigger else ZERO_MS
                if ws <= 0:
                    ws = we - self.L
                k = 0
                while k < len(self.inputs) and self.inputs[k] < we:
                    k += 1
                del self.inputs[:k]
                out_s.append(ws), out_e.append(we), out_w.append(w)
                self.has_trigger, self.trigger_time = True, we
                self.last_ticked = ticked
                we, ticked = self._next(w)
        for i in range(j, len(ev_a)):   # accepted after the batch's last tuple: released by a later one
            heapq.heappush(self.pending, (ev_t[i], ev_a[i]))
        wm = dict(wm)
        wm["sess_start"] = np.asarray(out_s, np.int64)
        wm["sess_end"] = np.asarray(out_e, np.int64)
        wm["sess_wm"] = np.asarray(out_w, np.int64)
        return wm


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
    ss = np.ascontiguousarray(wm.get("sess_start", np.zeros(0)), dtype=np.int64)
    se = np.ascontiguousarray(wm.get("sess_end", np.zeros(0)), dtype=np.int64)
    sw = np.ascontiguousarray(wm.get("sess_wm", np.zeros(0)), dtype=np.int64)
    g.sess_start = ss.ctypes.data if len(ss) else None
    g.sess_end = se.ctypes.data if len(se) else None
    g.sess_wm = sw.ctypes.data if len(sw) else None
    g.n_sess = len(ss)
    g._keep = (ra, wa, wt, ta, tt, ss, se, sw)
    return g


def merge_triggers(parts):
    """Global trigger list from every shard's (arrival, ts) lists (after the all-gather): arrival order."""
    if not parts:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    a = np.concatenate([np.asarray(p[0], np.int64) for p in parts])
    t = np.concatenate([np.asarray(p[1], np.int64) for p in parts])
    o = np.argsort(a, kind="stable")
    return a[o], t[o]


def device_watermark(ts, arr, tol: int, dist, want_list: bool, dense_limit: int = 1 << 24) -> dict:
    """The rule's WatermarkOp over the WHOLE stream (GlobalWatermark.track, watermark_op.go:144-225) computed by the
    ranks from their own rows (torch tensors: this rank's ts and global arrival indices, on any device) with
    collectives of `dist` (RCCL on GPUs, gloo on CPUs): F[v] = first global arrival with ts == v; the running max
    advances exactly at the arrivals F[v] < min over u > v of F[u] (no earlier arrival reached v) — those are the
    WatermarkTuples (watermark = v - tol); each rank checks its rows against the tuple before them (accepted iff
    ts >= mark - tol) and one all_reduce MIN gives all_accepted.
    F is a dense array over the batch's ts range combined by one all_reduce(MIN) when the range holds at most
    `dense_limit` ms, otherwise the ranks' distinct timestamps (with their first arrival) are all-gathered and merged:
    memory O(distinct ts) instead of O(ts range) (a batch spanning a day at ms resolution is 86.4 M entries).
    Returns the tuple dict make_ctx takes: the full tuple list when `want_list` (range-mode windows) or when some row
    is late, else only the batch's last tuple with the all_accepted / max_wm_step hints (a pane-mode shard needs
    nothing else, include/ekgpu.h ek_global_ctx)."""
    import torch
    i64max = torch.iinfo(torch.int64).max
    dev = ts.device
    mm = torch.stack([-ts.min(), ts.max()]) if ts.numel() else torch.tensor([-i64max, -i64max], device=dev)
    dist.all_reduce(mm, op=dist.ReduceOp.MAX)
    lo, hi = -int(mm[0]), int(mm[1])
    if hi == -i64max:
        # no rank holds a row (a watermark-only step): no tuple, nothing late; every rank takes this branch together
        empty = np.zeros(0, np.int64)
        return {"arrivals_end": None, "all_accepted": True, "max_wm_step": 0, "origin_known": False, "origin_ts": 0,
                "origin_arrival": 0, "wm_arrival": empty, "wm_ts": empty}
    if hi - lo + 1 <= dense_limit:
        F = torch.full((hi - lo + 1,), i64max, dtype=torch.int64, device=dev)
        if ts.numel():
            F.scatter_reduce_(0, ts - lo, arr, reduce="amin", include_self=True)
        dist.all_reduce(F, op=dist.ReduceOp.MIN)
        S = torch.flip(torch.cummin(torch.flip(F, [0]), 0).values, [0])
        nxt = torch.cat([S[1:], torch.tensor([i64max], dtype=torch.int64, device=dev)])
        tv = torch.nonzero(F < nxt).squeeze(1)
        t_arr = F[tv].contiguous()
        t_mark = tv + lo
        first_lo = F[0]
    else:
        # sparse: this rank's distinct ts with their first arrival, all-gathered (padded to the longest list)
        u, inv = torch.unique(ts, return_inverse=True)
        fa = torch.full((u.numel(),), i64max, dtype=torch.int64, device=dev)
        if ts.numel():
            fa.scatter_reduce_(0, inv, arr, reduce="amin", include_self=True)
        world = dist.get_world_size()
        cnt = torch.tensor([u.numel()], dtype=torch.int64, device=dev)
        cnts = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(cnts, cnt)
        m = int(max(int(c) for c in cnts))
        pad_t = torch.full((m,), i64max, dtype=torch.int64, device=dev)
        pad_a = torch.full((m,), i64max, dtype=torch.int64, device=dev)
        pad_t[:u.numel()] = u
        pad_a[:u.numel()] = fa
        gt = [torch.empty_like(pad_t) for _ in range(world)]
        ga = [torch.empty_like(pad_a) for _ in range(world)]
        dist.all_gather(gt, pad_t)
        dist.all_gather(ga, pad_a)
        allt, alla = torch.cat(gt), torch.cat(ga)
        keep = allt != i64max
        allt, alla = allt[keep], alla[keep]
        vt, vinv = torch.unique(allt, return_inverse=True)   # sorted distinct ts of the stream
        F = torch.full((vt.numel(),), i64max, dtype=torch.int64, device=dev)
        F.scatter_reduce_(0, vinv, alla, reduce="amin", include_self=True)
        S = torch.flip(torch.cummin(torch.flip(F, [0]), 0).values, [0])
        nxt = torch.cat([S[1:], torch.tensor([i64max], dtype=torch.int64, device=dev)])
        k = torch.nonzero(F < nxt).squeeze(1)
        t_arr = F[k].contiguous()
        t_mark = vt[k].contiguous()
        first_lo = F[0]
    k = torch.searchsorted(t_arr, arr) - 1
    zero_mark = ZERO_MS + tol          # the stream mark before the first event (watermark_op.go:55-58)
    mb = torch.where(k >= 0, t_mark[k.clamp(min=0)], torch.full_like(k, zero_mark))
    acc = torch.tensor([int(bool((ts >= mb - tol).all())) if ts.numel() else 1], dtype=torch.int64, device=dev)
    dist.all_reduce(acc, op=dist.ReduceOp.MIN)
    wm_ts = t_mark - tol
    steps = wm_ts[1:] - wm_ts[:-1]
    j = torch.searchsorted(wm_ts, torch.tensor([lo], dtype=torch.int64, device=dev))
    jj = int(j.clamp(max=len(wm_ts) - 1))
    head = torch.stack([acc[0], steps.max() if steps.numel() else torch.tensor(0, device=dev), t_arr[jj], first_lo,
                        t_arr[-1], wm_ts[-1]]).cpu().tolist()
    all_acc, max_step, o_arr, first_lo = bool(head[0]), int(head[1]), int(head[2]), int(head[3])
    out = {"arrivals_end": None, "all_accepted": all_acc, "max_wm_step": max_step,
           # the first window's anchor: the earliest event (ts = lo) is released at the first tuple reaching it
           "origin_known": all_acc and first_lo <= o_arr, "origin_ts": lo, "origin_arrival": o_arr}
    if want_list or not all_acc:
        out["wm_arrival"] = t_arr.cpu().numpy()
        out["wm_ts"] = wm_ts.cpu().numpy()
    else:
        out["wm_arrival"] = np.array([int(head[4])], np.int64)
        out["wm_ts"] = np.array([int(head[5])], np.int64)
    return out
