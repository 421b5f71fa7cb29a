"""Shared pieces of the sharding tests: synthetic global streams (out of order, late events, gaps, ties),
routing by key hash with the global WatermarkOp (ekgpu.shard.GlobalWatermark), and the comparison of the
shards' union with the single-stream oracle on EVERY window (start/end/status, membership, rows)."""
import numpy as np

from ekgpu import abi as A
from ekgpu.shard import GlobalSession, GlobalWatermark, ShardDictionary, make_ctx, merge_triggers, shard_of

T0 = 1541152480000
SCHEMA = {"deviceId": "key", "ts": "bigint", "temperature": "float", "humidity": "float", "trig": "bigint"}

CASES = {
    # name: (sql, late_tolerance_ms, is_event_time, stream kind)
    "tumbling_ooo_late": ("SELECT deviceId, avg(temperature), max(humidity), count(*), stddev(temperature) FROM demo "
                          "GROUP BY deviceId, TUMBLINGWINDOW(ss, 2)", 0, True, "ooo"),
    "tumbling_ooo_tol": ("SELECT deviceId, avg(temperature), min(humidity), count(*) FROM demo "
                         "GROUP BY deviceId, TUMBLINGWINDOW(ss, 2)", 700, True, "ooo"),
    "hopping_gaps": ("SELECT deviceId, sum(temperature), max(temperature), count(*) FROM demo "
                     "GROUP BY deviceId, HOPPINGWINDOW(ss, 3, 1)", 0, True, "gaps"),
    "sliding_over_when": ("SELECT deviceId, stddev(temperature), var(temperature), count(*) FROM demo "
                          "GROUP BY deviceId, SLIDINGWINDOW(ss, 2) OVER (WHEN trig = 1) HAVING count(*) > 1", 0, True, "ooo"),
    "sliding_over_when_tol": ("SELECT deviceId, avg(temperature), count(*) FROM demo "
                              "GROUP BY deviceId, SLIDINGWINDOW(ss, 2) OVER (WHEN trig = 1)", 300, True, "ooo"),
    # delayed sliding: each global trigger queues t + D, the window [t - L, t + D) fires at a later global tuple
    "sliding_delay": ("SELECT deviceId, count(*), sum(temperature), max(humidity) FROM demo "
                      "GROUP BY deviceId, SLIDINGWINDOW(ms, 700, 300) OVER (WHEN trig = 1)", 0, True, "ooo"),
    "sliding_delay_tol": ("SELECT deviceId, avg(temperature), count(*) FROM demo "
                          "GROUP BY deviceId, SLIDINGWINDOW(ss, 1, 1) OVER (WHEN trig = 1)", 250, True, "ooo"),
    "count_window": ("SELECT deviceId, stddev(temperature), var(temperature), count(*) FROM demo "
                     "GROUP BY deviceId, COUNTWINDOW(1000) HAVING count(*) > 1", 0, False, "sorted"),
    "tumbling_median": ("SELECT deviceId, median(temperature), count(*) FROM demo "
                        "GROUP BY deviceId, TUMBLINGWINDOW(ss, 2)", 0, True, "ooo"),
    # sessions closed by the timeout (bursts separated by 8 s gaps) and by the length ticks (a continuous stream)
    "session_gaps": ("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
                     "GROUP BY deviceId, SESSIONWINDOW(ss, 5, 2)", 0, True, "gaps"),
    "session_ooo_tol": ("SELECT deviceId, sum(temperature), min(humidity), count(*) FROM demo "
                        "GROUP BY deviceId, SESSIONWINDOW(ss, 1, 1)", 300, True, "ooo"),
}


def global_stream(kind, n=40_000, keys=300, seed=7):
    """key, ts, temperature, humidity, trig. 'ooo': 2 events/ms with jitter (ties, out of order, late
    events); 'gaps': bursts separated by gaps wider than the hopping window; 'sorted': in order."""
    rng = np.random.default_rng(seed)
    i = np.arange(n, dtype=np.int64)
    if kind == "gaps":
        burst = i // 5000
        ts = T0 + burst * 9000 + (i % 5000) // 5
    else:
        ts = T0 + i // 2
    if kind == "ooo":
        # 5 % of events up to 600 ms behind (late when lateTolerance is smaller), 0.2 % up to 5 ms ahead
        u = rng.random(n)
        ts = ts - rng.integers(0, 600, n) * (u < 0.05) + rng.integers(1, 6, n) * (u > 0.998)
    key = rng.integers(0, keys, n).astype(np.uint32)
    temp = rng.integers(0, 1000, n).astype(np.float64) / 8.0     # exact binary fractions: sums are exact
    hum = rng.uniform(0, 100, n)
    trig = (rng.random(n) < 0.01).astype(np.int64)
    return [key, ts.astype(np.int64), temp, hum, trig]


def route(cols, world, batches, late_tol, is_event_time, sql=None):
    """Per rank, per batch: (local cols, row_arrival, wm dict). Dictionaries are per rank (dense local ids).
    A SESSIONWINDOW rule (sql) also gets the router's global session list (GlobalSession) in every wm dict."""
    n = len(cols[0])
    cuts = np.linspace(0, n, batches + 1).astype(np.int64)
    gw = GlobalWatermark(late_tol)
    gs = None
    if sql is not None and "SESSIONWINDOW" in sql.upper():
        from ekgpu.rule import compile_rule
        gs = GlobalSession(compile_rule(sql, SCHEMA, num_keys=1, late_tolerance_ms=late_tol,
                                        is_event_time=is_event_time).plan)
    owner = shard_of(cols[0], world)
    dicts = [ShardDictionary() for _ in range(world)]
    out = [[] for _ in range(world)]
    for b in range(batches):
        lo, hi = cuts[b], cuts[b + 1]
        if is_event_time:
            wm = gw.track(cols[1][lo:hi])
            if gs is not None:
                wm = gs.step(cols[1][lo:hi], wm)
        else:
            gw.arrivals += hi - lo
            wm = {"wm_arrival": np.zeros(0, np.int64), "wm_ts": np.zeros(0, np.int64), "arrivals_end": gw.arrivals,
                  "origin_known": False, "origin_ts": 0, "origin_arrival": 0}
        for r in range(world):
            own = lo + np.nonzero(owner[lo:hi] == r)[0]
            local = [c[own] for c in cols]
            local[0] = dicts[r].encode(local[0]) if len(own) else local[0].astype(np.uint32)
            out[r].append((local, own.astype(np.int64), wm))
    return out, dicts


def whole_ctx(batches_of_rank, trig=None):
    """One ek_global_ctx over a rank's whole stream (the oracle's shard model runs the stream at once)."""
    cols = [np.concatenate([b[0][k] for b in batches_of_rank]) for k in range(len(batches_of_rank[0][0]))]
    arr = np.concatenate([b[1] for b in batches_of_rank])
    wm = {"wm_arrival": np.concatenate([b[2]["wm_arrival"] for b in batches_of_rank]),
          "wm_ts": np.concatenate([b[2]["wm_ts"] for b in batches_of_rank]),
          "arrivals_end": batches_of_rank[-1][2]["arrivals_end"]}
    last = batches_of_rank[-1][2]
    wm.update(origin_known=last["origin_known"], origin_ts=last["origin_ts"], origin_arrival=last["origin_arrival"])
    if "sess_end" in last:
        for f in ("sess_start", "sess_end", "sess_wm"):
            wm[f] = np.concatenate([b[2][f] for b in batches_of_rank])
    ta, tt = trig if trig is not None else (None, None)
    return cols, arr, make_ctx(wm, arr, ta, tt)


def windows_payload(windows, decode):
    """Picklable per-window summary with global keys."""
    out = []
    for w in windows:
        g = decode(w.keys) if len(w.keys) else np.zeros(0, np.int64)
        out.append({"start": w.start, "end": w.end, "status": w.status, "mc": w.member_count, "mh": w.member_hash,
                    "keys": g.astype(np.int64), "values": [v.copy() for v in w.values], "tags": [t.copy() for t in w.tags]})
    return out


def assert_union_equals(plan, shards, single):
    """shards: per rank a list of window payloads; single: oracle windows of the whole stream."""
    for r, s in enumerate(shards):
        assert len(s) == len(single), f"rank {r}: {len(s)} windows, single stream {len(single)}"
    for w, e in enumerate(single):
        parts = [s[w] for s in shards]
        for p in parts:
            assert (p["start"], p["end"]) == (e.start, e.end), f"window {w}: {(p['start'], p['end'])} vs {(e.start, e.end)}"
        status = max(p["status"] for p in parts)
        assert status == e.status, f"window {w}: status {status} vs {e.status}"
        assert sum(p["mc"] for p in parts) == e.member_count, f"window {w}: member count"
        assert sum(p["mh"] for p in parts) % (1 << 64) == e.member_hash, f"window {w}: member hash"
        if status != 0:
            continue
        got = {}
        for p in parts:
            for r, k in enumerate(p["keys"].tolist()):
                assert k not in got, f"window {w}: key {k} emitted by two shards"
                got[k] = tuple((int(p["tags"][a][r]), int(p["values"][a][r])) for a in range(plan.n_aggs))
        exp = {int(k): tuple((int(e.tags[a][r]), int(e.values[a][r])) for a in range(plan.n_aggs))
               for r, k in enumerate(e.keys.tolist())}
        assert got.keys() == exp.keys(), f"window {w} (end {e.end}): key sets differ " \
                                         f"(missing {sorted(exp.keys() - got.keys())[:5]}, extra {sorted(got.keys() - exp.keys())[:5]})"
        bad = [k for k in exp if got[k] != exp[k] and not _fp_close(plan, got[k], exp[k])]
        assert not bad, f"window {w} (end {e.end}): {len(bad)} rows differ, e.g. key {bad[0]}: {got[bad[0]]} vs {exp[bad[0]]}"


def _fp_close(plan, g, e):
    from parity import FP_TOL_FNS, REL_TOL
    for a, ((tg, vg), (te, ve)) in enumerate(zip(g, e)):
        if tg != te:
            return False
        if vg == ve:
            continue
        if te != A.EK_TAG_F64 or plan.aggs[a].fn not in FP_TOL_FNS:
            return False
        x = np.array([vg], np.int64).view(np.float64)[0]
        y = np.array([ve], np.int64).view(np.float64)[0]
        if not abs(x - y) <= REL_TOL * max(abs(x), abs(y)):
            return False
    return True


def gather_triggers(rank_triggers):
    return merge_triggers(rank_triggers)
