"""The multi-GPU protocol on the CPU (gloo, world_size 2 and 4): key-hash shards of ONE global stream with the
global WatermarkOp (ekgpu.shard.GlobalWatermark: WatermarkTuples broadcast to every shard, global arrival
indices, the global first-window anchor) and the sliding-trigger exchange (every rank evaluates OVER (WHEN ...)
on its own rows, the lists are all-gathered). Each rank runs the shard model of the protocol (oracle
eko_run_shard, the CPU restatement of ek_push_batch_global); rank 0 checks that the union of the shards equals
the single-stream oracle on EVERY window — including the windows closed by the global watermark, out-of-order
streams with late events, lateTolerance > 0, hopping windows across event-time gaps, COUNTWINDOW(1000) over the
global arrival order, SLIDINGWINDOW ... OVER (WHEN ...) and SESSIONWINDOW (the router's global session list,
ekgpu.shard.GlobalSession)."""
import os
import socket

import numpy as np
import pytest

import shard_harness as H
from ekgpu.rule import compile_rule


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from ekgpu.dist import all_gather_objects, exchange_triggers
    from oracle import ekoracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sql, tol, iet, kind = H.CASES[case]
        cols = H.global_stream(kind)
        per_rank, dicts = H.route(cols, world, batches=5, late_tol=tol, is_event_time=iet, sql=sql)
        mine = per_rank[rank]
        rule = compile_rule(sql, H.SCHEMA, num_keys=max(1, len(dicts[rank].global_of)), late_tolerance_ms=tol,
                            is_event_time=iet)
        lcols, arr, ctx = H.whole_ctx(mine)
        trig = None
        if "SLIDING" in sql:
            ta, tt = ekoracle.shard_triggers(rule.plan, lcols, ctx)
            trig = exchange_triggers(ta, tt)   # the exchange step (all_gather)
            lcols, arr, ctx = H.whole_ctx(mine, trig)
        run = ekoracle.run_shard(rule.plan, lcols, ctx)
        payload = H.windows_payload(run.windows, dicts[rank].decode)
        got = all_gather_objects(payload)
        if rank == 0:
            q.put(got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("case", sorted(H.CASES))
def test_sharded_union_equals_single_stream(oracle, case, world):
    if case == "tumbling_median" and world == 4:
        pytest.skip("covered at world 2")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    shards = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sql, tol, iet, kind = H.CASES[case]
    cols = H.global_stream(kind)
    rule = compile_rule(sql, H.SCHEMA, num_keys=300, late_tolerance_ms=tol, is_event_time=iet)
    single = oracle.run(rule.plan, cols, None).windows
    assert len(single) >= 5
    H.assert_union_equals(rule.plan, shards, single)


def test_global_watermark_matches_single_stream_tuples():
    """GlobalWatermark over 7 micro-batches = the per-event WatermarkOp: tuples, acceptance, first anchor."""
    from ekgpu.shard import GlobalWatermark, ZERO_MS
    cols = H.global_stream("ooo", n=20_000)
    ts = cols[1]
    for tol in (0, 500):
        gw = GlobalWatermark(tol)
        parts = [gw.track(x) for x in np.array_split(ts, 7)]
        wa = np.concatenate([p["wm_arrival"] for p in parts])
        wt = np.concatenate([p["wm_ts"] for p in parts])
        acc = np.concatenate([p["accepted"] for p in parts])
        # per-event restatement of watermark_op.go:144-225
        mark, last, ea, et, eacc, buf_min, origin = ZERO_MS + tol, ZERO_MS, [], [], [], None, None
        for i, t in enumerate(ts.tolist()):
            ok = t >= last
            eacc.append(ok)
            if t > mark:
                mark = t
            if ok:
                buf_min = t if buf_min is None else min(buf_min, t)
            w = mark - tol
            if w > last:
                ea.append(i)
                et.append(w)
                if origin is None and buf_min is not None and buf_min <= w:
                    origin = (buf_min, i)
                last = w
        assert wa.tolist() == ea and wt.tolist() == et
        assert acc.tolist() == eacc
        assert (gw.origin_ts, gw.origin_arrival) == origin
