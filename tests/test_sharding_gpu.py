"""The shard mode of the ENGINE (ek_push_batch_global / ek_shard_triggers / ek_advance_watermark) on one GPU:
2 and 4 handles, each owning a key-hash shard of one global stream, driven batch by batch exactly like the
multi-GPU deployment (global WatermarkOp on the host, sliding-trigger exchange between the shards). Checked:
  * every shard equals the CPU shard model of the protocol (oracle eko_run_shard): every window, membership
    fingerprint and row;
  * the union of the shards equals the single-stream oracle on EVERY window (incl. windows closed by the global
    watermark, late events, lateTolerance > 0, hopping gaps, COUNTWINDOW(1000), SLIDINGWINDOW OVER (WHEN)).
"""
import numpy as np
import pytest

import shard_harness as H
from ekgpu import abi as A
from ekgpu.rule import compile_rule
from ekgpu.shard import make_ctx, merge_triggers
from parity import assert_windows_equal
from test_engine_gpu import engine_mod  # noqa: F401

pytestmark = pytest.mark.gpu


def _run_engines(engine_mod, case, world, batches=5, debug=True):
    sql, tol, iet, kind = H.CASES[case]
    cols = H.global_stream(kind)
    per_rank, dicts = H.route(cols, world, batches=batches, late_tol=tol, is_event_time=iet, sql=sql)
    rules = [compile_rule(sql, H.SCHEMA, num_keys=max(1, len(dicts[r].global_of)), late_tolerance_ms=tol,
                          is_event_time=iet, debug_membership=debug) for r in range(world)]
    engs = [engine_mod.Engine(rules[r].plan) for r in range(world)]
    sliding = "SLIDING" in sql
    all_trig = []
    for b in range(batches):
        trig = (None, None)
        if sliding:
            parts = []
            for r in range(world):
                local, arr, wm = per_rank[r][b]
                parts.append(engs[r].shard_triggers(local, make_ctx(wm, arr)))
            trig = merge_triggers(parts)          # the all-gather of the multi-GPU deployment
            all_trig.append(trig)
        for r in range(world):
            local, arr, wm = per_rank[r][b]
            engs[r].push_global(local, make_ctx(wm, arr, *trig))
    got = [e.poll() for e in engs]
    for e in engs:
        e.close()
    if sliding:
        all_trig = (np.concatenate([t[0] for t in all_trig]), np.concatenate([t[1] for t in all_trig]))
    return cols, per_rank, dicts, rules, got, (all_trig if sliding else None)


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("case", sorted(H.CASES))
def test_engine_shards_union_and_model(oracle, engine_mod, case, world):
    sql, tol, iet, kind = H.CASES[case]
    cols, per_rank, dicts, rules, got, trig = _run_engines(engine_mod, case, world)
    # every shard = the CPU shard model of the protocol
    for r in range(world):
        lcols, arr, ctx = H.whole_ctx(per_rank[r], trig)
        if trig is not None:
            ta, tt = oracle.shard_triggers(rules[r].plan, lcols, H.whole_ctx(per_rank[r])[2])
            mine = np.isin(trig[0], arr)
            assert np.array_equal(trig[0][mine], ta) and np.array_equal(trig[1][mine], tt), "engine triggers != model"
        model = oracle.run_shard(rules[r].plan, lcols, ctx)
        assert_windows_equal(rules[r].plan, got[r], model.windows, check_members=True)
    # the union = the single-stream oracle
    rule = compile_rule(sql, H.SCHEMA, num_keys=300, late_tolerance_ms=tol, is_event_time=iet)
    single = oracle.run(rule.plan, cols, None).windows
    assert len(single) >= 5
    shards = [H.windows_payload(got[r], dicts[r].decode) for r in range(world)]
    H.assert_union_equals(rule.plan, shards, single)


def test_advance_watermark_closes_windows(oracle, engine_mod):
    """ek_advance_watermark = a WatermarkTuple without rows: the shard closes every window it reaches."""
    sql, tol, iet, kind = H.CASES["tumbling_ooo_late"]
    cols = H.global_stream(kind)
    per_rank, dicts = H.route(cols, 2, batches=3, late_tol=tol, is_event_time=iet)
    rule = compile_rule(sql, H.SCHEMA, num_keys=len(dicts[0].global_of), debug_membership=True)
    eng = engine_mod.Engine(rule.plan)
    for local, arr, wm in per_rank[0]:
        eng.push_global(local, make_ctx(wm, arr))
    before = eng.poll()
    last = per_rank[0][-1][2]
    w_end = int(last["wm_ts"][-1]) + 10_000
    eng.advance_watermark(w_end, last["arrivals_end"])
    after = eng.poll()
    eng.close()
    assert len(after) >= 4 and all(w.end <= w_end for w in after)
    # the model with the same extra tuple
    lcols, arr, _ = H.whole_ctx(per_rank[0])
    wm = {"wm_arrival": np.concatenate([b[2]["wm_arrival"] for b in per_rank[0]] + [[last["arrivals_end"] - 1]]),
          "wm_ts": np.concatenate([b[2]["wm_ts"] for b in per_rank[0]] + [[w_end]]),
          "arrivals_end": last["arrivals_end"], "origin_known": last["origin_known"], "origin_ts": last["origin_ts"],
          "origin_arrival": last["origin_arrival"]}
    model = oracle.run_shard(rule.plan, lcols, make_ctx(wm, arr))
    assert_windows_equal(rule.plan, before + after, model.windows, check_members=True)


def test_shard_mode_rejections(engine_mod):
    """Windows whose content depends on every row of the stream are not shardable; local and shard pushes
    do not mix on one handle."""
    sess = compile_rule("SELECT deviceId, count(*) FROM demo GROUP BY deviceId, STATEWINDOW(trig = 1, humidity > 99)",
                        H.SCHEMA, num_keys=4)
    eng = engine_mod.Engine(sess.plan)
    wm = {"wm_arrival": np.zeros(0, np.int64), "wm_ts": np.zeros(0, np.int64), "arrivals_end": 0,
          "origin_known": False, "origin_ts": 0, "origin_arrival": 0}
    with pytest.raises(engine_mod.EngineError) as ei:
        eng.advance_watermark(1541152480000, 1)
    assert ei.value.code == A.EK_ERR_UNSUPPORTED
    eng.close()
    # send-twice keeps an expired prefix of every input of the stream: not shardable by key
    st2 = compile_rule(H.CASES["sliding_delay"][0], H.SCHEMA, num_keys=4, sliding_send_twice=True)
    eng = engine_mod.Engine(st2.plan)
    with pytest.raises(engine_mod.EngineError) as ei:
        eng.advance_watermark(1541152480000, 1)
    assert ei.value.code == A.EK_ERR_UNSUPPORTED
    eng.close()
    tum = compile_rule(H.CASES["tumbling_ooo_late"][0], H.SCHEMA, num_keys=300)
    eng = engine_mod.Engine(tum.plan)
    cols = H.global_stream("sorted", n=100)
    eng.push_host(cols)
    with pytest.raises(engine_mod.EngineError) as ei:
        eng.push_global(cols, make_ctx(wm, np.arange(100)))
    assert ei.value.code == A.EK_ERR_STATE
    eng.close()


def test_session_shard_watermark_takes_session_list(engine_mod):
    """A SESSIONWINDOW shard: ek_advance_watermark (no session list) is refused rather than losing the sessions the
    tuple closes; Engine.advance_watermark(..., sessions=) delivers them through ek_push_batch_global; session ends
    must advance across pushes."""
    rule = compile_rule(H.CASES["session_gaps"][0], H.SCHEMA, num_keys=4)
    eng = engine_mod.Engine(rule.plan)
    with pytest.raises(engine_mod.EngineError) as ei:
        eng.advance_watermark(1541152480000, 1)
    assert ei.value.code == A.EK_ERR_INVALID
    eng.advance_watermark(1541152490000, 1, sessions=[(1541152480000, 1541152485000)])
    with pytest.raises(engine_mod.EngineError) as ei:
        eng.advance_watermark(1541152500000, 1, sessions=[(1541152481000, 1541152484000)])
    assert ei.value.code == A.EK_ERR_INVALID
    eng.close()
