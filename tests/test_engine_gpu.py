"""GPU parity tests: the HIP engine (through the C ABI) against the CPU oracle on the same seeded inputs."""
import json
import os

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def engine_mod():
    # torch ships its own HIP/HSA runtime copy: it must open the device before libekgpu's runtime
    # does, or torch reports no GPUs ("sharing a process with PyTorch")
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:
        pass
    from ekgpu import engine
    if engine.lib().ek_device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")
    return engine


def run_both(oracle, engine_mod, rule, cols, batches=1, validity=None, shuffle_seed=None):
    exp = oracle.run(rule.plan, cols, validity)
    eng = engine_mod.Engine(rule.plan)
    n = len(cols[0])
    cuts = np.linspace(0, n, batches + 1).astype(np.int64)
    for b in range(batches):
        lo, hi = cuts[b], cuts[b + 1]
        eng.push_host([c[lo:hi] for c in cols], None if validity is None else
                      [None if v is None else v[lo:hi] for v in validity])
    got = eng.poll()
    st = eng.stats()
    eng.close()
    return got, exp, st


# ------------------------------------------------------------------ reference known-answer window tests
def _kat_cases():
    g = json.load(open(os.path.join(GOLD, "kat_window_rules.json")))
    return [c for c in g["tests"] if "SLIDING" not in c["sql"].upper()]


@pytest.mark.parametrize("case", _kat_cases(), ids=lambda c: c["name"])
def test_window_rule_kat_engine(oracle, engine_mod, case):
    g = json.load(open(os.path.join(GOLD, "kat_window_rules.json")))
    rows = np.array(g["streams"][case["stream"]]["rows"], dtype=object)
    cols = [np.array(rows[:, 0], np.int64), np.array(rows[:, 1], np.int64), np.array(rows[:, 2], np.uint32),
            np.array(rows[:, 3], np.float64)]
    schema = {"ts": "bigint", "size": "bigint", "color": "key", "temp": "float"}
    rule = compile_rule(case["sql"], schema, late_tolerance_ms=1000, num_keys=4, debug_membership=True,
                        is_event_time=case.get("event_time", True))
    got, exp, st = run_both(oracle, engine_mod, rule, cols)
    assert len(got) == case["windows_out"]
    assert st.records_late == case["late"]
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    # and, one event per micro-batch (the reference's per-tuple arrival)
    got1, _, _ = run_both(oracle, engine_mod, rule, cols, batches=len(cols[0]))
    assert_windows_equal(rule.plan, got1, exp.windows, check_members=True)


# ------------------------------------------------------------------ C2 shape at reduced size
C2_SQL = ("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
          "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)")


def _iot_cols(n, keys, seed=44, epm=100):
    key, ts, temp, hum = iot_stream(n, keys, seed=seed, events_per_ms=epm)
    return [key, ts, temp, hum]


@pytest.mark.parametrize("n,keys,batches", [(300_000, 1000, 1), (300_000, 1000, 7), (240_000, 65536, 3)])
def test_c2_tumbling_parity(oracle, engine_mod, n, keys, batches):
    rule = compile_rule(C2_SQL, IOT_SCHEMA, num_keys=keys, debug_membership=True)
    cols = _iot_cols(n, keys, epm=10 if keys < 10000 else 5)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
    assert len(got) >= 2
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_hopping_sum_min_max(oracle, engine_mod):
    sql = ("SELECT deviceId, sum(temperature), min(temperature), max(temperature) FROM demo "
           "GROUP BY deviceId, HOPPINGWINDOW(ss, 60, 5)")
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=2000, debug_membership=True)
    cols = _iot_cols(400_000, 2000, seed=45, epm=2)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=3)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_where_having_var(oracle, engine_mod):
    sql = ("SELECT deviceId, stddev(temperature), var(temperature), stddevs(humidity), vars(humidity), count(*) "
           "FROM demo WHERE temperature > 20 AND humidity < 90 GROUP BY deviceId, TUMBLINGWINDOW(ss, 5) "
           "HAVING count(*) > 1")
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=3000, debug_membership=True)
    cols = _iot_cols(250_000, 3000, seed=46, epm=10)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=2)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_out_of_order_late_events(oracle, engine_mod):
    sql = "SELECT deviceId, count(*), sum(temperature), max(humidity) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 2)"
    rule = compile_rule(sql, IOT_SCHEMA, num_keys=50, late_tolerance_ms=700, debug_membership=True)
    key, ts, temp, hum = iot_stream(20_000, 50, seed=47, events_per_ms=2)
    rng = np.random.default_rng(7)
    ts = ts + rng.integers(-1500, 1500, size=len(ts))   # jitter: some events become late
    cols = [key, ts.astype(np.int64), temp, hum]
    for batches in (1, 13):
        got, exp, st = run_both(oracle, engine_mod, rule, cols, batches=batches)
        assert exp.records_late > 0 and st.records_late == exp.records_late
        assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_int_columns_and_nulls(oracle, engine_mod):
    schema = {"k": "key", "ts": "bigint", "a": "bigint", "x": "float"}
    sql = ("SELECT k, count(*), count(a), sum(a), avg(a), min(a), max(a), var(a), avg(x), min(x) FROM s "
           "GROUP BY k, TUMBLINGWINDOW(ss, 1)")
    rule = compile_rule(sql, schema, num_keys=17, nullable=("a", "x"), debug_membership=True)
    n = 30_000
    rng = np.random.default_rng(3)
    k = rng.integers(0, 17, n).astype(np.uint32)
    ts = (1541152480000 + np.arange(n) // 5).astype(np.int64)
    a = rng.integers(-1000, 1000, n).astype(np.int64)
    x = rng.normal(size=n)
    va = (rng.random(n) > 0.3).astype(np.uint8)
    vx = (rng.random(n) > 0.9).astype(np.uint8)     # mostly NULL: some groups all-nil -> NULL results
    got, exp, _ = run_both(oracle, engine_mod, rule, [k, ts, a, x], batches=2, validity=[None, None, va, vx])
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_no_group_by(oracle, engine_mod):
    sql = "SELECT count(*), avg(temperature), max(humidity) FROM demo GROUP BY TUMBLINGWINDOW(ss, 10)"
    rule = compile_rule(sql, IOT_SCHEMA, debug_membership=True)
    cols = _iot_cols(100_000, 10, seed=48, epm=5)
    got, exp, _ = run_both(oracle, engine_mod, rule, cols)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)


def test_full_size_c2_properties(engine_mod):
    """BASELINE configs[1] at full size (1e8 events, 64 Ki keys) on the device, checked through
    size-independent properties: every emitted window holds exactly 1e6 events (100 per ms x 10 s),
    count(*) sums to that per window, max(humidity) lies in [0, 100), the last window stays open."""
    import torch
    n, keys = 100_000_000, 65536
    rule = compile_rule(C2_SQL, IOT_SCHEMA, num_keys=keys)
    dev = torch.device("cuda:0")
    from bench import make_device_stream
    cols = make_device_stream(n, keys, dev)
    eng = engine_mod.Engine(rule.plan)
    eng.push_device(n, [c.data_ptr() for c in cols])
    wins = eng.poll()
    assert len(wins) == 99
    for w in wins:
        assert w.status == 0
        assert (w.tags[2] == A.EK_TAG_I64).all() and (w.tags[0] == A.EK_TAG_F64).all()
        assert w.values[2].sum() == 1_000_000
        assert len(np.unique(w.keys)) == len(w.keys)
        mx = w.values[1].view(np.float64)
        assert (mx >= 0).all() and (mx < 100).all()
        avg = w.values[0].view(np.float64)
        assert (avg >= 0).all() and (avg < 100).all()
    eng.close()


def test_key_sharded_engines_union(oracle, engine_mod):
    """Two engine handles as two key-hash shards on one device: the union of their
    rows equals the single-stream oracle result; the handles share nothing."""
    from ekgpu.shard import ShardDictionary, shard_batch
    sql = "SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)"
    keys, world = 4000, 2
    cols = _iot_cols(300_000, keys, seed=52, epm=10)
    ref = {w.end: w.rows() for w in oracle.run(compile_rule(sql, IOT_SCHEMA, num_keys=keys).plan, cols).windows}
    shards = []
    for r in range(world):
        d = ShardDictionary()
        local, _ = shard_batch(cols, 0, world, r, d)
        eng = engine_mod.Engine(compile_rule(sql, IOT_SCHEMA, num_keys=len(d.global_of)).plan)
        for lo in range(0, len(local[0]), 50_000):
            eng.push_host([c[lo:lo + 50_000] for c in local])
        wins = eng.poll()
        eng.close()
        rows = {}
        for w in wins:
            rr = w.rows()
            g = d.decode(np.fromiter(rr.keys(), dtype=np.int64, count=len(rr)))
            rows[w.end] = {int(k): v for k, v in zip(g, rr.values())}
        shards.append((rows, int(local[1].max())))
    closed = min(m for _, m in shards)
    ends = [e for e in ref if e <= closed]
    assert len(ends) >= 2
    for e in ends:
        union = {}
        for rows, _ in shards:
            part = rows.get(e, {})
            assert not (set(part) & set(union))
            union.update(part)
        assert set(union) == set(ref[e])
        for k, v in ref[e].items():
            g = union[k]
            assert g[1:] == v[1:] and abs(g[0] - v[0]) <= 1e-6 * abs(v[0])

