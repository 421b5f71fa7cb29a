"""min / max over a string column (common_array_funcs.go:49,86: bytewise comparison, seed = the first valid value):
the column travels as order-preserving int64 codes (ekgpu.keys.OrderedStringDict), so the engine's integer min / max is
the lexicographic one and CompiledRule.decode_value maps the code back. CPU: the dictionary's order invariant and the
oracle against Python's min / max per (window, key); GPU: engine parity in pane and range mode, with nulls."""
import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.keys import OrderedStringDict
from ekgpu.rule import compile_rule

T0 = 1541152480000
SCHEMA = {"k": "key", "ts": "bigint", "name": "string", "x": "float"}


def _words(rng, n):
    alpha = np.array(list("abcxyzé中"))
    return ["".join(rng.choice(alpha, rng.integers(0, 5))) for _ in range(n)]


def test_ordered_codes_follow_string_order():
    rng = np.random.default_rng(3)
    d = OrderedStringDict()
    words = _words(rng, 3000)
    codes = d.encode(words)
    pairs = sorted(set(zip(words, codes.tolist())))
    assert [c for _, c in pairs] == sorted(c for _, c in pairs)          # code order == string order
    assert d.decode(codes[:50]) == words[:50]
    assert all(s.encode() < t.encode() for s, t in zip(d.sorted, d.sorted[1:]))   # Go's bytewise order


@pytest.mark.parametrize("order", ["ascending", "descending", "ascending_inside_gap", "descending_inside_gap"])
def test_ordered_codes_monotone_runs(order):
    """Monotone runs (ISO timestamps, sequence ids) must not exhaust the code space (midpoint placement
    failed at the 63rd ascending value)."""
    d = OrderedStringDict()
    vals = [f"id{i:07d}" for i in range(10_000)]
    if order.startswith("descending"):
        vals = vals[::-1]
    if order.endswith("inside_gap"):
        d.encode(["id", "iz"])            # every run value sorts between these two
    codes = d.encode(vals)
    srt = sorted(zip(vals, codes.tolist()))
    assert all(a[1] < b[1] for a, b in zip(srt, srt[1:]))
    assert d.decode(codes[:5]) == vals[:5]
    # interleaved random insertions after the run still find room
    rng = np.random.default_rng(0)
    more = [f"id{int(x):07d}x" for x in rng.integers(0, 10_000, 2000)]
    c2 = d.encode(more)
    allv = sorted(set(zip(vals + more, codes.tolist() + c2.tolist())))
    assert all(a[1] < b[1] for a, b in zip(allv, allv[1:]))


def test_string_nil_rows_are_not_dictionary_entries():
    """None (or validity 0) rows of a nullable string column take a placeholder code and validity 0."""
    d = OrderedStringDict()
    out = d.encode(["a", None, "b"])
    assert len(d.sorted) == 2 and out[1] == 0
    out = d.encode(["c", "zz"], np.array([1, 0], np.uint8))
    assert "zz" not in d.code
    rule = compile_rule("SELECT k, min(name), max(name) FROM s GROUP BY k, TUMBLINGWINDOW(ms, 300)", SCHEMA,
                        num_keys=4, nullable=("name",))
    cols, valid = rule.device_columns([np.zeros(3, np.uint32), np.full(3, T0, np.int64), ["q", None, "r"],
                                       np.zeros(3)])
    assert valid is not None and list(valid[2]) == [1, 0, 1]
    strict = compile_rule("SELECT k, min(name) FROM s GROUP BY k, TUMBLINGWINDOW(ms, 300)", SCHEMA, num_keys=4)
    with pytest.raises(ValueError):
        strict.device_columns([np.zeros(2, np.uint32), np.full(2, T0, np.int64), ["q", None], np.zeros(2)])


def _stream(n, keys, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, keys, n).astype(np.uint32), (T0 + np.arange(n) // 5).astype(np.int64), _words(rng, n),
            rng.uniform(0, 1, n)]


def test_oracle_string_min_max_matches_python(oracle):
    rule = compile_rule("SELECT k, min(name), max(name), count(name) FROM s GROUP BY k, TUMBLINGWINDOW(ms, 300)",
                        SCHEMA, num_keys=20)
    assert rule.plan.column_type[2] == A.EK_COL_I64
    raw = _stream(20_000, 20, 5)
    cols, _ = rule.device_columns(raw)
    run = oracle.run(rule.plan, cols)
    ts, k, names = raw[1], raw[0], np.array(raw[2], dtype=object)
    checked = 0
    assert len(run.windows) > 5
    for w in run.windows[1:]:          # (the first tumbling window also holds everything before it)
        mn = dict(zip(map(int, w.keys), rule.decode_value(0, w.values[0], w.tags[0])))
        mx = dict(zip(map(int, w.keys), rule.decode_value(1, w.values[1], w.tags[1])))
        inw = (ts >= w.start) & (ts < w.end)
        for key in mn:
            sel = list(names[inw & (k == key)])
            assert mn[key] == min(sel) and mx[key] == max(sel)
            checked += 1
    assert checked > 100


@pytest.mark.gpu
@pytest.mark.parametrize("window", ["TUMBLINGWINDOW(ms, 300)", "SLIDINGWINDOW(ms, 400) OVER (WHEN x > 0.995)"])
def test_engine_string_min_max(oracle, window):
    from ekgpu.engine import Engine
    from parity import assert_windows_equal
    rule = compile_rule(f"SELECT k, min(name), max(name), count(name), name FROM s GROUP BY k, {window}", SCHEMA,
                        num_keys=50, nullable=("name",), debug_membership=True)
    raw = _stream(40_000, 50, 7)
    cols, _ = rule.device_columns(raw)
    valid = [None, None, (np.random.default_rng(1).random(40_000) > 0.1).astype(np.uint8), None]
    exp = oracle.run(rule.plan, cols, valid)
    eng = Engine(rule.plan)
    for a, b in ((0, 15_000), (15_000, 40_000)):
        eng.push_host([c[a:b] for c in cols], [None if v is None else v[a:b] for v in valid])
    got = eng.poll()
    eng.close()
    assert len(exp.windows) >= 10
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
