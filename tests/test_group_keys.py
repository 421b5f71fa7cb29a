"""Multi-dimension / string GROUP BY through the host key dictionary (ekgpu/keys.py): the reference's group key is
the concatenation of fmt.Sprintf("%v,", dim) over the dimensions (aggregate_operator.go:49-56). CPU tests: the Go
%v formatting, the key-string equivalence (including the comma collision and nil), the dictionary's vectorised
numeric path against a per-row restatement, and the rule lowering + oracle on a composite key."""
import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.keys import GroupKeyDict, go_v, go_v_float, group_key_string
from ekgpu.rule import GROUP_KEY, RuleError, compile_rule
from parity import assert_windows_equal
from test_engine_gpu import engine_mod, run_both  # noqa: F401  (fixture + helper)

# fmt.Println outputs of float64 values: %v is strconv's shortest %g, exponent form when the decimal exponent is
# < -4 or >= 6 (fmt.Println(1e6) prints 1e+06, fmt.Println(123456.0) prints 123456)
GO_V_FLOAT = [
    (1.0, "1"), (0.1, "0.1"), (100000.0, "100000"), (123456.0, "123456"), (1e6, "1e+06"),
    (1234567.0, "1.234567e+06"), (0.0001, "0.0001"), (0.00001, "1e-05"), (1.2e-5, "1.2e-05"), (-2.5, "-2.5"),
    (1e21, "1e+21"), (3.14159, "3.14159"), (-0.0, "-0"), (0.0, "0"), (float("nan"), "NaN"),
    (float("inf"), "+Inf"), (float("-inf"), "-Inf"), (5e-324, "5e-324"), (1.7976931348623157e308, "1.7976931348623157e+308"),
]


@pytest.mark.parametrize("x,s", GO_V_FLOAT, ids=[s for _, s in GO_V_FLOAT])
def test_go_v_float(x, s):
    assert go_v_float(x) == s


def test_go_v_other_types():
    assert go_v(None) == "<nil>"
    assert go_v(True) == "true" and go_v(False) == "false"
    assert go_v(np.int64(-7)) == "-7" and go_v("a b") == "a b"


def test_group_key_string_quirks():
    # aggregate_operator.go:49-56: "%v," per dimension, so comma-bearing values can collide
    assert group_key_string(["a,b", "c"]) == group_key_string(["a", "b,c"]) == "a,b,c,"
    assert group_key_string([1, "x"]) == "1,x,"
    assert group_key_string([None, 2.0]) == "<nil>,2,"
    assert group_key_string([1, 1.0]) == group_key_string([1.0, 1]) == "1,1,"   # int 1 and float 1 print alike


def _naive_ids(rows):
    ids, out = {}, []
    for r in rows:
        out.append(ids.setdefault(group_key_string(r), len(ids)))
    return np.array(out)


def _same_partition(a, b):
    """a and b induce the same equivalence classes (and the same first-seen numbering)."""
    return np.array_equal(np.asarray(a), np.asarray(b))


def test_dictionary_numeric_path_matches_key_strings():
    rng = np.random.default_rng(3)
    n = 5000
    a = rng.integers(-3, 3, n)
    f = rng.choice(np.array([0.5, -0.0, 0.0, np.nan, 1e6, 2.0]), n)
    va = (rng.random(n) > 0.1).astype(np.uint8)
    d = GroupKeyDict(["a", "f"], ["bigint", "float"], 10_000)
    got = np.concatenate([d.encode([a[:2000], f[:2000]], [va[:2000], None]), d.encode([a[2000:], f[2000:]], [va[2000:], None])])
    rows = [(None if not va[i] else int(a[i]), float(f[i])) for i in range(n)]
    assert _same_partition(got, _naive_ids(rows))
    # first row's values per id
    for i in range(n):
        r = d.decode([got[i]])[0]
        assert group_key_string(r) == group_key_string(rows[i])


@pytest.mark.parametrize("as_object", [False, True])
def test_single_float_dimension_signed_zero(as_object):
    """fmt %v prints -0.0 as "-0" and 0.0 as "0": two groups in the reference (aggregate_operator.go:49-56); every NaN
    prints "NaN": one group. A single float dimension (numpy or object column) keeps that split."""
    f = np.array([0.0, -0.0, 1.5, np.nan, -0.0, 0.0, np.nan, 1.5])
    col = np.array(list(f), dtype=object) if as_object else f
    d = GroupKeyDict(["f"], ["float"], 100)
    got = d.encode([col], [None])
    rows = [(float(x),) for x in f]
    assert _same_partition(got, _naive_ids(rows))
    assert len(set(got.tolist())) == 4
    for i in range(len(f)):
        assert group_key_string(d.decode([got[i]])[0]) == group_key_string(rows[i])


def test_dictionary_string_path_collisions():
    d = GroupKeyDict(["s", "t"], ["string", "string"], 100)
    ids = d.encode([np.array(["a,b", "a", "x", "a,b"], object), np.array(["c", "b,c", "y", "c"], object)])
    assert list(ids) == [0, 0, 1, 0]
    assert d.decode([0]) == [("a,b", "c")]                 # the group's first row
    with pytest.raises(OverflowError):
        GroupKeyDict(["s"], ["string"], 1).encode([np.array(["p", "q"], object)])


SCHEMA = {"deviceId": "bigint", "color": "string", "ts": "bigint", "temperature": "float", "humidity": "float"}
SQL = ("SELECT deviceId, color, avg(temperature), max(humidity), count(*) FROM demo "
       "GROUP BY deviceId, color, TUMBLINGWINDOW(ss, 1)")


def _stream(n=20_000, seed=5):
    rng = np.random.default_rng(seed)
    dev = rng.integers(0, 30, n).astype(np.int64)
    color = rng.choice(np.array(["red", "green", "blue,green", "blue"], object), n)
    ts = (1541152480000 + np.arange(n) // 5).astype(np.int64)
    return [dev, color, ts, rng.random(n) * 100, rng.random(n) * 100]


def test_composite_rule_lowering():
    r = compile_rule(SQL, SCHEMA, num_keys=1000)
    assert r.group_dims == ["deviceId", "color"] and r.columns[-1] == GROUP_KEY
    assert r.plan.key_column == len(SCHEMA) and r.plan.column_type[len(SCHEMA)] == A.EK_COL_U32
    assert [f.kind for f in r.fields] == ["dim", "dim", "agg", "agg", "agg"]
    with pytest.raises(RuleError):   # a string column inside an aggregate
        compile_rule("SELECT avg(color) FROM demo GROUP BY deviceId, color, TUMBLINGWINDOW(ss, 1)", SCHEMA, num_keys=10)
    # one key-typed dimension keeps the direct path
    r1 = compile_rule("SELECT k, count(*) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1)", {"k": "key", "ts": "bigint"}, num_keys=4)
    assert r1.key_dict is None and r1.plan.key_column == 0


def test_composite_groups_match_reference_grouping(oracle):
    """Oracle over the dictionary-encoded key == per-window grouping by the reference's key strings."""
    rule = compile_rule(SQL, SCHEMA, num_keys=1000)
    cols = _stream()
    dcols, _ = rule.device_columns(cols)
    res = oracle.run(rule.plan, dcols)
    assert len(res.windows) >= 3
    ts = cols[2]
    for w in res.windows:
        m = (ts >= w.start) & (ts < w.end)
        exp = {}
        for i in np.nonzero(m)[0]:
            k = group_key_string((int(cols[0][i]), cols[1][i]))
            c, s, mx = exp.get(k, (0, 0.0, -1.0))
            exp[k] = (c + 1, s + cols[3][i], max(mx, cols[4][i]))
        got = {group_key_string(rule.decode_keys([key])[0]): vals for key, vals in w.rows().items()}
        assert set(got) == set(exp)
        for k, (c, s, mx) in exp.items():
            avg, hmax, cnt = got[k]
            assert cnt == c and hmax == mx and abs(avg - s / c) <= 1e-9 * max(1.0, abs(s / c))


@pytest.mark.gpu
@pytest.mark.parametrize("sql", [
    SQL,
    "SELECT color, deviceId, stddev(temperature), min(humidity) FROM demo "
    "GROUP BY color, deviceId, SLIDINGWINDOW(ms, 700) OVER (WHEN humidity > 99.5) HAVING count(*) > 1",
])
def test_composite_key_engine_parity(oracle, engine_mod, sql):
    """The engine over the dictionary-encoded key == the oracle on the same columns; the decoded dimensions of
    each window's rows are distinct reference keys."""
    rule = compile_rule(sql, SCHEMA, num_keys=1000, debug_membership=True)
    dcols, dval = rule.device_columns(_stream(40_000, seed=8))
    got, exp, _ = run_both(oracle, engine_mod, rule, dcols, batches=3, validity=dval)
    assert len(got) >= 3
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    for w in got:
        ks = [group_key_string(t) for t in rule.decode_keys(w.keys)]
        assert len(set(ks)) == len(ks)


# ---------------------------------------------------------------- nullable GROUP BY key: nil is its own group "<nil>,"
NK_SCHEMA = {"k": "key", "ts": "bigint", "v": "float"}
NK_SQLS = [
    "SELECT k, count(*), avg(v), max(v) FROM s GROUP BY k, TUMBLINGWINDOW(ms, 500)",
    "SELECT k, stddev(v), min(v) FROM s GROUP BY k, SLIDINGWINDOW(ms, 300) OVER (WHEN v > 99.0) HAVING count(*) > 1",
    "SELECT k, median(v), count(*) FROM s GROUP BY k, HOPPINGWINDOW(ms, 600, 200)",
]


def _nk_stream(n=30_000, seed=9):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, 40, n).astype(np.uint32)
    valid = (rng.random(n) > 0.1).astype(np.uint8)   # 10 % nil keys
    k[valid == 0] = rng.integers(0, 40, int((valid == 0).sum()))   # (a nil row's stored value is arbitrary)
    ts = (1541152480000 + np.arange(n) // 7).astype(np.int64)
    return [k, ts, rng.random(n) * 100], [valid, None, None]


def _by_key(rule, w, direct):
    """A window's rows keyed by the reference's group key string (the nil group is "<nil>,")."""
    out = {}
    for key, vals in w.rows().items():
        if direct:
            dim = (None,) if int(key) in (-1, 0xFFFFFFFF) else (int(key),)
        else:
            dim = rule.decode_keys([key])[0]
        out[group_key_string(dim)] = vals
    return out


@pytest.mark.parametrize("sql", NK_SQLS)
def test_nullable_key_lowering_matches_direct_oracle(oracle, sql):
    """Lowering (nullable key -> group-key dictionary, nil an id of its own) == the oracle grouping the nullable key
    column directly (ekoracle.c run_window: a nil key is the group of key -1, i.e. "<nil>,")."""
    cols, valid = _nk_stream()
    rule = compile_rule(sql, NK_SCHEMA, num_keys=64, nullable=("k",))
    assert rule.key_dict is not None and rule.plan.key_column == len(NK_SCHEMA)
    dcols, dval = rule.device_columns(cols, valid)
    lowered = oracle.run(rule.plan, dcols, dval).windows
    direct_rule = compile_rule(sql, NK_SCHEMA, num_keys=64)
    assert direct_rule.key_dict is None
    direct_rule.plan.nullable_mask |= 1 << 0
    direct = oracle.run(direct_rule.plan, cols, valid).windows
    assert len(lowered) == len(direct) >= 3
    n_nil = 0
    for a, b in zip(lowered, direct):
        assert (a.start, a.end, a.status) == (b.start, b.end, b.status)
        ga, gb = _by_key(rule, a, False), _by_key(direct_rule, b, True)
        assert ga.keys() == gb.keys()
        for k in ga:
            for x, y in zip(ga[k], gb[k]):
                assert x == y or (isinstance(x, float) and abs(x - y) <= 1e-9 * max(1.0, abs(y)))
        n_nil += "<nil>," in ga
    assert n_nil >= len(lowered) // 2


@pytest.mark.gpu
@pytest.mark.parametrize("sql", NK_SQLS)
def test_nullable_key_engine_parity(oracle, engine_mod, sql):
    """The engine over the lowered rule == the oracle grouping the nullable key directly, window by window."""
    from parity import assert_windows_equal
    cols, valid = _nk_stream(60_000, seed=10)
    rule = compile_rule(sql, NK_SCHEMA, num_keys=64, nullable=("k",), debug_membership=True)
    dcols, dval = rule.device_columns(cols, valid)
    got, exp, _ = run_both(oracle, engine_mod, rule, dcols, batches=3, validity=dval)
    assert_windows_equal(rule.plan, got, exp.windows, check_members=True)
    direct_rule = compile_rule(sql, NK_SCHEMA, num_keys=64)
    direct_rule.plan.nullable_mask |= 1 << 0
    direct = oracle.run(direct_rule.plan, cols, valid).windows
    assert len(got) == len(direct)
    for a, b in zip(got, direct):
        ks = {group_key_string(t) for t in rule.decode_keys(a.keys)}
        assert ks == set(_by_key(direct_rule, b, True))
