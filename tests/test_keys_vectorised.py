"""The host dictionaries (ekgpu/keys.py) factorise columns in C and loop over distinct values only; checked against
the per-row definitions they replace (aggregate_operator.go:49-56 group key strings in first-seen order, nil rows,
"%v," collisions, -0 / NaN floats) on random columns, batch after batch."""
import numpy as np

from ekgpu.keys import GroupKeyDict, OrderedStringDict, StringDict, group_key_string


def _rows(n, rng):
    s = np.array([rng.choice(["a", "b", "a,b", "c", "b,c", ""]) for _ in range(n)], dtype=object)
    f = rng.choice([0.0, -0.0, 1.5, np.nan, 5.0], n)
    k = rng.integers(0, 7, n)
    vs = (rng.random(n) > 0.1).astype(np.uint8)
    vf = (rng.random(n) > 0.1).astype(np.uint8)
    return [s, f, k], [vs, vf, None]


def test_group_key_dict_matches_per_row_strings():
    rng = np.random.default_rng(3)
    d = GroupKeyDict(["s", "f", "k"], ["string", "float", "bigint"], capacity=1 << 20)
    ref_ids, ref_first = {}, []
    for _ in range(4):
        cols, valids = _rows(3000, rng)
        got = d.encode(cols, valids)
        for i in range(len(got)):
            row = tuple(None if (m is not None and not m[i]) else (c[i].item() if hasattr(c[i], "item") else c[i])
                        for c, m in zip(cols, valids))
            key = group_key_string(row)
            if key not in ref_ids:
                ref_ids[key] = len(ref_first)
                ref_first.append(row)
            assert got[i] == ref_ids[key]
    assert len(d) == len(ref_first)
    for a, b in zip(d.first, ref_first):
        assert group_key_string(a) == group_key_string(b)


def test_string_dicts_match_per_row():
    rng = np.random.default_rng(5)
    sd, od = StringDict(), OrderedStringDict()
    seen = []
    for _ in range(3):
        col = np.array([f"dev{rng.integers(0, 500):04d}" if rng.random() > 0.05 else None for _ in range(5000)],
                       dtype=object)
        valid = (rng.random(5000) > 0.05).astype(np.uint8)
        c1 = sd.encode(col, valid)
        c2 = od.encode(col, valid)
        for i, s in enumerate(col):
            if s is None or not valid[i]:
                assert c1[i] == 0 and c2[i] == 0
                continue
            if s not in seen:
                seen.append(s)
            assert sd.values[c1[i]] == s and seen.index(s) == c1[i]
            assert od.decode([c2[i]])[0] == s
    # order-preserving codes
    ss = sorted(seen)
    codes = [od.code[s] for s in ss]
    assert codes == sorted(codes)


def _per_row_ids(cols, valids):
    ids, out = {}, []
    for i in range(len(cols[0])):
        row = tuple(None if (m is not None and not m[i]) else c[i] for c, m in zip(cols, valids))
        out.append(ids.setdefault(group_key_string(row), len(ids)))
    return out


def test_mixed_type_object_dimension_keys_by_go_strings():
    """True == 1 == 1.0 in Python, but the reference's group key is the %v string: 1 and 1.0 print "1" (one group),
    true prints "true" (the group of the string "true", not of 1)."""
    col = np.array([True, 1, 1.0, "1", "true", None, 2.5, False, 0, "x"] * 3, dtype=object)
    d = GroupKeyDict(["v"], ["string"], capacity=64)
    got = list(d.encode([col], [None]))
    assert got == _per_row_ids([col], [None])
    assert got[0] == got[4] and got[1] == got[2] == got[3] and got[0] != got[1] and got[7] != got[8]


def test_factorize_without_pandas(monkeypatch):
    """pandas is optional: the numpy fallback gives the same first-seen codes."""
    import sys
    from ekgpu import keys
    rng = np.random.default_rng(11)
    cols, valids = _rows(2000, rng)
    with_pd = [keys._factorize(c, v) for c, v in zip(cols, valids)]
    monkeypatch.setitem(sys.modules, "pandas", None)
    without = [keys._factorize(c, v) for c, v in zip(cols, valids)]
    for (c1, u1), (c2, u2) in zip(with_pd, without):
        assert np.array_equal(c1, c2)
        assert [group_key_string([x]) for x in u1] == [group_key_string([x]) for x in u2]
