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
