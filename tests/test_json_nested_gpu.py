"""GPU tests of the nested JSON forms of the columnar ingest (ABI v14, ek_json_*).

* converter cases: the struct / array rows of TestFastJsonConverterWithSchema, TestFastJsonConverterWithSchemaError,
  TestArrayWithArray and TestTypeNull (internal/converter/json/converter_test.go:32-182,184-342,354-393,395-577),
  decoded from their raw payloads, each also sent as a one-element top-level array as the reference's second loop
  does (:172-181, :556-576);
* a number sent for a STRING field: cast.ToStringAlways(float64) = Go's %v (converter.go:446-451; the %v spellings are
  fmt's shortest 'g' with exponent threshold 6, hand-derived: parity unpinned by a reference fixture);
* subnormal FLOAT literals: bit-identical to Python's correctly rounded float() (strconv.ParseFloat returns them
  without error);
* top-level array payloads (decodeWithSchema's []map case, converter.go:141-158): one row per element, in order;
* random nested payloads against a restatement of decodeObject / decodeArray over the columns' paths (this file's
  go_extract: Go map assignment = Python's last-duplicate-wins dict, "has wrong type" for a container of the wrong
  kind).
"""
import json
import struct

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.engine import device_to_host
from test_engine_gpu import engine_mod  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu

OK, SYN, TYP, NUM = A.EK_JSON_OK, A.EK_JSON_ERR_SYNTAX, A.EK_JSON_ERR_TYPE, A.EK_JSON_ERR_NUMBER
_NP = {"bigint": np.int64, "float": np.float64, "boolean": np.int64, "key": np.uint32, "string": np.uint32}


def read_rows(dec, schema, batch):
    """Decoded rows as python values (scalar columns straight from the batch's device columns; LIST columns through
    ek_json_list; STRING columns through the decoder's dictionary)."""
    n = int(batch.n_rows)
    cols = []
    for c, (name, t) in enumerate(schema.items()):
        if t.startswith("array<"):
            cols.append(dec.lists(c, batch))
            continue
        if n == 0:
            cols.append([])
            continue
        v = device_to_host(batch.columns[c], n, _NP[t])
        ok = device_to_host(batch.validity[c], n, np.uint8) if batch.validity[c] else np.ones(n, np.uint8)
        if t == "float":
            vals = [float(x) for x in v]
        elif t == "boolean":
            vals = [bool(x) for x in v]
        elif t == "string":
            tab = dec.strings(c)
            vals = [tab[x] for x in v]
        else:
            vals = [int(x) for x in v]
        cols.append([x if o else None for x, o in zip(vals, ok)])
    return [tuple(col[r] for col in cols) for r in range(n)]


def decode(engine_mod, schema, msgs, paths=True):
    dec = engine_mod.JsonDecoder(schema, paths=paths)
    b = dec.decode(msgs)
    idx, code = dec.errors()
    return dec, b, dict(zip(idx.tolist(), code.tolist()))


# (schema, payload, expected row | error code) — converter_test.go
CONVERTER_CASES = [
    ({"a": "array<boolean>"}, b'{"a":["true"]}', ([True],)),                              # :40-53
    ({"a": "array<boolean>"}, b'{"a":[true]}', ([True],)),                                # :54-67
    ({"a.b": "bigint"}, b'{"a":{"b":1}}', (1,)),                                          # :145-162
    ({"a": "array<bigint>"}, b'{"a":123}', TYP),                                          # :226-234 expect:array
    ({"a.b": "bigint"}, b'{"a":123}', TYP),                                               # :235-243 expect:struct
    ({"a": "array<bigint>"}, b'{"a":[{"b":1}]}', TYP),                                    # :262-273
    ({"a[0][0]": "bigint"}, b'{"a":[123]}', TYP),                                         # :286-297 items array
    ({"a[0].b": "bigint"}, b'{"a":[123]}', TYP),                                          # :298-309 items struct
    ({"a": "array<boolean>"}, b'{"a":[{"b":1}]}', TYP),                                   # :310-321
    ({"a": "bigint"}, b'123', SYN),                                                       # :199-207 "only map ..."
    ({"a": "bigint"}, b'{123}', SYN),                                                     # :190-198
    ({"a[0][0].c": "bigint"}, b'{"a":[[{"c":1}]]}', (1,)),                                # TestArrayWithArray :354-393
    ({"a": "array<float>"}, b'{"a":[null]}', ([None],)),                                  # TestTypeNull :430-442
    ({"a": "array<bigint>"}, b'{"a":[null]}', ([None],)),                                 # :443-456
    ({"a": "array<boolean>"}, b'{"a":[null]}', ([None],)),                                # :457-470
    ({"a.b": "bigint"}, b'{"a":{"b":null}}', (None,)),                                    # :537-554
    ({"a": "array<float>"}, b'{"a":null}', (None,)),
    ({"a": "array<float>"}, b'{"a":[1, 2.5, -3e2]}', ([1.0, 2.5, -300.0],)),
    ({"a": "array<bigint>"}, b'{"a":[1, 2.5]}', NUM),
    ({"a": "array<bigint>"}, b'{"a":[]}', ([],)),
    ({"a": "array<bigint>"}, b'{"a":[1,]}', SYN),
    ({"a.b": "float", "a.c": "bigint"}, b'{"a":{"c":2,"b":0.5,"z":[{"q":1}]}}', (0.5, 2)),
    ({"a.b": "float"}, b'{"a":{"b":1},"a":{"c":2}}', (None,)),   # a repeated key replaces the subtree (map assignment)
    ({"a.b": "float"}, b'{"a":{"b":1},"a":null}', (None,)),
    ({"a.b": "float"}, b'{"a":null,"a":{"b":3}}', (3.0,)),
    ({"a.b": "float"}, b'{"a":5,"a":{"b":3}}', TYP),   # Visit reports the first occurrence's error (converter.go:249-260)
    ({"a.b.c": "bigint"}, b'{"a":{"b":{"c":7}}}', (7,)),
    ({"a.b.c": "bigint"}, b'{"a":{"b":[1]}}', TYP),
    ({"x[2]": "float"}, b'{"x":[1,2]}', (None,)),                 # index past the end: nil
    ({"x[1]": "float"}, b'{"x":[1,{"q":[2]},3.5]}', TYP),   # an element of the wrong kind for FLOAT
    ({"x[2]": "float"}, b'{"x":[1,{"q":[2]},3.5]}', (3.5,)),
    ({"s": "string"}, b'{"s":1000000}', ("1e+06",)),              # cast.ToStringAlways(float64) = %v
    ({"s": "string"}, b'{"s":2.5}', ("2.5",)),
    ({"s": "string"}, b'{"s":100000}', ("100000",)),
    ({"s": "string"}, b'{"s":0.00001}', ("1e-05",)),
    ({"s": "string"}, b'{"s":-123456789}', ("-1.23456789e+08",)),
    ({"s": "string"}, b'{"s":0.0001}', ("0.0001",)),
]


@pytest.mark.parametrize("k", range(len(CONVERTER_CASES)))
def test_converter_cases(engine_mod, k):
    schema, payload, exp = CONVERTER_CASES[k]
    # the payload as sent, then as a one-element top-level array (converter_test.go:172-181)
    dec, b, errs = decode(engine_mod, schema, [payload, b"[" + payload + b"]"])
    if isinstance(exp, tuple):
        assert errs == {}, errs
        assert read_rows(dec, schema, b) == [exp, exp]
        assert dec.rows_of().tolist() == [1, 1]
    else:
        assert errs.get(0) == exp, errs
        # (a non-object element fails the array message too; a syntax error inside stays a syntax error)
        assert 1 in errs
        assert b.n_rows == 0
    dec.close()


def test_number_string_dictionary(engine_mod):
    """A STRING column receiving strings and numbers: the numbers' %v spellings share the dictionary with strings."""
    schema = {"s": "string", "v": "bigint"}
    msgs = [b'{"s":"1e+06","v":1}', b'{"s":1000000,"v":2}', b'{"s":1e6,"v":3}', b'{"s":"x","v":4}', b'{"s":7,"v":5}']
    dec, b, errs = decode(engine_mod, schema, msgs)
    assert errs == {}
    rows = read_rows(dec, schema, b)
    assert rows == [("1e+06", 1), ("1e+06", 2), ("1e+06", 3), ("x", 4), ("7", 5)]
    assert dec.strings(0) == ["1e+06", "x", "7"]
    # second batch: the strings are dictionary hits now, the numbers still resolve through the host
    b = dec.decode(msgs[::-1])
    assert read_rows(dec, schema, b) == rows[::-1]
    dec.close()


def _bits(x):
    return struct.unpack("<q", struct.pack("<d", x))[0]


def test_subnormal_floats(engine_mod):
    rng = np.random.default_rng(21)
    lits = ["4.9e-324", "5e-324", "2.4703282292062327e-324", "2.4703282292062328e-324", "1e-323",
            "2.225073858507201e-308", "2.2250738585072009e-308", "2.2250738585072014e-308", "1e-310", "-3.5e-320",
            "0.000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000"
            "0000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000"
            "000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000"
            "00000000000123"]
    for _ in range(3000):
        m = int(rng.integers(1, 10**int(rng.integers(1, 18))))
        e = int(rng.integers(-343, -307))
        lits.append(f"{m}e{e}")
    msgs = [f'{{"x":{s}}}'.encode() for s in lits]
    dec, b, errs = decode(engine_mod, {"x": "float"}, msgs, paths=False)
    assert errs == {}, [(lits[i], c) for i, c in list(errs.items())[:5]]
    got = device_to_host(b.columns[0], len(lits), np.int64)
    exp = np.array([_bits(float(s)) for s in lits], np.int64)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(lits[i], got[i], exp[i]) for i in bad[:5]]
    dec.close()


def test_top_level_arrays(engine_mod):
    schema = {"id": "bigint", "v": "float"}
    msgs = [b'{"id":1,"v":0.5}', b'[{"id":2},{"id":3,"v":1}]', b'[]', b' [ {"v":2} ] ', b'[{"id":4},5]',
            b'[{"id":5}', b'{"id":6}', b'[{"id":7,"v":null},{"id":8,"v":"x"}]', b'[{"id":9}] x']
    dec, b, errs = decode(engine_mod, schema, msgs, paths=False)
    assert errs == {4: TYP, 5: SYN, 7: TYP, 8: SYN}, errs
    assert read_rows(dec, schema, b) == [(1, 0.5), (2, None), (3, 1.0), (None, 2.0), (6, None)]
    assert dec.rows_of().tolist() == [1, 2, 0, 1, 0, 0, 1, 0, 0]
    s = dec.stats()
    assert s.messages == len(msgs) and s.errors == 4
    dec.close()


# ---------------------------------------------------------------- random nested payloads vs a decodeObject restatement
class _Err(Exception):
    def __init__(self, code):
        super().__init__(code)
        self.code = code


class _Pairs(list):
    """A JSON object as its (key, value) pairs in document order (duplicates kept)."""


def _tree(schema):
    """Column paths -> a schema tree: dict (struct: key -> node), {"#": {index: node}} (array), or (column, type)."""
    root = {}
    for col, (name, t) in enumerate(schema.items()):
        node = root
        segs = _parse_path(name)
        for k, seg in enumerate(segs):
            last = k == len(segs) - 1
            if isinstance(seg, str):
                node = node.setdefault(seg, (col, t) if last else ({"#": {}} if isinstance(segs[k + 1], int) else {}))
            else:
                node = node["#"].setdefault(seg, (col, t) if last else ({"#": {}} if isinstance(segs[k + 1], int) else {}))
    return root


def _leaves(node):
    if isinstance(node, tuple):
        return [node[0]]
    kids = node["#"].values() if "#" in node else node.values()
    return [c for k in kids for c in _leaves(k)]


def go_walk(val, node, out):
    """decodeObject / decodeArray (converter.go:173-409) restated over the schema tree: every occurrence of a schema
    key is decoded (an error in any occurrence fails the message, Visit keeps going but the error stays), the last
    occurrence's subtree is the map's value (Go map assignment); array elements other than the indexed ones carry no
    schema (decoded unchecked). Leaves get their value in out[column]."""
    if isinstance(node, tuple):
        col, t = node
        out[col] = None if val is None else _leaf(val, t)
        return
    if val is None:
        for c in _leaves(node):
            out[c] = None
        return
    if "#" in node:
        if not isinstance(val, list) or isinstance(val, _Pairs):
            raise _Err(TYP)
        for ix, child in node["#"].items():
            if ix < len(val):
                go_walk(val[ix], child, out)
            else:
                for c in _leaves(child):
                    out[c] = None
        return
    if not isinstance(val, _Pairs):
        raise _Err(TYP)
    for key, child in node.items():
        for c in _leaves(child):
            out[c] = None
    for key, v in val:
        if key in node:
            for c in _leaves(node[key]):
                out[c] = None
            go_walk(v, node[key], out)


def _leaf(v, t):
    if t.startswith("array<"):
        if not isinstance(v, list) or isinstance(v, _Pairs):
            raise _Err(TYP)
        return [None if x is None else _scalar(x, t[6:-1]) for x in v]
    return _scalar(v, t)


def _scalar(v, t):
    if isinstance(v, list):   # (objects are _Pairs, a list too)
        raise _Err(TYP)
    if t == "bigint":
        if isinstance(v, float):
            raise _Err(NUM)   # fastfloat.ParseInt64 of a non-integer literal
        if isinstance(v, bool) or not isinstance(v, int):
            raise _Err(TYP)
        return v
    if t == "float":
        if isinstance(v, bool) or not isinstance(v, (int, float)):
            raise _Err(TYP)
        return float(v)
    if t == "boolean":
        if isinstance(v, bool):
            return v
        if isinstance(v, (int, float)):
            return v != 0
        s = {"1": True, "t": True, "T": True, "TRUE": True, "true": True, "True": True,
             "0": False, "f": False, "F": False, "FALSE": False, "false": False, "False": False}
        if isinstance(v, str) and v in s:
            return s[v]
        raise _Err(TYP)
    raise AssertionError(t)


def _parse_path(p):
    out = []
    for part in p.split("."):
        k = part.split("[")[0]
        if k:
            out.append(k)
        for ix in part.split("[")[1:]:
            out.append(int(ix.rstrip("]")))
    return out


def _rand_value(rng, depth):
    r = rng.random()
    if depth >= 3 or r < 0.45:
        c = rng.integers(0, 6)
        return [None, True, int(rng.integers(-50, 50)), float(rng.integers(-400, 400)) / 8, "t", 7][int(c)]
    if r < 0.75:
        keys = ["a", "b", "c", "x"]
        return {keys[int(rng.integers(0, 4))]: _rand_value(rng, depth + 1) for _ in range(int(rng.integers(0, 4)))}
    return [_rand_value(rng, depth + 1) for _ in range(int(rng.integers(0, 4)))]


def _guided(node, rng, depth=0):
    """A random value for a schema node: of the shape the schema wants with probability 0.9 (its leaves typed right
    with probability 0.95), else any value; objects get extra keys outside the schema, arrays extra elements."""
    if rng.random() < 0.1:
        return _rand_value(rng, depth)
    if isinstance(node, tuple):
        t = node[1]
        if rng.random() < 0.05:
            return _rand_value(rng, 3)
        if rng.random() < 0.1:
            return None
        if t.startswith("array<"):
            return [_guided((0, t[6:-1]), rng, depth + 1) if rng.random() < 0.97 else _rand_value(rng, 3)
                    for _ in range(int(rng.integers(0, 5)))]
        if t == "bigint":
            return int(rng.integers(-2**62, 2**62))
        if t == "float":
            return float(rng.standard_normal() * 1e3) if rng.random() < 0.7 else int(rng.integers(-99, 99))
        return [True, False, 0, 1, 2.5, "true", "F", "1"][int(rng.integers(0, 8))]
    if "#" in node:
        n = max(node["#"]) + int(rng.integers(-1, 3))
        return [_guided(node["#"][i], rng, depth + 1) if i in node["#"] else _rand_value(rng, depth + 1)
                for i in range(max(n, 0))]
    out = {}
    for k, child in node.items():
        if rng.random() < 0.8:
            out[k] = _guided(child, rng, depth + 1)
    if rng.random() < 0.3:
        out["z"] = _rand_value(rng, depth + 1)
    return out


def _dump(v, rng):
    """JSON text with random whitespace and, for objects, occasional duplicated keys."""
    ws = lambda: " " * int(rng.integers(0, 2))  # noqa: E731
    if isinstance(v, dict):
        parts = []
        for k, x in v.items():
            if rng.random() < 0.15:   # an earlier occurrence of the key
                parts.append(f'{ws()}"{k}"{ws()}:{ws()}{_dump(_rand_value(rng, 2), rng)}')
            parts.append(f'{ws()}"{k}"{ws()}:{ws()}{_dump(x, rng)}')
        return "{" + ",".join(parts) + ws() + "}"
    if isinstance(v, list):
        return "[" + ",".join(ws() + _dump(x, rng) for x in v) + ws() + "]"
    return json.dumps(v)


def test_random_nested_parity(engine_mod):
    schema = {"a.b": "float", "a.c": "bigint", "x[0]": "float", "x[1].b": "boolean", "b[0][1]": "bigint",
              "c": "array<float>", "a.x[2].c": "float", "a.a": "array<boolean>"}
    tree = _tree(schema)
    rng = np.random.default_rng(5)
    msgs, exp = [], []
    for _ in range(20000):
        doc = _guided(tree, rng)
        if not isinstance(doc, dict):
            doc = {"a": doc}
        txt = _dump(doc, rng)
        back = json.loads(txt, object_pairs_hook=_Pairs)
        out = [None] * len(schema)
        try:
            go_walk(back, tree, out)
            row = tuple(out)
        except _Err as e:
            row = e.code
        msgs.append(txt.encode())
        exp.append(row)
    dec, b, errs = decode(engine_mod, schema, msgs)
    exp_fail = {i: r for i, r in enumerate(exp) if not isinstance(r, tuple)}
    assert set(errs) == set(exp_fail), sorted(set(errs) ^ set(exp_fail))[:10]
    assert all(c in (TYP, NUM) for c in errs.values())
    got = read_rows(dec, schema, b)
    want = [r for r in exp if isinstance(r, tuple)]
    assert len(got) == len(want)
    bad = [(g, w) for g, w in zip(got, want) if g != w]
    assert not bad, bad[:5]
    assert 1000 < len(want) < 19000   # both outcomes are exercised
    dec.close()
