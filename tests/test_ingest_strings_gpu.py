"""GPU tests of STRING and BOOLEAN fields in the columnar JSON ingest (ek_json_*) and of BOOLEAN columns in the engine.

* converter cases: the string / boolean rows of TestFastJsonConverterWithSchema and TestFastJsonConverterWithSchemaError
  (internal/converter/json/converter_test.go:90-122,217-252) plus getBooleanFromValue's conversions
  (converter.go:600-625 over pkg/cast/cast.go:809-837: a number is != 0, a string goes through strconv.ParseBool) and
  the JSON string escapes (valyala/fastjson v1.6.4 unescapeStringBestEffort; hand-derived, parity unpinned by a
  reference fixture).
* a C2-shaped rule whose deviceId is a JSON string, decoded from raw payloads (host and device memory), against the
  oracle run on the same rows with the host dictionary (ekgpu.keys.StringDict) giving the ids: the decoder's ids are
  first-seen ids too, so keys, values and the id -> string tables are identical.
* BOOLEAN columns in WHERE (bare, = true, AND), count(bool), SELECT * (Go bool values) and the evaluation error texts
  of a bool against a number, against the oracle.
"""
import json

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.keys import StringDict
from ekgpu.rule import compile_rule
from ekgpu.synth import iot_stream
from parity import assert_windows_equal
from test_engine_gpu import engine_mod  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu

STR_SCHEMA = {"deviceId": "string", "ts": "bigint", "temperature": "float", "humidity": "float"}


def _read_back(engine_mod, dec, schema, batch):
    """The decoded rows through SELECT * (the product path) as python values; string ids -> the decoder's strings."""
    rule = compile_rule("SELECT * FROM s", dec.rule_schema(), is_event_time=False, nullable=tuple(schema))
    eng = engine_mod.Engine(rule.plan)
    eng.push_batch(batch)
    w = eng.poll()[0]
    eng.close()
    names = list(schema)
    tables = {c: dec.strings(c) for c, t in enumerate(schema.values()) if t == "string"}
    rows = []
    for r in range(len(w.keys)):
        row = []
        for c in range(len(names)):
            v = w.value(c, r)
            row.append(tables[c][v] if (c in tables and v is not None) else v)
        rows.append(tuple(row))
    return rows


CONVERTER_CASES = [
    # (schema type, payload, expected value | error code)
    ("string", b'{"a":"a"}', "a"),                                   # converter_test.go:90-100
    ("boolean", b'{"a":true}', True),                                # converter_test.go:112-122
    ("string", b'{"a":{"b":1}}', A.EK_JSON_ERR_TYPE),                # :217-225 "a has wrong type:object, expect:string"
    ("boolean", b'{"a":{"b":1}}', A.EK_JSON_ERR_TYPE),               # :244-252 "... expect:boolean"
    ("boolean", b'{"a":false}', False),
    ("boolean", b'{"a":"true"}', True),                              # strconv.ParseBool
    ("boolean", b'{"a":"F"}', False),
    ("boolean", b'{"a":"1"}', True),
    ("boolean", b'{"a":"yes"}', A.EK_JSON_ERR_TYPE),                 # ParseBool: invalid syntax
    ("boolean", b'{"a":"tRUE"}', A.EK_JSON_ERR_TYPE),
    ("boolean", b'{"a":1.5}', True),                                 # cast.ToBool(float64): != 0
    ("boolean", b'{"a":0}', False),
    ("boolean", b'{"a":-0.0}', False),
    ("boolean", b'{"a":[true]}', A.EK_JSON_ERR_TYPE),
    ("boolean", b'{"a":null}', None),
    ("string", b'{"a":true}', A.EK_JSON_ERR_TYPE),                   # extractBooleanFromValue: wrong type
    ("string", b'{"a":12}', "12"),                                    # cast.ToStringAlways(float64): %v (ABI v14)
    ("string", b'{"a":[1]}', A.EK_JSON_ERR_TYPE),
    ("string", b'{"a":null}', None),
    ("string", b'{}', None),
    ("string", b'{"a":""}', ""),
    ("string", b'{"a":"x\\"y\\\\z"}', 'x"y\\z'),
    ("string", b'{"a":"\\u00e9t\\u00e9\\n"}', "\u00e9t\u00e9\n"),
    ("string", b'{"a":"\\ud83d\\ude00!"}', "\U0001F600!"),           # a surrogate pair is one rune
    ("string", b'{"a":"\\ud83d\\u0041"}', "\ufffd"),                 # utf16.DecodeRune of a bad pair
    ("string", b'{"a":"\\ud83dxy"}', "\\ud83dxy"),                   # an unpaired surrogate stays escaped
    ("string", b'{"a":"\\q\\/"}', "\\q/"),                           # an unknown escape is kept
    ("string", b'{"a":"a"}', "a"),                                   # a repeat: the same id
    ("string", b'{"a":"\\u0061"}', "a"),                             # escaped spelling of a known string
    ("string", b'{"a":"caf\xc3\xa9"}', "caf\u00e9"),                 # raw UTF-8
]


@pytest.mark.parametrize("typ", ["string", "boolean"])
def test_converter_string_bool_cases(engine_mod, typ):
    cases = [c for c in CONVERTER_CASES if c[0] == typ]
    schema = {"a": typ}
    dec = engine_mod.JsonDecoder(schema)
    batch = dec.decode([c[1] for c in cases])
    idx, code = dec.errors()
    exp_err = [(i, c[2]) for i, c in enumerate(cases) if isinstance(c[2], int) and not isinstance(c[2], bool)]
    assert list(zip(idx.tolist(), code.tolist())) == exp_err
    ok = [(c[2],) for c in cases if not (isinstance(c[2], int) and not isinstance(c[2], bool))]
    rows = _read_back(engine_mod, dec, schema, batch)
    assert rows == ok
    assert all(type(g) is type(e) for r, x in zip(rows, ok) for g, e in zip(r, x))   # Go bool / string, not ints
    if typ == "string":
        strs = dec.strings("a")
        assert len(strs) == len(set(strs))                    # one id per distinct string (escaped spellings merge)
        assert strs[0] == "a"                                  # first-seen order
    dec.close()


def _str_msgs(key, ts, temp, hum, rng):
    names = [f"dev-{k:04d}" for k in range(int(key.max()) + 1)]
    msgs = []
    for k, t, a, b in zip(key.tolist(), ts.tolist(), temp.tolist(), hum.tolist()):
        s = json.dumps(names[k])
        if rng.random() < 0.01:   # the same string spelled with an escape: must land on the same id
            s = s.replace("-", "\\u002d")
        msgs.append(f'{{"deviceId":{s},"ts":{t},"temperature":{a!r},"humidity":{b!r}}}'.encode())
    return names, msgs


@pytest.mark.parametrize("memory", ["host", "device"])
def test_json_string_key_c2_shape(oracle, engine_mod, memory):
    """C2-shaped rule (GROUP BY deviceId, TUMBLINGWINDOW) with deviceId a JSON string, from raw payloads."""
    import torch
    key, ts, temp, hum = iot_stream(200_000, 1000, seed=21, events_per_ms=10)
    rng = np.random.default_rng(21)
    names, msgs = _str_msgs(key, ts, temp, hum, rng)
    dec = engine_mod.JsonDecoder(STR_SCHEMA)
    assert dec.rule_schema() == dict(STR_SCHEMA, deviceId="key")   # the ids are the engine's dense key column
    rule = compile_rule("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
                        "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)", dec.rule_schema(), num_keys=1000,
                        debug_membership=True)
    eng = engine_mod.Engine(rule.plan)
    step = 50_000
    keep = []
    for lo in range(0, len(msgs), step):
        part = msgs[lo:lo + step]
        if memory == "host":
            eng.push_batch(dec.decode(part))
            continue
        lens = np.fromiter((len(m) for m in part), np.int64, len(part))
        offs = np.zeros(len(part) + 1, np.int64)
        np.cumsum(lens, out=offs[1:])
        d_blob = torch.frombuffer(bytearray(b"".join(part)), dtype=torch.uint8).cuda()
        d_offs = torch.from_numpy(offs).cuda()
        torch.cuda.synchronize()
        keep.append((d_blob, d_offs))
        eng.push_batch(dec.decode_device(d_blob.data_ptr(), int(offs[-1]), d_offs.data_ptr(), len(part)))
    got = eng.poll()
    eng.close()
    # the oracle over the python-decoded rows, ids from the host dictionary (first-seen order, as the decoder's)
    sd = StringDict()
    dev = [json.loads(m)["deviceId"] for m in msgs]
    ids = sd.encode(np.array(dev, dtype=object))
    assert dec.strings("deviceId") == sd.values
    assert sorted(sd.values) == sorted(names[k] for k in set(key.tolist()))
    dec.close()
    exp = oracle.run(rule.plan, [ids, ts, temp, hum]).windows
    assert len(got) >= 1
    assert_windows_equal(rule.plan, got, exp, check_members=True)


BOOL_SCHEMA = {"ts": "bigint", "ok": "boolean", "v": "float"}


def _bool_rows(n, seed):
    rng = np.random.default_rng(seed)
    ts = 1541152480000 + np.sort(rng.integers(0, 60_000, n)).astype(np.int64)
    ok = rng.integers(0, 2, n).astype(np.int64)
    v = np.round(rng.uniform(0, 100, n), 2)
    return ts, ok, v


@pytest.mark.parametrize("where", ["ok", "ok = true", "ok != false AND v > 50", "NOT_ok_or_v", "ok = 1"])
def test_bool_where_parity(oracle, engine_mod, where):
    ts, ok, v = _bool_rows(20_000, 5)
    sql_where = "v < 10 OR ok = false" if where == "NOT_ok_or_v" else where
    rule = compile_rule(f"SELECT count(*), avg(v), count(ok) FROM demo WHERE {sql_where} "
                        "GROUP BY TUMBLINGWINDOW(ss, 10)", BOOL_SCHEMA, late_tolerance_ms=0)
    msgs = [f'{{"ts":{t},"ok":{"true" if o else "false"},"v":{x!r}}}'.encode()
            for t, o, x in zip(ts.tolist(), ok.tolist(), v.tolist())]
    dec = engine_mod.JsonDecoder(BOOL_SCHEMA)
    eng = engine_mod.Engine(rule.plan)
    eng.push_batch(dec.decode(msgs))
    got = eng.poll()
    eng.close()
    dec.close()
    run = oracle.run(rule.plan, [ts, ok, v])
    assert_windows_equal(rule.plan, got, run.windows)
    assert [w.error for w in got] == [run.errors[k] or "" for k in range(len(got))]
    if where == "ok = 1":   # bool = int64: "invalid operation bool(true) = int64(1)" (valuer.go:1243-1245)
        assert got and all(w.status == A.EK_WIN_WHERE_ERROR for w in got)
        assert all(w.error.startswith("run Where error: invalid operation bool(") for w in got)


def test_bool_select_star_and_refusals(oracle, engine_mod):
    ts, ok, v = _bool_rows(1000, 6)
    rule = compile_rule("SELECT * FROM demo WHERE ok", BOOL_SCHEMA, is_event_time=False)
    eng = engine_mod.Engine(rule.plan)
    eng.push_host([ts, ok, v])
    w = eng.poll()[0]
    eng.close()
    exp = oracle.run(rule.plan, [ts, ok, v]).windows[0]
    assert len(w.keys) == int(ok.sum()) == len(exp.keys)
    assert all(w.value(1, r) is True for r in range(len(w.keys)))
    assert [w.value(0, r) for r in range(len(w.keys))] == [exp.value(0, r) for r in range(len(exp.keys))]
    assert [exp.value(1, r) for r in range(len(exp.keys))] == [True] * len(exp.keys)
    for sql in ("SELECT sum(ok) FROM demo GROUP BY TUMBLINGWINDOW(ss, 10)",
                "SELECT max(ok) FROM demo GROUP BY TUMBLINGWINDOW(ss, 10)"):
        with pytest.raises(engine_mod.EngineError, match="BOOLEAN"):
            engine_mod.Engine(compile_rule(sql, BOOL_SCHEMA).plan)
