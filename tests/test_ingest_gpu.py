"""GPU tests of the columnar JSON ingest (ek_json_*) and the window-less FilterOp path (C1).

* C1 known-answer test: test/iot_data.txt sent as the reference's JMeter payload
  {"temperature": T, "humidity" : H} (test/select_condition_rule.jmx:134,174,275), decoded on the GPU,
  filtered by SELECT * FROM demo WHERE temperature > 30 -> test/select_condition_iot_data.txt.
* number conversion: FLOAT fields are bit-identical to Python's correctly rounded float(), BIGINT fields
  follow fastfloat.ParseInt64; error classes of converter.go (syntax / wrong type / number).
* JSON -> windowed GROUP BY end to end against the oracle run on the original columns.
"""
import json
import os
import struct

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule
from ekgpu.synth import IOT_SCHEMA, iot_stream
from parity import assert_windows_equal, assert_windows_equal_np
from test_engine_gpu import engine_mod  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
C1_SCHEMA = {"temperature": "float", "humidity": "bigint"}   # select_condition_rule.jmx:134


def _bits(x: float) -> int:
    return struct.unpack("<q", struct.pack("<d", x))[0]


def _decode_cols(engine_mod, schema, msgs):
    dec = engine_mod.JsonDecoder(schema)
    b = dec.decode(msgs)
    return dec, b


def test_c1_kat_json_filter(oracle, engine_mod):
    rows = np.loadtxt(os.path.join(GOLD, "iot_data.txt"), delimiter=",", dtype=np.int64, ndmin=2)
    exp = np.loadtxt(os.path.join(GOLD, "select_condition_iot_data.txt"), delimiter=",", dtype=np.int64, ndmin=2)
    msgs = [f'{{"temperature": {t}, "humidity" : {h}}}'.encode() for _, t, h in rows]
    dec, batch = _decode_cols(engine_mod, C1_SCHEMA, msgs)
    assert batch.n_rows == len(rows)
    rule = compile_rule("SELECT * FROM demo WHERE temperature > 30", C1_SCHEMA, is_event_time=False)
    eng = engine_mod.Engine(rule.plan)
    eng.push_batch(batch)
    got = eng.poll()
    eng.close()
    dec.close()
    assert len(got) == 1
    w = got[0]
    out = [(w.value(0, r), w.value(1, r)) for r in range(len(w.keys))]
    assert out == [(float(t), int(h)) for _, t, h in exp]
    assert all(isinstance(t, float) and isinstance(h, int) for t, h in out)


def test_c1_synthetic_filter_parity(oracle, engine_mod):
    """C1 shape: 1e6 payloads {"temperature":T,"humidity":H}, T,H uniform integers in [0, 100]."""
    n = 1_000_000
    rng = np.random.default_rng(11)
    t = rng.integers(0, 101, n)
    h = rng.integers(0, 101, n)
    msgs = [f'{{"temperature":{a},"humidity":{b}}}'.encode() for a, b in zip(t.tolist(), h.tolist())]
    dec, batch = _decode_cols(engine_mod, C1_SCHEMA, msgs)
    rule = compile_rule("SELECT * FROM demo WHERE temperature > 50", C1_SCHEMA, is_event_time=False)
    eng = engine_mod.Engine(rule.plan)
    eng.push_batch(batch)
    got = eng.poll()
    eng.close()
    exp = oracle.run(rule.plan, [t.astype(np.float64), h.astype(np.int64)]).windows
    assert_windows_equal(rule.plan, got, exp)
    assert len(got[0].keys) == int((t > 50).sum())


def _num_cases(rng, k):
    out = []
    for _ in range(k):
        kind = rng.integers(0, 6)
        if kind == 0:
            s = str(int(rng.integers(-10**6, 10**6)))
        elif kind == 1:
            s = f"{rng.uniform(-1e3, 1e3):.{int(rng.integers(1, 17))}f}"
        elif kind == 2:
            s = f"{rng.uniform(1, 10):.{int(rng.integers(1, 17))}f}e{int(rng.integers(-300, 300))}"
        elif kind == 3:    # long mantissas (> 19 significant digits)
            s = "".join(str(d) for d in rng.integers(0, 10, int(rng.integers(20, 40))))
            s = s.lstrip("0") or "0"
            s = s[: int(rng.integers(1, len(s)))] + "." + s[len(s) // 2:] if len(s) > 2 else s
        elif kind == 4:
            s = repr(float(rng.standard_normal() * 10 ** int(rng.integers(-20, 20))))
            s = s.replace("e+", "e")
        else:
            s = f"{int(rng.integers(0, 2**53))}e{int(rng.integers(-30, 30))}"
        if rng.random() < 0.2 and not s.startswith("-"):
            s = "-" + s
        out.append(s)
    return out


def test_json_float_conversion_exact(engine_mod):
    rng = np.random.default_rng(12)
    nums = _num_cases(rng, 20000)
    nums = [s for s in nums if abs(float(s)) < 1.7e308]   # (subnormal results decode too: ABI v14)
    msgs = [f'{{"x": {s}}}'.encode() for s in nums]
    dec, batch = _decode_cols(engine_mod, {"x": "float"}, msgs)
    assert batch.n_rows == len(msgs), dec.errors()
    _, w = _read_back(engine_mod, {"x": "float"}, batch)
    got = w.values[0]
    exp = np.array([_bits(float(s)) for s in nums], dtype=np.int64)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(nums[i], got[i], exp[i]) for i in bad[:5]]
    dec.close()


def _read_back(engine_mod, schema, batch):
    """The decoded rows through a SELECT * rule without WHERE (the product path), as python values."""
    rule = compile_rule("SELECT * FROM s", schema, is_event_time=False, nullable=tuple(schema))
    eng = engine_mod.Engine(rule.plan)
    eng.push_batch(batch)
    w = eng.poll()[0]
    eng.close()
    assert len(w.keys) == batch.n_rows and (w.keys == np.arange(batch.n_rows)).all()
    return [tuple(w.value(c, r) for c in range(len(schema))) for r in range(len(w.keys))], w


def test_json_fields_nulls_and_errors(engine_mod):
    schema = {"id": "key", "ts": "bigint", "v": "float"}
    cases = [
        (b'{"id": 3, "ts": 1541152480000, "v": 1.5}', A.EK_JSON_OK, (3, 1541152480000, 1.5)),
        (b' { "v" : -0.25 ,"ts":7 , "id":0 } ', A.EK_JSON_OK, (0, 7, -0.25)),
        (b'{"id": 1, "ts": 2, "v": null}', A.EK_JSON_OK, (1, 2, None)),
        (b'{"id": 1, "v": 2}', A.EK_JSON_OK, (1, None, 2.0)),                       # absent ts -> nil
        (b'{"id": 1, "ts": 5, "v": 2, "extra": {"a": [1, "x}"], "b": "q\\"}"}, "s": "t"}', A.EK_JSON_OK, (1, 5, 2.0)),
        (b'{"id": 1, "ts": 5, "ts": 6, "v": 0}', A.EK_JSON_OK, (1, 6, 0.0)),       # last duplicate wins
        (b'{"id": 1, "ts": 12.5, "v": 0}', A.EK_JSON_ERR_NUMBER, None),              # float for BIGINT
        (b'{"id": 1, "ts": 99999999999999999999, "v": 0}', A.EK_JSON_ERR_NUMBER, None),
        (b'{"id": -1, "ts": 1, "v": 0}', A.EK_JSON_ERR_NUMBER, None),                # negative key id
        (b'{"id": 1, "ts": "5", "v": 0}', A.EK_JSON_ERR_TYPE, None),                 # string for a number
        (b'{"id": 1, "ts": 5, "v": true}', A.EK_JSON_ERR_TYPE, None),
        (b'{"id": 1, "ts": 5, "v": [1]}', A.EK_JSON_ERR_TYPE, None),
        (b'{"id": 1, "ts": 5, "v": 1.}', A.EK_JSON_ERR_SYNTAX, None),
        (b'{"id": 1, "ts": 5 "v": 1}', A.EK_JSON_ERR_SYNTAX, None),
        (b'{"id": 1, "ts": 5, "v": 1} x', A.EK_JSON_ERR_SYNTAX, None),
        (b'[{"id": 1}]', A.EK_JSON_OK, (1, None, None)),                             # top-level array: one row per object
        (b'{"id": 1, "ts": 5,}', A.EK_JSON_ERR_SYNTAX, None),                      # trailing comma
        (b'{"id": 2, "e": {"a": [1, "x}"], "b": "q\\"}"}, "ts": 4}', A.EK_JSON_OK, (2, 4, None)),
        (b'{"id": 7, "ts": -3, "v": 1e2}', A.EK_JSON_OK, (7, -3, 100.0)),
        (b'{}', A.EK_JSON_OK, (None, None, None)),
    ]
    dec, batch = _decode_cols(engine_mod, schema, [c[0] for c in cases])
    idx, code = dec.errors()
    exp_err = [(i, c[1]) for i, c in enumerate(cases) if c[1] != A.EK_JSON_OK]
    assert list(zip(idx.tolist(), code.tolist())) == exp_err
    ok = [c[2] for c in cases if c[1] == A.EK_JSON_OK]
    assert batch.n_rows == len(ok)
    rows, _ = _read_back(engine_mod, schema, batch)
    assert rows == ok
    assert all(type(g) is type(e) for r, x in zip(rows, ok) for g, e in zip(r, x))
    s = dec.stats()
    assert s.messages == len(cases) and s.errors == len(exp_err)
    dec.close()


def test_json_to_tumbling_group_by(oracle, engine_mod):
    """JSON payloads -> GPU decode -> C2-shaped windowed GROUP BY, against the oracle on the same columns."""
    key, ts, temp, hum = iot_stream(200_000, 1000, seed=13, events_per_ms=10)
    msgs = [json.dumps({"deviceId": int(k), "ts": int(t), "temperature": float(a), "humidity": float(b)}).encode()
            for k, t, a, b in zip(key, ts, temp, hum)]
    rule = compile_rule("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
                        "GROUP BY deviceId, TUMBLINGWINDOW(ss, 10)", IOT_SCHEMA, num_keys=1000, debug_membership=True)
    dec = engine_mod.JsonDecoder(IOT_SCHEMA)
    eng = engine_mod.Engine(rule.plan)
    for lo in range(0, len(msgs), 50_000):
        eng.push_batch(dec.decode(msgs[lo:lo + 50_000]))
    got = eng.poll()
    eng.close()
    dec.close()
    exp = oracle.run(rule.plan, [key, ts, temp, hum]).windows
    assert len(got) >= 1
    assert_windows_equal(rule.plan, got, exp, check_members=True)


def test_c1_schemaless_json_filter(oracle, engine_mod):
    """C1 as SURVEY.md §8(d) states it: a schemaless stream, 1e6 payloads {"temperature":T,"humidity":H} with integer
    T, H in [0, 100]: every number decodes as float64 (converter.go:507-520), SELECT * ... WHERE temperature > 50."""
    n = 1_000_000
    rng = np.random.default_rng(12)
    t = rng.integers(0, 101, n)
    h = rng.integers(0, 101, n)
    msgs = [f'{{"temperature":{a},"humidity":{b}}}'.encode() for a, b in zip(t.tolist(), h.tolist())]
    dec = engine_mod.JsonDecoder.schemaless(["temperature", "humidity"])
    batch = dec.decode(msgs)
    assert batch.n_rows == n
    schema = {"temperature": "float", "humidity": "float"}
    rule = compile_rule("SELECT * FROM demo WHERE temperature > 50", schema, is_event_time=False)
    exp = oracle.run(rule.plan, [t.astype(np.float64), h.astype(np.float64)])
    eng = engine_mod.Engine(rule.plan)
    eng.push_batch(batch)
    got = eng.poll()
    eng.close()
    dec.close()
    assert_windows_equal_np(rule.plan, got, exp.windows)
    w = got[0]
    assert len(w.keys) == int((t > 50).sum()) and set(np.unique(w.tags[1])) == {A.EK_TAG_F64}
