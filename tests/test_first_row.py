"""Non-aggregate select fields of an aggregate rule take the column's value in the group's FIRST row (row.go:720-726:
GroupedTuples.Value reads Content[0]; project_operator.go:136-207). The lowering turns such a field into the engine's
EK_AGG_FIRST; the oracle restates it as "row 0 of the group in window order". Pinned by the reference's own
ProjectOp cases project_test.go #11 / #12 (`SELECT id1 FROM src1 GROUP BY TUMBLINGWINDOW(ss, 10), f1`: the v1 group
[id1 1, id1 3] -> 1, the v2 group [id1 2] -> 2; a first row without id1 -> the field is absent, i.e. nil)."""
import numpy as np

from ekgpu import abi as A
from ekgpu.rule import compile_rule

SCHEMA = {"id1": "bigint", "f1": "key", "ts": "bigint"}
SQL = "SELECT id1 FROM src1 GROUP BY TUMBLINGWINDOW(ss, 10), f1"
T0 = 1541152480000


def kat_columns(case12: bool):
    # window [T0, T0 + 10 s): v1 rows id1 = 1 then 3, v2 row id1 = 2 (missing in case 12); a later row closes it
    id1 = np.array([1, 2, 3, 9], np.int64)
    f1 = np.array([0, 1, 0, 0], np.uint32)
    ts = np.array([T0 + 100, T0 + 200, T0 + 300, T0 + 10_000], np.int64)
    valid = [np.array([1, 0 if case12 else 1, 1, 1], np.uint8), None, None]
    return [id1, f1, ts], valid


def test_lowering_first_row_field():
    rule = compile_rule(SQL, SCHEMA, num_keys=2, nullable=("id1",))
    assert rule.plan.n_aggs == 1 and rule.plan.aggs[0].fn == A.EK_AGG_FIRST and rule.plan.aggs[0].column == 0
    assert [(f.name, f.kind, f.slot) for f in rule.fields] == [("id1", "agg", 0)]
    r2 = compile_rule("SELECT f1, temp, avg(temp) AS a FROM s GROUP BY f1, TUMBLINGWINDOW(ss, 1)",
                      {"f1": "key", "ts": "bigint", "temp": "float"}, num_keys=4)
    assert [f.kind for f in r2.fields] == ["key", "agg", "agg"]
    assert [r2.plan.aggs[k].fn for k in range(r2.plan.n_aggs)] == [A.EK_AGG_AVG, A.EK_AGG_FIRST]


def test_oracle_project_kat_first_row(oracle):
    for case12, expect in ((False, {0: ("i", 1), 1: ("i", 2)}), (True, {0: ("i", 1), 1: ("nil", None)})):
        cols, valid = kat_columns(case12)
        rule = compile_rule(SQL, SCHEMA, num_keys=2, nullable=("id1",))
        run = oracle.run(rule.plan, cols, valid)
        w = [w for w in run.windows if len(w.keys)]
        assert len(w) == 1
        got = {}
        for key, tag, val in zip(w[0].keys, w[0].tags[0], w[0].values[0]):
            got[int(key)] = ("nil", None) if tag == A.EK_TAG_NULL else ("i", int(val))
        assert got == expect


def test_first_row_string_field_lowering_and_oracle(oracle):
    """A first-row field over a string column carries the column's dictionary code; decode_value maps it back."""
    schema = {"k": "key", "ts": "bigint", "name": "string", "x": "float"}
    rule = compile_rule("SELECT k, name, max(x) FROM s GROUP BY k, TUMBLINGWINDOW(ss, 1)", schema, num_keys=3)
    assert rule.plan.aggs[1].fn == A.EK_AGG_FIRST
    names = ["b", "a", "c", "b", "z"]
    cols, _ = rule.device_columns([np.array([0, 1, 0, 1, 2], np.uint32),
                                   np.array([T0, T0 + 1, T0 + 2, T0 + 3, T0 + 1000], np.int64), names,
                                   np.array([1.0, 2.0, 3.0, 4.0, 5.0])])
    run = oracle.run(rule.plan, cols)
    w = [w for w in run.windows if len(w.keys)][0]
    got = dict(zip((int(k) for k in w.keys), rule.decode_value(1, w.values[1], w.tags[1])))
    assert got == {0: "b", 1: "a"}
