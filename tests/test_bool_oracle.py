"""BOOLEAN columns and the literals true / false (ast.BooleanLiteral) in the plan ISA: compilation and the CPU oracle.

A Go bool compares with a bool by = / != only and is an AND / OR operand; against a number every operator is
invalidOpError "invalid operation bool(true) > int64(1)" (pkg/ast valuer.go SimpleDataEval, :1243-1245). A bare bool
column is a WHERE condition (filter_operator.go:63-77: true keeps the row)."""
import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import RuleError, compile_rule

SCHEMA = {"ts": "bigint", "ok": "boolean", "v": "float"}
T0 = 1541152480000


def _rows():
    ts = np.array([T0, T0 + 1, T0 + 2, T0 + 3, T0 + 30_000], np.int64)
    ok = np.array([1, 0, 1, 1, 0], np.int64)
    v = np.array([5.0, 60.0, 70.0, 20.0, 0.0])
    return [ts, ok, v]


def test_literals_compile_to_const_bool():
    rule = compile_rule("SELECT count(*) FROM demo WHERE ok = true OR false GROUP BY TUMBLINGWINDOW(ss, 10)", SCHEMA)
    prog = [(rule.plan.where_prog[k].op, rule.plan.where_prog[k].i64) for k in range(rule.plan.n_where)]
    assert prog == [(A.EK_OP_COL, 0), (A.EK_OP_CONST_BOOL, 1), (A.EK_OP_EQ, 0), (A.EK_OP_CONST_BOOL, 0), (A.EK_OP_OR, 0)]
    assert rule.plan.column_type[1] == A.EK_COL_BOOL
    with pytest.raises(RuleError, match="numeric"):
        compile_rule("SELECT sum(ok + 1) FROM demo GROUP BY TUMBLINGWINDOW(ss, 10)", SCHEMA)


@pytest.mark.parametrize("where,count", [("ok", 3), ("ok = true", 3), ("ok = false", 1), ("ok != true AND v > 50", 1),
                                         ("ok AND v > 50", 1), ("NOT_USED", 4)])
def test_bool_where(oracle, where, count):
    sql = "SELECT count(*), count(ok) FROM demo " + ("" if where == "NOT_USED" else f"WHERE {where} ") + \
          "GROUP BY TUMBLINGWINDOW(ss, 10)"
    run = oracle.run(compile_rule(sql, SCHEMA).plan, _rows())
    w = run.windows[0]
    assert w.status == A.EK_WIN_OK and w.value(0, 0) == count and w.value(1, 0) == count


def test_bool_number_mix_is_an_error(oracle):
    run = oracle.run(compile_rule("SELECT count(*) FROM demo WHERE ok > 1 GROUP BY TUMBLINGWINDOW(ss, 10)",
                                  SCHEMA).plan, _rows())
    assert run.windows[0].status == A.EK_WIN_WHERE_ERROR
    assert run.errors[0] == "run Where error: invalid operation bool(true) > int64(1)"


def test_select_star_yields_go_bools(oracle):
    rule = compile_rule("SELECT * FROM demo WHERE v > 10", SCHEMA, is_event_time=False)
    w = oracle.run(rule.plan, _rows()).windows[0]
    assert [w.value(1, r) for r in range(len(w.keys))] == [False, True, True]
    assert {int(t) for t in w.tags[1]} == {A.EK_TAG_BOOL}
