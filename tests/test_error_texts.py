"""The reference's window error texts on the CPU oracle (ek_window_error's parity target), pinned to the strings the
Go operators print for hand-checked inputs:

* FilterOp  "run Where error: %s" / "run Where error: invalid condition that returns non-bool value %T(%v)"
  (internal/topo/operator/filter_operator.go:60-81) over the window's rows in order, the first failure wins;
* HavingOp  "run Having error: ..." (having_operator.go:41-56); the reference ranges a Go map of groups
  (aggregate_operator.go:44-72), so any failed group's text is one it can print: the oracle (and the engine) take the
  failed group with the smallest key;
* ProjectOp "run Select error: %s" (project_operator.go:79-102) with funcs_agg.go's percentile texts;
* valuer.go: "divided by zero" (:897-979), invalidOpError "invalid operation %T(%v) %s %T(%v)" (:1243-1245), and
  Go's %v of float64 (strconv 'g', shortest: 37.5, 1.234567e+06, 1e-05).

Expected strings are written out by hand from those Go sources (no Go toolchain here: parity of the float
formatting is pinned to Go's documented strconv rules, not to a run of the reference)."""
import numpy as np
import pytest

from ekgpu.rule import compile_rule

SCHEMA = {"ts": "bigint", "size": "bigint", "color": "key", "temp": "float"}
#         ts     size color temp
ROWS = [(1000, 5, 1, 25.0),
        (1100, 0, 0, 1.234567),
        (1200, 2, 1, 0.00001),
        (2000, 1, 2, 4.0),
        (2500, 3, 2, 2.5),
        (2600, 4, 3, 8.0),
        (3500, 1, 0, 1.0)]


def _cols():
    r = np.array(ROWS, dtype=object)
    return [np.array(r[:, 0], np.int64), np.array(r[:, 1], np.int64), np.array(r[:, 2], np.uint32),
            np.array(r[:, 3], np.float64)]


CASES = [
    ("where_div0", "SELECT count(*) FROM demo WHERE 10 / size > 1 GROUP BY color, TUMBLINGWINDOW(ss, 1)",
     ["run Where error: divided by zero", ""]),
    ("where_nonbool_float", "SELECT count(*) FROM demo WHERE temp * 1.5 GROUP BY color, TUMBLINGWINDOW(ss, 1)",
     ["run Where error: invalid condition that returns non-bool value float64(37.5)",
      "run Where error: invalid condition that returns non-bool value float64(6)"]),
    ("where_float_exp", "SELECT count(*) FROM demo WHERE temp * 1000000.0 > size AND temp * 1000000.0 "
                        "GROUP BY color, TUMBLINGWINDOW(ss, 1)",
     ["run Where error: invalid operation bool(true) AND float64(2.5e+07)",
      "run Where error: invalid operation bool(true) AND float64(4e+06)"]),
    ("where_bool_plus_int", "SELECT count(*) FROM demo WHERE (size > 1) + 2 > 1 GROUP BY color, TUMBLINGWINDOW(ss, 1)",
     ["run Where error: invalid operation bool(true) + int64(2)",
      "run Where error: invalid operation bool(false) + int64(2)"]),
    ("where_int_and", "SELECT count(*) FROM demo WHERE size AND size > 1 GROUP BY color, TUMBLINGWINDOW(ss, 1)",
     ["run Where error: invalid operation int64(5) AND bool(true)",
      "run Where error: invalid operation int64(1) AND bool(false)"]),
    ("having_nonbool", "SELECT count(*) FROM demo GROUP BY color, TUMBLINGWINDOW(ss, 1) HAVING sum(size)",
     ["run Having error: invalid condition that returns non-bool value int64(0)",
      "run Having error: invalid condition that returns non-bool value int64(4)"]),
    ("having_div0", "SELECT count(*) FROM demo GROUP BY color, TUMBLINGWINDOW(ss, 1) "
                    "HAVING sum(size) / (count(*) - 1) > 2",
     ["run Having error: divided by zero", "run Having error: divided by zero"]),
    ("having_float_plus_bool", "SELECT count(*) FROM demo GROUP BY color, TUMBLINGWINDOW(ss, 1) "
                               "HAVING avg(temp) + (count(*) > 1) > 0",
     ["run Having error: invalid operation float64(1.234567) + bool(false)",
      "run Having error: invalid operation float64(3.25) + bool(true)"]),
    ("select_percentile", "SELECT percentile_cont(temp, 1.5) FROM demo GROUP BY color, TUMBLINGWINDOW(ss, 1)",
     ["run Select error: percentile exec with error: Input is outside of range.",
      "run Select error: percentile exec with error: Input is outside of range."]),
    ("having_reads_percentile", "SELECT count(*) FROM demo GROUP BY color, TUMBLINGWINDOW(ss, 1) "
                                "HAVING percentile_disc(temp, 1.5) > 1",
     ["run Having error: PopulationVariance exec with error: Input is outside of range.",
      "run Having error: PopulationVariance exec with error: Input is outside of range."]),
]


@pytest.mark.parametrize("name,sql,texts", CASES, ids=[c[0] for c in CASES])
def test_oracle_window_error_texts(oracle, name, sql, texts):
    rule = compile_rule(sql, SCHEMA, num_keys=4)
    run = oracle.run(rule.plan, _cols())
    got = {w.end: e for w, e in zip(run.windows, run.errors) if w.end > w.start}   # the windows [1000, 2000), [2000, 3000)
    assert got == dict(zip((2000, 3000), texts))
    for w, e in zip(run.windows, run.errors):
        assert (w.status != 0) == bool(e)
