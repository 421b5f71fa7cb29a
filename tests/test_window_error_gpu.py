"""ek_window_error on the GPU: the error text of every failed window equals the oracle's (tests/test_error_texts.py pins
the oracle's texts to the Go operators' strings). Covers the paths that record a witness: pane mode (k_part /
k_ung_tile -> pane witness -> k_finalize), range mode (k_part over virtual panes -> k_agg), the small-window kernel
(k_small_win, WHERE and HAVING), the key-major walks (HAVING over count(*) alone, order statistics) and
the order-statistic Select error."""
import os
import re
import zlib

import numpy as np
import pytest

from ekgpu import abi as A
from ekgpu.rule import compile_rule
from parity import REL_TOL
from test_engine_gpu import engine_mod, run_both  # noqa: F401  (fixture + helper)
from test_error_texts import CASES, SCHEMA, _cols

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["pane", "range"])
def mode(request):
    if request.param == "range":
        os.environ["EKGPU_FORCE_RANGE"] = "1"
    yield request.param
    os.environ.pop("EKGPU_FORCE_RANGE", None)


_F64 = re.compile(r"float64\(([^)]*)\)")


def _text_equal(a, b):
    """Equal texts, except that a float64(...) value computed from an f64 aggregate may differ within the north-star
    tolerance (parity.REL_TOL: the engine folds f64 sums in pane / partition order, the reference sequentially)."""
    if _F64.sub("float64(x)", a) != _F64.sub("float64(x)", b):
        return False
    for x, y in zip(_F64.findall(a), _F64.findall(b)):
        fx, fy = float(x.replace("+Inf", "inf")), float(y.replace("+Inf", "inf"))
        if not (fx == fy or abs(fx - fy) <= REL_TOL * max(abs(fx), abs(fy))):
            return False
    return True


def _assert_errors(got, exp):
    assert len(got) == len(exp.windows)
    for w, (g, e, t) in enumerate(zip(got, exp.windows, exp.errors)):
        assert g.status == e.status, f"window {w}: status {g.status} != {e.status}"
        assert _text_equal(g.error, t), f"window {w} [{e.start}, {e.end}): {g.error!r} != {t!r}"


@pytest.mark.parametrize("name,sql,texts", CASES, ids=[c[0] for c in CASES])
def test_window_error_texts_kat(oracle, engine_mod, mode, name, sql, texts):
    rule = compile_rule(sql, SCHEMA, num_keys=4)
    cols = _cols()
    for batches in (1, len(cols[0])):
        got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=batches)
        _assert_errors(got, exp)


def _stream(n, keys, seed):
    rng = np.random.default_rng(seed)
    ts = (1541152480000 + np.sort(rng.integers(0, n // 4, n))).astype(np.int64)
    size = rng.integers(0, 40, n).astype(np.int64)          # zero in 1 row of 40
    color = rng.integers(0, keys, n).astype(np.uint32)
    temp = rng.normal(20.0, 7.0, n)
    return [ts, size, color, temp]


BIG = [
    ("tumbling_where_nonbool", "SELECT count(*) FROM demo WHERE temp * 1.5 GROUP BY color, TUMBLINGWINDOW(ss, 1)"),
    ("hopping_where_div0", "SELECT count(*), avg(temp) FROM demo WHERE 1000 / size > 30 GROUP BY color, "
                           "HOPPINGWINDOW(ss, 2, 1)"),
    ("ungrouped_where_nonbool", "SELECT count(*), sum(size) FROM demo WHERE size + 0 GROUP BY TUMBLINGWINDOW(ss, 1)"),
    ("sliding_small_where", "SELECT count(*) FROM demo WHERE 1000 / size > 30 GROUP BY color, SLIDINGWINDOW(ms, 40)"),
    ("sliding_small_nonbool", "SELECT count(*) FROM demo WHERE temp * 2.0 GROUP BY color, SLIDINGWINDOW(ms, 40)"),
    ("sliding_having_nonbool", "SELECT count(*) FROM demo GROUP BY color, SLIDINGWINDOW(ms, 40) HAVING sum(size)"),
    ("sliding_having_star_div0", "SELECT count(*) FROM demo GROUP BY color, SLIDINGWINDOW(ms, 40) "
                                 "HAVING 10 / (count(*) - 1) > 1"),
    ("tumbling_having_type", "SELECT count(*) FROM demo GROUP BY color, TUMBLINGWINDOW(ss, 1) "
                             "HAVING avg(temp) + (count(*) > 30) > 0"),
    ("tumbling_percentile", "SELECT percentile_cont(temp, 1.5), count(*) FROM demo GROUP BY color, TUMBLINGWINDOW(ss, 1)"),
    ("sliding_large_having", "SELECT count(*), max(temp) FROM demo GROUP BY color, SLIDINGWINDOW(ss, 2) OVER (WHEN size = 0) "
                             "HAVING max(temp) / (count(*) - 1) > 0.1"),
]


@pytest.mark.parametrize("name,sql", BIG, ids=[c[0] for c in BIG])
def test_window_error_texts_stream(oracle, engine_mod, name, sql):
    """A 20 k-row stream over 37 keys: many failed windows, value-dependent texts (the first failed row in window
    order, the failed group with the smallest key) through the kernels each window shape takes."""
    rule = compile_rule(sql, SCHEMA, num_keys=37)
    cols = _stream(20_000, 37, seed=zlib.crc32(name.encode()))
    got, exp, _ = run_both(oracle, engine_mod, rule, cols, batches=3)
    assert any(e for e in exp.errors), "the case must fail some windows"
    _assert_errors(got, exp)


def test_window_error_abi(engine_mod):
    """ek_window_error: length query, truncation with NUL, "" for an OK window, EK_ERR_INVALID out of range."""
    import ctypes as C
    from ekgpu.engine import lib
    rule = compile_rule(CASES[0][1], SCHEMA, num_keys=4)
    eng = engine_mod.Engine(rule.plan)
    eng.push_host(_cols())
    r = A.ek_result()
    assert lib().ek_poll_results(eng.h, A.EK_MEM_HOST, C.byref(r)) == 0
    st = np.ctypeslib.as_array(r.win_status, shape=(r.n_windows,)).copy()
    w_err = int(np.nonzero(st)[0][0])
    w_ok = int(np.nonzero(st == 0)[0][0])
    n = C.c_int64(-1)
    assert lib().ek_window_error(eng.h, w_err, None, 0, C.byref(n)) == 0
    assert n.value == len("run Where error: divided by zero")
    buf = C.create_string_buffer(8)
    assert lib().ek_window_error(eng.h, w_err, buf, 8, C.byref(n)) == 0
    assert buf.value == b"run Whe"
    assert lib().ek_window_error(eng.h, w_ok, buf, 8, C.byref(n)) == 0 and n.value == 0 and buf.value == b""
    assert lib().ek_window_error(eng.h, int(r.n_windows), buf, 8, C.byref(n)) == A.EK_ERR_INVALID
    lib().ek_release_results(eng.h, C.byref(r))
    eng.close()


def test_window_error_texts_across_restore(oracle, engine_mod):
    """A checkpoint taken while panes hold failed rows carries their witnesses (state v4): the restored handle
    prints the same texts as one uninterrupted run."""
    sql = "SELECT count(*) FROM demo WHERE temp * 1.5 GROUP BY color, HOPPINGWINDOW(ss, 2, 1)"
    rule = compile_rule(sql, SCHEMA, num_keys=37)
    cols = _stream(20_000, 37, seed=5)
    exp = oracle.run(rule.plan, cols)
    half = 10_037
    a = engine_mod.Engine(rule.plan)
    a.push_host([c[:half] for c in cols])
    got = a.poll()
    blob = a.export_state()
    a.close()
    b = engine_mod.Engine(rule.plan)
    b.import_state(blob)
    b.push_host([c[half:] for c in cols])
    got += b.poll()
    b.close()
    assert any(exp.errors)
    _assert_errors(got, exp)
