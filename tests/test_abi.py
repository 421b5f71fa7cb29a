import numpy as np
"""CPU-side checks of the boundary: the C-ABI library loads and exports every declared symbol; the
ctypes mirror matches the header; the rule compiler builds the plans the configs need."""
import ctypes as C
import os
import re

import pytest

from ekgpu import abi as A
from ekgpu.rule import RuleError, compile_rule
from ekgpu.synth import IOT_SCHEMA

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ekgpu.h")


def declared_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(ek_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    from ekgpu import engine
    L = engine.lib()
    names = declared_functions()
    assert len(names) >= 12
    for name in names:
        assert hasattr(L, name), name
    assert set(names) <= set(engine.EXPORTED_SYMBOLS)
    assert L.ek_abi_version() == A.EKGPU_ABI_VERSION


def test_header_constants_match_ctypes():
    txt = open(HEADER).read()
    for name in ("EK_MAX_COLUMNS", "EK_MAX_AGGS", "EK_MAX_PROG", "EKGPU_ABI_VERSION"):
        m = re.search(rf"#define {name} (\d+)", txt)
        assert int(m.group(1)) == getattr(A, name)
    for name, val in re.findall(r"(EK_(?:WINDOW|AGG|OP|UNIT|COL|TAG|WIN|MEM)_[A-Z_]+)\s*=\s*(-?\d+)", txt):
        assert getattr(A, name) == int(val), name


def test_plan_struct_layout():
    # offsets the C side sees (computed by the compiler through a tiny probe library)
    import subprocess, tempfile
    src = r'''
#include <stddef.h>
#include "ekgpu.h"
size_t off_aggs(void){return offsetof(ek_plan,aggs);} size_t off_having(void){return offsetof(ek_plan,having_prog);}
size_t size_plan(void){return sizeof(ek_plan);} size_t size_result(void){return sizeof(ek_result);}
size_t off_rkey(void){return offsetof(ek_result,key);} size_t size_batch(void){return sizeof(ek_batch);}
size_t size_stats(void){return sizeof(ek_stats);} size_t off_kmaj(void){return offsetof(ek_stats,windows_keymajor);}
size_t off_bts(void){return offsetof(ek_batch,ts_stats);} size_t size_tss(void){return sizeof(ek_ts_stats);}
size_t off_tss_step(void){return offsetof(ek_ts_stats,max_step);} size_t off_tss_data(void){return offsetof(ek_ts_stats,ts_data);}
'''
    d = tempfile.mkdtemp()
    with open(os.path.join(d, "p.c"), "w") as f:
        f.write(src)
    so = os.path.join(d, "p.so")
    subprocess.check_call(["gcc", "-shared", "-fPIC", "-I", os.path.join(ROOT, "include"), "-o", so, os.path.join(d, "p.c")])
    P = C.CDLL(so)
    for fn in ("off_aggs", "off_having", "size_plan", "size_result", "off_rkey", "size_batch", "size_stats", "off_kmaj",
               "off_bts", "size_tss", "off_tss_step", "off_tss_data"):
        getattr(P, fn).restype = C.c_size_t
    assert P.off_aggs() == A.ek_plan.aggs.offset
    assert P.off_having() == A.ek_plan.having_prog.offset
    assert P.size_plan() == C.sizeof(A.ek_plan)
    assert P.size_result() == C.sizeof(A.ek_result)
    assert P.off_rkey() == A.ek_result.key.offset
    assert P.size_batch() == C.sizeof(A.ek_batch)
    assert P.size_stats() == C.sizeof(A.ek_stats)
    assert P.off_kmaj() == A.ek_stats.windows_keymajor.offset
    assert P.off_bts() == A.ek_batch.ts_stats.offset
    assert P.size_tss() == C.sizeof(A.ek_ts_stats)
    assert P.off_tss_step() == A.ek_ts_stats.max_step.offset
    assert P.off_tss_data() == A.ek_ts_stats.ts_data.offset


def test_compile_baseline_configs():
    r = compile_rule("SELECT deviceId, avg(temperature), max(humidity), count(*) FROM demo "
                     "GROUP BY deviceId, TUMBLINGWINDOW(ss,10)", IOT_SCHEMA, num_keys=65536)
    p = r.plan
    assert (p.window_type, p.time_unit, p.length, p.key_column, p.n_aggs) == (A.EK_WINDOW_TUMBLING, A.EK_UNIT_SS, 10, 0, 3)
    assert [p.aggs[k].fn for k in range(3)] == [A.EK_AGG_AVG, A.EK_AGG_MAX, A.EK_AGG_COUNT_STAR]
    assert [f.name for f in r.fields] == ["deviceId", "avg", "max", "count"]
    r = compile_rule("SELECT deviceId, sum(temperature), min(temperature), max(temperature) FROM demo "
                     "GROUP BY deviceId, HOPPINGWINDOW(ss, 60, 5)", IOT_SCHEMA, num_keys=1 << 20)
    assert (r.plan.window_type, r.plan.length, r.plan.interval) == (A.EK_WINDOW_HOPPING, 60, 5)
    r = compile_rule("SELECT deviceId, stddev(temperature), var(temperature) FROM demo GROUP BY deviceId, "
                     "COUNTWINDOW(1000) HAVING count(*) > 1", IOT_SCHEMA, num_keys=1 << 20, is_event_time=False)
    assert (r.plan.window_type, r.plan.length, r.plan.n_having) == (A.EK_WINDOW_COUNT, 1000, 3)
    assert r.plan.aggs[2].fn == A.EK_AGG_COUNT_STAR
    r = compile_rule("SELECT deviceId, median(temperature), percentile_cont(temperature, 0.9) FROM demo "
                     "GROUP BY deviceId, TUMBLINGWINDOW(ss, 60)", IOT_SCHEMA, num_keys=100)
    assert r.plan.aggs[1].fn == A.EK_AGG_PERCENTILE_CONT and r.plan.aggs[1].param == 0.9
    # a non-aggregate, non-dimension field: the group's first row (row.go:720-726) -> EK_AGG_FIRST
    r = compile_rule("SELECT temperature FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss,10)", IOT_SCHEMA, num_keys=4)
    assert r.plan.n_aggs == 1 and r.plan.aggs[0].fn == A.EK_AGG_FIRST
    with pytest.raises(RuleError):   # string columns: dimensions, min / max / count arguments, first-row fields
        compile_rule("SELECT sum(name) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss,10)", dict(IOT_SCHEMA, name="string"),
                     num_keys=4)


def test_engine_without_gpu_fails_loudly():
    """No CPU fallback: creating an engine without a HIP device must raise, not silently compute."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ekgpu.engine import Engine, EngineError
    r = compile_rule("SELECT deviceId, count(*) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss,10)",
                     IOT_SCHEMA, num_keys=16)
    with pytest.raises(EngineError):
        Engine(r.plan)


def test_expression_argument_lowering():
    """agg(<arithmetic over columns>) lowers to derived columns (row.go:712-718); identical arguments share one;
    int op int stays int, a float operand promotes; division only by a non-zero constant."""
    r = compile_rule("SELECT deviceId, avg(temperature * 1.8 + 32), max(temperature * 1.8 + 32), sum(humidity), "
                     "count(temperature - humidity) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss,10)",
                     IOT_SCHEMA, num_keys=16)
    p = r.plan
    assert p.n_derived == 2 and p.n_columns == 4
    assert [p.aggs[k].column for k in range(4)] == [4, 4, 3, 5]
    assert [p.derived_type[d] for d in range(2)] == [A.EK_COL_F64, A.EK_COL_F64]
    schema = {"k": "key", "ts": "bigint", "a": "bigint", "x": "float"}
    r = compile_rule("SELECT k, sum(a * 3 / 2), sum(a % 5 + x) FROM s GROUP BY k, TUMBLINGWINDOW(ss,1)", schema,
                     num_keys=4)
    assert [r.plan.derived_type[d] for d in range(2)] == [A.EK_COL_I64, A.EK_COL_F64]
    for bad in ("sum(a / x)", "sum(a % 0)", "sum(a / 0.0)"):
        with pytest.raises(RuleError):
            compile_rule(f"SELECT k, {bad} FROM s GROUP BY k, TUMBLINGWINDOW(ss,1)", schema, num_keys=4)


def test_oracle_expression_argument_is_per_row(oracle):
    """The oracle's derived column equals the per-row formula: avg(t*1.8+32) == avg(t)*1.8+32 per window (CPU,
    no engine)."""
    from ekgpu.synth import iot_stream
    cols = list(iot_stream(20_000, 8, events_per_ms=5))
    sql = "SELECT deviceId, avg(temperature * 1.8 + 32), avg(temperature) FROM demo GROUP BY deviceId, TUMBLINGWINDOW(ss, 1)"
    exp = oracle.run(compile_rule(sql, IOT_SCHEMA, num_keys=8).plan, cols, None)
    assert len(exp.windows) >= 3
    for w in exp.windows:
        a, b = (np.ascontiguousarray(w.values[k]).view(np.float64) for k in (0, 1))   # f64 bit patterns
        assert np.allclose(a, b * 1.8 + 32, rtol=1e-12, atol=1e-9)


def test_sliding_send_twice_plan():
    """enableSlidingWindowSendTwice (def/rule.go:104-112) lowers to ek_plan.sliding_send_twice for a delayed
    SLIDINGWINDOW only (window_op.go:98); every other window ignores it."""
    from ekgpu.rule import compile_rule
    sql = "SELECT count(*) FROM s GROUP BY SLIDINGWINDOW(ss, 10, 2)"
    assert compile_rule(sql, {"a": "bigint", "ts": "bigint"}, num_keys=1).plan.sliding_send_twice == 0
    r = compile_rule(sql, {"a": "bigint", "ts": "bigint"}, num_keys=1, sliding_send_twice=True)
    assert r.plan.sliding_send_twice == 1 and r.plan.delay == 2
    for other in ("SLIDINGWINDOW(ss, 10)", "TUMBLINGWINDOW(ss, 10)", "HOPPINGWINDOW(ss, 10, 5)"):
        r = compile_rule(f"SELECT count(*) FROM s GROUP BY {other}", {"a": "bigint", "ts": "bigint"}, num_keys=1,
                         sliding_send_twice=True)
        assert r.plan.delay == 0 and r.plan.sliding_send_twice == 0


def test_window_filter_lowering():
    """GROUP BY <window> FILTER (WHERE <cond>) (planner.go:388-392) lowers to ek_plan.filter_prog; WHERE stays."""
    from ekgpu import abi as A
    from ekgpu.rule import compile_rule
    r = compile_rule("SELECT count(*) FROM s WHERE a > 1 GROUP BY SLIDINGWINDOW(ss, 5) FILTER (WHERE a < 9) OVER (WHEN a = 3)",
                     {"a": "bigint", "ts": "bigint"}, num_keys=1)
    assert r.plan.n_where == 3 and r.plan.n_filter == 3 and r.plan.n_trigger == 3
    assert [r.plan.filter_prog[k].op for k in range(3)] == [A.EK_OP_COL, A.EK_OP_CONST_I64, A.EK_OP_LT]
