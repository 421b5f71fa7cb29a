"""ctypes binding of the CPU ORACLE (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module. The product
path (ekgpu package, libekgpu.so) never imports, links or executes anything under oracle/.
"""
import ctypes as C
import os
import subprocess
import sys
from typing import Dict, List, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "ekuiper-vioneta_amd"))
from ekgpu import abi as A  # noqa: E402
from ekgpu.results import result_to_python  # noqa: E402

# EKO_LIB: an alternative build of the same sources (tests/test_oracle_asan.py loads the ASan/UBSan one)
LIB_PATH = os.environ.get("EKO_LIB") or os.path.join(HERE, "libekoracle.so")


class eko_output(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("error", C.c_char * 256),
        ("records_late", C.c_int64),
        ("r", A.ek_result),
        ("member_offset", C.POINTER(C.c_int64)),
        ("members", C.POINTER(C.c_int64)),
        ("win_error", C.c_void_p),
        ("records_filter_error", C.c_int64),
    ]


class eko_restart(C.Structure):
    _fields_ = [("split", C.c_int64), ("export_ms", C.c_int64), ("restart_ms", C.c_int64)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.eko_run.argtypes = [C.POINTER(A.ek_plan), C.c_int64, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                 C.POINTER(eko_output)]
        _lib.eko_run.restype = C.c_int
        _lib.eko_free.argtypes = [C.POINTER(eko_output)]
        _lib.eko_aligned_window_end.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_int32]
        _lib.eko_aligned_window_end.restype = C.c_int64
        _lib.eko_agg_exec.argtypes = [C.c_int32, C.c_int32, C.c_int64, C.c_void_p, C.c_void_p, C.c_double,
                                      C.POINTER(C.c_int64), C.POINTER(C.c_uint8), C.c_char_p, C.c_int32]
        _lib.eko_agg_exec.restype = C.c_int
        _lib.eko_run_shard.argtypes = [C.POINTER(A.ek_plan), C.c_int64, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                       C.POINTER(A.ek_global_ctx), C.POINTER(eko_output)]
        _lib.eko_run_shard.restype = C.c_int
        _lib.eko_run_proc.argtypes = [C.POINTER(A.ek_plan), C.c_int64, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                      C.c_int64, C.c_int64, C.POINTER(eko_output)]
        _lib.eko_run_proc.restype = C.c_int
        _lib.eko_run_proc_restart.argtypes = [C.POINTER(A.ek_plan), C.c_int64, C.POINTER(C.c_void_p),
                                              C.POINTER(C.c_void_p), C.c_int64, C.c_int64, C.POINTER(eko_restart),
                                              C.POINTER(eko_output)]
        _lib.eko_run_proc_restart.restype = C.c_int
        _lib.eko_shard_triggers.argtypes = [C.POINTER(A.ek_plan), C.c_int64, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                            C.POINTER(A.ek_global_ctx), C.c_void_p, C.c_void_p]
        _lib.eko_shard_triggers.restype = C.c_int64
    return _lib


class OracleRun:
    def __init__(self, windows, members: List[np.ndarray], records_late: int, errors: List[str],
                 records_filter_error: int = 0):
        self.windows = windows
        self.members = members
        self.records_late = records_late
        self.errors = errors
        self.records_filter_error = records_filter_error


def _col_arrays(plan: A.ek_plan, columns: List[np.ndarray]):
    dtypes = {A.EK_COL_I64: np.int64, A.EK_COL_F64: np.float64, A.EK_COL_U32: np.uint32, A.EK_COL_BOOL: np.int64}
    keep = []
    for k in range(plan.n_columns):
        keep.append(np.ascontiguousarray(columns[k], dtype=dtypes[plan.column_type[k]]))
    return keep


def _ptrs(plan, columns, validity):
    cols = _col_arrays(plan, columns)
    n = len(cols[0]) if cols else 0
    cptr = (C.c_void_p * A.EK_MAX_COLUMNS)()
    vptr = (C.c_void_p * A.EK_MAX_COLUMNS)()
    keep = list(cols)
    for k, a in enumerate(cols):
        cptr[k] = a.ctypes.data
        if validity is not None and validity[k] is not None:
            v = np.ascontiguousarray(validity[k], dtype=np.uint8)
            keep.append(v)
            vptr[k] = v.ctypes.data
    return n, cptr, vptr, keep


def _collect(L, out) -> OracleRun:
    try:
        wins = result_to_python(out.r)
        nw = int(out.r.n_windows)
        moff = np.ctypeslib.as_array(out.member_offset, shape=(nw + 1,)).copy()
        mem = np.ctypeslib.as_array(out.members, shape=(max(int(moff[-1]), 1),)).copy()[: int(moff[-1])]
        members = [mem[moff[w]:moff[w + 1]] for w in range(nw)]
        raw = C.string_at(out.win_error, 128 * max(nw, 1))
        errors = [raw[128 * w:128 * (w + 1)].split(b"\0")[0].decode() for w in range(nw)]
        return OracleRun(wins, members, int(out.records_late), errors, int(out.records_filter_error))
    finally:
        L.eko_free(C.byref(out))


def run(plan: A.ek_plan, columns: List[np.ndarray], validity: Optional[List[Optional[np.ndarray]]] = None) -> OracleRun:
    L = lib()
    n, cptr, vptr, _keep = _ptrs(plan, columns, validity)
    out = eko_output()
    rc = L.eko_run(C.byref(plan), n, cptr, vptr, C.byref(out))
    if rc != 0:
        msg = out.error.decode()
        raise RuntimeError(f"oracle error {rc}: {msg}")
    return _collect(L, out)


def run_proc(plan: A.ek_plan, columns: List[np.ndarray], start_ms: int, end_ms: int,
             validity: Optional[List[Optional[np.ndarray]]] = None) -> OracleRun:
    """Processing-time windows under a deterministic clock (eko_run_proc): the rule opens at start_ms, every row is
    delivered at its timestamp (arrival time), then the clock moves to end_ms."""
    L = lib()
    n, cptr, vptr, _keep = _ptrs(plan, columns, validity)
    out = eko_output()
    rc = L.eko_run_proc(C.byref(plan), n, cptr, vptr, int(start_ms), int(end_ms), C.byref(out))
    if rc != 0:
        msg = out.error.decode()
        raise RuntimeError(f"oracle error {rc}: {msg}")
    return _collect(L, out)


def run_proc_restart(plan: A.ek_plan, columns: List[np.ndarray], start_ms: int, end_ms: int, split: int,
                     export_ms: int, restart_ms: int,
                     validity: Optional[List[Optional[np.ndarray]]] = None) -> OracleRun:
    """run_proc with a checkpoint after row `split` at clock export_ms and the rule restarted at restart_ms
    (eko_run_proc_restart: timers dropped, tickers re-aligned, restored inputs replayed, window_op.go:268-325)."""
    L = lib()
    n, cptr, vptr, _keep = _ptrs(plan, columns, validity)
    out = eko_output()
    rs = eko_restart(int(split), int(export_ms), int(restart_ms))
    rc = L.eko_run_proc_restart(C.byref(plan), n, cptr, vptr, int(start_ms), int(end_ms), C.byref(rs), C.byref(out))
    if rc != 0:
        msg = out.error.decode()
        raise RuntimeError(f"oracle error {rc}: {msg}")
    return _collect(L, out)


def run_shard(plan: A.ek_plan, columns: List[np.ndarray], ctx: A.ek_global_ctx,
              validity: Optional[List[Optional[np.ndarray]]] = None) -> OracleRun:
    """Shard model of the multi-GPU protocol (eko_run_shard): one shard's rows + the whole stream's context."""
    L = lib()
    n, cptr, vptr, _keep = _ptrs(plan, columns, validity)
    out = eko_output()
    rc = L.eko_run_shard(C.byref(plan), n, cptr, vptr, C.byref(ctx), C.byref(out))
    if rc != 0:
        msg = out.error.decode()
        raise RuntimeError(f"oracle error {rc}: {msg}")
    return _collect(L, out)


def shard_triggers(plan: A.ek_plan, columns: List[np.ndarray], ctx: A.ek_global_ctx,
                   validity: Optional[List[Optional[np.ndarray]]] = None):
    L = lib()
    n, cptr, vptr, _keep = _ptrs(plan, columns, validity)
    oa = np.zeros(max(n, 1), np.int64)
    ot = np.zeros(max(n, 1), np.int64)
    k = int(L.eko_shard_triggers(C.byref(plan), n, cptr, vptr, C.byref(ctx), oa.ctypes.data, ot.ctypes.data))
    return oa[:k], ot[:k]


def aligned_window_end(ts_ms: int, interval: int, unit: int, tz_offset_s: int = 0) -> int:
    return int(lib().eko_aligned_window_end(ts_ms, interval, unit, tz_offset_s))


def agg_exec(fn: int, col_type: int, values, valid=None, param: float = 0.0):
    """Direct builtins[name].exec call (funcs_agg_test.go style). Returns (value|None) or raises ValueError(msg)."""
    dt = {A.EK_COL_I64: np.int64, A.EK_COL_F64: np.float64, A.EK_COL_U32: np.uint32}[col_type]
    arr = np.ascontiguousarray(np.asarray(values, dtype=dt) if len(values) else np.zeros(0, dt))
    vv = None if valid is None else np.ascontiguousarray(np.asarray(valid, dtype=np.uint8))
    out_v = C.c_int64()
    out_t = C.c_uint8()
    err = C.create_string_buffer(256)
    rc = lib().eko_agg_exec(fn, col_type, len(arr), arr.ctypes.data if len(arr) else None,
                            vv.ctypes.data if vv is not None else None, param, C.byref(out_v), C.byref(out_t), err, 256)
    if rc != 0:
        raise ValueError(err.value.decode())
    if out_t.value == A.EK_TAG_NULL:
        return None
    if out_t.value == A.EK_TAG_I64:
        return int(out_v.value)
    return float(np.array([out_v.value], dtype=np.int64).view(np.float64)[0])
