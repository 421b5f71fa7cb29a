"""Convert a host-side ek_result into numpy / python structures.

Rows of window w are [win_row_offset[w], +win_row_count[w]) (ekgpu.h). Values are 8-byte slots
typed per row by agg_tag (EK_TAG_NULL / I64 / F64), i.e. the Go dynamic type of the reference's
aggregate result (funcs_agg.go: count -> int, avg(int) -> int64, median(int, even n) -> float64, ...).
"""
from dataclasses import dataclass
from typing import Dict, List

import numpy as np

from . import abi as A


@dataclass
class WindowResult:
    start: int
    end: int
    status: int
    member_count: int
    member_hash: int
    keys: np.ndarray            # uint32 [rows]
    values: List[np.ndarray]    # per agg: int64 bit patterns [rows]
    tags: List[np.ndarray]      # per agg: uint8 tags [rows]
    error: str = ""             # status != EK_WIN_OK: the reference's error text (ek_window_error)

    def value(self, a: int, r: int):
        t = int(self.tags[a][r])
        if t == A.EK_TAG_NULL:
            return None
        v = self.values[a][r:r + 1]
        if t == A.EK_TAG_BOOL:
            return bool(v[0])
        return int(v[0]) if t == A.EK_TAG_I64 else float(v.view(np.float64)[0])

    def rows(self) -> Dict[int, tuple]:
        return {int(self.keys[r]): tuple(self.value(a, r) for a in range(len(self.values)))
                for r in range(len(self.keys))}


def _arr(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


def result_to_python(res: A.ek_result) -> List[WindowResult]:
    if res.memory != A.EK_MEM_HOST:
        raise ValueError("result must be polled into host memory")
    nw, nr, na = int(res.n_windows), int(res.n_rows), int(res.n_aggs)
    ws = _arr(res.win_start, nw, np.int64)
    we = _arr(res.win_end, nw, np.int64)
    off = _arr(res.win_row_offset, nw, np.int64)
    cnt = _arr(res.win_row_count, nw, np.int64)
    st = _arr(res.win_status, nw, np.int32)
    mc = _arr(res.win_member_count, nw, np.int64) if res.win_member_count else np.zeros(nw, np.int64)
    mh = _arr(res.win_member_hash, nw, np.uint64) if res.win_member_hash else np.zeros(nw, np.uint64)
    total = int((off + cnt).max()) if nw else 0
    total = max(total, nr)
    keys = _arr(res.key, total, np.uint32)
    vals = [_arr(res.agg_value[a], total, np.int64) for a in range(na)]
    tags = [_arr(res.agg_tag[a], total, np.uint8) for a in range(na)]
    out = []
    for w in range(nw):
        o, c = int(off[w]), int(cnt[w])
        out.append(WindowResult(int(ws[w]), int(we[w]), int(st[w]), int(mc[w]), int(mh[w]), keys[o:o + c],
                                [v[o:o + c] for v in vals], [t[o:o + c] for t in tags]))
    return out
