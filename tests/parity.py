"""Parity helpers: compare engine windows with oracle windows (SURVEY.md §8(d) parity rule).

* windows compared in trigger order: window_start, window_end, status (and membership when enabled)
* rows compared as sets keyed by (window_end, key) — the reference emits groups in Go map order
* bit-exact: count, min, max, integer sum/avg, HAVING decisions, value types (tags)
* relative <= 1e-6 (the north-star tolerance): f64 sum, avg, stddev(s), var(s)
"""
import math

from ekgpu import abi as A

FP_TOL_FNS = {A.EK_AGG_SUM, A.EK_AGG_AVG, A.EK_AGG_STDDEV, A.EK_AGG_STDDEVS, A.EK_AGG_VAR, A.EK_AGG_VARS,
              A.EK_AGG_PERCENTILE_CONT}
REL_TOL = 1e-6


def col_type(plan, c):
    """Column type of an aggregate's argument; c >= n_columns names a derived (expression) column."""
    return plan.column_type[c] if c < plan.n_columns else plan.derived_type[c - plan.n_columns]


def _close(a, b, rel):
    if a is None or b is None:
        return a is b
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    return abs(a - b) <= rel * max(abs(a), abs(b), 1e-300) or a == b


def assert_windows_equal(plan, got, exp, check_members=False, max_report=5):
    assert len(got) == len(exp), f"window count {len(got)} != {len(exp)}"
    for w, (g, e) in enumerate(zip(got, exp)):
        assert (g.start, g.end, g.status) == (e.start, e.end, e.status), \
            f"window {w}: got {(g.start, g.end, g.status)} expected {(e.start, e.end, e.status)}"
        if check_members:
            assert (g.member_count, g.member_hash) == (e.member_count, e.member_hash), \
                f"window {w} membership: got {(g.member_count, g.member_hash)} expected {(e.member_count, e.member_hash)}"
        gr, er = g.rows(), e.rows()
        assert set(gr) == set(er), f"window {w} (end {e.end}): key sets differ: " \
                                   f"missing {sorted(set(er) - set(gr))[:5]} extra {sorted(set(gr) - set(er))[:5]}"
        bad = []
        for key, ev in er.items():
            gv = gr[key]
            for a in range(plan.n_aggs):
                fn = plan.aggs[a].fn
                c = plan.aggs[a].column
                is_float_col = c >= 0 and col_type(plan, c) == A.EK_COL_F64
                x, y = gv[a], ev[a]
                if type(x) is not type(y):
                    bad.append((key, a, x, y, "type"))
                elif fn in FP_TOL_FNS and isinstance(y, float) and (is_float_col or fn != A.EK_AGG_SUM):
                    if not _close(x, y, REL_TOL):
                        bad.append((key, a, x, y, "tol"))
                elif not (x == y or (isinstance(x, float) and math.isnan(x) and math.isnan(y))):
                    bad.append((key, a, x, y, "exact"))
        assert not bad, f"window {w} (end {e.end}): {len(bad)} mismatches, e.g. {bad[:max_report]}"


def assert_windows_equal_np(plan, got, exp, check_members=False):
    """assert_windows_equal for full-size runs (millions of rows): the same rule, vectorised per window.
    Rows are matched by key after sorting both sides; tags (Go dynamic types) must match exactly, values
    bit-exactly (NaN == NaN) except the FP_TOL_FNS over float results (relative <= REL_TOL)."""
    import numpy as np
    assert len(got) == len(exp), f"window count {len(got)} != {len(exp)}"
    tol_aggs = set()
    for a in range(plan.n_aggs):
        fn, c = plan.aggs[a].fn, plan.aggs[a].column
        is_float_col = c >= 0 and col_type(plan, c) == A.EK_COL_F64
        if fn in FP_TOL_FNS and (is_float_col or fn != A.EK_AGG_SUM):
            tol_aggs.add(a)
    for w, (g, e) in enumerate(zip(got, exp)):
        assert (g.start, g.end, g.status) == (e.start, e.end, e.status), \
            f"window {w}: got {(g.start, g.end, g.status)} expected {(e.start, e.end, e.status)}"
        if check_members:
            assert (g.member_count, g.member_hash) == (e.member_count, e.member_hash), \
                f"window {w} membership: got {(g.member_count, g.member_hash)} expected {(e.member_count, e.member_hash)}"
        go, eo = np.argsort(g.keys, kind="stable"), np.argsort(e.keys, kind="stable")
        gk, ek = g.keys[go], e.keys[eo]
        assert len(gk) == len(ek) and np.array_equal(gk, ek), \
            f"window {w} (end {e.end}): key sets differ ({len(gk)} vs {len(ek)} rows; " \
            f"missing {np.setdiff1d(ek, gk)[:5]}, extra {np.setdiff1d(gk, ek)[:5]})"
        assert len(np.unique(gk)) == len(gk), f"window {w}: duplicate keys"
        for a in range(plan.n_aggs):
            gt, et = g.tags[a][go], e.tags[a][eo]
            bad = np.nonzero(gt != et)[0]
            assert len(bad) == 0, f"window {w} agg {a}: {len(bad)} type mismatches, e.g. key {gk[bad[0]]}: {gt[bad[0]]} vs {et[bad[0]]}"
            gv, ev = g.values[a][go], e.values[a][eo]
            isf = et == A.EK_TAG_F64
            gf, ef = gv.view(np.float64), ev.view(np.float64)
            nan_both = isf & np.isnan(gf) & np.isnan(ef)
            if a in tol_aggs:
                with np.errstate(invalid="ignore", over="ignore"):
                    scale = np.maximum(np.maximum(np.abs(gf), np.abs(ef)), 1e-300)
                    ok_f = (np.abs(gf - ef) <= REL_TOL * scale) | (gf == ef) | nan_both
                ok = np.where(isf, ok_f, gv == ev)
            else:
                ok = (gv == ev) | nan_both
            ok |= et == A.EK_TAG_NULL
            bad = np.nonzero(~ok)[0]
            assert len(bad) == 0, f"window {w} (end {e.end}) agg {a}: {len(bad)} value mismatches, e.g. key {gk[bad[0]]}: " \
                                  f"{gv[bad[0]]} vs {ev[bad[0]]}"
