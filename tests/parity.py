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
                is_float_col = c >= 0 and plan.column_type[c] == A.EK_COL_F64
                x, y = gv[a], ev[a]
                if type(x) is not type(y):
                    bad.append((key, a, x, y, "type"))
                elif fn in FP_TOL_FNS and isinstance(y, float) and (is_float_col or fn != A.EK_AGG_SUM):
                    if not _close(x, y, REL_TOL):
                        bad.append((key, a, x, y, "tol"))
                elif not (x == y or (isinstance(x, float) and math.isnan(x) and math.isnan(y))):
                    bad.append((key, a, x, y, "exact"))
        assert not bad, f"window {w} (end {e.end}): {len(bad)} mismatches, e.g. {bad[:max_report]}"
