"""Global (un-grouped) aggregates over key-hash shards.

A rule without a GROUP BY key (e.g. C5's ``SELECT count(*) FROM demo GROUP BY TUMBLINGWINDOW(ss, 60)``)
cannot be split by key: every shard sees part of every window. Each rank therefore runs a *partial*
plan on its own shard (count / sum / min / max / var partials, funcs_agg.go:56-297 decomposed), and the
per-window partial rows are exchanged with one ``all_gather`` over the default process group (RCCL over
xGMI when the backend is "nccl", gloo on the CPU) and merged on every rank:

  count(*) / count(x)  sum of partial counts
  sum(x)               sum of partial sums (int: wrap-around int64; float: f64, rank order)
  avg(x)               sum / count, int columns truncating like funcs_agg.go:56-86
  min(x) / max(x)      min / max of the partials (nil partials skipped)
  var/vars/stddev(s)   Chan et al. merge of (n, mean, M2) partials (M2 = var_pop * n)
  median/percentile_*  not decomposable: rejected (run them GROUP BY key, or on one rank)

HAVING is evaluated after the merge (having_operator.go:32-104 semantics: only true keeps the window's
row; nil or non-bool -> window error). The exchange carries 8-16 B per partial and window, so it is
latency-bound; windows are matched by their end time.
"""
import copy
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi as A
from .rule import CompiledRule

_DECOMPOSABLE = {A.EK_AGG_COUNT_STAR, A.EK_AGG_COUNT, A.EK_AGG_SUM, A.EK_AGG_AVG, A.EK_AGG_MIN, A.EK_AGG_MAX,
                 A.EK_AGG_VAR, A.EK_AGG_VARS, A.EK_AGG_STDDEV, A.EK_AGG_STDDEVS}


class GlobalAggError(ValueError):
    pass


@dataclass
class GlobalWindow:
    start: int
    end: int
    status: int
    values: Optional[Tuple]      # one merged value per final aggregate, or None (no row)


@dataclass
class PartialPlan:
    """The plan every rank runs, and how final aggregate k is rebuilt from partial slots."""
    plan: A.ek_plan
    final: List[Tuple[int, int, Tuple[int, ...]]] = field(default_factory=list)   # (fn, column, partial slots)
    final_is_float: List[bool] = field(default_factory=list)
    having: List[Tuple] = field(default_factory=list)


def make_partial_plan(rule: CompiledRule) -> PartialPlan:
    src = rule.plan
    if src.key_column >= 0:
        raise GlobalAggError("rule has a GROUP BY key: shard by key instead (results are disjoint per shard)")
    plan = copy.deepcopy(src)
    plan.n_having = 0
    slots: List[Tuple[int, int]] = []

    def slot(fn, col):
        if (fn, col) not in slots:
            slots.append((fn, col))
        return slots.index((fn, col))

    pp = PartialPlan(plan=plan)
    for k in range(src.n_aggs):
        fn, col = src.aggs[k].fn, src.aggs[k].column
        if fn not in _DECOMPOSABLE:
            raise GlobalAggError("median / percentile are not decomposable across shards")
        isf = col >= 0 and src.column_type[col] == A.EK_COL_F64
        if fn in (A.EK_AGG_COUNT_STAR, A.EK_AGG_COUNT, A.EK_AGG_SUM, A.EK_AGG_MIN, A.EK_AGG_MAX):
            parts = (slot(fn, col),)
        elif fn == A.EK_AGG_AVG:
            parts = (slot(A.EK_AGG_SUM, col), slot(A.EK_AGG_COUNT, col))
        else:
            parts = (slot(A.EK_AGG_COUNT, col), slot(A.EK_AGG_SUM, col), slot(A.EK_AGG_VAR, col))
        pp.final.append((fn, col, parts))
        pp.final_is_float.append(isf)
    if len(slots) > A.EK_MAX_AGGS:
        raise GlobalAggError("too many partial aggregates")
    plan.n_aggs = len(slots)
    for k, (fn, col) in enumerate(slots):
        plan.aggs[k].fn = fn
        plan.aggs[k].column = col
        plan.aggs[k].param = 0.0
    pp.having = [(src.having_prog[k].op, src.having_prog[k].arg, src.having_prog[k].i64, src.having_prog[k].f64)
                 for k in range(src.n_having)]
    return pp


# ------------------------------------------------------------------ packing / exchange
def pack_windows(windows, n_partials: int) -> np.ndarray:
    """int64 [n_windows, 4 + 2 * n_partials]: end, start, status, has_row, (value bits, tag) * n."""
    out = np.zeros((len(windows), 4 + 2 * n_partials), dtype=np.int64)
    for i, w in enumerate(windows):
        out[i, 0], out[i, 1], out[i, 2] = w.end, w.start, w.status
        if len(w.keys) and w.status == A.EK_WIN_OK:
            out[i, 3] = 1
            for a in range(n_partials):
                out[i, 4 + 2 * a] = w.values[a][0]
                out[i, 5 + 2 * a] = w.tags[a][0]
    return out


def all_gather_partials(local: np.ndarray, group=None) -> List[np.ndarray]:
    """One all_gather of the packed partial rows of every rank (padded to the longest)."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    world = dist.get_world_size(group)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    counts = [int(x.item()) for x in ns]
    width = local.shape[1]
    m = max(counts + [1])
    buf = torch.zeros((m, width), dtype=torch.int64, device=dev)
    if local.shape[0]:
        buf[: local.shape[0]] = torch.from_numpy(local).to(dev)
    outs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return [o[:c].cpu().numpy() for o, c in zip(outs, counts)]


def exchange_triggers(trig_arrival: np.ndarray, trig_ts: np.ndarray, group=None) -> Tuple[np.ndarray, np.ndarray]:
    """The sliding-window trigger exchange of a key-hash-sharded rule: every rank's accepted OVER (WHEN ...) rows
    (global arrival, ts) of the micro-batch (ek_shard_triggers) go to every rank with one all_gather (RCCL over
    xGMI with backend "nccl"); the merged list, in global arrival order, is the ek_global_ctx trigger list every
    shard fires its windows for (event_window_trigger.go:190-192: a trigger opens a window over ALL keys)."""
    from .shard import merge_triggers
    local = np.stack([np.asarray(trig_arrival, np.int64), np.asarray(trig_ts, np.int64)], axis=1) \
        if len(trig_arrival) else np.zeros((0, 2), np.int64)
    parts = all_gather_partials(local, group)
    return merge_triggers([(p[:, 0], p[:, 1]) for p in parts])


def all_gather_objects(obj, group=None) -> list:
    """Picklable per-rank results to every rank (result gather of the tests / tools; not on the data path)."""
    import torch.distributed as dist
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


# ------------------------------------------------------------------ merge
def _val(bits: int, tag: int):
    if tag == A.EK_TAG_NULL:
        return None
    if tag == A.EK_TAG_I64:
        return int(bits)
    return float(np.array([bits], dtype=np.int64).view(np.float64)[0])


def _wrap64(x: int) -> int:
    return (x + (1 << 63)) % (1 << 64) - (1 << 63)


def _merge_one(fn: int, isf: bool, parts: List[List]):
    """parts[p] = list over ranks of the partial values of slot p (None = nil partial)."""
    if fn in (A.EK_AGG_COUNT_STAR, A.EK_AGG_COUNT):
        return sum(v for v in parts[0] if v is not None)
    if fn in (A.EK_AGG_MIN, A.EK_AGG_MAX):
        vs = [v for v in parts[0] if v is not None]
        if not vs:
            return None
        return min(vs) if fn == A.EK_AGG_MIN else max(vs)
    if fn == A.EK_AGG_SUM:
        vs = [v for v in parts[0] if v is not None]
        if not vs:
            return None
        if isf:
            t = 0.0
            for v in vs:
                t += v
            return t
        return _wrap64(sum(vs))
    if fn == A.EK_AGG_AVG:
        sums, cnts = parts
        n = sum(c for c in cnts if c is not None)
        vs = [v for v in sums if v is not None]
        if n == 0 or not vs:
            return None
        if isf:
            t = 0.0
            for v in vs:
                t += v
            return t / n
        t = _wrap64(sum(vs))
        q = abs(t) // n
        return q if t >= 0 else -q                 # Go integer division truncates toward zero
    # var family: Chan merge of (n, mean, M2)
    cnts, sums, vars_ = parts
    n_tot, mean, m2 = 0, 0.0, 0.0
    for c, s, v in zip(cnts, sums, vars_):
        if not c:
            continue
        mb = float(s) / c
        m2b = v * c
        if n_tot == 0:
            n_tot, mean, m2 = c, mb, m2b
            continue
        d = mb - mean
        n_new = n_tot + c
        m2 = m2 + m2b + d * d * (n_tot * c / n_new)
        mean = mean + d * c / n_new
        n_tot = n_new
    if n_tot == 0:
        return None
    sample = fn in (A.EK_AGG_VARS, A.EK_AGG_STDDEVS)
    var = m2 / (n_tot - 1) if sample else m2 / n_tot
    if sample and n_tot == 1:
        var = float("nan")
    return math.sqrt(var) if fn in (A.EK_AGG_STDDEV, A.EK_AGG_STDDEVS) else var


def _eval_having(prog, aggs):
    """Postfix HAVING program over the merged values (valuer.go:574-1000 subset); returns value or 'ERR'."""
    st = []
    for op, arg, i64, f64 in prog:
        if op == A.EK_OP_AGG:
            st.append(aggs[arg])
        elif op == A.EK_OP_CONST_I64:
            st.append(int(i64))
        elif op == A.EK_OP_CONST_F64:
            st.append(float(f64))
        elif op == A.EK_OP_CONST_BOOL:
            st.append(bool(i64))
        elif op == A.EK_OP_COL:
            return "ERR"
        else:
            r, l = st.pop(), st.pop()
            if l == "ERR" or r == "ERR":
                st.append("ERR")
                continue
            if op in (A.EK_OP_AND, A.EK_OP_OR):
                if l is None or r is None:
                    st.append(False)
                elif not isinstance(l, bool) or not isinstance(r, bool):
                    st.append("ERR")
                else:
                    st.append((l and r) if op == A.EK_OP_AND else (l or r))
                continue
            if l is None or r is None:
                st.append(False if op <= A.EK_OP_GTE else None)
                continue
            if isinstance(l, bool) or isinstance(r, bool):   # bools compare with bools by = / != only (valuer.go)
                ok = isinstance(l, bool) and isinstance(r, bool) and op in (A.EK_OP_EQ, A.EK_OP_NEQ)
                st.append(((l == r) if op == A.EK_OP_EQ else (l != r)) if ok else "ERR")
                continue
            if isinstance(l, float) or isinstance(r, float):
                l, r = float(l), float(r)
            if op == A.EK_OP_EQ: st.append(l == r)
            elif op == A.EK_OP_NEQ: st.append(l != r)
            elif op == A.EK_OP_LT: st.append(l < r)
            elif op == A.EK_OP_LTE: st.append(l <= r)
            elif op == A.EK_OP_GT: st.append(l > r)
            elif op == A.EK_OP_GTE: st.append(l >= r)
            elif op == A.EK_OP_ADD: st.append(l + r)
            elif op == A.EK_OP_SUB: st.append(l - r)
            elif op == A.EK_OP_MUL: st.append(l * r)
            elif op in (A.EK_OP_DIV, A.EK_OP_MOD):
                if r == 0:
                    st.append("ERR")
                elif op == A.EK_OP_MOD:
                    st.append(math.fmod(l, r) if isinstance(l, float) else int(math.fmod(l, r)))
                else:
                    st.append(l / r if isinstance(l, float) else int(l / r))
    return st[-1] if st else None


def merge_partials(pp: PartialPlan, per_rank: Sequence[np.ndarray], closed_end: Optional[int] = None) -> List[GlobalWindow]:
    """Merge the packed partial windows of all ranks; windows are matched by end time and emitted in
    end order. With closed_end, only windows with end <= closed_end are merged (the rest stay open)."""
    by_end: Dict[int, List[np.ndarray]] = {}
    for arr in per_rank:
        for row in arr:
            by_end.setdefault(int(row[0]), []).append(row)
    out = []
    for end in sorted(by_end):
        if closed_end is not None and end > closed_end:
            continue
        rows = by_end[end]
        start = min(int(r[1]) for r in rows)
        status = 0
        for r in rows:
            status |= int(r[2])
        have = [r for r in rows if r[3]]
        if status or not have:
            out.append(GlobalWindow(start, end, status, None))
            continue
        vals = []
        for k, (fn, col, slots) in enumerate(pp.final):
            parts = [[_val(int(r[4 + 2 * s]), int(r[5 + 2 * s])) for r in have] for s in slots]
            vals.append(_merge_one(fn, pp.final_is_float[k], parts))
        if pp.having:
            h = _eval_having(pp.having, vals)
            if not isinstance(h, bool):
                out.append(GlobalWindow(start, end, A.EK_WIN_HAVING_ERROR, None))
                continue
            if not h:
                out.append(GlobalWindow(start, end, 0, None))
                continue
        out.append(GlobalWindow(start, end, 0, tuple(vals)))
    return out


def global_windows(pp: PartialPlan, local_windows, group=None, closed_end: Optional[int] = None) -> List[GlobalWindow]:
    """Collective: every rank passes the partial windows its engine emitted; returns the merged windows."""
    local = pack_windows(local_windows, pp.plan.n_aggs)
    return merge_partials(pp, all_gather_partials(local, group), closed_end)
