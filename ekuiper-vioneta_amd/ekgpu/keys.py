"""Host dictionaries of GROUP BY keys: multi-dimension and string GROUP BY on top of the engine's dense u32 key.

The reference groups a window's rows by a STRING key built from every dimension
(internal/topo/operator/aggregate_operator.go:49-56):

    for _, d := range dimensions { name += fmt.Sprintf("%v,", ve.Eval(d.Expr)) }

so two rows share a group iff their concatenations are equal — including the quirk that dimensions whose values
contain commas can collide ("a,b" + "c" and "a" + "b,c" both give "a,b,c,"), and that nil prints as "<nil>".
`GroupKeyDict` assigns each distinct key string a dense id in first-seen order (the engine's u32 key column) and
keeps the first row's dimension values per id, which is what a SELECT of a dimension shows
(internal/xsql/row.go:720-726: non-aggregate fields come from the group's first row). Without a string dimension
the %v strings are injective on the values (numbers never print a comma), so the dictionary keys on the value
tuples directly (vectorised) instead of formatting strings.

`StringDict` gives a string column dense u32 codes so it can travel to the device as a key-typed column.
"""
import math
from decimal import Decimal
from typing import Dict, List, Optional, Sequence

import numpy as np


def go_v_float(x: float) -> str:
    """fmt.Sprintf("%v", float64): strconv.FormatFloat(x, 'g', -1, 64) — shortest digits; exponent form when the
    decimal exponent is < -4 or >= 6 (strconv/ftoa.go: shortest %g uses eprec 6), at least two exponent digits."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "+Inf" if x > 0 else "-Inf"
    if x == 0:
        return "-0" if math.copysign(1.0, x) < 0 else "0"
    t = Decimal(repr(abs(x))).normalize().as_tuple()   # shortest round-trip digits, as strconv's shortest
    digits = "".join(map(str, t.digits))
    nd = len(digits)
    dp = nd + t.exponent                  # decimal point position after the first dp digits
    exp = dp - 1
    sign = "-" if x < 0 else ""
    if exp < -4 or exp >= 6:
        m = digits[0] + ("." + digits[1:] if nd > 1 else "")
        es = "-" if exp < 0 else "+"
        return f"{sign}{m}e{es}{abs(exp):02d}"
    if dp <= 0:
        return f"{sign}0.{'0' * (-dp)}{digits}"
    if dp >= nd:
        return f"{sign}{digits}{'0' * (dp - nd)}"
    return f"{sign}{digits[:dp]}.{digits[dp:]}"


def go_v(v) -> str:
    """fmt.Sprintf("%v", v) of a decoded column value (nil, bool, int64, float64 or string)."""
    if v is None:
        return "<nil>"
    if isinstance(v, (bool, np.bool_)):
        return "true" if v else "false"
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, (float, np.floating)):
        return go_v_float(float(v))
    return str(v)


def group_key_string(values: Sequence) -> str:
    """aggregate_operator.go:49-56: the key of one row."""
    return "".join(go_v(v) + "," for v in values)


def _factorize_dense(a):
    """(codes, uniques) of a nil-free array, uniques in first-seen order: pandas.factorize when pandas is importable
    (hashing in C), numpy otherwise (a sort: np.unique, then the first-seen order restored).
    A float array is keyed by its bit patterns: -0.0 and 0.0 are two keys, as their %v strings "-0" and "0" are in the
    reference's group key, while every NaN is one ("NaN")."""
    if isinstance(a, np.ndarray) and a.dtype.kind == "f":
        bits = np.ascontiguousarray(a, dtype=np.float64).view(np.int64).copy()
        bits[np.isnan(a)] = np.array([np.nan], np.float64).view(np.int64)[0]
        codes, ub = _factorize_dense(bits)
        return codes, np.asarray(np.asarray(ub, np.int64).view(np.float64), dtype=object)
    try:
        import pandas as pd
    except ImportError:
        pd = None
    if pd is not None:
        codes, uniques = pd.factorize(a, use_na_sentinel=False)
        return np.asarray(codes, np.int64), np.asarray(uniques, dtype=object)
    if len(a) == 0:
        return np.zeros(0, np.int64), np.zeros(0, dtype=object)
    uniq, first, inv = np.unique(a, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")
    rank = np.empty(len(order), np.int64)
    rank[order] = np.arange(len(order))
    return rank[np.asarray(inv).reshape(-1)], np.asarray(uniq[order], dtype=object)


def _factorize(col, valid=None):
    """(codes, uniques) of a column: uniques in first-seen order over the non-nil rows, codes[i] = -1 for nil rows
    (None, or validity 0). The dictionaries below loop over the distinct values only, not over the rows.
    An object column holding values of several Python types is keyed by their Go %v strings (the reference's group
    key, aggregate_operator.go:49-56): Python-equal values of different types (True == 1 == 1.0) are one key only
    where Go prints them alike (1 and 1.0 both print "1", true does not)."""
    a = col if isinstance(col, np.ndarray) and col.dtype.kind in "iuf" else np.asarray(col, dtype=object)
    n = len(a)
    keep = None
    if valid is not None:
        keep = np.asarray(valid, np.uint8) != 0
    if a.dtype == object:
        nn = np.not_equal(a, None)
        keep = nn if keep is None else keep & nn
        live = a if keep.all() else a[keep]
        types = {type(x) for x in live}
        if len(types) > 1:
            a = np.array([None if x is None else go_v(x) for x in a], dtype=object)
        elif types and issubclass(next(iter(types)), (float, np.floating)):
            a = np.array([np.nan if x is None else x for x in a], dtype=np.float64)   # bit-pattern keys (-0 vs 0)
    if keep is None or keep.all():
        return _factorize_dense(a)
    idx = np.nonzero(keep)[0]
    sub, uniques = _factorize_dense(a[idx])
    codes = np.full(n, -1, np.int64)
    codes[idx] = sub
    return codes, uniques


def _first_rows(codes: np.ndarray) -> np.ndarray:
    """First row of every code of a first-seen-order factorisation: the rows where the running max of the codes
    grows (nil rows carry -1 and never do)."""
    if len(codes) == 0:
        return np.zeros(0, np.int64)
    run = np.maximum.accumulate(codes)
    grow = np.empty(len(codes), bool)
    grow[0] = codes[0] >= 0
    grow[1:] = run[1:] > run[:-1]
    return np.nonzero(grow)[0]


class StringDict:
    """Dense u32 codes of a string column (first-seen order). Rows that are nil (None, or validity 0) take the
    placeholder code 0 and are not entered in the dictionary (the engine never reads a nil row's value)."""

    def __init__(self):
        self.ids: Dict[str, int] = {}
        self.values: List[str] = []

    def encode(self, col, valid=None) -> np.ndarray:
        codes, uniq = _factorize(col, valid)
        ids = self.ids
        m = np.zeros(len(uniq) + 1, np.uint32)       # slot -1 (nil) -> placeholder 0
        for u in range(len(uniq)):                    # first-seen order
            s = uniq[u]
            c = ids.get(s)
            if c is None:
                c = ids[s] = len(self.values)
                self.values.append(s)
            m[u] = c
        return m[codes]

    def decode(self, codes) -> List[str]:
        return [self.values[int(c)] for c in codes]


class OrderedStringDict:
    """Order-preserving int64 codes of a string column whose min / max the rule aggregates
    (internal/binder/function/common_array_funcs.go:49,86: Go compares strings bytewise, which for UTF-8 is code point
    order, i.e. Python's str order). Codes already on the device never change, so the engine's integer min / max over
    codes is the lexicographic min / max.

    Placement of a new string between its sorted neighbours' codes (lo, hi) — codes live in +-2^62:
      * past either end, or right after / before the previously inserted string (a monotone run: ISO timestamps,
        sequence ids, sorted names), the new code takes a share of the gap next to that neighbour that halves with
        every step of the run down to 2^-20, so the rest of the gap stays open for the run: tens of millions of
        strings of one monotone run fit;
      * anywhere else it takes the midpoint.
    Only an adversarial order (e.g. a zig-zag converging on one point, ~60 levels deep) can exhaust a gap; that
    raises ValueError rather than re-coding values already pushed to the device. Nil rows (None, or validity 0)
    take the placeholder code 0 and are not entered in the dictionary."""

    LO, HI = -(1 << 62), 1 << 62
    RUN_SHIFT = 20

    def __init__(self):
        self.code: Dict[str, int] = {}
        self.sorted: List[str] = []
        self.codes: List[int] = []          # codes of self.sorted, ascending
        self.by_code: Dict[int, str] = {}
        self._last: Optional[str] = None     # the string inserted last (monotone-run detection)
        self._dir, self._run = 0, 0          # direction and length of the current run

    def _add(self, s: str) -> int:
        import bisect
        i = bisect.bisect_left(self.sorted, s)
        lo = self.codes[i - 1] if i > 0 else self.LO
        hi = self.codes[i] if i < len(self.codes) else self.HI
        gap = hi - lo
        if gap < 2:
            raise ValueError("ordered string dictionary: no code left between the neighbours of %r "
                             "(adversarial insertion order)" % s)
        ascending = i == len(self.sorted) or (i > 0 and self.sorted[i - 1] == self._last)
        descending = i == 0 or (i < len(self.sorted) and self.sorted[i] == self._last)
        run = self._run + 1 if (ascending and self._dir > 0) or (descending and self._dir < 0) else 0
        step = max(1, gap >> min(self.RUN_SHIFT, run + 1))   # midpoint first; a growing run takes ever less
        if not self.sorted:
            c, self._dir = 0, 0
        elif ascending:
            c, self._dir = lo + step, 1
        elif descending:
            c, self._dir = hi - step, -1
        else:
            c, self._dir, run = lo + gap // 2, 0, 0
        self._run = run
        self.sorted.insert(i, s)
        self.codes.insert(i, c)
        self.code[s] = c
        self.by_code[c] = s
        self._last = s
        return c

    def encode(self, col, valid=None) -> np.ndarray:
        codes, uniq = _factorize(col, valid)
        code = self.code
        m = np.zeros(len(uniq) + 1, np.int64)        # slot -1 (nil) -> placeholder 0
        for u in range(len(uniq)):                    # insertion in first-seen order
            s = uniq[u]
            c = code.get(s)
            m[u] = c if c is not None else self._add(s)
        return m[codes]

    def decode(self, codes) -> List[str]:
        return [self.by_code[int(c)] for c in codes]

    @property
    def values(self):
        return _ByCode(self.by_code)


class _ByCode:
    def __init__(self, by_code):
        self.by_code = by_code

    def __getitem__(self, c):
        return self.by_code[int(c)]


def _canon_bits(col: np.ndarray) -> np.ndarray:
    """Value identity of a numeric column as int64: floats by bit pattern (so -0 and 0 stay apart, as "%v" prints
    them apart) with every NaN folded into one pattern ("NaN")."""
    if col.dtype.kind == "f":
        c = np.array(col, np.float64)
        b = c.view(np.int64).copy()
        b[np.isnan(c)] = 0x7FF8000000000000
        return b
    return np.asarray(col).astype(np.int64)


class GroupKeyDict:
    """Dense ids of GROUP BY keys over `dims` (names, in GROUP BY order) with their schema types
    ("bigint" | "float" | "key" | "string"). `capacity` bounds the ids (the plan's num_keys)."""

    def __init__(self, dims: Sequence[str], types: Sequence[str], capacity: int):
        self.dims = list(dims)
        self.types = list(types)
        self.capacity = int(capacity)
        self.by_string = any(t == "string" for t in self.types)
        self.ids: Dict[object, int] = {}
        self.first: List[tuple] = []      # id -> first row's dimension values

    def __len__(self):
        return len(self.first)

    def _new(self, k, vals) -> int:
        i = len(self.first)
        if i >= self.capacity:
            raise OverflowError(f"GROUP BY dictionary full ({self.capacity} keys): raise num_keys")
        self.ids[k] = i
        self.first.append(tuple(vals))
        return i

    def encode(self, cols: Sequence, valids: Optional[Sequence] = None) -> np.ndarray:
        """cols: one array per dimension (numbers, or python strings for string dims); valids: optional u8 masks
        (0 = nil). Returns the u32 key column."""
        n = len(cols[0]) if cols else 0
        valids = list(valids) if valids is not None else [None] * len(cols)
        vals = []
        for c, v, t in zip(cols, valids, self.types):
            if t == "string":
                a = np.asarray(c, dtype=object)
            elif t == "float":
                a = np.asarray(c, np.float64)
            else:
                a = np.asarray(c).astype(np.int64)
            vals.append((a, None if v is None else np.asarray(v, np.uint8)))
        out = np.empty(n, np.uint32)
        if self.by_string:
            # one code per dimension (nil its own code), the rows' code tuples factorised, and the key string built
            # once per distinct tuple in first-seen order (distinct tuples can still share a string: "%v," collisions)
            if n == 0:
                return out
            comb = np.zeros(n, np.int64)
            for a, m in vals:
                codes, uniq = _factorize(a if a.dtype == object else _canon_bits(a), m)
                card = len(uniq) + 1
                if int(comb.max()) + 1 > (1 << 62) // card:
                    comb = _factorize(comb)[0]   # re-densify before the product could overflow
                comb = comb * card + (codes + 1)
            tcodes, _ = _factorize(comb)
            tfirst = _first_rows(tcodes)
            m_id = np.empty(len(tfirst), np.uint32)
            for u in range(len(tfirst)):                # first-seen order
                i = int(tfirst[u])
                row = tuple(None if (mm is not None and not mm[i]) else (a[i].item() if hasattr(a[i], "item") else a[i])
                            for a, mm in vals)
                k = group_key_string(row)
                j = self.ids.get(k)
                m_id[u] = self._new(k, row) if j is None else j
            out[:] = m_id[tcodes]
            return out
        # numeric dimensions: key on the value tuples (nil -> its own value)
        fields = []
        for a, m in vals:
            b = _canon_bits(a)
            nil = np.zeros(n, np.int64) if m is None else (m == 0).astype(np.int64)
            if m is not None:
                b = np.where(m == 0, 0, b)
            fields += [nil, b]
        rec = np.rec.fromarrays(fields) if fields else np.zeros(n)
        uniq, first_idx, inv = np.unique(rec, return_index=True, return_inverse=True)
        order = np.argsort(first_idx, kind="stable")          # first-seen order inside the batch
        uid = np.empty(len(uniq), np.uint32)
        for u in order:
            key = tuple(int(x) for x in uniq[u])
            j = self.ids.get(key)
            if j is None:
                i0 = first_idx[u]
                row = tuple(None if (m is not None and not m[i0]) else a[i0].item() for a, m in vals)
                j = self._new(key, row)
            uid[u] = j
        out[:] = uid[inv.reshape(-1)]
        return out

    def decode(self, ids) -> List[tuple]:
        return [self.first[int(i)] for i in ids]
