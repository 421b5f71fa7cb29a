/*
 * ekoracle.c — CPU ORACLE for parity testing (test infrastructure only; see ekoracle.h).
 *
 * Restates, event by event, the reference's operator chain for a windowed GROUP BY rule:
 *   WatermarkOp       internal/topo/node/watermark_op.go:144-225
 *   WindowOperator    internal/topo/node/event_window_trigger.go:57-209, window_op.go:194-227,390-418,
 *                     502-551,553-574,605-739
 *   FilterOp          internal/topo/operator/filter_operator.go:36-90
 *   AggregateOp       internal/topo/operator/aggregate_operator.go:34-82
 *   HavingOp          internal/topo/operator/having_operator.go:32-104
 *   aggregates        internal/binder/function/funcs_agg.go:28-428, common_array_funcs.go:27-247,
 *                     function.go:155-171 (check guard), pkg/cast/cast.go:322-420,915-966,
 *                     github.com/montanaflynn/stats v0.7.1 (Mean/Variance/Percentile/PercentileNearestRank,
 *                     restated from the library's published source; not vendored in the reference)
 *   expressions       internal/xsql/valuer.go:574-660 (evalBinaryExpr), 823-1000 (SimpleDataEval)
 *
 * Compiled with -ffp-contract=off so that every floating-point operation rounds like Go's.
 */
#include "ekoracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* Go's time.Time{} (year 1) in Unix ms, used for IsZero() comparisons. */
#define ZERO_MS (-62135596800000LL)
/* pkg/timex/time.go:28 Maxtime = 9999-12-31T23:59:59.999999999Z (ms, rounded up) */
#define MAXT_MS (253402300800000LL)

/* ------------------------------------------------------------------ vectors */
typedef struct { int64_t* a; int64_t n, cap; } vec64;
static void v_push(vec64* v, int64_t x) {
    if (v->n == v->cap) { v->cap = v->cap ? v->cap * 2 : 64; v->a = (int64_t*)realloc(v->a, (size_t)v->cap * 8); }
    v->a[v->n++] = x;
}
static void v_erase_front(vec64* v, int64_t k) {
    if (k <= 0) return;
    if (k >= v->n) { v->n = 0; return; }
    memmove(v->a, v->a + k, (size_t)(v->n - k) * 8);
    v->n -= k;
}

/* ------------------------------------------------------------------ time */
static int64_t floordiv(int64_t a, int64_t b) { int64_t q = a / b; if ((a % b) != 0 && ((a < 0) != (b < 0))) q--; return q; }

int64_t eko_aligned_window_end(int64_t ts_ms, int32_t interval, int32_t unit, int32_t tz_offset_s) {
    /* window_op.go:194-227 */
    int64_t off = (int64_t)tz_offset_s * 1000;
    int64_t local = ts_ms + off;
    int64_t day0 = floordiv(local, 86400000LL) * 86400000LL;
    int64_t gap = interval;
    switch (unit) {
    case EK_UNIT_DD:
        return day0 + (int64_t)interval * 86400000LL - off;
    case EK_UNIT_HH: {
        int64_t hour = (local - day0) / 3600000LL;
        if (hour > interval) gap = (int64_t)interval * (hour / interval + 1);
        return day0 + gap * 3600000LL - off;
    }
    case EK_UNIT_MI: {
        int64_t h0 = floordiv(local, 3600000LL) * 3600000LL;
        int64_t minute = (local - h0) / 60000LL;
        if (minute > interval) gap = (int64_t)interval * (minute / interval + 1);
        return h0 + gap * 60000LL - off;
    }
    case EK_UNIT_SS: {
        int64_t m0 = floordiv(local, 60000LL) * 60000LL;
        int64_t sec = (local - m0) / 1000LL;
        if (sec > interval) gap = (int64_t)interval * (sec / interval + 1);
        return m0 + gap * 1000LL - off;
    }
    case EK_UNIT_MS: {
        int64_t s0 = floordiv(local, 1000LL) * 1000LL;
        int64_t milli = local - s0;
        if (milli > interval) gap = (int64_t)interval * (milli / interval + 1);
        return s0 + gap - off;
    }
    default:
        return ts_ms;
    }
}

static int64_t unit_ms(int32_t unit) {
    /* planner.go:463-478 convertFromDuration */
    switch (unit) {
    case EK_UNIT_DD: return 86400000LL;
    case EK_UNIT_HH: return 3600000LL;
    case EK_UNIT_MI: return 60000LL;
    case EK_UNIT_SS: return 1000LL;
    case EK_UNIT_MS: return 1LL;
    }
    return 1000LL;
}

/* ------------------------------------------------------------------ values */
enum { V_NULL = 0, V_BOOL = 1, V_I64 = 2, V_F64 = 3, V_ERR = 4 };
typedef struct { int tag; int64_t i; double f; } val_t;

typedef struct {
    const ek_plan* p;
    int64_t n;
    const void* const* cols;
    const uint8_t* const* valid;
    const int64_t* arrival;    /* shard model: global arrival index of each row (NULL: row index = arrival) */
} dataset;

static int64_t row_arrival(const dataset* d, int64_t e) { return d->arrival ? d->arrival[e] : e; }

static val_t eval_prog(const ek_instr* prog, int n, const dataset* d, int64_t row, const val_t* aggs);

/* column c of a row; c in [n_columns, n_columns + n_derived) is an aggregate argument expression, evaluated on the
 * row like GroupedTuples.AggregateEval (internal/xsql/row.go:712-718) */
static val_t col_val(const dataset* d, int c, int64_t row) {
    val_t v; v.tag = V_NULL; v.i = 0; v.f = 0;
    if (c >= d->p->n_columns && c < d->p->n_columns + d->p->n_derived) {
        const int k = c - d->p->n_columns;
        v = eval_prog(d->p->derived_prog[k], d->p->n_derived_prog[k], d, row, NULL);
        if (v.tag != V_I64 && v.tag != V_F64) { v.tag = V_NULL; v.i = 0; v.f = 0; }
        return v;
    }
    if (c < 0 || c >= d->p->n_columns || !d->cols[c]) return v;
    if (d->valid && d->valid[c] && !d->valid[c][row]) return v;
    switch (d->p->column_type[c]) {
    case EK_COL_I64: v.tag = V_I64; v.i = ((const int64_t*)d->cols[c])[row]; break;
    case EK_COL_U32: v.tag = V_I64; v.i = ((const uint32_t*)d->cols[c])[row]; break;
    case EK_COL_F64: v.tag = V_F64; v.f = ((const double*)d->cols[c])[row]; break;
    case EK_COL_BOOL: v.tag = V_BOOL; v.i = ((const int64_t*)d->cols[c])[row] != 0; break;   /* Go bool */
    }
    return v;
}

static val_t mk_bool(int b) { val_t v; v.tag = V_BOOL; v.i = b ? 1 : 0; v.f = 0; return v; }
static val_t mk_null(void) { val_t v; v.tag = V_NULL; v.i = 0; v.f = 0; return v; }

/* ------------------------------------------------------------------ error texts
 * An error value carries its text (v.i indexes a ring of texts, enough for one program's evaluation): valuer.go's
 * "divided by zero" (:897-979) and invalidOpError "invalid operation %T(%v) %s %T(%v)" (:1243-1245) with the
 * ast.Tokens spellings (pkg/ast/token.go:135-193). Go's %v of a float64 is strconv.FormatFloat(f, 'g', -1, 64):
 * the shortest round-trip digits, exponent form when the decimal exponent is below -4 or at least 6
 * (strconv/ftoa.go %g with the shortest precision), e.g. 2.5, 123456, 1.234567e+06, 1e-05. */
static char eko_errtab[64][160];
static unsigned eko_errn;
static val_t mk_err_text(const char* fmt, ...) {
    const unsigned k = (eko_errn++) & 63u;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(eko_errtab[k], sizeof eko_errtab[k], fmt, ap);
    va_end(ap);
    val_t v; v.tag = V_ERR; v.i = (int64_t)k; v.f = 0;
    return v;
}
static const char* err_text(val_t v) { return eko_errtab[v.i & 63]; }
static void go_float_v(char* out, size_t cap, double x) {
    if (x != x) { snprintf(out, cap, "NaN"); return; }
    if (isinf(x)) { snprintf(out, cap, x > 0 ? "+Inf" : "-Inf"); return; }
    if (x == 0) { snprintf(out, cap, signbit(x) ? "-0" : "0"); return; }
    char e[48];
    for (int prec = 0; prec < 17; ++prec) {   /* shortest %.{prec}e that reads back as x */
        snprintf(e, sizeof e, "%.*e", prec, x);
        if (strtod(e, NULL) == x) break;
    }
    /* e = [-]D[.DDD]e(+|-)XX: digits without the point, decimal exponent */
    char dig[32];
    int nd = 0, neg = e[0] == '-';
    const char* q = e + neg;
    for (; *q && *q != 'e'; ++q) if (*q != '.') dig[nd++] = *q;
    while (nd > 1 && dig[nd - 1] == '0') --nd;
    dig[nd] = 0;
    const int x10 = atoi(q + 1);
    char* o = out;
    size_t left = cap;
#define EKO_PUT(...) do { int m_ = snprintf(o, left, __VA_ARGS__); if (m_ < 0 || (size_t)m_ >= left) return; o += m_; left -= (size_t)m_; } while (0)
    if (neg) EKO_PUT("-");
    if (x10 < -4 || x10 >= 6) {
        EKO_PUT("%c", dig[0]);
        if (nd > 1) EKO_PUT(".%s", dig + 1);
        EKO_PUT("e%c%02d", x10 < 0 ? '-' : '+', x10 < 0 ? -x10 : x10);
    } else if (x10 < 0) {
        EKO_PUT("0.");
        for (int k = 0; k < -x10 - 1; ++k) EKO_PUT("0");
        EKO_PUT("%s", dig);
    } else {
        for (int k = 0; k <= x10 || k < nd; ++k) {
            if (k == x10 + 1) EKO_PUT(".");
            EKO_PUT("%c", k < nd ? dig[k] : '0');
        }
    }
#undef EKO_PUT
}
/* %T(%v) of a value */
static void go_typed(char* out, size_t cap, val_t v) {
    char f[48];
    switch (v.tag) {
    case V_BOOL: snprintf(out, cap, "bool(%s)", v.i ? "true" : "false"); break;
    case V_I64: snprintf(out, cap, "int64(%lld)", (long long)v.i); break;
    case V_F64: go_float_v(f, sizeof f, v.f); snprintf(out, cap, "float64(%s)", f); break;
    default: snprintf(out, cap, "<nil>(<nil>)"); break;
    }
}
static const char* go_token(int op) {
    static const char* t[] = {"", "", "", "", "", "=", "!=", "<", "<=", ">", ">=", "AND", "OR", "+", "-", "*", "/", "%"};
    return op >= 0 && op <= EK_OP_MOD ? t[op] : "?";
}
static val_t invalid_op(val_t l, int op, val_t r) {
    char a[64], b[64];
    go_typed(a, sizeof a, l);
    go_typed(b, sizeof b, r);
    return mk_err_text("invalid operation %s %s %s", a, go_token(op), b);
}
static val_t div_zero(void) { return mk_err_text("divided by zero"); }

/* valuer.go:823-1000 SimpleDataEval for the op subset of the plan ISA */
static val_t simple_eval(val_t l, val_t r, int op) {
    if (l.tag == V_NULL || r.tag == V_NULL) {
        switch (op) {
        case EK_OP_AND: case EK_OP_OR: case EK_OP_EQ: case EK_OP_NEQ: case EK_OP_GT: case EK_OP_GTE:
        case EK_OP_LT: case EK_OP_LTE:
            return mk_bool(0);
        default:
            return mk_null();
        }
    }
    if (l.tag == V_BOOL) {
        if (r.tag != V_BOOL) return invalid_op(l, op, r);
        switch (op) {
        case EK_OP_AND: return mk_bool(l.i && r.i);
        case EK_OP_OR: return mk_bool(l.i || r.i);
        case EK_OP_EQ: return mk_bool(l.i == r.i);
        case EK_OP_NEQ: return mk_bool(l.i != r.i);
        default: return invalid_op(l, op, r);
        }
    }
    if (r.tag == V_BOOL) return invalid_op(l, op, r);
    if (l.tag == V_F64 || r.tag == V_F64) {
        double a = l.tag == V_F64 ? l.f : (double)l.i;
        double b = r.tag == V_F64 ? r.f : (double)r.i;
        val_t v; v.tag = V_F64; v.i = 0;
        switch (op) {
        case EK_OP_EQ: return mk_bool(a == b);
        case EK_OP_NEQ: return mk_bool(a != b);
        case EK_OP_LT: return mk_bool(a < b);
        case EK_OP_LTE: return mk_bool(a <= b);
        case EK_OP_GT: return mk_bool(a > b);
        case EK_OP_GTE: return mk_bool(a >= b);
        case EK_OP_ADD: v.f = a + b; return v;
        case EK_OP_SUB: v.f = a - b; return v;
        case EK_OP_MUL: v.f = a * b; return v;
        case EK_OP_DIV: if (b == 0) return div_zero(); v.f = a / b; return v;
        case EK_OP_MOD: if (b == 0) return div_zero(); v.f = fmod(a, b); return v;
        default: { val_t lf = v, rf = v; lf.f = a; rf.f = b; return invalid_op(lf, op, rf); }
        }
    }
    {
        int64_t a = l.i, b = r.i;
        val_t v; v.tag = V_I64; v.f = 0;
        switch (op) {
        case EK_OP_EQ: return mk_bool(a == b);
        case EK_OP_NEQ: return mk_bool(a != b);
        case EK_OP_LT: return mk_bool(a < b);
        case EK_OP_LTE: return mk_bool(a <= b);
        case EK_OP_GT: return mk_bool(a > b);
        case EK_OP_GTE: return mk_bool(a >= b);
        case EK_OP_ADD: v.i = (int64_t)((uint64_t)a + (uint64_t)b); return v;
        case EK_OP_SUB: v.i = (int64_t)((uint64_t)a - (uint64_t)b); return v;
        case EK_OP_MUL: v.i = (int64_t)((uint64_t)a * (uint64_t)b); return v;
        case EK_OP_DIV: if (b == 0) return div_zero(); v.i = (a == INT64_MIN && b == -1) ? a : a / b; return v;
        case EK_OP_MOD: if (b == 0) return div_zero(); v.i = (b == -1) ? 0 : a % b; return v;
        default: return invalid_op(l, op, r);
        }
    }
}

/* Postfix evaluation equivalent to the tree walk of valuer.go:574-660 (AND/OR short-circuit on
 * a decided lhs is reproduced: a false lhs of AND / true lhs of OR wins over an rhs error). */
static val_t eval_prog(const ek_instr* prog, int n, const dataset* d, int64_t row, const val_t* aggs) {
    val_t st[EK_MAX_PROG];
    int sp = 0;
    for (int k = 0; k < n; ++k) {
        const ek_instr* in = &prog[k];
        switch (in->op) {
        case EK_OP_COL: st[sp++] = col_val(d, in->arg, row); break;
        case EK_OP_AGG: st[sp++] = aggs ? aggs[in->arg] : mk_null(); break;
        case EK_OP_CONST_I64: { val_t v; v.tag = V_I64; v.i = in->i64; v.f = 0; st[sp++] = v; } break;
        case EK_OP_CONST_F64: { val_t v; v.tag = V_F64; v.i = 0; v.f = in->f64; st[sp++] = v; } break;
        case EK_OP_CONST_BOOL: st[sp++] = mk_bool(in->i64 != 0); break;   /* ast.BooleanLiteral */
        default: {
            if (sp < 2) return mk_err_text("malformed program");
            val_t r = st[--sp], l = st[--sp], res;
            if (l.tag == V_ERR) res = l;
            else if (in->op == EK_OP_AND && l.tag == V_BOOL && !l.i) res = mk_bool(0);
            else if (in->op == EK_OP_OR && l.tag == V_BOOL && l.i) res = mk_bool(1);
            else if (r.tag == V_ERR) res = r;
            else res = simple_eval(l, r, in->op);
            st[sp++] = res;
        }
        }
    }
    return sp ? st[sp - 1] : mk_null();
}

/* ------------------------------------------------------------------ aggregates */
static int cmp_f64(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    /* sort.Float64s order (NaN first); ties keep no particular order (value-equal) */
    int xn = x != x, yn = y != y;
    if (xn || yn) return yn - xn;
    return (x < y) ? -1 : (x > y) ? 1 : 0;
}
static int cmp_i64(const void* a, const void* b) {
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return (x < y) ? -1 : (x > y) ? 1 : 0;
}

typedef struct { int tag; int64_t i; double f; int err; char msg[160]; } agg_out;

static void set_err(agg_out* o, const char* fmt, ...) {
    va_list ap; va_start(ap, fmt); vsnprintf(o->msg, sizeof o->msg, fmt, ap); va_end(ap);
    o->err = 1; o->tag = EK_TAG_NULL;
}

/* vals: typed values of the argument column over the group rows in window order, vnull[i] = 1 if nil */
static void agg_eval(int fn, int is_float, int64_t n, const int64_t* iv, const double* fv, const uint8_t* vnull,
                     double param, agg_out* o) {
    memset(o, 0, sizeof *o);
    o->tag = EK_TAG_NULL;
    int64_t cnt = 0, first = -1;
    for (int64_t k = 0; k < n; ++k) if (!vnull[k]) { if (first < 0) first = k; cnt++; }
    switch (fn) {
    case EK_AGG_COUNT_STAR: o->tag = EK_TAG_I64; o->i = n; return;
    case EK_AGG_FIRST:                                                 /* row.go:720-726: the group's first row */
        if (n == 0 || vnull[0]) return;                                /* nil */
        if (is_float) { o->tag = EK_TAG_F64; o->f = fv[0]; } else { o->tag = EK_TAG_I64; o->i = iv[0]; }
        return;
    case EK_AGG_COUNT: o->tag = EK_TAG_I64; o->i = cnt; return;        /* getCount */
    case EK_AGG_SUM:                                                   /* funcs_agg.go:114-143 */
    case EK_AGG_AVG: {                                                 /* funcs_agg.go:56-86 */
        if (n == 0 || first < 0) return;                              /* nil */
        if (!is_float) {
            int64_t t = 0;
            for (int64_t k = 0; k < n; ++k) if (!vnull[k]) t = (int64_t)((uint64_t)t + (uint64_t)iv[k]);
            o->tag = EK_TAG_I64;
            o->i = (fn == EK_AGG_SUM) ? t : ((t == INT64_MIN && cnt == -1) ? t : t / cnt);
        } else {
            double t = 0;
            for (int64_t k = 0; k < n; ++k) if (!vnull[k]) t += fv[k];
            o->tag = EK_TAG_F64;
            o->f = (fn == EK_AGG_SUM) ? t : t / (double)cnt;
        }
        return;
    }
    case EK_AGG_MIN:
    case EK_AGG_MAX: {                                                 /* common_array_funcs.go:27-247 */
        if (first < 0) return;
        if (!is_float) {
            int64_t m = iv[first];
            for (int64_t k = 0; k < n; ++k) if (!vnull[k]) {
                if (fn == EK_AGG_MAX ? (iv[k] > m) : (iv[k] < m)) m = iv[k];
            }
            o->tag = EK_TAG_I64; o->i = m;
        } else {
            double m = fv[first];
            for (int64_t k = 0; k < n; ++k) if (!vnull[k]) {
                if (fn == EK_AGG_MAX ? (m < fv[k]) : (m > fv[k])) m = fv[k];
            }
            o->tag = EK_TAG_F64; o->f = m;
        }
        return;
    }
    case EK_AGG_STDDEV: case EK_AGG_STDDEVS: case EK_AGG_VAR: case EK_AGG_VARS: {
        /* cast.ToFloat64Slice(IGNORE_NIL) then stats v0.7.1 _variance: mean = Sum/len (sequential),
         * Σ (x-m)*(x-m) sequential, / len or / (len-1); empty -> EmptyInputErr -> nil */
        if (cnt == 0) return;
        double s = 0;
        for (int64_t k = 0; k < n; ++k) if (!vnull[k]) s += is_float ? fv[k] : (double)iv[k];
        double m = s / (double)cnt, v = 0;
        for (int64_t k = 0; k < n; ++k) if (!vnull[k]) {
            double x = is_float ? fv[k] : (double)iv[k];
            double dx = x - m;
            v += dx * dx;
        }
        int sample = (fn == EK_AGG_STDDEVS || fn == EK_AGG_VARS);
        v = v / (double)(cnt - sample);
        if (fn == EK_AGG_STDDEV || fn == EK_AGG_STDDEVS) v = sqrt(v);
        o->tag = EK_TAG_F64; o->f = v;
        return;
    }
    case EK_AGG_MEDIAN: {                                              /* funcs_agg.go:29-55,415-428 */
        if (n < 1) { o->tag = EK_TAG_I64; o->i = 0; return; }
        if (vnull[0]) { set_err(o, "<nil> should be number"); return; }
        if (is_float) {
            double* a = (double*)malloc((size_t)cnt * 8); int64_t m = 0;
            for (int64_t k = 0; k < n; ++k) if (!vnull[k]) a[m++] = fv[k];
            qsort(a, (size_t)m, 8, cmp_f64);
            if (m % 2 == 1) { o->tag = EK_TAG_F64; o->f = a[m / 2]; }
            else { o->tag = EK_TAG_F64; o->f = (a[m / 2 - 1] + a[m / 2]) / 2; }
            free(a);
        } else {
            if (cnt != n) { set_err(o, "cannot convert <nil> to int64"); return; } /* ToInt64Slice SAMEKIND */
            int64_t* a = (int64_t*)malloc((size_t)n * 8);
            memcpy(a, iv, (size_t)n * 8);
            qsort(a, (size_t)n, 8, cmp_i64);
            if (n % 2 == 1) { o->tag = EK_TAG_I64; o->i = a[n / 2]; }
            else { o->tag = EK_TAG_F64; o->f = (double)(int64_t)((uint64_t)a[n / 2 - 1] + (uint64_t)a[n / 2]) / 2; }
            free(a);
        }
        return;
    }
    case EK_AGG_PERCENTILE_CONT:
    case EK_AGG_PERCENTILE_DISC: {
        if (cnt == 0) return;                                          /* EmptyInputErr -> nil */
        double percent = param * 100;
        double* c = (double*)malloc((size_t)cnt * 8); int64_t m = 0;
        for (int64_t k = 0; k < n; ++k) if (!vnull[k]) c[m++] = is_float ? fv[k] : (double)iv[k];
        if (fn == EK_AGG_PERCENTILE_CONT) {
            /* stats.Percentile v0.7.1 */
            if (m == 1) { o->tag = EK_TAG_F64; o->f = c[0]; free(c); return; }
            if (percent <= 0 || percent > 100) { set_err(o, "percentile exec with error: Input is outside of range."); free(c); return; }
            qsort(c, (size_t)m, 8, cmp_f64);
            double index = (percent / 100) * (double)m;
            if (index == (double)(int64_t)index) {
                int64_t i = (int64_t)index;
                o->tag = EK_TAG_F64; o->f = c[i - 1];
            } else if (index > 1) {
                int64_t i = (int64_t)index;
                double s = 0; s += c[i - 1]; s += c[i];
                o->tag = EK_TAG_F64; o->f = s / 2;
            } else {
                set_err(o, "percentile exec with error: Input is outside of range.");
            }
        } else {
            /* stats.PercentileNearestRank v0.7.1 */
            if (percent < 0 || percent > 100) { set_err(o, "PopulationVariance exec with error: Input is outside of range."); free(c); return; }
            qsort(c, (size_t)m, 8, cmp_f64);
            if (percent == 100.0) { o->tag = EK_TAG_F64; o->f = c[m - 1]; free(c); return; }
            int64_t r = (int64_t)ceil((double)m * percent / 100);
            o->tag = EK_TAG_F64; o->f = (r == 0) ? c[0] : c[r - 1];
        }
        free(c);
        return;
    }
    }
    set_err(o, "unsupported aggregate %d", fn);
}

int eko_agg_exec(int32_t fn, int32_t col_type, int64_t n, const void* values, const uint8_t* valid,
                 double param, int64_t* out_value, uint8_t* out_tag, char* err, int32_t err_len) {
    int is_float = col_type == EK_COL_F64;
    int64_t* iv = (int64_t*)calloc((size_t)(n ? n : 1), 8);
    double* fv = (double*)calloc((size_t)(n ? n : 1), 8);
    uint8_t* nul = (uint8_t*)calloc((size_t)(n ? n : 1), 1);
    for (int64_t k = 0; k < n; ++k) {
        nul[k] = valid ? !valid[k] : 0;
        if (is_float) fv[k] = ((const double*)values)[k];
        else if (col_type == EK_COL_U32) iv[k] = ((const uint32_t*)values)[k];
        else iv[k] = ((const int64_t*)values)[k];
    }
    agg_out o;
    agg_eval(fn, is_float, n, iv, fv, nul, param, &o);
    free(iv); free(fv); free(nul);
    if (o.err) { if (err && err_len > 0) snprintf(err, (size_t)err_len, "%s", o.msg); *out_tag = EK_TAG_NULL; return 1; }
    *out_tag = (uint8_t)o.tag;
    if (o.tag == EK_TAG_F64) memcpy(out_value, &o.f, 8); else *out_value = o.i;
    return 0;
}

/* ------------------------------------------------------------------ output building */
typedef struct {
    vec64 ws, we, roff, rcnt, st, mcnt, mhash, moff, mem;
    vec64 key;
    vec64 aval[EK_MAX_AGGS];
    vec64 atag[EK_MAX_AGGS];
    char* werr; int64_t werr_cap;
} outbuf;

/* Evaluate WHERE -> GROUP BY -> aggregates -> HAVING over one emitted window
 * (filter_operator.go:36-90, aggregate_operator.go:34-82, having_operator.go:32-104,
 *  project_operator.go:79-207 for the aggregate fields). */
#define EKO_MEMBER_CAP ((int64_t)1 << 24)
static void emit_window(const dataset* d, outbuf* ob, int64_t wstart, int64_t wend, const int64_t* content, int64_t nc) {
    const ek_plan* p = d->p;
    int64_t w = ob->ws.n;
    v_push(&ob->ws, wstart);
    v_push(&ob->we, wend);
    v_push(&ob->roff, ob->key.n);
    v_push(&ob->moff, ob->mem.n);
    uint64_t h = 0;
    /* the member lists themselves are kept only while they stay small (KAT-sized runs inspect them); full-size
     * runs compare membership through (count, Σ mix64(arrival)) and would otherwise hold GBs of lists */
    const int keep = ob->mem.n + nc <= EKO_MEMBER_CAP;
    for (int64_t k = 0; k < nc; ++k) {
        const int64_t a = row_arrival(d, content[k]);
        if (keep) v_push(&ob->mem, a);
        h += ek_mix64((uint64_t)a);
    }
    v_push(&ob->mcnt, nc);
    v_push(&ob->mhash, (int64_t)h);
    if (ob->werr_cap <= w) { ob->werr_cap = (w + 1) * 2; ob->werr = (char*)realloc(ob->werr, (size_t)ob->werr_cap * 128); }
    ob->werr[w * 128] = 0;
    int status = EK_WIN_OK;

    /* WHERE (after the window in event time: windowPlan.go:82-99) */
    int64_t* sel = (int64_t*)malloc((size_t)(nc ? nc : 1) * 8);
    int64_t ns = 0;
    for (int64_t k = 0; k < nc; ++k) {
        if (p->n_where <= 0) { sel[ns++] = content[k]; continue; }
        val_t r = eval_prog(p->where_prog, p->n_where, d, content[k], NULL);
        /* FilterOp over the window's rows in order: the first failure is the window's error (filter_operator.go:60-81) */
        if (r.tag == V_ERR) { status = EK_WIN_WHERE_ERROR; snprintf(ob->werr + w * 128, 128, "run Where error: %s", err_text(r)); break; }
        if (r.tag == V_BOOL) { if (r.i) sel[ns++] = content[k]; }
        else if (r.tag != V_NULL) {
            char tv[80];
            go_typed(tv, sizeof tv, r);
            status = EK_WIN_WHERE_ERROR;
            snprintf(ob->werr + w * 128, 128, "run Where error: invalid condition that returns non-bool value %s", tv);
            break;
        }
    }
    int64_t rows_before = ob->key.n;
    if (status == EK_WIN_OK && ns > 0) {
        /* GROUP BY key (first-appearance order; output order is unspecified in the reference) */
        int64_t ng = 0;
        int64_t* gstart = (int64_t*)malloc((size_t)ns * 8);  /* group id per selected row */
        int64_t* gkey = (int64_t*)malloc((size_t)ns * 8);
        int64_t* gcount = (int64_t*)calloc((size_t)ns, 8);
        int64_t* rowg = (int64_t*)malloc((size_t)ns * 8);
        if (p->key_column >= 0) {
            /* open-addressing map key -> group */
            int64_t cap = 16; while (cap < ns * 2) cap <<= 1;
            int64_t* slot = (int64_t*)malloc((size_t)cap * 8);
            for (int64_t k = 0; k < cap; ++k) slot[k] = -1;
            for (int64_t k = 0; k < ns; ++k) {
                val_t kv = col_val(d, p->key_column, sel[k]);
                int64_t key = kv.tag == V_NULL ? -1 : kv.i;
                uint64_t hh = ek_mix64((uint64_t)key) & (uint64_t)(cap - 1);
                while (slot[hh] >= 0 && gkey[slot[hh]] != key) hh = (hh + 1) & (uint64_t)(cap - 1);
                if (slot[hh] < 0) { slot[hh] = ng; gkey[ng] = key; ng++; }
                rowg[k] = slot[hh];
                gcount[slot[hh]]++;
            }
            free(slot);
        } else {
            ng = 1; gkey[0] = 0; gcount[0] = ns;
            for (int64_t k = 0; k < ns; ++k) rowg[k] = 0;
        }
        /* bucket rows per group preserving order */
        int64_t* goff = (int64_t*)calloc((size_t)ng + 1, 8);
        for (int64_t g = 0; g < ng; ++g) goff[g + 1] = goff[g] + gcount[g];
        int64_t* fill = (int64_t*)calloc((size_t)ng, 8);
        int64_t* grows = (int64_t*)malloc((size_t)ns * 8);
        for (int64_t k = 0; k < ns; ++k) { int64_t g = rowg[k]; grows[goff[g] + fill[g]++] = sel[k]; }
        int64_t* iv = (int64_t*)malloc((size_t)ns * 8);
        double* fv = (double*)malloc((size_t)ns * 8);
        uint8_t* nul = (uint8_t*)malloc((size_t)ns);
        val_t aggv[EK_MAX_AGGS];
        agg_out ao[EK_MAX_AGGS];
        /* every group is aggregated: HavingOp's error (any failed group: the reference ranges a Go map, the engine
         * reports the smallest failed key) wins over ProjectOp's (the first failed aggregate slot over the groups) */
        int64_t hkey = INT64_MAX, aslot = EK_MAX_AGGS;
        char htext[128] = "", atext[160] = "";
        for (int64_t g = 0; g < ng; ++g) {
            int64_t gn = goff[g + 1] - goff[g];
            const int64_t* rows = grows + goff[g];
            int gfail = 0;
            for (int a = 0; a < p->n_aggs; ++a) {
                const ek_agg_spec* as = &p->aggs[a];
                int c = as->column;
                int is_float = (c >= 0 && c < p->n_columns) ? (p->column_type[c] == EK_COL_F64)
                             : (c >= p->n_columns && c < p->n_columns + p->n_derived) ? (p->derived_type[c - p->n_columns] == EK_COL_F64) : 0;
                for (int64_t k = 0; k < gn; ++k) {
                    if (as->fn == EK_AGG_COUNT_STAR) { nul[k] = 0; iv[k] = 0; continue; }
                    val_t v = col_val(d, c, rows[k]);
                    nul[k] = v.tag == V_NULL;
                    iv[k] = v.i; fv[k] = v.f;
                }
                agg_eval(as->fn, is_float, gn, iv, fv, nul, as->param, &ao[a]);
                if (ao[a].err) {
                    status |= EK_WIN_AGG_ERROR;
                    if (a < aslot) { aslot = a; snprintf(atext, sizeof atext, "%s", ao[a].msg); }
                    gfail = 1;
                    break;
                }
                aggv[a].tag = ao[a].tag == EK_TAG_NULL ? V_NULL : (ao[a].tag == EK_TAG_I64 ? V_I64 : V_F64);
                aggv[a].i = ao[a].i; aggv[a].f = ao[a].f;
            }
            if (gfail) continue;   /* a failed aggregate: no HAVING, no row for this group */
            if (p->n_having > 0) {
                val_t r = eval_prog(p->having_prog, p->n_having, d, rows[0], aggv);
                if (r.tag != V_BOOL) {
                    status |= EK_WIN_HAVING_ERROR;
                    if (gkey[g] < hkey) {
                        hkey = gkey[g];
                        if (r.tag == V_ERR) snprintf(htext, sizeof htext, "run Having error: %s", err_text(r));
                        else {
                            char tv[80];
                            go_typed(tv, sizeof tv, r);
                            snprintf(htext, sizeof htext, "run Having error: invalid condition that returns non-bool value %s", tv);
                        }
                    }
                    continue;
                }
                if (!r.i) continue;
            }
            v_push(&ob->key, gkey[g]);
            for (int a = 0; a < p->n_aggs; ++a) {
                int64_t bits = ao[a].i;
                if (ao[a].tag == EK_TAG_F64) memcpy(&bits, &ao[a].f, 8);
                v_push(&ob->aval[a], bits);
                v_push(&ob->atag[a], ao[a].tag);
            }
        }
        if (htext[0]) snprintf(ob->werr + w * 128, 128, "%s", htext);
        else if (atext[0]) {
            /* HavingOp meets a failed aggregate it reads before ProjectOp does */
            int in_having = 0;
            for (int k = 0; k < p->n_having; ++k) in_having |= p->having_prog[k].op == EK_OP_AGG && p->having_prog[k].arg == aslot;
            snprintf(ob->werr + w * 128, 128, "%s%s", in_having ? "run Having error: " : "run Select error: ", atext);
        }
        free(gstart); free(gkey); free(gcount); free(rowg); free(goff); free(fill); free(grows);
        free(iv); free(fv); free(nul);
    }
    if (status != EK_WIN_OK) {
        /* the window's output is replaced by the error */
        ob->key.n = rows_before;
        for (int a = 0; a < p->n_aggs; ++a) { ob->aval[a].n = rows_before; ob->atag[a].n = rows_before; }
    }
    free(sel);
    v_push(&ob->rcnt, ob->key.n - rows_before);
    v_push(&ob->st, status);
}

/* ------------------------------------------------------------------ incremental-aggregation windows
 * The planner's opt-in incremental path (planner.go:905-997 rewriteIfIncAggStmt: every aggregate call becomes
 * a scalar inc_<fn> whose running state lives per (window, dimension); node.NewWindowIncAggOp,
 * window_inc_agg_op.go:59-101). Per row of a window, incAggCal (window_inc_agg_op.go:792-809) evaluates every
 * inc_<fn> and OVERWRITES the dimension's Fields with the result, and keeps the row as LastRow; the window
 * emits one row per dimension = LastRow + the Fields of its last evaluation (emit, :768-781). So a group's
 * value is the one computed at its LAST row: a nil argument there makes the field nil (the builtin's `check`
 * returnNilIfHasAnyNil skips exec, function.go:155-170, static_executor.go:59-71), and a nil row never
 * updates the state. State rules (funcs_inc_agg.go:266-325): inc_count +1 per non-nil row -> int64;
 * inc_sum float64 (cast.ToFloat64 CONVERT_ALL, first value taken as is, then prev + arg); inc_avg =
 * inc_sum / inc_count (float64); inc_min / inc_max = min/max over [arg, prev] (funcs_agg.go:96-113). */
typedef struct { int has; int lastnil; int64_t cnt; double fsum; val_t mm; } incstate;

static void inc_step(const dataset* d, int fn, int c, int64_t row, incstate* s) {
    if (fn == EK_AGG_COUNT_STAR) { s->cnt++; s->lastnil = 0; s->has = 1; return; }
    val_t v = col_val(d, c, row);
    if (v.tag == V_NULL) { s->lastnil = 1; return; }
    s->lastnil = 0;
    const double x = v.tag == V_F64 ? v.f : (double)v.i;
    switch (fn) {
    case EK_AGG_COUNT: s->cnt++; break;
    case EK_AGG_SUM: case EK_AGG_AVG:
        s->fsum = s->has ? s->fsum + x : x;
        s->cnt++;
        break;
    case EK_AGG_MIN: case EK_AGG_MAX:
        if (!s->has) s->mm = v;
        else {
            /* min/max(args) with args = [arg, prev] (funcs_inc_agg.go:234-264) */
            int64_t iv[2] = {v.i, s->mm.i};
            double fv[2] = {v.f, s->mm.f};
            uint8_t nul[2] = {0, 0};
            agg_out ao;
            agg_eval(fn, v.tag == V_F64, 2, iv, fv, nul, 0.0, &ao);
            s->mm.tag = ao.tag == EK_TAG_F64 ? V_F64 : V_I64;
            s->mm.i = ao.i; s->mm.f = ao.f;
        }
        break;
    }
    s->has = 1;
}

static val_t inc_value(int fn, const incstate* s) {
    val_t r; r.tag = V_NULL; r.i = 0; r.f = 0;
    if (s->lastnil || !s->has) return r;
    switch (fn) {
    case EK_AGG_COUNT_STAR: case EK_AGG_COUNT: r.tag = V_I64; r.i = s->cnt; break;
    case EK_AGG_SUM: r.tag = V_F64; r.f = s->fsum; break;
    case EK_AGG_AVG: r.tag = V_F64; r.f = s->fsum / (double)s->cnt; break;
    default: r = s->mm; break;
    }
    return r;
}

static int inc_supported_fn(int fn) {
    return fn == EK_AGG_COUNT_STAR || fn == EK_AGG_COUNT || fn == EK_AGG_SUM || fn == EK_AGG_AVG || fn == EK_AGG_MIN ||
           fn == EK_AGG_MAX;
}

/* One incremental window: content = the rows incAggCal added, in processing order. A window none of whose
 * rows was added (created by a row outside its own range) is not reported. */
static void emit_inc_window_ex(const dataset* d, outbuf* ob, int64_t wstart, int64_t wend, const int64_t* content, int64_t nc,
                               int report_empty) {
    const ek_plan* p = d->p;
    if (nc == 0 && !report_empty) return;
    int64_t w = ob->ws.n;
    v_push(&ob->ws, wstart);
    v_push(&ob->we, wend);
    v_push(&ob->roff, ob->key.n);
    v_push(&ob->moff, ob->mem.n);
    uint64_t h = 0;
    for (int64_t k = 0; k < nc; ++k) {
        const int64_t a = row_arrival(d, content[k]);
        v_push(&ob->mem, a);
        h += ek_mix64((uint64_t)a);
    }
    v_push(&ob->mcnt, nc);
    v_push(&ob->mhash, (int64_t)h);
    if (ob->werr_cap <= w) { ob->werr_cap = (w + 1) * 2; ob->werr = (char*)realloc(ob->werr, (size_t)ob->werr_cap * 128); }
    ob->werr[w * 128] = 0;
    int status = EK_WIN_OK;
    int64_t rows_before = ob->key.n;
    /* dimensions in first-appearance order (the reference iterates a Go map: unspecified order) */
    int64_t cap = 16; while (cap < nc * 2) cap <<= 1;
    int64_t* slot = (int64_t*)malloc((size_t)cap * 8);
    int64_t* gkey = (int64_t*)malloc((size_t)nc * 8);
    int64_t* glast = (int64_t*)malloc((size_t)nc * 8);
    incstate* st = (incstate*)calloc((size_t)nc * (p->n_aggs ? p->n_aggs : 1), sizeof(incstate));
    for (int64_t k = 0; k < cap; ++k) slot[k] = -1;
    int64_t ng = 0;
    for (int64_t k = 0; k < nc; ++k) {
        int64_t g = 0;
        if (p->key_column >= 0) {
            val_t kv = col_val(d, p->key_column, content[k]);
            int64_t key = kv.tag == V_NULL ? -1 : kv.i;
            uint64_t hh = ek_mix64((uint64_t)key) & (uint64_t)(cap - 1);
            while (slot[hh] >= 0 && gkey[slot[hh]] != key) hh = (hh + 1) & (uint64_t)(cap - 1);
            if (slot[hh] < 0) { slot[hh] = ng; gkey[ng] = key; ng++; }
            g = slot[hh];
        } else {
            if (ng == 0) { gkey[0] = 0; ng = 1; }
        }
        glast[g] = content[k];
        for (int a = 0; a < p->n_aggs; ++a) inc_step(d, p->aggs[a].fn, p->aggs[a].column, content[k], &st[g * p->n_aggs + a]);
    }
    val_t aggv[EK_MAX_AGGS];
    /* WHERE above the incremental window (FilterPlan over IncWindowPlan, planner.go:702-708; incAggPlan.go:76-78):
     * FilterOp.Apply over the emitted collection (filter_operator.go:59-90), each row a group's LAST row: nil / false
     * drops the row, an error or a non-bool replaces the window ("run Where error: ..."). The collection comes out of
     * a Go map (window_inc_agg_op.go:443-457): of several failing rows, the one with the smallest key is reported. */
    uint8_t* gkeep = (uint8_t*)malloc((size_t)(ng ? ng : 1));
    for (int64_t g = 0; g < ng; ++g) gkeep[g] = 1;
    if (p->n_where > 0) {
        int64_t bad = -1;
        val_t badv = mk_null();
        for (int64_t g = 0; g < ng; ++g) {
            const val_t r = eval_prog(p->where_prog, p->n_where, d, glast[g], NULL);
            gkeep[g] = r.tag == V_BOOL && r.i;
            if (r.tag != V_BOOL && r.tag != V_NULL && (bad < 0 || gkey[g] < gkey[bad])) { bad = g; badv = r; }
        }
        if (bad >= 0) {
            status = EK_WIN_WHERE_ERROR;
            if (badv.tag == V_ERR) snprintf(ob->werr + w * 128, 128, "run Where error: %s", err_text(badv));
            else {
                char tv[80];
                go_typed(tv, sizeof tv, badv);
                snprintf(ob->werr + w * 128, 128, "run Where error: invalid condition that returns non-bool value %s", tv);
            }
            ng = 0;
        }
    }
    int64_t hkey = INT64_MAX;   /* HAVING: of several failing groups, the one with the smallest key is reported */
    for (int64_t g = 0; g < ng; ++g) {
        if (!gkeep[g]) continue;
        for (int a = 0; a < p->n_aggs; ++a) aggv[a] = inc_value(p->aggs[a].fn, &st[g * p->n_aggs + a]);
        if (p->n_having > 0) {
            /* HavingOp IsIncAgg branch (having_operator.go:73-98): evaluated on each emitted row */
            val_t r = eval_prog(p->having_prog, p->n_having, d, glast[g], aggv);
            if (r.tag != V_BOOL) {
                status = EK_WIN_HAVING_ERROR;
                if (gkey[g] < hkey) {
                    hkey = gkey[g];
                    if (r.tag == V_ERR) snprintf(ob->werr + w * 128, 128, "run Having error: %s", err_text(r));
                    else {
                        char tv[80];
                        go_typed(tv, sizeof tv, r);
                        snprintf(ob->werr + w * 128, 128, "run Having error: invalid condition that returns non-bool value %s", tv);
                    }
                }
                continue;
            }
            if (!r.i) continue;
        }
        v_push(&ob->key, gkey[g]);
        for (int a = 0; a < p->n_aggs; ++a) {
            int64_t bits = aggv[a].i;
            if (aggv[a].tag == V_F64) memcpy(&bits, &aggv[a].f, 8);
            v_push(&ob->aval[a], aggv[a].tag == V_NULL ? 0 : bits);
            v_push(&ob->atag[a], aggv[a].tag == V_NULL ? EK_TAG_NULL : (aggv[a].tag == V_F64 ? EK_TAG_F64 : EK_TAG_I64));
        }
    }
    if (status != EK_WIN_OK) {
        ob->key.n = rows_before;
        for (int a = 0; a < p->n_aggs; ++a) { ob->aval[a].n = rows_before; ob->atag[a].n = rows_before; }
    }
    free(slot); free(gkey); free(glast); free(st); free(gkeep);
    v_push(&ob->rcnt, ob->key.n - rows_before);
    v_push(&ob->st, status);
}
static void emit_inc_window(const dataset* d, outbuf* ob, int64_t wstart, int64_t wend, const int64_t* content, int64_t nc) {
    emit_inc_window_ex(d, ob, wstart, wend, content, nc, 0);
}

/* HoppingWindowIncAggEventOp (window_inc_agg_event_op.go:26-146), also TUMBLING (:298-307, Length = Interval) */
typedef struct { int64_t start; vec64 mem; } incwin;
typedef struct {
    const dataset* d;
    outbuf* ob;
    int64_t L, I;
    int32_t raw_interval, unit, tz;
    int has_T; int64_t T;      /* NextTriggerWindowTime (zero time before the first row) */
    incwin* w; int64_t nw, cap;
    int64_t* ts;
} incop;

static void inc_on_event(incop* o, int64_t e) {
    const int64_t t = o->ts[e];
    /* triggerWindow (:130-137): a row later than NextTriggerWindowTime opens [next - Interval, +Length) */
    if (!o->has_T || o->T < t) {
        o->T = eko_aligned_window_end(t, o->raw_interval, o->unit, o->tz);
        o->has_T = 1;
        if (o->nw == o->cap) { o->cap = o->cap ? 2 * o->cap : 16; o->w = (incwin*)realloc(o->w, (size_t)o->cap * sizeof(incwin)); }
        memset(&o->w[o->nw], 0, sizeof(incwin));
        o->w[o->nw++].start = o->T - o->I;
    }
    /* calIncAggWindow (:104-111): every open window whose [start, start + Length) holds t */
    for (int64_t k = 0; k < o->nw; ++k)
        if (o->w[k].start <= t && t < o->w[k].start + o->L) v_push(&o->w[k].mem, e);
}

static void inc_on_watermark(incop* o, int64_t wm) {
    /* emitWindow (:113-119) then gcIncAggWindow (window_inc_agg_op.go:843-857) */
    for (int64_t k = 0; k < o->nw; ++k)
        if (o->w[k].start + o->L <= wm) emit_inc_window(o->d, o->ob, o->w[k].start, o->w[k].start + o->L, o->w[k].mem.a, o->w[k].mem.n);
    int64_t g = 0;
    while (g < o->nw && wm - o->w[g].start >= o->L) { free(o->w[g].mem.a); g++; }
    if (g > 0) { memmove(o->w, o->w + g, (size_t)(o->nw - g) * sizeof(incwin)); o->nw -= g; }
}

/* SlidingWindowIncAggEventOp without delay (window_inc_agg_event_op.go:193-273): a trigger row opens a window at its
 * ts (newIncAggWindow); every row joins the open windows with start <= ts < start + Length (incAggCal); a trigger row
 * then queues a clone of the OLDEST open window (CurrWindowList[0].Clone) whose StartTime becomes the row's ts; the
 * next WatermarkTuple emits every queued clone (zero EventTime + 0 <= watermark) with WindowRange (StartTime,
 * watermark) and drops the open windows with watermark - start >= Length (gcIncAggWindow, window_inc_agg_op.go:843-857). */
typedef struct {
    const dataset* d;
    outbuf* ob;
    int64_t L;
    incwin* w; int64_t nw, cap;    /* CurrWindowList */
    incwin* e; int64_t ne, ecap;   /* EmitList (start = the trigger row's ts) */
    const int64_t* ts;
} incslide;

static void incslide_on_event(incslide* o, int64_t e) {
    const ek_plan* p = o->d->p;
    const int64_t t = o->ts[e];
    int trig = 1;
    if (p->n_trigger > 0) { val_t r = eval_prog(p->trigger_prog, p->n_trigger, o->d, e, NULL); trig = r.tag == V_BOOL && r.i; }
    if (trig) {
        if (o->nw == o->cap) { o->cap = o->cap ? 2 * o->cap : 16; o->w = (incwin*)realloc(o->w, (size_t)o->cap * sizeof(incwin)); }
        memset(&o->w[o->nw], 0, sizeof(incwin));
        o->w[o->nw++].start = t;
    }
    for (int64_t k = 0; k < o->nw; ++k)
        if (o->w[k].start <= t && t < o->w[k].start + o->L) v_push(&o->w[k].mem, e);
    if (trig) {
        if (o->ne == o->ecap) { o->ecap = o->ecap ? 2 * o->ecap : 16; o->e = (incwin*)realloc(o->e, (size_t)o->ecap * sizeof(incwin)); }
        incwin* c = &o->e[o->ne++];
        memset(c, 0, sizeof *c);
        c->start = t;
        for (int64_t k = 0; k < o->w[0].mem.n; ++k) v_push(&c->mem, o->w[0].mem.a[k]);
    }
}

static void incslide_on_watermark(incslide* o, int64_t wm) {
    for (int64_t k = 0; k < o->ne; ++k) {
        emit_inc_window(o->d, o->ob, o->e[k].start, wm, o->e[k].mem.a, o->e[k].mem.n);
        free(o->e[k].mem.a);
    }
    o->ne = 0;
    int64_t g = 0;
    while (g < o->nw && wm - o->w[g].start >= o->L) { free(o->w[g].mem.a); g++; }
    if (g > 0) { memmove(o->w, o->w + g, (size_t)(o->nw - g) * sizeof(incwin)); o->nw -= g; }
}

/* CountWindowIncAggEventOp (window_inc_agg_event_op.go:351-408): consecutive blocks of CountLength released rows
 * (StartTime = the first row's ts); the next WatermarkTuple emits the completed blocks, WindowRange (StartTime, wm). */
typedef struct {
    const dataset* d;
    outbuf* ob;
    int64_t n;
    vec64 cur; int64_t cur_start;
    incwin* e; int64_t ne, ecap;
    const int64_t* ts;
} inccount;

static void inccount_on_event(inccount* o, int64_t e) {
    if (o->cur.n == 0) o->cur_start = o->ts[e];
    v_push(&o->cur, e);
    if (o->cur.n >= o->n) {
        if (o->ne == o->ecap) { o->ecap = o->ecap ? 2 * o->ecap : 16; o->e = (incwin*)realloc(o->e, (size_t)o->ecap * sizeof(incwin)); }
        o->e[o->ne].start = o->cur_start;
        o->e[o->ne].mem = o->cur;
        o->ne++;
        memset(&o->cur, 0, sizeof o->cur);
    }
}

static void inccount_on_watermark(inccount* o, int64_t wm) {
    /* every queued block started at or before the watermark (its rows were released by it) */
    for (int64_t k = 0; k < o->ne; ++k) {
        emit_inc_window(o->d, o->ob, o->e[k].start, wm, o->e[k].mem.a, o->e[k].mem.n);
        free(o->e[k].mem.a);
    }
    o->ne = 0;
}

/* ------------------------------------------------------------------ window operator (event time) */
typedef struct {
    const dataset* d;
    outbuf* ob;
    int wtype;
    int64_t L, I, D;           /* ms */
    int32_t raw_interval, unit, tz;
    vec64 inputs;              /* event indices, release order */
    int unsorted;              /* an input was released out of ts order (never in event time; kept as a guard) */
    int has_trigger; int64_t trigger_time;
    int64_t next_end, prev_end; /* prev_end ZERO_MS = IsZero */
    vec64 trigger_ts, delay_ts;
    int last_ticked;
    int send_twice;            /* enableSlidingWindowSendTwice (window_op.go:98): delayed sliding windows only */
    int64_t* ts;
    vec64 content;
    /* shard model (eko_run_shard): the window op of one key-hash shard fed the global WatermarkTuples */
    int shard;
    int origin_known;
    int64_t origin_ts, origin_arrival, cur_wm_arrival;
    /* shard model, SESSIONWINDOW: the router's global session list (ek_global_ctx sess_*) and the next one */
    const int64_t *sess_start, *sess_end, *sess_wm;
    int64_t n_sess, i_sess;
} winop;

static int64_t ev_ts(const winop* o, int64_t e) { return o->ts[e]; }

/* window_op.go:553-574 */
static int is_time_related(const winop* o) {
    switch (o->wtype) {
    case EK_WINDOW_SLIDING: return o->D > 0;
    case EK_WINDOW_TUMBLING: case EK_WINDOW_HOPPING: case EK_WINDOW_SESSION: return 1;
    }
    return 0;
}
static int is_overlap(const winop* o) { return o->wtype == EK_WINDOW_HOPPING || o->wtype == EK_WINDOW_SLIDING; }

/* window_op.go:605-655 handleInputs; event time => calDelta == 0 once triggerTime is set (it is set by the
 * first event, event_window_trigger.go:187-189), else MaxInt16 ns which is invisible at ms resolution. */
static void handle_inputs(winop* o, int64_t right, int64_t* keep_from) {
    int64_t length = o->L + o->D;
    int64_t left = right - length;
    int64_t nextleft = -1;
    int all_discarded = 0;
    int ov = is_overlap(o), tr = is_time_related(o);
    o->content.n = 0;
    for (int64_t i = 0; i < o->inputs.n; ++i) {
        int64_t t = ev_ts(o, o->inputs.a[i]);
        if (ov && !all_discarded) {
            if (t < left) continue;
        }
        all_discarded = 1;
        int meet = tr ? (t < right) : (t <= right);
        if (meet) {
            v_push(&o->content, o->inputs.a[i]);
            if (nextleft < 0 && ov) nextleft = i;
        } else {
            if (nextleft < 0 && !ov) nextleft = i;
        }
    }
    if (nextleft < 0 && ov && o->shard) {
        /* shard model: an empty LOCAL window is not an empty global one (the global discard quirk is decided per
         * event at acceptance, hop_discard below); only the expired rows go */
        nextleft = 0;
        while (nextleft < o->inputs.n && ev_ts(o, o->inputs.a[nextleft]) < left) nextleft++;
    }
    *keep_from = nextleft < 0 ? o->inputs.n : nextleft;
}

/* window_op.go:576-603 handleInputsForSlidingWindow (enableSlidingWindowSendTwice): content = the inputs with
 * windowStart < ts <= windowEnd; an input with ts < discardedLeft = windowEnd - (length + delay) (- calDelta: 0 once
 * triggerTime is set, MaxInt16 ns before, invisible at ms resolution) is expired and nextleft = the LAST expired index;
 * the inputs kept are inputs[:nextleft+1] — the expired prefix: the reference keeps those and drops the rest —
 * unless no input expired (unchanged) or every one did (none). */
static void handle_inputs_sliding(winop* o, int64_t ws, int64_t we) {
    const int64_t dl = we - (o->L + o->D);
    int64_t nextleft = -1;
    o->content.n = 0;
    for (int64_t i = 0; i < o->inputs.n; ++i) {
        const int64_t t = ev_ts(o, o->inputs.a[i]);
        if (t < dl) { nextleft = i; continue; }
        if (t > ws && t <= we) v_push(&o->content, o->inputs.a[i]);
    }
    if (nextleft < 0) return;
    o->inputs.n = nextleft == o->inputs.n - 1 ? 0 : nextleft + 1;
}

/* window_op.go:675-721 scan */
static void scan(winop* o, int64_t t, int64_t length, int is_first_part) {
    if (o->send_twice && o->wtype == EK_WINDOW_SLIDING) {
        handle_inputs_sliding(o, t - length, t);
        /* WindowRange: [t - length, t] for both parts (the second part's third field is its trigger, t - delay) */
        emit_window(o->d, o->ob, t - length, t, o->content.a, o->content.n);
        o->trigger_time = t; o->has_trigger = 1;
        return;
    }
    int64_t keep_from;
    handle_inputs(o, t, &keep_from);
    int64_t tt = o->has_trigger ? o->trigger_time : ZERO_MS;
    int64_t ws = 0;
    switch (o->wtype) {
    case EK_WINDOW_TUMBLING: case EK_WINDOW_SESSION: ws = tt; break;
    case EK_WINDOW_HOPPING: ws = tt - o->I; break;
    case EK_WINDOW_SLIDING: ws = t - length; break;
    }
    if (ws <= 0) ws = t - length;
    int64_t we = t;
    if (!is_first_part) { ws = 0; we = 0; } /* WindowRange left unset (delayed sliding, no send-twice) */
    emit_window(o->d, o->ob, ws, we, o->content.a, o->content.n);
    v_erase_front(&o->inputs, keep_from);
    o->trigger_time = t; o->has_trigger = 1;
}

/* event_window_trigger.go:211-219 */
static int64_t earliest(const winop* o, int64_t start, int64_t end) {
    int64_t m = MAXT_MS;
    if (!o->unsorted) {
        /* inputs hold released events in release order, i.e. non-decreasing ts: the minimum of the ts in
         * (start, end] is the first ts > start (same result as the scan below, without its O(n) per watermark) */
        int64_t lo = 0, hi = o->inputs.n;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (ev_ts(o, o->inputs.a[mid]) > start) hi = mid; else lo = mid + 1;
        }
        if (lo < o->inputs.n && ev_ts(o, o->inputs.a[lo]) <= end) m = ev_ts(o, o->inputs.a[lo]);
        return m;
    }
    for (int64_t i = 0; i < o->inputs.n; ++i) {
        int64_t t = ev_ts(o, o->inputs.a[i]);
        if (t > start && t <= end && t < m) m = t;
    }
    return m;
}

/* event_window_trigger.go:57-75 */
static int64_t next_window(const winop* o, int64_t current, int64_t wm) {
    switch (o->wtype) {
    case EK_WINDOW_TUMBLING: case EK_WINDOW_HOPPING: {
        int64_t interval = o->wtype == EK_WINDOW_TUMBLING ? o->L : o->I;
        if (current != ZERO_MS) return current + interval;
        if (o->shard) {
            /* the first end is anchored on the GLOBAL earliest released event, known from the tuple that released it */
            if (!o->origin_known || o->cur_wm_arrival < o->origin_arrival) return MAXT_MS;
            return eko_aligned_window_end(o->origin_ts, o->raw_interval, o->unit, o->tz);
        }
        int64_t nt = earliest(o, ZERO_MS, wm);
        if (nt == MAXT_MS) return nt;
        return eko_aligned_window_end(nt, o->raw_interval, o->unit, o->tz);
    }
    case EK_WINDOW_SLIDING:
        return earliest(o, current, wm);
    }
    return MAXT_MS;
}

/* event_window_trigger.go:77-110 */
static int64_t next_session(const winop* o, int64_t now, int* ticked) {
    *ticked = 0;
    if (o->inputs.n > 0) {
        int64_t timeout = o->I, duration = o->L;
        int64_t et = ev_ts(o, o->inputs.a[0]);
        int64_t tick = eko_aligned_window_end(et, o->raw_interval, o->unit, o->tz);
        int64_t p = ZERO_MS;
        for (int64_t i = 0; i < o->inputs.n; ++i) {
            int64_t t = ev_ts(o, o->inputs.a[i]);
            int64_t r = MAXT_MS;
            if (p != ZERO_MS && t - p > timeout) r = p + timeout;
            if (t > tick) {
                if (tick - duration > et && tick < r) { r = tick; *ticked = 1; }
                tick = tick + duration;
            }
            if (r < MAXT_MS) return r;
            p = t;
        }
        if (p != ZERO_MS && now - p > timeout) return p + timeout;
    }
    *ticked = 0;
    return MAXT_MS;
}

static int match_trigger(const winop* o, int64_t e) {
    const ek_plan* p = o->d->p;
    if (p->n_trigger <= 0 || o->wtype != EK_WINDOW_SLIDING) return 1;
    val_t r = eval_prog(p->trigger_prog, p->n_trigger, o->d, e, NULL);
    return r.tag == V_BOOL && r.i; /* window_op.go:741-768: nil/error/non-bool -> false */
}

/* event_window_trigger.go:182-196 (EventRow branch) */
static void win_on_event(winop* o, int64_t e) {
    if (!o->has_trigger) { o->has_trigger = 1; o->trigger_time = o->shard ? o->origin_ts : ev_ts(o, e); }
    if (o->wtype == EK_WINDOW_SLIDING && !o->shard && match_trigger(o, e)) v_push(&o->trigger_ts, ev_ts(o, e));
    if (o->inputs.n > 0 && ev_ts(o, e) < ev_ts(o, o->inputs.a[o->inputs.n - 1])) o->unsorted = 1;
    v_push(&o->inputs, e);
}

/* event_window_trigger.go:124-180 (WatermarkTuple branch) */
static void win_on_watermark(winop* o, int64_t wm) {
    if (o->wtype == EK_WINDOW_SLIDING) {
        while (o->delay_ts.n > 0 && wm >= o->delay_ts.a[0]) {
            scan(o, o->delay_ts.a[0], o->D, 0);
            v_erase_front(&o->delay_ts, 1);
        }
    }
    if (o->shard && o->wtype == EK_WINDOW_SESSION) {
        /* shard model: the sessions the WHOLE stream's tuple closed (ekgpu/shard.py GlobalSession), each over
         * this shard's inputs with ts < end (handleInputs of a non-overlapping window, window_op.go:605-655) */
        while (o->i_sess < o->n_sess && o->sess_wm[o->i_sess] <= wm) {
            o->trigger_time = o->sess_start[o->i_sess]; o->has_trigger = 1;
            scan(o, o->sess_end[o->i_sess], o->L, 1);
            o->i_sess++;
        }
        return;
    }
    int64_t we = o->next_end;
    int ticked = 0;
    if (we == MAXT_MS || o->wtype == EK_WINDOW_SESSION || o->wtype == EK_WINDOW_SLIDING) {
        if (o->wtype == EK_WINDOW_SESSION) we = next_session(o, wm, &ticked);
        else we = next_window(o, o->prev_end, wm);
    }
    if (o->shard && o->wtype == EK_WINDOW_SLIDING) {
        /* shard model: every trigger fires at the tuple that released it (its window = the rows released so far);
         * with a delay it queues t + D and the window (t - L, t + D] fires at a later tuple reaching it (the delay
         * loop above), as in the trigger loop below (event_window_trigger.go:154-166) */
        while (o->trigger_ts.n > 0 && o->trigger_ts.a[0] <= wm) {
            if (o->D > 0) v_push(&o->delay_ts, o->trigger_ts.a[0] + o->D);
            else scan(o, o->trigger_ts.a[0], o->L, 1);
            v_erase_front(&o->trigger_ts, 1);
        }
        return;
    }
    while (we != ZERO_MS && we <= wm) {
        if (o->wtype == EK_WINDOW_SESSION && !o->last_ticked && o->inputs.n > 0) {
            o->trigger_time = ev_ts(o, o->inputs.a[0]); o->has_trigger = 1;
        }
        if (o->wtype == EK_WINDOW_SLIDING) {
            while (o->trigger_ts.n > 0 && o->trigger_ts.a[0] <= wm) {
                if (o->D > 0) {
                    v_push(&o->delay_ts, o->trigger_ts.a[0] + o->D);
                    if (o->send_twice) scan(o, o->trigger_ts.a[0], o->L, 1);   /* the first part, at the trigger */
                } else {
                    scan(o, o->trigger_ts.a[0], o->L + o->D, 1);
                }
                v_erase_front(&o->trigger_ts, 1);
            }
        } else {
            scan(o, we, o->L + o->D, 1);
        }
        o->prev_end = we;
        o->last_ticked = ticked;
        if (o->wtype == EK_WINDOW_SESSION) we = next_session(o, wm, &ticked);
        else we = next_window(o, o->prev_end, wm);
    }
    o->next_end = we;
}

/* ------------------------------------------------------------------ state window (WindowV2Operator) */
/* StateWindowOp.exec (window_v2_op.go:111-148); rows arrive in arrival order (processing time) or in
 * WatermarkOp release order (event time; watermark tuples are ignored by this op). */
typedef struct {
    const dataset* d;
    outbuf* ob;
    int on;                    /* onBegin */
    vec64 rows;                /* WindowScanner.tuples */
    const int64_t* ts;         /* event time: row timestamps; NULL in processing time */
} stateop;

/* isMatchCondition (window_v2_op.go:212-238): nil condition -> true; nil / error / non-bool result -> false */
static int cond_true(const dataset* d, const ek_instr* prog, int n, int64_t e) {
    if (n <= 0) return 1;
    val_t r = eval_prog(prog, n, d, e, NULL);
    return r.tag == V_BOOL && r.i;
}

static void state_on_row(stateop* o, int64_t e) {
    const ek_plan* p = o->d->p;
    int can_begin = 0, can_emit = 0;
    if (!o->on) {
        can_begin = cond_true(o->d, p->begin_prog, p->n_begin, e);
        if (can_begin) o->on = 1;
    }
    if (o->on) {
        v_push(&o->rows, e);
        can_emit = cond_true(o->d, p->emit_prog, p->n_emit, e);
    }
    if (o->on && can_emit) {
        /* emitWindow(time.Time{}, InfTime) -> scanWindow (window_v2_op.go:75-87,252-263): rows with a timestamp
         * after time.Time{} (processing-time rows carry the ingest wall clock) */
        int64_t nc = 0;
        for (int64_t k = 0; k < o->rows.n; ++k)
            if (!o->ts || o->ts[o->rows.a[k]] > ZERO_MS) o->rows.a[nc++] = o->rows.a[k];
        emit_window(o->d, o->ob, EK_STATE_WINDOW_START_MS, EK_STATE_WINDOW_END_MS, o->rows.a, nc);
        o->rows.n = 0;          /* scanner.gc(InfTime) */
        o->on = 0;
    }
    if (can_begin && !o->on) o->on = 1;
}

/* EventSlidingWindowOp without delay (window_v2_event_op.go:78-96): each released row joins the scanner; a row
 * matching the trigger condition emits scanWindow(ts - L, ts): the rows added so far with ts in (ts - L, ts]
 * (window_v2_op.go:252-263). The scanner is in release order, so the scan stops at the first later row. */
static void v2slide_on_row(winop* o, int64_t e) {
    v_push(&o->inputs, e);
    const ek_plan* p = o->d->p;
    if (p->n_trigger > 0) {
        val_t r = eval_prog(p->trigger_prog, p->n_trigger, o->d, e, NULL);
        if (!(r.tag == V_BOOL && r.i)) return;
    }
    const int64_t t = ev_ts(o, e), ws = t - o->L;
    if (o->D > 0) { v_push(&o->delay_ts, t + o->D); return; }   /* delayTS (window_v2_event_op.go:90-93) */
    o->content.n = 0;
    for (int64_t i = 0; i < o->inputs.n; ++i) {
        const int64_t x = ev_ts(o, o->inputs.a[i]);
        if (x > ws && x <= t) v_push(&o->content, o->inputs.a[i]);
        else if (x > t) break;
    }
    emit_window(o->d, o->ob, ws, t, o->content.a, o->content.n);
}

/* EventSlidingWindowOp's WatermarkTuple branch (window_v2_event_op.go:56-76): every queued delay time at or before the
 * watermark emits scanWindow(delay - length - D, watermark) — WindowRange ends at the WATERMARK — and the queue drops
 * the emitted prefix only when a later entry is still pending (newIndex != -1): while every entry is due, all of them
 * are emitted again at each later watermark. Then scanner.gc(watermark - length - D). */
static void v2slide_on_watermark(winop* o, int64_t wm) {
    int64_t keep_from = -1;
    for (int64_t k = 0; k < o->delay_ts.n; ++k) {
        const int64_t dts = o->delay_ts.a[k];
        if (dts <= wm) {
            const int64_t ws = dts - o->L - o->D;
            o->content.n = 0;
            for (int64_t i = 0; i < o->inputs.n; ++i) {
                const int64_t x = ev_ts(o, o->inputs.a[i]);
                if (x > ws && x <= wm) v_push(&o->content, o->inputs.a[i]);
                else if (x > wm) break;
            }
            emit_window(o->d, o->ob, ws, wm, o->content.a, o->content.n);
        } else {
            keep_from = k;
            break;
        }
    }
    if (keep_from >= 0) v_erase_front(&o->delay_ts, keep_from);
    int64_t g = 0;
    while (g < o->inputs.n && ev_ts(o, o->inputs.a[g]) <= wm - o->L - o->D) g++;
    v_erase_front(&o->inputs, g);
}

/* ------------------------------------------------------------------ driver */
static void set_status(eko_output* out, int st, const char* msg) {
    out->status = st;
    snprintf(out->error, sizeof out->error, "%s", msg);
}

static int64_t* take(vec64* v) { int64_t* a = v->a; v->a = NULL; v->n = v->cap = 0; return a ? a : (int64_t*)calloc(1, 8); }

/* the outbuf of a run -> the eko_output arrays */
static void finish_output(const ek_plan* p, outbuf* ob, eko_output* out) {
    out->r.n_windows = ob->ws.n;
    out->r.n_rows = ob->key.n;
    out->r.n_aggs = p->window_type == EK_WINDOW_NONE ? p->n_columns : p->n_aggs;
    out->r.memory = EK_MEM_HOST;
    v_push(&ob->moff, ob->mem.n);
    out->r.win_start = take(&ob->ws);
    out->r.win_end = take(&ob->we);
    out->r.win_row_offset = take(&ob->roff);
    out->r.win_row_count = take(&ob->rcnt);
    out->r.win_member_count = take(&ob->mcnt);
    out->r.win_member_hash = (uint64_t*)take(&ob->mhash);
    {
        int64_t* st = take(&ob->st);
        out->r.win_status = (int32_t*)calloc((size_t)(out->r.n_windows ? out->r.n_windows : 1), 4);
        for (int64_t w = 0; w < out->r.n_windows; ++w) out->r.win_status[w] = (int32_t)st[w];
        free(st);
    }
    {
        int64_t* k = take(&ob->key);
        out->r.key = (uint32_t*)calloc((size_t)(out->r.n_rows ? out->r.n_rows : 1), 4);
        for (int64_t r = 0; r < out->r.n_rows; ++r) out->r.key[r] = (uint32_t)k[r];
        free(k);
    }
    for (int a = 0; a < out->r.n_aggs; ++a) {
        out->r.agg_value[a] = take(&ob->aval[a]);
        int64_t* t = take(&ob->atag[a]);
        out->r.agg_tag[a] = (uint8_t*)calloc((size_t)(out->r.n_rows ? out->r.n_rows : 1), 1);
        for (int64_t r = 0; r < out->r.n_rows; ++r) out->r.agg_tag[a][r] = (uint8_t)t[r];
        free(t);
    }
    out->member_offset = take(&ob->moff);
    out->members = take(&ob->mem);
    out->win_error = ob->werr ? ob->werr : (char*)calloc(1, 128);
}

/* FilterOp.Apply of the window's FILTER (WHERE ...) clause on one row (filter_operator.go:41-57): true keeps it;
 * nil / false drop it; an evaluation error or a non-bool drops it and is counted (the reference forwards that error) */
static int filter_pass(const dataset* d, int64_t row, int64_t* n_err) {
    const ek_plan* p = d->p;
    if (p->n_filter <= 0) return 1;
    val_t r = eval_prog(p->filter_prog, p->n_filter, d, row, NULL);
    if (r.tag == V_BOOL) return r.i != 0;
    if (r.tag != V_NULL && n_err) (*n_err)++;
    return 0;
}

/* The FilterOp in front of a processing-time window (windowPlan.PushDownPredicate, windowPlan.go:82-99, planner.go:
 * 388-392): combine(WHERE, FILTER) evaluated as the binary AND of valuer.go:574-660 (a false / error lhs decides;
 * nil AND x -> false unless x errors); an error or a non-bool drops the row and is counted */
static int pushdown_pass(const dataset* d, int64_t i, int64_t* n_err) {
    const ek_plan* p = d->p;
    if (p->n_where <= 0 && p->n_filter <= 0) return 1;
    val_t r = mk_bool(1);
    if (p->n_where > 0) r = eval_prog(p->where_prog, p->n_where, d, i, NULL);
    if (p->n_filter > 0 && r.tag != V_ERR && !(r.tag == V_BOOL && !r.i)) {
        const val_t rf = eval_prog(p->filter_prog, p->n_filter, d, i, NULL);
        r = p->n_where > 0 ? (rf.tag == V_ERR ? rf : simple_eval(r, rf, EK_OP_AND)) : rf;
    }
    if (r.tag == V_BOOL && r.i) return 1;
    if (r.tag != V_BOOL && r.tag != V_NULL && n_err) (*n_err)++;
    return 0;
}

int eko_run(const ek_plan* p, int64_t n, const void* const* columns, const uint8_t* const* validity, eko_output* out) {
    memset(out, 0, sizeof *out);
    if (!p || p->abi_version != EKGPU_ABI_VERSION) { set_status(out, EK_ERR_INVALID, "abi version mismatch"); return out->status; }
    if (p->n_aggs < 0 || p->n_aggs > EK_MAX_AGGS) { set_status(out, EK_ERR_INVALID, "bad n_aggs"); return out->status; }
    dataset d = { p, n, columns, validity, NULL };
    outbuf ob; memset(&ob, 0, sizeof ob);

    /* rewriteIfIncAggStmt (planner.go:910-997): every aggregate must be incremental, and the window type one of
     * COUNT (without interval) / SLIDING / HOPPING / TUMBLING; otherwise the regular operator chain is planned */
    int inc_ok = p->incremental != 0 && p->n_aggs > 0;
    for (int a = 0; a < p->n_aggs; ++a) inc_ok &= inc_supported_fn(p->aggs[a].fn);
    if (p->window_type == EK_WINDOW_COUNT && p->interval > 0) inc_ok = 0;
    if (p->window_type == EK_WINDOW_SESSION || p->window_type == EK_WINDOW_NONE || p->window_type == EK_WINDOW_STATE) inc_ok = 0;
    if (inc_ok && p->window_type == EK_WINDOW_SLIDING && (!p->is_event_time || p->delay != 0)) {
        set_status(out, EK_ERR_UNSUPPORTED, "incremental sliding windows are restated in event time without delay only"); return out->status;
    }
    const int v2slide = p->window_version == 2 && p->window_type == EK_WINDOW_SLIDING;
    if (v2slide && !p->is_event_time) {
        set_status(out, EK_ERR_UNSUPPORTED, "processing-time v2 sliding windows run under the clock (eko_run_proc)"); return out->status;
    }
    stateop so; memset(&so, 0, sizeof so);
    so.d = &d; so.ob = &ob;
    if (p->is_event_time) {
        /* NewEventTimeTrigger (event_window_trigger.go:35-53); STATEWINDOW runs in WindowV2Operator (window_v2_op.go:39-58) */
        if ((p->window_type == EK_WINDOW_COUNT || p->window_type > EK_WINDOW_COUNT || p->window_type < 0) &&
            p->window_type != EK_WINDOW_STATE && !(inc_ok && p->window_type == EK_WINDOW_COUNT)) {
            set_status(out, EK_ERR_UNSUPPORTED, "unsupported window type"); return out->status;
        }
        if (p->ts_column < 0) { set_status(out, EK_ERR_INVALID, "event time requires a timestamp column"); return out->status; }
        int64_t* ts = (int64_t*)malloc((size_t)(n ? n : 1) * 8);
        for (int64_t i = 0; i < n; ++i) { val_t v = col_val(&d, p->ts_column, i); ts[i] = v.tag == V_F64 ? (int64_t)v.f : v.i; }
        const int inc = p->incremental && (p->window_type == EK_WINDOW_TUMBLING || p->window_type == EK_WINDOW_HOPPING) && inc_ok;
        const int inc_slide = inc_ok && p->window_type == EK_WINDOW_SLIDING;
        const int inc_count = inc_ok && p->window_type == EK_WINDOW_COUNT;
        incslide isl; memset(&isl, 0, sizeof isl);
        isl.d = &d; isl.ob = &ob; isl.ts = ts; isl.L = (int64_t)p->length * unit_ms(p->time_unit);
        inccount icn; memset(&icn, 0, sizeof icn);
        icn.d = &d; icn.ob = &ob; icn.ts = ts; icn.n = p->length;
        incop io; memset(&io, 0, sizeof io);
        io.d = &d; io.ob = &ob; io.ts = ts;
        {
            int64_t uu = unit_ms(p->time_unit);
            io.L = (int64_t)p->length * uu;
            io.I = (int64_t)(p->window_type == EK_WINDOW_HOPPING ? p->interval : p->length) * uu;
            io.raw_interval = p->window_type == EK_WINDOW_HOPPING ? p->interval : p->length;
            io.unit = p->time_unit; io.tz = p->tz_offset_s;
        }
        winop o; memset(&o, 0, sizeof o);
        o.d = &d; o.ob = &ob; o.wtype = p->window_type; o.ts = ts;
        so.ts = ts;
        int64_t u = unit_ms(p->time_unit);
        o.L = (int64_t)p->length * u; o.I = (int64_t)p->interval * u; o.D = (int64_t)p->delay * u;
        o.raw_interval = (p->window_type == EK_WINDOW_HOPPING) ? p->interval : p->length; /* planner.go:394-400 */
        o.unit = p->time_unit; o.tz = p->tz_offset_s;
        o.next_end = MAXT_MS; o.prev_end = ZERO_MS;
        o.send_twice = p->sliding_send_twice && p->window_type == EK_WINDOW_SLIDING && o.D > 0;

        /* WatermarkOp (single stream) watermark_op.go:54-67,144-225 */
        int64_t lateTol = p->late_tolerance_ms;
        int64_t stream_wm = ZERO_MS + lateTol;
        int64_t last_wm = ZERO_MS;
        vec64 buf; memset(&buf, 0, sizeof buf);
        for (int64_t i = 0; i < n; ++i) {
            int64_t t = ts[i];
            if (t > stream_wm) stream_wm = t;
            if (!(t >= last_wm)) { out->records_late++; continue; }
            /* insert after all events with ts <= t (sort.Search(After)) */
            int64_t lo = 0, hi = buf.n;
            while (lo < hi) { int64_t mid = (lo + hi) / 2; if (ts[buf.a[mid]] > t) hi = mid; else lo = mid + 1; }
            v_push(&buf, 0);
            memmove(buf.a + lo + 1, buf.a + lo, (size_t)(buf.n - 1 - lo) * 8);
            buf.a[lo] = i;
            int64_t wm = stream_wm - lateTol;
            if (wm > last_wm) {
                if (wm >= ts[buf.a[0]]) {
                    int64_t c = buf.n;
                    for (int64_t k = 0; k < buf.n; ++k) if (ts[buf.a[k]] > wm) { c = k; break; }
                    for (int64_t k = 0; k < c; ++k) {
                        /* the window's FILTER (WHERE ...) op between WatermarkOp and the window (planner.go:388-392) */
                        if (!filter_pass(&d, buf.a[k], &out->records_filter_error)) continue;
                        if (p->window_type == EK_WINDOW_STATE) state_on_row(&so, buf.a[k]);
                        else if (inc_slide) incslide_on_event(&isl, buf.a[k]);
                        else if (inc_count) inccount_on_event(&icn, buf.a[k]);
                        else if (v2slide) v2slide_on_row(&o, buf.a[k]);
                        else if (inc) inc_on_event(&io, buf.a[k]);
                        else win_on_event(&o, buf.a[k]);
                    }
                    v_erase_front(&buf, c);
                }
                if (p->window_type == EK_WINDOW_STATE) { /* WatermarkTuple: no effect on StateWindowOp */ }
                else if (inc_slide) incslide_on_watermark(&isl, wm);
                else if (inc_count) inccount_on_watermark(&icn, wm);
                else if (v2slide) v2slide_on_watermark(&o, wm);
                else if (inc) inc_on_watermark(&io, wm); else win_on_watermark(&o, wm);
                last_wm = wm;
            }
        }
        for (int64_t k = 0; k < io.nw; ++k) free(io.w[k].mem.a);
        free(io.w);
        for (int64_t k = 0; k < isl.nw; ++k) free(isl.w[k].mem.a);
        for (int64_t k = 0; k < isl.ne; ++k) free(isl.e[k].mem.a);
        free(isl.w); free(isl.e);
        for (int64_t k = 0; k < icn.ne; ++k) free(icn.e[k].mem.a);
        free(icn.e); free(icn.cur.a);
        free(buf.a); free(o.inputs.a); free(o.trigger_ts.a); free(o.delay_ts.a); free(o.content.a);
        free(ts);
    } else if (p->window_type == EK_WINDOW_STATE) {
        /* processing time: WHERE is pushed below the window with the FILTER (windowPlan.go:82-99): the rows it keeps
         * reach StateWindowOp; WHERE above the window then holds for every row (emit_window re-tests it: a no-op) */
        for (int64_t i = 0; i < n; ++i)
            if (pushdown_pass(&d, i, &out->records_filter_error)) state_on_row(&so, i);
    } else {
        if (p->window_type == EK_WINDOW_NONE) {
            /* window-less rule: FilterOp.Apply per event (filter_operator.go:36-90) + SELECT * projection.
             * One output segment: rows = passing events in arrival order, key = row index, value c = column c. */
            if (p->n_aggs != 0) { set_status(out, EK_ERR_UNSUPPORTED, "aggregates need a window"); return out->status; }
            v_push(&ob.ws, 0); v_push(&ob.we, 0); v_push(&ob.roff, 0); v_push(&ob.moff, 0);
            uint64_t h = 0;
            for (int64_t i = 0; i < n; ++i) {
                v_push(&ob.mem, i);
                h += ek_mix64((uint64_t)i);
                if (p->n_where > 0) {
                    val_t r = eval_prog(p->where_prog, p->n_where, &d, i, NULL);
                    if (!(r.tag == V_BOOL && r.i)) continue;   /* nil/false dropped; an error drops the event */
                }
                v_push(&ob.key, i);
                for (int c = 0; c < p->n_columns; ++c) {
                    val_t v = col_val(&d, c, i);
                    int64_t bits = v.i;
                    if (v.tag == V_F64) memcpy(&bits, &v.f, 8);
                    v_push(&ob.aval[c], v.tag == V_NULL ? 0 : bits);
                    v_push(&ob.atag[c], v.tag == V_NULL ? EK_TAG_NULL
                                        : v.tag == V_F64 ? EK_TAG_F64 : v.tag == V_BOOL ? EK_TAG_BOOL : EK_TAG_I64);
                }
            }
            v_push(&ob.mcnt, n);
            v_push(&ob.mhash, (int64_t)h);
            v_push(&ob.rcnt, ob.key.n);
            v_push(&ob.st, EK_WIN_OK);
            ob.werr = (char*)calloc(128, 1);
            ob.werr_cap = 1;
        } else if (p->window_type != EK_WINDOW_COUNT) {
            set_status(out, EK_ERR_UNSUPPORTED, "processing-time oracle supports COUNTWINDOW only"); return out->status;
        } else {
        /* window_op.go:390-418 + TupleList 502-551; CountInterval defaults to CountLength (window_op.go:100-103) */
        int64_t len = p->length, itv = p->interval > 0 ? p->interval : p->length;
        if (len <= 0) { set_status(out, EK_ERR_INVALID, "Window size should not be less than zero."); return out->status; }
        vec64 inputs; memset(&inputs, 0, sizeof inputs);
        int64_t msg = 0;
        for (int64_t i = 0; i < n; ++i) {
            if (!filter_pass(&d, i, &out->records_filter_error)) continue;   /* window FILTER before the window */
            v_push(&inputs, i);
            msg++;
            if (msg % itv != 0) continue;
            msg = 0;
            if (inputs.n >= len) {
                /* CountWindowIncAggOp (window_inc_agg_op.go:239-314): the same consecutive blocks of len rows */
                if (inc_ok) emit_inc_window(&d, &ob, 0, 0, inputs.a + (inputs.n - len), len);
                else emit_window(&d, &ob, 0, 0, inputs.a + (inputs.n - len), len);  /* wall-clock range: not comparable */
                v_erase_front(&inputs, inputs.n - len + 1);
            }
        }
        free(inputs.a);
        }
    }

    free(so.rows.a);
    finish_output(p, &ob, out);
    return 0;
}

/* ------------------------------------------------------------------ processing time (deterministic clock)
 * WindowOperator.execProcessingWindow (window_op.go:235-470) for TUMBLING / HOPPING / SLIDING / SESSION, driven by a
 * clock the way the reference's own tests drive it (pkg/timex/time.go:31-100 mock clock; topotest/mock_topo.go:208-235,
 * 263-268): the rule opens at start_ms (Exec sets triggerTime = now, window_op.go:149-151); before row i is delivered
 * the clock is set to its timestamp ts_i (the row's arrival time) and every timer due at or before ts_i fires first,
 * in due order (a ticker before a session timeout due at the same instant); after the last row the clock moves to
 * end_ms.
 *   tickers (getFirstTimer + setupTicker, window_op.go:228-233,250-260,471-481): the first tick at
 *     getAlignedWindowEndTime(start_ms, rawInterval) (rawInterval = length for tumbling / session, interval for
 *     hopping, planner.go:394-400), then every length (tumbling, session) or interval (hopping);
 *   tick (window_op.go:483-499): scan(tick); a session window scans only when it has inputs and the first one is at
 *     least `length` before the tick;
 *   rows (window_op.go:343-419): appended to the inputs; SLIDING: a row matching OVER (WHEN) scans at its own
 *     timestamp, or with a delay D arms a timer due at ts + D (window_op.go:355-373) that scans [ts - length, ts + D)
 *     — with enableSlidingWindowSendTwice the row first scans its first part (ts - length, ts] and the timer the second
 *     part (ts, ts + D]; any other row garbage-collects the inputs that expired (gcInputs, window_op.go:657-673:
 *     ts + length + delay <= t); SESSION: the timeout timer is (re)armed at ts + timeout, the first row of a session
 *     sets triggerTime;
 *   session timeout (window_op.go:448-461): scan(now) over the whole inputs, then every input is dropped.
 * WHERE / FILTER: windowPlan.PushDownPredicate (windowPlan.go:82-99) moves WHERE AND the window's FILTER below a
 * processing-time TUMBLING / HOPPING / SESSION window: a row whose combined condition is not true never reaches the
 * window (an evaluation error drops the row; the reference forwards that error by itself, not as a window result).
 * Under SLIDING the FILTER op alone sits before the window (planner.go:388-392) and WHERE stays above it.
 * Restart (rs != NULL, rs->split >= 0): rows [0, split) are delivered, the clock moves to rs->export_ms and the rule
 * is checkpointed — inputs, triggerTime once a scan or a session's first row stored it (TriggerTimeKey) — then it
 * restarts at rs->restart_ms: the timers are gone (a session's timeout is re-armed by its next row), the tickers are
 * re-aligned to the restart, triggerTime is the restored one or the restart time, and the restored inputs are
 * replayed (window_op.go:268-325): TUMBLING / HOPPING scan at triggerTime + k * interval while <= restart + interval;
 * SESSION scans at the next session end computed over the inputs while <= restart + timeout (the reference panics on
 * inputs[0] once a replay emptied the inputs and re-scans the same end forever when none is found: both stop the
 * replay here). Rows must arrive with non-decreasing ts. */
/* ------------------------------------------------------------------ processing-time incremental windows
 * TumblingWindowIncAggOp / HoppingWindowIncAggOp / SlidingWindowIncAggOp (window_inc_agg_op.go:316-790) under the
 * same deterministic clock as eko_run_proc (rows delivered at their arrival ts, every timer due at or before a row
 * fires first; timers at one instant in creation order). A window's content = the rows incAggCal added to it, in
 * delivery order; emit() broadcasts the window even when no row joined it (WindowRange [StartTime, now]).
 *   TUMBLING (:359-457): aligned (EnableAlignWindow, the default): the window opened at the rule's start, the
 *     FirstTimer at getAlignedWindowEndTime(start, rawInterval = length) emits it, then a ticker every length emits the
 *     open window if a row opened one (newIncAggWindow at that row's ts); unaligned: ticker every length from the
 *     start, no window before the first row.
 *   HOPPING (:666-760): aligned: a window at the start that nothing emits (no timer), the FirstTimer at
 *     getAlignedWindowEndTime(start, rawInterval = interval) then every interval opens a window with an emit timer at
 *     its start + length; unaligned: the same from a window opened at the start; a row joins every window with
 *     start <= ts < start + length (calIncAggWindow; gcIncAggWindow only drops windows no later row can join).
 *   SLIDING (:536-566): per row: gcIncAggWindow(length + delay), a new window at its ts, the row joins every window;
 *     a row matching OVER (WHEN) emits the oldest window (CurrWindowList[0]) at once, or with a delay D arms a timer
 *     due at ts + D that gcs (length + delay) and emits the oldest window if any.
 * The window FILTER op sits before the window (planner.go:360-365). WHERE stays above it (IncWindowPlan keeps the
 * predicate, incAggPlan.go:76-78): it filters the emitted rows, each a group's LAST row (emit_inc_window_ex). */
typedef struct { int64_t due, widx; } inc_timer;
static int proc_inc_run(const ek_plan* p, const dataset* d, outbuf* ob, const int64_t* ts, int64_t n, int64_t start_ms,
                        int64_t end_ms, int64_t* n_filter_err) {
    const int wt = p->window_type;
    const int64_t u = unit_ms(p->time_unit);
    const int64_t L = (int64_t)p->length * u, D = wt == EK_WINDOW_SLIDING ? (int64_t)p->delay * u : 0;
    const int64_t I = wt == EK_WINDOW_HOPPING ? (int64_t)p->interval * u : L;   /* IncWindowPlan.Init: tumbling I = L */
    const int32_t raw = wt == EK_WINDOW_HOPPING ? p->interval : p->length;
    const int aligned = !p->inc_unaligned;
    incwin* w = NULL; int64_t nw = 0, cap = 0;   /* every window ever opened (index = creation order) */
    inc_timer* tm = NULL; int64_t ntm = 0, tcap = 0, thead = 0;   /* emit timers (hopping / delayed sliding), due order */
    int64_t cur = -1;                            /* tumbling: the open window */
    int64_t head = 0;                            /* sliding: CurrWindowList = windows [head, nw) */
#define PI_OPEN(st) do { if (nw == cap) { cap = cap ? 2 * cap : 16; w = (incwin*)realloc(w, (size_t)cap * sizeof(incwin)); } \
                         memset(&w[nw], 0, sizeof(incwin)); w[nw++].start = (st); } while (0)
#define PI_TIMER(d_, wi) do { if (ntm == tcap) { tcap = tcap ? 2 * tcap : 16; tm = (inc_timer*)realloc(tm, (size_t)tcap * sizeof(inc_timer)); } \
                              tm[ntm].due = (d_); tm[ntm].widx = (wi); ntm++; } while (0)
    int64_t tick = MAXT_MS;
    if (wt == EK_WINDOW_TUMBLING) {
        if (aligned) { PI_OPEN(start_ms); cur = nw - 1; tick = eko_aligned_window_end(start_ms, raw, p->time_unit, p->tz_offset_s); }
        else tick = start_ms + I;
    } else if (wt == EK_WINDOW_HOPPING) {
        PI_OPEN(start_ms);
        if (aligned) tick = eko_aligned_window_end(start_ms, raw, p->time_unit, p->tz_offset_s);
        else { PI_TIMER(start_ms + L, nw - 1); tick = start_ms + I; }
    }
    /* timers due at or before `now`: the ticker (tumbling / hopping) and the emit timers, earliest first (an emit
     * timer before a tick at the same instant: either order emits the same windows) */
    for (int64_t i = 0; i <= n; ++i) {
        const int64_t now = i < n ? ts[i] : end_ms;
        for (;;) {
            const int em = thead < ntm && tm[thead].due <= now;
            const int tk = tick <= now;
            if (em && (!tk || tm[thead].due <= tick)) {
                const inc_timer t = tm[thead++];
                if (wt == EK_WINDOW_SLIDING) {
                    while (head < nw && t.due - w[head].start >= L + D) head++;   /* gcIncAggWindow(length + delay) */
                    if (head < nw) emit_inc_window_ex(d, ob, w[head].start, t.due, w[head].mem.a, w[head].mem.n, 1);
                } else {
                    emit_inc_window_ex(d, ob, w[t.widx].start, t.due, w[t.widx].mem.a, w[t.widx].mem.n, 1);
                }
            } else if (tk) {
                if (wt == EK_WINDOW_TUMBLING) {
                    if (cur >= 0) emit_inc_window_ex(d, ob, w[cur].start, tick, w[cur].mem.a, w[cur].mem.n, 1);
                    cur = -1;
                } else {
                    PI_OPEN(tick);
                    PI_TIMER(tick + L, nw - 1);
                }
                tick += I;
            } else break;
        }
        if (i == n) break;
        if (!filter_pass(d, i, n_filter_err)) continue;   /* the window FILTER op before the window */
        const int64_t t = ts[i];
        if (wt == EK_WINDOW_TUMBLING) {
            if (cur < 0) { PI_OPEN(t); cur = nw - 1; }
            v_push(&w[cur].mem, i);
        } else if (wt == EK_WINDOW_HOPPING) {
            for (int64_t k = 0; k < nw; ++k)
                if (w[k].start <= t && t < w[k].start + L) v_push(&w[k].mem, i);
        } else {
            while (head < nw && t - w[head].start >= L + D) head++;
            PI_OPEN(t);
            for (int64_t k = head; k < nw; ++k)
                if (w[k].start <= t && t < w[k].start + L + D) v_push(&w[k].mem, i);
            int trig = 1;
            if (p->n_trigger > 0) { const val_t r = eval_prog(p->trigger_prog, p->n_trigger, d, i, NULL); trig = r.tag == V_BOOL && r.i; }
            if (trig) {
                if (D > 0) PI_TIMER(t + D, -1);
                else emit_inc_window_ex(d, ob, w[head].start, t, w[head].mem.a, w[head].mem.n, 1);
            }
        }
    }
#undef PI_OPEN
#undef PI_TIMER
    for (int64_t k = 0; k < nw; ++k) free(w[k].mem.a);
    free(w); free(tm);
    return 0;
}

/* WindowV2Operator SlidingWindowOp (window_v2_op.go:160-215) in processing time, under the same clock: a row at t
 * (its arrival = tuple.Timestamp) first gcs the scanner (WindowScanner.gc(t - length): rows with ts <= t - length go),
 * is added, and when it matches OVER (WHEN) (isMatchCondition) emits scanWindow(t - length, t) — the scanner's rows with
 * t - length < ts <= t (window_v2_op.go:252-263) — or, with a delay D, arms a timer due at t + D that emits
 * scanWindow(t - length, t + D) over the scanner as the later rows' gcs left it. WindowRange [start, end]. The window
 * FILTER op sits in front (planner.go:388-392); WHERE stays above the window (emit_window). */
static void proc_v2slide_run(const ek_plan* p, const dataset* d, outbuf* ob, const int64_t* ts, int64_t n, int64_t end_ms,
                             int64_t* n_filter_err) {
    const int64_t u = unit_ms(p->time_unit);
    const int64_t L = (int64_t)p->length * u, D = (int64_t)p->delay * u;
    vec64 tup; memset(&tup, 0, sizeof tup);   /* the scanner: delivered rows, [head, n) live */
    int64_t head = 0;
    vec64 dq; memset(&dq, 0, sizeof dq);      /* timers: the trigger ts, due at ts + D */
    int64_t dq_head = 0;
    vec64 c; memset(&c, 0, sizeof c);
    for (int64_t i = 0; i <= n; ++i) {
        const int64_t now = i < n ? ts[i] : end_ms;
        while (dq_head < dq.n && dq.a[dq_head] + D <= now) {
            const int64_t t = dq.a[dq_head++], we = t + D, wsb = t - L;
            c.n = 0;
            for (int64_t k = head; k < tup.n; ++k) {
                const int64_t x = ts[tup.a[k]];
                if (x > wsb && x <= we) v_push(&c, tup.a[k]);
                else if (x > we) break;
            }
            emit_window(d, ob, wsb, we, c.a, c.n);
        }
        if (i == n) break;
        if (!filter_pass(d, i, n_filter_err)) continue;
        const int64_t t = ts[i];
        while (head < tup.n && ts[tup.a[head]] <= t - L) head++;   /* gc(t - length) */
        v_push(&tup, i);
        int trig = 1;
        if (p->n_trigger > 0) { const val_t r = eval_prog(p->trigger_prog, p->n_trigger, d, i, NULL); trig = r.tag == V_BOOL && r.i; }
        if (!trig) continue;
        if (D > 0) { v_push(&dq, t); continue; }
        c.n = 0;
        for (int64_t k = head; k < tup.n; ++k)
            if (ts[tup.a[k]] > t - L && ts[tup.a[k]] <= t) v_push(&c, tup.a[k]);
        emit_window(d, ob, t - L, t, c.a, c.n);
    }
    free(tup.a); free(dq.a); free(c.a);
}

int eko_run_proc_restart(const ek_plan* p, int64_t n, const void* const* columns, const uint8_t* const* validity,
                         int64_t start_ms, int64_t end_ms, const eko_restart* rs, eko_output* out) {
    memset(out, 0, sizeof *out);
    if (!p || p->abi_version != EKGPU_ABI_VERSION) { set_status(out, EK_ERR_INVALID, "abi version mismatch"); return out->status; }
    const int wt = p->window_type;
    if (p->is_event_time || !(wt == EK_WINDOW_TUMBLING || wt == EK_WINDOW_HOPPING || wt == EK_WINDOW_SLIDING || wt == EK_WINDOW_SESSION)) {
        set_status(out, EK_ERR_UNSUPPORTED, "processing-time clock runs are for TUMBLING / HOPPING / SLIDING / SESSION"); return out->status;
    }
    int inc_ok = p->incremental != 0 && p->n_aggs > 0 && wt != EK_WINDOW_SESSION;
    for (int a = 0; a < p->n_aggs; ++a) inc_ok &= inc_supported_fn(p->aggs[a].fn);
    const int v2slide = p->window_version == 2 && wt == EK_WINDOW_SLIDING && !inc_ok;
    if (p->window_version == 2 && !v2slide) { set_status(out, EK_ERR_UNSUPPORTED, "v2 windows are not restated in processing time"); return out->status; }
    if (p->ts_column < 0) { set_status(out, EK_ERR_INVALID, "processing-time rows need their arrival timestamp column"); return out->status; }
    if (inc_ok || v2slide) {
        if (rs && rs->split >= 0) { set_status(out, EK_ERR_UNSUPPORTED, "restart of processing-time incremental / v2 windows is not restated"); return out->status; }
        dataset d = { p, n, columns, validity, NULL };
        outbuf ob; memset(&ob, 0, sizeof ob);
        int64_t* ts = (int64_t*)malloc((size_t)(n ? n : 1) * 8);
        for (int64_t i = 0; i < n; ++i) { val_t v = col_val(&d, p->ts_column, i); ts[i] = v.tag == V_F64 ? (int64_t)v.f : v.i; }
        for (int64_t i = 0; i < n; ++i)
            if ((i > 0 && ts[i] < ts[i - 1]) || ts[i] < start_ms) {
                free(ts); set_status(out, EK_ERR_INVALID, "processing-time rows must arrive with non-decreasing timestamps after the start"); return out->status;
            }
        if (v2slide) proc_v2slide_run(p, &d, &ob, ts, n, end_ms, &out->records_filter_error);
        else proc_inc_run(p, &d, &ob, ts, n, start_ms, end_ms, &out->records_filter_error);
        free(ts);
        finish_output(p, &ob, out);
        return 0;
    }
    const int64_t split = rs && rs->split >= 0 ? (rs->split < n ? rs->split : n) : -1;
    if (split >= 0 && (rs->export_ms < start_ms || rs->restart_ms < rs->export_ms)) {
        set_status(out, EK_ERR_INVALID, "restart: start <= export <= restart"); return out->status;
    }
    dataset d = { p, n, columns, validity, NULL };
    outbuf ob; memset(&ob, 0, sizeof ob);
    int64_t* ts = (int64_t*)malloc((size_t)(n ? n : 1) * 8);
    for (int64_t i = 0; i < n; ++i) { val_t v = col_val(&d, p->ts_column, i); ts[i] = v.tag == V_F64 ? (int64_t)v.f : v.i; }
    for (int64_t i = 0; i < n; ++i)
        if ((i > 0 && ts[i] < ts[i - 1]) || ts[i] < start_ms || (split >= 0 && i < split && ts[i] > rs->export_ms) ||
            (split >= 0 && i >= split && ts[i] < rs->restart_ms)) {
            free(ts); set_status(out, EK_ERR_INVALID, "processing-time rows must arrive with non-decreasing timestamps after the start"); return out->status;
        }
    winop o; memset(&o, 0, sizeof o);
    o.d = &d; o.ob = &ob; o.wtype = wt; o.ts = ts;
    const int64_t u = unit_ms(p->time_unit);
    o.L = (int64_t)p->length * u; o.I = (int64_t)p->interval * u; o.D = (int64_t)p->delay * u;
    o.raw_interval = wt == EK_WINDOW_HOPPING ? p->interval : p->length;
    o.unit = p->time_unit; o.tz = p->tz_offset_s;
    o.send_twice = p->sliding_send_twice && wt == EK_WINDOW_SLIDING && o.D > 0;
    /* Exec: triggerTime = now in processing time (window_op.go:149-151) */
    o.has_trigger = 1; o.trigger_time = start_ms;
    int trig_saved = 0;   /* TriggerTimeKey was put (a tick / timeout scan, a session's first row) */
    const int pushdown = wt != EK_WINDOW_SLIDING;
    const int has_tick = wt != EK_WINDOW_SLIDING;
    int64_t tick = has_tick ? eko_aligned_window_end(start_ms, o.raw_interval, o.unit, o.tz) : MAXT_MS;
    const int64_t period = wt == EK_WINDOW_HOPPING ? o.I : o.L;
    int to_exists = 0, to_armed = 0;
    int64_t to_due = 0;
    vec64 dq; memset(&dq, 0, sizeof dq);   /* delayed sliding timers: due times, in order */
    int64_t dq_head = 0;
    /* every timer due at or before `now`, in due order (ticker first on a tie; delay timers are sliding-only) */
#define EKO_ADVANCE(now)                                                                                        \
    for (;;) {                                                                                                  \
        const int tk = has_tick && tick <= (now);                                                               \
        const int tm = wt == EK_WINDOW_SESSION && to_armed && to_due <= (now) && (!tk || to_due < tick);        \
        const int dl = dq_head < dq.n && dq.a[dq_head] <= (now);                                                \
        if (tm) {                                                                                               \
            to_armed = 0;                                                                                       \
            if (o.inputs.n > 0) { scan(&o, to_due, o.L + o.D, 1); o.inputs.n = 0; to_exists = 0; trig_saved = 1; } \
        } else if (tk) {                                                                                        \
            if (wt != EK_WINDOW_SESSION || (o.inputs.n > 0 && tick - ts[o.inputs.a[0]] >= o.L)) {               \
                scan(&o, tick, o.L + o.D, 1); trig_saved = 1;                                                   \
            }                                                                                                   \
            tick += period;                                                                                     \
        } else if (dl) {                                                                                        \
            const int64_t due = dq.a[dq_head++];                                                                \
            if (o.send_twice) scan(&o, due, o.D, 0);   /* the last part (t, t + D] */                           \
            else scan(&o, due, o.L + o.D, 1);                                                                   \
        } else break;                                                                                           \
    }
    for (int64_t i = 0; i <= n; ++i) {
        if (i == split) {
            EKO_ADVANCE(rs->export_ms)
            /* checkpoint at export_ms, restart at restart_ms: timers gone, tickers re-aligned, inputs replayed */
            to_armed = 0; to_exists = 0; dq_head = dq.n;
            if (!trig_saved) { o.trigger_time = rs->restart_ms; o.has_trigger = 1; }
            const int64_t R = rs->restart_ms;
            if (o.inputs.n > 0 && (wt == EK_WINDOW_TUMBLING || wt == EK_WINDOW_HOPPING)) {
                const int64_t itv = wt == EK_WINDOW_HOPPING ? o.I : o.L, next_tick = R + itv;
                for (int64_t next = o.trigger_time + itv; next <= next_tick; next += itv) scan(&o, next, o.L + o.D, 1);
            } else if (o.inputs.n > 0 && wt == EK_WINDOW_SESSION) {
                const int64_t timeout = o.I, duration = o.L, next_tick = R + o.I;
                while (o.inputs.n > 0) {
                    const int64_t et = ts[o.inputs.a[0]];
                    const int64_t dd = et % duration;
                    int64_t tk2 = dd == 0 ? et : et + duration - dd;
                    int64_t pp = ZERO_MS, next = MAXT_MS;
                    for (int64_t k = 0; k < o.inputs.n; ++k) {
                        const int64_t tt = ts[o.inputs.a[k]];
                        int64_t r = MAXT_MS;
                        if (pp != ZERO_MS && tt - pp > timeout) r = pp + timeout;
                        if (tt > tk2) {
                            if (tk2 - et > duration && tk2 < r) r = tk2;
                            tk2 += duration;
                        }
                        if (r < MAXT_MS) { next = r; break; }
                        pp = tt;
                    }
                    if (next == MAXT_MS || next > next_tick) break;
                    scan(&o, next, o.L + o.D, 1);
                }
            }
            if (has_tick) tick = eko_aligned_window_end(R, o.raw_interval, o.unit, o.tz);
        }
        if (i == n) break;
        EKO_ADVANCE(ts[i])
        if (pushdown) {
            /* WHERE AND FILTER below the window */
            if (!pushdown_pass(&d, i, &out->records_filter_error)) continue;
        } else if (!filter_pass(&d, i, &out->records_filter_error)) {
            continue;   /* the window's FILTER op before a sliding window */
        }
        v_push(&o.inputs, i);
        if (wt == EK_WINDOW_SESSION) {
            if (!to_exists) { to_exists = 1; o.trigger_time = ts[i]; o.has_trigger = 1; trig_saved = 1; }
            to_armed = 1;
            to_due = ts[i] + o.I;
        } else if (wt == EK_WINDOW_SLIDING) {
            if (match_trigger(&o, i)) {
                if (o.D > 0) {
                    if (o.send_twice) scan(&o, ts[i], o.L, 1);   /* the first part (t - length, t] */
                    v_push(&dq, ts[i] + o.D);
                } else {
                    scan(&o, ts[i], o.L + o.D, 1);
                }
            } else {
                int64_t g = 0;   /* gcInputs(inputs, ts + 1ns): drop the prefix with ts_k + length + delay <= ts */
                while (g < o.inputs.n && ts[o.inputs.a[g]] + o.L + o.D <= ts[i]) g++;
                v_erase_front(&o.inputs, g);
            }
        }
    }
    EKO_ADVANCE(end_ms)
#undef EKO_ADVANCE
    free(o.inputs.a); free(o.trigger_ts.a); free(o.delay_ts.a); free(o.content.a); free(dq.a);
    free(ts);
    finish_output(p, &ob, out);
    return 0;
}

int eko_run_proc(const ek_plan* p, int64_t n, const void* const* columns, const uint8_t* const* validity,
                 int64_t start_ms, int64_t end_ms, eko_output* out) {
    return eko_run_proc_restart(p, n, columns, validity, start_ms, end_ms, NULL, out);
}

/* ------------------------------------------------------------------ shard model (multi-GPU protocol)
 * One key-hash shard of a rule: the shard's own rows (global arrival indices g->row_arrival) plus the global
 * WatermarkTuples (wm list), the global window anchor (origin) and the global sliding triggers — exactly what
 * ek_push_batch_global hands one engine handle. The WatermarkOp tracking runs over the WHOLE stream on the host
 * (ekgpu/shard.py GlobalWatermark, watermark_op.go:144-225); here, per shard:
 *   track:    a row is accepted iff ts >= the last watermark emitted before its arrival (watermark_op.go:144-155)
 *   release:  at each WatermarkTuple, the buffered rows / trigger ghosts with ts <= watermark, in (ts, arrival)
 *             order (watermark_op.go:157-204), then the window op's WatermarkTuple branch
 *   hopping:  the "empty window discards every input" quirk (window_op.go:605-655) for lateTolerance 0, decided
 *             per event: event i reaches no window iff ts_i > W_{i-1} and e_max(ts_i) - L > W_{i-1}
 *   count:    processing-time COUNTWINDOW blocks over the GLOBAL arrival order (window_op.go:390-418)
 *   session:  the sessions the router closed over the WHOLE stream (g->sess_*), each at its tuple, over the
 *             shard's inputs with ts < end
 *   sliding:  every global trigger fires at the tuple releasing it; with a delay D it queues t + D and the window
 *             [t - L, t + D) over the shard's inputs fires at the first LATER tuple reaching it (send-twice is not
 *             shardable: its expired-prefix rule depends on every input of the stream)
 * The union of the shards' rows (and the sum of their membership fingerprints) is compared with eko_run on the
 * whole stream by the tests. */
int eko_run_shard(const ek_plan* p, int64_t n, const void* const* columns, const uint8_t* const* validity,
                  const ek_global_ctx* g, eko_output* out) {
    memset(out, 0, sizeof *out);
    if (!p || p->abi_version != EKGPU_ABI_VERSION || !g) { set_status(out, EK_ERR_INVALID, "bad plan / context"); return out->status; }
    if (p->incremental || p->window_version == 2 || p->window_type == EK_WINDOW_STATE ||
        p->window_type == EK_WINDOW_NONE || (p->window_type == EK_WINDOW_SLIDING && p->delay != 0 && p->sliding_send_twice) ||
        (p->window_type == EK_WINDOW_HOPPING && p->late_tolerance_ms != 0) ||
        (p->window_type == EK_WINDOW_COUNT && p->is_event_time)) {
        set_status(out, EK_ERR_UNSUPPORTED, "window not shardable"); return out->status;
    }
    dataset d = { p, n, columns, validity, g->row_arrival };
    outbuf ob; memset(&ob, 0, sizeof ob);
    if (!p->is_event_time) {
        /* COUNTWINDOW(len, itv) over the global arrival order: window k = arrivals [k*itv - len, k*itv) */
        const int64_t len = p->length, itv = p->interval > 0 ? p->interval : p->length;
        int64_t lo = 0;
        for (int64_t e = itv; e <= g->arrivals_end; e += itv) {
            if (e < len) continue;
            while (lo < n && g->row_arrival[lo] < e - len) lo++;
            int64_t hi = lo;
            while (hi < n && g->row_arrival[hi] < e) hi++;
            vec64 c; memset(&c, 0, sizeof c);
            for (int64_t k = lo; k < hi; ++k) v_push(&c, k);
            emit_window(&d, &ob, 0, 0, c.a, c.n);
            free(c.a);
        }
        finish_output(p, &ob, out);
        return 0;
    }
    if (p->ts_column < 0) { set_status(out, EK_ERR_INVALID, "event time requires a timestamp column"); return out->status; }
    /* ts of own rows [0, n) and of the trigger ghosts [n, n + n_trig) */
    const int64_t nt = p->window_type == EK_WINDOW_SLIDING ? g->n_trig : 0;
    int64_t* ts = (int64_t*)malloc((size_t)(n + nt + 1) * 8);
    for (int64_t i = 0; i < n; ++i) { val_t v = col_val(&d, p->ts_column, i); ts[i] = v.i; }
    for (int64_t k = 0; k < nt; ++k) ts[n + k] = g->trig_ts[k];
    winop o; memset(&o, 0, sizeof o);
    o.d = &d; o.ob = &ob; o.wtype = p->window_type; o.ts = ts;
    const int64_t u = unit_ms(p->time_unit);
    o.L = (int64_t)p->length * u; o.I = (int64_t)p->interval * u;
    o.D = p->window_type == EK_WINDOW_SLIDING ? (int64_t)p->delay * u : 0;   /* delayed sliding: the delay loop */
    o.raw_interval = (p->window_type == EK_WINDOW_HOPPING) ? p->interval : p->length;
    o.unit = p->time_unit; o.tz = p->tz_offset_s;
    o.next_end = MAXT_MS; o.prev_end = ZERO_MS;
    o.shard = 1;
    o.origin_known = g->origin_known; o.origin_ts = g->origin_ts; o.origin_arrival = g->origin_arrival;
    if (p->window_type == EK_WINDOW_SESSION) {
        if (g->n_sess > 0 && (!g->sess_start || !g->sess_end || !g->sess_wm)) {
            free(ts); set_status(out, EK_ERR_INVALID, "missing session list"); return out->status;
        }
        o.I = (int64_t)p->interval * u;   /* the session timeout */
        o.sess_start = g->sess_start; o.sess_end = g->sess_end; o.sess_wm = g->sess_wm; o.n_sess = g->n_sess;
    }
    const int64_t H = p->window_type == EK_WINDOW_HOPPING ? o.I : o.L;
    int64_t last_wm = ZERO_MS;
    vec64 buf; memset(&buf, 0, sizeof buf);   /* own rows (< n) and trigger ghosts (>= n), release order */
    int64_t ir = 0, iw = 0, itr = 0;
    for (;;) {
        int64_t a = INT64_MAX;
        if (ir < n) a = g->row_arrival[ir];
        if (itr < nt && g->trig_arrival[itr] < a) a = g->trig_arrival[itr];
        if (iw < g->n_wm && g->wm_arrival[iw] < a) a = g->wm_arrival[iw];
        if (a == INT64_MAX) break;
        int64_t add[2]; int na = 0;
        if (ir < n && g->row_arrival[ir] == a) {
            const int64_t t = ts[ir];
            int ok = t >= last_wm;
            if (!ok) out->records_late++;
            if (ok && p->window_type == EK_WINDOW_HOPPING && o.origin_known && t > last_wm) {
                const int64_t e1 = eko_aligned_window_end(o.origin_ts, o.raw_interval, o.unit, o.tz);
                if (t >= e1) {
                    const int64_t emax = e1 + floordiv(t - e1, H) * H;
                    if (emax - o.L > last_wm) ok = 0;   /* reaches no window: discarded with the empty window */
                }
            }
            if (ok) add[na++] = ir;
            ir++;
        }
        if (itr < nt && g->trig_arrival[itr] == a) add[na++] = n + itr++;
        for (int k = 0; k < na; ++k) {
            const int64_t e = add[k], t = ts[e];
            int64_t lo = 0, hi = buf.n;
            while (lo < hi) { int64_t mid = (lo + hi) / 2; if (ts[buf.a[mid]] > t) hi = mid; else lo = mid + 1; }
            v_push(&buf, 0);
            memmove(buf.a + lo + 1, buf.a + lo, (size_t)(buf.n - 1 - lo) * 8);
            buf.a[lo] = e;
        }
        if (iw < g->n_wm && g->wm_arrival[iw] == a) {
            const int64_t wm = g->wm_ts[iw++];
            o.cur_wm_arrival = a;
            int64_t c = 0;
            while (c < buf.n && ts[buf.a[c]] <= wm) c++;
            for (int64_t k = 0; k < c; ++k) {
                const int64_t e = buf.a[k];
                if (e < n) win_on_event(&o, e);
                else v_push(&o.trigger_ts, ts[e]);
            }
            v_erase_front(&buf, c);
            win_on_watermark(&o, wm);
            last_wm = wm;
        }
    }
    free(buf.a); free(o.inputs.a); free(o.trigger_ts.a); free(o.delay_ts.a); free(o.content.a); free(ts);
    finish_output(p, &ob, out);
    return 0;
}

/* The shard's accepted trigger rows (ek_shard_triggers): OVER (WHEN ...) true (every row without OVER) and
 * ts >= the last global watermark before the row's arrival. out_* sized n. Returns the count. */
int64_t eko_shard_triggers(const ek_plan* p, int64_t n, const void* const* columns, const uint8_t* const* validity,
                           const ek_global_ctx* g, int64_t* out_arrival, int64_t* out_ts) {
    dataset d = { p, n, columns, validity, g->row_arrival };
    int64_t k = 0, iw = 0, last_wm = ZERO_MS;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t a = g->row_arrival[i];
        while (iw < g->n_wm && g->wm_arrival[iw] < a) last_wm = g->wm_ts[iw++];
        const int64_t t = col_val(&d, p->ts_column, i).i;
        if (t < last_wm) continue;
        if (p->n_trigger > 0) {
            val_t r = eval_prog(p->trigger_prog, p->n_trigger, &d, i, NULL);
            if (!(r.tag == V_BOOL && r.i)) continue;
        }
        out_arrival[k] = a;
        out_ts[k] = t;
        k++;
    }
    return k;
}

void eko_free(eko_output* o) {
    if (!o) return;
    free(o->r.win_start); free(o->r.win_end); free(o->r.win_row_offset); free(o->r.win_row_count);
    free(o->r.win_status); free(o->r.win_member_count); free(o->r.win_member_hash); free(o->r.key);
    for (int a = 0; a < EK_MAX_AGGS; ++a) { free(o->r.agg_value[a]); free(o->r.agg_tag[a]); }
    free(o->member_offset); free(o->members); free(o->win_error);
    memset(o, 0, sizeof *o);
}
