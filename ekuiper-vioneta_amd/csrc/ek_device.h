// ek_device.h — device-side plan descriptor and helpers shared by the gfx950 kernels.
//
// Semantics restated from the reference:
//   expression evaluation      internal/xsql/valuer.go:574-660 (evalBinaryExpr), :823-1000 (SimpleDataEval)
//   aggregate finalisation     internal/binder/function/funcs_agg.go:28-297, common_array_funcs.go:27-247
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ekgpu.h"

namespace ek {

constexpr int kBlock = 256;       // 4 wave64s per workgroup
constexpr int kMaxVC = 4;         // value columns referenced by aggregates
constexpr uint32_t kPseudoKeys = 65536;   // partial slots of an un-grouped pane-mode rule

// fields kept per (pane, key) in the pane-partial state and per key in LDS tables
enum : int { NEED_CNT = 1, NEED_SUM = 2, NEED_MIN = 4, NEED_MAX = 8, NEED_M2 = 16, NEED_FSUM = 32, NEED_SORT = 64 };
constexpr int kMaxScol = 2;       // value columns of median / percentile_* (key-grouped scatter each)
constexpr int kMaxSortAggs = 4;   // median / percentile_* calls per rule
constexpr int kHStarTab = 2049;   // HAVING over count(*) alone decided per row count 0..2048 (k_small_win's windows)

struct DPlan {
    int32_t n_columns;
    int32_t col_type[EK_MAX_COLUMNS];
    int32_t ts_col;
    int32_t key_col;
    uint32_t num_keys;
    int32_t n_where, n_having, n_trigger;
    ek_instr where_prog[EK_MAX_PROG];
    ek_instr having_prog[EK_MAX_PROG];
    ek_instr trigger_prog[EK_MAX_PROG];
    int32_t n_vc;                 // distinct value columns used by aggregates
    int32_t vc_col[kMaxVC];       // -> plan column
    int32_t vc_flags[kMaxVC];     // NEED_*
    int32_t vc_is_float[kMaxVC];
    int32_t n_aggs;
    int32_t agg_fn[EK_MAX_AGGS];
    int32_t agg_vc[EK_MAX_AGGS];  // -1 for count(*)
    double agg_p[EK_MAX_AGGS];
    // order-statistic aggregates (median, percentile_cont/disc): per sort slot s < n_sagg its column slot
    int32_t n_scol;
    int32_t scol_vc[kMaxScol];    // value column (vc index) of sort column slot
    int32_t n_sagg;
    int32_t agg_sidx[EK_MAX_AGGS];  // sort slot of aggregate k (-1 otherwise)
    int32_t sagg_scol[kMaxSortAggs];
    int32_t sagg_agg[kMaxSortAggs];
    int32_t inc;                  // incremental-window semantics (inc_sum / inc_avg float64, funcs_inc_agg.go:56-117)
    int32_t n_begin, n_emit;      // STATEWINDOW(begin, emit) conditions (window_v2_op.go:111-148)
    int32_t n_user_cols;          // columns of the caller's batch; [n_user_cols, n_columns) are derived (aggregate args)
    int32_t n_derived_prog[EK_MAX_DERIVED];
    ek_instr derived_prog[EK_MAX_DERIVED][EK_MAX_PROG];
    int32_t n_first;              // EK_AGG_FIRST aggregates (non-aggregate select fields; range mode)
    int32_t first_col[EK_MAX_AGGS];   // their source columns (the aggregate itself is the min buffer position)
    int32_t pseudo_keys;          // no GROUP BY in pane mode: rows spread over kPseudoKeys partial slots by row index
                                  // (merged per window by k_finalize_merge) instead of one partition
    ek_instr begin_prog[EK_MAX_PROG];
    ek_instr emit_prog[EK_MAX_PROG];
    int32_t having_star;          // HAVING reads no aggregate but count(*): decidable from a group's row count alone
    // median over a nullable f64 column: its hidden EK_AGG_FIRST slot (the group's first row), -1 otherwise; a nil
    // there is the reference's "<nil> should be number" (funcs_agg.go:36-52)
    int32_t med_first[EK_MAX_AGGS];
    // having_star: the decision for a group of c rows (1 keep, 0 drop, -1 non-bool), c < kHStarTab, filled on the
    // device at create time by k_hstar_tab (the same evaluator), so k_small_win<HS> carries no interpreter
    int8_t hstar_tab[kHStarTab];
};

// Columns of one micro-batch (device pointers).
struct DBatch {
    const void* col[EK_MAX_COLUMNS];
    const uint8_t* valid[EK_MAX_COLUMNS];
    int64_t n;
};

// Pane-partial state: SoA field arrays of [slots * K] entries.
struct DState {
    int64_t* cnt;                 // count(*) of rows passing WHERE
    int64_t* vcnt[kMaxVC];        // non-nil count per value column
    int64_t* sum[kMaxVC];         // i64 sum or f64 bits
    int64_t* mn[kMaxVC];          // i64 or f64 bits
    int64_t* mx[kMaxVC];
    double* m2[kMaxVC];           // Σ (x - mean)^2 (two-pass per partial, Chan merge across partials)
    double* fsum[kMaxVC];         // f64 sum of an int column (for var on int columns)
    int64_t K;                    // keys per slot (padded)
};

// ---------------------------------------------------------------- ordered bits for f64 min/max
__device__ __forceinline__ uint64_t f64_to_ord(double d) {
    uint64_t u = (uint64_t)__double_as_longlong(d);
    return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double ord_to_f64(uint64_t o) {
    uint64_t u = (o & 0x8000000000000000ull) ? (o & 0x7FFFFFFFFFFFFFFFull) : ~o;
    return __longlong_as_double((long long)u);
}
__device__ __forceinline__ uint64_t i64_to_ord(int64_t v) { return (uint64_t)v ^ 0x8000000000000000ull; }
__device__ __forceinline__ int64_t ord_to_i64(uint64_t o) { return (int64_t)(o ^ 0x8000000000000000ull); }

// ---------------------------------------------------------------- column access
__device__ __forceinline__ bool col_valid(const DBatch& b, int c, int64_t i) {
    return b.valid[c] == nullptr || b.valid[c][i] != 0;
}
__device__ __forceinline__ int64_t col_i64(const DPlan& p, const DBatch& b, int c, int64_t i) {
    return p.col_type[c] == EK_COL_U32 ? (int64_t)((const uint32_t*)b.col[c])[i] : ((const int64_t*)b.col[c])[i];
}
__device__ __forceinline__ double col_f64(const DBatch& b, int c, int64_t i) { return ((const double*)b.col[c])[i]; }

// ---------------------------------------------------------------- expression interpreter
enum : int { V_NULL = 0, V_BOOL = 1, V_I64 = 2, V_F64 = 3, V_ERR = 4 };
struct Val {
    int tag;
    int64_t i;
    double f;
};
__device__ __forceinline__ Val mkb(bool b) { return Val{V_BOOL, b ? 1 : 0, 0.0}; }
// column c of row i as an evaluator value (NULL when invalid; a BOOLEAN column is a bool)
__device__ __forceinline__ Val col_val(const DPlan& p, const DBatch& b, int c, int64_t i) {
    if (!col_valid(b, c, i)) return Val{V_NULL, 0, 0.0};
    const int t = p.col_type[c];
    if (t == EK_COL_F64) return Val{V_F64, 0, col_f64(b, c, i)};
    const int64_t v = col_i64(p, b, c, i);
    return t == EK_COL_BOOL ? mkb(v != 0) : Val{V_I64, v, 0.0};
}

// valuer.go:823-1000 SimpleDataEval over the plan ISA
__device__ inline Val simple_eval(Val l, Val r, int op) {
    if (l.tag == V_NULL || r.tag == V_NULL) {
        if (op >= EK_OP_EQ && op <= EK_OP_OR) return mkb(false);
        return Val{V_NULL, 0, 0.0};
    }
    if (l.tag == V_BOOL || r.tag == V_BOOL) {
        if (l.tag != V_BOOL || r.tag != V_BOOL) return Val{V_ERR, 0, 0.0};
        switch (op) {
        case EK_OP_AND: return mkb(l.i && r.i);
        case EK_OP_OR: return mkb(l.i || r.i);
        case EK_OP_EQ: return mkb(l.i == r.i);
        case EK_OP_NEQ: return mkb(l.i != r.i);
        default: return Val{V_ERR, 0, 0.0};
        }
    }
    if (l.tag == V_F64 || r.tag == V_F64) {
        double a = l.tag == V_F64 ? l.f : (double)l.i;
        double c = r.tag == V_F64 ? r.f : (double)r.i;
        switch (op) {
        case EK_OP_EQ: return mkb(a == c);
        case EK_OP_NEQ: return mkb(a != c);
        case EK_OP_LT: return mkb(a < c);
        case EK_OP_LTE: return mkb(a <= c);
        case EK_OP_GT: return mkb(a > c);
        case EK_OP_GTE: return mkb(a >= c);
        case EK_OP_ADD: return Val{V_F64, 0, __dadd_rn(a, c)};
        case EK_OP_SUB: return Val{V_F64, 0, __dsub_rn(a, c)};
        case EK_OP_MUL: return Val{V_F64, 0, __dmul_rn(a, c)};
        case EK_OP_DIV: return c == 0 ? Val{V_ERR, 0, 0.0} : Val{V_F64, 0, __ddiv_rn(a, c)};
        case EK_OP_MOD: return c == 0 ? Val{V_ERR, 0, 0.0} : Val{V_F64, 0, fmod(a, c)};
        default: return Val{V_ERR, 0, 0.0};
        }
    }
    int64_t a = l.i, c = r.i;
    switch (op) {
    case EK_OP_EQ: return mkb(a == c);
    case EK_OP_NEQ: return mkb(a != c);
    case EK_OP_LT: return mkb(a < c);
    case EK_OP_LTE: return mkb(a <= c);
    case EK_OP_GT: return mkb(a > c);
    case EK_OP_GTE: return mkb(a >= c);
    case EK_OP_ADD: return Val{V_I64, (int64_t)((uint64_t)a + (uint64_t)c), 0.0};
    case EK_OP_SUB: return Val{V_I64, (int64_t)((uint64_t)a - (uint64_t)c), 0.0};
    case EK_OP_MUL: return Val{V_I64, (int64_t)((uint64_t)a * (uint64_t)c), 0.0};
    case EK_OP_DIV: return c == 0 ? Val{V_ERR, 0, 0.0} : Val{V_I64, (a == INT64_MIN && c == -1) ? a : a / c, 0.0};
    case EK_OP_MOD: return c == 0 ? Val{V_ERR, 0, 0.0} : Val{V_I64, (c == -1) ? 0 : a % c, 0.0};
    default: return Val{V_ERR, 0, 0.0};
    }
}

// Register-resident evaluation stack: kEvalDepth slots addressed through switches, so the interpreter never
// touches per-lane scratch memory (a dynamically indexed array would live there). ek_create rejects deeper
// programs.
constexpr int kEvalDepth = 8;
// Evaluation stack of eight values kept in registers as a shift register: the top is always s0, push shifts down,
// pop shifts up. No access uses a runtime index, so nothing can be lowered to a private (scratch) array — a
// switch over the slots was turned into an indexed load from a stack-allocated struct (136 B of scratch traffic per
// HAVING / WHERE evaluation).
struct EvalStack {
    Val s0, s1, s2, s3, s4, s5, s6, s7;
    __device__ __forceinline__ void push(Val v) { s7 = s6; s6 = s5; s5 = s4; s4 = s3; s3 = s2; s2 = s1; s1 = s0; s0 = v; }
    __device__ __forceinline__ Val pop() {
        const Val v = s0;
        s0 = s1; s1 = s2; s2 = s3; s3 = s4; s4 = s5; s5 = s6; s6 = s7;
        return v;
    }
};

// Postfix program over one row; aggf(k) yields aggregate slot k (HAVING). Mirrors evalBinaryExpr's
// short-circuit: a decided lhs of AND/OR wins over an error on the rhs.
template <typename AGGF>
__device__ inline Val eval_prog(const ek_instr* prog, int n, const DPlan& p, const DBatch* b, int64_t row, AGGF aggf) {
    EvalStack st;
    int sp = 0;
    for (int k = 0; k < n; ++k) {
        const int op = prog[k].op;
        const int arg = prog[k].arg;
        if (op == EK_OP_COL) {
            st.push(b ? col_val(p, *b, arg, row) : Val{V_NULL, 0, 0.0});
            sp++;
        } else if (op == EK_OP_AGG) {
            st.push(aggf(arg));
            sp++;
        } else if (op == EK_OP_CONST_I64) {
            st.push(Val{V_I64, prog[k].i64, 0.0});
            sp++;
        } else if (op == EK_OP_CONST_F64) {
            st.push(Val{V_F64, 0, prog[k].f64});
            sp++;
        } else if (op == EK_OP_CONST_BOOL) {
            st.push(mkb(prog[k].i64 != 0));
            sp++;
        } else {
            const Val r = st.pop();
            const Val l = st.pop();
            sp -= 2;
            Val res;
            if (l.tag == V_ERR) res = l;
            else if (op == EK_OP_AND && l.tag == V_BOOL && !l.i) res = mkb(false);
            else if (op == EK_OP_OR && l.tag == V_BOOL && l.i) res = mkb(true);
            else if (r.tag == V_ERR) res = r;
            else res = simple_eval(l, r, op);
            st.push(res);
            sp++;
        }
    }
    return sp ? st.s0 : Val{V_NULL, 0, 0.0};
}
struct NoAggs {
    __device__ __forceinline__ Val operator()(int) const { return Val{V_NULL, 0, 0.0}; }
};

// WHERE decision: 1 keep, 0 drop, -1 error (filter_operator.go:63-77: nil -> drop, non-bool -> error)
__device__ inline int where_decide_slow(const DPlan& p, const DBatch& b, int64_t row) {
    Val v = eval_prog(p.where_prog, p.n_where, p, &b, row, NoAggs{});
    if (v.tag == V_BOOL) return v.i ? 1 : 0;
    if (v.tag == V_NULL) return 0;
    return -1;
}

__device__ __forceinline__ uint64_t d_mix64(uint64_t x) {  // == ek_mix64 (ekgpu.h)
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ int64_t floordiv64(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b) != 0 && ((a < 0) != (b < 0))) q--;
    return q;
}

}  // namespace ek
