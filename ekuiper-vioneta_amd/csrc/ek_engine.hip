// ek_engine.hip — host side of the MI355X window/aggregate engine: the C ABI of include/ekgpu.h.
//
// Replaces, for one rule, the reference's per-tuple operator chain
//   WatermarkOp (internal/topo/node/watermark_op.go:144-225)
//   WindowOperator event-time trigger (event_window_trigger.go:112-209, window_op.go:194-227,605-739)
//   FilterOp / AggregateOp / HavingOp / ProjectOp aggregate fields (internal/topo/operator/*.go)
// with columnar micro-batches processed by the gfx950 kernels of ek_kernels.h.
//
// Event-time semantics kept exactly (see DESIGN.md §2 for the derivation):
//   * late drop: event i accepted iff ts_i >= max(ts_<i) - lateTol            watermark_op.go:144-155
//   * watermark after a batch W = max ts - lateTol; windows with end <= W are emitted in order, none at EOF
//   * first window end E1 = getAlignedWindowEndTime(min accepted ts)         event_window_trigger.go:57-75
//   * tumbling window j: ts < E1 (j = 0) or [E_{j-1}, E_j); hopping j: [E_j - L, E_j)
//   * window_start quirks of scan()                                          window_op.go:697-707
// Aggregation is pane-based: each (pane, key) keeps a partial (count, sum, min, max, M2), windows
// merge their panes when they close.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "ek_kernels.h"
#include "ek_lib.h"
#include "ek_range.h"
#include "ek_global.h"
#include "ek_keymajor.h"
#include "ek_launch.h"
#include "ek_errmsg.h"

using namespace ek;

namespace {

constexpr int64_t kMinTs = INT64_MIN;
constexpr int64_t kYear1Ms = -62135596800000LL;   // Go's time.Time{} (0001-01-01T00:00:00Z) in Unix ms

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct WinInfo {
    int64_t j;           // window index (0 = first)
    int64_t start, end;
    int64_t out_base;    // first row of the window's result region
    int32_t slot;        // index into win_cnt / win_err device arrays
    bool direct;         // rows emitted by k_agg (whole tumbling pane inside one group)
};

int64_t floordiv_h(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b) != 0 && ((a < 0) != (b < 0))) q--;
    return q;
}

int64_t gcd64(int64_t a, int64_t b) {
    while (b) { int64_t t = a % b; a = b; b = t; }
    return a;
}

int64_t unit_ms(int32_t u) {
    switch (u) {
    case EK_UNIT_DD: return 86400000LL;
    case EK_UNIT_HH: return 3600000LL;
    case EK_UNIT_MI: return 60000LL;
    case EK_UNIT_SS: return 1000LL;
    case EK_UNIT_MS: return 1LL;
    }
    return 0;
}

// window_op.go:194-227 getAlignedWindowEndTime (time.Local = UTC + tz_offset_s, no DST)
int64_t aligned_end(int64_t ts, int32_t interval, int32_t unit, int32_t tz) {
    int64_t off = (int64_t)tz * 1000;
    int64_t local = ts + off;
    int64_t day0 = floordiv_h(local, 86400000LL) * 86400000LL;
    int64_t gap = interval;
    switch (unit) {
    case EK_UNIT_DD: return day0 + (int64_t)interval * 86400000LL - off;
    case EK_UNIT_HH: {
        int64_t hour = (local - day0) / 3600000LL;
        if (hour > interval) gap = (int64_t)interval * (hour / interval + 1);
        return day0 + gap * 3600000LL - off;
    }
    case EK_UNIT_MI: {
        int64_t h0 = floordiv_h(local, 3600000LL) * 3600000LL;
        int64_t minute = (local - h0) / 60000LL;
        if (minute > interval) gap = (int64_t)interval * (minute / interval + 1);
        return h0 + gap * 60000LL - off;
    }
    case EK_UNIT_SS: {
        int64_t m0 = floordiv_h(local, 60000LL) * 60000LL;
        int64_t sec = (local - m0) / 1000LL;
        if (sec > interval) gap = (int64_t)interval * (sec / interval + 1);
        return m0 + gap * 1000LL - off;
    }
    case EK_UNIT_MS: {
        int64_t s0 = floordiv_h(local, 1000LL) * 1000LL;
        int64_t milli = local - s0;
        if (milli > interval) gap = (int64_t)interval * (milli / interval + 1);
        return s0 + gap - off;
    }
    }
    return ts;
}

int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

int prog_depth_ok(const ek_instr* prog, int n) {
    int sp = 0;
    for (int k = 0; k < n; ++k) {
        int op = prog[k].op;
        if (op == EK_OP_COL || op == EK_OP_AGG || op == EK_OP_CONST_I64 || op == EK_OP_CONST_F64 || op == EK_OP_CONST_BOOL) sp++;
        else if (op >= EK_OP_EQ && op <= EK_OP_MOD) { if (sp < 2) return 0; sp--; }
        else return 0;
        if (sp > kEvalDepth) return 0;   // the device interpreter's register stack
    }
    return n == 0 || sp == 1;
}

// Whether a (depth-checked) condition can fail at run time — an error or a non-bool result (filter_operator.go:45-58,
// having_operator.go:45-55) — by the static types of its operands: numbers (columns, constants, aggregates) and bools
// (comparisons, AND / OR). Division / modulo by a possible zero, bool-number mixes, AND / OR over numbers, a non-bool
// root and order statistics (their "Input is outside of range") can; a plan whose conditions cannot fail records no
// error witnesses.
bool prog_can_fail(const ek_instr* prog, int n, const int32_t* agg_fn, const int32_t* col_type) {
    bool st[EK_MAX_PROG + 1];   // true: bool-typed
    int sp = 0;
    bool f = false;
    for (int k = 0; k < n; ++k) {
        const int op = prog[k].op;
        if (op == EK_OP_CONST_BOOL) { st[sp++] = true; continue; }
        if (op == EK_OP_COL) { st[sp++] = col_type[prog[k].arg] == EK_COL_BOOL; continue; }
        if (op == EK_OP_CONST_I64 || op == EK_OP_CONST_F64) { st[sp++] = false; continue; }
        if (op == EK_OP_AGG) {
            const int fn = agg_fn[prog[k].arg];
            f |= fn == EK_AGG_PERCENTILE_CONT || fn == EK_AGG_PERCENTILE_DISC;
            st[sp++] = false;
            continue;
        }
        const bool r = st[--sp], l = st[--sp];
        if (op == EK_OP_EQ || op == EK_OP_NEQ) f |= l != r;
        else if (op >= EK_OP_LT && op <= EK_OP_GTE) f |= l || r;
        else if (op == EK_OP_AND || op == EK_OP_OR) f |= !l || !r;
        else f |= l || r || op == EK_OP_DIV || op == EK_OP_MOD;
        st[sp++] = op <= EK_OP_OR;
    }
    return f || sp != 1 || !st[0];
}

}  // namespace

struct Engine {
    ek_plan plan{};
    int user_cols = 0;                  // columns of the caller's batches (plan.n_columns also counts the derived ones)
    DevBuf der_val[EK_MAX_DERIVED], der_valid[EK_MAX_DERIVED];
    DPlan dp{};
    DPlan* d_plan = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // per-phase timing: event pairs recorded around launches, summed when the push completes
    struct PhaseEv { hipEvent_t a, b; int phase; };
    std::vector<PhaseEv> phase_ev;
    size_t phase_used = 0;
    int phase_begin(int ph) {
        if (!phase_events) return -1;
        if (phase_used == phase_ev.size()) {
            PhaseEv e{nullptr, nullptr, 0};
            hipEventCreate(&e.a);
            hipEventCreate(&e.b);
            phase_ev.push_back(e);
        }
        phase_ev[phase_used].phase = ph;
        hipEventRecord(phase_ev[phase_used].a, stream);
        return (int)phase_used++;
    }
    void phase_end(int idx) { if (idx >= 0) hipEventRecord(phase_ev[idx].b, stream); }
    bool phase_events = true;   // ek_set_phase_timing (EKGPU_PHASE_EVENTS=0 at create: off)

    // ---- derived configuration
    int wtype = 0;
    int n_out = 0;                     // value arrays per result row: aggregates, or every column (filter rules)
    int64_t L = 0, H = 0, P = 0;       // ms
    int64_t ppw = 1, hpp = 1;          // panes per window, panes per hop
    int32_t raw_interval = 0;
    uint32_t K = 1;                    // keys
    int kbits = 0, NB = 1;
    int64_t Kpad = 1;
    int ring = 16;
    int max_panes_group = 8;
    int64_t group_events = 8 << 20;
    int chunk = 16384;
    LdsLayout lay{};
    int np_max = 8192;

    // ---- processing time (execProcessingWindow under the caller's clock, ek_advance_time)
    bool proc = false;                 // processing-time TUMBLING / HOPPING / SLIDING / SESSION
    bool proc_inc = false;             // processing-time incremental TUMBLING / HOPPING / SLIDING (proc_inc_triggers)
    bool proc_v2s = false;             // processing-time v2 SLIDINGWINDOW (SlidingWindowOp; proc_inc_triggers replays it)
    bool inc_where = false;            // WHERE above an incremental window: filters the groups' last rows (k_inc_where)
    int inc_hidden = -1;               // its hidden result slot: the group's last row (MAX of the position column)
    int n_res = 0;                     // value arrays per result row (n_out + the hidden slot)
    DPlan* d_plan_incw = nullptr;      // the plan with WHERE and HAVING, for k_inc_where (d_plan aggregates without them)
    DPlan dp_incw{};                   // its host copy (the window error texts re-evaluate its programs)
    bool proc_pushdown = false;        // WHERE / FILTER moved below the window (windowPlan.go:82-99): rows are pre-filtered
    bool pre_filter = false;           // a FilterOp in front of the window (pushed-down WHERE and / or the window FILTER)
    DPlan* d_plan_where = nullptr;     // the plan with WHERE, for the pre-filter (d_plan has n_where = 0 then)
    bool clock_started = false;        // the rule's start: the first ek_advance_time, or the first row
    int64_t clock_ms = 0;              // the clock (every timer due at or before it has fired)
    // session timers (window_op.go:363-373,448-461): ticker due ps_tick, timeout due ps_to_due; next row to deliver
    int64_t ps_tick = 0;
    bool ps_to_exists = false, ps_to_armed = false;
    int64_t ps_to_due = 0;
    int64_t ps_next_abs = 0;
    int64_t ps_last_nonmatch = INT64_MIN;   // SLIDING: ts of the latest delivered row not matching OVER (WHEN)

    // ---- stream state
    bool has_M = false;
    int64_t M = kMinTs;                // max ts over all arrivals
    bool has_W = false;
    int64_t W = kMinTs;                // last watermark
    bool e1_known = false;
    int64_t E1 = 0, first_ts = 0;
    int64_t next_win = 0;              // next window index to emit
    int64_t arrivals = 0;
    bool time_pending = false;         // the last push's end event is recorded but not yet read (fold_time)
    bool async_push = false;           // ek_set_async: pushes return with their work queued
    hipEvent_t ev_h2d = nullptr;       // asynchronous pushes: the host batch's copies are done
    bool h2d_pending = false;
    std::vector<int64_t> slot_pane;    // pane id held by each ring slot (INT64_MIN = free)
    PaneGrid grid{};
    ek_stats stats{};

    // ---- device memory
    DevBuf state_buf, pane_err, pane_mcnt, pane_mhash;
    // error witnesses (ek_window_error): allocated only for plans whose WHERE / HAVING / order statistics can fail
    bool where_can_fail = false, having_can_fail = false, agg_can_fail = false;
    DevBuf pane_wit;                   // [ring] WitRec: each pane slot's first failed WHERE row
    DevBuf r_wwit, r_aslot;
    DevBuf vp_wit;                     // range mode: the launch's window witnesses (its virtual panes)            // [2 per window] WitRec (WHERE, HAVING), [window] failed order statistic
    int64_t wit_seq = 0;               // launch counter: the release-order tie-break of pane witnesses
    std::vector<std::string> poll_msgs;   // the last poll's window error texts
    DState dstate{};
    DevBuf bstats, bstats_part;        // BatchStats, per-block partials of k_stats
    BatchStats* h_stats = nullptr;     // pinned
    int64_t* h_small = nullptr;        // pinned scratch (bounds)
    size_t h_small_cap = 0;
    DevBuf cmax, acc, bounds_val, bounds_idx, chist, totals, pstart, pcursor, direct_d;
    DevBuf st_klo, st_val[kMaxVC], st_valid[kMaxVC];
    int64_t st_cap = 0;
    DevBuf in_cols[EK_MAX_COLUMNS], in_valid[EK_MAX_COLUMNS];   // H2D staging for host batches
    // accepted events that arrived before the first watermark release (host copy, tiny)
    DevBuf pend_cols[EK_MAX_COLUMNS], pend_valid[EK_MAX_COLUMNS], pend_arr_d;
    std::vector<char> pend_host[EK_MAX_COLUMNS];
    std::vector<uint8_t> pend_vhost[EK_MAX_COLUMNS];
    std::vector<int64_t> pend_arr;
    int64_t pend_n = 0, pend_min = INT64_MAX, pend_max = INT64_MIN;
    bool pend_has_valid[EK_MAX_COLUMNS] = {};
    DevBuf wdesc;                      // WinDesc array
    WinDesc* h_wdesc = nullptr;        // pinned, bump-allocated per push (reset after the stats sync)
    size_t h_wdesc_cap = 0, h_wdesc_used = 0;

    // ---- results (device, accumulated until poll)
    DevBuf r_key, r_val[EK_MAX_AGGS], r_tag[EK_MAX_AGGS], r_wcnt, r_werr, r_wmc, r_wmh;
    int64_t r_rows_cap = 0, r_rows_used = 0;
    int64_t r_win_cap = 0;
    std::vector<WinInfo> wins;         // windows since last poll
    // host copies handed out by poll (EK_MEM_HOST)
    std::vector<int64_t> h_ws, h_we, h_off, h_cnt, h_mc;
    std::vector<uint64_t> h_mh;
    std::vector<int32_t> h_st;
    std::vector<uint32_t> h_key;
    std::vector<int64_t> h_val[EK_MAX_AGGS];
    std::vector<uint8_t> h_tag[EK_MAX_AGGS];
    std::vector<int64_t> d_off_host;   // offsets for device results

    int fail(int code, const char* fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }

    int ensure(DevBuf& b, size_t bytes) {
        if (b.bytes >= bytes && b.p) return 0;
        if (b.p) { hipStreamSynchronize(stream); hipFree(b.p); b.p = nullptr; b.bytes = 0; }
        size_t nb = std::max(bytes, (size_t)256);
        if (hipMalloc(&b.p, nb) != hipSuccess) return fail(EK_ERR_NOMEM, "hipMalloc(%zu) failed", nb);
        b.bytes = nb;
        return 0;
    }
    void release(DevBuf& b) {
        if (b.p) hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
    }

    // ------------------------------------------------------------------ create
    int init(const ek_plan* p, int dev) {
        plan = *p;
        device = dev;
        if (plan.abi_version != EKGPU_ABI_VERSION) return fail(EK_ERR_INVALID, "abi version %d != %d", plan.abi_version, EKGPU_ABI_VERSION);
        if (plan.n_columns <= 0 || plan.n_columns > EK_MAX_COLUMNS) return fail(EK_ERR_INVALID, "bad n_columns");
        if (plan.n_aggs < 0 || plan.n_aggs > EK_MAX_AGGS) return fail(EK_ERR_INVALID, "bad n_aggs");
        if (plan.n_where < 0 || plan.n_where > EK_MAX_PROG || plan.n_having < 0 || plan.n_having > EK_MAX_PROG ||
            plan.n_trigger < 0 || plan.n_trigger > EK_MAX_PROG || plan.n_begin < 0 || plan.n_begin > EK_MAX_PROG ||
            plan.n_emit < 0 || plan.n_emit > EK_MAX_PROG)
            return fail(EK_ERR_INVALID, "bad program length");
        if (!prog_depth_ok(plan.where_prog, plan.n_where) || !prog_depth_ok(plan.having_prog, plan.n_having) ||
            !prog_depth_ok(plan.trigger_prog, plan.n_trigger) || !prog_depth_ok(plan.begin_prog, plan.n_begin) ||
            !prog_depth_ok(plan.emit_prog, plan.n_emit))
            return fail(EK_ERR_INVALID, "malformed expression program");
        for (int c = 0; c < plan.n_columns; ++c)
            if (plan.column_type[c] != EK_COL_I64 && plan.column_type[c] != EK_COL_F64 && plan.column_type[c] != EK_COL_U32 &&
                plan.column_type[c] != EK_COL_BOOL)
                return fail(EK_ERR_INVALID, "bad column type %d", c);
        auto col_ok = [&](int c) { return c >= 0 && c < plan.n_columns; };
        for (int k = 0; k < plan.n_where; ++k)
            if (plan.where_prog[k].op == EK_OP_COL && !col_ok(plan.where_prog[k].arg)) return fail(EK_ERR_INVALID, "WHERE column out of range");
            else if (plan.where_prog[k].op == EK_OP_AGG) return fail(EK_ERR_INVALID, "aggregate in WHERE");
        for (const ek_instr* pr : {plan.trigger_prog, plan.begin_prog, plan.emit_prog})
            for (int k = 0; k < EK_MAX_PROG; ++k) {
                const int n = pr == plan.trigger_prog ? plan.n_trigger : pr == plan.begin_prog ? plan.n_begin : plan.n_emit;
                if (k >= n) break;
                if (pr[k].op == EK_OP_COL && !col_ok(pr[k].arg)) return fail(EK_ERR_INVALID, "condition column out of range");
                if (pr[k].op == EK_OP_AGG) return fail(EK_ERR_INVALID, "aggregate in a window condition");
            }
        // the window's FILTER (WHERE ...) clause (ABI v8): a row condition over the stream's columns
        if (plan.n_filter < 0 || plan.n_filter > EK_MAX_PROG || !prog_depth_ok(plan.filter_prog, plan.n_filter))
            return fail(EK_ERR_INVALID, "malformed window FILTER program");
        for (int k = 0; k < plan.n_filter; ++k) {
            if (plan.filter_prog[k].op == EK_OP_COL && !col_ok(plan.filter_prog[k].arg)) return fail(EK_ERR_INVALID, "FILTER column out of range");
            if (plan.filter_prog[k].op == EK_OP_AGG) return fail(EK_ERR_INVALID, "aggregate in a window FILTER");
        }
        if (plan.n_filter > 0 && plan.window_type == EK_WINDOW_NONE) return fail(EK_ERR_INVALID, "FILTER belongs to a window");
        // derived columns (expression arguments of aggregates): validated here, then appended to the engine's copy of
        // the plan as ordinary columns [user_cols, user_cols + n_derived) computed per batch by k_derive
        user_cols = plan.n_columns;
        if (plan.n_derived < 0 || plan.n_derived > EK_MAX_DERIVED || plan.n_columns + plan.n_derived > EK_MAX_COLUMNS)
            return fail(EK_ERR_INVALID, "bad n_derived");
        if (plan.n_derived > 0 && plan.window_type == EK_WINDOW_NONE) return fail(EK_ERR_INVALID, "derived columns need aggregates");
        for (int d = 0; d < plan.n_derived; ++d) {
            const ek_instr* pr = plan.derived_prog[d];
            const int np = plan.n_derived_prog[d];
            if (np <= 0 || np > EK_MAX_PROG || !prog_depth_ok(pr, np)) return fail(EK_ERR_INVALID, "malformed derived column program %d", d);
            if (plan.derived_type[d] != EK_COL_I64 && plan.derived_type[d] != EK_COL_F64) return fail(EK_ERR_INVALID, "bad derived column type");
            bool nullable = false;
            for (int k = 0; k < np; ++k) {
                const int op = pr[k].op;
                if (op == EK_OP_COL) {
                    if (!col_ok(pr[k].arg)) return fail(EK_ERR_INVALID, "derived column reference out of range");
                    if (plan.column_type[pr[k].arg] == EK_COL_BOOL)
                        return fail(EK_ERR_UNSUPPORTED, "derived columns are arithmetic over numeric columns");
                    nullable |= (plan.nullable_mask >> pr[k].arg) & 1u;
                } else if (op == EK_OP_AGG || op == EK_OP_CONST_BOOL || (op >= EK_OP_EQ && op <= EK_OP_OR)) {
                    return fail(EK_ERR_UNSUPPORTED, "derived columns are arithmetic over columns and constants");
                } else if (op == EK_OP_DIV || op == EK_OP_MOD) {
                    const ek_instr& r = pr[k - 1];   // postfix: the divisor is the instruction before the operator
                    const bool cz = (r.op == EK_OP_CONST_I64 && r.i64 != 0) || (r.op == EK_OP_CONST_F64 && r.f64 != 0.0);
                    if (!cz) return fail(EK_ERR_UNSUPPORTED, "derived columns divide only by a non-zero constant "
                                                             "(a zero divisor is a per-row evaluation error)");
                }
            }
            const int c = plan.n_columns + d;
            plan.column_type[c] = plan.derived_type[d];
            if (nullable) plan.nullable_mask |= 1u << c;
        }
        plan.n_columns += plan.n_derived;
        if (plan.window_version == 2 && plan.window_type == EK_WINDOW_SLIDING) {
            // WindowV2Operator sliding windows (window_v2_op.go:39-58): SlidingWindowOp (processing time, under the caller's
            // clock, delay included) and EventSlidingWindowOp (its delayed form re-emits every due delay at each later
            // WatermarkTuple until a newer one is pending, window_v2_event_op.go:56-76: v2_delay_triggers)
        } else if (plan.window_version != 0 && plan.window_version != 1 && plan.window_type != EK_WINDOW_STATE) {
            return fail(EK_ERR_UNSUPPORTED, "window version %d (WindowV2Operator) is built for STATEWINDOW and SLIDINGWINDOW only",
                        plan.window_version);
        }
        for (int k = 0; k < plan.n_having; ++k) {
            if (plan.having_prog[k].op == EK_OP_COL) return fail(EK_ERR_UNSUPPORTED, "non-aggregate column in HAVING");
            if (plan.having_prog[k].op == EK_OP_AGG && (plan.having_prog[k].arg < 0 || plan.having_prog[k].arg >= plan.n_aggs))
                return fail(EK_ERR_INVALID, "HAVING aggregate slot out of range");
        }
        wtype = plan.window_type;
        bool sort_aggs = false, has_first = false;
        for (int k = 0; k < plan.n_aggs; ++k) {
            sort_aggs |= plan.aggs[k].fn == EK_AGG_MEDIAN || plan.aggs[k].fn == EK_AGG_PERCENTILE_CONT ||
                         plan.aggs[k].fn == EK_AGG_PERCENTILE_DISC;
            has_first |= plan.aggs[k].fn == EK_AGG_FIRST;
        }
        n_out = plan.n_aggs;
        n_res = n_out;
        if (wtype == EK_WINDOW_NONE) {
            // a rule without window and aggregates: FilterOp (WHERE) + SELECT * per event (C1 shape)
            if (plan.n_aggs != 0 || plan.key_column >= 0 || plan.n_having)
                return fail(EK_ERR_UNSUPPORTED, "aggregates need a window in GROUP BY");
            if (plan.is_event_time) return fail(EK_ERR_UNSUPPORTED, "event-time ordering of a window-less rule is not on this path");
            n_out = n_res = plan.n_columns;
            if (hipSetDevice(device) != hipSuccess) return fail(EK_ERR_DEVICE, "hipSetDevice(%d) failed", device);
            if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return fail(EK_ERR_DEVICE, "stream create failed");
            own_stream = true;
            hipEventCreate(&ev0);
            hipEventCreate(&ev1);
            dp = DPlan{};
            dp.n_columns = plan.n_columns;
            for (int c = 0; c < plan.n_columns; ++c) dp.col_type[c] = plan.column_type[c];
            dp.ts_col = plan.ts_column;
            dp.key_col = -1;
            dp.n_where = plan.n_where;
            memcpy(dp.where_prog, plan.where_prog, sizeof plan.where_prog);
            if (hipMalloc((void**)&d_plan, sizeof(DPlan)) != hipSuccess) return fail(EK_ERR_NOMEM, "plan alloc");
            if (hipMemcpy(d_plan, &dp, sizeof(DPlan), hipMemcpyHostToDevice) != hipSuccess) return fail(EK_ERR_DEVICE, "plan copy");
            if (hipHostMalloc((void**)&h_stats, sizeof(BatchStats)) != hipSuccess) return fail(EK_ERR_NOMEM, "pinned alloc");
            reset_state();
            return 0;
        }
        if (wtype == EK_WINDOW_STATE) {
            // WindowV2Operator / StateWindowOp (window_v2_op.go:39-58,94-148): rows in arrival order (processing
            // time) or in WatermarkOp release order (event time); no time grid. WHERE is pushed below a
            // processing-time window (windowPlan.go:82-99): with the FILTER it is the FilterOp in front of the window
            // (planner.go:388-392), so only the rows it keeps reach the begin / emit conditions (proc_prefilter)
            proc_pushdown = !plan.is_event_time && plan.n_where > 0;
        } else if (plan.is_event_time) {
            // NewEventTimeTrigger (event_window_trigger.go:35-53): COUNTWINDOW is rejected in event time, except on the
            // incremental path (CountWindowIncAggEventOp, window_inc_agg_event_op.go:340-439), decided below
            const bool inc_count = plan.incremental && wtype == EK_WINDOW_COUNT && plan.interval <= 0;
            if ((wtype <= EK_WINDOW_NONE || wtype > EK_WINDOW_SESSION) && !inc_count)
                return fail(EK_ERR_UNSUPPORTED, "unsupported window type %d", wtype);
        } else if (wtype != EK_WINDOW_COUNT) {
            // execProcessingWindow (window_op.go:235-470) under the caller's clock (ek_advance_time): tickers aligned
            // to the rule's start, rows delivered at their arrival timestamps
            if (wtype != EK_WINDOW_TUMBLING && wtype != EK_WINDOW_HOPPING && wtype != EK_WINDOW_SLIDING && wtype != EK_WINDOW_SESSION)
                return fail(EK_ERR_UNSUPPORTED, "unsupported processing-time window type %d", wtype);
            if (plan.window_version == 2 && wtype != EK_WINDOW_SLIDING)
                return fail(EK_ERR_UNSUPPORTED, "v2 processing-time windows other than SLIDINGWINDOW are not built");
            if (!col_ok(plan.ts_column) || plan.column_type[plan.ts_column] != EK_COL_I64 || (plan.nullable_mask & (1u << plan.ts_column)))
                return fail(EK_ERR_INVALID, "processing-time windows need the rows' arrival timestamps (a non-nullable i64 column)");
            proc = true;
            // windowPlan.PushDownPredicate (windowPlan.go:82-99): WHERE below a processing-time TUMBLING / HOPPING / SESSION
            // rows a FilterOp drops before they reach the window, compacted at delivery (proc_prefilter): WHERE AND the
            // window FILTER pushed below TUMBLING / HOPPING / SESSION (windowPlan.PushDownPredicate, windowPlan.go:82-99),
            // the FILTER op alone before SLIDING (planner.go:388-392; WHERE stays above the window)
            proc_pushdown = (plan.n_where > 0 && wtype != EK_WINDOW_SLIDING) || plan.n_filter > 0;
            if (wtype == EK_WINDOW_SLIDING && plan.delay > 0) {
                slide_delay = (int64_t)plan.delay * unit_ms(plan.time_unit);
                send_twice = plan.sliding_send_twice != 0;
            }
        }
        // incremental-aggregation window (planOptimizeStrategy.enableIncrementalWindow): the planner rewrites the
        // rule only when every aggregate is incremental and the window is COUNT (no interval) / SLIDING / HOPPING /
        // TUMBLING (rewriteIfIncAggStmt + supportedWindowType, planner.go:910-1017); otherwise the regular chain runs
        {
            bool fns = plan.n_aggs > 0;
            for (int k = 0; k < plan.n_aggs; ++k) fns &= plan.aggs[k].fn >= EK_AGG_COUNT_STAR && plan.aggs[k].fn <= EK_AGG_MAX;
            const bool win = (wtype == EK_WINDOW_COUNT && plan.interval <= 0) || wtype == EK_WINDOW_SLIDING ||
                             wtype == EK_WINDOW_HOPPING || wtype == EK_WINDOW_TUMBLING;
            inc = plan.incremental != 0 && fns && win;
        }
        if (proc && plan.window_version == 2 && !inc) {
            // WindowV2Operator SlidingWindowOp (window_v2_op.go:160-215): replayed on the host like the incremental ops;
            // the window FILTER op in front of it, WHERE above it
            proc_v2s = true;
            proc_pushdown = plan.n_filter > 0;
            slide_delay = 0;
            send_twice = false;
        }
        if (inc && proc) {
            // TumblingWindowIncAggOp / HoppingWindowIncAggOp / SlidingWindowIncAggOp (window_inc_agg_op.go:316-790) under
            // the caller's clock; WHERE stays above the window (IncWindowPlan.PushDownPredicate, incAggPlan.go:76-78): only
            // the window FILTER op is in front of it (planner.go:360-365)
            proc_inc = true;
            proc_pushdown = plan.n_filter > 0;
            slide_delay = 0;
            send_twice = false;
        }
        if (inc) {
            if (wtype == EK_WINDOW_SLIDING && plan.delay != 0 && !proc)
                return fail(EK_ERR_UNSUPPORTED, "delayed incremental sliding windows (appendDelayIncAggWindowInEvent, "
                                                "window_inc_agg_event_op.go:275-296: a window per row) are not built");
            if (plan.n_where > 0) {
                // FilterPlan above IncWindowPlan (planner.go:702-708): WHERE filters the emitted last rows (k_inc_where)
                if (plan.n_aggs >= EK_MAX_AGGS) return fail(EK_ERR_UNSUPPORTED, "WHERE over an incremental window needs a free aggregate slot");
                inc_where = true;
            }
            if (has_first)
                return fail(EK_ERR_UNSUPPORTED, "incremental windows emit the group's LAST row (window_inc_agg_op.go:443-457): "
                                                "first-row select fields are not on that path");
            for (int k = 0; k < plan.n_aggs; ++k)
                if (plan.aggs[k].fn != EK_AGG_COUNT_STAR && ((plan.nullable_mask >> plan.aggs[k].column) & 1u))
                    return fail(EK_ERR_UNSUPPORTED, "incremental aggregates over a nullable column (nil at a group's last row) are not built");
        }
        // hopping with lateTolerance > 0: the empty-window discard (window_op.go:605-655) can drop inputs released by
        // earlier pushes, so the events are kept (range mode) instead of being folded into pane partials
        range_mode = wtype == EK_WINDOW_SLIDING || wtype == EK_WINDOW_SESSION || wtype == EK_WINDOW_COUNT ||
                     (wtype == EK_WINDOW_HOPPING && plan.is_event_time && plan.late_tolerance_ms > 0) ||
                     wtype == EK_WINDOW_STATE || sort_aggs || has_first ||
                     inc || env_int("EKGPU_FORCE_RANGE", 0) != 0;
        if (plan.sliding_send_twice && wtype == EK_WINDOW_SLIDING && plan.delay > 0 && plan.is_event_time &&
            plan.window_version != 2 && !inc) {
            // event_window_trigger.go:129-135,156-161: the first part at the trigger, the last part at its delay
            // (et2_triggers); WindowV2's EventSlidingWindowOp and the incremental op have no send-twice
            send_twice = true;
        }
        if (plan.is_event_time && wtype == EK_WINDOW_COUNT && !inc)
            return fail(EK_ERR_UNSUPPORTED, "COUNTWINDOW in event time needs the incremental path (every aggregate incremental)");
        need_rel = (wtype == EK_WINDOW_SLIDING && !proc) || (inc && wtype == EK_WINDOW_COUNT) ||
                   (wtype == EK_WINDOW_SESSION && plan.late_tolerance_ms > 0 && !proc);
        if (proc && plan.late_tolerance_ms != 0) return fail(EK_ERR_INVALID, "lateTolerance applies to event time only");
        if (plan.is_event_time) {
            if (!col_ok(plan.ts_column) || plan.column_type[plan.ts_column] != EK_COL_I64)
                return fail(EK_ERR_INVALID, "event time needs an i64 timestamp column");
            if (plan.nullable_mask & (1u << plan.ts_column)) return fail(EK_ERR_INVALID, "nullable timestamp column");
        }
        if (plan.key_column >= 0) {
            if (!col_ok(plan.key_column) || plan.column_type[plan.key_column] != EK_COL_U32)
                return fail(EK_ERR_INVALID, "GROUP BY key must be a u32 dictionary column");
            if (plan.num_keys == 0) return fail(EK_ERR_INVALID, "num_keys must be > 0");
            if (plan.nullable_mask & (1u << plan.key_column)) return fail(EK_ERR_UNSUPPORTED, "nullable GROUP BY key");
        }
        if (plan.length <= 0 && wtype != EK_WINDOW_STATE) return fail(EK_ERR_INVALID, "Window size should not be less than zero.");
        if (wtype == EK_WINDOW_STATE) {
            L = H = P = 1;   // no time grid
        } else if (wtype == EK_WINDOW_COUNT) {
            // window_op.go:100-103: CountInterval defaults to CountLength
            if (plan.interval < 0) return fail(EK_ERR_INVALID, "count window interval must be >= 0");
            L = plan.length;
            H = plan.interval > 0 ? plan.interval : plan.length;
            P = 1;
        } else {
            int64_t u = unit_ms(plan.time_unit);
            if (u == 0) return fail(EK_ERR_INVALID, "bad time unit");
            L = (int64_t)plan.length * u;
            if (plan.delay != 0 && wtype != EK_WINDOW_SLIDING) return fail(EK_ERR_UNSUPPORTED, "window delay is only defined for sliding windows");
            if (plan.delay < 0) return fail(EK_ERR_INVALID, "negative window delay");
            if (wtype == EK_WINDOW_TUMBLING || wtype == EK_WINDOW_SLIDING) {
                H = L; P = L; raw_interval = plan.length;
            } else if (wtype == EK_WINDOW_SESSION) {
                // SESSIONWINDOW(unit, length, timeout): raw interval of the tick grid = length (planner.go:394-400)
                if (plan.interval <= 0) return fail(EK_ERR_INVALID, "session timeout must be > 0");
                H = (int64_t)plan.interval * u; P = L; raw_interval = plan.length;
            } else {
                if (plan.interval <= 0) return fail(EK_ERR_INVALID, "hopping interval must be > 0");
                H = (int64_t)plan.interval * u;
                if (H > L && !range_mode) return fail(EK_ERR_UNSUPPORTED, "hopping interval larger than the window length");
                P = gcd64(L, H);
                raw_interval = plan.interval;
            }
        }
        ppw = L / P;
        hpp = H / P;

        // ---- device plan + aggregate field needs
        dp = DPlan{};
        dp.n_columns = plan.n_columns;
        for (int c = 0; c < plan.n_columns; ++c) dp.col_type[c] = plan.column_type[c];
        dp.n_user_cols = user_cols;
        for (int d = 0; d < plan.n_derived; ++d) {
            dp.n_derived_prog[d] = plan.n_derived_prog[d];
            memcpy(dp.derived_prog[d], plan.derived_prog[d], sizeof plan.derived_prog[d]);
        }
        dp.ts_col = plan.ts_column;
        dp.key_col = plan.key_column;
        dp.num_keys = plan.key_column >= 0 ? plan.num_keys : 1u;
        // un-grouped pane-mode rule: spread the rows over kPseudoKeys partial slots (row index) so a pane is aggregated
        // by many workgroups; k_finalize_merge folds the slots of a window into its one group
        if (plan.key_column < 0 && !range_mode && env_int("EKGPU_PSEUDO_KEYS", 1)) {
            dp.pseudo_keys = 1;
            dp.num_keys = kPseudoKeys;
        }
        dp.n_where = plan.n_where;
        dp.n_having = plan.n_having;
        dp.n_trigger = plan.n_trigger;
        memcpy(dp.where_prog, plan.where_prog, sizeof plan.where_prog);
        memcpy(dp.having_prog, plan.having_prog, sizeof plan.having_prog);
        memcpy(dp.trigger_prog, plan.trigger_prog, sizeof plan.trigger_prog);
        if (wtype == EK_WINDOW_STATE) {
            dp.n_begin = plan.n_begin;
            dp.n_emit = plan.n_emit;
            memcpy(dp.begin_prog, plan.begin_prog, sizeof plan.begin_prog);
            memcpy(dp.emit_prog, plan.emit_prog, sizeof plan.emit_prog);
        }
        dp.n_aggs = plan.n_aggs;
        dp.inc = inc ? 1 : 0;
        dp.having_star = plan.n_having > 0 ? 1 : 0;
        for (int i = 0; i < plan.n_having; ++i)
            if (plan.having_prog[i].op == EK_OP_AGG &&
                (plan.having_prog[i].arg < 0 || plan.having_prog[i].arg >= plan.n_aggs ||
                 plan.aggs[plan.having_prog[i].arg].fn != EK_AGG_COUNT_STAR))
                dp.having_star = 0;
        for (int k = 0; k < plan.n_aggs; ++k) {
            const ek_agg_spec& a = plan.aggs[k];
            dp.agg_fn[k] = a.fn;
            dp.agg_p[k] = a.param;
            dp.agg_vc[k] = -1;
            dp.agg_sidx[k] = -1;
            if (a.fn < EK_AGG_COUNT_STAR || a.fn > EK_AGG_FIRST) return fail(EK_ERR_INVALID, "bad aggregate %d", a.fn);
            if (a.fn == EK_AGG_COUNT_STAR) continue;
            if (a.fn == EK_AGG_FIRST) {
                // the group's first row = the minimum of the hidden position column (value = event-buffer index,
                // buffer_view) over its rows; k_first_fetch reads the source column there
                if (!col_ok(a.column)) return fail(EK_ERR_INVALID, "first-row field column out of range");
                if (plan.column_type[a.column] == EK_COL_BOOL) return fail(EK_ERR_UNSUPPORTED, "a BOOLEAN column is a count() argument only");
                if (rowpos_col < 0) {
                    if (plan.n_columns >= EK_MAX_COLUMNS) return fail(EK_ERR_UNSUPPORTED, "too many columns for a first-row field");
                    rowpos_col = plan.n_columns;
                    dp.col_type[rowpos_col] = EK_COL_I64;
                }
                int v = -1;
                for (int x = 0; x < dp.n_vc; ++x) if (dp.vc_col[x] == rowpos_col) v = x;
                if (v < 0) {
                    if (dp.n_vc >= kMaxVC) return fail(EK_ERR_UNSUPPORTED, "too many aggregated columns");
                    v = dp.n_vc++;
                    dp.vc_col[v] = rowpos_col;
                    dp.vc_is_float[v] = 0;
                    dp.vc_flags[v] = 0;
                }
                dp.agg_vc[k] = v;
                dp.vc_flags[v] |= NEED_MIN;
                dp.first_col[k] = a.column;
                dp.n_first++;
                continue;
            }
            if (!col_ok(a.column)) return fail(EK_ERR_INVALID, "aggregate column out of range");
            if (plan.column_type[a.column] == EK_COL_BOOL && a.fn != EK_AGG_COUNT)
                return fail(EK_ERR_UNSUPPORTED, "a BOOLEAN column is a count() argument only");
            int v = -1;
            for (int x = 0; x < dp.n_vc; ++x) if (dp.vc_col[x] == a.column) v = x;
            if (v < 0) {
                if (dp.n_vc >= kMaxVC) return fail(EK_ERR_UNSUPPORTED, "too many aggregated columns");
                v = dp.n_vc++;
                dp.vc_col[v] = a.column;
                dp.vc_is_float[v] = plan.column_type[a.column] == EK_COL_F64;
                dp.vc_flags[v] = 0;
            }
            dp.agg_vc[k] = v;
            const bool nullable = (plan.nullable_mask >> a.column) & 1u;
            const bool fl = dp.vc_is_float[v];
            int f = 0;
            switch (a.fn) {
            case EK_AGG_COUNT: f = NEED_CNT; break;
            // inc_sum / inc_avg accumulate float64 even over a BIGINT column (funcs_inc_agg.go:56-75,102-117)
            case EK_AGG_SUM: f = NEED_SUM | (inc && !fl ? NEED_FSUM : 0); break;
            case EK_AGG_AVG: f = NEED_SUM | NEED_CNT | (inc && !fl ? NEED_FSUM : 0); break;
            case EK_AGG_MIN: f = NEED_MIN; break;
            case EK_AGG_MAX: f = NEED_MAX; break;
            case EK_AGG_MEDIAN: case EK_AGG_PERCENTILE_CONT: case EK_AGG_PERCENTILE_DISC: {
                // order statistics over the group's values (range mode, k_agg sort pass)
                if (a.fn == EK_AGG_MEDIAN && nullable) {
                    // funcs_agg.go:29-55: a group whose first value is nil is a type error, an f64 column ignores the
                    // other nils. Built for f64 columns without HAVING (the check runs on the emitted rows); a BIGINT
                    // column fails on any nil with a text naming the whole group
                    if (!fl || plan.n_having > 0)
                        return fail(EK_ERR_UNSUPPORTED, "median over a nullable %s column (nil first element is a type error)",
                                    fl ? "float column with HAVING" : "bigint");
                    med_nullable.push_back(k);
                }
                if (dp.n_sagg >= kMaxSortAggs) return fail(EK_ERR_UNSUPPORTED, "too many median/percentile calls");
                int sc = -1;
                for (int x = 0; x < dp.n_scol; ++x) if (dp.scol_vc[x] == v) sc = x;
                if (sc < 0) {
                    if (dp.n_scol >= kMaxScol) return fail(EK_ERR_UNSUPPORTED, "median/percentile over more than %d columns", kMaxScol);
                    sc = dp.n_scol++;
                    dp.scol_vc[sc] = v;
                }
                dp.agg_sidx[k] = dp.n_sagg;
                dp.sagg_scol[dp.n_sagg] = sc;
                dp.sagg_agg[dp.n_sagg] = k;
                dp.n_sagg++;
                f = NEED_SORT | NEED_CNT;
                break;
            }
            default: f = NEED_M2 | NEED_CNT | (fl ? NEED_SUM : NEED_FSUM); break;   // var family
            }
            if (fl && (f & NEED_SUM) == 0 && (f & NEED_M2)) f |= NEED_SUM;
            if (!nullable) f &= ~NEED_CNT;   // vcnt == count(*) when the column has no NULLs
            dp.vc_flags[v] |= f;
        }
        if (inc_where) {
            // the group's last row: MAX of the hidden position column (event-buffer index) in slot plan.n_aggs
            if (rowpos_col < 0) {
                if (plan.n_columns >= EK_MAX_COLUMNS) return fail(EK_ERR_UNSUPPORTED, "too many columns for WHERE over an incremental window");
                rowpos_col = plan.n_columns;
                dp.col_type[rowpos_col] = EK_COL_I64;
            }
            int v = -1;
            for (int x = 0; x < dp.n_vc; ++x) if (dp.vc_col[x] == rowpos_col) v = x;
            if (v < 0) {
                if (dp.n_vc >= kMaxVC) return fail(EK_ERR_UNSUPPORTED, "too many aggregated columns");
                v = dp.n_vc++;
                dp.vc_col[v] = rowpos_col;
                dp.vc_is_float[v] = 0;
                dp.vc_flags[v] = 0;
            }
            inc_hidden = plan.n_aggs;
            dp.agg_fn[inc_hidden] = EK_AGG_MAX;
            dp.agg_vc[inc_hidden] = v;
            dp.agg_sidx[inc_hidden] = -1;
            dp.vc_flags[v] |= NEED_MAX;
            dp.n_aggs = plan.n_aggs + 1;
        }
        for (int k = 0; k < EK_MAX_AGGS; ++k) dp.med_first[k] = -1;
        for (int k : med_nullable) {
            // the group's first row over the median's column: a hidden EK_AGG_FIRST slot (k_first_fetch checks it)
            if (dp.n_aggs >= EK_MAX_AGGS) return fail(EK_ERR_UNSUPPORTED, "median over a nullable column needs a free aggregate slot");
            if (rowpos_col < 0) {
                if (plan.n_columns >= EK_MAX_COLUMNS) return fail(EK_ERR_UNSUPPORTED, "too many columns for a first-row field");
                rowpos_col = plan.n_columns;
                dp.col_type[rowpos_col] = EK_COL_I64;
            }
            int v = -1;
            for (int x = 0; x < dp.n_vc; ++x) if (dp.vc_col[x] == rowpos_col) v = x;
            if (v < 0) {
                if (dp.n_vc >= kMaxVC) return fail(EK_ERR_UNSUPPORTED, "too many aggregated columns");
                v = dp.n_vc++;
                dp.vc_col[v] = rowpos_col;
                dp.vc_is_float[v] = 0;
                dp.vc_flags[v] = 0;
            }
            const int h = dp.n_aggs++;
            dp.agg_fn[h] = EK_AGG_FIRST;
            dp.agg_vc[h] = v;
            dp.agg_sidx[h] = -1;
            dp.agg_p[h] = 0;
            dp.vc_flags[v] |= NEED_MIN;
            dp.first_col[h] = plan.aggs[k].column;
            dp.n_first++;
            dp.med_first[k] = h;
        }
        n_res = dp.n_aggs > n_out ? dp.n_aggs : n_out;
        for (int v = 0; v < dp.n_vc; ++v) {
            // float sums feed the M2 merge and avg; int sums keep a float shadow only for var
            if (!dp.vc_is_float[v] && (dp.vc_flags[v] & NEED_M2)) dp.vc_flags[v] |= NEED_FSUM;
        }

        // ---- key bucketing: keys per bucket (1 << kbits) sized so the LDS partial fits
        K = dp.num_keys;
        int bytes_per_key = 4;
        for (int v = 0; v < dp.n_vc; ++v) {
            int f = dp.vc_flags[v];
            bytes_per_key += (f & NEED_CNT ? 4 : 0) + (f & NEED_SUM ? 8 : 0) + (f & NEED_MIN ? 8 : 0) + (f & NEED_MAX ? 8 : 0) +
                             (f & NEED_M2 ? 8 : 0) + (f & NEED_FSUM ? 8 : 0);
        }
        if (dp.n_sagg > 0) bytes_per_key += 8 + 9 * dp.n_sagg;   // key offsets + cursors, results + tags
        int want = env_int("EKGPU_KBITS", 11);
        kbits = 0;
        while ((1u << kbits) < K && kbits < want) kbits++;
        while (kbits > 0 && ((1 << kbits) * bytes_per_key) > 48 * 1024) kbits--;
        if ((1 << kbits) > kMaxBucketKeys) kbits = 13;   // k_agg's present mask (kMaxBucketKeys)
        NB = (int)((K + (1u << kbits) - 1) >> kbits);
        Kpad = (int64_t)NB << kbits;
        // LDS layout (8-byte fields first for alignment)
        {
            int kk = 1 << kbits;
            int o = 0;
            for (int v = 0; v < dp.n_vc; ++v) {
                int f = dp.vc_flags[v];
                if (f & NEED_SUM) { lay.off_sum[v] = o; o += 8 * kk; }
                if (f & NEED_MIN) { lay.off_min[v] = o; o += 8 * kk; }
                if (f & NEED_MAX) { lay.off_max[v] = o; o += 8 * kk; }
                if (f & NEED_M2) { lay.off_m2[v] = o; o += 8 * kk; }
                if (f & NEED_FSUM) { lay.off_fsum[v] = o; o += 8 * kk; }
            }
            if (dp.n_sagg > 0) { lay.off_sres = o; o += 8 * kk * dp.n_sagg; }
            lay.off_cnt = o; o += 4 * kk;
            for (int v = 0; v < dp.n_vc; ++v) if (dp.vc_flags[v] & NEED_CNT) { lay.off_vcnt[v] = o; o += 4 * kk; }
            if (dp.n_sagg > 0) {
                lay.off_koff = o; o += 4 * (kk + 1);
                lay.off_kcur = o; o += 4 * kk;
                lay.off_stag = o; o += dp.n_sagg * kk;
            }
            // the sparse-partition path of k_agg stages its rows in the same LDS
            lay.bytes = (int32_t)std::max<size_t>((size_t)((o + 15) & ~15), (sparse_lds_bytes(dp.n_vc) + 15) & ~(size_t)15);
        }
        chunk = env_int("EKGPU_CHUNK", 8192);
        sorted_chunk = env_int("EKGPU_SORTED_CHUNK", kTile);
        // the fused sorted pass is built and parity-tested but off by default: measured on MI355X it moves the same
        // bytes at the same mixed read/write rate as k_stats + k_part and keeps two round trips
        fz_on = env_int("EKGPU_FUSED", 0);
        small_win_on = env_int("EKGPU_SMALL_WIN", 1) != 0;
        sw_grid = std::max(1, env_int("EKGPU_SW_GRID", 4096));
        fin_ring = env_int("EKGPU_FIN_RING", 1) != 0;
        fin_ring_chunks = env_int("EKGPU_FIN_RING_CHUNKS", 0);
        fin_ring_split = env_int("EKGPU_FIN_RING_SPLIT", 0);
        km_mode = env_int("EKGPU_KEYMAJOR", 2);
        ung_mode = env_int("EKGPU_UNG", 1);
        km_one = env_int("EKGPU_KM_ONE", 1);
        km_packed = env_int("EKGPU_KM_PACKED", 1);
        km_states = env_int("EKGPU_KM_STATES", 1);
        km_single = env_int("EKGPU_KM_SINGLE", 1);
        km_merge_sort = env_int("EKGPU_KM_MERGE_SORT", 1);
        km_msd_on = env_int("EKGPU_KM_MSD", 1);
        count_direct = env_int("EKGPU_COUNT_DIRECT", 1);
        sw_cap_on = env_int("EKGPU_SW_CAP", 1);
        grp_on = env_int("EKGPU_GRP", 1);
        eb_need_init();
        agg_small = env_int("EKGPU_AGG_SMALL", 1) != 0;
        phase_events = env_int("EKGPU_PHASE_EVENTS", 1) != 0;
        stats_blocks = std::max(1, env_int("EKGPU_STATS_BLOCKS", 1024));
        variant = env_int("EKGPU_VARIANT", 0);
        // one group per batch by default (full-chip launches); bounded by the per-partition run list of k_agg
        group_events = (int64_t)env_int("EKGPU_GROUP_EVENTS", 1 << 30);
        // chunk-local partitions k_part can sort through LDS: 8 B each next to the 4096-row staging (~13 K)
        np_max = env_int("EKGPU_NP_MAX", 13000);
        max_panes_group = env_int("EKGPU_MAX_GROUP_PANES", 4096);
        // pane-state ring: pane mode only (range-mode windows aggregate from the event buffer; a COUNTWINDOW(1000) ring
        // of 2 ppw + 16 slots held 2016 x K x 24 B — 387 GB at 8 M keys)
        ring = range_mode ? 4 : (int)(2 * ppw + 16);

        // ---- HIP resources
        if (hipSetDevice(device) != hipSuccess) return fail(EK_ERR_DEVICE, "hipSetDevice(%d) failed", device);
        if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return fail(EK_ERR_DEVICE, "stream create failed");
        own_stream = true;
        hipEventCreate(&ev0);
        hipEventCreate(&ev1);
        // the pre-window filter plan (d_plan_where: its where_prog is the program of the FilterOp in front of the window):
        // processing time — WHERE AND FILTER pushed below TUMBLING / HOPPING / SESSION, FILTER alone before SLIDING,
        // COUNT and STATE windows (rows compacted at delivery, proc_prefilter); event time — FILTER alone, applied to
        // the rows WatermarkOp accepted (filter_accept)
        pre_filter = proc_pushdown || plan.n_filter > 0;
        if (pre_filter) {
            const bool push_where = ((proc && !proc_inc && wtype != EK_WINDOW_SLIDING) || (wtype == EK_WINDOW_STATE && !plan.is_event_time)) &&
                                    plan.n_where > 0;
            std::vector<ek_instr> prog;
            if (push_where) prog.insert(prog.end(), plan.where_prog, plan.where_prog + plan.n_where);
            if (plan.n_filter > 0) {
                prog.insert(prog.end(), plan.filter_prog, plan.filter_prog + plan.n_filter);
                if (push_where) { ek_instr a{}; a.op = EK_OP_AND; prog.push_back(a); }   // combine(where, filter)
            }
            if ((int)prog.size() > EK_MAX_PROG || !prog_depth_ok(prog.data(), (int)prog.size()))
                return fail(EK_ERR_UNSUPPORTED, "WHERE AND FILTER pushed below the window: the combined condition is longer "
                                                "than %d instructions or nests deeper than %d operands", EK_MAX_PROG, kEvalDepth);
            DPlan pre = dp;
            pre.n_where = (int)prog.size();
            memcpy(pre.where_prog, prog.data(), prog.size() * sizeof(ek_instr));
            if (hipMalloc((void**)&d_plan_where, sizeof(DPlan)) != hipSuccess) return fail(EK_ERR_NOMEM, "plan alloc");
            if (hipMemcpy(d_plan_where, &pre, sizeof(DPlan), hipMemcpyHostToDevice) != hipSuccess) return fail(EK_ERR_DEVICE, "plan copy");
            if (push_where) dp.n_where = 0;   // the pre-filter already dropped every row whose WHERE is not true
        }
        if (inc_where) {
            // k_inc_where's plan keeps WHERE and HAVING; the aggregation runs without either
            DPlan w = dp;
            dp_incw = dp;
            if (hipMalloc((void**)&d_plan_incw, sizeof(DPlan)) != hipSuccess) return fail(EK_ERR_NOMEM, "plan alloc");
            if (hipMemcpy(d_plan_incw, &w, sizeof(DPlan), hipMemcpyHostToDevice) != hipSuccess) return fail(EK_ERR_DEVICE, "plan copy");
            where_can_fail = prog_can_fail(dp.where_prog, dp.n_where, dp.agg_fn, dp.col_type);
            having_can_fail = dp.n_having > 0 && prog_can_fail(dp.having_prog, dp.n_having, dp.agg_fn, dp.col_type);
            dp.n_where = 0;
            dp.n_having = 0;
            dp.having_star = 0;
        } else {
            where_can_fail = dp.n_where > 0 && prog_can_fail(dp.where_prog, dp.n_where, dp.agg_fn, dp.col_type);
            having_can_fail = dp.n_having > 0 && prog_can_fail(dp.having_prog, dp.n_having, dp.agg_fn, dp.col_type);
        }
        for (int k = 0; k < dp.n_aggs; ++k)
            agg_can_fail |= dp.agg_fn[k] == EK_AGG_PERCENTILE_CONT || dp.agg_fn[k] == EK_AGG_PERCENTILE_DISC || dp.med_first[k] >= 0;
        if (hipMalloc((void**)&d_plan, sizeof(DPlan)) != hipSuccess) return fail(EK_ERR_NOMEM, "plan alloc");
        if (hipMemcpy(d_plan, &dp, sizeof(DPlan), hipMemcpyHostToDevice) != hipSuccess) return fail(EK_ERR_DEVICE, "plan copy");
        if (dp.having_star) {
            // HAVING over count(*) alone, decided once per row count by the device evaluator (k_small_win<HS> reads it)
            hipLaunchKernelGGL(k_hstar_tab, dim3(1), dim3(256), 0, stream, d_plan);
            if (hipMemcpyAsync(dp.hstar_tab, d_plan->hstar_tab, sizeof dp.hstar_tab, hipMemcpyDeviceToHost, stream) != hipSuccess ||
                hipStreamSynchronize(stream) != hipSuccess)
                return fail(EK_ERR_DEVICE, "HAVING table failed");
        }
        if (hipHostMalloc((void**)&h_stats, sizeof(BatchStats)) != hipSuccess) return fail(EK_ERR_NOMEM, "pinned alloc");
        if (int rc = ensure(bstats, sizeof(BatchStats))) return rc;
        if (int rc = alloc_state()) return rc;
        reset_state();
        return 0;
    }

    int n_state_fields() const {
        int nf = 1;
        for (int v = 0; v < dp.n_vc; ++v) {
            int f = dp.vc_flags[v];
            nf += !!(f & NEED_CNT) + !!(f & NEED_SUM) + !!(f & NEED_MIN) + !!(f & NEED_MAX) + !!(f & NEED_M2) + !!(f & NEED_FSUM);
        }
        return nf;
    }
    // SoA fields, each R * Kpad entries of 8 bytes, carved from one allocation
    DState carve_state(void* base, int R) const {
        size_t per = (size_t)R * Kpad * 8;
        char* b = (char*)base;
        DState d{};
        d.K = Kpad;
        d.cnt = (int64_t*)b; b += per;
        for (int v = 0; v < dp.n_vc; ++v) {
            int f = dp.vc_flags[v];
            if (f & NEED_CNT) { d.vcnt[v] = (int64_t*)b; b += per; }
            if (f & NEED_SUM) { d.sum[v] = (int64_t*)b; b += per; }
            if (f & NEED_MIN) { d.mn[v] = (int64_t*)b; b += per; }
            if (f & NEED_MAX) { d.mx[v] = (int64_t*)b; b += per; }
            if (f & NEED_M2) { d.m2[v] = (double*)b; b += per; }
            if (f & NEED_FSUM) { d.fsum[v] = (double*)b; b += per; }
        }
        return d;
    }
    int alloc_state() {
        if (int rc = ensure(state_buf, (size_t)ring * Kpad * 8 * n_state_fields())) return rc;
        dstate = carve_state(state_buf.p, ring);
        if (int rc = ensure(pane_err, (size_t)ring * 4)) return rc;
        if (int rc = ensure(pane_mcnt, (size_t)ring * 8)) return rc;
        if (int rc = ensure(pane_mhash, (size_t)ring * 8)) return rc;
        if (where_can_fail) {
            if (int rc = ensure(pane_wit, (size_t)ring * sizeof(WitRec))) return rc;
            hipMemsetAsync(pane_wit.p, 0, (size_t)ring * sizeof(WitRec), stream);
        }
        return 0;
    }
    // Grow the pane ring to at least `need` slots, moving the partials of live panes.
    int ensure_ring(int64_t need) {
        if (need <= ring) return 0;
        int R = (int)std::max<int64_t>(need, (int64_t)ring * 2);
        hipStreamSynchronize(stream);
        const int nf = n_state_fields();
        DevBuf nsb, npe, npm, nph, npw;
        if (hipMalloc(&nsb.p, (size_t)R * Kpad * 8 * nf) != hipSuccess) return fail(EK_ERR_NOMEM, "pane state alloc (%d slots)", R);
        nsb.bytes = (size_t)R * Kpad * 8 * nf;
        if (hipMalloc(&npe.p, (size_t)R * 4) != hipSuccess || hipMalloc(&npm.p, (size_t)R * 8) != hipSuccess ||
            hipMalloc(&nph.p, (size_t)R * 8) != hipSuccess)
            return fail(EK_ERR_NOMEM, "pane scalar alloc");
        npe.bytes = (size_t)R * 4; npm.bytes = nph.bytes = (size_t)R * 8;
        if (where_can_fail) {
            if (hipMalloc(&npw.p, (size_t)R * sizeof(WitRec)) != hipSuccess) return fail(EK_ERR_NOMEM, "pane witness alloc");
            npw.bytes = (size_t)R * sizeof(WitRec);
            hipMemsetAsync(npw.p, 0, npw.bytes, stream);
        }
        DState nd = carve_state(nsb.p, R);
        std::vector<int64_t> nslot(R, INT64_MIN);
        const int64_t first_live = win_first_pane(next_win);
        const size_t per = (size_t)Kpad * 8;
        for (int so = 0; so < ring; ++so) {
            int64_t q = slot_pane[so];
            if (q == INT64_MIN || q < first_live) continue;
            int sn = (int)(q % R);
            nslot[sn] = q;
            auto mv = [&](void* dst, void* src) { if (src) hipMemcpyAsync((char*)dst + sn * per, (char*)src + so * per, per, hipMemcpyDeviceToDevice, stream); };
            mv(nd.cnt, dstate.cnt);
            for (int v = 0; v < dp.n_vc; ++v) {
                if (dstate.vcnt[v]) mv(nd.vcnt[v], dstate.vcnt[v]);
                if (dstate.sum[v]) mv(nd.sum[v], dstate.sum[v]);
                if (dstate.mn[v]) mv(nd.mn[v], dstate.mn[v]);
                if (dstate.mx[v]) mv(nd.mx[v], dstate.mx[v]);
                if (dstate.m2[v]) mv(nd.m2[v], dstate.m2[v]);
                if (dstate.fsum[v]) mv(nd.fsum[v], dstate.fsum[v]);
            }
            hipMemcpyAsync((char*)npe.p + sn * 4, (char*)pane_err.p + so * 4, 4, hipMemcpyDeviceToDevice, stream);
            hipMemcpyAsync((char*)npm.p + sn * 8, (char*)pane_mcnt.p + so * 8, 8, hipMemcpyDeviceToDevice, stream);
            hipMemcpyAsync((char*)nph.p + sn * 8, (char*)pane_mhash.p + so * 8, 8, hipMemcpyDeviceToDevice, stream);
            if (npw.p)
                hipMemcpyAsync((char*)npw.p + sn * sizeof(WitRec), (char*)pane_wit.p + so * sizeof(WitRec), sizeof(WitRec),
                               hipMemcpyDeviceToDevice, stream);
        }
        hipStreamSynchronize(stream);
        release(state_buf); release(pane_err); release(pane_mcnt); release(pane_mhash); release(pane_wit);
        state_buf = nsb; pane_err = npe; pane_mcnt = npm; pane_mhash = nph; pane_wit = npw;
        dstate = nd;
        slot_pane = nslot;
        ring = R;
        return 0;
    }

    void reset_state() {
        has_M = has_W = e1_known = false;
        M = W = kMinTs;
        E1 = first_ts = 0;
        next_win = 0;
        reg_win = 0;
        arrivals = 0;
        pend_n = 0;
        pend_min = INT64_MAX;
        pend_max = INT64_MIN;
        pend_arr.clear();
        for (int c = 0; c < EK_MAX_COLUMNS; ++c) { pend_host[c].clear(); pend_vhost[c].clear(); pend_has_valid[c] = false; }
        slot_pane.assign(ring, INT64_MIN);
        // range mode
        eb.n = 0;
        eb_arr_impl = true;
        eb_arr0 = 0;
        eb_base = 0;
        eb_rel = 0;
        eb_floor = 0;
        sW = -1;
        range_wins = 0;
        delayq.clear();
        delayq_head = 0;
        h_rts.clear();
        h_rwp.clear();
        h_rts_base = 0;
        sess_last_ticked = sess_has_trigger = false;
        sess_trigger = 0;
        st_on = false;
        st_start_abs = 0;
        count_k = 1;
        inc_has_T = false;
        inc_T = 0;
        inc_pend.clear();
        gmode = 0;
        g_row_arr = nullptr;
        clock_started = false;
        clock_ms = kMinTs;
        ps_tick = 0;
        ps_to_exists = ps_to_armed = false;
        ps_to_due = 0;
        ps_next_abs = 0;
        ps_last_nonmatch = INT64_MIN;
        proc_dq.clear();
        proc_dq_head = 0;
        sw2_e.clear();
        sw2_cut = 0;
        sw2_gcb = INT64_MIN;
        sw2_gcx = 0;
        h_rtrig.clear();
        et2_prev = kYear1Ms;
        zero_pend.n = 0;
        pi_reset();
        v2q.clear();
        v2q_head = v2q_seen = 0;
        v2_lastW = INT64_MIN;
        g_wa = g_wt = nullptr;
        g_nwm = 0;
        g_sess_last_end = INT64_MIN;
        g_trig.clear();
        wins.clear();
        r_rows_used = 0;
        // counters restart with the stream; the running device-time totals (ek_stats *_total) span resets
        const ek_stats keep = stats;
        stats = ek_stats{};
        stats.device_ms_total = keep.device_ms_total;
        stats.pushes_timed = keep.pushes_timed;
        for (int k = 0; k < 4; ++k) { stats.phase_ms_total[k] = keep.phase_ms_total[k]; stats.phase_launches_total[k] = keep.phase_launches_total[k]; }
    }

    // ------------------------------------------------------------------ pane geometry
    int64_t win_end(int64_t j) const { return E1 + j * H; }
    int64_t win_first_pane(int64_t j) const { return wtype == EK_WINDOW_TUMBLING ? j : j * hpp; }
    int64_t win_last_pane(int64_t j) const { return wtype == EK_WINDOW_TUMBLING ? j : j * hpp + ppw - 1; }
    int64_t pane_host(int64_t ts) const {
        if (wtype == EK_WINDOW_TUMBLING) return ts < E1 ? 0 : floordiv_h(ts - E1, P) + 1;
        int64_t o = E1 - L;
        return ts < o ? -1 : floordiv_h(ts - o, P);
    }
    int64_t pane_start(int64_t q) const {
        if (wtype == EK_WINDOW_TUMBLING) return q == 0 ? INT64_MIN : E1 + (q - 1) * P;
        return E1 - L + q * P;
    }

    // Bind panes [qa, qb] to ring slots. A pane new to its slot is "fresh": its partials are written
    // (not merged) by the next k_agg, or zeroed here when `zero` (panes no group ever touched).
    int claim_slots(int64_t qa, int64_t qb, uint8_t* fresh, bool zero) {
        int64_t first_live = win_first_pane(next_win);
        if (int rc = ensure_ring(qb - std::min(first_live, qa) + 3)) return rc;
        if (fresh) memset(fresh, 0, (size_t)(qb - qa + 1));
        for (int64_t q = qa; q <= qb; ++q) {
            int s = (int)(q % ring);
            if (slot_pane[s] == q) continue;
            if (slot_pane[s] != INT64_MIN && slot_pane[s] >= first_live)
                return fail(EK_ERR_UNSUPPORTED, "pane ring overflow (pane %lld needs slot %d held by live pane %lld)",
                            (long long)q, s, (long long)slot_pane[s]);
            slot_pane[s] = q;
            if (fresh) fresh[q - qa] = 1;
            if (!zero) continue;
            // queued: flush_zero_slots zeroes the whole list in one launch
            if (zero_pend.n == kZeroSlotsMax) flush_zero_slots();
            zero_pend.s[zero_pend.n++] = s;
        }
        return 0;
    }
    SlotList zero_pend{};
    void flush_zero_slots() {
        if (zero_pend.n == 0) return;
        const int64_t per_words = Kpad;
        const int bx = (int)std::min<int64_t>(64, (per_words + 4095) / 4096);
        hipLaunchKernelGGL(k_zero_slots, dim3(bx, zero_pend.n), dim3(256), 0, stream, zero_pend, (uint64_t*)dstate.cnt,
                           per_words, (int32_t*)pane_err.p, (int64_t*)pane_mcnt.p, (uint64_t*)pane_mhash.p,
                           (uint8_t*)pane_wit.p, (int)sizeof(WitRec));
        zero_pend.n = 0;
    }

    // pinned host bump buffer for small per-launch descriptors (reset once per push, after a sync)
    int64_t* h_desc = nullptr;
    size_t h_desc_cap = 0, h_desc_used = 0;
    int64_t* desc_alloc(size_t n) {
        if (h_desc_used + n > h_desc_cap) {
            hipStreamSynchronize(stream);
            drain_downs();   // staged device -> host copies leave the block before it is recycled
            if (h_desc_cap < n) {
                if (h_desc) hipHostFree(h_desc);
                h_desc_cap = std::max<size_t>(n, 1 << 16);
                if (hipHostMalloc((void**)&h_desc, h_desc_cap * 8) != hipSuccess) { h_desc = nullptr; h_desc_cap = 0; return nullptr; }
            }
            h_desc_used = 0;
        }
        int64_t* r = h_desc + h_desc_used;
        h_desc_used += n;
        return r;
    }
    // n elements of a host array staged through the pinned block and copied to dst on the stream (the block is only
    // recycled after a sync, so the caller's array may change at once)
    template <typename T>
    int up_pinned(void* dst, const T* src, size_t n) {
        if (n == 0) return 0;
        int64_t* h = desc_alloc((n * sizeof(T) + 7) / 8);
        if (!h) return fail(EK_ERR_NOMEM, "pinned");
        memcpy(h, src, n * sizeof(T));
        hipMemcpyAsync(dst, h, n * sizeof(T), hipMemcpyHostToDevice, stream);
        return 0;
    }
    // device -> host through the pinned block: the copy is queued now, the bytes land in dst at sync_downs() (or when
    // the block is recycled)
    struct Down { void* dst; const int64_t* h; size_t bytes; };
    std::vector<Down> downs;
    int down_pinned(void* dst, const void* src, size_t bytes) {
        if (bytes == 0) return 0;
        int64_t* h = desc_alloc((bytes + 7) / 8);
        if (!h) return fail(EK_ERR_NOMEM, "pinned");
        hipMemcpyAsync(h, src, bytes, hipMemcpyDeviceToHost, stream);
        downs.push_back(Down{dst, h, bytes});
        return 0;
    }
    void drain_downs() {
        for (const Down& d : downs) memcpy(d.dst, d.h, d.bytes);
        downs.clear();
    }
    int sync_downs(const char* what) {
        if (hipStreamSynchronize(stream) != hipSuccess) { downs.clear(); return fail(EK_ERR_DEVICE, "%s", what); }
        drain_downs();
        return 0;
    }
    DevBuf aux_d;
    size_t aux_used = 0;

    // ------------------------------------------------------------------ results
    int ensure_results(int64_t add_rows, int64_t add_wins) {
        int64_t need_rows = r_rows_used + add_rows;
        if (need_rows > r_rows_cap) {
            int64_t cap = std::max<int64_t>(need_rows, r_rows_cap * 2);
            cap = std::max<int64_t>(cap, 1024);
            // grow with copy of the live rows
            auto grow = [&](DevBuf& b, size_t esz) -> int {
                DevBuf nb;
                if (hipMalloc(&nb.p, (size_t)cap * esz) != hipSuccess) return fail(EK_ERR_NOMEM, "result alloc");
                nb.bytes = (size_t)cap * esz;
                if (b.p && r_rows_used) hipMemcpyAsync(nb.p, b.p, (size_t)r_rows_used * esz, hipMemcpyDeviceToDevice, stream);
                if (b.p) { hipStreamSynchronize(stream); hipFree(b.p); }
                b = nb;
                return 0;
            };
            if (int rc = grow(r_key, 4)) return rc;
            for (int k = 0; k < n_res; ++k) {
                if (int rc = grow(r_val[k], 8)) return rc;
                if (int rc = grow(r_tag[k], 1)) return rc;
            }
            r_rows_cap = cap;
        }
        int64_t need_w = (int64_t)wins.size() + add_wins;
        if (need_w > r_win_cap) {
            int64_t cap = std::max<int64_t>(need_w, std::max<int64_t>(r_win_cap * 2, 256));
            auto growz = [&](DevBuf& b, size_t esz) -> int {
                DevBuf nb;
                if (hipMalloc(&nb.p, (size_t)cap * esz) != hipSuccess) return fail(EK_ERR_NOMEM, "window alloc");
                nb.bytes = (size_t)cap * esz;
                hipMemsetAsync(nb.p, 0, (size_t)cap * esz, stream);
                if (b.p && !wins.empty()) hipMemcpyAsync(nb.p, b.p, wins.size() * esz, hipMemcpyDeviceToDevice, stream);
                if (b.p) { hipStreamSynchronize(stream); hipFree(b.p); }
                b = nb;
                return 0;
            };
            if (int rc = growz(r_wcnt, 8)) return rc;
            if (int rc = growz(r_werr, 4)) return rc;
            if (int rc = growz(r_wmc, 8)) return rc;
            if (int rc = growz(r_wmh, 8)) return rc;
            if (where_can_fail || having_can_fail)
                if (int rc = growz(r_wwit, 2 * sizeof(WitRec))) return rc;
            if (agg_can_fail)
                if (int rc = growz(r_aslot, 4)) return rc;
            r_win_cap = cap;
        }
        return 0;
    }

    Results results_view() {
        Results r{};
        r.key = (uint32_t*)r_key.p;
        for (int k = 0; k < n_res; ++k) { r.val[k] = (int64_t*)r_val[k].p; r.tag[k] = (uint8_t*)r_tag[k].p; }
        r.win_cnt = (int64_t*)r_wcnt.p;
        r.win_err = (int32_t*)r_werr.p;
        r.wwit = (WitRec*)r_wwit.p;
        r.pwit = (const WitRec*)pane_wit.p;
        r.aslot = (int32_t*)r_aslot.p;
        return r;
    }

    // window_op.go:688-716 scan(): windowStart by type, then the <= 0 fallback
    int64_t window_start(int64_t j) const {
        int64_t trig = j == 0 ? first_ts : win_end(j - 1);
        int64_t ws = wtype == EK_WINDOW_TUMBLING ? trig : trig - H;
        if (ws <= 0) ws = win_end(j) - L;
        return ws;
    }

    // Windows are registered (result region + index) strictly in trigger order, possibly before
    // their rows exist: a tumbling pane emitted directly by k_agg registers every earlier window first.
    int64_t reg_win = 0;               // next window index to register
    int register_until(int64_t j) {
        while (reg_win <= j) {
            if (int rc = ensure_results(Krows(), 1)) return rc;
            WinInfo wi{};
            wi.j = reg_win;
            wi.end = win_end(reg_win);
            wi.start = window_start(reg_win);
            wi.out_base = r_rows_used;
            wi.slot = (int32_t)wins.size();
            wi.direct = false;
            r_rows_used += Krows();
            wins.push_back(wi);
            reg_win++;
        }
        return 0;
    }
    WinInfo& win_info(int64_t j) { return wins[(size_t)(j - wins.front().j)]; }
    int64_t Krows() const { return dp.pseudo_keys ? 1 : (int64_t)K; }   // result rows a window can hold

    // Emit every window j >= next_win with E_j <= W whose panes are complete (last pane <= q_done). A window none of
    // whose panes a row touched is empty: it is reported with no rows and takes neither result rows nor pane slots,
    // and the windows before it are merged first, so an idle stretch of N windows (a clock jump, an event-time gap)
    // costs O(N) host work and no memory (the reference fires one scan per tick, window_op.go:483-499).
    int finalize_ready(int64_t q_done) {
        if (!e1_known || !has_W) return 0;
        int64_t j1 = next_win;
        while (win_end(j1) <= W && win_last_pane(j1) <= q_done) j1++;
        int64_t seg = next_win;
        for (int64_t j = next_win; j < j1; ++j) {
            if (j < reg_win || pane_touched(j)) continue;
            if (int rc = finalize_range(seg, j)) return rc;
            if (int rc = ensure_results(0, 1)) return rc;
            WinInfo wi{};
            wi.j = j;
            wi.end = win_end(j);
            wi.start = window_start(j);
            wi.out_base = r_rows_used;
            wi.slot = (int32_t)wins.size();
            wi.direct = true;
            wins.push_back(wi);
            reg_win = j + 1;
            next_win = j + 1;
            stats.windows_out++;
            seg = j + 1;
        }
        return finalize_range(seg, j1);
    }
    // a row reached one of window j's panes (its pane is bound to a ring slot)
    bool pane_touched(int64_t j) const {
        for (int64_t q = std::max<int64_t>(0, win_first_pane(j)); q <= win_last_pane(j); ++q)
            if (slot_pane[(size_t)(q % ring)] == q) return true;
        return false;
    }
    // Merge and emit windows [j0, j1) (all registered or registrable, none empty-skipped).
    int finalize_range(int64_t j0, int64_t j1) {
        if (j1 <= j0) return 0;
        int64_t n = j1 - j0;
        if (int rc = register_until(j1 - 1)) return rc;
        // panes no group touched hold no events: bind and zero them so the merge reads empty partials
        for (int64_t j = j0; j < j1; ++j) {
            if (win_info(j).direct) continue;
            if (int rc = claim_slots(std::max<int64_t>(0, win_first_pane(j)), win_last_pane(j), nullptr, true)) return rc;
        }
        flush_zero_slots();
        if (h_wdesc_used + n > h_wdesc_cap) {
            hipStreamSynchronize(stream);  // every earlier descriptor upload has completed
            if (h_wdesc_cap < (size_t)n) {
                if (h_wdesc) hipHostFree(h_wdesc);
                h_wdesc_cap = std::max<size_t>(n, 4096);
                if (hipHostMalloc((void**)&h_wdesc, h_wdesc_cap * sizeof(WinDesc)) != hipSuccess) return fail(EK_ERR_NOMEM, "pinned");
            }
            h_wdesc_used = 0;
        }
        WinDesc* hd = h_wdesc + h_wdesc_used;
        h_wdesc_used += n;
        if (int rc = ensure(wdesc, (size_t)n * sizeof(WinDesc))) return rc;
        // descriptors: windows needing the pane merge first, then the direct ones (membership only)
        int64_t nf = 0;
        for (int64_t j = j0; j < j1; ++j) nf += win_info(j).direct ? 0 : 1;
        int64_t k = 0;
        for (int pass = 0; pass < 2; ++pass)
            for (int64_t j = j0; j < j1; ++j) {
                const WinInfo& wi = win_info(j);
                if (wi.direct != (pass == 1)) continue;
                WinDesc& d = hd[k++];
                d.q_first = std::max<int64_t>(0, win_first_pane(j));
                d.q_last = win_last_pane(j);
                d.out_base = wi.out_base;
                d.idx = wi.slot;
            }
        if (nf || plan.debug_membership)
            hipMemcpyAsync(wdesc.p, hd, (size_t)n * sizeof(WinDesc), hipMemcpyHostToDevice, stream);
        if (nf) {
            const int nvc = std::max(1, dp.n_vc);
            Results rv = results_view();
            const WinDesc* wd = (const WinDesc*)wdesc.p;
            const int ph = phase_begin(EK_PHASE_FINALIZE);
            // consecutive hopping windows over one count / sum / min / max column: the register-ring walk reads each
            // pane once (k_finalize_ring); anything else merges per (window, key block) (k_finalize)
            int64_t span = 0;
            bool ordered = true;
            for (int64_t i = 0; i < nf; ++i) {
                span = std::max(span, hd[i].q_last - hd[i].q_first + 1);
                if (i && (hd[i].q_first < hd[i - 1].q_first || hd[i].q_last <= hd[i - 1].q_last)) ordered = false;
            }
            bool ring_ok = fin_ring && nf >= 2 && ordered && span <= 16 && !dp.pseudo_keys && dp.n_vc == 1 &&
                           dp.n_sagg == 0 && (dp.vc_flags[0] & ~(NEED_CNT | NEED_SUM | NEED_MIN | NEED_MAX)) == 0;
            for (int k = 0; k < dp.n_aggs && ring_ok; ++k)   // the ring's own emission: count / sum / avg / min / max
                ring_ok = dp.agg_fn[k] == EK_AGG_COUNT_STAR ||
                          (dp.agg_vc[k] == 0 && (dp.agg_fn[k] == EK_AGG_COUNT || dp.agg_fn[k] == EK_AGG_SUM ||
                                                 dp.agg_fn[k] == EK_AGG_AVG || dp.agg_fn[k] == EK_AGG_MIN ||
                                                 dp.agg_fn[k] == EK_AGG_MAX));
            if (ring_ok) {
                const int64_t kb = (K + kBlock - 1) / kBlock;
                int64_t chunks = fin_ring_chunks > 0 ? fin_ring_chunks
                                                     : std::max<int64_t>(1, std::min<int64_t>(nf / (4 * span), (1024 + kb - 1) / kb));
                chunks = std::max<int64_t>(1, std::min<int64_t>(chunks, nf));
                const int64_t cw = (nf + chunks - 1) / chunks;
                dim3 grid_r((unsigned)kb, (unsigned)((nf + cw - 1) / cw));
                const bool vcr = (dp.vc_flags[0] & NEED_CNT) != 0;
                // split walk (no HAVING, both halves needed): count / sum, then min / max, each at twice the occupancy
                const int fl = dp.vc_flags[0];
                const bool split = fin_ring_split && dp.n_having == 0 && (fl & NEED_SUM) && (fl & (NEED_MIN | NEED_MAX));
                if (split) {
                    if (int rc = ensure(ring_gbase, (size_t)grid_r.x * grid_r.y * cw * 4 + 64)) return rc;
                    ek::launch_fin_ring((int)span, vcr, false, 1, grid_r, stream, d_plan, wd, (int32_t)nf, (int32_t)cw, dstate, ring,
                                        (const int32_t*)pane_err.p, rv, (uint32_t*)ring_gbase.p);
                    ek::launch_fin_ring((int)span, vcr, false, 2, grid_r, stream, d_plan, wd, (int32_t)nf, (int32_t)cw, dstate, ring,
                                        (const int32_t*)pane_err.p, rv, (uint32_t*)ring_gbase.p);
                } else {
                    ek::launch_fin_ring((int)span, vcr, dp.n_having > 0, 0, grid_r, stream, d_plan, wd, (int32_t)nf, (int32_t)cw, dstate,
                                        ring, (const int32_t*)pane_err.p, rv, nullptr);
                }
            } else {
                dim3 grid_f((unsigned)((K + kBlock - 1) / kBlock), (unsigned)nf);
                ek::launch_fin(nvc, dp.pseudo_keys != 0, grid_f, stream, d_plan, wd, dstate, ring, (const int32_t*)pane_err.p, rv);
            }
            phase_end(ph);
        }
        if (plan.debug_membership) {
            hipLaunchKernelGGL(k_win_members, dim3((unsigned)n), dim3(64), 0, stream, (const WinDesc*)wdesc.p, ring,
                               (const int64_t*)pane_mcnt.p, (const unsigned long long*)pane_mhash.p, (int64_t*)r_wmc.p,
                               (unsigned long long*)r_wmh.p);
        }
        next_win = j1;
        stats.windows_out += n;
        return 0;
    }

    // ------------------------------------------------------------------ batch processing
    int process(const DBatch& db, bool sorted, int64_t start, const uint8_t* d_acc, int64_t min_acc, int64_t max_ts,
                const int64_t* d_arrival) {
        int64_t n = db.n;
        // size the result store once for the windows this batch will close that can hold rows (the windows of an
        // event-time gap before the batch are empty: no result rows)
        if (W >= win_end(next_win)) {
            const int64_t nclose = (W - win_end(next_win)) / H + 1;
            const int64_t nrows = std::min<int64_t>(nclose, (max_ts - min_acc) / H + 2 * ppw + 2);
            if (int rc = ensure_results(nrows * Krows(), nclose)) return rc;
        }
        int64_t q_lo = std::max<int64_t>(0, pane_host(min_acc));
        int64_t q_hi = pane_host(max_ts);
        if (q_hi < 0) return 0;   // every event precedes the first hopping window
        int64_t first_live = win_first_pane(next_win);
        q_lo = std::max(q_lo, first_live);

        struct Grp { int64_t lo, hi, qa, qb; int64_t q_done; int64_t bk; };
        const int64_t pane_cap = (int64_t)(kMaxRuns - 2) * chunk;   // k_agg run list bound per pane
        std::vector<Grp> groups;
        const int64_t* fz_b = nullptr;   // the fused sorted pass's pane bounds (k_part MODE 3 already ran)
        if (sorted) {
            int64_t nq = q_hi - q_lo + 1;
            int nb = (int)nq + 1;
            if (fz_pass.on) {
                if (fz_pass.q_lo != q_lo || fz_pass.nq != nq) return fail(EK_ERR_STATE, "fused pass pane range mismatch");
                fz_b = fz_pass.pbnd;
            } else {
                // pane boundaries by binary search on the sorted ts column
                if (h_small_cap < (size_t)(2 * nb)) {
                    if (h_small) { hipStreamSynchronize(stream); hipHostFree(h_small); }
                    h_small_cap = std::max<size_t>(2 * nb, 4096);
                    if (hipHostMalloc((void**)&h_small, h_small_cap * 8) != hipSuccess) return fail(EK_ERR_NOMEM, "pinned");
                }
                if (int rc = ensure(bounds_idx, (size_t)nb * 8)) return rc;
                hipLaunchKernelGGL(k_pane_bounds, dim3((nb + kBoundsBlock / 64 - 1) / (kBoundsBlock / 64)), dim3(kBoundsBlock), 0, stream,
                                   (const int64_t*)db.col[dp.ts_col], start, n, grid, q_lo, nb, (int64_t*)bounds_idx.p);
                hipMemcpyAsync(h_small + nb, bounds_idx.p, (size_t)nb * 8, hipMemcpyDeviceToHost, stream);
                if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "bounds sync failed");
            }
            const int64_t* b = fz_b ? fz_b : h_small + nb;
            // greedy grouping of consecutive panes; a pane larger than the target is split
            int64_t k = 0;
            while (k < nq) {
                int64_t lo = b[k];
                int64_t kk = k;
                int64_t hi = b[k + 1];
                const int64_t cap = std::min(group_events, pane_cap);
                if (hi - lo > cap) {
                    // split one big pane into several groups
                    for (int64_t s = lo; s < hi; s += cap) {
                        int64_t e = std::min(hi, s + cap);
                        groups.push_back(Grp{s, e, q_lo + k, q_lo + k, e == hi ? q_lo + k : q_lo + k - 1, -1});
                    }
                    k++;
                    continue;
                }
                while (kk + 1 < nq && (b[kk + 2] - lo) <= group_events && (kk + 1 - k + 1) <= max_panes_group &&
                       b[kk + 2] - b[kk + 1] <= pane_cap) {
                    kk++;
                    hi = b[kk + 1];
                }
                groups.push_back(Grp{lo, std::max(lo, hi), q_lo + k, q_lo + kk, q_lo + kk, k});
                k = kk + 1;
            }
        } else {
            if ((q_hi - q_lo + 1) * NB > np_max)
                return fail(EK_ERR_UNSUPPORTED, "out-of-order batch spans %lld panes (max %d): split the batch",
                            (long long)(q_hi - q_lo + 1), np_max / NB);
            // every index range may hold events of any pane: finalise only after the last one
            const int64_t cap = (int64_t)(kMaxRuns - 2) * chunk;
            for (int64_t s = start; s < n; s += cap) {
                int64_t e = std::min(n, s + cap);
                groups.push_back(Grp{s, e, q_lo, q_hi, e == n ? q_hi : q_lo - 1, e == n && s == start ? 0 : -2});
            }
        }

        const int64_t* bidx = sorted ? (fz_b ? fz_b : h_small + (q_hi - q_lo + 2)) : nullptr;
        if (fz_pass.on && groups.size() != 1) return fail(EK_ERR_STATE, "fused pass split into %zu groups", groups.size());
        for (const Grp& g : groups) {
            if (g.hi > g.lo) {
                // pane boundaries of the group (sorted batches): pbnd[k] = first event of pane qa + k
                std::vector<int64_t> pb;
                if (sorted) {
                    int npn = (int)(g.qb - g.qa + 1);
                    pb.resize(npn + 1);
                    for (int k = 0; k <= npn; ++k) pb[k] = g.bk >= 0 ? bidx[g.bk + k] : (k == 0 ? g.lo : g.hi);
                    pb[0] = g.lo;
                    pb[npn] = g.hi;
                }
                // whole_panes: the group holds every event of this batch for each of its panes
                if (int rc = run_group(db, g.lo, g.hi, g.qa, g.qb, d_acc, sorted ? pb.data() : nullptr,
                                       g.bk >= 0)) return rc;
                if (plan.debug_membership) {
                    hipLaunchKernelGGL(k_members, dim3(256), dim3(kBlock), 0, stream, d_plan, db, grid, d_acc,
                                       (int)(d_acc != nullptr), g.lo, g.hi, arrivals, d_arrival, g.qa, g.qb, ring,
                                       (int64_t*)pane_mcnt.p, (unsigned long long*)pane_mhash.p);
                }
            }
            if (int rc = finalize_ready(g.q_done)) return rc;
        }
        return finalize_ready(q_hi);
    }

    size_t direct_used = 0;
    int run_group(const DBatch& db, int64_t lo, int64_t hi, int64_t qa, int64_t qb, const uint8_t* d_acc,
                  const int64_t* pbnd_host, bool whole_panes) {
        GroupDesc gd{};
        const int npn = (int)(qb - qa + 1);
        // per-pane descriptors: [pbnd n+1][dbase n][didx n (i32)][fresh n (u8)] in one pinned block -> one upload
        const size_t aux_words = aux_layout_words(npn);
        int64_t* aux = desc_alloc(aux_words);
        if (!aux) return fail(EK_ERR_NOMEM, "pinned");
        int64_t* h_pbnd = aux;
        int64_t* h_dbase = h_pbnd + npn + 1;
        int32_t* h_didx = (int32_t*)(h_dbase + npn);
        uint8_t* h_fresh = (uint8_t*)(h_didx + 2 * ((npn + 1) / 2));
        if (int rc = claim_slots(qa, qb, h_fresh, false)) return rc;
        bool any_fresh = false;
        for (int r = 0; r < npn; ++r) any_fresh |= h_fresh[r] != 0;
        gd.lo = lo;
        gd.hi = hi;
        gd.q_lo = qa;
        gd.n_panes = (int32_t)(qb - qa + 1);
        gd.nb = NB;
        gd.kbits = kbits;
        gd.abase = lo & ~(int64_t)15;
        gd.hi = hi;
        gd.n_panes = npn;
        // chunk size of this group: halve while a chunk would span more panes than k_part sorts in LDS
        // sorted groups start from single-tile chunks (keys read once, k_part's count pass skipped) and
        // grow the chunk only while a pane would span more chunk runs than k_agg walks
        int64_t csz = pbnd_host ? std::min<int64_t>(sorted_chunk, chunk) : chunk;
        int mp = max_panes_in_chunk(pbnd_host, gd, csz);
        while (pbnd_host && csz < chunk && max_chunks_in_pane(pbnd_host, gd, csz) > kMaxRuns) {
            csz <<= 1;
            mp = max_panes_in_chunk(pbnd_host, gd, csz);
        }
        while (csz > 1024 && pbnd_host && (mp > kMaxChunkBnd + 1 || (int64_t)NB * mp > np_max)) {
            csz >>= 1;
            mp = max_panes_in_chunk(pbnd_host, gd, csz);
        }
        if (fz_pass.on && (csz != kTile || mp > fz_pass.mp))
            return fail(EK_ERR_STATE, "fused pass geometry mismatch (chunk %lld, %d panes per chunk)", (long long)csz, mp);
        gd.chunk = csz;
        gd.key_col = dp.key_col;
        gd.ts_col = dp.ts_col;
        gd.n_where = dp.n_where;
        gd.num_keys = dp.num_keys;
        gd.nbatch = db.n;
        gd.nch = (int32_t)((hi - gd.abase + csz - 1) / csz);
        gd.np = gd.n_panes * NB;
        gd.ring = ring;
        gd.has_accept = d_acc != nullptr;
        gd.sorted = pbnd_host != nullptr;
        gd.pad = env_int("EKGPU_DEBUG_AGG", 0);   // diagnostic knobs (timing only; results invalid when set)
        gd.pad2 = variant;
        gd.pwit = (WitRec*)pane_wit.p;   // pane witnesses in release order: (ts, this launch, row)
        gd.wit_ts = 1;
        gd.wit_o2 = (wit_seq++) << 36;

        for (int k = 0; k <= npn; ++k) h_pbnd[k] = pbnd_host ? pbnd_host[k] : 0;
        for (int r = 0; r < npn; ++r) { h_dbase[r] = -1; h_didx[r] = -1; }
        // direct emission: a fresh tumbling pane whose whole content is in this group and whose window
        // closes at this batch's watermark is finalised by k_agg itself (no pane-state round trip)
        if (wtype == EK_WINDOW_TUMBLING && has_W && whole_panes && !dp.pseudo_keys) {
            for (int r = 0; r < npn; ++r) {
                int64_t q = qa + r;
                if (!h_fresh[r] || win_end(q) > W || q < next_win) continue;
                if (int rc = register_until(q)) return rc;
                WinInfo& wi = win_info(q);
                wi.direct = true;
                h_dbase[r] = wi.out_base;
                h_didx[r] = wi.slot;
            }
        }
        if (int rc = upload_aux(aux, aux_words, npn, gd)) return rc;
        // largest chunk-local partition count: sorted chunks touch at most the panes their index range spans
        const int lp_stride = fz_pass.on ? fz_pass.ls - 1 : (gd.sorted ? std::min(gd.np, NB * mp) : gd.np);
        if (lp_stride > np_max || (gd.sorted && mp > kMaxChunkBnd + 1))
            return fail(EK_ERR_UNSUPPORTED, "chunk spans %d partitions (split the batch)", lp_stride);
        const int mc = max_chunks_in_pane(pbnd_host, gd, gd.chunk);
        if (mc > kMaxRuns) return fail(EK_ERR_UNSUPPORTED, "a pane spans %d chunks of one group (max %d)", mc, kMaxRuns);
        gd.mruns = std::max(1, mc);
        return launch_part_agg(db, gd, gd.sorted ? 1 : 0, d_acc, (int32_t*)pane_err.p, (int64_t*)pane_mcnt.p,
                               (unsigned long long*)pane_mhash.p, lp_stride, any_fresh);
    }

    // one pinned block [pbnd n+1][dbase n][didx n (i32)][fresh n (u8)][voff n] -> device, pointers into gd
    int upload_aux(int64_t* aux, size_t aux_words, int npn, GroupDesc& gd) {
        size_t need = (aux_used + aux_words) * 8;
        if (need > aux_d.bytes) {
            hipStreamSynchronize(stream);
            aux_used = 0;
            if (int rc = ensure(aux_d, std::max<size_t>(aux_words * 8 * 4, 1 << 20))) return rc;
        }
        int64_t* dst = (int64_t*)aux_d.p + aux_used;
        aux_used += aux_words;
        hipMemcpyAsync(dst, aux, aux_words * 8, hipMemcpyHostToDevice, stream);
        gd.pbnd = dst;
        gd.dbase = dst + npn + 1;
        gd.didx = (const int32_t*)(gd.dbase + npn);
        gd.fresh = (const uint8_t*)(gd.didx + 2 * ((npn + 1) / 2));
        gd.voff = (const int64_t*)(dst + aux_layout_voff(npn));
        return 0;
    }
    static size_t aux_layout_voff(int npn) { return (size_t)(npn + 1) + npn + (npn + 1) / 2 + (npn + 7) / 8; }
    static size_t aux_layout_words(int npn) { return aux_layout_voff(npn) + npn + 2; }

    // k_part (MODE 0 unsorted / 1 sorted / 2 virtual panes) + k_agg for one group
    int launch_part_agg(const DBatch& db, GroupDesc gd, int mode, const uint8_t* d_acc, int32_t* perr,
                        int64_t* pmc, unsigned long long* pmh, int lp_stride, bool any_fresh) {
        if (dp.pseudo_keys && mode == 1 && dp.n_sagg == 0 && ung_mode) return launch_ung(db, gd, d_acc, perr, pmc, pmh, any_fresh);
        const int64_t rs = gd.chunk;                                // staging region per chunk
        int64_t ne = (int64_t)gd.nch * rs + 64;
        if (ne > st_cap) {
            if (int rc = ensure(st_klo, (size_t)ne * 2)) return rc;
            for (int v = 0; v < dp.n_vc; ++v) {
                if (int rc = ensure(st_val[v], (size_t)ne * 8)) return rc;
                if ((plan.nullable_mask >> dp.vc_col[v]) & 1u)
                    if (int rc = ensure(st_valid[v], (size_t)ne)) return rc;
            }
            st_cap = ne;
        }
        Staging st{};
        st.klo = (uint16_t*)st_klo.p;
        bool any_nullable = false;
        for (int v = 0; v < dp.n_vc; ++v) {
            st.val[v] = (int64_t*)st_val[v].p;
            if (db.valid[dp.vc_col[v]]) {
                st.valid[v] = (uint8_t*)st_valid[v].p;
                st.nullable_mask |= 1u << v;
                any_nullable = true;
            }
        }
        const int ls = lp_stride + 1;
        if (int rc = ensure(chist, (size_t)gd.nch * ls * 4)) return rc;
        if (int rc = ensure(chunk_pa, (size_t)gd.nch * 4)) return rc;
        gd.cpa = (int32_t*)chunk_pa.p;
        if (any_fresh)
            hipLaunchKernelGGL(k_group_prep, dim3((gd.n_panes + 255) / 256), dim3(256), 0, stream, gd, perr, pmc, pmh);
        const bool wh = dp.n_where > 0;
        if (!fz_pass.on) {   // (the fused sorted pass already partitioned the batch: same staging, ctab and cpa)
            const int nvc = std::max(1, dp.n_vc);
            const size_t lds_p = part_lds_bytes(nvc, lp_stride, any_nullable, gd.chunk <= kTile);
            uint32_t* ct = (uint32_t*)chist.p;
            dim3 gp(gd.nch);
            const int ph = phase_begin(EK_PHASE_PARTITION);
            ek::launch_part(mode, wh, nvc, gp, lds_p, stream, d_plan, db, grid, gd, d_acc, st, ct, ls, rs, perr);
            phase_end(ph);
        }
        {
            const int nvc = std::max(1, dp.n_vc);
            Results rv = results_view();
            rv.pwit = gd.pwit;   // the group's pane (range mode: window) witnesses
            dim3 ga(gd.np);
            const uint32_t* ct = (const uint32_t*)chist.p;
            const int ph = phase_begin(EK_PHASE_AGGREGATE);
            // order statistics: scratch region per partition = exclusive prefix of the partition sizes
            const int64_t* pbase = nullptr;
            uint64_t* scr = nullptr;
            const int64_t scr_stride = gd.hi - gd.lo;
            if (dp.n_sagg > 0) {
                if (int rc = ensure(sort_pbase, (size_t)(gd.np + 1) * 8)) return rc;
                if (int rc = ensure(sort_scr, (size_t)std::max<int64_t>(scr_stride, 1) * 8 * dp.n_scol)) return rc;
                hipLaunchKernelGGL(k_part_sizes, dim3((gd.np + 255) / 256), dim3(256), 0, stream, gd, ct, ls, (int64_t*)sort_pbase.p);
                hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, stream, (int64_t*)sort_pbase.p, gd.np);
                pbase = (const int64_t*)sort_pbase.p;
                scr = (uint64_t*)sort_scr.p;
            }
            const size_t lds_a = (size_t)lay.bytes + agg_run_lds_bytes(gd.mruns);
            // partitions averaging under 8 192 rows: the fold with 4 rows in flight per lane (k_agg<.., UR = 4>)
            const bool small = agg_small && (gd.hi - gd.lo) < (int64_t)gd.np * 8192;
            ek::launch_agg(nvc, pbase != nullptr, dp.n_having > 0, small, ga, lds_a, stream, d_plan, gd, lay, ct, ls, rs, st, dstate, rv, perr, pbase, scr,
                       scr_stride);
            phase_end(ph);
        }
        if (hipGetLastError() != hipSuccess) return fail(EK_ERR_DEVICE, "kernel launch failed");
        return 0;
    }

    // Un-grouped rule over a ts-sorted group (k_ung_tile): one pass over the referenced columns, a partial per
    // (tile, pane segment) merged into pseudo-key slot tile mod kPseudoKeys (EKGPU_UNG=0: the k_part + k_agg path).
    int ung_mode = 1;
    int64_t sorted_chunk = kTile;   // first chunk size tried for a sorted group (single-tile chunks: no count pass)
    int rowpos_col = -1;      // hidden position column of first-row fields (buffer_view: event-buffer index)
    DevBuf rowpos;            // its values 0, 1, 2, ... (grown with the buffer)
    int64_t rowpos_n = 0;
    int ensure_rowpos(int64_t n) {
        if (rowpos_col < 0 || n <= rowpos_n) return 0;
        const int64_t want = std::max<int64_t>(n, std::max<int64_t>(2 * rowpos_n, 1 << 16));
        if (int rc = ensure(rowpos, (size_t)want * 8)) return rc;
        hipLaunchKernelGGL(k_iota64, dim3((unsigned)std::min<int64_t>(8192, (want + 255) / 256)), dim3(256), 0, stream,
                           (int64_t*)rowpos.p, (int64_t)0, want);
        rowpos_n = want;
        return 0;
    }
    // first-row select fields of the windows this fire emitted: swap each slot's position for the value
    int first_fetch(const std::vector<int32_t>& slots, const std::vector<int64_t>& obase) {
        std::vector<int32_t> ws;
        std::vector<int64_t> wb;
        for (size_t w = 0; w < slots.size(); ++w)
            if (slots[w] >= 0) { ws.push_back(slots[w]); wb.push_back(obase[w]); }
        if (ws.empty()) return 0;
        const size_t nw = ws.size();
        if (int rc = ensure(ff_d, nw * 12 + 16)) return rc;
        int64_t* d_wb = (int64_t*)ff_d.p;
        int32_t* d_ws = (int32_t*)(d_wb + nw);
        hipMemcpyAsync(d_wb, wb.data(), nw * 8, hipMemcpyHostToDevice, stream);
        hipMemcpyAsync(d_ws, ws.data(), nw * 4, hipMemcpyHostToDevice, stream);
        hipLaunchKernelGGL(k_first_fetch, dim3((unsigned)nw), dim3(256), 0, stream, d_plan, buffer_view(), (const int32_t*)d_ws,
                           (const int64_t*)d_wb, results_view());
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "first-row fetch failed");
        return 0;
    }
    DevBuf ff_d;
    // WHERE (and HAVING) over the fired incremental windows' last rows (ek_range.h k_inc_where)
    int inc_where_pass(const std::vector<int32_t>& slots, const std::vector<int64_t>& obase) {
        std::vector<int32_t> ws;
        std::vector<int64_t> wb;
        for (size_t w = 0; w < slots.size(); ++w)
            if (slots[w] >= 0) { ws.push_back(slots[w]); wb.push_back(obase[w]); }
        if (ws.empty()) return 0;
        const size_t nw = ws.size();
        if (int rc = ensure(ff_d, nw * 12 + 16)) return rc;
        int64_t* d_wb = (int64_t*)ff_d.p;
        int32_t* d_ws = (int32_t*)(d_wb + nw);
        hipMemcpyAsync(d_wb, wb.data(), nw * 8, hipMemcpyHostToDevice, stream);
        hipMemcpyAsync(d_ws, ws.data(), nw * 4, hipMemcpyHostToDevice, stream);
        hipLaunchKernelGGL(k_inc_where, dim3((unsigned)nw), dim3(256), 0, stream, d_plan_incw, buffer_view(), (const int32_t*)d_ws,
                           (const int64_t*)d_wb, inc_hidden, n_res, results_view());
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "incremental WHERE pass failed");
        return 0;
    }
    int launch_ung(const DBatch& db, GroupDesc gd, const uint8_t* d_acc, int32_t* perr, int64_t* pmc,
                   unsigned long long* pmh, bool any_fresh) {
        if (any_fresh) {
            hipLaunchKernelGGL(k_group_prep, dim3((gd.n_panes + 255) / 256), dim3(256), 0, stream, gd, perr, pmc, pmh);
            hipLaunchKernelGGL(k_ung_zero, dim3(64, gd.n_panes), dim3(256), 0, stream, gd, dstate);
        }
        const int64_t rows = gd.hi - gd.lo;
        int64_t tile = 8192;
        while ((rows + tile - 1) / tile > (int64_t)kPseudoKeys) tile <<= 1;
        const int64_t nt = std::max<int64_t>(1, (rows + tile - 1) / tile);
        const int nvc = std::max(1, dp.n_vc);
        const bool wh = dp.n_where > 0;
        const int ph = phase_begin(EK_PHASE_AGGREGATE);
        ek::launch_ung(nvc, wh, dim3((unsigned)nt), stream, d_plan, db, gd, d_acc, dstate, tile, perr);
        phase_end(ph);
        if (hipGetLastError() != hipSuccess) return fail(EK_ERR_DEVICE, "kernel launch failed");
        return 0;
    }

    // Largest number of panes one chunk of the aligned grid spans (sorted groups): 1 + the most pane starts that
    // fall strictly inside one chunk (the device's chunk_panes: pa = last pane with pbnd <= c0, pb = last < c1).
    // O(panes), not O(chunks): the host computes this for every group of every push.
    int max_panes_in_chunk(const int64_t* pb, const GroupDesc& gd, int64_t chunk_sz) const {
        if (!pb) return gd.n_panes;
        int best = 0, run = 0;
        int64_t cur = -1;
        for (int k = 1; k < gd.n_panes; ++k) {
            const int64_t x = pb[k];
            if (x >= gd.hi) break;
            const int64_t c = (x - gd.abase) / chunk_sz;
            if (x <= std::max(gd.lo, gd.abase + c * chunk_sz)) continue;
            if (c != cur) { cur = c; run = 0; }
            best = std::max(best, ++run);
        }
        return best + 1;
    }
    // Largest number of chunks one pane spans (bounded by k_agg's per-partition run list).
    int max_chunks_in_pane(const int64_t* pb, const GroupDesc& gd, int64_t chunk_sz) const {
        if (!pb) return (int)((gd.hi - gd.abase + chunk_sz - 1) / chunk_sz);
        int64_t best = 0;
        for (int k = 0; k < gd.n_panes; ++k) {
            if (pb[k + 1] <= pb[k]) continue;
            best = std::max(best, (pb[k + 1] - 1 - gd.abase) / chunk_sz - (pb[k] - gd.abase) / chunk_sz + 1);
        }
        return (int)best;
    }

    // Accepted events that arrived before the first watermark release are kept (host side, tiny:
    // at most lateTolerance worth of events) until the first window end can be aligned
    // (getNextWindow on the first released event, event_window_trigger.go:57-75).
    int append_pending(const DBatch& db, const uint8_t* d_acc, int64_t arrival_base) {
        int64_t n = db.n;
        std::vector<uint8_t> acc_h;
        if (d_acc) {
            acc_h.resize(n);
            hipMemcpyAsync(acc_h.data(), d_acc, n, hipMemcpyDeviceToHost, stream);
        }
        std::vector<char> colh[EK_MAX_COLUMNS];
        std::vector<uint8_t> valh[EK_MAX_COLUMNS];
        for (int c = 0; c < plan.n_columns; ++c) {
            size_t es = plan.column_type[c] == EK_COL_U32 ? 4 : 8;
            colh[c].resize(n * es);
            hipMemcpyAsync(colh[c].data(), db.col[c], n * es, hipMemcpyDeviceToHost, stream);
            if (db.valid[c]) {
                valh[c].resize(n);
                hipMemcpyAsync(valh[c].data(), db.valid[c], n, hipMemcpyDeviceToHost, stream);
            }
        }
        std::vector<int64_t> garr;
        if (g_row_arr) {   // shard mode: global arrivals
            garr.resize(n);
            hipMemcpyAsync(garr.data(), g_row_arr, n * 8, hipMemcpyDeviceToHost, stream);
        }
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "pending copy failed");
        const int64_t* ts = (const int64_t*)colh[dp.ts_col].data();
        for (int64_t i = 0; i < n; ++i) {
            if (d_acc && !acc_h[i]) continue;
            for (int c = 0; c < plan.n_columns; ++c) {
                size_t es = plan.column_type[c] == EK_COL_U32 ? 4 : 8;
                pend_host[c].insert(pend_host[c].end(), colh[c].data() + i * es, colh[c].data() + (i + 1) * es);
                if (db.valid[c] && !pend_has_valid[c]) { pend_vhost[c].assign(pend_n, 1); pend_has_valid[c] = true; }
                if (pend_has_valid[c]) pend_vhost[c].push_back(db.valid[c] ? valh[c][i] : 1);
            }
            pend_arr.push_back(g_row_arr ? garr[i] : arrival_base + i);
            pend_min = std::min(pend_min, ts[i]);
            pend_max = std::max(pend_max, ts[i]);
            pend_n++;
        }
        return 0;
    }

    int flush_pending() {
        DBatch pb{};
        pb.n = pend_n;
        for (int c = 0; c < plan.n_columns; ++c) {
            size_t es = plan.column_type[c] == EK_COL_U32 ? 4 : 8;
            if (int rc = ensure(pend_cols[c], pend_n * es)) return rc;
            hipMemcpyAsync(pend_cols[c].p, pend_host[c].data(), pend_n * es, hipMemcpyHostToDevice, stream);
            pb.col[c] = pend_cols[c].p;
            if (pend_has_valid[c]) {
                if (int rc = ensure(pend_valid[c], pend_n)) return rc;
                hipMemcpyAsync(pend_valid[c].p, pend_vhost[c].data(), pend_n, hipMemcpyHostToDevice, stream);
                pb.valid[c] = (const uint8_t*)pend_valid[c].p;
            }
        }
        if (int rc = ensure(pend_arr_d, pend_n * 8)) return rc;
        hipMemcpyAsync(pend_arr_d.p, pend_arr.data(), pend_n * 8, hipMemcpyHostToDevice, stream);
        int rc = process(pb, false, 0, nullptr, pend_min, pend_max, (const int64_t*)pend_arr_d.p);
        hipStreamSynchronize(stream);   // host vectors may be released now
        pend_n = 0;
        pend_arr.clear();
        for (int c = 0; c < EK_MAX_COLUMNS; ++c) { pend_host[c].clear(); pend_vhost[c].clear(); pend_has_valid[c] = false; }
        return rc;
    }

    // ================================================================== RANGE mode
    // The accepted events stay in a device-resident event buffer in the order the reference's
    // WindowOperator holds them (`inputs`, window_op.go:576-739); each triggered window is an index range
    // [a, b) of it, aggregated as one "virtual pane" (k_part MODE 2 + k_agg direct emission).
    // Used for SLIDINGWINDOW, SESSIONWINDOW, COUNTWINDOW, and for tumbling/hopping windows whose
    // aggregates need the raw values (median, percentile_*).
    bool range_mode = false;
    struct EvBuf {
        DevBuf col[EK_MAX_COLUMNS], valid[EK_MAX_COLUMNS], arr, rel;
        int64_t cap = 0, n = 0;
    };
    EvBuf eb, eb_alt;
    int64_t eb_base = 0;               // absolute stream position of buffer index 0
    bool eb_valid_on[EK_MAX_COLUMNS] = {};
    // columns a range-mode kernel can read from the buffer (key, ts, aggregated / sorted value columns, WHERE /
    // trigger / STATEWINDOW condition columns, first-row sources); eb_append skips the others (the buffer keeps
    // their slot, contents unspecified and never read)
    bool eb_need[EK_MAX_COLUMNS] = {};
    void eb_need_init() {
        for (int c = 0; c < EK_MAX_COLUMNS; ++c) eb_need[c] = false;
        auto mark = [&](int c) { if (c >= 0 && c < EK_MAX_COLUMNS) eb_need[c] = true; };
        mark(dp.key_col);
        mark(dp.ts_col);
        for (int v = 0; v < dp.n_vc; ++v) mark(dp.vc_col[v]);
        for (int k = 0; k < plan.n_aggs; ++k) if (plan.aggs[k].fn == EK_AGG_FIRST) mark(plan.aggs[k].column);
        auto prog = [&](const ek_instr* pr, int n) { for (int k = 0; k < n; ++k) if (pr[k].op == EK_OP_COL) mark(pr[k].arg); };
        prog(plan.where_prog, plan.n_where);
        prog(plan.trigger_prog, plan.n_trigger);
        prog(plan.begin_prog, plan.n_begin);
        prog(plan.emit_prog, plan.n_emit);
        if (env_int("EKGPU_EB_ALL_COLUMNS", 0)) for (int c = 0; c < EK_MAX_COLUMNS; ++c) eb_need[c] = true;
    }
    bool need_rel = false;             // sliding windows: per-event release step (closed right boundary)
    int64_t eb_rel = 0;                // released prefix (buffer index)
    int64_t eb_floor = 0;              // smallest buffer index a future window can start at
    // The arrival column is implicit (arrival(i) = eb_arr0 + i, nothing stored) while the buffer is filled only by
    // in-order appends of consecutive arrivals; an out-of-order merge, shard mode or a state restore materialises it.
    bool eb_arr_impl = true;
    int64_t eb_arr0 = 0;
    const int64_t* arr_ptr() const { return eb_arr_impl ? nullptr : (const int64_t*)eb.arr.p; }
    int arr_materialize() {
        if (!eb_arr_impl) return 0;
        if (int rc = ensure(eb.arr, (size_t)std::max<int64_t>(eb.cap, 1) * 8)) return rc;
        if (eb.n > 0) {
            const int g = (int)std::min<int64_t>(4096, (eb.n + 255) / 256);
            hipLaunchKernelGGL(k_iota64, dim3(g), dim3(256), 0, stream, (int64_t*)eb.arr.p, eb_arr0, eb.n);
        }
        eb_arr_impl = false;
        return 0;
    }
    int64_t sW = -1;                   // arrival index at which the watermark reached W
    int64_t range_wins = 0;            // windows triggered so far
    // sliding windows with delay: queued triggers (event_window_trigger.go:129-135,156-161)
    struct DelayTrig { int64_t pos_abs, ts, w_rel; };
    std::vector<DelayTrig> delayq;
    size_t delayq_head = 0;
    // session windows: host mirror of the released timestamps [h_rts_base, h_rts_base + size)
    std::vector<int64_t> h_rts;
    std::vector<int64_t> h_rwp;        // lateTolerance > 0: watermark just before each mirrored row's release step
    int64_t h_rts_base = 0;
    bool sess_last_ticked = false, sess_has_trigger = false;
    int64_t sess_trigger = 0;
    int64_t count_k = 1;               // COUNTWINDOW: next window index
    // STATEWINDOW (StateWindowOp.onBegin): a window is open from absolute stream position st_start_abs
    bool st_on = false;
    int64_t st_start_abs = 0;
    // incremental-aggregation windows (window_inc_agg_event_op.go:26-146): NextTriggerWindowTime and the
    // windows opened by rows but not emitted yet (creation order == end order)
    bool inc = false;
    bool inc_has_T = false;
    int64_t inc_T = 0;
    struct IncWin { int64_t start, end, floor_abs; };
    std::vector<IncWin> inc_pend;
    DevBuf rq_d, ab_d, slot_d, trig_d, flags_d, cnts_d, runmax_d, runcm_d, mrg_keys[2], mrg_src[2], mrg_tmp, mrg_tail,
        mrg_bidx, mrg_col, vp_err, vp_mc, vp_mh, sort_pbase, sort_scr, chunk_pa;
    std::vector<int64_t> h_ab;
    DevBuf sw_d;                        // small-window launch lists
    bool small_win_on = true;           // EKGPU_SMALL_WIN=0: every range window through k_part + k_agg
    int stats_blocks = 1024;            // k_stats grid (EKGPU_STATS_BLOCKS)
    int variant = 0;                    // layout variants under measurement (EKGPU_VARIANT bits)
    bool agg_small = true;              // EKGPU_AGG_SMALL=0: k_agg keeps 8 rows per lane for small partitions too

    size_t col_es(int c) const { return plan.column_type[c] == EK_COL_U32 ? 4 : 8; }

    DBatch buffer_view() const {
        DBatch d{};
        d.n = eb.n;
        for (int c = 0; c < plan.n_columns; ++c) {
            d.col[c] = eb.col[c].p;
            d.valid[c] = eb_valid_on[c] ? (const uint8_t*)eb.valid[c].p : nullptr;
        }
        if (rowpos_col >= 0) d.col[rowpos_col] = rowpos.p;
        return d;
    }

    // Make room for `add` more rows: drop the consumed prefix [0, eb_floor) and/or grow (double buffer).
    int eb_reserve(int64_t add) {
        const int64_t drop = std::max<int64_t>(0, std::min(eb_floor, eb.n));
        const bool compact = drop > 0 && (drop >= (eb.n >> 1) || eb.n + add > eb.cap);
        if (eb.n + add <= eb.cap && !compact) return 0;
        const int64_t live = eb.n - (compact ? drop : 0);
        int64_t cap = eb.cap;
        if (live + add > cap) cap = std::max<int64_t>(2 * (live + add), (int64_t)1 << 16);
        const int64_t d = compact ? drop : 0;
        auto mv = [&](DevBuf& dst, DevBuf& src, size_t es) -> int {
            if (dst.bytes < (size_t)cap * es) {
                release(dst);
                if (int rc = ensure(dst, (size_t)cap * es)) return rc;
            }
            if (src.p && live) hipMemcpyAsync(dst.p, (char*)src.p + d * es, (size_t)live * es, hipMemcpyDeviceToDevice, stream);
            return 0;
        };
        for (int c = 0; c < plan.n_columns; ++c) {
            if (int rc = mv(eb_alt.col[c], eb.col[c], col_es(c))) return rc;
            if (eb_valid_on[c]) if (int rc = mv(eb_alt.valid[c], eb.valid[c], 1)) return rc;
        }
        if (!eb_arr_impl) if (int rc = mv(eb_alt.arr, eb.arr, 8)) return rc;
        if (need_rel) if (int rc = mv(eb_alt.rel, eb.rel, 8)) return rc;
        std::swap(eb, eb_alt);
        if (eb_arr_impl) eb_arr0 += d;
        eb.cap = cap;
        eb.n = live;
        eb_alt.n = 0;
        eb_base += d;
        eb_rel -= d;
        eb_floor -= d;
        return 0;
    }

    void fill_valid_ones(int c, int64_t from, int64_t cnt) {
        if (cnt > 0) hipMemsetAsync((uint8_t*)eb.valid[c].p + from, 1, (size_t)cnt, stream);
    }
    // a batch brings validity for column c the buffer has not carried so far: all earlier rows are valid
    int eb_enable_valid(int c) {
        if (eb_valid_on[c]) return 0;
        if (int rc = ensure(eb.valid[c], (size_t)std::max<int64_t>(eb.cap, 1))) return rc;
        fill_valid_ones(c, 0, eb.n);
        eb_valid_on[c] = true;
        return 0;
    }

    // Append rows [start, start + cnt) of a batch (already in buffer order) to the buffer.
    int eb_append(const DBatch& db, int64_t start, int64_t cnt, int64_t arr_base) {
        for (int c = 0; c < plan.n_columns; ++c)
            if (db.valid[c]) if (int rc = eb_enable_valid(c)) return rc;
        if (int rc = eb_reserve(cnt)) return rc;
        // every copied column (and validity, and shard-mode arrivals) in one k_eb_copy launch
        CopySegs cs{};
        int ns = 0;
        auto seg = [&](const void* src, void* dst, int64_t bytes, int es) {
            if (bytes > 0) cs.s[ns++] = CopySeg{(const unsigned char*)src, (unsigned char*)dst, bytes, es, 0};
        };
        for (int c = 0; c < plan.n_columns; ++c) {
            const size_t es = col_es(c);
            if (eb_need[c]) seg((const char*)db.col[c] + start * es, (char*)eb.col[c].p + eb.n * es, cnt * (int64_t)es, (int)es);
            if (eb_valid_on[c]) {
                if (db.valid[c]) seg(db.valid[c] + start, (uint8_t*)eb.valid[c].p + eb.n, cnt, 1);
                else fill_valid_ones(c, eb.n, cnt);
            }
        }
        if (g_row_arr) {   // shard mode: the rows' global arrival indices
            if (int rc = arr_materialize()) return rc;
            seg(g_row_arr + start, (int64_t*)eb.arr.p + eb.n, cnt * 8, 8);
        }
        if (ns > 0) {
            int64_t mx = 0;
            for (int k = 0; k < ns; ++k) mx = std::max(mx, cs.s[k].bytes);
            const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (mx + 16 * 256 * 4 - 1) / (16 * 256 * 4)));
            hipLaunchKernelGGL(k_eb_copy, dim3(gx, (unsigned)ns), dim3(256), 0, stream, cs);
        }
        if (g_row_arr) {
            // (shard mode: the global arrivals were copied above)
        } else if (eb_arr_impl && (eb.n == 0 || arr_base + start == eb_arr0 + eb.n)) {
            if (eb.n == 0) eb_arr0 = arr_base + start;   // consecutive arrivals: the column stays implicit
        } else {
            if (int rc = arr_materialize()) return rc;
            const int g = (int)std::min<int64_t>(4096, (cnt + 255) / 256);
            hipLaunchKernelGGL(k_iota64, dim3(std::max(g, 1)), dim3(256), 0, stream, (int64_t*)eb.arr.p + eb.n, arr_base + start, cnt);
        }
        if (need_rel) hipMemsetAsync((int64_t*)eb.rel.p + eb.n, 0x7f, (size_t)cnt * 8, stream);   // "not released"
        eb.n += cnt;
        return 0;
    }

    // Merge the accepted rows of an out-of-order batch (or one that starts below the buffer's tail) into the
    // ts-ordered buffer: the buffer rows with ts >= min_acc and the new rows are stably sorted by ts
    // (buffer rows first on ties, then arrival order = watermark_op.go:158-168 insertion "after equal").
    int eb_merge(const DBatch& db, int64_t start, const uint8_t* d_acc, int64_t n_acc, int64_t min_acc, int64_t max_acc,
                 int64_t arr_base) {
        const int64_t n = db.n;
        const int tsc = dp.ts_col;
        for (int c = 0; c < plan.n_columns; ++c)
            if (db.valid[c]) if (int rc = eb_enable_valid(c)) return rc;
        if (int rc = eb_reserve(n_acc)) return rc;
        if (int rc = arr_materialize()) return rc;
        // accepted row indices of the batch, in arrival order
        if (int rc = ensure(mrg_bidx, (size_t)std::max<int64_t>(n, 1) * 8)) return rc;
        int64_t* bidx = (int64_t*)mrg_bidx.p;
        if (d_acc) {
            const int nb = (int)((n + kCompactTile - 1) / kCompactTile);
            if (int rc = ensure(cnts_d, (size_t)(nb + 1) * 8)) return rc;
            hipLaunchKernelGGL(k_flag_count, dim3(nb), dim3(kBlock), 0, stream, d_acc, n, (int64_t*)cnts_d.p);
            hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, stream, (int64_t*)cnts_d.p, nb);
            hipLaunchKernelGGL(k_flag_write, dim3(nb), dim3(kBlock), 0, stream, d_acc, n, (const int64_t*)cnts_d.p, (int64_t)0, bidx);
        } else {
            const int g = (int)std::min<int64_t>(4096, (n_acc + 255) / 256);
            hipLaunchKernelGGL(k_iota64, dim3(std::max(g, 1)), dim3(256), 0, stream, bidx, start, n_acc);
        }
        // tail of the buffer that interleaves with the batch
        if (int rc = ensure(bounds_val, 8)) return rc;
        if (int rc = ensure(bounds_idx, 8)) return rc;
        hipMemcpyAsync(bounds_val.p, &min_acc, 8, hipMemcpyHostToDevice, stream);
        hipLaunchKernelGGL(k_lower_bound, dim3(1), dim3(64), 0, stream, (const int64_t*)eb.col[tsc].p, (int64_t)0, eb.n,
                           (const int64_t*)bounds_val.p, 1, (int64_t*)bounds_idx.p);
        int64_t p = 0;
        hipMemcpyAsync(&p, bounds_idx.p, 8, hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "merge bound failed");
        const int64_t ntail = eb.n - p, nm = ntail + n_acc;
        // saved tail (every column + arrivals + release steps), 8-byte slots
        const int nsv = plan.n_columns + 1 + (need_rel ? 1 : 0);
        if (int rc = ensure(mrg_tail, (size_t)std::max<int64_t>(ntail, 1) * 8 * (nsv + plan.n_columns))) return rc;
        auto tail_slot = [&](int k) { return (char*)mrg_tail.p + (size_t)k * std::max<int64_t>(ntail, 1) * 8; };
        for (int c = 0; c < plan.n_columns; ++c) {
            hipMemcpyAsync(tail_slot(c), (char*)eb.col[c].p + p * col_es(c), (size_t)ntail * col_es(c), hipMemcpyDeviceToDevice, stream);
            if (eb_valid_on[c]) hipMemcpyAsync(tail_slot(nsv + c), (uint8_t*)eb.valid[c].p + p, (size_t)ntail, hipMemcpyDeviceToDevice, stream);
        }
        hipMemcpyAsync(tail_slot(plan.n_columns), (int64_t*)eb.arr.p + p, (size_t)ntail * 8, hipMemcpyDeviceToDevice, stream);
        if (need_rel) hipMemcpyAsync(tail_slot(plan.n_columns + 1), (int64_t*)eb.rel.p + p, (size_t)ntail * 8, hipMemcpyDeviceToDevice, stream);
        // sort keys = ts - min_acc (the tail starts at ts >= min_acc), stable
        for (int k = 0; k < 2; ++k) {
            if (int rc = ensure(mrg_keys[k], (size_t)nm * 8)) return rc;
            if (int rc = ensure(mrg_src[k], (size_t)nm * 8)) return rc;
        }
        const int g = (int)std::min<int64_t>(8192, (nm + 255) / 256);
        hipLaunchKernelGGL(k_merge_keys, dim3(g), dim3(256), 0, stream, (const int64_t*)tail_slot(tsc), ntail,
                           (const int64_t*)db.col[tsc], (const int64_t*)bidx, n_acc, min_acc, (uint64_t*)mrg_keys[0].p,
                           (int64_t*)mrg_src[0].p);
        int64_t hi_ts = std::max(max_acc, M);
        uint64_t range = (uint64_t)(hi_ts - min_acc);
        int end_bit = 1;
        while (end_bit < 64 && (range >> end_bit)) end_bit++;
        size_t tb = 0;
        ekl_sort_pairs_u64(nullptr, &tb, nullptr, nullptr, nullptr, nullptr, nm, end_bit, stream);
        if (int rc = ensure(mrg_tmp, tb + 256)) return rc;
        tb = mrg_tmp.bytes;
        if (ekl_sort_pairs_u64(mrg_tmp.p, &tb, (const uint64_t*)mrg_keys[0].p, (uint64_t*)mrg_keys[1].p,
                               (const int64_t*)mrg_src[0].p, (int64_t*)mrg_src[1].p, nm, end_bit, stream))
            return fail(EK_ERR_DEVICE, "radix sort failed");
        const int64_t* perm = (const int64_t*)mrg_src[1].p;
        for (int c = 0; c < plan.n_columns; ++c) {
            if (col_es(c) == 4)
                hipLaunchKernelGGL(k_gather4, dim3(g), dim3(256), 0, stream, perm, nm, ntail, (const uint32_t*)tail_slot(c),
                                   (const uint32_t*)db.col[c], (const int64_t*)bidx, (uint32_t*)eb.col[c].p + p);
            else
                hipLaunchKernelGGL(k_gather8, dim3(g), dim3(256), 0, stream, perm, nm, ntail, (const int64_t*)tail_slot(c),
                                   (const int64_t*)db.col[c], (const int64_t*)bidx, (int64_t*)eb.col[c].p + p);
            if (eb_valid_on[c])
                hipLaunchKernelGGL(k_gather1, dim3(g), dim3(256), 0, stream, perm, nm, ntail, (const uint8_t*)tail_slot(nsv + c),
                                   db.valid[c], (const int64_t*)bidx, (uint8_t*)eb.valid[c].p + p);
        }
        // arrivals of the batch rows: arr_base + row
        if (int rc = ensure(mrg_col, (size_t)std::max<int64_t>(n, 1) * 8)) return rc;
        if (g_row_arr)
            hipMemcpyAsync(mrg_col.p, g_row_arr, (size_t)n * 8, hipMemcpyDeviceToDevice, stream);
        else
            hipLaunchKernelGGL(k_iota64, dim3((int)std::min<int64_t>(4096, (n + 255) / 256)), dim3(256), 0, stream,
                               (int64_t*)mrg_col.p, arr_base, n);
        hipLaunchKernelGGL(k_gather8, dim3(g), dim3(256), 0, stream, perm, nm, ntail, (const int64_t*)tail_slot(plan.n_columns),
                           (const int64_t*)mrg_col.p, (const int64_t*)bidx, (int64_t*)eb.arr.p + p);
        if (need_rel) {
            hipMemsetAsync(mrg_col.p, 0x7f, (size_t)n * 8, stream);
            hipLaunchKernelGGL(k_gather8, dim3(g), dim3(256), 0, stream, perm, nm, ntail,
                               (const int64_t*)tail_slot(plan.n_columns + 1), (const int64_t*)mrg_col.p,
                               (const int64_t*)bidx, (int64_t*)eb.rel.p + p);
        }
        eb.n = p + nm;
        return 0;
    }

    // Per-event running max of the batch (arrival order) -> runmax_d
    int batch_runmax(const int64_t* ts, int64_t n, int64_t seed) {
        int nch = (int)((n + kAccChunk - 1) / kAccChunk);
        if (int rc = ensure(runcm_d, (size_t)nch * 8)) return rc;
        if (int rc = ensure(runmax_d, (size_t)n * 8)) return rc;
        hipLaunchKernelGGL(k_chunk_max, dim3(nch), dim3(kBlock), 0, stream, ts, n, (int64_t*)runcm_d.p);
        hipLaunchKernelGGL(k_scan_max, dim3(1), dim3(1024), 0, stream, (int64_t*)runcm_d.p, nch, seed);
        hipLaunchKernelGGL(k_runmax, dim3(nch), dim3(kBlock), 0, stream, ts, n, (const int64_t*)runcm_d.p, (int64_t*)runmax_d.p);
        runmax_p = (const int64_t*)runmax_d.p;
        return 0;
    }
    // the running max of the current batch (arrival order): runmax_d, or the batch's own ts column when the batch is
    // ts-sorted and starts at or above the carried max (then runmax[i] == ts[i]: no kernels, no copy)
    const int64_t* runmax_p = nullptr;

    // one scalar device -> host (synchronous)
    int64_t* h_scalar = nullptr;   // pinned landing word (a pageable 8-byte copy costs tens of µs of staging)
    int64_t fetch_i64(const void* dptr) {
        if (!h_scalar && hipHostMalloc((void**)&h_scalar, 64) != hipSuccess) h_scalar = nullptr;
        int64_t v = 0;
        hipMemcpyAsync(h_scalar ? (void*)h_scalar : (void*)&v, dptr, 8, hipMemcpyDeviceToHost, stream);
        hipStreamSynchronize(stream);
        if (h_scalar) v = *h_scalar;
        return v;
    }

    // A triggered window before its range is resolved
    struct PendWin { RangeQ q; int64_t start, end; };
    bool hop_discard_pending = false;   // fire_windows applies the hopping empty-window discard to this set

    // Resolve the ranges of `pw` on the device, register the windows, launch their aggregation.
    // k_small_win over nb windows (persistent waves, one window at a time each; see ek_range.h), specialised by value
    // columns, WHERE and rows per lane
    int sw_grid = 4096;   // EKGPU_SW_GRID: waves of a k_small_win launch
    bool fin_ring = true;       // EKGPU_FIN_RING=0: hopping windows always through k_finalize
    int fin_ring_chunks = 0;    // EKGPU_FIN_RING_CHUNKS: window chunks of a k_finalize_ring launch (0: by the key blocks)
    int fin_ring_split = 0;     // EKGPU_FIN_RING_SPLIT=1: the split walk (count / sum, then min / max; measured slower on C3)
    DevBuf ring_gbase;          // split walk: each (window, key block)'s row base, written by part 1 and read by part 2
    // HS: HAVING absent or over count(*) alone (decided from dp.hstar_tab): the kernel carries no interpreter. When the
    // full candidate tables would cost more LDS than the bitmaps, the launch caps them (kSwCandCap rows) and a second
    // launch redoes the few windows with more candidates (their list and count stay on the device)
    DevBuf sw_redo;
    int sw_cap_on = 1;   // EKGPU_SW_CAP=0: one launch with the full tables
    int small_win_launch(int nb, const DBatch& src, const int64_t* ab, const int32_t* wl, const int32_t* slot,
                         const int64_t* ob, int max_n, SwArith ar) {
        const int nvc = std::max(1, dp.n_vc), rm = max_n <= 16 * kSwLanes ? 16 : kSwRows;
        const bool hs = dp.n_having == 0 || dp.having_star;
        const bool capped = sw_cap_on && sw_lds_bytes_capped(max_n) < sw_lds_bytes(max_n);
        SwRedo rd{};
        if (capped) {
            if (int rc = ensure(sw_redo, ((size_t)nb + 1) * 4)) return rc;
            rd.cap = kSwCandCap;
            rd.cnt = (int32_t*)sw_redo.p;
            rd.out = rd.cnt + 1;
            hipMemsetAsync(rd.cnt, 0, 4, stream);
        }
        ek::launch_small_win(nvc, dp.n_where > 0, rm, hs, std::min(nb, sw_grid), nb,
                             capped ? sw_lds_bytes_capped(max_n) : sw_lds_bytes(max_n), stream, d_plan, src, ab, wl, slot, ob,
                             results_view(), ar, rd);
        if (capped) {
            SwRedo r2{};
            r2.cnt = rd.cnt;
            r2.in = rd.out;
            ek::launch_small_win(nvc, dp.n_where > 0, rm, hs, std::min(nb, 256), nb, sw_lds_bytes(max_n), stream, d_plan, src, ab,
                                 wl, slot, ob, results_view(), ar, r2);
        }
        return 0;
    }

    int fire_windows(std::vector<PendWin>& pw) {
        const int nq = (int)pw.size();
        if (nq == 0) { hop_discard_pending = false; return 0; }
        if (int rc = ensure_rowpos(eb.n)) return rc;
        if (int rc = ensure(rq_d, (size_t)nq * sizeof(RangeQ))) return rc;
        if (int rc = ensure(ab_d, (size_t)nq * 16)) return rc;
        // descriptors in and ranges out through the pinned block (a pageable copy costs tens of µs of host staging)
        {
            RangeQ* hq = (RangeQ*)desc_alloc(((size_t)nq * sizeof(RangeQ) + 7) / 8);
            if (!hq) return fail(EK_ERR_NOMEM, "pinned");
            for (int w = 0; w < nq; ++w) hq[w] = pw[w].q;
            hipMemcpyAsync(rq_d.p, hq, (size_t)nq * sizeof(RangeQ), hipMemcpyHostToDevice, stream);
        }
        hipLaunchKernelGGL(k_window_ranges, dim3((nq + 255) / 256), dim3(256), 0, stream, (const int64_t*)eb.col[std::max(0, dp.ts_col)].p,
                           need_rel ? (const int64_t*)eb.rel.p : nullptr, arr_ptr(), eb_arr0, eb_rel, (const RangeQ*)rq_d.p, nq,
                           (int64_t*)ab_d.p);
        {
            int64_t* hab = desc_alloc((size_t)nq * 2);
            if (!hab) return fail(EK_ERR_NOMEM, "pinned");
            hipMemcpyAsync(hab, ab_d.p, (size_t)nq * 16, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "window range kernel failed");
            h_ab.assign(hab, hab + (size_t)nq * 2);
        }
        // every aggregation kernel below reads rows [a, b) of the buffer: check the ranges on the host first
        for (int w = 0; w < nq; ++w)
            if (h_ab[2 * w] < 0 || h_ab[2 * w] > h_ab[2 * w + 1] || h_ab[2 * w + 1] > eb.n)
                return fail(EK_ERR_STATE, "internal: window %d of %d has rows [%lld, %lld) outside the buffer [0, %lld) "
                                          "(kind %d, pos %lld, rstep %lld)", w, nq, (long long)h_ab[2 * w],
                            (long long)h_ab[2 * w + 1], (long long)eb.n, (int)pw[w].q.kind, (long long)pw[w].q.pos,
                            (long long)pw[w].q.rstep);
        if (hop_discard_pending) {
            hop_discard_pending = false;
            if (int rc = hopping_discard(pw)) return rc;
        }
        // register in trigger order; rows reserved = min(K, members)
        int64_t rows = 0;
        for (int w = 0; w < nq; ++w) rows += std::min<int64_t>(K, h_ab[2 * w + 1] - h_ab[2 * w]);
        // incremental windows none of whose rows joined them (opened by a row outside their range) are not reported; a
        // processing-time incremental window is broadcast even when no row joined it (emit, window_inc_agg_op.go:443-457)
        const auto skip = [&](int w) { return inc && !proc_inc && h_ab[2 * w + 1] == h_ab[2 * w]; };
        if (int rc = ensure_results(rows, nq)) return rc;
        std::vector<int32_t> slots(nq);
        std::vector<int64_t> obase(nq);
        for (int w = 0; w < nq; ++w) {
            if (skip(w)) { slots[w] = -1; obase[w] = -1; continue; }
            WinInfo wi{};
            wi.j = range_wins++;
            wi.start = pw[w].start;
            wi.end = pw[w].end;
            wi.out_base = r_rows_used;
            wi.slot = (int32_t)wins.size();
            wi.direct = true;
            r_rows_used += std::min<int64_t>(K, h_ab[2 * w + 1] - h_ab[2 * w]);
            wins.push_back(wi);
            slots[w] = wi.slot;
            obase[w] = wi.out_base;
        }
        for (int w = 0; w < nq; ++w) stats.windows_out += skip(w) ? 0 : 1;
        if (plan.debug_membership) {
            if (int rc = ensure(slot_d, (size_t)nq * 4)) return rc;
            if (int rc = up_pinned(slot_d.p, slots.data(), (size_t)nq)) return rc;
            hipLaunchKernelGGL(k_range_members, dim3(nq), dim3(kBlock), 0, stream, arr_ptr(),
                               (const int64_t*)ab_d.p, (const int32_t*)slot_d.p, (int64_t*)r_wmc.p,
                               (unsigned long long*)r_wmh.p, eb_arr_impl ? eb_arr0 : (int64_t)0);
        }
        // small windows: one workgroup each (k_small_win); no order statistics on that path
        std::vector<uint8_t> small(nq, 0);
        if (dp.n_sagg == 0 && small_win_on) {
            std::vector<int32_t> wl;
            for (int w = 0; w < nq; ++w) {
                const int64_t sz = h_ab[2 * w + 1] - h_ab[2 * w];
                if (slots[w] >= 0 && sz > 0 && sz <= kSmallWin) { small[w] = 1; wl.push_back(w); }
            }
            if (!wl.empty()) {
                const int nw = (int)wl.size();
                int max_n = 1;
                for (int w : wl) max_n = std::max<int>(max_n, (int)(h_ab[2 * w + 1] - h_ab[2 * w]));
                if (int rc = ensure(sw_d, (size_t)nw * 4 + (size_t)nq * 12 + 16)) return rc;
                int32_t* d_wl = (int32_t*)sw_d.p;
                int32_t* d_slot = d_wl + nw;
                int64_t* d_ob = (int64_t*)(((uintptr_t)(d_slot + nq) + 7) & ~(uintptr_t)7);
                if (int rc = up_pinned(d_wl, wl.data(), (size_t)nw)) return rc;
                if (int rc = up_pinned(d_slot, slots.data(), (size_t)nq)) return rc;
                if (int rc = up_pinned(d_ob, obase.data(), (size_t)nq)) return rc;
                const int ph = phase_begin(EK_PHASE_AGGREGATE);
                if (int rc = small_win_launch(nw, buffer_view(), (const int64_t*)ab_d.p, d_wl, d_slot, d_ob, max_n, SwArith{})) return rc;
                phase_end(ph);
            }
        }
        // key-major aggregation of the other windows when the cost rule picks it (ek_keymajor.h)
        {
            std::vector<int> rest;
            for (int w = 0; w < nq; ++w)
                if (!small[w] && slots[w] >= 0 && h_ab[2 * w + 1] > h_ab[2 * w]) rest.push_back(w);
            if (!rest.empty())
                if (int rc = km_try(rest, obase, slots, small)) return rc;   // marks the windows it aggregated
        }
        // virtual-pane groups of consecutive non-empty windows
        const int64_t vcap = (int64_t)env_int("EKGPU_RANGE_GROUP_EVENTS", 1 << 26);
        int w = 0;
        while (w < nq) {
            std::vector<int> members;
            int64_t V = 0;
            while (w < nq && (int)members.size() < max_panes_group) {
                const int64_t sz = h_ab[2 * w + 1] - h_ab[2 * w];
                if (sz == 0 || small[w]) { w++; continue; }   // empty window: no output (aggregate_operator.go:66-75)
                if (!members.empty() && V + sz > vcap) break;
                members.push_back(w);
                V += sz;
                w++;
            }
            if (members.empty()) continue;
            if (int rc = run_vgroup(members, V, obase, slots)) return rc;
        }
        if (dp.n_first > 0)
            if (int rc = first_fetch(slots, obase)) return rc;
        if (inc_where)
            if (int rc = inc_where_pass(slots, obase)) return rc;
        // windows never start below the last fired one's start (overlapping) or end (disjoint); send-twice windows do
        // not fire in start order (a timer's (t, t + D] precedes the next trigger's (t' - L, t']): proc_slide_delayed
        // and proc_slide_floor keep their floor
        const bool overlap = wtype == EK_WINDOW_SLIDING || wtype == EK_WINDOW_HOPPING || wtype == EK_WINDOW_COUNT;
        if (!send_twice) eb_floor = std::max(eb_floor, overlap ? h_ab[2 * (nq - 1)] : h_ab[2 * (nq - 1) + 1]);
        if (hop_floor >= 0) { eb_floor = std::max(eb_floor, hop_floor); hop_floor = -1; }
        return 0;
    }

    // Hopping windows fired by this push, in order (handleInputs, window_op.go:605-655): a window's content starts at
    // the inputs the previous window kept (nextleft = its first member); a window with no member drops EVERY input
    // present at the WatermarkTuple that fired it, so the next windows start past the rows released by then.
    int hopping_discard(const std::vector<PendWin>& pw) {
        const int nq = (int)pw.size();
        std::vector<int64_t> ends(nq), pre(nq);
        for (int w = 0; w < nq; ++w) ends[w] = pw[w].end;
        if (int rc = ensure(mrg_col, (size_t)nq * 16)) return rc;
        int64_t* d_ends = (int64_t*)mrg_col.p;
        hipMemcpyAsync(d_ends, ends.data(), (size_t)nq * 8, hipMemcpyHostToDevice, stream);
        hipLaunchKernelGGL(k_fire_prefix, dim3((nq + 255) / 256), dim3(256), 0, stream, runmax_p, cur_nb,
                           cur_arr_base, plan.late_tolerance_ms, (const int64_t*)eb.col[dp.ts_col].p, arr_ptr(), eb_arr0,
                           eb.n, d_ends, nq, d_ends + nq);
        hipMemcpyAsync(pre.data(), d_ends + nq, (size_t)nq * 8, hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "fire prefix kernel failed");
        int64_t floor = eb_floor;
        for (int w = 0; w < nq; ++w) {
            const int64_t a = std::max(h_ab[2 * w], floor), b = h_ab[2 * w + 1];
            if (a >= b) {
                // inputs released by the firing tuple beyond this window are dropped with it
                stats.records_discarded += std::max<int64_t>(0, pre[w] - std::max(a, b));
                h_ab[2 * w] = h_ab[2 * w + 1] = a;
                floor = std::max(floor, pre[w]);
            } else {
                h_ab[2 * w] = a;
                floor = a;
            }
        }
        hop_floor = floor;
        hipMemcpyAsync(ab_d.p, h_ab.data(), (size_t)nq * 16, hipMemcpyHostToDevice, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "window range upload failed");
        return 0;
    }
    int64_t hop_floor = -1;

    // ---- key-major aggregation (ek_keymajor.h): the span of a run of fired windows is sorted once by key and one
    // thread per key walks the windows. Picked (EKGPU_KEYMAJOR=2, default) for big key spaces when the windows overlap
    // heavily (each event re-aggregated >= 4 times by the window-major path) or need order statistics over short
    // per-key runs; 1 = whenever eligible, 0 = never. Ineligible: no GROUP BY, non-monotone window ranges, WHERE
    // errors in the span (attributed per window by the window-major path), order statistics over a (key, window)
    // run longer than kKmSegMax. The windows it aggregates are marked in `done`.
    int km_mode = 2;
    DevBuf km_k[2], km_p[2], km_tmp, km_start, km_val[kMaxVC], km_ok[kMaxVC], km_ab, km_bcnt, km_flag;
    unsigned int* h_kmf = nullptr;     // pinned: WHERE errors, longest key run, long order-statistic run, scratch
    std::vector<int64_t> km_hab;

    int km_try(const std::vector<int>& rest, const std::vector<int64_t>& obase, const std::vector<int32_t>& slots,
               std::vector<uint8_t>& done) {
        if (km_mode == 0 || dp.key_col < 0 || dp.pseudo_keys || K < 2) return 0;
        for (size_t i = 1; i < rest.size(); ++i)
            if (h_ab[2 * rest[i]] < h_ab[2 * rest[i - 1]] || h_ab[2 * rest[i] + 1] < h_ab[2 * rest[i - 1] + 1]) return 0;
        for (size_t c0 = 0; c0 < rest.size(); c0 += kKmMaxWin) {
            const size_t c1 = std::min(rest.size(), c0 + (size_t)kKmMaxWin);
            std::vector<int> wl(rest.begin() + c0, rest.begin() + c1);
            bool ok = false;
            if (int rc = km_run(wl, obase, slots, &ok)) return rc;
            if (ok) for (int w : wl) done[w] = 1;
        }
        return 0;
    }

    int km_one = 1;   // EKGPU_KM_ONE=0: one-window launches take the count + scan + write passes too
    int km_packed = 1;   // EKGPU_KM_PACKED=0: the write pass stores the result columns directly
    int count_direct = 1;   // EKGPU_COUNT_DIRECT=0: every COUNTWINDOW row goes through the event buffer
    int km_states = 1;   // EKGPU_KM_STATES=0: multi-window launches emit one record per (state, window) (k_km_unpack)
    int km_single = 1;   // EKGPU_KM_SINGLE=0: state emission keeps the count pass (states sorted as they are stored)
    int km_merge_sort = 1;   // EKGPU_KM_MERGE_SORT=0: order-statistic launches walk by binary search over the window bounds
    DevBuf km_rbase, km_rec, km_skend, km_urec, km_ukend, km_scount, km_ex;
    int grp_on = 1;   // EKGPU_GRP=0: one-window launches over huge key spaces use the radix-sorted key-major walk
    DevBuf grp_tiles, grp_cnt, grp_base;

    // ek_keymajor.h k_grp_*: two MSD partition passes (8-bit digits of the key) into sub-buckets of 2^s2 keys,
    // then one workgroup per sub-bucket groups its rows by key in LDS and emits. *ok = false: a sub-bucket holds
    // more rows than kGrpCap (skewed keys) -> the caller's radix-sorted path (nothing was written).
    int grp_run(const DBatch& bv, int64_t lo, int64_t n, int32_t wslot, int64_t wobase, bool sort, bool* ok) {
        *ok = false;
        int kb = 17;
        while ((1ull << kb) < (uint64_t)K) kb++;
        const int s1 = kb - 8, s2 = s1 - 8;
        const int nb1 = (int)(((uint64_t)K - 1) >> s1) + 1, nsub = nb1 * 256;
        const uint32_t* key0 = (const uint32_t*)bv.col[dp.key_col] + lo;
        const int64_t* val0 = (const int64_t*)bv.col[dp.vc_col[0]] + lo;
        for (int i = 0; i < 2; ++i) {
            if (int rc = ensure(km_k[i], (size_t)n * 4)) return rc;
            if (int rc = ensure(km_val[i], (size_t)n * 8)) return rc;
        }
        const int64_t nt1 = (n + kGrpTile - 1) / kGrpTile;
        if (int rc = ensure(grp_tiles, (size_t)(nt1 + nt1 + 256) * sizeof(GrpTile))) return rc;
        constexpr int kRep1 = 64;   // counter replicas of the first pass (k_grp_hist)
        const int n1 = kRep1 * 256;
        if (int rc = ensure(grp_cnt, (size_t)(n1 + nsub) * 2 * 4)) return rc;
        if (int rc = ensure(grp_base, (size_t)(n1 + nsub + 1) * 8)) return rc;
        GrpTile* d_t1 = (GrpTile*)grp_tiles.p;
        GrpTile* d_t2 = d_t1 + nt1;
        unsigned int* tot1 = (unsigned int*)grp_cnt.p;
        unsigned int* cur1 = tot1 + n1;
        unsigned int* tot2 = cur1 + n1;
        unsigned int* cur2 = tot2 + nsub;
        int64_t* base1 = (int64_t*)grp_base.p;
        int64_t* base2 = base1 + n1;
        // offsets and pass-2 tiles planned on the device (k_msd_plan1 / k_msd_plan2, as km_msd): one host round trip,
        // after the second scatter, for the largest sub-bucket (register depth of the walk, or the fallback)
        if (int rc = ensure(km_flag, 64)) return rc;
        if (!h_kmf && hipHostMalloc((void**)&h_kmf, 32) != hipSuccess) { h_kmf = nullptr; return fail(EK_ERR_NOMEM, "pinned"); }
        unsigned int* d_flag = (unsigned int*)km_flag.p;
        if (msd_ht_n != n) {   // pass 1's tiles: the span in kGrpTile pieces (pinned, shared with km_msd)
            if (msd_ht_cap < (size_t)nt1) {
                if (msd_ht) { hipStreamSynchronize(stream); hipHostFree(msd_ht); }
                msd_ht_cap = (size_t)nt1;
                if (hipHostMalloc((void**)&msd_ht, msd_ht_cap * sizeof(GrpTile)) != hipSuccess) { msd_ht = nullptr; msd_ht_cap = 0; return fail(EK_ERR_NOMEM, "pinned"); }
            } else {
                hipStreamSynchronize(stream);   // the previous launch's copy has completed
            }
            for (int64_t t = 0; t < nt1; ++t)
                msd_ht[t] = GrpTile{t * kGrpTile, (int32_t)std::min<int64_t>(kGrpTile, n - t * kGrpTile), 0};
            msd_ht_n = n;
        }
        const int64_t nt2c = nt1 + 256;
        hipMemcpyAsync(d_t1, msd_ht, (size_t)nt1 * sizeof(GrpTile), hipMemcpyHostToDevice, stream);
        hipMemsetAsync(grp_cnt.p, 0, (size_t)(2 * n1 + 2 * nsub) * 4, stream);
        hipMemsetAsync(d_flag, 0, 64, stream);
        const int ph = phase_begin(EK_PHASE_PARTITION);
        hipLaunchKernelGGL(k_grp_hist, dim3((unsigned)nt1), dim3(kGrpBlock), 0, stream, key0, (const GrpTile*)d_t1, s1, 255u, K,
                           kRep1, tot1);
        hipLaunchKernelGGL(k_msd_plan1, dim3(1), dim3(1024), 0, stream, (const unsigned int*)tot1, kRep1, 8, (int)nt2c, base1, d_t2);
        hipLaunchKernelGGL(k_grp_scatter<false>, dim3((unsigned)nt1), dim3(kGrpScatBlock), 0, stream, key0, val0, (const GrpTile*)d_t1, s1,
                           255u, K, kRep1, (const int64_t*)base1, cur1, (uint32_t*)km_k[0].p, (int64_t*)km_val[0].p, (const uint32_t*)nullptr,
                           (uint32_t*)nullptr);
        hipLaunchKernelGGL(k_grp_hist, dim3((unsigned)nt2c), dim3(kGrpBlock), 0, stream, (const uint32_t*)km_k[0].p,
                           (const GrpTile*)d_t2, s2, 255u, K, 1, tot2);
        hipLaunchKernelGGL(k_msd_plan2, dim3(1), dim3(1024), 0, stream, (const unsigned int*)tot2, nsub, base2, (unsigned int)kGrpCap,
                           d_flag + 4);
        hipLaunchKernelGGL(k_grp_scatter<false>, dim3((unsigned)nt2c), dim3(kGrpScatBlock), 0, stream, (const uint32_t*)km_k[0].p,
                           (const int64_t*)km_val[0].p, (const GrpTile*)d_t2, s2, 255u, K, 1, (const int64_t*)base2, cur2,
                           (uint32_t*)km_k[1].p, (int64_t*)km_val[1].p, (const uint32_t*)nullptr, (uint32_t*)nullptr);
        phase_end(ph);
        hipMemcpyAsync(h_kmf, d_flag, 32, hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "grouping partition failed");
        const unsigned int mx = h_kmf[5];
        if (h_kmf[4]) return 0;   // a sub-bucket above kGrpCap rows (skewed keys): the caller's path
        GrpDesc g{};
        g.base2 = base2;
        g.keys = (const uint32_t*)km_k[1].p;
        g.vals = (const int64_t*)km_val[1].p;
        g.s1 = s1;
        g.s2 = s2;
        g.obase = wobase;
        g.widx = wslot;
        const Results rv = results_view();
        const int ph2 = phase_begin(EK_PHASE_AGGREGATE);
        // register depth (and LDS slab) sized to the largest sub-bucket of this launch
        const int rdep = mx <= 8u * kGrpWalkBlock ? 8 : mx <= 12u * kGrpWalkBlock ? 12 : 16;
        const size_t gl = grp_walk_lds(s2, rdep);
        const dim3 gg((unsigned)nsub), gb(kGrpWalkBlock);
        const bool isf = dp.vc_is_float[0] != 0;
        ek::launch_grp_walk(sort, isf, rdep, dp.n_having > 0, gg, gb, gl, stream, d_plan, g, rv);
        phase_end(ph2);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "grouping walk failed");
        *ok = true;
        return 0;
    }
    // Key-major span sort by MSD partition (replaces the radix sort of (key, position) pairs and the value gather by
    // position): two k_grp_scatter<true> passes on 8-bit digits of the dense key carry (key, value, position) into
    // sub-buckets of 2^s2 keys, k_kmsd_fix sorts each sub-bucket by (key, position) in LDS and writes kstart and the
    // longest key run. Input: km_k[0] (k_km_keys: dropped rows carry key K). Output, sorted by (key, position):
    // keys km_k[0], positions km_p[1], values km_val[0]. *ok = false: a sub-bucket exceeds kGrpCap rows (skewed keys;
    // the caller takes the radix sort — its inputs must be rebuilt, km_k[0] is overwritten).
    int km_msd(const int64_t* val0, int64_t n, unsigned int* d_flag) {
        int kb = 17;
        while ((1ull << kb) < (uint64_t)K) kb++;
        // sub-buckets of 2^s2 keys holding ~1 000 rows (<= kKmFixCap with room for the spread): one k_kmsd_fix thread per
        // key (up to 256), one workgroup per sub-bucket; the second pass's digit is the s1 - s2 (<= 8) bits between
        const int s1 = kb - 8;
        int s2 = 8;
        while (s2 > 1 && ((double)n / (double)K) * (double)(1 << s2) > 1000.0) s2--;
        s2 = std::max(s2, s1 - 8);
        const int w2 = s1 - s2;
        const int nb1 = (int)(((uint64_t)K - 1) >> s1) + 1, nsub = nb1 << w2;
        for (int i = 0; i < 2; ++i) {
            if (int rc = ensure(km_k[i], (size_t)n * 4)) return rc;
            if (int rc = ensure(km_p[i], (size_t)n * 4)) return rc;
            if (int rc = ensure(km_val[i], (size_t)n * 8)) return rc;
        }
        const int64_t nt1 = (n + kGrpTile - 1) / kGrpTile;
        const int64_t nt2c = nt1 + 256;   // pass 2's tiles: at most one partial tile per digit beyond pass 1's count
        if (int rc = ensure(grp_tiles, (size_t)(nt1 + nt2c) * sizeof(GrpTile))) return rc;
        constexpr int kRep1 = 64;
        const int n1 = kRep1 * 256;
        if (int rc = ensure(grp_cnt, (size_t)(n1 + nsub) * 2 * 4)) return rc;
        if (int rc = ensure(grp_base, (size_t)(n1 + nsub + 1) * 8)) return rc;
        if (int rc = ensure(km_start, ((size_t)K + 2) * 4)) return rc;
        GrpTile* d_t1 = (GrpTile*)grp_tiles.p;
        GrpTile* d_t2 = d_t1 + nt1;
        unsigned int* tot1 = (unsigned int*)grp_cnt.p;
        unsigned int* cur1 = tot1 + n1;
        unsigned int* tot2 = cur1 + n1;
        unsigned int* cur2 = tot2 + nsub;
        int64_t* base1 = (int64_t*)grp_base.p;
        int64_t* base2 = base1 + n1;
        const uint32_t* key0 = (const uint32_t*)km_k[0].p;
        if (msd_ht_n != n) {   // pass 1's tiles: the span in kGrpTile pieces (pinned: the copy is asynchronous)
            if (msd_ht_cap < (size_t)nt1) {
                if (msd_ht) { hipStreamSynchronize(stream); hipHostFree(msd_ht); }
                msd_ht_cap = (size_t)nt1;
                if (hipHostMalloc((void**)&msd_ht, msd_ht_cap * sizeof(GrpTile)) != hipSuccess) { msd_ht = nullptr; msd_ht_cap = 0; return fail(EK_ERR_NOMEM, "pinned"); }
            } else {
                hipStreamSynchronize(stream);   // the previous launch's copy has completed
            }
            for (int64_t t = 0; t < nt1; ++t)
                msd_ht[t] = GrpTile{t * kGrpTile, (int32_t)std::min<int64_t>(kGrpTile, n - t * kGrpTile), 0};
            msd_ht_n = n;
        }
        hipMemcpyAsync(d_t1, msd_ht, (size_t)nt1 * sizeof(GrpTile), hipMemcpyHostToDevice, stream);
        hipMemsetAsync(grp_cnt.p, 0, (size_t)(2 * n1 + 2 * nsub) * 4, stream);
        hipLaunchKernelGGL(k_grp_hist, dim3((unsigned)nt1), dim3(kGrpBlock), 0, stream, key0, (const GrpTile*)d_t1, s1, 255u, K, kRep1, tot1);
        hipLaunchKernelGGL(k_msd_plan1, dim3(1), dim3(1024), 0, stream, (const unsigned int*)tot1, kRep1, w2, (int)nt2c, base1, d_t2);
        hipLaunchKernelGGL(k_grp_scatter<true>, dim3((unsigned)nt1), dim3(kGrpScatBlock), 0, stream, key0, val0, (const GrpTile*)d_t1,
                           s1, 255u, K, kRep1, (const int64_t*)base1, cur1, (uint32_t*)km_k[1].p, (int64_t*)km_val[1].p,
                           (const uint32_t*)nullptr, (uint32_t*)km_p[0].p);
        const uint32_t m2 = (1u << w2) - 1u;
        hipLaunchKernelGGL(k_grp_hist, dim3((unsigned)nt2c), dim3(kGrpBlock), 0, stream, (const uint32_t*)km_k[1].p,
                           (const GrpTile*)d_t2, s2, m2, K, 1, tot2);
        // LDS per k_kmsd_fix workgroup sized for twice the mean sub-bucket (a sub-bucket beyond it: the radix-sort fallback)
        const double mean = (double)n / (double)nsub;
        const int cap = (int)std::min<double>(kKmFixCap, std::max(512.0, std::ceil(2.0 * mean / 256.0) * 256.0));
        hipLaunchKernelGGL(k_msd_plan2, dim3(1), dim3(1024), 0, stream, (const unsigned int*)tot2, nsub, base2, (unsigned int)cap,
                           d_flag + 4);
        hipLaunchKernelGGL(k_grp_scatter<true>, dim3((unsigned)nt2c), dim3(kGrpScatBlock), 0, stream, (const uint32_t*)km_k[1].p,
                           (const int64_t*)km_val[1].p, (const GrpTile*)d_t2, s2, m2, K, 1, (const int64_t*)base2, cur2,
                           (uint32_t*)km_k[0].p, (int64_t*)km_val[0].p, (const uint32_t*)km_p[0].p, (uint32_t*)km_p[1].p);
        const int nk = 1 << s2;
        const size_t flds = (((size_t)(2 * nk + 1) * 4 + 15) & ~(size_t)15) + (size_t)cap * 12 + 16;
        hipLaunchKernelGGL(k_kmsd_fix, dim3((unsigned)nsub), dim3(kKmFixBlock), flds, stream, (const int64_t*)base2, nsub, s2, K,
                           (const uint32_t*)km_k[0].p, (uint32_t*)km_p[1].p, (int64_t*)km_val[0].p, (uint32_t*)km_start.p,
                           d_flag + 1, cap);
        return 0;
    }
    GrpTile* msd_ht = nullptr;   // km_msd's pass-1 tiles (pinned, rebuilt when the span length changes)
    size_t msd_ht_cap = 0;
    int64_t msd_ht_n = -1;
    int km_msd_on = 1;   // EKGPU_KM_MSD=0: the key-major span sort is the radix sort + value gather

    int km_run(const std::vector<int>& wl, const std::vector<int64_t>& obase, const std::vector<int32_t>& slots,
               bool* handled) {
        *handled = false;
        const int nw = (int)wl.size();
        const int64_t lo = h_ab[2 * wl[0]], hi = h_ab[2 * wl.back() + 1];
        const int64_t n = hi - lo;
        if (n <= 0 || n >= (1LL << 31)) return 0;
        int64_t V = 0;
        for (int w : wl) V += h_ab[2 * w + 1] - h_ab[2 * w];
        const bool sort = dp.n_sagg > 0;
        const double overlap = (double)V / (double)n, rows_kw = (double)V / nw / (double)K;
        if (km_mode == 2 && !(K >= 16384 && (sort ? rows_kw <= 16.0 : overlap >= 4.0))) return 0;
        int end_bit = 1;
        while (end_bit < 32 && (1ull << end_bit) <= (uint64_t)K) end_bit++;
        const DBatch bv = buffer_view();
        // one window, one value column without validity, no WHERE, 2^16 < K <= 2^27: MSD-partitioned grouping
        if (nw == 1 && km_one && grp_on && dp.n_where == 0 && dp.n_vc == 1 && !bv.valid[dp.vc_col[0]] && K > 65536 &&
            K <= (1u << 27)) {
            bool ok = false;
            if (int rc = grp_run(bv, lo, n, slots[wl[0]], obase[wl[0]], sort, &ok)) return rc;
            if (ok) {
                stats.windows_keymajor += 1;
                *handled = true;
                return 0;
            }
        }
        // one window over the whole span: the walk needs no positions; with one value column (no validity) the
        // column itself is sorted by key (no position payload, no gather)
        const bool one = nw == 1 && km_one;
        if (int rc = ensure(km_flag, 64)) return rc;   // [0..3] flags, [8..15] EK_KM_CHECK report
        if (!h_kmf && hipHostMalloc((void**)&h_kmf, 32) != hipSuccess) { h_kmf = nullptr; return fail(EK_ERR_NOMEM, "pinned"); }
        unsigned int* d_flag = (unsigned int*)km_flag.p;
        const dim3 gk((unsigned)std::min<int64_t>(8192, (n + kBlock - 1) / kBlock));
        // the (key, position) order of the span's rows, with the value column carried along (km_msd) or gathered after
        // the radix sort
        bool msd = km_msd_on && dp.n_vc == 1 && !bv.valid[dp.vc_col[0]] && K >= 65536 && K <= (1u << 27) && (double)n <= 64.0 * K;
        int ph = -1;
        if (msd) {
            if (int rc = ensure(km_k[0], (size_t)n * 4)) return rc;
            hipMemsetAsync(d_flag, 0, 64, stream);
            ph = phase_begin(EK_PHASE_PARTITION);
            hipLaunchKernelGGL(k_km_keys, gk, dim3(kBlock), 0, stream, d_plan, bv, lo, n, (uint32_t*)km_k[0].p, (uint32_t*)nullptr, d_flag);
            if (int rc = km_msd((const int64_t*)bv.col[dp.vc_col[0]] + lo, n, d_flag)) return rc;
            phase_end(ph);
            hipMemcpyAsync(h_kmf, d_flag, 32, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "key partition failed");
            if (h_kmf[4]) msd = false;   // a sub-bucket above kKmFixCap rows (skewed keys): the radix sort below
        }
        const bool vsort = !msd && one && dp.n_vc == 1 && !bv.valid[dp.vc_col[0]];
        if (!msd) {
            size_t tb = 0;
            if (vsort) ekl_sort_pairs_u32_i64(nullptr, &tb, nullptr, nullptr, nullptr, nullptr, n, end_bit, stream);
            else ekl_sort_pairs_u32(nullptr, &tb, nullptr, nullptr, nullptr, nullptr, n, end_bit, stream);
            for (int i = 0; i < 2; ++i) {
                if (int rc = ensure(km_k[i], (size_t)n * 4)) return rc;
                if (!vsort)
                    if (int rc = ensure(km_p[i], (size_t)n * 4)) return rc;
            }
            if (vsort)
                if (int rc = ensure(km_val[0], (size_t)n * 8)) return rc;
            if (int rc = ensure(km_tmp, tb)) return rc;
            if (int rc = ensure(km_start, ((size_t)K + 2) * 4)) return rc;
            hipMemsetAsync(d_flag, 0, 64, stream);
            ph = phase_begin(EK_PHASE_PARTITION);
            hipLaunchKernelGGL(k_km_keys, gk, dim3(kBlock), 0, stream, d_plan, bv, lo, n, (uint32_t*)km_k[0].p,
                               vsort ? (uint32_t*)nullptr : (uint32_t*)km_p[0].p, d_flag);
            if (vsort) {
                if (ekl_sort_pairs_u32_i64(km_tmp.p, &tb, (const uint32_t*)km_k[0].p, (uint32_t*)km_k[1].p,
                                           (const int64_t*)bv.col[dp.vc_col[0]] + lo, (int64_t*)km_val[0].p, n, end_bit, stream))
                    return fail(EK_ERR_DEVICE, "key sort failed");
            } else if (ekl_sort_pairs_u32(km_tmp.p, &tb, (const uint32_t*)km_k[0].p, (uint32_t*)km_k[1].p, (const uint32_t*)km_p[0].p,
                                          (uint32_t*)km_p[1].p, n, end_bit, stream))
                return fail(EK_ERR_DEVICE, "key sort failed");
        }
        const uint32_t* sk = (const uint32_t*)km_k[msd ? 0 : 1].p;
        const uint32_t* spos = vsort ? nullptr : (const uint32_t*)km_p[1].p;
        uint32_t* kstart = (uint32_t*)km_start.p;
        if (!msd) {
            hipLaunchKernelGGL(k_km_starts, dim3((unsigned)std::min<int64_t>(8192, (n + 1 + 255) / 256)), dim3(256), 0, stream, sk, n,
                               K, kstart);
            hipLaunchKernelGGL(k_km_maxrun, dim3((unsigned)std::min<int64_t>(256, ((int64_t)K + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                               stream, (const uint32_t*)kstart, K, d_flag + 1);
            phase_end(ph);
            hipMemcpyAsync(h_kmf, d_flag, 32, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "key-major sort failed");
        }
        if (h_kmf[0] > 0) return 0;                                                       // WHERE errors
        if (km_mode == 2 && !sort && (double)h_kmf[1] * overlap > (double)(1 << 22)) return 0;   // one key dominates
        if (one && sort && h_kmf[1] > (unsigned)kKmSegMax) return 0;   // single pass: no (key, window) run too long
        // value columns in key order
        KmCols cols{};
        cols.no_vals = msd ? 1 : 0;   // km_msd carried the value column: the gather computes E / X only
        for (int v = 0; v < dp.n_vc; ++v) {
            if (int rc = ensure(km_val[v], (size_t)n * 8)) return rc;
            cols.val[v] = (int64_t*)km_val[v].p;
            if (bv.valid[dp.vc_col[v]]) {
                if (int rc = ensure(km_ok[v], (size_t)n)) return rc;
                cols.ok[v] = (uint8_t*)km_ok[v].p;
            }
        }
        const int nvc = std::max(1, dp.n_vc);
        const int nblk = (int)(((int64_t)K + kKmBlock - 1) / kKmBlock);
        if (int rc = ensure(km_ab, (size_t)nw * 28)) return rc;
        if (int rc = ensure(km_bcnt, (size_t)nw * (nblk + 1) * 4)) return rc;
        km_hab.resize((size_t)nw * 3);
        int64_t* h_rab = km_hab.data();
        int64_t* h_rob = h_rab + 2 * nw;
        for (int i = 0; i < nw; ++i) {
            h_rab[2 * i] = h_ab[2 * wl[i]] - lo;
            h_rab[2 * i + 1] = h_ab[2 * wl[i] + 1] - lo;
            h_rob[i] = obase[wl[i]];
        }
        std::vector<int32_t> h_wi(nw);
        for (int i = 0; i < nw; ++i) h_wi[i] = slots[wl[i]];
        int64_t* d_ab = (int64_t*)km_ab.p;
        int32_t* d_wi = (int32_t*)(d_ab + 3 * nw);
        if (int rc = up_pinned(d_ab, h_rab, (size_t)nw * 3)) return rc;
        if (int rc = up_pinned(d_wi, h_wi.data(), (size_t)nw)) return rc;
        KmDesc d{};
        d.n = n;
        d.nw = nw;
        d.nblk = nblk;
        d.nkeys = K;
        d.ab = d_ab;
        d.obase = d_ab + 2 * nw;
        d.widx = d_wi;
        d.kstart = kstart;
        d.spos = spos;
        for (int v = 0; v < kMaxVC; ++v) { d.sval[v] = cols.val[v]; d.sok[v] = cols.ok[v]; }
        d.bcnt = (uint32_t*)km_bcnt.p;
        d.flags = (int32_t*)(d_flag + 2);
#ifdef EK_KM_CHECK
        d.dbg = (int32_t*)(d_flag + 8);
        cols.dbg = d.dbg;
        d.dbg_mode = km_merge_sort == 3 ? 1 : 0;
#endif
        cols.n = n;
        const Results rv = results_view();
        // kept-row counters / cursors per window (+ the order-statistic lanes)
        const size_t lds = sort ? (size_t)((3 * nw + 1) & ~1) * 4 + (size_t)kKmSegMax * kKmBlock * 8 : (size_t)nw * 4;
        const int ph2 = phase_begin(EK_PHASE_AGGREGATE);
        const dim3 gg((unsigned)std::min<int64_t>(8192, (n + kBlock - 1) / kBlock));
        size_t glds = 0;
        if (!one && (!sort || km_merge_sort)) {   // multi-window walk by merge: each row's first window and first window past it
            if (int rc = ensure(km_ex, (size_t)n * 4)) return rc;
            cols.E = (uint16_t*)km_ex.p;
            cols.X = cols.E + n;
            cols.ab = d_ab;
            cols.nw = nw;
            if (!(sort && km_merge_sort == 2)) {   // 2 (diagnostic): E / X computed, the walk binary-searches
                d.sE = cols.E;
                d.sX = cols.X;
            }
            glds = (size_t)nw * 8;
        }
        if (!vsort && !(msd && !cols.E)) switch (nvc) {
        case 1: hipLaunchKernelGGL(k_km_gather<1>, gg, dim3(kBlock), glds, stream, d_plan, bv, lo, spos, (const uint32_t*)kstart, cols); break;
        case 2: hipLaunchKernelGGL(k_km_gather<2>, gg, dim3(kBlock), glds, stream, d_plan, bv, lo, spos, (const uint32_t*)kstart, cols); break;
        case 3: hipLaunchKernelGGL(k_km_gather<3>, gg, dim3(kBlock), glds, stream, d_plan, bv, lo, spos, (const uint32_t*)kstart, cols); break;
        default: hipLaunchKernelGGL(k_km_gather<4>, gg, dim3(kBlock), glds, stream, d_plan, bv, lo, spos, (const uint32_t*)kstart, cols); break;
        }
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return fail(EK_ERR_DEVICE, "key-major gather launch: %s", hipGetErrorName(e));
#ifdef EK_KM_CHECK
        if (hipError_t e = hipStreamSynchronize(stream); e != hipSuccess)
            return fail(EK_ERR_DEVICE, "key-major gather failed: %s", hipGetErrorName(e));
        if (int rc = km_check_report("gather")) return rc;
#endif
        // HAVING absent, or over count(*) alone with every key run (h_kmf[1], the longest) inside the decision table:
        // the walk decides each state from DPlan.hstar_tab and carries no interpreter
        const bool hs = !sort && (dp.n_having == 0 || (dp.having_star && h_kmf[1] < (unsigned)kHStarTab));
        auto walk = [&](bool write) { ek::launch_km_walk(nvc, sort, write, false, hs, nblk, lds, stream, d_plan, d, rv); };
        if (one) {
            ek::launch_km_walk(nvc, sort, true, true, hs, nblk, lds, stream, d_plan, d, rv);
            phase_end(ph2);
            if (hipGetLastError() != hipSuccess) return fail(EK_ERR_DEVICE, "key-major launch failed");
            stats.windows_keymajor += nw;
            *handled = true;
            return 0;
        }
        // state emission: each kept membership state stored once and fanned out to its windows by k_km_expand
        const bool states = km_packed && km_states && dp.n_aggs <= kKmRecAggs && nw > 1 && nw <= 65535;
        int R = 0;
        if (states) {
            // R = the most windows one buffer position belongs to (attained at some window start; a, b monotone)
            for (int i = 0; i < nw; ++i) {
                const int64_t x = h_rab[2 * i];
                int lo_j = 0, hi_j = i;   // first j <= i with b_j > x
                while (lo_j < hi_j) { const int mid = (lo_j + hi_j) >> 1; if (h_rab[2 * mid + 1] > x) hi_j = mid; else lo_j = mid + 1; }
                int a_lo = i + 1, a_hi = nw;   // first j > i with a_j > x
                while (a_lo < a_hi) { const int mid = (a_lo + a_hi) >> 1; if (h_rab[2 * mid] > x) a_hi = mid; else a_lo = mid + 1; }
                R = std::max(R, a_lo - lo_j);
            }
            if (int rc = ensure(km_skend, 64)) return rc;
            d.skend = (uint16_t*)km_skend.p;   // the count pass only tests it
        }
        // single pass (no order statistics, so nothing can send the launch back to the window-major path after the
        // walk): the walk stores its states unsorted per block and counts them, k_km_sscatter sorts them by bucket
        const bool single = states && !sort && km_single && (double)n * 2.0 * 36.0 <= 8e9;
        if (single) {
            if (int rc = ensure(km_urec, (size_t)n * 2 * 32)) return rc;
            if (int rc = ensure(km_ukend, (size_t)n * 2 * 2 * 2)) return rc;
            if (int rc = ensure(km_scount, (size_t)nblk * 4)) return rc;
            KmDesc du = d;
            du.rec = (uint4*)km_urec.p;
            du.skend = (uint16_t*)km_ukend.p;
            du.sk = du.skend + (size_t)n * 2;
            du.scount = (uint32_t*)km_scount.p;
            ek::launch_km_walk(nvc, sort, true, false, hs, nblk, lds, stream, d_plan, du, rv);
            hipLaunchKernelGGL(k_km_scan, dim3(nw), dim3(1024), 0, stream, d, rv);
            if (int rc = ensure(km_rbase, (size_t)(nw + 1) * 8)) return rc;
            hipLaunchKernelGGL(k_km_rbase, dim3(1), dim3(1024), 0, stream, d, (int64_t*)km_rbase.p);
            const int64_t nrec = fetch_i64((int64_t*)km_rbase.p + nw);
            if (nrec > 0) {
                if (int rc = ensure(km_rec, (size_t)nrec * 32)) return rc;
                if (int rc = ensure(km_skend, (size_t)std::max<int64_t>(nrec, 32) * 2)) return rc;
                d.rbase = (const int64_t*)km_rbase.p;
                d.rec = (uint4*)km_rec.p;
                d.skend = (uint16_t*)km_skend.p;
                d.scount = du.scount;
                hipLaunchKernelGGL(k_km_sscatter, dim3((unsigned)nblk), dim3(kKmBlock), (size_t)nw * 4, stream, d,
                                   (const uint4*)du.rec, (const uint16_t*)du.skend, (const uint16_t*)du.sk);
                hipLaunchKernelGGL(k_km_expand, dim3((unsigned)(8 * ((nw + 7) / 8) * kKmExpChunks)), dim3(kKmExpBlock), 0, stream, d,
                                   dp.n_aggs, R, rv);
            }
            phase_end(ph2);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "key-major aggregation failed");
            if (int rc = km_check_report("single pass")) return rc;
            stats.windows_keymajor += nw;
            *handled = true;
            return 0;
        }
        walk(false);
        if (hipError_t e = hipGetLastError(); e != hipSuccess)
            return fail(EK_ERR_DEVICE, "key-major count pass launch (lds %zu, nw %d): %s", lds, nw, hipGetErrorName(e));
        if (sort) {
            hipMemcpyAsync(h_kmf, d_flag, 16, hipMemcpyDeviceToHost, stream);
            if (hipError_t e = hipStreamSynchronize(stream); e != hipSuccess)
                return fail(EK_ERR_DEVICE, "key-major count pass failed: %s", hipGetErrorName(e));
            if (int rc = km_check_report("count pass")) return rc;
            if (h_kmf[2]) { phase_end(ph2); return 0; }   // a (key, window) run too long for one thread: window-major path
        }
        hipLaunchKernelGGL(k_km_scan, dim3(nw), dim3(1024), 0, stream, d, rv);
        // packed emission: the windows' kept totals -> record offsets (one sync to size the record buffer)
        const bool packed = km_packed && dp.n_aggs <= kKmRecAggs;
        int64_t nrec = 0;
        if (packed) {
            if (int rc = ensure(km_rbase, (size_t)(nw + 1) * 8)) return rc;
            hipLaunchKernelGGL(k_km_rbase, dim3(1), dim3(1024), 0, stream, d, (int64_t*)km_rbase.p);
            nrec = fetch_i64((int64_t*)km_rbase.p + nw);
            if (int rc = ensure(km_rec, (size_t)std::max<int64_t>(nrec, 1) * 32)) return rc;
            d.rbase = (const int64_t*)km_rbase.p;
            d.rec = (uint4*)km_rec.p;
            if (states) {
                if (int rc = ensure(km_skend, (size_t)std::max<int64_t>(nrec, 32) * 2)) return rc;
                d.skend = (uint16_t*)km_skend.p;
            }
        }
        walk(true);
        if (states) {
            if (nrec > 0)
                hipLaunchKernelGGL(k_km_expand, dim3((unsigned)(8 * ((nw + 7) / 8) * kKmExpChunks)), dim3(kKmExpBlock), 0, stream, d,
                                   dp.n_aggs, R, rv);
        } else if (packed && nrec > 0) {
            const int64_t per = (nrec + nw - 1) / nw;
            const dim3 gu((unsigned)std::max<int64_t>(1, std::min<int64_t>(64, (per + kBlock - 1) / kBlock)), (unsigned)nw);
            hipLaunchKernelGGL(k_km_unpack, gu, dim3(kBlock), 0, stream, d, dp.n_aggs, rv);
        }
        phase_end(ph2);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "key-major aggregation failed");
        if (int rc = km_check_report("write pass")) return rc;
        stats.windows_keymajor += nw;
        *handled = true;
        return 0;
    }
    // EK_KM_CHECK builds: the first bound a key-major kernel found violated (ek_keymajor.h km_bad)
    int km_check_report(const char* where) {
#ifdef EK_KM_CHECK
        int32_t r[8];
        if (hipMemcpy(r, (const unsigned int*)km_flag.p + 8, sizeof r, hipMemcpyDeviceToHost) != hipSuccess)
            return fail(EK_ERR_DEVICE, "check read failed");
        if (r[0]) return fail(EK_ERR_DEVICE, "key-major bound check %d after the %s: %d %d %d %d (block %d thread %d)", r[0], where,
                              r[1], r[2], r[3], r[4], r[5], r[6]);
#else
        (void)where;
#endif
        return 0;
    }

    int run_vgroup(const std::vector<int>& members, int64_t V, const std::vector<int64_t>& obase, const std::vector<int32_t>& slots) {
        const int npn = (int)members.size();
        const size_t aux_words = aux_layout_words(npn);
        int64_t* aux = desc_alloc(aux_words);
        if (!aux) return fail(EK_ERR_NOMEM, "pinned");
        int64_t* h_pbnd = aux;
        int64_t* h_dbase = h_pbnd + npn + 1;
        int32_t* h_didx = (int32_t*)(h_dbase + npn);
        uint8_t* h_fresh = (uint8_t*)(h_didx + 2 * ((npn + 1) / 2));
        int64_t* h_voff = aux + aux_layout_voff(npn);
        int64_t v = 0;
        for (int r = 0; r < npn; ++r) {
            const int w = members[r];
            const int64_t a = h_ab[2 * w], b = h_ab[2 * w + 1];
            h_pbnd[r] = v;
            h_voff[r] = a - v;
            h_dbase[r] = obase[w];
            h_didx[r] = slots[w];
            h_fresh[r] = 1;
            v += b - a;
        }
        h_pbnd[npn] = v;
        GroupDesc gd{};
        gd.lo = 0;
        gd.hi = V;
        gd.q_lo = 0;
        gd.n_panes = npn;
        gd.nb = NB;
        gd.kbits = kbits;
        gd.abase = 0;
        gd.sorted = 1;
        gd.ring = npn;
        // chunk size: small windows -> shorter chunks (a chunk sorts at most kMaxChunkBnd+1 panes in LDS);
        // big windows -> longer chunks (k_agg walks at most kMaxRuns chunk runs per pane)
        int64_t csz = kTile;
        int mp = max_panes_in_chunk(h_pbnd, gd, csz);
        while (csz > 256 && (mp > kMaxChunkBnd + 1 || (int64_t)NB * mp > np_max)) { csz >>= 1; mp = max_panes_in_chunk(h_pbnd, gd, csz); }
        while (max_chunks_in_pane(h_pbnd, gd, csz) > kMaxRuns && csz < (1 << 22)) { csz <<= 1; mp = max_panes_in_chunk(h_pbnd, gd, csz); }
        const int lp_stride = std::min(npn * NB, NB * mp);
        if (mp > kMaxChunkBnd + 1 || lp_stride > np_max || max_chunks_in_pane(h_pbnd, gd, csz) > kMaxRuns)
            return fail(EK_ERR_UNSUPPORTED, "window sizes in one launch too uneven (%d windows per chunk, %lld events)",
                        mp, (long long)V);
        gd.chunk = (int32_t)csz;
        gd.mruns = std::max(1, max_chunks_in_pane(h_pbnd, gd, csz));
        gd.key_col = dp.key_col;
        gd.ts_col = dp.ts_col;
        gd.n_where = dp.n_where;
        gd.num_keys = dp.num_keys;
        gd.nbatch = eb.n;
        gd.nch = (int32_t)((V + csz - 1) / csz);
        gd.np = npn * NB;
        gd.has_accept = 0;
        gd.pad = env_int("EKGPU_DEBUG_AGG", 0);   // diagnostic knobs (timing only; results invalid when set)
        gd.pad2 = variant;
        if (int rc = upload_aux(aux, aux_words, npn, gd)) return rc;
        if (int rc = ensure(vp_err, (size_t)npn * 4)) return rc;
        if (int rc = ensure(vp_mc, (size_t)npn * 8)) return rc;
        if (int rc = ensure(vp_mh, (size_t)npn * 8)) return rc;
        if (where_can_fail) {   // window witnesses in buffer order (k_group_prep zeroes them: every pane is fresh)
            if (int rc = ensure(vp_wit, (size_t)npn * sizeof(WitRec))) return rc;
            gd.pwit = (WitRec*)vp_wit.p;
        }
        return launch_part_agg(buffer_view(), gd, 2, nullptr, (int32_t*)vp_err.p, (int64_t*)vp_mc.p,
                               (unsigned long long*)vp_mh.p, lp_stride, true);
    }

    // ---- triggers per window type (host side of event_window_trigger.go:112-209 over the buffer)
    int range_triggers(int64_t rel_prev) {
        std::vector<PendWin> pw;
        const int64_t n_new = eb_rel - rel_prev;
        if (proc_inc || proc_v2s) return proc_inc_triggers(rel_prev);
        if (inc && wtype == EK_WINDOW_SLIDING) return inc_slide_triggers(rel_prev);
        if (inc && wtype == EK_WINDOW_COUNT) return inc_count_triggers(rel_prev);
        if (wtype == EK_WINDOW_SLIDING && gmode) {
            if (int rc = global_slide_triggers(pw)) return rc;
        } else if (wtype == EK_WINDOW_SLIDING && proc) {
            if (int rc = proc_slide_triggers(rel_prev, pw)) return rc;
        } else if (wtype == EK_WINDOW_SLIDING) {
            const int64_t D = (int64_t)plan.delay * unit_ms(plan.time_unit);
            std::vector<DelayTrig> et2_new;   // send-twice: this push's triggers (abs position, ts, release step)
            if (n_new > 0) {
                // trigger events among the newly released rows (OVER (WHEN ...)), in release order
                if (int rc = ensure(flags_d, (size_t)n_new)) return rc;
                if (int rc = ensure(trig_d, (size_t)n_new * 8)) return rc;
                const int nb = (int)((n_new + kCompactTile - 1) / kCompactTile);
                if (int rc = ensure(cnts_d, (size_t)(nb + 1) * 8)) return rc;
                const DBatch bv = buffer_view();
                hipLaunchKernelGGL(k_trigger_flags, dim3((int)std::min<int64_t>(4096, (n_new + 255) / 256)), dim3(256), 0, stream,
                                   d_plan, bv, rel_prev, eb_rel, (uint8_t*)flags_d.p);
                hipLaunchKernelGGL(k_flag_count, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n_new, (int64_t*)cnts_d.p);
                hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, stream, (int64_t*)cnts_d.p, nb);
                hipLaunchKernelGGL(k_flag_write, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n_new,
                                   (const int64_t*)cnts_d.p, rel_prev, (int64_t*)trig_d.p);
                const int64_t nt = fetch_i64((const int64_t*)cnts_d.p + nb);
                if (nt > 0) {
                    std::vector<int64_t> pos(nt), tts(nt), trel(nt);
                    // positions, ts and release step of each trigger (device gathers; one round trip, pinned copies)
                    if (int rc = ensure(mrg_col, (size_t)nt * 16)) return rc;
                    int64_t* g_ts = (int64_t*)mrg_col.p;
                    const int gg = (int)std::min<int64_t>(4096, (nt + 255) / 256);
                    hipLaunchKernelGGL(k_gather8, dim3(gg), dim3(256), 0, stream, (const int64_t*)trig_d.p, nt, INT64_MAX,
                                       (const int64_t*)eb.col[dp.ts_col].p, (const int64_t*)nullptr, (const int64_t*)nullptr, g_ts);
                    hipLaunchKernelGGL(k_gather8, dim3(gg), dim3(256), 0, stream, (const int64_t*)trig_d.p, nt, INT64_MAX,
                                       (const int64_t*)eb.rel.p, (const int64_t*)nullptr, (const int64_t*)nullptr, g_ts + nt);
                    if (int rc = down_pinned(pos.data(), trig_d.p, (size_t)nt * 8)) return rc;
                    if (int rc = down_pinned(tts.data(), g_ts, (size_t)nt * 8)) return rc;
                    if (int rc = down_pinned(trel.data(), g_ts + nt, (size_t)nt * 8)) return rc;
                    if (int rc = sync_downs("trigger copy failed")) return rc;
                    for (int64_t k = 0; k < nt; ++k) {
                        const int64_t i = pos[k], t = tts[k], r = trel[k];
                        if (plan.window_version == 2 && D > 0) {
                            // EventSlidingWindowOp with a delay: the trigger queues ts + D (delayTS, emitted at the
                            // WatermarkTuples, v2_delay_triggers below)
                            v2q.push_back(V2Delay{t + D, r == INT64_MAX ? cur_arr_base + cur_nb : r});
                        } else if (plan.window_version == 2) {
                            // EventSlidingWindowOp (window_v2_event_op.go:78-96): scanWindow over the rows added so far,
                            // left-open (t - L, t] (window_v2_op.go:252-263); WindowRange (t - L, t)
                            PendWin p{};
                            p.q.kind = RB_UPTO;
                            p.q.lo_ts = t - L + 1;
                            p.q.pos = i;
                            p.q.floor = eb_floor;
                            p.start = t - L;
                            p.end = t;
                            pw.push_back(p);
                        } else if (D == 0) {
                            PendWin p{};
                            p.q.kind = RB_SLIDE;
                            p.q.lo_ts = t - L;
                            p.q.hi_ts = t;
                            p.q.pos = i;
                            p.q.rstep = r;
                            p.q.floor = eb_floor;
                            p.start = t - L;   // scan(): windowStart = t - length (window_op.go:697-707)
                            p.end = t;
                            pw.push_back(p);
                        } else if (send_twice) {
                            et2_new.push_back(DelayTrig{eb_base + i, t, r});
                        } else {
                            // W at the release step: the delayed window fires at a LATER watermark advance
                            delayq.push_back(DelayTrig{eb_base + i, t, r == INT64_MAX ? W : relstep_w(r)});
                        }
                    }
                }
            }
            if (D > 0 && plan.window_version == 2) {
                if (int rc = v2_delay_triggers(rel_prev, pw)) return rc;
            } else if (D > 0 && send_twice) {
                if (int rc = et2_triggers(rel_prev, et2_new, pw)) return rc;
            } else if (D > 0) {
                while (delayq_head < delayq.size()) {
                    const DelayTrig& d = delayq[delayq_head];
                    if (!(W >= d.ts + D && W > d.w_rel)) break;
                    PendWin p{};
                    p.q.kind = RB_LB;
                    p.q.lo_ts = d.ts - L;
                    p.q.hi_ts = d.ts + D;
                    p.q.floor = eb_floor;
                    p.start = 0;     // second-part scan leaves WindowRange unset
                    p.end = 0;
                    pw.push_back(p);
                    delayq_head++;
                }
                if (delayq_head > 4096 && delayq_head * 2 > delayq.size()) {
                    delayq.erase(delayq.begin(), delayq.begin() + (int64_t)delayq_head);
                    delayq_head = 0;
                }
            }
        } else if (inc) {
            if (int rc = inc_triggers(rel_prev, pw)) return rc;
            int rc = fire_windows(pw);
            // rows a pending window will aggregate stay in the buffer (windows opened later start at >= eb_rel)
            eb_floor = inc_pend.empty() ? eb_rel : std::min(eb_rel, inc_pend.front().floor_abs - eb_base);
            return rc;
        } else if (wtype == EK_WINDOW_TUMBLING || wtype == EK_WINDOW_HOPPING) {
            if (!e1_known && eb_rel > 0 && !gmode) {
                e1_known = true;
                first_ts = fetch_i64(eb.col[dp.ts_col].p);
                E1 = aligned_end(first_ts, raw_interval, plan.time_unit, plan.tz_offset_s);
            }
            if (e1_known && has_W) {
                // (processing time: a tick fires before any later row arrives, so the discard of an empty window
                // never reaches a row the window could not hold; it is not applied)
                hop_discard_pending = wtype == EK_WINDOW_HOPPING && !gmode && !proc;
                while (win_end(next_win) <= W) {
                    const int64_t j = next_win++;
                    PendWin p{};
                    p.q.kind = RB_LB;
                    p.q.lo_ts = wtype == EK_WINDOW_TUMBLING ? (j == 0 ? INT64_MIN : win_end(j - 1)) : win_end(j) - L;
                    p.q.hi_ts = win_end(j);
                    p.q.floor = eb_floor;
                    p.start = window_start(j);
                    p.end = win_end(j);
                    pw.push_back(p);
                }
            }
        } else if (wtype == EK_WINDOW_SESSION && proc) {
            if (int rc = proc_session_triggers(rel_prev, pw)) return rc;
        } else if (wtype == EK_WINDOW_SESSION) {
            if (int rc = session_triggers(rel_prev, pw)) return rc;
        } else if (wtype == EK_WINDOW_STATE) {
            return state_scan(rel_prev, eb_rel);
        }
        return fire_windows(pw);
    }

    // ---- STATEWINDOW (StateWindowOp.exec, window_v2_op.go:111-148) over buffer rows [lo, hi), in order:
    //   if no window is open, a row whose begin condition holds opens one (canBegin);
    //   a row of an open window joins it; if its emit condition holds the window [start, row] is emitted and closed;
    //   a row that opened AND closed a window re-opens one at once (`if canBegin && !s.onBegin`), starting at the next row.
    // Only rows whose begin or emit condition holds can change the state: the device evaluates both conditions,
    // compacts those rows, and the host walks them.
    int state_scan(int64_t lo, int64_t hi) {
        std::vector<PendWin> pw;
        const int64_t n_new = hi - lo;
        if (n_new > 0) {
            if (int rc = ensure(flags_d, (size_t)n_new)) return rc;
            if (int rc = ensure(trig_d, (size_t)n_new * 8)) return rc;
            const int nb = (int)((n_new + kCompactTile - 1) / kCompactTile);
            if (int rc = ensure(cnts_d, (size_t)(nb + 1) * 8)) return rc;
            const DBatch bv = buffer_view();
            const int g = (int)std::min<int64_t>(4096, (n_new + 255) / 256);
            hipLaunchKernelGGL(k_state_flags, dim3(g), dim3(256), 0, stream, d_plan, bv, lo, hi, (uint8_t*)flags_d.p);
            hipLaunchKernelGGL(k_flag_count, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n_new, (int64_t*)cnts_d.p);
            hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, stream, (int64_t*)cnts_d.p, nb);
            hipLaunchKernelGGL(k_flag_write, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n_new,
                               (const int64_t*)cnts_d.p, lo, (int64_t*)trig_d.p);
            const int64_t nt = fetch_i64((const int64_t*)cnts_d.p + nb);
            if (nt > 0) {
                std::vector<int64_t> pos(nt);
                std::vector<uint8_t> fl(nt);
                if (int rc = ensure(mrg_col, (size_t)nt)) return rc;
                const int gg = (int)std::min<int64_t>(4096, (nt + 255) / 256);
                hipLaunchKernelGGL(k_gather_flags, dim3(gg), dim3(256), 0, stream, (const int64_t*)trig_d.p, nt, lo,
                                   (const uint8_t*)flags_d.p, (uint8_t*)mrg_col.p);
                hipMemcpyAsync(pos.data(), trig_d.p, (size_t)nt * 8, hipMemcpyDeviceToHost, stream);
                hipMemcpyAsync(fl.data(), mrg_col.p, (size_t)nt, hipMemcpyDeviceToHost, stream);
                if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "state condition copy failed");
                for (int64_t k = 0; k < nt; ++k) {
                    const int64_t i = pos[k];
                    bool can_begin = false;
                    if (!st_on) {
                        can_begin = (fl[k] & 1) != 0;
                        if (!can_begin) continue;
                        st_on = true;
                        st_start_abs = eb_base + i;
                    }
                    if (fl[k] & 2) {
                        PendWin p{};
                        p.q.kind = RB_FIXED;
                        p.q.pos = st_start_abs - eb_base;
                        p.q.rstep = i + 1;
                        p.start = EK_STATE_WINDOW_START_MS;
                        p.end = EK_STATE_WINDOW_END_MS;
                        pw.push_back(p);
                        st_on = can_begin;   // opened and closed by this row: the next window starts at the next row
                        st_start_abs = eb_base + i + 1;
                    }
                }
            }
        }
        if (!pw.empty() && plan.is_event_time && eb.n > 0) {
            // emitWindow(time.Time{}, InfTime) -> scanWindow keeps rows whose timestamp is After(time.Time{})
            // (window_v2_op.go:77-87,254-263): in the ts-ordered buffer those are the rows from lb(year 1 + 1 ms) on
            const int64_t bound = kYear1Ms + 1;
            if (int rc = ensure(bounds_val, 8)) return rc;
            if (int rc = ensure(bounds_idx, 8)) return rc;
            hipMemcpyAsync(bounds_val.p, &bound, 8, hipMemcpyHostToDevice, stream);
            hipLaunchKernelGGL(k_lower_bound, dim3(1), dim3(64), 0, stream, (const int64_t*)eb.col[dp.ts_col].p, (int64_t)0,
                               eb.n, (const int64_t*)bounds_val.p, 1, (int64_t*)bounds_idx.p);
            const int64_t y1 = fetch_i64(bounds_idx.p);
            for (PendWin& p : pw) p.q.pos = std::max(p.q.pos, std::min(y1, p.q.rstep));
        }
        int rc = fire_windows(pw);
        // rows before the open window (or every scanned row) are never needed again (scanner.gc(InfTime))
        eb_floor = std::max(eb_floor, st_on ? st_start_abs - eb_base : hi);
        return rc;
    }

    // ---- incremental-aggregation windows, event time (HoppingWindowIncAggEventOp, window_inc_agg_event_op.go:71-146;
    // TUMBLING = the same op with Length = Interval, :298-307). Over the rows released in release order:
    //   triggerWindow: a row with ts > T (NextTriggerWindowTime) sets T = getAlignedWindowEndTime(ts) and opens
    //                  the window [T - Interval, T - Interval + Length);
    //   calIncAggWindow: the row joins every open window whose range holds its ts;
    //   at a watermark, windows with end <= watermark are emitted (emitWindow) and dropped (gcIncAggWindow).
    // A window therefore holds the rows with ts in its range from the row that opened it on: an index range
    // [first row >= max(opener, lb(start)), lb(end)) of the ts-sorted buffer -> RangeQ RB_LB with floor = opener.
    // getAlignedWindowEndTime is monotone in ts and piecewise constant on "cells" [lo_k, lo_k+1) with end e_k; inside
    // a cell only the first row with ts > T opens a window (T becomes e_k), except rows with ts > e_k (the second
    // "second == interval" of window_op.go:194-227), each of which opens one. All the row indices the rule needs
    // are lower bounds in the sorted buffer: one batched search per push, no per-row host work.
    int64_t next_cell_lo(int64_t x) const {
        const int64_t e = aligned_end(x, raw_interval, plan.time_unit, plan.tz_offset_s);
        int64_t lo = x + 1, hi = std::max(x, e) + 2 * 86400000LL;   // aligned_end(hi) > e
        while (lo < hi) {
            const int64_t m = lo + ((hi - lo) >> 1);
            if (aligned_end(m, raw_interval, plan.time_unit, plan.tz_offset_s) > e) hi = m; else lo = m + 1;
        }
        return lo;
    }

    int inc_triggers(int64_t rel_prev, std::vector<PendWin>& pw) {
        const int64_t I = H;
        if (eb_rel > rel_prev) {
            const int64_t* bts = (const int64_t*)eb.col[dp.ts_col].p;
            int64_t t01[2];
            hipMemcpyAsync(&t01[0], bts + rel_prev, 8, hipMemcpyDeviceToHost, stream);
            hipMemcpyAsync(&t01[1], bts + eb_rel - 1, 8, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "inc window ts fetch failed");
            // cells covering [t0, t1]
            std::vector<int64_t> clo, ce;
            for (int64_t x = t01[0]; x <= t01[1];) {
                clo.push_back(x);
                ce.push_back(aligned_end(x, raw_interval, plan.time_unit, plan.tz_offset_s));
                x = next_cell_lo(x);
                if (clo.size() > ((size_t)1 << 22)) return fail(EK_ERR_UNSUPPORTED, "incremental window: too many window cells in one batch");
            }
            const int K = (int)clo.size();
            // bounds: F_k = lb(lo_k), U_k = lb(e_k + 1) (first row with ts > e_k), Q = lb(T + 1)
            std::vector<int64_t> q((size_t)2 * K + 1);
            for (int k = 0; k < K; ++k) { q[k] = clo[k]; q[K + k] = ce[k] + 1; }
            q[2 * K] = inc_has_T ? inc_T + 1 : INT64_MIN;
            const int nq = 2 * K + 1;
            if (int rc = ensure(bounds_val, (size_t)nq * 8)) return rc;
            if (int rc = ensure(bounds_idx, (size_t)nq * 8)) return rc;
            hipMemcpyAsync(bounds_val.p, q.data(), (size_t)nq * 8, hipMemcpyHostToDevice, stream);
            hipLaunchKernelGGL(k_lower_bound, dim3((nq + 255) / 256), dim3(256), 0, stream, bts, rel_prev, eb_rel,
                               (const int64_t*)bounds_val.p, nq, (int64_t*)bounds_idx.p);
            std::vector<int64_t> b((size_t)nq);
            hipMemcpyAsync(b.data(), bounds_idx.p, (size_t)nq * 8, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "inc window bounds failed");
            int64_t T = inc_T, ubT = b[2 * K];
            bool hasT = inc_has_T;
            const int64_t dup_cap = env_int("EKGPU_INC_MAX_OPEN", 65536);
            int64_t opened = 0;
            auto open_win = [&](int64_t e, int64_t row) -> int {
                if (++opened > dup_cap)
                    return fail(EK_ERR_UNSUPPORTED, "incremental window: more than %lld windows opened in one batch (the reference "
                                                    "opens one per row in the second where the alignment ends before the row)",
                                (long long)dup_cap);
                inc_pend.push_back(IncWin{e - I, e - I + L, eb_base + row});
                return 0;
            };
            for (int k = 0; k < K; ++k) {
                const int64_t s0 = k == 0 ? rel_prev : b[k];
                const int64_t s1 = k + 1 < K ? b[k + 1] : eb_rel;
                if (s0 >= s1) continue;
                const int64_t Uk = b[K + k];
                const int64_t nend = std::min(Uk, s1);        // rows with ts <= e_k
                const int64_t r = hasT ? std::max(s0, ubT) : s0;
                if (r < nend) {
                    if (int rc = open_win(ce[k], r)) return rc;
                    T = ce[k]; ubT = Uk; hasT = true;
                }
                const int64_t a0 = std::max(Uk, s0);          // rows with ts > e_k: each opens a window
                if (a0 < s1) {
                    T = ce[k]; ubT = Uk; hasT = true;
                    // with Length == Interval those windows end at e_k, before their rows: nothing to report
                    if (L > I)
                        for (int64_t row = a0; row < s1; ++row) if (int rc = open_win(ce[k], row)) return rc;
                }
            }
            inc_T = T;
            inc_has_T = hasT;
        }
        // emitWindow at the watermark: every open window with end <= W, in opening order
        size_t nf = 0;
        while (has_W && nf < inc_pend.size() && inc_pend[nf].end <= W) {
            const IncWin& iw = inc_pend[nf++];
            PendWin p{};
            p.q.kind = RB_LB;
            p.q.lo_ts = iw.start;
            p.q.hi_ts = iw.end;
            p.q.floor = iw.floor_abs - eb_base;
            p.start = iw.start;
            p.end = iw.end;
            pw.push_back(p);
        }
        inc_pend.erase(inc_pend.begin(), inc_pend.begin() + (int64_t)nf);
        return 0;
    }

    // Watermarks at / before the release steps of the listed buffer rows (k_step_wm); rows must be released in this batch
    int step_watermarks(const int64_t* d_pos, int64_t nt, std::vector<int64_t>& w_step, std::vector<int64_t>& w_prev) {
        if (int rc = ensure(mrg_col, (size_t)nt * 24)) return rc;
        int64_t* g_rel = (int64_t*)mrg_col.p;
        const int gg = (int)std::min<int64_t>(4096, (nt + 255) / 256);
        hipLaunchKernelGGL(k_gather8, dim3(gg), dim3(256), 0, stream, d_pos, nt, INT64_MAX, (const int64_t*)eb.rel.p,
                           (const int64_t*)nullptr, (const int64_t*)nullptr, g_rel);
        hipLaunchKernelGGL(k_step_wm, dim3(gg), dim3(256), 0, stream, (const int64_t*)g_rel, nt, runmax_p,
                           cur_nb, cur_arr_base, cur_prevmax, plan.late_tolerance_ms, g_rel + nt, g_rel + 2 * nt);
        w_step.resize(nt);
        w_prev.resize(nt);
        hipMemcpyAsync(w_step.data(), g_rel + nt, (size_t)nt * 8, hipMemcpyDeviceToHost, stream);
        hipMemcpyAsync(w_prev.data(), g_rel + 2 * nt, (size_t)nt * 8, hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "step watermark gather failed");
        return 0;
    }

    // ---- incremental sliding window, event time, no delay (SlidingWindowIncAggEventOp.appendIncAggWindowInEvent +
    // emitList + gcIncAggWindow, window_inc_agg_event_op.go:193-273). Per released row in release order: a trigger
    // row opens a window starting at its ts; every row joins the open windows whose [start, start + L) holds its ts;
    // a trigger row then queues a CLONE OF THE OLDEST OPEN WINDOW (CurrWindowList[0]) with StartTime = its ts, which
    // the next WatermarkTuple emits with WindowRange (ts, watermark); at each watermark windows with
    // watermark - start >= L are dropped. The oldest open window at trigger row j is the first trigger k whose
    // window survived the watermark before j's release step, and its rows are [k, min(j + 1, lb(ts_k + L))) of the
    // ts-sorted buffer. Open windows: inc_pend (start = ts, floor_abs = row).
    int inc_slide_triggers(int64_t rel_prev) {
        std::vector<PendWin> pw;
        const int64_t n_new = eb_rel - rel_prev;
        if (n_new > 0) {
            if (int rc = ensure(flags_d, (size_t)n_new)) return rc;
            if (int rc = ensure(trig_d, (size_t)n_new * 8)) return rc;
            const int nb = (int)((n_new + kCompactTile - 1) / kCompactTile);
            if (int rc = ensure(cnts_d, (size_t)(nb + 1) * 8)) return rc;
            const DBatch bv = buffer_view();
            hipLaunchKernelGGL(k_trigger_flags, dim3((int)std::min<int64_t>(4096, (n_new + 255) / 256)), dim3(256), 0, stream,
                               d_plan, bv, rel_prev, eb_rel, (uint8_t*)flags_d.p);
            hipLaunchKernelGGL(k_flag_count, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n_new, (int64_t*)cnts_d.p);
            hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, stream, (int64_t*)cnts_d.p, nb);
            hipLaunchKernelGGL(k_flag_write, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n_new,
                               (const int64_t*)cnts_d.p, rel_prev, (int64_t*)trig_d.p);
            const int64_t nt = fetch_i64((const int64_t*)cnts_d.p + nb);
            if (nt > 0) {
                std::vector<int64_t> pos(nt), tts(nt), w_step, w_prev;
                if (int rc = step_watermarks((const int64_t*)trig_d.p, nt, w_step, w_prev)) return rc;
                if (int rc = ensure(bounds_val, (size_t)nt * 8)) return rc;
                const int gg = (int)std::min<int64_t>(4096, (nt + 255) / 256);
                hipLaunchKernelGGL(k_gather8, dim3(gg), dim3(256), 0, stream, (const int64_t*)trig_d.p, nt, INT64_MAX,
                                   (const int64_t*)eb.col[dp.ts_col].p, (const int64_t*)nullptr, (const int64_t*)nullptr,
                                   (int64_t*)bounds_val.p);
                hipMemcpyAsync(pos.data(), trig_d.p, (size_t)nt * 8, hipMemcpyDeviceToHost, stream);
                hipMemcpyAsync(tts.data(), bounds_val.p, (size_t)nt * 8, hipMemcpyDeviceToHost, stream);
                if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "trigger copy failed");
                size_t head = 0;
                for (int64_t k = 0; k < nt; ++k) {
                    const int64_t wp = w_prev[k];
                    while (wp != INT64_MIN && head < inc_pend.size() && wp - inc_pend[head].start >= L) head++;
                    inc_pend.push_back(IncWin{tts[k], 0, eb_base + pos[k]});
                    const IncWin& f = inc_pend[head];
                    PendWin p{};
                    p.q.kind = RB_CAP;
                    p.q.pos = f.floor_abs - eb_base;
                    p.q.rstep = pos[k] + 1;
                    p.q.hi_ts = f.start + L;
                    p.start = tts[k];
                    p.end = w_step[k];
                    pw.push_back(p);
                }
                inc_pend.erase(inc_pend.begin(), inc_pend.begin() + (int64_t)head);
            }
        }
        // the batch's last watermark: gcIncAggWindow
        size_t head = 0;
        while (has_W && head < inc_pend.size() && W - inc_pend[head].start >= L) head++;
        inc_pend.erase(inc_pend.begin(), inc_pend.begin() + (int64_t)head);
        const int rc = fire_windows(pw);
        eb_floor = std::max(eb_floor, inc_pend.empty() ? eb_rel : inc_pend.front().floor_abs - eb_base);
        return rc;
    }

    // ---- incremental count window, event time (CountWindowIncAggEventOp, window_inc_agg_event_op.go:351-408): the
    // released rows form consecutive blocks of n; a block is emitted by the WatermarkTuple after its last row, with
    // WindowRange (ts of its first row, watermark). inc_T = absolute buffer position of the open block's first row.
    int inc_count_triggers(int64_t rel_prev) {
        std::vector<PendWin> pw;
        const int64_t n = plan.length;
        if (!inc_has_T) { inc_has_T = true; inc_T = eb_base + rel_prev; }
        std::vector<int64_t> firsts, lasts;
        for (int64_t s = inc_T; s + n <= eb_base + eb_rel; s += n) {
            firsts.push_back(s - eb_base);
            lasts.push_back(s + n - 1 - eb_base);
        }
        const int64_t nw = (int64_t)firsts.size();
        if (nw > 0) {
            if (int rc = ensure(trig_d, (size_t)nw * 16)) return rc;
            hipMemcpyAsync(trig_d.p, lasts.data(), (size_t)nw * 8, hipMemcpyHostToDevice, stream);
            hipMemcpyAsync((int64_t*)trig_d.p + nw, firsts.data(), (size_t)nw * 8, hipMemcpyHostToDevice, stream);
            std::vector<int64_t> w_step, w_prev, t0(nw);
            if (int rc = step_watermarks((const int64_t*)trig_d.p, nw, w_step, w_prev)) return rc;
            if (int rc = ensure(bounds_val, (size_t)nw * 8)) return rc;
            const int gg = (int)std::min<int64_t>(4096, (nw + 255) / 256);
            hipLaunchKernelGGL(k_gather8, dim3(gg), dim3(256), 0, stream, (const int64_t*)trig_d.p + nw, nw, INT64_MAX,
                               (const int64_t*)eb.col[dp.ts_col].p, (const int64_t*)nullptr, (const int64_t*)nullptr,
                               (int64_t*)bounds_val.p);
            hipMemcpyAsync(t0.data(), bounds_val.p, (size_t)nw * 8, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "count window ts gather failed");
            for (int64_t w = 0; w < nw; ++w) {
                PendWin p{};
                p.q.kind = RB_FIXED;
                p.q.pos = firsts[w];
                p.q.rstep = lasts[w] + 1;
                p.start = t0[w];
                p.end = w_step[w];
                pw.push_back(p);
            }
            inc_T += nw * n;
        }
        const int rc = fire_windows(pw);
        eb_floor = std::max(eb_floor, inc_T - eb_base);
        return rc;
    }

    // ---- processing-time incremental windows (TumblingWindowIncAggOp / HoppingWindowIncAggOp / SlidingWindowIncAggOp,
    // window_inc_agg_op.go:316-790) under the caller's clock. The rows arrive in the buffer in delivery order, so every
    // window's content is a contiguous buffer range [first, upto): the host replays the op's timers over a mirror of the
    // delivered arrival timestamps (h_rts) — every timer due at or before a row fires before it, an emit timer before a
    // tick at the same instant — and fires each emitted window as a fixed range with WindowRange [StartTime, now]:
    //   TUMBLING: aligned (default): the window opened at the start is emitted by the FirstTimer at
    //     getAlignedWindowEndTime(start, length), then each tick (every length) emits the window the first row after the
    //     previous emit opened (StartTime = that row's ts), if any; unaligned (inc_unaligned): ticks every length from the
    //     start, no window before the first row;
    //   HOPPING: each tick (the FirstTimer at getAlignedWindowEndTime(start, interval), then every interval; unaligned:
    //     the start itself, then every interval) opens a window [T, T + length) emitted at T + length (the aligned
    //     op's window opened at the start has no emit timer: never emitted);
    //   SLIDING: a row matching OVER (WHEN) emits the oldest live window, i.e. the rows since the first one with
    //     ts > t - length (gcIncAggWindow(length + delay)), StartTime = that row's ts; with a delay D a timer at t + D
    //     emits the rows since the first one with ts > t - length that were delivered before it.
    struct PiHop { int64_t start, first_abs; };
    int64_t pi_tick = INT64_MAX;        // next tick (tumbling / hopping)
    int64_t pi_D = 0;                   // sliding delay (ms)
    bool pi_cur = false;                // tumbling: a window is open
    int64_t pi_cur_start = 0, pi_cur_first = 0;   // its StartTime and first row (absolute buffer index; -1: not yet known)
    std::vector<PiHop> pi_hop;          // hopping: opened, not yet emitted windows (emit due = start + length)
    size_t pi_hop_head = 0;
    std::vector<int64_t> pi_dq;         // sliding: delay timers (trigger ts), due order
    size_t pi_dq_head = 0;
    int64_t pi_next_abs = 0;            // first mirrored row not yet replayed
    void pi_reset() {
        pi_tick = INT64_MAX;
        pi_cur = false;
        pi_cur_start = pi_cur_first = 0;
        pi_hop.clear();
        pi_hop_head = 0;
        pi_dq.clear();
        pi_dq_head = 0;
        pi_next_abs = 0;
    }
    void pi_start(int64_t t0) {
        const bool aligned = plan.inc_unaligned == 0;
        pi_D = wtype == EK_WINDOW_SLIDING ? (int64_t)plan.delay * unit_ms(plan.time_unit) : 0;
        if (wtype == EK_WINDOW_TUMBLING) {
            if (aligned) { pi_cur = true; pi_cur_start = t0; pi_cur_first = -1; }
            pi_tick = aligned ? aligned_end(t0, raw_interval, plan.time_unit, plan.tz_offset_s) : t0 + H;
        } else if (wtype == EK_WINDOW_HOPPING) {
            if (aligned) pi_tick = aligned_end(t0, raw_interval, plan.time_unit, plan.tz_offset_s);
            else { pi_hop.push_back(PiHop{t0, -1}); pi_tick = t0 + H; }
        }
    }
    int proc_inc_triggers(int64_t rel_prev) {
        std::vector<PendWin> pw;
        const int64_t n_new = eb_rel - rel_prev;
        if (h_rts.empty()) { h_rts_base = eb_base + rel_prev; if (pi_next_abs < h_rts_base) pi_next_abs = h_rts_base; }
        if (n_new > 0) {
            const size_t o = h_rts.size();
            h_rts.resize(o + n_new);
            hipMemcpyAsync(h_rts.data() + o, (const int64_t*)eb.col[dp.ts_col].p + rel_prev, (size_t)n_new * 8, hipMemcpyDeviceToHost, stream);
            if (wtype == EK_WINDOW_SLIDING) {   // OVER (WHEN) of every delivered row
                if (int rc = ensure(flags_d, (size_t)n_new)) return rc;
                const DBatch bv = buffer_view();
                hipLaunchKernelGGL(k_trigger_flags, dim3((int)std::min<int64_t>(4096, (n_new + 255) / 256)), dim3(256), 0, stream,
                                   d_plan, bv, rel_prev, eb_rel, (uint8_t*)flags_d.p);
                h_rtrig.resize(h_rts.size());
                hipMemcpyAsync(h_rtrig.data() + o, flags_d.p, (size_t)n_new, hipMemcpyDeviceToHost, stream);
            }
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "incremental window mirror copy failed");
        }
        const int64_t L_ = L, D = pi_D;
        auto ts_at = [&](int64_t abs) { return h_rts[abs - h_rts_base]; };
        auto first_gt = [&](int64_t hi_abs, int64_t x) {   // first mirrored row before hi_abs with ts > x (ts non-decreasing)
            return h_rts_base + (std::upper_bound(h_rts.begin(), h_rts.begin() + (hi_abs - h_rts_base), x) - h_rts.begin());
        };
        auto emit = [&](int64_t start, int64_t now, int64_t a_abs, int64_t b_abs) {
            PendWin p{};
            p.q.kind = RB_FIXED;
            p.q.pos = a_abs - eb_base;
            p.q.rstep = b_abs - eb_base;
            p.start = start;
            p.end = now;
            pw.push_back(p);
        };
        // every timer due at or before `now`, `upto` rows delivered (emit timers before a tick at the same instant)
        auto timers = [&](int64_t now, int64_t upto) {
            for (;;) {
                const int64_t due_h = pi_hop_head < pi_hop.size() ? pi_hop[pi_hop_head].start + L_ : INT64_MAX;
                const int64_t due_s = pi_dq_head < pi_dq.size() ? pi_dq[pi_dq_head] + D : INT64_MAX;
                const int64_t due_e = std::min(due_h, due_s);
                if (due_e <= now && due_e <= pi_tick) {
                    if (due_h <= due_s) {
                        PiHop& hw = pi_hop[pi_hop_head++];
                        const int64_t a = hw.first_abs < 0 ? upto : hw.first_abs;
                        emit(hw.start, due_h, a, upto);
                    } else if (proc_v2s) {
                        // scanWindow(t - length, t + D) over the scanner as the rows delivered since left it (each row's
                        // gc(ts - length)): rows with ts > max(t - length, last delivered ts - length)
                        pi_dq_head++;
                        const int64_t t = due_s - D;
                        const int64_t g = upto > h_rts_base ? ts_at(upto - 1) - L_ : INT64_MIN;
                        const int64_t a = first_gt(upto, std::max(t - L_, g));
                        emit(t - L_, due_s, a, upto);
                    } else {
                        pi_dq_head++;
                        const int64_t a = first_gt(upto, due_s - L_ - D);
                        if (a < upto) emit(ts_at(a), due_s, a, upto);
                    }
                } else if (pi_tick <= now) {
                    if (wtype == EK_WINDOW_TUMBLING) {
                        if (pi_cur) emit(pi_cur_start, pi_tick, pi_cur_first < 0 ? upto : pi_cur_first, upto);
                        pi_cur = false;
                    } else {
                        pi_hop.push_back(PiHop{pi_tick, -1});
                    }
                    pi_tick += H;
                } else {
                    break;
                }
            }
        };
        const int64_t end_abs = eb_base + eb_rel;
        for (int64_t r = pi_next_abs; r < end_abs; ++r) {
            const int64_t t = ts_at(r);
            timers(t, r);
            if (wtype == EK_WINDOW_TUMBLING) {
                if (!pi_cur) { pi_cur = true; pi_cur_start = t; pi_cur_first = r; }
                else if (pi_cur_first < 0) pi_cur_first = r;
            } else if (wtype == EK_WINDOW_HOPPING) {
                // a window's rows start at the first row delivered after its tick (windows still waiting for one are the
                // newest; an open window's start + length is past t, or its emit timer would have fired before this row)
                for (size_t k = pi_hop.size(); k > pi_hop_head && pi_hop[k - 1].first_abs < 0; --k) pi_hop[k - 1].first_abs = r;
            } else if (h_rtrig[r - h_rts_base]) {
                if (D > 0) pi_dq.push_back(t);
                else { const int64_t a = first_gt(r + 1, t - L_); emit(proc_v2s ? t - L_ : ts_at(a), t, a, r + 1); }
            }
        }
        pi_next_abs = end_abs;
        timers(W, end_abs);
        const int rc = fire_windows(pw);
        // rows a later emission can still hold: the open tumbling / hopping windows' rows, the sliding windows' rows
        // with ts > clock - length - delay (every later timer or trigger is at or after the clock)
        int64_t keep = end_abs;
        if (wtype == EK_WINDOW_TUMBLING && pi_cur && pi_cur_first >= 0) keep = std::min(keep, pi_cur_first);
        for (size_t k = pi_hop_head; k < pi_hop.size(); ++k) if (pi_hop[k].first_abs >= 0) keep = std::min(keep, pi_hop[k].first_abs);
        if (wtype == EK_WINDOW_SLIDING) keep = std::min(keep, first_gt(end_abs, W - L_ - D));
        eb_floor = std::max(eb_floor, keep - eb_base);
        const int64_t drop = keep - h_rts_base;
        if (drop > 65536 && drop * 2 > (int64_t)h_rts.size()) {
            h_rts.erase(h_rts.begin(), h_rts.begin() + drop);
            if (!h_rtrig.empty()) h_rtrig.erase(h_rtrig.begin(), h_rtrig.begin() + drop);
            h_rts_base = keep;
        }
        if (pi_hop_head > 1024 && pi_hop_head * 2 > pi_hop.size()) { pi_hop.erase(pi_hop.begin(), pi_hop.begin() + (int64_t)pi_hop_head); pi_hop_head = 0; }
        if (pi_dq_head > 4096 && pi_dq_head * 2 > pi_dq.size()) { pi_dq.erase(pi_dq.begin(), pi_dq.begin() + (int64_t)pi_dq_head); pi_dq_head = 0; }
        return rc;
    }

    // ---- EventSlidingWindowOp with a delay (window_v2_event_op.go:56-76,90-93): each trigger queues ts + D (v2q, in
    // release order); at every WatermarkTuple W (each accepted arrival that raises the running max,
    // watermark_op.go:170-213) the queued delays <= W emit scanWindow(delay - L - D, W) over the scanner — the rows
    // released by then with ts > the previous WatermarkTuple's gc(W' - L - D) — with WindowRange [delay - L - D, W], and
    // the queue drops that prefix only when a later delay is still pending (newIndex != -1; otherwise every due delay
    // is emitted again at the next WatermarkTuple). The WatermarkTuples of this push are replayed on the host from the
    // batch's running max; the scanner's content is the buffer range [first ts > bound, rows released by the tuple).
    struct V2Delay { int64_t due, step; };
    std::vector<V2Delay> v2q;
    size_t v2q_head = 0, v2q_seen = 0;   // v2q[v2q_seen..) were triggered in this push and not yet queued
    int64_t v2_lastW = INT64_MIN;        // the previous WatermarkTuple (its gc bound)
    int v2_delay_triggers(int64_t rel_prev, std::vector<PendWin>& pw) {
        const int64_t D = (int64_t)plan.delay * unit_ms(plan.time_unit), tol = plan.late_tolerance_ms;
        const int64_t n_new = eb_rel - rel_prev;
        std::vector<int64_t> h_rm((size_t)std::max<int64_t>(cur_nb, 0)), h_rel((size_t)std::max<int64_t>(n_new, 0));
        if (cur_nb > 0 && runmax_p) hipMemcpyAsync(h_rm.data(), runmax_p, (size_t)cur_nb * 8, hipMemcpyDeviceToHost, stream);
        if (n_new > 0) hipMemcpyAsync(h_rel.data(), (const int64_t*)eb.rel.p + rel_prev, (size_t)n_new * 8, hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "watermark replay copy failed");
        int64_t prevmax = cur_prevmax;
        for (int64_t i = 0; i < cur_nb && runmax_p; ++i) {
            const int64_t m = h_rm[(size_t)i];
            if (prevmax != INT64_MIN && m <= prevmax) continue;
            prevmax = m;
            const int64_t Wj = m - tol, step = cur_arr_base + i;
            while (v2q_seen < v2q.size() && v2q[v2q_seen].step <= step) v2q_seen++;   // released before this tuple
            if (v2q_head < v2q_seen) {
                const int64_t rel_end = rel_prev + (int64_t)(std::upper_bound(h_rel.begin(), h_rel.end(), step) - h_rel.begin());
                size_t k = v2q_head;
                for (; k < v2q_seen && v2q[k].due <= Wj; ++k) {
                    const int64_t ws = v2q[k].due - L - D;
                    const int64_t bound = v2_lastW == INT64_MIN ? ws : std::max(ws, v2_lastW - L - D);
                    PendWin p{};
                    p.q.kind = RB_UPTO;
                    p.q.lo_ts = bound + 1;
                    p.q.pos = rel_end - 1;
                    p.q.floor = eb_floor;
                    p.start = ws;
                    p.end = Wj;
                    pw.push_back(p);
                }
                if (k < v2q_seen) v2q_head = k;
            }
            v2_lastW = Wj;
        }
        if (v2q_head > 4096 && v2q_head * 2 > v2q.size()) {
            v2q.erase(v2q.begin(), v2q.begin() + (int64_t)v2q_head);
            v2q_seen -= v2q_head;
            v2q_head = 0;
        }
        return 0;
    }

    // ---- Delayed SLIDINGWINDOW with enableSlidingWindowSendTwice in event time (event_window_trigger.go:124-180,
    // window_op.go:576-603,675-721). At every WatermarkTuple W (replayed from the batch's running max, as above):
    //   1. each queued delay t + D <= W scans the last part (t, t + D];
    //   2. getNextWindow(prevWindowEndTs, W) — the earliest input in (prevWindowEndTs, W] — gates the triggers: when it
    //      finds one, every queued trigger t scans the first part (t - L, t] and queues t + D; prevWindowEndTs then walks
    //      to the last input <= W. With no input in that range the triggers stay queued.
    // Each scan keeps, by handleInputsForSlidingWindow, only the EXPIRED prefix of the inputs (ts < windowEnd - L - D)
    // whenever some but not all inputs expired (all expired: none kept). Restated on the host like the processing-time
    // rule: sw2_e holds the ts of the expired inputs kept (never in a later window: every later window starts at or
    // after their bound), the buffer rows [sw2_cut, released by the tuple) are the live inputs, a window is the fixed
    // range of live rows with ts in its bounds. Triggers wait in delayq (pos_abs, ts, release step), timers in proc_dq.
    int64_t et2_prev = kYear1Ms;          // prevWindowEndTs
    std::vector<int> med_nullable;        // median slots over a nullable f64 column (their nil-first check)
    int et2_triggers(int64_t rel_prev, const std::vector<DelayTrig>& trig, std::vector<PendWin>& pw) {
        const int64_t D = slide_delay_et(), tol = plan.late_tolerance_ms;
        const int64_t n_new = eb_rel - rel_prev;
        std::vector<int64_t> h_rm((size_t)std::max<int64_t>(cur_nb, 0)), h_rel((size_t)std::max<int64_t>(n_new, 0));
        if (h_rts.empty()) h_rts_base = eb_base + rel_prev;
        const size_t o = h_rts.size();
        h_rts.resize(o + (size_t)std::max<int64_t>(n_new, 0));
        if (cur_nb > 0 && runmax_p) hipMemcpyAsync(h_rm.data(), runmax_p, (size_t)cur_nb * 8, hipMemcpyDeviceToHost, stream);
        if (n_new > 0) {
            hipMemcpyAsync(h_rel.data(), (const int64_t*)eb.rel.p + rel_prev, (size_t)n_new * 8, hipMemcpyDeviceToHost, stream);
            hipMemcpyAsync(h_rts.data() + o, (const int64_t*)eb.col[dp.ts_col].p + rel_prev, (size_t)n_new * 8,
                           hipMemcpyDeviceToHost, stream);
        }
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "send-twice replay copy failed");
        if (sw2_cut < h_rts_base) sw2_cut = h_rts_base;
        auto ts_at = [&](int64_t abs) { return h_rts[abs - h_rts_base]; };
        auto first_gt = [&](int64_t lo, int64_t hi, int64_t x) {   // first abs index in [lo, hi) with ts > x
            return h_rts_base + (std::upper_bound(h_rts.begin() + (lo - h_rts_base), h_rts.begin() + (hi - h_rts_base), x) - h_rts.begin());
        };
        auto first_ge = [&](int64_t lo, int64_t hi, int64_t x) {   // first abs index in [lo, hi) with ts >= x
            return h_rts_base + (std::lower_bound(h_rts.begin() + (lo - h_rts_base), h_rts.begin() + (hi - h_rts_base), x) - h_rts.begin());
        };
        // the last input present with rows [.., P) released (none: INT64_MIN)
        auto last_input = [&](int64_t P) {
            if (P > sw2_cut) return ts_at(P - 1);
            return sw2_e.empty() ? INT64_MIN : sw2_e.back();
        };
        auto scan2 = [&](int64_t ws, int64_t we, int64_t P) {
            const int64_t a = first_gt(sw2_cut, P, ws);
            const int64_t b = std::max(a, first_gt(a, P, we));
            PendWin p{};
            p.q.kind = RB_FIXED;
            p.q.pos = a - eb_base;
            p.q.rstep = b - eb_base;
            p.start = ws;   // WindowRange: [t - L, t] for the first part, [t, t + D] for the last (window_op.go:683-703)
            p.end = we;
            pw.push_back(p);
            const int64_t dl = we - (L + D);
            const int64_t ne = std::lower_bound(sw2_e.begin(), sw2_e.end(), dl) - sw2_e.begin();
            const int64_t nl = first_ge(sw2_cut, P, dl) - sw2_cut;
            const int64_t present = (int64_t)sw2_e.size() + (P - sw2_cut);
            if (ne + nl == 0) return;
            if (ne + nl == present) {
                sw2_e.clear();
            } else {
                sw2_e.resize((size_t)ne);
                for (int64_t k = 0; k < nl; ++k) sw2_e.push_back(ts_at(sw2_cut + k));
            }
            sw2_cut = P;
        };
        const int64_t rel0 = eb_base + rel_prev;
        size_t tk = 0;                  // this push's triggers not queued yet
        int64_t lazy_P = -1;            // a WatermarkTuple that only moved prevWindowEndTs (applied before the next scan)
        auto settle = [&]() {
            if (lazy_P < 0) return;
            const int64_t x = last_input(lazy_P);
            if (x != INT64_MIN && x > et2_prev) et2_prev = x;
            lazy_P = -1;
        };
        int64_t prevmax = cur_prevmax;
        for (int64_t i = 0; i < cur_nb && runmax_p; ++i) {
            const int64_t m = h_rm[(size_t)i];
            if (prevmax != INT64_MIN && m <= prevmax) continue;
            prevmax = m;
            const int64_t Wj = m - tol, step = cur_arr_base + i;
            const int64_t P = rel0 + (int64_t)(std::upper_bound(h_rel.begin(), h_rel.end(), step) - h_rel.begin());
            while (tk < trig.size() && trig[tk].w_rel <= step) delayq.push_back(trig[tk++]);
            const bool due = proc_dq_head < proc_dq.size() && proc_dq[proc_dq_head] + D <= Wj;
            if (!due && delayq_head == delayq.size()) { lazy_P = P; continue; }
            settle();
            while (proc_dq_head < proc_dq.size() && proc_dq[proc_dq_head] + D <= Wj) {
                const int64_t t = proc_dq[proc_dq_head++];
                scan2(t, t + D, P);   // the last part
            }
            // getNextWindow: the earliest input in (prevWindowEndTs, W] (expired inputs kept count too)
            int64_t we1 = INT64_MAX;
            {
                auto e = std::upper_bound(sw2_e.begin(), sw2_e.end(), et2_prev);
                if (e != sw2_e.end()) we1 = *e;
                const int64_t f = first_gt(sw2_cut, P, et2_prev);
                if (f < P) we1 = std::min(we1, ts_at(f));
            }
            if (we1 == INT64_MAX || we1 > Wj) continue;
            for (; delayq_head < delayq.size(); ++delayq_head) {
                const int64_t t = delayq[delayq_head].ts;
                proc_dq.push_back(t);
                scan2(t - L, t, P);   // the first part
            }
            const int64_t x = last_input(P);
            et2_prev = std::max(we1, x);
        }
        while (tk < trig.size()) delayq.push_back(trig[tk++]);   // (a release step past this batch's tuples)
        settle();
        eb_floor = std::max(eb_floor, sw2_cut - eb_base);
        const int64_t drop = sw2_cut - h_rts_base;
        if (drop > 65536 && drop * 2 > (int64_t)h_rts.size()) {
            h_rts.erase(h_rts.begin(), h_rts.begin() + drop);
            h_rts_base = sw2_cut;
        }
        if (delayq_head > 4096 && delayq_head * 2 > delayq.size()) {
            delayq.erase(delayq.begin(), delayq.begin() + (int64_t)delayq_head);
            delayq_head = 0;
        }
        if (proc_dq_head > 4096 && proc_dq_head * 2 > proc_dq.size()) {
            proc_dq.erase(proc_dq.begin(), proc_dq.begin() + (int64_t)proc_dq_head);
            proc_dq_head = 0;
        }
        return 0;
    }
    int64_t slide_delay_et() const { return (int64_t)plan.delay * unit_ms(plan.time_unit); }

    // W at a release step r (arrival index inside the current batch): runmax[r - batch base] - lateTol
    int64_t cur_arr_base = 0, cur_nb = 0, cur_prevmax = INT64_MIN;
    int64_t relstep_w(int64_t r) {
        const int64_t j = r - cur_arr_base;
        if (j < 0 || !runmax_p) return W;
        return fetch_i64(runmax_p + j) - plan.late_tolerance_ms;
    }

    // SESSIONWINDOW(unit, L, timeout): getNextSessionWindow (event_window_trigger.go:77-110) over the released
    // timestamps, evaluated at the batch's final watermark.
    int session_triggers(int64_t rel_prev, std::vector<PendWin>& pw) {
        // mirror the newly released timestamps
        const int64_t n_new = eb_rel - rel_prev;
        if (h_rts.empty()) h_rts_base = eb_base + rel_prev;
        if (n_new > 0) {
            const size_t o = h_rts.size();
            h_rts.resize(o + n_new);
            hipMemcpyAsync(h_rts.data() + o, (const int64_t*)eb.col[dp.ts_col].p + rel_prev, (size_t)n_new * 8, hipMemcpyDeviceToHost, stream);
            if (need_rel && !gmode) {
                // the watermark before each new row's release step (k_step_wm over the batch's running max)
                if (int rc = ensure(mrg_col, (size_t)n_new * 16)) return rc;
                int64_t* g = (int64_t*)mrg_col.p;
                hipLaunchKernelGGL(k_step_wm, dim3((int)std::min<int64_t>(4096, (n_new + 255) / 256)), dim3(256), 0, stream,
                                   (const int64_t*)eb.rel.p + rel_prev, n_new, runmax_p, cur_nb, cur_arr_base,
                                   cur_prevmax, plan.late_tolerance_ms, g, g + n_new);
                if (h_rwp.size() != o) h_rwp.assign(o, INT64_MIN);   // rows mirrored before (e.g. restored): unknown
                h_rwp.resize(o + n_new);
                hipMemcpyAsync(h_rwp.data() + o, g + n_new, (size_t)n_new * 8, hipMemcpyDeviceToHost, stream);
            }
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "session mirror copy failed");
        }
        const int64_t timeout = H, duration = L;
        int64_t floor_abs = eb_base + eb_floor;
        auto next_session = [&](int64_t from_abs, bool* ticked) -> int64_t {
            *ticked = false;
            const int64_t i0 = from_abs - h_rts_base, i1 = (int64_t)h_rts.size();
            if (i0 >= i1) return INT64_MAX;
            const int64_t et = h_rts[i0];
            int64_t tick = aligned_end(et, raw_interval, plan.time_unit, plan.tz_offset_s);
            int64_t p = INT64_MIN;
            for (int64_t i = i0; i < i1; ++i) {
                const int64_t t = h_rts[i];
                // lateTolerance > 0: a WatermarkTuple before this row's release already saw p as the last input and
                // closed the session by the trailing check (now - p > timeout), before any tick at this row
                if (need_rel && p != INT64_MIN && i < (int64_t)h_rwp.size() && h_rwp[i] != INT64_MIN && h_rwp[i] - p > timeout)
                    return p + timeout;
                int64_t r = INT64_MAX;
                if (p != INT64_MIN && t - p > timeout) r = p + timeout;
                if (t > tick) {
                    if (tick - duration > et && tick < r) { r = tick; *ticked = true; }
                    tick += duration;
                }
                if (r < INT64_MAX) return r;
                p = t;
            }
            if (p != INT64_MIN && W - p > timeout) return p + timeout;
            *ticked = false;
            return INT64_MAX;
        };
        if (gmode) {
            // shard mode: the sessions the router closed over the whole stream (GlobalSession), each over this
            // shard's released rows with ts < end (a session window is not overlapping: window_op.go:605-655)
            for (const GSess& gs : g_sess) {
                const int64_t i0 = std::max<int64_t>(0, floor_abs - h_rts_base);
                const int64_t b_abs = i0 >= (int64_t)h_rts.size()
                    ? floor_abs
                    : h_rts_base + (std::lower_bound(h_rts.begin() + i0, h_rts.end(), gs.end) - h_rts.begin());
                PendWin p{};
                p.q.kind = RB_FIXED;
                p.q.pos = floor_abs - eb_base;
                p.q.rstep = b_abs - eb_base;
                p.start = gs.start;
                p.end = gs.end;
                pw.push_back(p);
                floor_abs = b_abs;
            }
            g_sess.clear();
        }
        bool ticked = false;
        int64_t we = gmode ? INT64_MAX : next_session(floor_abs, &ticked);
        while (we != INT64_MAX && we <= W) {
            const int64_t i0 = floor_abs - h_rts_base;
            const bool has_inputs = i0 < (int64_t)h_rts.size();
            if (!sess_last_ticked && has_inputs) { sess_trigger = h_rts[i0]; sess_has_trigger = true; }
            // content: remaining inputs with ts < we
            const int64_t b_abs = h_rts_base + (std::lower_bound(h_rts.begin() + i0, h_rts.end(), we) - h_rts.begin());
            PendWin p{};
            p.q.kind = RB_FIXED;
            p.q.pos = floor_abs - eb_base;
            p.q.rstep = b_abs - eb_base;
            int64_t ws = sess_has_trigger ? sess_trigger : 0;
            if (ws <= 0) ws = we - L;
            p.start = ws;
            p.end = we;
            pw.push_back(p);
            floor_abs = b_abs;
            sess_trigger = we;
            sess_has_trigger = true;
            sess_last_ticked = ticked;
            we = next_session(floor_abs, &ticked);
        }
        // trim the mirror below the floor
        const int64_t drop = floor_abs - h_rts_base;
        if (drop > 65536 && drop * 2 > (int64_t)h_rts.size()) {
            h_rts.erase(h_rts.begin(), h_rts.begin() + drop);
            if (!h_rwp.empty()) h_rwp.erase(h_rwp.begin(), h_rwp.begin() + drop);
            h_rts_base = floor_abs;
        }
        return 0;
    }

    // ================================================================== processing time (ek_advance_time)
    // WindowOperator.execProcessingWindow (window_op.go:235-470) with the caller's clock, as the reference's own tests
    // drive it (pkg/timex mock clock, topotest/mock_topo.go:208-235): the rule opens at the first ek_advance_time (or
    // at the first row); a row is delivered when the clock reaches its arrival timestamp, after every timer due at or
    // before it; ek_advance_time(now) moves the clock without rows. Rows arrive in timestamp order.
    //   TUMBLING / HOPPING: tickers from getAlignedWindowEndTime(start, rawInterval) every length / interval
    //     (window_op.go:228-233,250-260,471-481); a tick scans the rows with ts < tick (time-related windows) - the
    //     event-time pane / range machinery with E1 = the first tick and the watermark = the clock;
    //   SLIDING (no delay): each row matching OVER (WHEN) scans at its own timestamp over the rows delivered so far
    //     (window_op.go:353-379), [ts - length, ts] of the arrival prefix; a non-matching row garbage-collects the
    //     rows with ts + length <= its ts (gcInputs, window_op.go:657-673), which only matters for a row exactly at
    //     the left edge of a later trigger with the same timestamp;
    //   SESSION: the timeout timer re-armed by every row, the ticker every length (window_op.go:363-373,448-461,483-492).
    //   WHERE below TUMBLING / HOPPING / SESSION (windowPlan.go:82-99): rows are pre-filtered at delivery.
    void start_clock(int64_t t0) {
        clock_started = true;
        clock_ms = t0;
        if (wtype == EK_WINDOW_TUMBLING || wtype == EK_WINDOW_HOPPING) {
            e1_known = true;
            first_ts = t0;  // Exec sets triggerTime = now in processing time (window_op.go:149-151): the first windowStart
            E1 = aligned_end(t0, raw_interval, plan.time_unit, plan.tz_offset_s);
            grid.tumbling = wtype == EK_WINDOW_TUMBLING;
            grid.origin = grid.tumbling ? E1 : E1 - L;
            grid.P = P;
        } else if (wtype == EK_WINDOW_SESSION) {
            ps_tick = aligned_end(t0, raw_interval, plan.time_unit, plan.tz_offset_s);
        }
        if (proc_inc || proc_v2s) pi_start(t0);
    }

    // ---- batch statistics: one pass over ts (k_stats), or the shared ek_ts_stats the pushed batch carries (ABI v10:
    // computed once by ek_batch_ts_stats for every rule over the same source). GAP (hopping, lateTolerance 0): also the
    // widest arrival gap, seeded with the carried stream maximum.
    const ek_ts_stats* ts_hint = nullptr;   // set by push / push_global for the batch being pushed

    struct HintScope {   // the hint points into the caller's batch: valid for one push only
        const ek_ts_stats*& h;
        ~HintScope() { h = nullptr; }
    };

    void set_ts_hint(const ek_batch* b) {
        const ek_ts_stats* t = b ? b->ts_stats : nullptr;
        // bound to the exact column: same row count, ts column id AND column pointer (ABI v11)
        ts_hint = t && t->n_rows == b->n_rows && t->ts_column == dp.ts_col && dp.ts_col < user_cols &&
                          t->ts_data == b->columns[dp.ts_col] ? t : nullptr;
    }

    int batch_stats(const int64_t* ts, int64_t n, bool gap, int64_t seed, BatchStats* out) {
        if (ts_hint && ts_hint->n_rows == n) {
            BatchStats s{};
            s.min_ts = ts_hint->ts_min;
            s.max_ts = ts_hint->ts_max;
            s.unsorted = ts_hint->unsorted != 0;
            s.min_accepted = INT64_MAX;
            s.max_gap = INT64_MIN;
            if (gap) {
                s.max_gap = ts_hint->max_step;
                if (seed != INT64_MIN && n > 0) s.max_gap = std::max(s.max_gap, ts_hint->ts_first - seed);
            }
            *out = s;
            // the device copy too, as k_stats_reduce leaves it: later passes accumulate into it (k_hop_drop's
            // n_dropped); and the callers rely on the stats sync having drained the stream (pinned buffers are reused)
            if (int rc = ensure(bstats, sizeof(BatchStats))) return rc;
            *h_stats = s;
            hipMemcpyAsync(bstats.p, h_stats, sizeof(BatchStats), hipMemcpyHostToDevice, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "stream sync failed");
            return 0;
        }
        const int sblocks = (int)std::min<int64_t>(stats_blocks, std::max<int64_t>(1, (n / 2 + kBlock - 1) / kBlock));
        if (int rc = ensure(bstats_part, (size_t)sblocks * sizeof(BatchStats))) return rc;
        const int ph_s = phase_begin(EK_PHASE_STATS);
        if (gap)
            hipLaunchKernelGGL(k_stats<true>, dim3(sblocks), dim3(kBlock), 0, stream, ts, n, seed, (BatchStats*)bstats_part.p);
        else
            hipLaunchKernelGGL(k_stats<false>, dim3(sblocks), dim3(kBlock), 0, stream, ts, n, INT64_MIN, (BatchStats*)bstats_part.p);
        hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(1024), 0, stream, (const BatchStats*)bstats_part.p, sblocks,
                           (BatchStats*)bstats.p);
        phase_end(ph_s);
        hipMemcpyAsync(h_stats, bstats.p, sizeof(BatchStats), hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "stats kernel failed");
        *out = *h_stats;
        return 0;
    }

    // ---- the fused sorted pass (k_part MODE 3): a pane-mode batch presumed ts-sorted is partitioned straight from
    // its first and last timestamps, and the partition pass itself checks the presumption (sortedness, panes per
    // chunk, the hopping gap), writes the pane bounds and reports back in one read-back; the separate ts pass
    // (k_stats), its reduction, the pane-bounds search and one host round trip are gone. A batch that fails the
    // check is redone on the general path before any engine state changes (the pass only wrote scratch).
    struct FzPass { bool on; int64_t q_lo, nq; int mp, ls; const int64_t* pbnd; };
    FzPass fz_pass{};
    int fz_on = 0;            // EKGPU_FUSED=1: try the fused pass (default off)
    int fz_skip = 0;          // pushes that skip the attempt after a discarded pass (an unsorted stream pays once)
    DevBuf fz_buf;            // [FzStatus][ends 2][pbnd_out n_panes + 1]
    int64_t* h_fz = nullptr;  // pinned landing block
    size_t h_fz_cap = 0;
    static constexpr int kFzFallback = -1;
    static constexpr int64_t kFzMinRows = 1 << 16;

    bool fz_eligible(int64_t n) {
        // (WHERE plans keep the general path: k_part<3, WHERE> measured corrupted value registers on MI355X — the
        // interpreter call inside the partition loop with the direct-to-LDS ts loads of the tile)
        if (!fz_on || range_mode || gmode || ts_hint || plan.n_filter > 0 || dp.n_where > 0 || dp.pseudo_keys) return false;
        if (wtype != EK_WINDOW_TUMBLING && wtype != EK_WINDOW_HOPPING) return false;
        if (n < kFzMinRows || sorted_chunk != kTile || chunk < kTile) return false;
        if (fz_skip > 0) { fz_skip--; return false; }
        return true;
    }

    int push_fused(const DBatch& db, const int64_t* ts, int64_t n) {
        const size_t hdr = (sizeof(FzStatus) + 7) / 8 + 2;   // words before pbnd_out
        if (int rc = ensure(fz_buf, hdr * 8 + 64 * 8)) return rc;
        if (h_fz_cap < hdr + 64) {
            if (h_fz) { hipStreamSynchronize(stream); hipHostFree(h_fz); }
            h_fz_cap = std::max<size_t>(hdr + 64, 4096);
            if (hipHostMalloc((void**)&h_fz, h_fz_cap * 8) != hipSuccess) { h_fz = nullptr; h_fz_cap = 0; return fail(EK_ERR_NOMEM, "pinned"); }
        }
        FzStatus* d_st = (FzStatus*)fz_buf.p;
        int64_t* d_ends = (int64_t*)fz_buf.p + hdr - 2;
        hipLaunchKernelGGL(k_fz_prep, dim3(1), dim3(64), 0, stream, ts, n, d_st, d_ends);
        hipMemcpyAsync(h_fz, d_ends, 16, hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "fused pass: ts read failed");
        const int64_t t0 = h_fz[0], t1 = h_fz[1];
        const int64_t T = plan.late_tolerance_ms;
        if (t0 > t1) { fz_skip = 8; return kFzFallback; }     // not sorted: the general path
        if (has_M && t0 < M - T) return kFzFallback;           // a late prefix: the general path drops it
        const int64_t M1 = has_M ? std::max(M, t1) : t1, W1 = M1 - T;
        const bool hop_gap = wtype == EK_WINDOW_HOPPING && T == 0;
        if (hop_gap && has_M && t0 - M > L) return kFzFallback;   // the empty-window discard pass (k_hop_drop)
        // the first window's alignment, tentatively (restored if the pass is discarded)
        const bool e1_was = e1_known;
        const int64_t E1_was = E1, first_was = first_ts;
        const PaneGrid grid_was = grid;
        auto restore = [&]() { e1_known = e1_was; E1 = E1_was; first_ts = first_was; grid = grid_was; };
        if (!e1_known) {
            if (pend_n != 0 || W1 < t0) return kFzFallback;
            first_ts = t0;
            E1 = aligned_end(first_ts, raw_interval, plan.time_unit, plan.tz_offset_s);
            grid.tumbling = wtype == EK_WINDOW_TUMBLING;
            grid.origin = grid.tumbling ? E1 : E1 - L;
            grid.P = P;
        }
        int64_t q_lo = std::max<int64_t>(0, pane_host(t0));
        const int64_t q_hi = pane_host(t1);
        q_lo = std::max(q_lo, win_first_pane(next_win));
        const int64_t nq = q_hi - q_lo + 1;
        if (q_hi < 0 || nq < 1 || nq > max_panes_group || n > group_events || (size_t)nq + 1 + hdr > (size_t)INT32_MAX) {
            restore();
            return kFzFallback;
        }
        // panes a 4096-row chunk may span: from the batch's mean rows per pane (a chunk past it discards the pass)
        const int64_t per_pane = std::max<int64_t>(1, n / nq);
        int mp = (int)std::min<int64_t>(nq, std::max<int64_t>(2, (kTile + per_pane - 1) / per_pane + 1));
        mp = std::min(mp, std::min(kMaxChunkBnd + 1, np_max / std::max(1, NB)));
        if (mp < 1 || (int64_t)NB * mp > np_max) { restore(); return kFzFallback; }
        if (int rc = ensure(fz_buf, (hdr + (size_t)nq + 1) * 8)) { restore(); return rc; }
        if (h_fz_cap < hdr + (size_t)nq + 1) {
            hipHostFree(h_fz);
            h_fz_cap = std::max<size_t>(hdr + nq + 1, 2 * h_fz_cap);
            if (hipHostMalloc((void**)&h_fz, h_fz_cap * 8) != hipSuccess) { h_fz = nullptr; h_fz_cap = 0; restore(); return fail(EK_ERR_NOMEM, "pinned"); }
        }
        hipMemsetAsync(fz_buf.p, 0, sizeof(FzStatus), stream);   // (ensure may have moved the block)
        GroupDesc gd{};
        gd.lo = 0;
        gd.hi = n;
        gd.q_lo = q_lo;
        gd.n_panes = (int32_t)nq;
        gd.nb = NB;
        gd.kbits = kbits;
        gd.chunk = kTile;
        gd.abase = 0;
        gd.nch = (int32_t)((n + kTile - 1) / kTile);
        gd.np = (int32_t)nq * NB;
        gd.ring = ring;
        gd.has_accept = 0;
        gd.sorted = 1;
        gd.key_col = dp.key_col;
        gd.ts_col = dp.ts_col;
        gd.n_where = dp.n_where;
        gd.num_keys = dp.num_keys;
        gd.nbatch = n;
        gd.pad = env_int("EKGPU_DEBUG_AGG", 0);
        gd.pad2 = variant;
        gd.fz_mp = mp;
        gd.fz_gap = hop_gap ? 1 : 0;
        gd.pbnd_out = (int64_t*)fz_buf.p + hdr;
        gd.fz_st = (FzStatus*)fz_buf.p;
        const int ls = NB * mp + 1;
        // the same staging / run-table buffers (and sizes) launch_part_agg uses for this group
        const int64_t ne = (int64_t)gd.nch * kTile + 64;
        if (ne > st_cap) {
            if (int rc = ensure(st_klo, (size_t)ne * 2)) { restore(); return rc; }
            for (int v = 0; v < dp.n_vc; ++v) {
                if (int rc = ensure(st_val[v], (size_t)ne * 8)) { restore(); return rc; }
                if ((plan.nullable_mask >> dp.vc_col[v]) & 1u)
                    if (int rc = ensure(st_valid[v], (size_t)ne)) { restore(); return rc; }
            }
            st_cap = ne;
        }
        Staging st{};
        st.klo = (uint16_t*)st_klo.p;
        bool any_nullable = false;
        for (int v = 0; v < dp.n_vc; ++v) {
            st.val[v] = (int64_t*)st_val[v].p;
            if (db.valid[dp.vc_col[v]]) {
                st.valid[v] = (uint8_t*)st_valid[v].p;
                st.nullable_mask |= 1u << v;
                any_nullable = true;
            }
        }
        if (int rc = ensure(chist, (size_t)gd.nch * ls * 4)) { restore(); return rc; }
        if (int rc = ensure(chunk_pa, (size_t)gd.nch * 4)) { restore(); return rc; }
        gd.cpa = (int32_t*)chunk_pa.p;
        {
            const int nvc = std::max(1, dp.n_vc);
            const size_t lds_p = std::max(part_lds_bytes(nvc, ls - 1, any_nullable, true), fz_lds_bytes(ls - 1));
            const int ph = phase_begin(EK_PHASE_PARTITION);
            ek::launch_part(3, dp.n_where > 0, nvc, dim3(gd.nch), lds_p, stream, d_plan, db, grid, gd, nullptr, st,
                            (uint32_t*)chist.p, ls, kTile, (int32_t*)pane_err.p);
            phase_end(ph);
        }
        hipMemcpyAsync(h_fz, fz_buf.p, (hdr + (size_t)nq + 1) * 8, hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) { restore(); return fail(EK_ERR_DEVICE, "fused partition pass failed"); }
        const FzStatus fs = *(const FzStatus*)h_fz;
        int64_t* pb = h_fz + hdr;
        pb[0] = 0;
        pb[nq] = n;
        bool ok = !fs.unsorted && !fs.overflow && (!hop_gap || (int64_t)fs.max_gap <= L);
        if (ok) {
            // the general path's grouping would form exactly this one group with single-tile chunks
            const int64_t pane_cap = (int64_t)(kMaxRuns - 2) * chunk;
            for (int64_t k = 0; k < nq && ok; ++k) ok = pb[k + 1] - pb[k] <= std::min(group_events, pane_cap);
            GroupDesc chk = gd;
            ok = ok && max_chunks_in_pane(pb, chk, kTile) <= kMaxRuns && max_panes_in_chunk(pb, chk, kTile) <= mp;
        }
        if (!ok) {
            restore();
            fz_skip = 8;
            stats.fused_discarded++;
            return kFzFallback;
        }
        // ---- commit: the batch is sorted, nothing is late; the rest is the general path's sorted branch
        int64_t arrival_base = arrivals;
        arrivals += n;
        h_wdesc_used = 0;   // the read-back sync drained every earlier descriptor upload
        h_desc_used = 0;
        aux_used = 0;
        if (!has_M || t1 > M) {
            M = t1;
            has_M = true;
            W = M - T;
            has_W = true;
        }
        if (!e1_was) e1_known = true;   // (E1 / grid / first_ts set above, as the general path's step 4)
        stats.fused_batches++;
        fz_pass = FzPass{true, q_lo, nq, mp, ls, pb};
        int64_t save = arrivals;
        arrivals = arrival_base;
        const int rc = process(db, true, 0, nullptr, t0, t1, nullptr);
        arrivals = save;
        fz_pass = FzPass{};
        return rc;
    }

    // ek_batch_ts_stats: the shareable form of the statistics above
    int ts_stats_of(const ek_batch* b, ek_ts_stats* out) {
        if (!b || !out) return fail(EK_ERR_INVALID, "null batch / output");
        if (dp.ts_col < 0 || dp.ts_col >= user_cols) return fail(EK_ERR_STATE, "the rule has no timestamp column");
        const int64_t n = b->n_rows;
        if (n < 0 || !b->columns[dp.ts_col]) return fail(EK_ERR_INVALID, "bad batch");
        ek_ts_stats t{};
        t.n_rows = n;
        t.ts_column = dp.ts_col;
        t.ts_min = INT64_MAX;
        t.ts_max = INT64_MIN;
        t.max_step = INT64_MIN;
        t.ts_data = b->columns[dp.ts_col];
        if (n > 0 && b->memory == EK_MEM_HOST) {
            const int64_t* ts = (const int64_t*)b->columns[dp.ts_col];
            t.ts_first = ts[0];
            for (int64_t i = 0; i < n; ++i) {
                t.ts_min = std::min(t.ts_min, ts[i]);
                t.ts_max = std::max(t.ts_max, ts[i]);
                if (i > 0) { t.unsorted |= ts[i] < ts[i - 1]; t.max_step = std::max(t.max_step, ts[i] - ts[i - 1]); }
            }
        } else if (n > 0) {
            const int64_t* ts = (const int64_t*)b->columns[dp.ts_col];
            const ek_ts_stats* keep = ts_hint;
            ts_hint = nullptr;
            BatchStats s;
            const int rc = batch_stats(ts, n, true, INT64_MIN, &s);
            ts_hint = keep;
            if (rc) return rc;
            hipMemcpyAsync(h_stats, ts, 8, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "ts copy failed");
            t.ts_first = h_stats->min_ts;   // the pinned stats block doubles as the 8-byte landing slot
            t.ts_min = s.min_ts;
            t.ts_max = s.max_ts;
            t.unsorted = s.unsorted != 0;
            t.max_step = s.max_gap;
        }
        *out = t;
        return 0;
    }

    int push_proc(DBatch db) {
        const int64_t n = db.n;
        const int64_t* ts = (const int64_t*)db.col[dp.ts_col];
        BatchStats s;
        if (int rc = batch_stats(ts, n, false, INT64_MIN, &s)) return rc;
        if (s.unsorted) return fail(EK_ERR_INVALID, "processing-time rows must arrive in timestamp order (their arrival times)");
        if (!clock_started) start_clock(s.min_ts);
        else if (s.min_ts < clock_ms)
            return fail(EK_ERR_INVALID, "processing-time row at %lld is older than the clock (%lld)", (long long)s.min_ts,
                        (long long)clock_ms);
        const int64_t arrival_base = arrivals;
        arrivals += n;
        h_wdesc_used = 0;   // the stats sync above drained every earlier descriptor upload
        h_desc_used = 0;
        aux_used = 0;
        if (proc_pushdown)
            if (int rc = proc_prefilter(db, arrival_base)) { g_row_arr = nullptr; return rc; }
        const int rc = proc_deliver(db, arrival_base, s.min_ts, s.max_ts);
        g_row_arr = nullptr;
        return rc;
    }

    // WHERE pushed below the window: the rows whose WHERE is true, compacted (stable), with their arrival indices as
    // the batch's row arrivals (g_row_arr). A row whose WHERE errors is dropped and counted (FilterOp forwards its error).
    DevBuf pf_cols[EK_MAX_COLUMNS], pf_valid[EK_MAX_COLUMNS], pf_arr, filt_d;
    int proc_prefilter(DBatch& db, int64_t arrival_base) {
        const int64_t n = db.n;
        if (int rc = ensure(flags_d, (size_t)n)) return rc;
        if (int rc = ensure(trig_d, (size_t)n * 8)) return rc;
        const int nb = (int)((n + kCompactTile - 1) / kCompactTile);
        if (int rc = ensure(cnts_d, (size_t)(nb + 2) * 8)) return rc;
        hipMemsetAsync((int64_t*)cnts_d.p + nb + 1, 0, 8, stream);
        hipLaunchKernelGGL(k_filter_flags, dim3((int)std::min<int64_t>(8192, (n + 255) / 256)), dim3(256), 0, stream, d_plan_where, db,
                           (uint8_t*)flags_d.p, (unsigned long long*)((int64_t*)cnts_d.p + nb + 1));
        hipLaunchKernelGGL(k_flag_count, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n, (int64_t*)cnts_d.p);
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, stream, (int64_t*)cnts_d.p, nb);
        hipLaunchKernelGGL(k_flag_write, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n, (const int64_t*)cnts_d.p,
                           (int64_t)0, (int64_t*)trig_d.p);
        int64_t sel_err[2] = {0, 0};
        hipMemcpyAsync(sel_err, (int64_t*)cnts_d.p + nb, 16, hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "pre-filter failed");
        const int64_t ns = sel_err[0];
        stats.records_filter_error += sel_err[1];
        DBatch fb{};
        fb.n = ns;
        const int g = (int)std::min<int64_t>(8192, std::max<int64_t>(1, (ns + 255) / 256));
        for (int c = 0; c < plan.n_columns; ++c) {
            const int es = plan.column_type[c] == EK_COL_U32 ? 4 : 8;
            if (int rc = ensure(pf_cols[c], (size_t)std::max<int64_t>(ns, 1) * es)) return rc;
            uint8_t* vd = nullptr;
            if (db.valid[c]) {
                if (int rc = ensure(pf_valid[c], (size_t)std::max<int64_t>(ns, 1))) return rc;
                vd = (uint8_t*)pf_valid[c].p;
            }
            if (ns > 0)
                hipLaunchKernelGGL(k_compact_col, dim3(g), dim3(256), 0, stream, (const int64_t*)trig_d.p, ns, db.col[c], es,
                                   db.valid[c], pf_cols[c].p, vd);
            fb.col[c] = pf_cols[c].p;
            fb.valid[c] = vd;
        }
        if (int rc = ensure(pf_arr, (size_t)std::max<int64_t>(ns, 1) * 8)) return rc;
        if (ns > 0)
            hipLaunchKernelGGL(k_offset_idx, dim3(g), dim3(256), 0, stream, (const int64_t*)trig_d.p, ns, arrival_base,
                               (int64_t*)pf_arr.p);
        g_row_arr = (const int64_t*)pf_arr.p;
        db = fb;
        return 0;
    }

    // the clock moves to max_ts delivering the batch's rows (timers due at or before each row fire first)
    int proc_deliver(const DBatch& db, int64_t arrival_base, int64_t min_ts, int64_t max_ts) {
        if (!has_M || max_ts > M) { M = max_ts; has_M = true; }
        W = max_ts;
        has_W = true;
        int rc = 0;
        if (range_mode) {
            if (db.n > 0)
                if (int r = eb_append(db, 0, db.n, arrival_base)) return r;
            const int64_t rel_prev = eb_rel;
            eb_rel = eb.n;
            rc = range_triggers(rel_prev);
            if (!rc && wtype == EK_WINDOW_SLIDING && !proc_inc && !proc_v2s) rc = proc_slide_floor();
        } else if (db.n > 0) {
            const int64_t save = arrivals;
            arrivals = arrival_base;
            rc = process(db, true, 0, nullptr, min_ts, max_ts, g_row_arr);
            arrivals = save;
        } else {
            rc = proc_close();
        }
        clock_ms = max_ts;
        return rc;
    }

    // pane mode, no rows: every window whose tick is due fires (its panes can no longer receive rows)
    int proc_close() {
        if (!e1_known || W < win_end(next_win)) return 0;
        return finalize_ready(INT64_MAX);   // windows no row reached are reported empty, without result rows
    }

    int advance_time(int64_t now) {
        if (!proc) return fail(EK_ERR_STATE, "ek_advance_time drives processing-time TUMBLING / HOPPING / SLIDING / SESSION windows");
        if (!clock_started) { start_clock(now); return 0; }
        if (now < clock_ms) return fail(EK_ERR_INVALID, "the clock cannot move back (%lld < %lld)", (long long)now, (long long)clock_ms);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "stream failed");
        if (int rc = fold_time()) return rc;
        hipEventRecord(ev0, stream);
        h_wdesc_used = 0;
        h_desc_used = 0;
        aux_used = 0;
        W = now;
        has_W = true;
        int rc = 0;
        if (range_mode) {
            rc = range_triggers(eb_rel);
            if (!rc && wtype == EK_WINDOW_SLIDING && !proc_inc && !proc_v2s) rc = proc_slide_floor();
        } else {
            rc = proc_close();
        }
        clock_ms = now;
        return rc ? rc : record_time();
    }

    // SLIDING: one window per delivered row matching OVER (WHEN), over the rows delivered up to it:
    // [lb(ts - length), row]; the left edge moves one ms in when a non-matching row with the same ts as the trigger
    // arrived before it (its gcInputs dropped the rows with ts + length <= ts).
    int proc_slide_triggers(int64_t rel_prev, std::vector<PendWin>& pw) {
        const int64_t n_new = eb_rel - rel_prev;
        if (n_new <= 0) return slide_delay > 0 ? proc_slide_delayed(rel_prev, {}, {}, pw) : 0;
        if (int rc = ensure(flags_d, (size_t)n_new)) return rc;
        if (int rc = ensure(trig_d, (size_t)n_new * 8)) return rc;
        const int nb = (int)((n_new + kCompactTile - 1) / kCompactTile);
        if (int rc = ensure(cnts_d, (size_t)(nb + 1) * 8)) return rc;
        const DBatch bv = buffer_view();
        hipLaunchKernelGGL(k_trigger_flags, dim3((int)std::min<int64_t>(4096, (n_new + 255) / 256)), dim3(256), 0, stream,
                           d_plan, bv, rel_prev, eb_rel, (uint8_t*)flags_d.p);
        hipLaunchKernelGGL(k_flag_count, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n_new, (int64_t*)cnts_d.p);
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, stream, (int64_t*)cnts_d.p, nb);
        hipLaunchKernelGGL(k_flag_write, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n_new,
                           (const int64_t*)cnts_d.p, rel_prev, (int64_t*)trig_d.p);
        const int64_t nt = fetch_i64((const int64_t*)cnts_d.p + nb);
        std::vector<int64_t> pos(std::max<int64_t>(nt, 0)), tts(std::max<int64_t>(nt, 0));
        if (nt > 0) hipMemcpyAsync(pos.data(), trig_d.p, (size_t)nt * 8, hipMemcpyDeviceToHost, stream);
        if (int rc = ensure(mrg_col, (size_t)(nt + 1) * 24)) return rc;
        int64_t* g_ts = (int64_t*)mrg_col.p;
        if (nt > 0) {
            hipLaunchKernelGGL(k_gather8, dim3((int)std::min<int64_t>(4096, (nt + 255) / 256)), dim3(256), 0, stream,
                               (const int64_t*)trig_d.p, nt, INT64_MAX, (const int64_t*)eb.col[dp.ts_col].p,
                               (const int64_t*)nullptr, (const int64_t*)nullptr, g_ts);
            hipMemcpyAsync(tts.data(), g_ts, (size_t)nt * 8, hipMemcpyDeviceToHost, stream);
        }
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "trigger copy failed");
        if (slide_delay > 0 && send_twice) {
            // send-twice keeps a host mirror of which delivered rows matched OVER (WHEN) (the others gcInputs)
            const size_t o = h_rtrig.size();
            h_rtrig.resize(o + n_new);
            hipMemcpyAsync(h_rtrig.data() + o, flags_d.p, (size_t)n_new, hipMemcpyDeviceToHost, stream);
        }
        if (slide_delay > 0) return proc_slide_delayed(rel_prev, pos, tts, pw);
        // the latest non-matching row before each trigger (its ts decides the gcInputs edge): the row just before the
        // trigger unless that row is a trigger too (then the same as that trigger's); rows before this batch: carried
        std::vector<int64_t> qpos;            // batch rows whose ts is needed (non-matching predecessors, the last row)
        std::vector<int64_t> nm_ref(std::max<int64_t>(nt, 0));   // >= 0: index into qpos; -1: the carried value
        for (int64_t k = 0; k < nt; ++k) {
            if (k > 0 && pos[k - 1] == pos[k] - 1) { nm_ref[k] = nm_ref[k - 1]; continue; }
            if (pos[k] - 1 >= rel_prev) { nm_ref[k] = (int64_t)qpos.size(); qpos.push_back(pos[k] - 1); }
            else nm_ref[k] = -1;
        }
        const bool last_is_trig = nt > 0 && pos[nt - 1] == eb_rel - 1;
        int64_t last_ref = -1;
        if (!last_is_trig) { last_ref = (int64_t)qpos.size(); qpos.push_back(eb_rel - 1); }
        std::vector<int64_t> qts(qpos.size());
        if (!qpos.empty()) {
            const int64_t nq = (int64_t)qpos.size();
            int64_t* d_q = g_ts + nt;
            hipMemcpyAsync(d_q, qpos.data(), (size_t)nq * 8, hipMemcpyHostToDevice, stream);
            hipLaunchKernelGGL(k_gather8, dim3((int)std::min<int64_t>(4096, (nq + 255) / 256)), dim3(256), 0, stream, d_q, nq,
                               INT64_MAX, (const int64_t*)eb.col[dp.ts_col].p, (const int64_t*)nullptr, (const int64_t*)nullptr,
                               d_q + nq);
            hipMemcpyAsync(qts.data(), d_q + nq, (size_t)nq * 8, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "trigger copy failed");
        }
        std::vector<int64_t> prevts(std::max<int64_t>(nt, 0));
        for (int64_t k = 0; k < nt; ++k) prevts[k] = nm_ref[k] >= 0 ? qts[nm_ref[k]] : ps_last_nonmatch;
        ps_last_nonmatch = last_is_trig ? prevts[nt - 1] : qts[last_ref];
        for (int64_t k = 0; k < nt; ++k) {
            const int64_t t = tts[k];
            PendWin p{};
            p.q.kind = RB_UPTO;
            p.q.lo_ts = prevts[k] == t ? t - L + 1 : t - L;
            p.q.pos = pos[k];
            p.q.floor = eb_floor;
            p.start = t - L;   // scan(): windowStart = t - length (window_op.go:697-707)
            p.end = t;
            pw.push_back(p);
        }
        return 0;
    }
    // Delayed SLIDINGWINDOW(unit, L, D) in processing time (window_op.go:355-373,325-337): a trigger row at t arms a
    // timer due at t + D; when the clock reaches it (before any row stamped t + D) the window scans [t - L, t + D).
    // With enableSlidingWindowSendTwice the trigger first scans (t - L, t] over the rows delivered up to it and the
    // timer (t, t + D]; handleInputsForSlidingWindow (window_op.go:576-603) then keeps only the EXPIRED prefix of the
    // inputs (ts < windowEnd - L - D) whenever some input expired: restated on the host over the mirror of the
    // delivered timestamps as an inert expired set sw2_e (its rows are never in a later window) and the index sw2_cut
    // from which delivered rows are live. Windows are fired in clock order, a timer before a trigger at the same ms.
    int64_t slide_delay = 0;            // SLIDINGWINDOW delay (ms); > 0: proc_dq holds the armed timers (trigger ts)
    bool send_twice = false;
    std::vector<int64_t> proc_dq;
    size_t proc_dq_head = 0;
    std::vector<int64_t> sw2_e;         // send-twice: ts of the expired inputs the reference keeps
    int64_t sw2_cut = 0;                // send-twice: absolute buffer index of the first live input
    int64_t sw2_gcb = INT64_MIN;        // send-twice: the gcInputs bound so far (inputs with ts <= it are gone)
    int64_t sw2_gcx = 0;                // send-twice: absolute index up to which sw2_gcb accounts for the rows
    std::vector<uint8_t> h_rtrig;       // send-twice: OVER (WHEN) flag of each mirrored row (h_rts)
    int proc_slide_delayed(int64_t rel_prev, const std::vector<int64_t>& pos, const std::vector<int64_t>& tts,
                           std::vector<PendWin>& pw) {
        const int64_t D = slide_delay;
        if (!send_twice) {
            for (int64_t t : tts) proc_dq.push_back(t);
            while (proc_dq_head < proc_dq.size() && proc_dq[proc_dq_head] + D <= W) {
                const int64_t t = proc_dq[proc_dq_head++];
                PendWin p{};
                p.q.kind = RB_LB;
                p.q.lo_ts = t - L;
                p.q.hi_ts = t + D;
                p.q.floor = eb_floor;
                p.start = t - L;   // scan(t + D, length + delay): windowStart = windowEnd - (L + D)
                p.end = t + D;
                pw.push_back(p);
            }
        } else {
            // host mirror of the delivered timestamps [h_rts_base, ...) (h_rtrig: their OVER (WHEN) flags, copied by
            // proc_slide_triggers)
            const int64_t n_new = eb_rel - rel_prev;
            if (h_rts.empty()) h_rts_base = eb_base + rel_prev;
            if (n_new > 0) {
                const size_t o = h_rts.size();
                h_rts.resize(o + n_new);
                hipMemcpyAsync(h_rts.data() + o, (const int64_t*)eb.col[dp.ts_col].p + rel_prev, (size_t)n_new * 8,
                               hipMemcpyDeviceToHost, stream);
                if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "timestamp mirror copy failed");
            }
            if (h_rtrig.size() < h_rts.size()) h_rtrig.resize(h_rts.size(), 0);
            if (sw2_cut < h_rts_base) sw2_cut = h_rts_base;
            auto ts_at = [&](int64_t abs) { return h_rts[abs - h_rts_base]; };
            auto first_gt = [&](int64_t lo, int64_t hi, int64_t x) {   // first abs index in [lo, hi) with ts > x
                return h_rts_base + (std::upper_bound(h_rts.begin() + (lo - h_rts_base), h_rts.begin() + (hi - h_rts_base), x) - h_rts.begin());
            };
            auto first_ge = [&](int64_t lo, int64_t hi, int64_t x) {   // first abs index in [lo, hi) with ts >= x
                return h_rts_base + (std::lower_bound(h_rts.begin() + (lo - h_rts_base), h_rts.begin() + (hi - h_rts_base), x) - h_rts.begin());
            };
            // gcInputs of every non-matching row delivered before index x (window_op.go:376-378): it drops the inputs
            // with ts + L + D <= its ts; the bound only grows, so applied lazily as "ts > gc bound"
            auto gc_bound = [&](int64_t x) {   // (rows before sw2_gcx are in sw2_gcb already: each row is walked once)
                for (int64_t k = x - 1; k >= std::max(sw2_gcx, h_rts_base); --k)
                    if (!h_rtrig[k - h_rts_base]) return std::max(sw2_gcb, ts_at(k) - L - D);
                return sw2_gcb;
            };
            // one scan over the inputs delivered before index `delivered`: content (ws, we], then the expired-prefix
            // rule of handleInputsForSlidingWindow
            auto scan2 = [&](int64_t ws, int64_t we, int64_t delivered) {
                const int64_t gcb = gc_bound(delivered);
                sw2_gcb = gcb;
                sw2_gcx = std::max(sw2_gcx, delivered);
                const int64_t live0 = std::max(sw2_cut, first_gt(sw2_cut, delivered, gcb));
                const int64_t a = std::max(live0, first_gt(live0, delivered, ws));
                const int64_t b = std::max(a, first_gt(a, delivered, we));
                PendWin p{};
                p.q.kind = RB_FIXED;
                p.q.pos = a - eb_base;
                p.q.rstep = b - eb_base;
                p.start = ws;
                p.end = we;
                pw.push_back(p);
                const int64_t dl = we - (L + D);
                const size_t e0 = std::upper_bound(sw2_e.begin(), sw2_e.end(), gcb) - sw2_e.begin();   // gc'd expired rows
                const int64_t ne = std::max<int64_t>(0, (std::lower_bound(sw2_e.begin(), sw2_e.end(), dl) - sw2_e.begin()) - (int64_t)e0);
                const int64_t nl = first_ge(live0, delivered, dl) - live0;
                const int64_t present = (int64_t)(sw2_e.size() - e0) + (delivered - live0);
                if (ne + nl == 0) return;
                if (ne + nl == present) {
                    sw2_e.clear();
                } else {
                    sw2_e.erase(sw2_e.begin(), sw2_e.begin() + (int64_t)e0);
                    sw2_e.resize((size_t)ne);
                    for (int64_t k = 0; k < nl; ++k) sw2_e.push_back(ts_at(live0 + k));
                }
                sw2_cut = delivered;
            };
            const int64_t end_abs = eb_base + eb_rel;
            size_t k = 0;
            for (;;) {
                const int64_t due = proc_dq_head < proc_dq.size() ? proc_dq[proc_dq_head] + D : INT64_MAX;
                const int64_t tn = k < tts.size() ? tts[k] : INT64_MAX;
                if (due <= tn && due <= W) {
                    // the second part (t, t + D] over the rows delivered before the timer (ts < t + D)
                    const int64_t t = proc_dq[proc_dq_head++];
                    scan2(t, t + D, first_ge(sw2_cut, end_abs, t + D));
                } else if (tn != INT64_MAX) {
                    // the first part (t - L, t] over the rows delivered up to the trigger
                    scan2(tn - L, tn, eb_base + pos[k] + 1);
                    proc_dq.push_back(tn);
                    ++k;
                } else {
                    break;
                }
            }
            sw2_gcb = gc_bound(end_abs);
            sw2_gcx = end_abs;
            eb_floor = std::max(eb_floor, sw2_cut - eb_base);
            const int64_t drop = sw2_cut - h_rts_base;
            if (drop > 65536 && drop * 2 > (int64_t)h_rts.size()) {
                h_rts.erase(h_rts.begin(), h_rts.begin() + drop);
                h_rtrig.erase(h_rtrig.begin(), h_rtrig.begin() + drop);
                h_rts_base = sw2_cut;
            }
        }
        if (proc_dq_head > 4096 && proc_dq_head * 2 > proc_dq.size()) {
            proc_dq.erase(proc_dq.begin(), proc_dq.begin() + (int64_t)proc_dq_head);
            proc_dq_head = 0;
        }
        return 0;
    }

    // rows older than clock - length - delay can no longer be in a window (every later trigger is at or after the
    // clock; a pending delayed window of trigger t > clock - delay starts at t - length)
    int proc_slide_floor() {
        if (eb_rel <= eb_floor) return 0;
        const int64_t bound = W - L - slide_delay;
        if (int rc = ensure(bounds_val, 8)) return rc;
        if (int rc = ensure(bounds_idx, 8)) return rc;
        hipMemcpyAsync(bounds_val.p, &bound, 8, hipMemcpyHostToDevice, stream);
        hipLaunchKernelGGL(k_lower_bound, dim3(1), dim3(64), 0, stream, (const int64_t*)eb.col[dp.ts_col].p, eb_floor, eb_rel,
                           (const int64_t*)bounds_val.p, 1, (int64_t*)bounds_idx.p);
        eb_floor = std::max(eb_floor, fetch_i64((const int64_t*)bounds_idx.p));
        return 0;
    }

    // SESSION: the delivered rows' timestamps are mirrored on the host and the timers replayed in due order:
    // the ticker (due ps_tick, every length) closes the inputs when the first one is at least length old; the timeout
    // (due ps_to_due, re-armed by every row) closes them. A close takes every input (all are older than the clock).
    int proc_session_triggers(int64_t rel_prev, std::vector<PendWin>& pw) {
        const int64_t n_new = eb_rel - rel_prev;
        if (h_rts.empty()) { h_rts_base = eb_base + rel_prev; if (ps_next_abs < h_rts_base) ps_next_abs = h_rts_base; }
        if (n_new > 0) {
            const size_t o = h_rts.size();
            h_rts.resize(o + n_new);
            hipMemcpyAsync(h_rts.data() + o, (const int64_t*)eb.col[dp.ts_col].p + rel_prev, (size_t)n_new * 8, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "session mirror copy failed");
        }
        int64_t floor_abs = eb_base + eb_floor;
        const int64_t end_abs = eb_base + eb_rel;
        auto close = [&](int64_t at, int64_t upto_abs) {
            PendWin p{};
            p.q.kind = RB_FIXED;
            p.q.pos = floor_abs - eb_base;
            p.q.rstep = upto_abs - eb_base;
            int64_t ws = sess_has_trigger ? sess_trigger : 0;
            if (ws <= 0) ws = at - L;
            p.start = ws;
            p.end = at;
            pw.push_back(p);
            floor_abs = upto_abs;
            sess_trigger = at;
            sess_has_trigger = true;
        };
        // timers due at or before `now` with `upto_abs` rows delivered (ticker first on a tie)
        auto timers = [&](int64_t now, int64_t upto_abs) {
            for (;;) {
                const bool tk = ps_tick <= now;
                const bool tm = ps_to_armed && ps_to_due <= now && (!tk || ps_to_due < ps_tick);
                if (tm) {
                    ps_to_armed = false;
                    if (floor_abs < upto_abs) { close(ps_to_due, upto_abs); ps_to_exists = false; }
                } else if (tk) {
                    if (floor_abs < upto_abs && ps_tick - h_rts[floor_abs - h_rts_base] >= L) close(ps_tick, upto_abs);
                    ps_tick += L;
                } else {
                    break;
                }
            }
        };
        for (int64_t r = ps_next_abs; r < end_abs; ++r) {
            const int64_t t = h_rts[r - h_rts_base];
            timers(t, r);
            if (!ps_to_exists) { ps_to_exists = true; sess_trigger = t; sess_has_trigger = true; }
            ps_to_armed = true;
            ps_to_due = t + H;
        }
        ps_next_abs = end_abs;
        timers(W, end_abs);
        const int64_t drop = floor_abs - h_rts_base;
        if (drop > 65536 && drop * 2 > (int64_t)h_rts.size()) {
            h_rts.erase(h_rts.begin(), h_rts.begin() + drop);
            h_rts_base = floor_abs;
        }
        return 0;
    }

    // Event-time push in range mode, after the shared late-drop / watermark steps.
    int push_range(const DBatch& db, bool sorted, int64_t start, const uint8_t* d_acc, int64_t n_acc, int64_t min_acc,
                   int64_t max_ts, int64_t arrival_base, int64_t M_prev, bool had_M, int64_t batch_min) {
        const int64_t n = db.n;
        const int64_t* ts = (const int64_t*)db.col[dp.ts_col];
        cur_arr_base = arrival_base;
        cur_nb = n;
        cur_prevmax = had_M ? M_prev : INT64_MIN;
        // running max of the batch: release steps (sliding) and the step at which W was reached
        if (sorted && (!had_M || batch_min >= M_prev)) runmax_p = ts;
        else if (int rc = batch_runmax(ts, n, had_M ? M_prev : INT64_MIN)) return rc;
        if (n_acc > 0) {
            if (sorted && !d_acc && (eb.n == 0 || !had_M || min_acc >= M_prev)) {
                if (int rc = eb_append(db, start, n_acc, arrival_base)) return rc;
            } else {
                int64_t max_acc = max_ts;
                if (int rc = eb_merge(db, start, d_acc, n_acc, min_acc, max_acc, arrival_base)) return rc;
            }
        }
        // the watermark's step: first arrival whose running max reached M (only if M advanced in this batch), and the
        // released end of the buffer at (W, sW): one launch, one round trip
        const int64_t rel_prev = eb_rel;
        const bool first = !had_M || max_ts > M_prev;
        if (first || eb.n > 0) {
            if (int rc = ensure(bounds_idx, 16)) return rc;
            hipLaunchKernelGGL(k_rel_bounds, dim3(1), dim3(64), 0, stream, runmax_p, n, max_ts, first ? 1 : 0, arrival_base, sW,
                               eb.n > 0 ? (const int64_t*)eb.col[dp.ts_col].p : (const int64_t*)nullptr, arr_ptr(), eb_arr0,
                               eb.n, W, (int64_t*)bounds_idx.p);
            int64_t out2[2] = {0, 0};
            hipMemcpyAsync(out2, bounds_idx.p, 16, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "release bounds failed");
            sW = out2[0];
            if (eb.n > 0) eb_rel = std::max(eb_rel, out2[1]);
        }
        if (need_rel && eb_rel > rel_prev) {
            const int g = (int)std::min<int64_t>(4096, (eb_rel - rel_prev + 255) / 256);
            hipLaunchKernelGGL(k_release_step, dim3(g), dim3(256), 0, stream, (const int64_t*)eb.col[dp.ts_col].p,
                               arr_ptr(), eb_arr0, rel_prev, eb_rel, runmax_p, n, arrival_base,
                               had_M ? M_prev : INT64_MIN, plan.late_tolerance_ms, (int64_t*)eb.rel.p);
        }
        const int rc = range_triggers(rel_prev);
        runmax_p = (const int64_t*)runmax_d.p;   // never an alias of a batch column past its push
        return rc;
    }

    // Window-less rule (SELECT * ... WHERE): FilterOp.Apply per event (filter_operator.go:36-90). Each push
    // yields one result segment whose rows are the events that passed, in arrival order: key = row index
    // in the batch, value k = column k (SELECT *). A row whose WHERE errors is dropped and counted
    // (the reference forwards that event's error instead of the event).
    int push_filter(const DBatch& db) {
        const int64_t n = db.n;
        if (int rc = ensure(flags_d, (size_t)n)) return rc;
        if (int rc = ensure(trig_d, (size_t)n * 8)) return rc;
        const int nb = (int)((n + kCompactTile - 1) / kCompactTile);
        if (int rc = ensure(cnts_d, (size_t)(nb + 2) * 8)) return rc;
        hipMemsetAsync((int64_t*)cnts_d.p + nb + 1, 0, 8, stream);
        const int ph = phase_begin(EK_PHASE_PARTITION);
        hipLaunchKernelGGL(k_filter_flags, dim3((int)std::min<int64_t>(8192, (n + 255) / 256)), dim3(256), 0, stream, d_plan, db,
                           (uint8_t*)flags_d.p, (unsigned long long*)((int64_t*)cnts_d.p + nb + 1));
        hipLaunchKernelGGL(k_flag_count, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n, (int64_t*)cnts_d.p);
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, stream, (int64_t*)cnts_d.p, nb);
        hipLaunchKernelGGL(k_flag_write, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n, (const int64_t*)cnts_d.p,
                           (int64_t)0, (int64_t*)trig_d.p);
        phase_end(ph);
        int64_t sel_err[2] = {0, 0};
        hipMemcpyAsync(sel_err, (int64_t*)cnts_d.p + nb, 16, hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "filter kernel failed");
        const int64_t ns = sel_err[0];
        stats.records_filter_error += sel_err[1];
        if (int rc = ensure_results(ns, 1)) return rc;
        WinInfo wi{};
        wi.j = range_wins++;
        wi.out_base = r_rows_used;
        wi.slot = (int32_t)wins.size();
        wi.direct = true;
        wins.push_back(wi);
        r_rows_used += ns;
        stats.windows_out++;
        if (ns > 0) {
            Results rv = results_view();
            const int ph2 = phase_begin(EK_PHASE_AGGREGATE);
            hipLaunchKernelGGL(k_filter_emit, dim3((int)std::min<int64_t>(8192, (ns + 255) / 256)), dim3(256), 0, stream, d_plan, db,
                               (const int64_t*)trig_d.p, ns, wi.out_base, wi.slot, rv);
            phase_end(ph2);
        }
        return 0;
    }

    // nq consecutive windows of len rows from src row a0 on (COUNTWINDOW blocks, no membership fingerprint): one
    // k_small_win launch with the arithmetic layout, no descriptor upload
    int fire_direct_arith(const DBatch& src, int64_t a0, int64_t len, int nq) {
        const int64_t rowcap = std::min<int64_t>(K, len);
        if (int rc = ensure_results(rowcap * nq, nq)) return rc;
        SwArith ar{};
        ar.a0 = a0;
        ar.len = (int32_t)len;
        ar.rowcap = rowcap;
        ar.ob0 = r_rows_used;
        ar.slot0 = (int32_t)wins.size();
        const int ph = phase_begin(EK_PHASE_AGGREGATE);
        if (int rc = small_win_launch(nq, src, nullptr, nullptr, nullptr, nullptr, (int)len, ar)) return rc;
        phase_end(ph);
        if (hipGetLastError() != hipSuccess) return fail(EK_ERR_DEVICE, "small-window launch failed");
        // the host's record of the windows (slot0 + w, rows from ob0 + w * rowcap) is written while the kernel runs:
        // for 10^5 windows a step it is a few hundred µs the device would otherwise wait for
        wins.resize(wins.size() + (size_t)nq);
        WinInfo* wp = wins.data() + ar.slot0;
        for (int w = 0; w < nq; ++w) {
            WinInfo& wi = wp[w];
            wi = WinInfo{};
            wi.j = range_wins + w;
            wi.out_base = ar.ob0 + (int64_t)w * rowcap;
            wi.slot = ar.slot0 + w;
            wi.direct = true;
        }
        range_wins += nq;
        r_rows_used += rowcap * nq;
        stats.windows_out += nq;
        return 0;
    }

    // COUNTWINDOW(n[, m]) in processing time (window_op.go:390-418, TupleList 502-551): every m-th arrival
    // emits the last n arrivals when at least n are buffered; arrival order, no watermark.
    // Small windows read straight from `src` (a batch in arrival order): hab = each window's row range in src, in
    // trigger order. Registers the windows like fire_windows and aggregates them with k_small_win.
    int fire_direct_small(const DBatch& src, const std::vector<int64_t>& hab, int64_t arr_base) {
        const int nq = (int)(hab.size() / 2);
        if (nq == 0) return 0;
        // consecutive equal-size windows (COUNTWINDOW blocks) and no membership fingerprint: arithmetic layout
        bool arith = !plan.debug_membership;
        for (int w = 1; w < nq && arith; ++w)
            arith = hab[2 * w] == hab[2 * w - 1] && hab[2 * w + 1] - hab[2 * w] == hab[1] - hab[0];
        if (arith) return fire_direct_arith(src, hab[0], hab[1] - hab[0], nq);
        if (int rc = ensure(ab_d, (size_t)nq * 16)) return rc;
        hipMemcpyAsync(ab_d.p, hab.data(), (size_t)nq * 16, hipMemcpyHostToDevice, stream);
        int64_t rows = 0;
        int max_n = 1;
        for (int w = 0; w < nq; ++w) {
            rows += std::min<int64_t>(K, hab[2 * w + 1] - hab[2 * w]);
            max_n = std::max<int>(max_n, (int)(hab[2 * w + 1] - hab[2 * w]));
        }
        if (int rc = ensure_results(rows, nq)) return rc;
        std::vector<int32_t> slots(nq), wl(nq);
        std::vector<int64_t> obase(nq);
        for (int w = 0; w < nq; ++w) {
            WinInfo wi{};
            wi.j = range_wins++;
            wi.out_base = r_rows_used;
            wi.slot = (int32_t)wins.size();
            wi.direct = true;
            r_rows_used += std::min<int64_t>(K, hab[2 * w + 1] - hab[2 * w]);
            wins.push_back(wi);
            slots[w] = wi.slot;
            obase[w] = wi.out_base;
            wl[w] = w;
        }
        stats.windows_out += nq;
        if (int rc = ensure(sw_d, (size_t)nq * 4 + (size_t)nq * 12 + 16)) return rc;
        int32_t* d_wl = (int32_t*)sw_d.p;
        int32_t* d_slot = d_wl + nq;
        int64_t* d_ob = (int64_t*)(((uintptr_t)(d_slot + nq) + 7) & ~(uintptr_t)7);
        hipMemcpyAsync(d_wl, wl.data(), (size_t)nq * 4, hipMemcpyHostToDevice, stream);
        hipMemcpyAsync(d_slot, slots.data(), (size_t)nq * 4, hipMemcpyHostToDevice, stream);
        hipMemcpyAsync(d_ob, obase.data(), (size_t)nq * 8, hipMemcpyHostToDevice, stream);
        if (plan.debug_membership)
            hipLaunchKernelGGL(k_range_members, dim3(nq), dim3(kBlock), 0, stream, (const int64_t*)nullptr, (const int64_t*)ab_d.p,
                               (const int32_t*)d_slot, (int64_t*)r_wmc.p, (unsigned long long*)r_wmh.p, arr_base);
        const int ph = phase_begin(EK_PHASE_AGGREGATE);
        if (int rc = small_win_launch(nq, src, (const int64_t*)ab_d.p, d_wl, d_slot, d_ob, max_n, SwArith{})) return rc;
        phase_end(ph);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "small-window launch failed");   // host lists reused
        return 0;
    }

    // COUNTWINDOW(n) (tumbling, processing time) over a batch holding whole windows (window_op.go:390-418): the window
    // that spans the carried rows and the batch head goes through the event buffer; every window wholly inside the
    // batch is aggregated straight from the batch's columns (no copy into the buffer); only the rows of the next,
    // unfinished window are appended. Windows, arrivals and membership are those of the buffered path.
    bool count_direct_ok(const DBatch& db) const {
        const int64_t len = plan.length;
        return count_direct && plan.interval <= 0 && !inc && !need_rel && !gmode && !g_row_arr && rowpos_col < 0 && dp.n_sagg == 0 &&
               small_win_on && len >= 1 && len <= kSmallWin && db.n >= 2 * len;
    }
    int push_count_direct(const DBatch& db) {
        const int64_t n = db.n, len = plan.length, A0 = arrivals, A1 = A0 + n;
        int64_t k = std::max<int64_t>(count_k, 1);   // next window: [k len - len, k len)
        int64_t e = k * len;
        if (e > A1) return 1;
        if (e - len < A0) {   // the window the carried rows began: the batch head completes it in the buffer
            const int64_t hcut = e - A0;
            if (int rc = eb_append(db, 0, hcut, A0)) return rc;
            eb_rel = eb.n;
            std::vector<PendWin> pw(1);
            pw[0].q.kind = RB_FIXED;
            pw[0].q.pos = e - len - eb_base;
            pw[0].q.rstep = e - eb_base;
            if (int rc = fire_windows(pw)) return rc;
            ++k;
            e += len;
        }
        if (!plan.debug_membership) {
            // the whole windows of the batch are consecutive blocks: no per-window host list before the launch
            const int64_t nw = e <= A1 ? (A1 - e) / len + 1 : 0;
            if (nw > 0)
                if (int rc = fire_direct_arith(db, e - len - A0, len, (int)nw)) return rc;
            k += nw;
            e += nw * len;
        } else {
            std::vector<int64_t> hab;
            for (; e <= A1; ++k, e += len) { hab.push_back(e - len - A0); hab.push_back(e - A0); }
            if (int rc = fire_direct_small(db, hab, A0)) return rc;
        }
        count_k = k;
        // every buffered row is consumed: the buffer restarts at the next window's first arrival with its rows
        const int64_t s_next = k * len - len;
        eb.n = 0;
        eb_base = s_next;
        eb_rel = 0;
        eb_floor = 0;
        if (int rc = eb_append(db, s_next - A0, A1 - s_next, A0)) return rc;
        arrivals = A1;
        eb_rel = eb.n;
        return 0;
    }

    int push_count(const DBatch& db) {
        if (count_direct_ok(db)) {
            const int rc = push_count_direct(db);
            if (rc <= 0) return rc;   // 1: the batch holds no whole window, buffered path
        }
        const int64_t n = db.n;
        const int64_t arrival_base = arrivals;
        if (int rc = eb_append(db, 0, n, arrival_base)) return rc;
        arrivals += n;
        eb_rel = eb.n;
        const int64_t len = plan.length, itv = plan.interval > 0 ? plan.interval : plan.length;
        std::vector<PendWin> pw;
        for (; count_k * itv <= arrivals; ++count_k) {
            const int64_t e = count_k * itv;
            if (e < len) continue;
            PendWin p{};
            p.q.kind = RB_FIXED;
            p.q.pos = e - len - eb_base;
            p.q.rstep = e - eb_base;
            p.start = 0;   // wall-clock WindowRange (not reproducible): reported as 0
            p.end = 0;
            pw.push_back(p);
        }
        int rc = fire_windows(pw);
        // the next window starts at (count_k * itv - len)
        eb_floor = std::max(eb_floor, count_k * itv - len - eb_base);
        return rc;
    }

    // the batch's columns on the device (host batches are copied to the handle's staging buffers)
    int stage_batch(const ek_batch* b, DBatch& db) {
        const int64_t n = b->n_rows;
        db.n = n;
        if (b->memory == EK_MEM_HOST) {
            for (int c = 0; c < user_cols; ++c) {
                size_t es = plan.column_type[c] == EK_COL_U32 ? 4 : 8;
                if (int rc = ensure(in_cols[c], (size_t)n * es)) return rc;
                hipMemcpyAsync(in_cols[c].p, b->columns[c], (size_t)n * es, hipMemcpyHostToDevice, stream);
                db.col[c] = in_cols[c].p;
                if (b->validity[c]) {
                    if (int rc = ensure(in_valid[c], (size_t)n)) return rc;
                    hipMemcpyAsync(in_valid[c].p, b->validity[c], (size_t)n, hipMemcpyHostToDevice, stream);
                    db.valid[c] = (const uint8_t*)in_valid[c].p;
                }
            }
            // a pinned caller buffer makes these copies truly asynchronous: an asynchronous push waits for them before
            // it returns (record_time), so a host batch is never borrowed past its push
            if (async_push) {
                if (!ev_h2d) hipEventCreateWithFlags(&ev_h2d, hipEventDisableTiming);
                hipEventRecord(ev_h2d, stream);
                h2d_pending = true;
            }
        } else {
            for (int c = 0; c < user_cols; ++c) { db.col[c] = b->columns[c]; db.valid[c] = b->validity[c]; }
        }
        return derive(db);
    }

    // the derived columns of a staged batch (k_derive): engine-owned buffers appended to the batch's columns
    int derive(DBatch& db) {
        const int nd = plan.n_columns - user_cols;
        if (nd <= 0 || db.n <= 0) return 0;
        int64_t* o[4] = {nullptr, nullptr, nullptr, nullptr};
        uint8_t* v[4] = {nullptr, nullptr, nullptr, nullptr};
        for (int d = 0; d < nd; ++d) {
            const int c = user_cols + d;
            if (int rc = ensure(der_val[d], (size_t)db.n * 8)) return rc;
            o[d] = (int64_t*)der_val[d].p;
            db.col[c] = o[d];
            db.valid[c] = nullptr;
            if ((plan.nullable_mask >> c) & 1u) {
                if (int rc = ensure(der_valid[d], (size_t)db.n)) return rc;
                v[d] = (uint8_t*)der_valid[d].p;
                db.valid[c] = v[d];
            }
        }
        hipLaunchKernelGGL(k_derive, dim3((int)std::min<int64_t>(8192, (db.n + 255) / 256)), dim3(256), 0, stream, d_plan, db, db.n,
                           o[0], o[1], o[2], o[3], v[0], v[1], v[2], v[3]);
        return 0;
    }

    int push(const ek_batch* b) {
        if (!b) return fail(EK_ERR_INVALID, "null batch");
        int64_t n = b->n_rows;
        if (n < 0) return fail(EK_ERR_INVALID, "negative row count");
        if (n == 0) return 0;
        if (n > ((int64_t)1 << 31) - 1) return fail(EK_ERR_UNSUPPORTED, "batch larger than 2^31-1 rows");
        for (int c = 0; c < user_cols; ++c) {
            if (!b->columns[c]) return fail(EK_ERR_INVALID, "column %d missing", c);
            if (b->validity[c] && !((plan.nullable_mask >> c) & 1u)) return fail(EK_ERR_INVALID, "column %d is not declared nullable", c);
        }
        if (gmode) return fail(EK_ERR_STATE, "the handle takes its watermark from ek_push_batch_global (shard mode)");
        if (int rc = fold_time()) return rc;
        hipEventRecord(ev0, stream);
        DBatch db{};
        if (int rc = stage_batch(b, db)) return rc;
        stats.records_in += n;
        set_ts_hint(b);
        const HintScope hint_scope{ts_hint};
        if (wtype == EK_WINDOW_NONE) {
            const int rc = push_filter(db);
            return rc ? rc : record_time();
        }
        if (!plan.is_event_time && (wtype == EK_WINDOW_COUNT || wtype == EK_WINDOW_STATE) && pre_filter) {
            // the window FILTER op in front of the count / state window: only the rows it keeps reach the window (they
            // keep their source arrival indices for the membership check)
            if (int rc = proc_prefilter(db, stats.records_in - n)) { g_row_arr = nullptr; return rc; }
        }
        if (wtype == EK_WINDOW_COUNT && !plan.is_event_time) {
            const int rc = push_count(db);
            g_row_arr = nullptr;
            return rc ? rc : record_time();
        }
        if (wtype == EK_WINDOW_STATE && !plan.is_event_time) {
            // processing time: the rows reach StateWindowOp in arrival order
            const int64_t m = db.n;
            int rc = eb_append(db, 0, m, arrivals);
            g_row_arr = nullptr;
            if (rc) return rc;
            arrivals += m;
            const int64_t lo = eb_rel;
            eb_rel = eb.n;
            rc = state_scan(lo, eb_rel);
            return rc ? rc : record_time();
        }
        if (proc) {
            const int rc = push_proc(db);
            return rc ? rc : record_time();
        }
        const int64_t* ts = (const int64_t*)db.col[dp.ts_col];
        if (fz_eligible(n)) {   // pane mode: the fused sorted pass (push_fused), or the general path below
            const int rc = push_fused(db, ts, n);
            if (rc != kFzFallback) return rc ? rc : record_time();
        }

        // ---- 1. batch statistics (one pass over ts, or the batch's shared ek_ts_stats)
        BatchStats s;
        const bool gap = wtype == EK_WINDOW_HOPPING && plan.late_tolerance_ms == 0;
        if (int rc = batch_stats(ts, n, gap, gap && has_M ? M : INT64_MIN, &s)) return rc;
        const int64_t T = plan.late_tolerance_ms;

        // ---- 2. late-event drop (watermark_op.go:144-155)
        bool sorted = !s.unsorted;
        int64_t start = 0, n_acc = n, min_acc = s.min_ts;
        const uint8_t* d_acc = nullptr;
        if (sorted && has_M && s.min_ts < M - T) {
            // sorted batch below the carried watermark: the late events are a prefix
            int64_t bound = M - T;
            if (int rc = ensure(bounds_val, 8)) return rc;
            if (int rc = ensure(bounds_idx, 8)) return rc;
            hipMemcpyAsync(bounds_val.p, &bound, 8, hipMemcpyHostToDevice, stream);
            hipLaunchKernelGGL(k_lower_bound, dim3(1), dim3(64), 0, stream, ts, (int64_t)0, n, (const int64_t*)bounds_val.p, 1,
                               (int64_t*)bounds_idx.p);
            hipMemcpyAsync(&start, bounds_idx.p, 8, hipMemcpyDeviceToHost, stream);
            hipStreamSynchronize(stream);
            n_acc = n - start;
            if (n_acc > 0) {
                hipMemcpyAsync(&min_acc, ts + start, 8, hipMemcpyDeviceToHost, stream);
                hipStreamSynchronize(stream);
            }
        } else if (!sorted) {
            int nch = (int)((n + kAccChunk - 1) / kAccChunk);
            if (int rc = ensure(cmax, (size_t)nch * 8 * 3)) return rc;   // chunk maxima + (count, min) partials
            if (int rc = ensure(acc, (size_t)n)) return rc;
            int64_t* cpart = (int64_t*)cmax.p + nch;
            hipLaunchKernelGGL(k_chunk_max, dim3(nch), dim3(kBlock), 0, stream, ts, n, (int64_t*)cmax.p);
            hipLaunchKernelGGL(k_scan_max, dim3(1), dim3(1024), 0, stream, (int64_t*)cmax.p, nch, has_M ? M : kMinTs);
            hipLaunchKernelGGL(k_accept, dim3(nch), dim3(kBlock), 0, stream, ts, n, (const int64_t*)cmax.p, T,
                               (uint8_t*)acc.p, cpart);
            hipLaunchKernelGGL(k_accept_reduce, dim3(1), dim3(1024), 0, stream, (const int64_t*)cpart, nch, (BatchStats*)bstats.p);
            hipMemcpyAsync(h_stats, bstats.p, sizeof(BatchStats), hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "accept kernel failed");
            n_acc = h_stats->n_accepted;
            min_acc = h_stats->min_accepted;
            d_acc = (const uint8_t*)acc.p;
        }
        stats.records_late += n - n_acc;
        // ---- 2b. the window's FILTER (WHERE ...) op between WatermarkOp and the window (planner.go:388-392): a row it
        // drops never reaches the window (no member, no trigger, not the first window's anchor) but moved the watermark
        bool filt_dropped = false;
        if (plan.n_filter > 0 && n_acc > 0) {
            if (int rc = ensure(filt_d, (size_t)n)) return rc;
            BatchStats* bs = (BatchStats*)bstats.p;
            hipMemsetAsync(&bs->n_accepted, 0, 8, stream);
            hipMemsetAsync(&bs->n_dropped, 0, 8, stream);
            const int64_t big = INT64_MAX;
            hipMemcpyAsync(&bs->min_accepted, &big, 8, hipMemcpyHostToDevice, stream);
            hipLaunchKernelGGL(k_filter_mask, dim3((int)std::min<int64_t>(4096, (n + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                               d_plan_where, db, d_acc, start, (uint8_t*)filt_d.p, bs);
            hipMemcpyAsync(h_stats, bstats.p, sizeof(BatchStats), hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "window filter kernel failed");
            stats.records_filter_error += h_stats->n_dropped;
            filt_dropped = h_stats->n_accepted < n_acc;
            n_acc = h_stats->n_accepted;
            if (n_acc > 0) min_acc = h_stats->min_accepted;   // none left: the batch only moves the watermark
            d_acc = (const uint8_t*)filt_d.p;
        }
        int64_t arrival_base = arrivals;
        arrivals += n;
        h_wdesc_used = 0;   // the stats sync above drained every earlier descriptor upload
        h_desc_used = 0;
        aux_used = 0;

        // ---- 3. watermark advance (watermark_op.go:157-214): W = max ts - lateTol
        const int64_t M_prev = M;
        const bool had_M = has_M;
        if (!has_M || s.max_ts > M) {
            M = s.max_ts;
            has_M = true;
            W = M - T;
            has_W = true;
        }
        bool hop_dropped = false;
        // ---- 3b. hopping empty-window discard (window_op.go:605-655, lateTolerance 0): only a batch with an
        // arrival gap wider than the window can trigger an empty window, so the mask pass runs only then
        if (wtype == EK_WINDOW_HOPPING && T == 0 && n_acc > 0 && s.max_gap > L) {
            // the first window end: E1 = aligned end of the first released event (= min accepted ts when T = 0)
            const int64_t e1 = e1_known ? E1 : aligned_end(min_acc, raw_interval, plan.time_unit, plan.tz_offset_s);
            const int nch = (int)((n + kAccChunk - 1) / kAccChunk);
            if (int rc = ensure(cmax, (size_t)nch * 8)) return rc;
            if (int rc = ensure(acc, (size_t)n)) return rc;
            hipLaunchKernelGGL(k_chunk_max, dim3(nch), dim3(kBlock), 0, stream, ts, n, (int64_t*)cmax.p);
            hipLaunchKernelGGL(k_scan_max, dim3(1), dim3(1024), 0, stream, (int64_t*)cmax.p, nch, had_M ? M_prev : INT64_MIN);
            hipLaunchKernelGGL(k_hop_drop, dim3(nch), dim3(kBlock), 0, stream, ts, n, (const int64_t*)cmax.p, start, d_acc,
                               e1, H, L, (uint8_t*)acc.p, (BatchStats*)bstats.p);
            int64_t dropped = 0;
            hipMemcpyAsync(&dropped, &((BatchStats*)bstats.p)->n_dropped, 8, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "hopping discard kernel failed");
            if (dropped) {
                d_acc = (const uint8_t*)acc.p;
                n_acc -= dropped;
                stats.records_discarded += dropped;
                hop_dropped = true;
            }
        }
        if (range_mode) {
            const int rc = push_range(db, sorted, start, d_acc, n_acc, min_acc, s.max_ts, arrival_base, M_prev, had_M, s.min_ts);
            return rc ? rc : record_time();
        }
        // a batch whose every accepted event was discarded (or filtered) still advanced the watermark: its windows close
        // below
        if (n_acc == 0 && !((hop_dropped || filt_dropped) && e1_known)) return record_time();

        // ---- 4. first window alignment once the first event is released
        if (!e1_known) {
            int64_t mn = std::min(min_acc, pend_min);
            if (!(has_W && W >= mn)) {
                int rc = append_pending(db, d_acc, arrival_base);
                return rc ? rc : record_time();
            }
            e1_known = true;
            first_ts = mn;
            E1 = aligned_end(first_ts, raw_interval, plan.time_unit, plan.tz_offset_s);
            grid.tumbling = wtype == EK_WINDOW_TUMBLING;
            grid.origin = grid.tumbling ? E1 : E1 - L;
            grid.P = P;
            if (pend_n) {
                if (int rc = flush_pending()) return rc;
            }
        }
        {
            int64_t save = arrivals;
            arrivals = arrival_base;
            int rc = process(db, sorted, start, d_acc, min_acc, s.max_ts, nullptr);
            arrivals = save;
            if (rc) return rc;
        }
        return record_time();
    }

    // Asynchronous pushes (ek_set_async) return once their work is queued: the end event is recorded here and read
    // back (fold_time) by the next push or by ek_get_stats — so the caller's own work between pushes overlaps the
    // device tail of the previous one instead of idling the GPU behind a host round trip.
    int record_time() {
        hipEventRecord(ev1, stream);
        time_pending = true;
        if (h2d_pending) {   // an asynchronous push of a host batch returns once its columns are copied
            h2d_pending = false;
            if (hipEventSynchronize(ev_h2d) != hipSuccess) return fail(EK_ERR_DEVICE, "host batch copy failed");
        }
        if (!async_push) return fold_time();   // synchronous pushes (the default) complete before they return
        return 0;
    }
    int fold_time() {
        // (not pending: phases recorded since the last fold — a shared ek_batch_ts_stats pass before this push — stay
        // and are folded with the push they serve)
        if (!time_pending) return 0;
        time_pending = false;
        // an asynchronous push's queued work that failed surfaces here: at the next push / advance / stats call
        const hipError_t qe = hipEventSynchronize(ev1);
        if (qe != hipSuccess) {
            phase_used = 0;
            return fail(EK_ERR_DEVICE, "queued work of the previous push failed: %s", hipGetErrorString(qe));
        }
        {
            float ms = 0;
            hipEventElapsedTime(&ms, ev0, ev1);
            stats.last_batch_device_ms = ms;
            stats.device_ms_total += ms;
            stats.pushes_timed++;
            for (int k = 0; k < 4; ++k) { stats.phase_ms[k] = 0; stats.phase_launches[k] = 0; }
            for (size_t k = 0; k < phase_used; ++k) {
                float t = 0;
                if (hipEventElapsedTime(&t, phase_ev[k].a, phase_ev[k].b) == hipSuccess) {
                    stats.phase_ms[phase_ev[k].phase] += t;
                    stats.phase_launches[phase_ev[k].phase]++;
                }
            }
            for (int k = 0; k < 4; ++k) {
                stats.phase_ms_total[k] += stats.phase_ms[k];
                stats.phase_launches_total[k] += stats.phase_launches[k];
            }
        }
        phase_used = 0;
        return 0;
    }



    // ================================================================== SHARD mode (global watermark)
    // One key-hash shard of a rule (include/ekgpu.h, ek_push_batch_global): the rows of this handle carry their
    // global arrival index; the WatermarkTuples of the whole stream come from the host that assigns the arrival
    // order (ekgpu/shard.py GlobalWatermark, watermark_op.go:144-225). Acceptance, release steps and window closing
    // follow those tuples instead of the handle's own rows. Rows are otherwise processed exactly as in the local
    // modes (pane partials for tumbling / hopping, the ts-ordered event buffer for sliding windows, the arrival
    // ordered buffer for processing-time count windows).
    int gmode = 0;                      // 1: shard mode (entered by the first global push, left by ek_reset)
    const int64_t* g_row_arr = nullptr; // device: global arrival of the current batch's rows
    // the current push's WatermarkTuples: the caller's host arrays (valid for the duration of the call)
    const int64_t* g_wa = nullptr;
    const int64_t* g_wt = nullptr;
    int64_t g_nwm = 0;
    bool g_wm_on_dev = false;           // uploaded to g_wm_d (only when a kernel needs the list)
    bool g_all_accepted = false;
    int64_t g_max_step = 0;
    DevBuf g_wm_d, g_arr_d, g_acc_d;
    struct GTrig { int64_t a, t; };
    std::vector<GTrig> g_trig;          // accepted global sliding triggers not released yet (arrival order)
    struct GSess { int64_t start, end; };
    std::vector<GSess> g_sess;          // sessions the router closed in this push (ek_global_ctx sess_*), in order
    int64_t g_sess_last_end = INT64_MIN;   // the last session end delivered (ends advance across pushes)

    int global_check() {
        if (plan.is_event_time) {
            if (inc || plan.window_version == 2 || wtype == EK_WINDOW_STATE)
                return fail(EK_ERR_UNSUPPORTED, "shard mode: state, v2 and incremental windows depend on every row "
                                                "of the stream (not shardable by key)");
            if (wtype == EK_WINDOW_SLIDING && plan.delay != 0 && send_twice)
                return fail(EK_ERR_UNSUPPORTED, "shard mode: send-twice sliding windows keep an expired prefix of EVERY "
                                                "input of the stream (window_op.go:576-603; not shardable by key)");
            if (wtype == EK_WINDOW_HOPPING && plan.late_tolerance_ms != 0)
                return fail(EK_ERR_UNSUPPORTED, "shard mode: the hopping empty-window discard is built for lateTolerance 0");
            if (plan.n_filter > 0)
                return fail(EK_ERR_UNSUPPORTED, "shard mode: a window FILTER is not built (the router would drop the rows)");
        } else if (wtype != EK_WINDOW_COUNT || inc || plan.n_filter > 0) {
            return fail(EK_ERR_UNSUPPORTED, "shard mode: processing time is built for COUNTWINDOW (without FILTER)");
        }
        return 0;
    }

    // the tuple list on the device (one upload per push, from a pinned staging block)
    int wm_to_device() {
        if (g_wm_on_dev || g_nwm == 0) return 0;
        if (int rc = ensure(g_wm_d, (size_t)g_nwm * 16)) return rc;
        int64_t* h = desc_alloc((size_t)g_nwm * 2);
        if (!h) return fail(EK_ERR_NOMEM, "pinned");
        memcpy(h, g_wa, (size_t)g_nwm * 8);
        memcpy(h + g_nwm, g_wt, (size_t)g_nwm * 8);
        hipMemcpyAsync(g_wm_d.p, h, (size_t)g_nwm * 16, hipMemcpyHostToDevice, stream);
        g_wm_on_dev = true;
        return 0;
    }
    // W before this push's tuples (carry) and the list on the device (call wm_to_device first)
    WmList wm_list(int64_t carry) const {
        WmList w{};
        w.arr = g_nwm ? (const int64_t*)g_wm_d.p : nullptr;
        w.ts = w.arr ? w.arr + g_nwm : nullptr;
        w.n = g_nwm;
        w.carry = carry;
        return w;
    }

    // host copies + one device upload of the tuple list; the rows' arrivals on the device
    int global_stage(const ek_global_ctx* g, int64_t n) {
        if (g->n_wm < 0 || g->n_trig < 0) return fail(EK_ERR_INVALID, "negative list length");
        if ((g->n_wm > 0 && (!g->wm_arrival || !g->wm_ts)) || (g->n_trig > 0 && (!g->trig_arrival || !g->trig_ts)))
            return fail(EK_ERR_INVALID, "missing watermark / trigger list");
        if (n > 0 && !g->row_arrival) return fail(EK_ERR_INVALID, "missing row arrivals");
        if (g->n_sess < 0 || (g->n_sess > 0 && (!g->sess_start || !g->sess_end)))
            return fail(EK_ERR_INVALID, "missing session list");
        g_sess.clear();
        if (wtype == EK_WINDOW_SESSION)
            for (int64_t k = 0; k < g->n_sess; ++k) {   // ends advance within the list and across pushes
                if (g->sess_end[k] <= (k ? g->sess_end[k - 1] : g_sess_last_end))
                    return fail(EK_ERR_INVALID, "session ends must advance (session %lld ends at %lld, after %lld)",
                                (long long)k, (long long)g->sess_end[k], (long long)(k ? g->sess_end[k - 1] : g_sess_last_end));
                g_sess.push_back(GSess{g->sess_start[k], g->sess_end[k]});
            }
        if (!g_sess.empty()) g_sess_last_end = g_sess.back().end;
        g_wa = g->wm_arrival;
        g_wt = g->wm_ts;
        g_nwm = g->n_wm;
        g_wm_on_dev = false;
        g_all_accepted = g->all_accepted != 0;
        g_max_step = g->max_wm_step;
        // the tuples advance (the whole list is checked when a kernel uploads it; here its ends)
        if (g_nwm > 0 && ((has_W && g_wt[0] <= W) || g_wt[g_nwm - 1] < g_wt[0] || g_wa[g_nwm - 1] < g_wa[0]))
            return fail(EK_ERR_INVALID, "WatermarkTuples must advance");
        g_row_arr = nullptr;
        if (n > 0) {
            if (g->memory == EK_MEM_HOST) {
                if (int rc = ensure(g_arr_d, (size_t)n * 8)) return rc;
                hipMemcpyAsync(g_arr_d.p, g->row_arrival, (size_t)n * 8, hipMemcpyHostToDevice, stream);
                g_row_arr = (const int64_t*)g_arr_d.p;
            } else {
                g_row_arr = g->row_arrival;
            }
        }
        return 0;
    }

    // accept mask of the staged batch (nullptr: every row accepted); n_acc / min_acc / dropped out
    int global_accept(const DBatch& db, int64_t min_ts, bool hop, int64_t e1, const uint8_t** d_acc, int64_t* n_acc,
                      int64_t* min_acc, int64_t* dropped) {
        const int64_t n = db.n;
        const int64_t carry = has_W ? W : INT64_MIN;
        int64_t wmax = carry;
        if (g_nwm > 0) wmax = std::max(wmax, g_wt[g_nwm - 1]);
        *d_acc = nullptr; *n_acc = n; *min_acc = min_ts; *dropped = 0;
        if (!hop && (wmax == INT64_MIN || min_ts >= wmax)) return 0;   // no row can be late
        // the host's WatermarkOp accepted every event and no tuple advanced by more than a hopping window
        if (g_all_accepted && (!hop || (g_max_step > 0 && g_max_step <= L))) return 0;
        if (int rc = wm_to_device()) return rc;
        const WmList w = wm_list(carry);
        if (int rc = ensure(g_acc_d, (size_t)n)) return rc;
        hipMemsetAsync(&((BatchStats*)bstats.p)->n_accepted, 0, 8, stream);
        hipMemsetAsync(&((BatchStats*)bstats.p)->n_dropped, 0, 8, stream);
        const int64_t big = INT64_MAX;
        hipMemcpyAsync(&((BatchStats*)bstats.p)->min_accepted, &big, 8, hipMemcpyHostToDevice, stream);
        hipLaunchKernelGGL(k_accept_global, dim3((int)std::min<int64_t>(4096, (n + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                           (const int64_t*)db.col[dp.ts_col], g_row_arr, n, w, hop ? 1 : 0, e1, H, L, (uint8_t*)g_acc_d.p,
                           (BatchStats*)bstats.p);
        hipMemcpyAsync(h_stats, bstats.p, sizeof(BatchStats), hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "global accept kernel failed");
        *n_acc = h_stats->n_accepted;
        *min_acc = h_stats->min_accepted;
        *dropped = h_stats->n_dropped;
        if (*n_acc < n) *d_acc = (const uint8_t*)g_acc_d.p;
        return 0;
    }

    int push_global(const ek_batch* b, const ek_global_ctx* g) {
        if (!g) return fail(EK_ERR_INVALID, "null global context");
        const int64_t n = b ? b->n_rows : 0;
        if (n < 0) return fail(EK_ERR_INVALID, "negative row count");
        if (n > ((int64_t)1 << 31) - 1) return fail(EK_ERR_UNSUPPORTED, "batch larger than 2^31-1 rows");
        if (wtype == EK_WINDOW_NONE) return fail(EK_ERR_UNSUPPORTED, "shard mode needs a window");
        if (!gmode) {
            if (stats.records_in > 0 || has_W) return fail(EK_ERR_STATE, "the handle already runs on its own watermark (ek_push_batch)");
            if (int rc = global_check()) return rc;
            gmode = 1;
        }
        if (g->arrivals_end < arrivals) return fail(EK_ERR_INVALID, "arrivals_end went backwards");
        if (n > 0) {
            for (int c = 0; c < user_cols; ++c) {
                if (!b->columns[c]) return fail(EK_ERR_INVALID, "column %d missing", c);
                if (b->validity[c] && !((plan.nullable_mask >> c) & 1u)) return fail(EK_ERR_INVALID, "column %d is not declared nullable", c);
            }
        }
        if (int rc = fold_time()) return rc;
        hipEventRecord(ev0, stream);
        h_wdesc_used = 0;
        h_desc_used = 0;
        aux_used = 0;
        hipStreamSynchronize(stream);   // the pinned descriptor blocks are reused below
        if (int rc = global_stage(g, n)) return rc;
        DBatch db{};
        if (n > 0) {
            if (int rc = stage_batch(b, db)) return rc;
        }
        stats.records_in += n;
        set_ts_hint(b);
        const HintScope hint_scope{ts_hint};
        int rc = 0;
        if (!plan.is_event_time) rc = push_count_global(db, g);
        else rc = push_global_event(db, g);
        g_row_arr = nullptr;
        g_wa = g_wt = nullptr;
        g_nwm = 0;
        if (rc) return rc;
        arrivals = g->arrivals_end;
        return record_time();
    }

    int push_global_event(const DBatch& db, const ek_global_ctx* g) {
        const int64_t n = db.n;
        const int64_t T = plan.late_tolerance_ms;
        BatchStats s{};
        s.min_ts = INT64_MAX;
        s.max_ts = INT64_MIN;
        if (n > 0) {
            const int64_t* ts = (const int64_t*)db.col[dp.ts_col];
            if (int rc = batch_stats(ts, n, false, INT64_MIN, &s)) return rc;
        }
        // the first window's anchor: the global earliest released event (getEarliestEventTs at that tuple)
        const bool origin_now = !e1_known && g->origin_known;
        const int64_t e1_anchor = g->origin_known ? aligned_end(g->origin_ts, raw_interval, plan.time_unit, plan.tz_offset_s) : 0;
        const bool hop = wtype == EK_WINDOW_HOPPING && T == 0 && (e1_known || g->origin_known);
        const uint8_t* d_acc = nullptr;
        int64_t n_acc = 0, min_acc = s.min_ts, dropped = 0;
        if (n > 0) {
            if (int rc = global_accept(db, s.min_ts, hop, e1_known ? E1 : e1_anchor, &d_acc, &n_acc, &min_acc, &dropped)) return rc;
        }
        stats.records_late += n - n_acc - dropped;
        stats.records_discarded += dropped;
        // the shard's own max ts (buffer order bookkeeping only: it does not move the watermark)
        const int64_t M_prev = M;
        const bool had_M = has_M;
        if (n > 0 && (!has_M || s.max_ts > M)) { M = s.max_ts; has_M = true; }
        const int64_t W_carry = has_W ? W : INT64_MIN;
        if (g_nwm > 0) {
            W = g_wt[g_nwm - 1];
            has_W = true;
            sW = g_wa[g_nwm - 1];
        }
        if (origin_now) {
            e1_known = true;
            first_ts = g->origin_ts;
            E1 = e1_anchor;
            grid.tumbling = wtype == EK_WINDOW_TUMBLING;
            grid.origin = grid.tumbling ? E1 : E1 - L;
            grid.P = P;
        }
        const int64_t arrival_base = arrivals;
        if (range_mode) {
            if (n_acc > 0) {
                if (!s.unsorted && !d_acc && (eb.n == 0 || !had_M || min_acc >= M_prev)) {
                    if (int rc = eb_append(db, 0, n_acc, arrival_base)) return rc;
                } else {
                    if (int rc = eb_merge(db, 0, d_acc, n_acc, min_acc, s.max_ts, arrival_base)) return rc;
                }
            }
            const int64_t rel_prev = eb_rel;
            if (has_W && eb.n > 0) {
                if (int rc = ensure(bounds_idx, 8)) return rc;
                hipLaunchKernelGGL(k_rel_end, dim3(1), dim3(64), 0, stream, (const int64_t*)eb.col[dp.ts_col].p,
                                   arr_ptr(), eb_arr0, eb.n, W, sW, (int64_t*)bounds_idx.p);
                eb_rel = std::max(eb_rel, fetch_i64(bounds_idx.p));
            }
            if (need_rel && eb_rel > rel_prev) {
                if (int rc = wm_to_device()) return rc;
                if (int rc = arr_materialize()) return rc;
                const int gg = (int)std::min<int64_t>(4096, (eb_rel - rel_prev + 255) / 256);
                hipLaunchKernelGGL(k_release_step_global, dim3(gg), dim3(256), 0, stream, (const int64_t*)eb.col[dp.ts_col].p,
                                   (const int64_t*)eb.arr.p, rel_prev, eb_rel, wm_list(W_carry), (int64_t*)eb.rel.p);
            }
            for (int64_t k = 0; k < g->n_trig; ++k) g_trig.push_back(GTrig{g->trig_arrival[k], g->trig_ts[k]});
            return range_triggers(rel_prev);
        }
        // pane mode: rows before the anchor wait (host side) until the first release is known
        if (!e1_known) {
            if (n_acc > 0) return append_pending(db, d_acc, arrival_base);
            return 0;
        }
        if (origin_now && pend_n) {
            if (int rc = flush_pending()) return rc;
        }
        if (n_acc > 0) {
            const int64_t save = arrivals;
            arrivals = arrival_base;
            int rc = process(db, !s.unsorted, 0, d_acc, min_acc, s.max_ts, g_row_arr);
            arrivals = save;
            if (rc) return rc;
        }
        // windows the global watermark closed beyond this shard's rows
        return finalize_ready(INT64_MAX / 4);
    }

    // SLIDINGWINDOW triggers of the whole stream (shard mode): a trigger fires at the tuple that releases it
    // (ts < W, or ts == W and it arrived no later than that tuple's event), over the rows released so far with
    // t - L <= ts <= t and release step <= the trigger's (window_op.go:605-655, event_window_trigger.go:147-166).
    int global_slide_triggers(std::vector<PendWin>& pw) {
        const int64_t D = (int64_t)plan.delay * unit_ms(plan.time_unit);
        if (D > 0) {
            // delayed: a released trigger queues t + D (event_window_trigger.go:154-166); its window [t - L, t + D) over
            // the shard's rows fires at the first LATER global tuple reaching t + D — in this push iff its last tuple
            // does (W only grows) — in trigger order, as the single-stream delay loop (the queue is ts-ordered)
            if (int rc = global_release_triggers([&](const GTrig& x, int64_t k) {
                    delayq.push_back(DelayTrig{x.a, x.t, g_wt[k]});
                    return 0;
                }))
                return rc;
            while (delayq_head < delayq.size()) {
                const DelayTrig& d = delayq[delayq_head];
                if (!(has_W && W >= d.ts + D && W > d.w_rel)) break;
                PendWin p{};
                p.q.kind = RB_LB;
                p.q.lo_ts = d.ts - L;
                p.q.hi_ts = d.ts + D;
                p.q.floor = eb_floor;
                p.start = 0;     // second-part scan leaves WindowRange unset
                p.end = 0;
                pw.push_back(p);
                delayq_head++;
            }
            if (delayq_head > 4096 && delayq_head * 2 > delayq.size()) {
                delayq.erase(delayq.begin(), delayq.begin() + (int64_t)delayq_head);
                delayq_head = 0;
            }
            return 0;
        }
        return global_release_triggers([&](const GTrig& x, int64_t k) {
            PendWin p{};
            p.q.kind = RB_SLIDE;
            p.q.lo_ts = x.t - L;
            p.q.hi_ts = x.t;
            p.q.pos = eb_floor - 1;      // the search starts at the floor: every row before the trigger's run is a member candidate
            p.q.rstep = g_wa[k];
            p.q.floor = eb_floor;
            p.start = x.t - L;
            p.end = x.t;
            pw.push_back(p);
            return 0;
        });
    }
    // the global triggers the push's tuples release, in (ts, arrival) order, each with the index of its releasing tuple
    template <typename F>
    int global_release_triggers(F on_release) {
        if (!has_W || g_trig.empty()) return 0;
        std::vector<GTrig> rel, keep;
        for (const GTrig& x : g_trig) {
            if (x.t < W || (x.t == W && x.a <= sW)) rel.push_back(x);
            else keep.push_back(x);
        }
        g_trig.swap(keep);
        std::stable_sort(rel.begin(), rel.end(), [](const GTrig& x, const GTrig& y) { return x.t < y.t || (x.t == y.t && x.a < y.a); });
        for (const GTrig& x : rel) {
            // the releasing tuple: the first one at or after its arrival whose watermark reaches its ts
            const int64_t k0 = std::lower_bound(g_wa, g_wa + g_nwm, x.a) - g_wa;
            const int64_t k1 = std::lower_bound(g_wt, g_wt + g_nwm, x.t) - g_wt;
            const int64_t k = std::max(k0, k1);
            if (k >= g_nwm) return fail(EK_ERR_INVALID, "trigger at arrival %lld is not released by this batch's tuples", (long long)x.a);
            if (int rc = on_release(x, k)) return rc;
        }
        return 0;
    }

    // COUNTWINDOW(n[, m]) of a shard: blocks of the GLOBAL arrival order (window_op.go:390-418)
    int push_count_global(const DBatch& db, const ek_global_ctx* g) {
        const int64_t n = db.n;
        if (n > 0) {
            if (int rc = eb_append(db, 0, n, 0)) return rc;
        }
        eb_rel = eb.n;
        const int64_t len = plan.length, itv = plan.interval > 0 ? plan.interval : plan.length;
        std::vector<PendWin> pw;
        for (; count_k * itv <= g->arrivals_end; ++count_k) {
            const int64_t e = count_k * itv;
            if (e < len) continue;
            PendWin p{};
            p.q.kind = RB_ARR;
            p.q.lo_ts = e - len;
            p.q.hi_ts = e;
            p.q.floor = eb_floor;
            pw.push_back(p);
        }
        return fire_windows(pw);
    }

    // ek_shard_triggers: accepted rows of the batch that match OVER (WHEN ...)
    int shard_triggers(const ek_batch* b, const ek_global_ctx* g, int64_t* out_a, int64_t* out_t, int64_t cap, int64_t* n_out) {
        if (!b || !g || !n_out) return fail(EK_ERR_INVALID, "null argument");
        if (wtype != EK_WINDOW_SLIDING || !plan.is_event_time) return fail(EK_ERR_UNSUPPORTED, "triggers belong to event-time sliding windows");
        if (!gmode) {
            if (stats.records_in > 0 || has_W) return fail(EK_ERR_STATE, "the handle already runs on its own watermark (ek_push_batch)");
            if (int rc = global_check()) return rc;
        }
        const int64_t n = b->n_rows;
        *n_out = 0;
        if (n <= 0) return 0;
        hipStreamSynchronize(stream);
        h_desc_used = 0;
        if (int rc = global_stage(g, n)) return rc;
        DBatch db{};
        if (int rc = stage_batch(b, db)) return rc;
        const uint8_t* d_acc = nullptr;
        int64_t n_acc = 0, min_acc = 0, dropped = 0;
        if (int rc = global_accept(db, INT64_MIN, false, 0, &d_acc, &n_acc, &min_acc, &dropped)) return rc;
        if (int rc = ensure(flags_d, (size_t)n)) return rc;
        if (int rc = ensure(trig_d, (size_t)n * 8)) return rc;
        const int nb = (int)((n + kCompactTile - 1) / kCompactTile);
        if (int rc = ensure(cnts_d, (size_t)(nb + 1) * 8)) return rc;
        const int gg = (int)std::min<int64_t>(4096, (n + 255) / 256);
        hipLaunchKernelGGL(k_trigger_flags, dim3(gg), dim3(256), 0, stream, d_plan, db, (int64_t)0, n, (uint8_t*)flags_d.p);
        if (d_acc) hipLaunchKernelGGL(k_and_flags, dim3(gg), dim3(256), 0, stream, (uint8_t*)flags_d.p, d_acc, n);
        hipLaunchKernelGGL(k_flag_count, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n, (int64_t*)cnts_d.p);
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, stream, (int64_t*)cnts_d.p, nb);
        hipLaunchKernelGGL(k_flag_write, dim3(nb), dim3(kBlock), 0, stream, (const uint8_t*)flags_d.p, n, (const int64_t*)cnts_d.p,
                           (int64_t)0, (int64_t*)trig_d.p);
        const int64_t nt = fetch_i64((const int64_t*)cnts_d.p + nb);
        *n_out = nt;
        const int64_t nc = std::min(nt, cap);
        if (nc > 0 && out_a && out_t) {
            if (int rc = ensure(mrg_col, (size_t)nc * 16)) return rc;
            int64_t* gbuf = (int64_t*)mrg_col.p;
            const int g2 = (int)std::min<int64_t>(4096, (nc + 255) / 256);
            hipLaunchKernelGGL(k_gather8, dim3(g2), dim3(256), 0, stream, (const int64_t*)trig_d.p, nc, INT64_MAX, g_row_arr,
                               (const int64_t*)nullptr, (const int64_t*)nullptr, gbuf);
            hipLaunchKernelGGL(k_gather8, dim3(g2), dim3(256), 0, stream, (const int64_t*)trig_d.p, nc, INT64_MAX,
                               (const int64_t*)db.col[dp.ts_col], (const int64_t*)nullptr, (const int64_t*)nullptr, gbuf + nc);
            hipMemcpyAsync(out_a, gbuf, (size_t)nc * 8, hipMemcpyDeviceToHost, stream);
            hipMemcpyAsync(out_t, gbuf + nc, (size_t)nc * 8, hipMemcpyDeviceToHost, stream);
        }
        g_row_arr = nullptr;
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "trigger evaluation failed");
        return 0;
    }

    // ------------------------------------------------------------------ poll
    int poll(int32_t memory, ek_result* out) {
        memset(out, 0, sizeof *out);
        int64_t nw = (int64_t)wins.size();
        out->n_windows = nw;
        out->n_aggs = n_out;
        out->memory = memory;
        std::vector<int64_t> wc(nw);
        std::vector<int32_t> we(nw);
        std::vector<int64_t> wmc(nw);
        std::vector<uint64_t> wmh(nw);
        if (nw) {
            hipMemcpyAsync(wc.data(), r_wcnt.p, nw * 8, hipMemcpyDeviceToHost, stream);
            hipMemcpyAsync(we.data(), r_werr.p, nw * 4, hipMemcpyDeviceToHost, stream);
            if (plan.debug_membership) {
                hipMemcpyAsync(wmc.data(), r_wmc.p, nw * 8, hipMemcpyDeviceToHost, stream);
                hipMemcpyAsync(wmh.data(), r_wmh.p, nw * 8, hipMemcpyDeviceToHost, stream);
            }
        }
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "poll sync failed");
        if (int rc = window_messages(we)) return rc;
        h_ws.assign(nw, 0); h_we.assign(nw, 0); h_off.assign(nw, 0); h_cnt.assign(nw, 0); h_st.assign(nw, 0);
        h_mc.assign(nw, 0); h_mh.assign(nw, 0);
        int64_t total = 0;
        for (int64_t w = 0; w < nw; ++w) {
            h_ws[w] = wins[w].start;
            h_we[w] = wins[w].end;
            h_st[w] = we[w];
            h_cnt[w] = we[w] ? 0 : wc[w];   // an errored window emits only its error (operations.go:108-113)
            h_mc[w] = wmc[w];
            h_mh[w] = wmh[w];
            total += h_cnt[w];
        }
        stats.rows_out += total;
        out->win_start = h_ws.data();
        out->win_end = h_we.data();
        out->win_row_count = h_cnt.data();
        out->win_status = h_st.data();
        out->win_member_count = h_mc.data();
        out->win_member_hash = h_mh.data();
        if (memory == EK_MEM_DEVICE) {
            for (int64_t w = 0; w < nw; ++w) h_off[w] = wins[w].out_base;
            out->win_row_offset = h_off.data();
            out->n_rows = r_rows_used;
            out->key = (uint32_t*)r_key.p;
            for (int k = 0; k < n_out; ++k) {
                out->agg_value[k] = (int64_t*)r_val[k].p;
                out->agg_tag[k] = (uint8_t*)r_tag[k].p;
            }
            return 0;
        }
        h_key.resize(total);
        for (int k = 0; k < n_out; ++k) { h_val[k].resize(total); h_tag[k].resize(total); }
        int64_t o = 0;
        for (int64_t w = 0; w < nw; ++w) {
            h_off[w] = o;
            int64_t c = h_cnt[w];
            if (c) {
                int64_t base = wins[w].out_base;
                hipMemcpyAsync(h_key.data() + o, (uint32_t*)r_key.p + base, c * 4, hipMemcpyDeviceToHost, stream);
                for (int k = 0; k < n_out; ++k) {
                    hipMemcpyAsync(h_val[k].data() + o, (int64_t*)r_val[k].p + base, c * 8, hipMemcpyDeviceToHost, stream);
                    hipMemcpyAsync(h_tag[k].data() + o, (uint8_t*)r_tag[k].p + base, c, hipMemcpyDeviceToHost, stream);
                }
            }
            o += c;
        }
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "poll copy failed");
        out->win_row_offset = h_off.data();
        out->n_rows = total;
        out->key = h_key.data();
        for (int k = 0; k < n_out; ++k) { out->agg_value[k] = h_val[k].data(); out->agg_tag[k] = h_tag[k].data(); }
        return 0;
    }

    // The error text of each failed window of this poll (ek_window_error): the operator's message re-evaluated on the
    // host over the window's witness (ek_errmsg.h). Precedence follows the reference's operator order: FilterOp, then
    // HavingOp, then ProjectOp (planner.go:387-446) — a window the WHERE failed never reaches HAVING.
    static const char* order_stat_error(int fn) {   // funcs_agg.go:321-326,357-362 over stats v0.7.1 ErrBounds
        if (fn == EK_AGG_MEDIAN) return "<nil> should be number";   // funcs_agg.go:51-52 (a nil first value)
        return fn == EK_AGG_PERCENTILE_DISC ? "PopulationVariance exec with error: Input is outside of range."
                                            : "percentile exec with error: Input is outside of range.";
    }
    HVal wit_value(const WitRec& r, int k, bool agg) const {
        HVal v;
        switch (r.tag[k]) {
        case V_BOOL: v.tag = HVal::BOOL; v.i = r.v[k]; break;
        case V_I64: v.tag = HVal::I64; v.i = r.v[k]; break;
        case V_F64: v.tag = HVal::F64; memcpy(&v.f, &r.v[k], 8); break;
        case V_ERR: v = hv_err(agg ? order_stat_error(dp.agg_fn[k]) : "invalid value"); break;
        default: break;
        }
        return v;
    }
    int window_messages(const std::vector<int32_t>& we) {
        const int64_t nw = (int64_t)we.size();
        poll_msgs.assign((size_t)nw, std::string());
        bool any = false;
        for (int32_t e : we) any |= e != 0;
        if (!any) return 0;
        std::vector<WitRec> wit;
        std::vector<int32_t> as;
        if (r_wwit.p) {
            wit.resize((size_t)nw * 2);
            hipMemcpyAsync(wit.data(), r_wwit.p, (size_t)nw * 2 * sizeof(WitRec), hipMemcpyDeviceToHost, stream);
        }
        if (r_aslot.p) {
            as.resize((size_t)nw);
            hipMemcpyAsync(as.data(), r_aslot.p, (size_t)nw * 4, hipMemcpyDeviceToHost, stream);
        }
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "error witness copy failed");
        const DPlan& dp = inc_where ? dp_incw : this->dp;   // WHERE over an incremental window: k_inc_where's programs
        for (int64_t w = 0; w < nw; ++w) {
            const int32_t st = we[w];
            if (!st) continue;
            std::string m;
            if (st == EK_WIN_WHERE_ERROR) {
                if (!wit.empty() && wit[2 * w].set) {
                    const WitRec& r = wit[2 * w];
                    const HVal v = h_eval_prog(dp.where_prog, dp.n_where, [&](int c) { return wit_value(r, c, false); },
                                               [&](int) { return HVal{}; });
                    m = condition_error("run Where error: ", v, true);
                }
                if (m.empty()) m = "run Where error: (no witness row recorded)";
            } else if (!wit.empty() && wit[2 * w + 1].set) {
                const WitRec& r = wit[2 * w + 1];
                const HVal v = h_eval_prog(dp.having_prog, dp.n_having, [&](int) { return HVal{}; },
                                           [&](int k) { return wit_value(r, k, true); });
                m = condition_error("run Having error: ", v, false);
            }
            if (m.empty() && !as.empty() && as[w] > 0) {
                // the first failed order statistic: HavingOp meets it first when HAVING reads it, ProjectOp otherwise
                const int a = kMaxSortAggs - as[w];
                const int slot = dp.sagg_agg[a];
                bool in_having = false;
                for (int k = 0; k < dp.n_having; ++k)
                    in_having |= dp.having_prog[k].op == EK_OP_AGG && dp.having_prog[k].arg == slot;
                m = std::string(in_having ? "run Having error: " : "run Select error: ") + order_stat_error(dp.agg_fn[slot]);
            }
            if (m.empty()) m = st == EK_WIN_HAVING_ERROR ? "run Having error: (no witness group recorded)" : "run Select error";
            poll_msgs[(size_t)w] = std::move(m);
        }
        return 0;
    }
    int window_error(int64_t w, char* buf, int64_t cap, int64_t* len) {
        if (w < 0 || w >= (int64_t)poll_msgs.size()) return fail(EK_ERR_INVALID, "window %lld not in the last poll", (long long)w);
        const std::string& m = poll_msgs[(size_t)w];
        if (len) *len = (int64_t)m.size();
        if (buf && cap > 0) {
            const size_t n = std::min<size_t>(m.size(), (size_t)cap - 1);
            memcpy(buf, m.data(), n);
            buf[n] = 0;
        }
        return 0;
    }

    int release_results() {
        // windows handed out are dropped; device regions are recycled
        int64_t nw = (int64_t)wins.size();
        if (nw && r_wcnt.p)
            hipLaunchKernelGGL(k_zero_wins, dim3((unsigned)std::min<int64_t>(1024, (nw + 255) / 256)), dim3(256), 0, stream, nw,
                               (int64_t*)r_wcnt.p, (int32_t*)r_werr.p, (int64_t*)r_wmc.p, (int64_t*)r_wmh.p);
        if (nw && r_wwit.p) hipMemsetAsync(r_wwit.p, 0, (size_t)nw * 2 * sizeof(WitRec), stream);
        if (nw && r_aslot.p) hipMemsetAsync(r_aslot.p, 0, (size_t)nw * 4, stream);
        wins.clear();
        r_rows_used = 0;
        return 0;
    }

    int reset() {
        // asynchronous mode: stream-ordered, the zeroing of the result counters queues behind the previous push
        if (!async_push) hipStreamSynchronize(stream);
        release_results();
        reset_state();
        return async_push || hipStreamSynchronize(stream) == hipSuccess ? 0 : fail(EK_ERR_DEVICE, "reset sync failed");
    }

    // ------------------------------------------------------------------ checkpoint (ek_export_state / ek_import_state)
    // The state the reference checkpoints through ctx.PutState — WatermarkOp's lastWatermarkTs and buffered events
    // (watermark_op.go:204-211), WindowOperator's inputs / triggerTime / msgCount (window_op.go:283-340,419-420,
    // event_window_trigger.go:196) — in this engine's representation: watermark and window cursor, the accepted
    // events still waiting for the first window end, and either the partials of every open pane (pane mode) or the
    // event-buffer rows a future window can still contain (range mode). Sections are 8-byte aligned, host order.
    static constexpr uint64_t kStateMagic = 0x31305453474B4545ull;   // "EEKGST01"
    static constexpr int64_t kStateVersion = 8;   // 3: the processing-time clock and timers; 4: pane WHERE witnesses;
                                                  // 5: processing-time incremental windows; 6: ek_stats totals;
                                                  // 7: event-time send-twice prevWindowEndTs; 8: ek_stats v13

    // FNV-1a over the plan fields that shape the state (a blob only restores into the same rule)
    uint64_t plan_hash() const {
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](const void* p, size_t n) {
            const uint8_t* b = (const uint8_t*)p;
            for (size_t k = 0; k < n; ++k) { h ^= b[k]; h *= 1099511628211ull; }
        };
        auto i32 = [&](int32_t v) { mix(&v, 4); };
        auto i64 = [&](int64_t v) { mix(&v, 8); };
        i32(plan.window_type); i32(plan.time_unit); i32(plan.length); i32(plan.interval); i32(plan.delay);
        i32(plan.is_event_time); i32(plan.tz_offset_s); i64(plan.late_tolerance_ms); i32(plan.n_columns);
        for (int c = 0; c < plan.n_columns; ++c) i32(plan.column_type[c]);
        i32(plan.ts_column); i32(plan.key_column); i32((int32_t)plan.num_keys); i32(plan.debug_membership);
        i32((int32_t)plan.nullable_mask); i32(plan.n_aggs);
        for (int k = 0; k < plan.n_aggs; ++k) {
            i32(plan.aggs[k].fn); i32(plan.aggs[k].column);
            if (plan.aggs[k].fn == EK_AGG_PERCENTILE_CONT || plan.aggs[k].fn == EK_AGG_PERCENTILE_DISC) mix(&plan.aggs[k].param, 8);
        }
        auto prog = [&](const ek_instr* p, int n) {
            i32(n);
            for (int k = 0; k < n; ++k) {
                i32(p[k].op); i32(p[k].arg);
                if (p[k].op == EK_OP_CONST_I64 || p[k].op == EK_OP_CONST_BOOL) i64(p[k].i64);
                if (p[k].op == EK_OP_CONST_F64) mix(&p[k].f64, 8);
            }
        };
        prog(plan.where_prog, plan.n_where);
        prog(plan.having_prog, plan.n_having);
        prog(plan.trigger_prog, plan.n_trigger);
        prog(plan.filter_prog, plan.n_filter);   // FILTER (WHERE ...) decides which rows the panes / buffer hold
        i32(plan.sliding_send_twice);
        i32(plan.inc_unaligned);
        if (wtype == EK_WINDOW_STATE) {
            prog(plan.begin_prog, plan.n_begin);
            prog(plan.emit_prog, plan.n_emit);
        }
        i32(range_mode ? 1 : 0);
        return h;
    }

    struct StateOut {
        std::vector<uint8_t> b;
        void put(const void* p, size_t n) {
            if (n) b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n);
            while (b.size() & 7) b.push_back(0);
        }
        void i64(int64_t v) { put(&v, 8); }
    };
    struct StateIn {
        const uint8_t* p;
        int64_t n, o;
        bool ok;
        const uint8_t* take(int64_t k) {
            if (!ok || k < 0 || k > n - o) { ok = false; return nullptr; }
            const uint8_t* r = p + o;
            o = std::min(n, o + ((k + 7) & ~(int64_t)7));
            return r;
        }
        bool read(void* dst, int64_t k) {
            const uint8_t* r = take(k);
            if (r && k) memcpy(dst, r, (size_t)k);
            return r != nullptr;
        }
        int64_t i64() { int64_t v = 0; read(&v, 8); return v; }
    };
    // device bytes -> blob (the stream was drained by the caller)
    int dev_append(StateOut& s, const void* d, size_t n) {
        const size_t o = s.b.size();
        s.b.resize(o + ((n + 7) & ~(size_t)7), 0);
        if (n && (hipMemcpyAsync(s.b.data() + o, d, n, hipMemcpyDeviceToHost, stream) != hipSuccess ||
                  hipStreamSynchronize(stream) != hipSuccess))
            return fail(EK_ERR_DEVICE, "state copy (device -> host) failed");
        return 0;
    }
    // blob -> device
    int dev_restore(StateIn& r, void* d, size_t n) {
        const uint8_t* p = r.take((int64_t)n);
        if (!p) return fail(EK_ERR_INVALID, "state blob truncated");
        if (n && hipMemcpyAsync(d, p, n, hipMemcpyHostToDevice, stream) != hipSuccess)
            return fail(EK_ERR_DEVICE, "state copy (host -> device) failed");
        return 0;
    }

    int export_state(void* buf, int64_t cap, int64_t* size) {
        if (!wins.empty()) return fail(EK_ERR_STATE, "poll and release the results before exporting the state");
        if (!range_mode && reg_win != next_win) return fail(EK_ERR_STATE, "windows registered but not emitted");
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "sync failed");
        StateOut s;
        s.i64((int64_t)kStateMagic);
        s.i64(kStateVersion);
        s.i64((int64_t)plan_hash());
        // watermark and window cursor (WatermarkKey, TriggerTimeKey, MsgCountKey)
        for (int64_t v : {(int64_t)has_M, M, (int64_t)has_W, W, (int64_t)e1_known, E1, first_ts, next_win, reg_win,
                          arrivals, grid.origin, grid.P, (int64_t)grid.tumbling})
            s.i64(v);
        s.put(&stats, sizeof stats);
        // accepted events before the first release (EventInputKey)
        s.i64(pend_n);
        s.i64(pend_min);
        s.i64(pend_max);
        for (int c = 0; c < plan.n_columns; ++c) {
            s.i64(pend_has_valid[c] ? 1 : 0);
            s.put(pend_host[c].data(), pend_host[c].size());
            if (pend_has_valid[c]) s.put(pend_vhost[c].data(), pend_vhost[c].size());
        }
        s.put(pend_arr.data(), pend_arr.size() * 8);
        // processing time: the caller's clock and the timers armed by it (tickers, session timeout, delayed sliding
        // triggers, the send-twice inputs state) — the import resumes the rule exactly where the export left it
        for (int64_t v : {(int64_t)clock_started, clock_ms, ps_tick, (int64_t)ps_to_exists, (int64_t)ps_to_armed, ps_to_due,
                          ps_next_abs, ps_last_nonmatch, sw2_cut, sw2_gcb, sw2_gcx})
            s.i64(v);
        s.i64((int64_t)(proc_dq.size() - proc_dq_head));
        s.put(proc_dq.data() + proc_dq_head, (proc_dq.size() - proc_dq_head) * 8);
        s.i64((int64_t)sw2_e.size());
        s.put(sw2_e.data(), sw2_e.size() * 8);
        if (wtype != EK_WINDOW_NONE && !range_mode) {
            // partials of every open pane: field-major SoA, field f of slot x at ((f * ring) + x) * Kpad
            const int nf = n_state_fields();
            const int64_t first_live = win_first_pane(next_win);
            std::vector<int> live;
            for (int x = 0; x < ring; ++x)
                if (slot_pane[x] != INT64_MIN && slot_pane[x] >= first_live) live.push_back(x);
            s.i64(Kpad);
            s.i64(nf);
            s.i64(ring);
            s.i64((int64_t)live.size());
            const size_t per = (size_t)Kpad * 8;
            for (int x : live) {
                s.i64(slot_pane[x]);
                for (int f = 0; f < nf; ++f)
                    if (int rc = dev_append(s, (char*)state_buf.p + ((size_t)f * ring + x) * per, per)) return rc;
                if (int rc = dev_append(s, (char*)pane_err.p + (size_t)x * 4, 4)) return rc;
                if (int rc = dev_append(s, (char*)pane_mcnt.p + (size_t)x * 8, 8)) return rc;
                if (int rc = dev_append(s, (char*)pane_mhash.p + (size_t)x * 8, 8)) return rc;
                if (pane_wit.p)   // the pane's WHERE witness (a plan whose WHERE can fail: the same plan on import)
                    if (int rc = dev_append(s, (char*)pane_wit.p + (size_t)x * sizeof(WitRec), sizeof(WitRec))) return rc;
            }
        }
        if (range_mode) {
            // event-buffer rows from the oldest row a future window can start at (WindowInputsKey)
            const int64_t drop = std::max<int64_t>(0, std::min(eb_floor, eb.n));
            const int64_t live = eb.n - drop;
            uint32_t vmask = 0;
            for (int c = 0; c < plan.n_columns; ++c) if (eb_valid_on[c]) vmask |= 1u << c;
            for (int64_t v : {eb_base + drop, eb_rel - drop, eb_floor - drop, live, sW, range_wins, count_k, (int64_t)vmask,
                              (int64_t)sess_last_ticked, (int64_t)sess_has_trigger, sess_trigger})
                s.i64(v);
            if (live) {
                for (int c = 0; c < plan.n_columns; ++c) {
                    if (int rc = dev_append(s, (char*)eb.col[c].p + drop * col_es(c), (size_t)live * col_es(c))) return rc;
                    if (eb_valid_on[c])
                        if (int rc = dev_append(s, (uint8_t*)eb.valid[c].p + drop, (size_t)live)) return rc;
                }
                if (int rc = arr_materialize()) return rc;
                if (int rc = dev_append(s, (int64_t*)eb.arr.p + drop, (size_t)live * 8)) return rc;
                if (need_rel) if (int rc = dev_append(s, (int64_t*)eb.rel.p + drop, (size_t)live * 8)) return rc;
            }
            const int64_t nd = (int64_t)(delayq.size() - delayq_head);   // queued delayed sliding triggers
            s.i64(nd);
            s.put(delayq.data() + delayq_head, (size_t)nd * sizeof(DelayTrig));
            s.i64(h_rts_base);                                                // session: released timestamps
            s.i64((int64_t)h_rts.size());
            s.put(h_rts.data(), h_rts.size() * 8);
            s.i64((int64_t)h_rtrig.size());                                   // send-twice: OVER (WHEN) flags
            s.put(h_rtrig.data(), h_rtrig.size());
            s.i64(inc_has_T ? 1 : 0);                                         // incremental windows: T + open windows
            s.i64(inc_T);
            s.i64((int64_t)inc_pend.size());
            s.put(inc_pend.data(), inc_pend.size() * sizeof(IncWin));
            s.i64(st_on ? 1 : 0);                                             // state window: onBegin + its first row
            s.i64(st_start_abs);
            // processing-time incremental windows (v5): ticker, the open windows, the delay timers
            for (int64_t v : {pi_tick, pi_D, (int64_t)pi_cur, pi_cur_start, pi_cur_first, pi_next_abs}) s.i64(v);
            s.i64((int64_t)(pi_hop.size() - pi_hop_head));
            s.put(pi_hop.data() + pi_hop_head, (pi_hop.size() - pi_hop_head) * sizeof(PiHop));
            s.i64((int64_t)(pi_dq.size() - pi_dq_head));
            s.put(pi_dq.data() + pi_dq_head, (pi_dq.size() - pi_dq_head) * 8);
            s.i64(v2_lastW);                                                  // delayed v2 sliding: delayTS queue
            s.i64((int64_t)(v2q.size() - v2q_head));
            s.put(v2q.data() + v2q_head, (v2q.size() - v2q_head) * sizeof(V2Delay));
            s.i64(et2_prev);                                                  // event-time send-twice (v7)
        }
        *size = (int64_t)s.b.size();
        if (!buf) return 0;
        if (cap < *size) return fail(EK_ERR_INVALID, "state buffer too small (%lld < %lld bytes)", (long long)cap, (long long)*size);
        memcpy(buf, s.b.data(), s.b.size());
        return 0;
    }

    int import_state(const void* buf, int64_t size) {
        if (!buf || size < 24) return fail(EK_ERR_INVALID, "state blob too short");
        StateIn r{(const uint8_t*)buf, size, 0, true};
        if ((uint64_t)r.i64() != kStateMagic || r.i64() != kStateVersion)
            return fail(EK_ERR_INVALID, "not an ekgpu state blob of version %lld", (long long)kStateVersion);
        if ((uint64_t)r.i64() != plan_hash()) return fail(EK_ERR_INVALID, "state blob was exported by a different plan");
        if (int rc = reset()) return rc;
        int rc = import_body(r, size);
        if (rc == 0 && !r.ok) rc = fail(EK_ERR_INVALID, "state blob truncated");
        if (rc == 0 && hipStreamSynchronize(stream) != hipSuccess) rc = fail(EK_ERR_DEVICE, "state restore sync failed");
        if (rc) {
            const std::string e = err;
            reset();
            err = e;
        }
        return rc;
    }

    int import_body(StateIn& r, int64_t size) {
        has_M = r.i64() != 0; M = r.i64();
        has_W = r.i64() != 0; W = r.i64();
        e1_known = r.i64() != 0; E1 = r.i64(); first_ts = r.i64();
        next_win = r.i64(); reg_win = r.i64(); arrivals = r.i64();
        grid.origin = r.i64(); grid.P = r.i64(); grid.tumbling = (int32_t)r.i64();
        r.read(&stats, sizeof stats);
        pend_n = r.i64(); pend_min = r.i64(); pend_max = r.i64();
        if (pend_n < 0 || pend_n > size) return fail(EK_ERR_INVALID, "bad pending-event count");
        for (int c = 0; c < plan.n_columns; ++c) {
            pend_has_valid[c] = r.i64() != 0;
            pend_host[c].resize((size_t)pend_n * col_es(c));
            r.read(pend_host[c].data(), (int64_t)pend_host[c].size());
            if (pend_has_valid[c]) {
                pend_vhost[c].resize((size_t)pend_n);
                r.read(pend_vhost[c].data(), pend_n);
            }
        }
        pend_arr.resize((size_t)pend_n);
        r.read(pend_arr.data(), pend_n * 8);
        clock_started = r.i64() != 0; clock_ms = r.i64(); ps_tick = r.i64();
        ps_to_exists = r.i64() != 0; ps_to_armed = r.i64() != 0; ps_to_due = r.i64();
        ps_next_abs = r.i64(); ps_last_nonmatch = r.i64(); sw2_cut = r.i64(); sw2_gcb = r.i64(); sw2_gcx = r.i64();
        {
            const int64_t nq = r.i64();
            if (!r.ok || nq < 0 || nq > size) return fail(EK_ERR_INVALID, "bad timer queue in state blob");
            proc_dq.resize((size_t)nq);
            proc_dq_head = 0;
            r.read(proc_dq.data(), nq * 8);
            const int64_t ne = r.i64();
            if (!r.ok || ne < 0 || ne > size) return fail(EK_ERR_INVALID, "bad send-twice state in state blob");
            sw2_e.resize((size_t)ne);
            r.read(sw2_e.data(), ne * 8);
        }
        if (!r.ok) return fail(EK_ERR_INVALID, "state blob truncated");
        if (wtype != EK_WINDOW_NONE && !range_mode) {
            const int64_t kp = r.i64(), nf = r.i64(), R = r.i64(), nl = r.i64();
            if (kp != Kpad || nf != n_state_fields() || R < 1 || R > (1 << 24) || nl < 0 || nl > R)
                return fail(EK_ERR_INVALID, "pane state does not match this plan");
            if (int rc = ensure_ring(R)) return rc;
            const size_t per = (size_t)Kpad * 8;
            for (int64_t l = 0; l < nl; ++l) {
                const int64_t q = r.i64();
                const int x = (int)(q % ring);
                if (!r.ok || q < 0 || slot_pane[x] != INT64_MIN) return fail(EK_ERR_INVALID, "bad pane in state blob");
                slot_pane[x] = q;
                for (int f = 0; f < nf; ++f)
                    if (int rc = dev_restore(r, (char*)state_buf.p + ((size_t)f * ring + x) * per, per)) return rc;
                if (int rc = dev_restore(r, (char*)pane_err.p + (size_t)x * 4, 4)) return rc;
                if (int rc = dev_restore(r, (char*)pane_mcnt.p + (size_t)x * 8, 8)) return rc;
                if (int rc = dev_restore(r, (char*)pane_mhash.p + (size_t)x * 8, 8)) return rc;
                if (pane_wit.p)
                    if (int rc = dev_restore(r, (char*)pane_wit.p + (size_t)x * sizeof(WitRec), sizeof(WitRec))) return rc;
            }
        }
        if (range_mode) {
            const int64_t base = r.i64(), rel = r.i64(), floor = r.i64(), live = r.i64();
            const int64_t sw = r.i64(), rw = r.i64(), ck = r.i64(), vmask = r.i64();
            const int64_t slt = r.i64(), sht = r.i64(), strig = r.i64();
            if (!r.ok || live < 0 || live > size) return fail(EK_ERR_INVALID, "bad event-buffer size in state blob");
            eb.n = 0;
            eb_floor = eb_rel = 0;
            for (int c = 0; c < plan.n_columns; ++c)
                if ((vmask >> c) & 1) if (int rc = eb_enable_valid(c)) return rc;
            if (int rc = eb_reserve(live)) return rc;
            for (int c = 0; c < plan.n_columns; ++c) {
                if (int rc = dev_restore(r, eb.col[c].p, (size_t)live * col_es(c))) return rc;
                if ((vmask >> c) & 1) { if (int rc = dev_restore(r, eb.valid[c].p, (size_t)live)) return rc; }
                else if (eb_valid_on[c]) fill_valid_ones(c, 0, live);
            }
            if (int rc = arr_materialize()) return rc;   // eb.n == 0 here: allocates the column
            if (int rc = dev_restore(r, eb.arr.p, (size_t)live * 8)) return rc;
            if (need_rel) if (int rc = dev_restore(r, eb.rel.p, (size_t)live * 8)) return rc;
            eb.n = live;
            eb_base = base;
            eb_rel = rel;
            eb_floor = floor;
            sW = sw;
            range_wins = rw;
            count_k = ck;
            sess_last_ticked = slt != 0;
            sess_has_trigger = sht != 0;
            sess_trigger = strig;
            const int64_t nd = r.i64();
            if (!r.ok || nd < 0 || nd > size) return fail(EK_ERR_INVALID, "bad delay queue in state blob");
            delayq.resize((size_t)nd);
            r.read(delayq.data(), nd * (int64_t)sizeof(DelayTrig));
            delayq_head = 0;
            h_rts_base = r.i64();
            const int64_t nr = r.i64();
            if (!r.ok || nr < 0 || nr > size) return fail(EK_ERR_INVALID, "bad session mirror in state blob");
            h_rts.resize((size_t)nr);
            r.read(h_rts.data(), nr * 8);
            const int64_t nf = r.i64();
            if (!r.ok || nf < 0 || nf > size) return fail(EK_ERR_INVALID, "bad trigger mirror in state blob");
            h_rtrig.resize((size_t)nf);
            r.read(h_rtrig.data(), nf);
            inc_has_T = r.i64() != 0;
            inc_T = r.i64();
            const int64_t ni = r.i64();
            if (!r.ok || ni < 0 || ni > size) return fail(EK_ERR_INVALID, "bad incremental windows in state blob");
            inc_pend.resize((size_t)ni);
            r.read(inc_pend.data(), ni * (int64_t)sizeof(IncWin));
            st_on = r.i64() != 0;
            st_start_abs = r.i64();
            pi_tick = r.i64(); pi_D = r.i64(); pi_cur = r.i64() != 0; pi_cur_start = r.i64(); pi_cur_first = r.i64();
            pi_next_abs = r.i64();
            const int64_t nh = r.i64();
            if (!r.ok || nh < 0 || nh > size) return fail(EK_ERR_INVALID, "bad incremental hopping windows in state blob");
            pi_hop.resize((size_t)nh);
            pi_hop_head = 0;
            r.read(pi_hop.data(), nh * (int64_t)sizeof(PiHop));
            const int64_t nq = r.i64();
            if (!r.ok || nq < 0 || nq > size) return fail(EK_ERR_INVALID, "bad incremental delay timers in state blob");
            pi_dq.resize((size_t)nq);
            pi_dq_head = 0;
            r.read(pi_dq.data(), nq * 8);
            v2_lastW = r.i64();
            const int64_t nv = r.i64();
            if (!r.ok || nv < 0 || nv > size) return fail(EK_ERR_INVALID, "bad v2 delay queue in state blob");
            v2q.resize((size_t)nv);
            v2q_head = 0;
            v2q_seen = (size_t)nv;
            r.read(v2q.data(), nv * (int64_t)sizeof(V2Delay));
            et2_prev = r.i64();
            if (!r.ok) return fail(EK_ERR_INVALID, "state blob truncated");
        }
        return 0;
    }

    ~Engine() {
        if (stream) hipStreamSynchronize(stream);
        release(state_buf); release(pane_err); release(pane_mcnt); release(pane_mhash); release(bstats); release(bstats_part);
        release(cmax); release(acc); release(bounds_val); release(bounds_idx); release(chist); release(totals);
        release(pstart); release(pcursor); release(direct_d);
        release(st_klo);
        for (int v = 0; v < kMaxVC; ++v) { release(st_val[v]); release(st_valid[v]); }
        for (int c = 0; c < EK_MAX_COLUMNS; ++c) { release(in_cols[c]); release(in_valid[c]); release(pend_cols[c]); release(pend_valid[c]); }
        release(pend_arr_d);
        release(wdesc); release(r_key); release(r_wcnt); release(r_werr); release(r_wmc); release(r_wmh);
        release(pane_wit); release(r_wwit); release(r_aslot); release(vp_wit);
        for (int k = 0; k < EK_MAX_AGGS; ++k) { release(r_val[k]); release(r_tag[k]); }
        if (d_plan) hipFree(d_plan);
        if (d_plan_where) hipFree(d_plan_where);
        if (d_plan_incw) hipFree(d_plan_incw);
        if (h_stats) hipHostFree(h_stats);
        if (h_small) hipHostFree(h_small);
        if (h_wdesc) hipHostFree(h_wdesc);
        if (h_desc) hipHostFree(h_desc);
        release(aux_d);
        for (EvBuf* e : {&eb, &eb_alt}) {
            for (int c = 0; c < EK_MAX_COLUMNS; ++c) { release(e->col[c]); release(e->valid[c]); }
            release(e->arr);
            release(e->rel);
        }
        for (DevBuf* d : {&rq_d, &ab_d, &slot_d, &trig_d, &flags_d, &cnts_d, &runmax_d, &runcm_d, &mrg_keys[0], &mrg_keys[1],
                          &mrg_src[0], &mrg_src[1], &mrg_tmp, &mrg_tail, &mrg_bidx, &mrg_col, &vp_err, &vp_mc, &vp_mh, &sort_pbase, &sort_scr, &chunk_pa, &sw_d,
                          &km_k[0], &km_k[1], &km_p[0], &km_p[1], &km_tmp, &km_start, &km_ab, &km_bcnt, &km_flag, &rowpos, &ff_d,
                          &grp_tiles, &grp_cnt, &grp_base, &sw_redo})
            release(*d);
        for (int v = 0; v < kMaxVC; ++v) { release(km_val[v]); release(km_ok[v]); }
        if (h_kmf) hipHostFree(h_kmf);
        if (h_scalar) hipHostFree(h_scalar);
        if (msd_ht) hipHostFree(msd_ht);
        if (ev0) hipEventDestroy(ev0);
        if (ev1) hipEventDestroy(ev1);
        if (ev_h2d) hipEventDestroy(ev_h2d);
        for (auto& e : phase_ev) { hipEventDestroy(e.a); hipEventDestroy(e.b); }
        phase_ev.clear();
        if (stream && own_stream) hipStreamDestroy(stream);
    }
};

// ---------------------------------------------------------------------- C ABI
static thread_local std::string g_create_error;

extern "C" {

int ek_abi_version(void) { return EKGPU_ABI_VERSION; }

int ek_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int ek_create(const ek_plan* plan, int device, void** out_handle) {
    if (!plan || !out_handle) return EK_ERR_INVALID;
    *out_handle = nullptr;
    // init selects `device`: give the calling thread its current device back
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    struct Restore { int d; ~Restore() { if (d >= 0) hipSetDevice(d); } } restore{prev};
    Engine* e = new (std::nothrow) Engine();
    if (!e) return EK_ERR_NOMEM;
    int rc = e->init(plan, device);
    if (rc) {
        g_create_error = e->err;
        delete e;
        return rc;
    }
    *out_handle = e;
    return 0;
}

// Every entry point runs on the handle's device whatever the calling thread's current device is (a Go node may call
// from any OS thread; the bench runs two rules on two host threads), and gives the caller its device back.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(void* h) {
        if (!h) return;
        const int dev = ((Engine*)h)->device;
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) hipSetDevice(dev);
        else prev = -1;
    }
    ~DeviceGuard() { if (prev >= 0) hipSetDevice(prev); }
};

int ek_push_batch(void* h, const ek_batch* batch) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    return ((Engine*)h)->push(batch);
}

int ek_batch_ts_stats(void* h, const ek_batch* batch, ek_ts_stats* out) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    return ((Engine*)h)->ts_stats_of(batch, out);
}

int ek_poll_results(void* h, int32_t memory, ek_result* out) {
    if (!h || !out) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    return ((Engine*)h)->poll(memory, out);
}

int ek_window_error(void* h, int64_t w, char* buf, int64_t cap, int64_t* len) {
    if (!h) return EK_ERR_INVALID;
    return ((Engine*)h)->window_error(w, buf, cap, len);
}

int ek_release_results(void* h, ek_result* res) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    if (res) memset(res, 0, sizeof *res);
    return ((Engine*)h)->release_results();
}

int ek_reset(void* h) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    return ((Engine*)h)->reset();
}

int ek_sync(void* h) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    return hipStreamSynchronize(((Engine*)h)->stream) == hipSuccess ? 0 : EK_ERR_DEVICE;
}

int ek_set_stream(void* h, void* s) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    Engine* e = (Engine*)h;
    hipStreamSynchronize(e->stream);
    if (s) {
        if (e->own_stream) hipStreamDestroy(e->stream);
        e->stream = (hipStream_t)s;
        e->own_stream = false;
    } else if (!e->own_stream) {
        hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
        e->own_stream = true;
    }
    return 0;
}

int ek_set_async(void* h, int32_t on) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    Engine* e = (Engine*)h;
    int rc = 0;
    if (!on) { hipStreamSynchronize(e->stream); rc = e->fold_time(); }
    e->async_push = on != 0;
    return rc;
}

int ek_set_phase_timing(void* h, int32_t on) {
    if (!h) return EK_ERR_INVALID;
    ((Engine*)h)->phase_events = on != 0;
    return 0;
}

int ek_get_stats(void* h, ek_stats* out) {
    if (!h || !out) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    const int rc = ((Engine*)h)->fold_time();
    *out = ((Engine*)h)->stats;
    return rc;
}

const char* ek_last_error(void* h) {
    if (!h) return g_create_error.c_str();
    return ((Engine*)h)->err.c_str();
}

int ek_destroy(void* h) {
    DeviceGuard dg(h);
    delete (Engine*)h;
    return 0;
}

int ek_push_batch_global(void* h, const ek_batch* batch, const ek_global_ctx* g) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    return ((Engine*)h)->push_global(batch, g);
}

int ek_advance_time(void* h, int64_t now_ms) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    return static_cast<Engine*>(h)->advance_time(now_ms);
}

int ek_advance_watermark(void* h, int64_t wm_ms, int64_t arrivals_end) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    Engine* e = (Engine*)h;
    if (e->wtype == EK_WINDOW_SESSION)   // the sessions a tuple closes travel in ek_global_ctx.sess_* only
        return e->fail(EK_ERR_INVALID, "a SESSIONWINDOW shard takes watermark advances through ek_push_batch_global "
                                       "(with the router's session list), not ek_advance_watermark");
    const int64_t a = std::max<int64_t>(0, arrivals_end - 1);
    ek_global_ctx g{};
    g.arrivals_end = arrivals_end;
    g.wm_arrival = &a;
    g.wm_ts = &wm_ms;
    g.n_wm = 1;
    g.memory = EK_MEM_HOST;
    return e->push_global(nullptr, &g);
}

int ek_shard_triggers(void* h, const ek_batch* batch, const ek_global_ctx* g, int64_t* out_arrival, int64_t* out_ts,
                      int64_t cap, int64_t* n_out) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    return ((Engine*)h)->shard_triggers(batch, g, out_arrival, out_ts, cap, n_out);
}

int ek_export_state(void* h, void* buf, int64_t cap, int64_t* size) {
    if (!h || !size) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    return ((Engine*)h)->export_state(buf, cap, size);
}

int ek_import_state(void* h, const void* buf, int64_t size) {
    if (!h) return EK_ERR_INVALID;
    DeviceGuard dg(h);
    return ((Engine*)h)->import_state(buf, size);
}

}  // extern "C"
