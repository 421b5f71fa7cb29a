/*
 * ekgpu.h — C ABI of the MI355X window & aggregate engine.
 *
 * This is the drop-in boundary for the hot path of an eKuiper rule:
 *   [Watermark] -> WindowOperator -> [FilterOp] -> AggregateOp -> [HavingOp] -> ProjectOp(agg fields)
 * i.e. the operator chain planned by internal/topo/planner/planner.go:387-446 (buildOps) and executed
 * by internal/topo/node/{watermark_op.go,window_op.go,event_window_trigger.go} and
 * internal/topo/operator/{filter,aggregate,having,project}_operator.go in the reference.
 *
 * One handle = one rule's window/aggregate node (reference: one WindowOperator goroutine,
 * window_op.go:131-192, plus the UnaryOperator chain behind it, node/operations.go:42-130).
 * A handle is single-consumer (not internally locked); distinct handles are independent.
 * All entry points return 0 on success and a negative EK_ERR_* code on failure; the message
 * is available from ek_last_error(h) and carries the reference's error prefixes
 * ("run Where error: ...", "run Having error: ...", "run Window error: ...").
 *
 * Plain C types only: no HIP or torch types cross this boundary.  Device pointers are passed
 * as void* together with EK_MEM_DEVICE.
 */
#ifndef EKGPU_H
#define EKGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EKGPU_ABI_VERSION 14
#define EK_MAX_COLUMNS 16
#define EK_MAX_AGGS 16
#define EK_MAX_PROG 48
#define EK_MAX_DERIVED 4

/* Window types: identical values to pkg/ast/statement.go:185-193 (ast.WindowType). */
enum {
    EK_WINDOW_NONE = 0,
    EK_WINDOW_TUMBLING = 1,
    EK_WINDOW_HOPPING = 2,
    EK_WINDOW_SLIDING = 3,
    EK_WINDOW_SESSION = 4,
    EK_WINDOW_COUNT = 5,
    EK_WINDOW_STATE = 6         /* STATEWINDOW(begin, emit): WindowV2Operator only (window_v2_op.go:94-148) */
};

/* WindowRange reported by a state window (window_v2_op.go:111-148 emitWindow(time.Time{}, InfTime)):
 * time.Time{}.UnixMilli() and InfTime.UnixMilli() (window_v2_op.go:30, the int64 product wraps in Go). */
#define EK_STATE_WINDOW_START_MS (-62135596800000LL)
#define EK_STATE_WINDOW_END_MS (-62135596800001LL)

/* Time units of the window literal (pkg/ast/token.go:117-121: DD, HH, MI, SS, MS). */
enum { EK_UNIT_DD = 1, EK_UNIT_HH = 2, EK_UNIT_MI = 3, EK_UNIT_SS = 4, EK_UNIT_MS = 5 };

/* Column storage types. Stream schema BIGINT -> EK_COL_I64, FLOAT -> EK_COL_F64
 * (converter/json/converter.go:429-460); group ids are dictionary-encoded EK_COL_U32. */
enum { EK_COL_I64 = 1, EK_COL_F64 = 2, EK_COL_U32 = 3 };
/* BOOLEAN (converter.go:362-380 -> Go bool): stored as int64 0 / 1, evaluated as a bool (the literals true / false are
 * EK_OP_CONST_BOOL); a WHERE / FILTER / window-condition operand, a count() argument and a SELECT * column.
 * EK_COL_STR is an ingest type only (ek_json_decode): the string's FNV-1a 64 hash in an int64 column plus its byte range
 * (ek_json_strings), resolved to a dense EK_COL_U32 id by the host dictionary before the engine sees it. */
enum { EK_COL_STR = 4, EK_COL_BOOL = 5 };
/* ABI v14. EK_COL_LIST is an ingest type only (ek_json_decode): a JSON array field (schema ARRAY(elem), converter.go
 * decodeArray :173-244) whose elements of type ek_json_schema.elem_type (EK_COL_I64 / EK_COL_F64 / EK_COL_BOOL) are
 * read through ek_json_list; the batch carries no column for it (columns[c] = NULL, validity = the array's own nil). */
enum { EK_COL_LIST = 6 };

/* Aggregate functions (internal/binder/function/funcs_agg.go:28-370). */
enum {
    EK_AGG_COUNT_STAR = 1,      /* count(*)                         funcs_agg.go:87-95            */
    EK_AGG_COUNT = 2,           /* count(col): non-nil values       common_array_funcs.go:101-109 */
    EK_AGG_SUM = 3,             /* funcs_agg.go:114-143                                           */
    EK_AGG_AVG = 4,             /* funcs_agg.go:56-86 (int: truncating int64 division)            */
    EK_AGG_MIN = 5,             /* funcs_agg.go:105-113, common_array_funcs.go:59-99              */
    EK_AGG_MAX = 6,             /* funcs_agg.go:96-104,  common_array_funcs.go:27-57              */
    EK_AGG_STDDEV = 7,          /* stats.StandardDeviation          funcs_agg.go:206-228          */
    EK_AGG_STDDEVS = 8,         /* stats.StandardDeviationSample    funcs_agg.go:229-251          */
    EK_AGG_VAR = 9,             /* stats.Variance                   funcs_agg.go:252-274          */
    EK_AGG_VARS = 10,           /* stats.SampleVariance             funcs_agg.go:275-297          */
    EK_AGG_MEDIAN = 11,         /* funcs_agg.go:29-55,415-428                                     */
    EK_AGG_PERCENTILE_CONT = 12,/* stats.Percentile(sorted, p*100)  funcs_agg.go:298-334          */
    EK_AGG_PERCENTILE_DISC = 13,/* stats.PercentileNearestRank      funcs_agg.go:335-370          */
    EK_AGG_FIRST = 14           /* a non-aggregate select field: the column's value in the group's
                                   FIRST row (row.go:720-726, project_operator.go:136-207); ABI v6   */
};

/* Expression programs (WHERE / HAVING / OVER(WHEN ...)) in postfix form.
 * Evaluation follows xsql.ValuerEval.evalBinaryExpr / SimpleDataEval (internal/xsql/valuer.go:574-1000):
 * nil in a relational or logical op yields false, nil in arithmetic yields nil, int64 op float64
 * promotes to float64, divide/mod by zero is an error. */
enum {
    EK_OP_COL = 1,       /* push column[arg] of the current row (NULL when invalid)          */
    EK_OP_AGG = 2,       /* push aggregate slot[arg] of the current group (HAVING only)       */
    EK_OP_CONST_I64 = 3, /* push i64                                                          */
    EK_OP_CONST_F64 = 4, /* push f64                                                          */
    EK_OP_EQ = 5, EK_OP_NEQ = 6, EK_OP_LT = 7, EK_OP_LTE = 8, EK_OP_GT = 9, EK_OP_GTE = 10,
    EK_OP_AND = 11, EK_OP_OR = 12,
    EK_OP_ADD = 13, EK_OP_SUB = 14, EK_OP_MUL = 15, EK_OP_DIV = 16, EK_OP_MOD = 17,
    EK_OP_CONST_BOOL = 18 /* push bool (i64 != 0): the literals true / false (ast.BooleanLiteral)     */
};

typedef struct {
    int32_t op;
    int32_t arg;
    int64_t i64;
    double f64;
} ek_instr;

typedef struct {
    int32_t fn;      /* EK_AGG_*                                   */
    int32_t column;  /* argument column (ignored for count(*))     */
    double param;    /* percentile fraction p (percentile_* only)  */
} ek_agg_spec;

/* Compiled rule. POD with fixed arrays so a cgo / ctypes caller can fill it in place. */
typedef struct {
    int32_t abi_version;          /* must be EKGPU_ABI_VERSION                                  */
    int32_t window_type;          /* EK_WINDOW_*                                                */
    int32_t time_unit;            /* EK_UNIT_* (time windows)                                   */
    int32_t length;               /* raw literal: TUMBLINGWINDOW(ss,10) -> 10; COUNTWINDOW(n) -> n */
    int32_t interval;             /* HOPPINGWINDOW hop / SESSIONWINDOW timeout / COUNTWINDOW m   */
    int32_t delay;                /* SLIDINGWINDOW delay                                         */
    int32_t is_event_time;        /* def.RuleOption.IsEventTime                                  */
    int32_t tz_offset_s;          /* local-time offset used by window alignment (time.Local)    */
    int64_t late_tolerance_ms;    /* def.RuleOption.LateTol                                      */
    int32_t n_columns;
    int32_t column_type[EK_MAX_COLUMNS];
    int32_t ts_column;            /* TIMESTAMP column (i64 epoch ms); -1 for processing time     */
    int32_t key_column;           /* GROUP BY dimension as dense u32 id; -1 = no GROUP BY       */
    uint32_t num_keys;            /* exclusive bound of key ids                                 */
    int32_t debug_membership;     /* 1: report per-window member count + member-set hash        */
    uint32_t nullable_mask;       /* bit c: column c may carry a validity array (NULLs)         */
    int32_t n_aggs;
    ek_agg_spec aggs[EK_MAX_AGGS];
    int32_t n_where;
    ek_instr where_prog[EK_MAX_PROG];
    int32_t n_having;
    ek_instr having_prog[EK_MAX_PROG];
    int32_t n_trigger;            /* SLIDINGWINDOW(...) OVER (WHEN <prog>)                       */
    ek_instr trigger_prog[EK_MAX_PROG];
    /* def.RuleOption.PlanOptimizeStrategy.EnableIncrementalWindow (def/rule.go:55-61): the planner's
     * incremental-aggregation window (planner.go:905-997 rewriteIfIncAggStmt -> IncWindowPlan ->
     * node.NewWindowIncAggOp, window_inc_agg_op.go:59-101 / window_inc_agg_event_op.go). Honoured for
     * event-time TUMBLING/HOPPING/SLIDING (no delay), COUNTWINDOW(n) in either time mode, when every aggregate is one of
     * count/sum/avg/min/max (function.IsSupportedIncAgg, funcs_inc_agg.go:28-41); with another aggregate
     * the reference planner keeps the regular path and so does the engine. Inc semantics: windows are
     * created by the events themselves (HoppingWindowIncAggEventOp.triggerWindow), each group reports
     * the inc_* values computed at its last row, inc_sum / inc_avg are float64 (funcs_inc_agg.go:56-117). */
    int32_t incremental;
    /* def.RuleOption.PlanOptimizeStrategy.WindowOption.WindowVersion (def/rule.go:68-76): 2 selects
     * node.NewWindowV2Op (planner.go:416-425). EK_WINDOW_STATE exists only there and is accepted with any
     * value; for the other window types only 0/1 (the regular WindowOperator) is built. */
    int32_t window_version;
    /* STATEWINDOW(<begin>, <emit>) (parser.go:1047-1053,1119-1124; StateWindowOp.exec, window_v2_op.go:111-148).
     * Rows are taken in arrival order (processing time) or release order (event time: after WatermarkOp).
     * While no window is open, a row whose begin condition is true opens one; every row of an open window
     * joins it and a row whose emit condition is true closes it and emits the rows since the opening row
     * (WindowRange = [time.Time{}, InfTime] in ms: -62135596800000, -62135596800001 after Go's int64 wrap).
     * A row that both opens and closes a window opens the next one at the following row. A nil, non-bool
     * or failing condition is false (isMatchCondition, window_v2_op.go:212-238). */
    int32_t n_begin;
    ek_instr begin_prog[EK_MAX_PROG];
    int32_t n_emit;
    ek_instr emit_prog[EK_MAX_PROG];
    /* Aggregate arguments that are expressions: GroupedTuples.AggregateEval evaluates the argument on every row of the
     * group (internal/xsql/row.go:712-718). Derived column d is column index n_columns + d (an aggregate's `column`
     * may name it); its value per row is derived_prog[d] over the stream's columns and constants with the valuer's
     * arithmetic (valuer.go:861-1000: int64 op int64 stays int64 - integer division truncates -, any float64
     * operand promotes, % on floats is math.Mod, a nil operand gives nil). Built for + - * and / % by a non-zero
     * constant (a zero divisor is an evaluation error the aggregate functions would have to see per row);
     * derived_type[d] is the expression's result type (EK_COL_I64 / EK_COL_F64). */
    int32_t n_derived;
    int32_t derived_type[EK_MAX_DERIVED];
    int32_t n_derived_prog[EK_MAX_DERIVED];
    ek_instr derived_prog[EK_MAX_DERIVED][EK_MAX_PROG];
    /* ABI v8. The window's FILTER (WHERE <cond>) clause (WindowPlan.condition, planner.go:388-392,639-641): a FilterOp
     * planned between the WatermarkOp and the window, so a row whose condition is not true never reaches the window —
     * it is no member, no OVER (WHEN) trigger and no gcInputs edge — while it still moved the watermark (event time).
     * An evaluation error drops the row and is counted in ek_stats.records_filter_error (the reference forwards that
     * row's error, filter_operator.go:41-57). In processing time under TUMBLING / HOPPING / SESSION the planner combines
     * it with WHERE and pushes both below the window (windowPlan.go:82-99: WHERE AND FILTER). */
    int32_t n_filter;
    ek_instr filter_prog[EK_MAX_PROG];
    /* ABI v8. def.RuleOption.PlanOptimizeStrategy.WindowOption.EnableSendSlidingWindowTwice (def/rule.go:104-112,
     * window_op.go:98): a SLIDINGWINDOW with a delay D emits the rows (t - length, t] when its trigger t fires and the
     * rows (t, t + D] when the delay expires (handleInputsForSlidingWindow, window_op.go:576-603; the second part's
     * WindowRange is [t, t + D]). Ignored for every other window. */
    int32_t sliding_send_twice;
    /* ABI v11. node.EnableAlignWindow = false (window_inc_agg_op.go:34-38,369-377,693-699; the reference's own tests set
     * it): processing-time incremental TUMBLING / HOPPING windows tick every interval from the rule's start instead of
     * from the aligned window end (getFirstTimer), and a tumbling window is opened by its first row only. 0 = the
     * production default (aligned). Ignored for every other window. */
    int32_t inc_unaligned;
} ek_plan;

enum { EK_MEM_HOST = 0, EK_MEM_DEVICE = 1 };

/* ABI v10. Statistics of a batch's timestamp column, computed once by ek_batch_ts_stats and shared by every rule that
 * reads the same batch: eKuiper fans one source out to all the rules subscribed to it (internal/topo/subtopo.go:
 * SrcSubTopo.AddOutput / the shared source node), and each rule's WatermarkOp then scans the same timestamps again
 * (watermark_op.go:118-155). A push whose batch carries matching statistics skips its own pass over the column. */
typedef struct {
    int64_t n_rows;      /* rows they describe (a push with another n_rows ignores them)             */
    int32_t ts_column;   /* the column they were computed over (a rule with another ts column ignores them) */
    int32_t unsorted;    /* 1 when some ts[i] < ts[i - 1]                                             */
    int64_t ts_min, ts_max;
    int64_t ts_first;    /* ts[0]                                                                     */
    int64_t max_step;    /* max over i >= 1 of ts[i] - ts[i - 1] (INT64_MIN for one row)              */
    const void* ts_data; /* ABI v11: the timestamp column they describe (batch->columns[ts_column] when computed);
                          * a push whose timestamp column is another pointer ignores them, so statistics left over from
                          * the previous micro-batch of the same size are never trusted                           */
} ek_ts_stats;

/* One columnar micro-batch in arrival order. */
typedef struct {
    int64_t n_rows;
    const void* columns[EK_MAX_COLUMNS];
    const uint8_t* validity[EK_MAX_COLUMNS]; /* 1 byte per row, 1 = valid; NULL = all valid */
    int32_t memory;                          /* EK_MEM_HOST or EK_MEM_DEVICE                */
    const ek_ts_stats* ts_stats;             /* ABI v10: host memory; NULL = none            */
} ek_batch;

/* Per-row value tags of aggregate outputs (Go dynamic type of the reference's result). */
enum { EK_TAG_NULL = 0, EK_TAG_I64 = 1, EK_TAG_F64 = 2, EK_TAG_BOOL = 3 /* value 0 / 1: a BOOLEAN column of SELECT * */ };

/* Window status (window-level error replaces the window's output, node/operations.go:108-113). */
enum { EK_WIN_OK = 0, EK_WIN_WHERE_ERROR = 1, EK_WIN_HAVING_ERROR = 2, EK_WIN_AGG_ERROR = 3 };

/* Results emitted since the previous poll, segmented by window in trigger order.
 * Rows of window w are [win_row_offset[w], win_row_offset[w] + win_row_count[w]).
 * Row order inside a window is unspecified (the reference emits groups in Go map order,
 * aggregate_operator.go:67-72). Values are 8-byte slots interpreted through the tags. */
typedef struct {
    int64_t n_windows;
    int64_t* win_start;            /* WindowRange.windowStart (window_op.go:688-716 quirks kept) */
    int64_t* win_end;
    int64_t* win_row_offset;
    int64_t* win_row_count;
    int32_t* win_status;
    int64_t* win_member_count;     /* debug_membership: events in the window before WHERE        */
    uint64_t* win_member_hash;     /* debug_membership: sum of ek_mix64(arrival index)           */
    int64_t n_rows;
    uint32_t* key;
    int64_t* agg_value[EK_MAX_AGGS];  /* bit pattern of int64 or double per tag */
    uint8_t* agg_tag[EK_MAX_AGGS];
    int32_t n_aggs;
    int32_t memory;                /* where the arrays live */
    void* _owner;                  /* engine-private */
} ek_result;

typedef struct {
    int64_t records_in;       /* events pushed                                  */
    int64_t records_late;     /* dropped by the watermark (watermark_op.go:144-155) */
    int64_t windows_out;      /* windows triggered                              */
    int64_t rows_out;         /* result rows                                    */
    double last_batch_device_ms; /* device time of the last push (HIP events)   */
    /* Device time of the last push per phase (HIP events on the engine stream around each launch):
     * [EK_PHASE_STATS] batch statistics + pane bounds, [EK_PHASE_PARTITION] k_part (with a fused sorted pass: the
     * ts read too),
     * [EK_PHASE_AGGREGATE] k_agg, [EK_PHASE_FINALIZE] k_finalize. */
    double phase_ms[4];
    int64_t phase_launches[4];
    int64_t records_filter_error; /* window-less rules: events whose WHERE evaluation errored      */
    int64_t records_discarded;    /* hopping windows: inputs dropped when a triggered window is empty
                                   * (handleInputs returns inputs[:0], window_op.go:605-655)          */
    int64_t windows_keymajor;     /* range windows aggregated key-major (sorted once by key, one thread
                                   * per key walks the windows)                        */
    /* Running totals over every timed push (ek_push_batch returns once its work is queued; its device time is read
     * back by the next push or by ek_get_stats, so per-push fields describe the last push read back). */
    double device_ms_total;
    double phase_ms_total[4];
    int64_t phase_launches_total[4];
    int64_t pushes_timed;
    /* ABI v13. Pane-mode batches taken by the fused sorted pass (the partition pass checks the batch's ts order, finds
     * its pane bounds and the hopping gap itself: no separate ts pass), and passes discarded because the batch was not
     * sorted (or spanned more panes per chunk than presumed): those batches ran the general path instead. */
    int64_t fused_batches;
    int64_t fused_discarded;
} ek_stats;

enum { EK_PHASE_STATS = 0, EK_PHASE_PARTITION = 1, EK_PHASE_AGGREGATE = 2, EK_PHASE_FINALIZE = 3 };

/* Error codes. */
enum {
    EK_OK = 0,
    EK_ERR_INVALID = -1,
    EK_ERR_UNSUPPORTED = -2,
    EK_ERR_DEVICE = -3,
    EK_ERR_NOMEM = -4,
    EK_ERR_STATE = -5
};

/* Library / device */
int ek_abi_version(void);
int ek_device_count(void);

/* Create an engine instance for a compiled rule on HIP device `device`.
 * Replaces node.NewWindowOp (window_op.go:93-122) + operator.{FilterOp,AggregateOp,HavingOp}
 * as wired by planner.buildOps (planner.go:387-446). Plan errors mirror NewEventTimeTrigger
 * (event_window_trigger.go:35-53), e.g. COUNTWINDOW with event time -> EK_ERR_UNSUPPORTED. */
int ek_create(const ek_plan* plan, int device, void** out_handle);

/* Ingest one micro-batch (arrival order). Replaces the per-tuple channel ingest of
 * WatermarkOp (watermark_op.go:118-129) and WindowOperator (event_window_trigger.go:182-196,
 * window_op.go:339-419). Windows whose end passes the new watermark are triggered and their
 * GROUP BY results become available to ek_poll_results. */
int ek_push_batch(void* h, const ek_batch* batch);

/* Compute `out` for `batch` over the handle's timestamp column, on the handle's stream (one pass over the column,
 * synchronous). Set batch->ts_stats = out before pushing the batch into this and every other event-time rule over the
 * same source. EK_ERR_STATE for a rule without a timestamp column. (ABI v10) */
int ek_batch_ts_stats(void* h, const ek_batch* batch, ek_ts_stats* out);

/* Take the results produced so far. memory = EK_MEM_HOST copies them to host memory owned by
 * the engine; EK_MEM_DEVICE hands out device pointers. Valid until ek_release_results. */
int ek_poll_results(void* h, int32_t memory, ek_result* out);
int ek_release_results(void* h, ek_result* res);

/* The error text of window w (0 <= w < n_windows) of the last ek_poll_results: what the reference's operator chain
 * broadcasts in place of a failed window's rows (node/operations.go:108-113) — FilterOp "run Where error: ..."
 * (filter_operator.go:45-58), HavingOp "run Having error: ..." (having_operator.go:45-55), ProjectOp
 * "run Select error: ..." (project_operator.go:79-102), e.g. "run Where error: divided by zero" or
 * "run Having error: invalid condition that returns non-bool value int64(3)"; "" when win_status is EK_WIN_OK.
 * The text comes from the window's first failed row in window order (WHERE) or its failed group with the smallest
 * key (HAVING: the reference's groups come out of a Go map, any failed group's text is one it can print).
 * *len = the text's length; buf (cap bytes) receives it NUL-terminated, truncated to cap - 1 (buf NULL: length only).
 * Valid until the next ek_poll_results. (ABI v9) */
int ek_window_error(void* h, int64_t w, char* buf, int64_t cap, int64_t* len);

/* Forget all stream state (watermark, open windows, unpolled results) but keep the device
 * allocations, so that a new stream can be pushed without re-creating the handle. */
int ek_reset(void* h);

/* Wait for all work queued on the handle's stream. */
int ek_sync(void* h);
/* Use the caller's HIP stream (hipStream_t passed as void*; NULL = handle-owned stream). */
int ek_set_stream(void* h, void* hip_stream);
/* Asynchronous pushes (on != 0; default off): ek_push_batch / ek_advance_time return once their work is queued on
 * the handle's stream, and ek_reset queues its zeroing behind it, so the caller's work between two pushes overlaps
 * the device tail of the first. A device-memory batch stays borrowed until the next push, ek_sync, ek_poll_results
 * or ek_get_stats returns; a host-memory batch (pageable or pinned) is copied before its push returns. An error of
 * queued work is returned by the next push, ek_advance_time, ek_get_stats or ek_set_async(h, 0) (EK_ERR_DEVICE).
 * Turning it off waits for queued work. */
int ek_set_async(void* h, int32_t on);
/* Per-phase device timing (on != 0, the default): every push brackets its statistics / partition / aggregate /
 * finalize launches with HIP events, read into ek_stats.phase_ms / phase_*_total. Each event is a queue marker that
 * costs the push ≈ 5-10 µs of device idle, so a caller that samples the phase times (bench.py: one step in four) turns
 * it off for the other pushes; their phase counters then do not move. Instrumentation only (no reference
 * counterpart; the reference exposes operator metrics, internal/topo/node/metric). */
int ek_set_phase_timing(void* h, int32_t on);
int ek_get_stats(void* h, ek_stats* out);
const char* ek_last_error(void* h);
int ek_destroy(void* h);

/* Checkpoint / restore of the stream state of a handle: what the reference's checkpoint coordinator
 * saves through ctx.PutState and restores through ctx.GetState for this chain —
 *   WatermarkOp: WatermarkKey / EventInputKey / StreamWMKey    (watermark_op.go:72-101,149,204-211)
 *   WindowOperator: WindowInputsKey / TriggerTimeKey / MsgCountKey (window_op.go:83-85,131-168,283-340,
 *                   event_window_trigger.go:196).
 * The blob holds the watermark, the window cursor, the partial aggregates of every open pane (pane mode)
 * or the buffered events a future window can still contain (range mode), and the counters. It is a
 * host-side byte string bound to the plan: a hash of the ek_plan fields is checked on import.
 * ek_export_state: results must have been polled and released first (EK_ERR_STATE otherwise).
 *   *size = bytes of the blob; buf == NULL only queries the size; cap < *size -> EK_ERR_INVALID.
 * ek_import_state: replaces the handle's stream state (ek_reset, then restore); unpolled results are dropped. */
int ek_export_state(void* h, void* buf, int64_t cap, int64_t* size);
int ek_import_state(void* h, const void* buf, int64_t size);

/* ---------------------------------------------------------------- external / global watermark (sharding)
 * The reference splits the chain into WatermarkOp -> WindowOperator: WatermarkOp tracks the stream, drops
 * late events and emits a WatermarkTuple at every advance (watermark_op.go:144-225); the WindowOperator closes
 * windows on those tuples (event_window_trigger.go:126-180). A key-hash shard of a rule (one handle per GPU)
 * keeps that split: the host that assigns the global arrival order runs the WatermarkOp tracking over the
 * WHOLE stream and broadcasts its WatermarkTuples; every shard receives only its own rows, each with its
 * global arrival index. A handle enters this mode at its first ek_push_batch_global / ek_advance_watermark
 * (before any ek_push_batch) and stays in it until ek_reset; its own rows no longer move its watermark.
 * Built for event-time TUMBLING / HOPPING / SLIDING (no delay) / SESSION and processing-time COUNTWINDOW
 * (global arrival blocks); other windows -> EK_ERR_UNSUPPORTED (state windows depend on every row of the
 * stream). A SESSIONWINDOW's gaps depend on every row's timestamp: the router runs getNextSessionWindow over
 * the whole stream (ekgpu/shard.py GlobalSession, event_window_trigger.go:77-180) and hands every shard the
 * sessions it closed (sess_*); a shard fires each over its own rows with ts < sess_end. Global un-grouped
 * aggregates are merged across shards by the caller (ekgpu/dist.py). */
typedef struct {
    const int64_t* row_arrival;   /* per row of the batch: global arrival index, strictly increasing       */
    int64_t arrivals_end;         /* global arrivals after this batch (>= last row_arrival + 1)           */
    /* WatermarkTuples emitted while the batch's global arrivals were tracked, in order: the tuple k follows
     * the event of global arrival wm_arrival[k] and carries watermark wm_ts[k] (strictly increasing)       */
    const int64_t* wm_arrival;
    const int64_t* wm_ts;
    int64_t n_wm;
    /* event time: the first window's alignment anchor (getEarliestEventTs at the first WatermarkTuple that
     * released an event, event_window_trigger.go:57-75,211-219): valid when origin_known != 0; the tuple
     * that released it is the last one with wm_arrival <= origin_arrival */
    int32_t origin_known;
    /* hints from the host's WatermarkOp (0 = unknown): all_accepted = no event of this batch was late;
     * max_wm_step = the largest advance between consecutive WatermarkTuples (from the previous batch's last one).
     * With all_accepted and (no hopping window with lateTolerance 0, or max_wm_step <= its length) a pane-mode
     * shard needs only the batch's last tuple: no per-row watermark search. */
    int32_t all_accepted;
    int64_t max_wm_step;
    int64_t origin_ts;
    int64_t origin_arrival;
    /* SLIDINGWINDOW: the accepted trigger events of the WHOLE stream in this batch (every shard's, from
     * ek_shard_triggers + an all-gather), in arrival order: (global arrival, ts) */
    const int64_t* trig_arrival;
    const int64_t* trig_ts;
    int64_t n_trig;
    int32_t memory;               /* EK_MEM_HOST or EK_MEM_DEVICE: where row_arrival lives (the other arrays
                                   * are always host memory) */
    int32_t pad2;
    /* SESSIONWINDOW (ABI v7): the sessions the WHOLE stream's WatermarkTuples of this batch closed, in order:
     * window [sess_start[k], sess_end[k]) fired at the tuple of watermark sess_wm[k] (a value of wm_ts) */
    const int64_t* sess_start;
    const int64_t* sess_end;
    const int64_t* sess_wm;
    int64_t n_sess;
} ek_global_ctx;

/* ---------------------------------------------------------------- key-hash router (ABI v13)
 * a multi-GPU rule partitions every micro-batch by gpu = hash(key) mod G. The reference has no
 * counterpart (one process; its channels fan a source out to rules, internal/topo/subtopo.go), so this entry point is
 * the router's own: the rows of a device batch (one rank's slice of the global stream, global arrivals arrival_base
 * + i) are split into n_dest segments of out_columns by owner = ek_mix64(key) & (2^62 - 1) mod n_dest, stably (each
 * segment keeps arrival order); the key column is renamed through key_map (device, key_map_size entries, global key
 * -> the owner's dense id; NULL keeps it; a key past the table is kept and the call returns EK_ERR_INVALID) and out_arrival (device, NULL = none) receives every routed row's global arrival. Segment d is
 * rows [sum(dest_counts[<d]), + dest_counts[d]) (dest_counts: host, n_dest entries). column_type gives each
 * column's width (EK_COL_U32: 4 bytes, else 8); the key column must be EK_COL_U32; validity is not routed.
 * Synchronous on `stream` (hipStream_t; NULL = the null stream) of HIP device `device`. */
int ek_route_partition(int device, void* stream, const ek_batch* batch, const int32_t* column_type, int32_t key_column,
                       int32_t n_dest, const uint32_t* key_map, uint32_t key_map_size, int64_t arrival_base,
                       void* const* out_columns, int64_t* out_arrival, int64_t* dest_counts);

/* ---------------------------------------------------------------- processing-time clock
 * Processing-time TUMBLING / HOPPING / SLIDING / SESSION windows (WindowOperator.execProcessingWindow,
 * window_op.go:235-470) run under the caller's clock, the way the reference's tests drive them with its mock clock
 * (pkg/timex/time.go:31-100): every row carries its arrival time in the plan's ts_column (non-decreasing); the clock
 * reaches a row's timestamp before the row is delivered, so every ticker / timeout due at or before it fires first.
 * ek_advance_time(h, now) moves the clock with no rows: the first call (before any row) is the rule's start, which
 * aligns the tickers (getAlignedWindowEndTime(start, rawInterval)); without it the first row's time is the start.
 * The clock never moves back (EK_ERR_INVALID). Windows the clock closes are polled like any other. */
int ek_advance_time(void* h, int64_t now_ms);

/* One micro-batch of a shard: the rows owned by this handle plus the global context above. */
int ek_push_batch_global(void* h, const ek_batch* batch, const ek_global_ctx* g);
/* A WatermarkTuple with no new rows (event_window_trigger.go:126-146): the global watermark reached wm_ms after
 * `arrivals_end` global arrivals. Equivalent to ek_push_batch_global with an empty batch and one tuple.
 * A SESSIONWINDOW shard is refused (EK_ERR_INVALID): the sessions such a tuple closes only travel in
 * ek_global_ctx.sess_*, so it takes ek_push_batch_global with an empty batch instead. */
int ek_advance_watermark(void* h, int64_t wm_ms, int64_t arrivals_end);
/* The rows of `batch` (global arrivals g->row_arrival) that are accepted by the global watermark and match
 * SLIDINGWINDOW ... OVER (WHEN ...) (every accepted row when there is no OVER): their global arrival and ts,
 * in arrival order, up to cap (n_out = the total). g->trig_* are ignored. */
int ek_shard_triggers(void* h, const ek_batch* batch, const ek_global_ctx* g, int64_t* out_arrival, int64_t* out_ts,
                      int64_t cap, int64_t* n_out);

/* ---------------------------------------------------------------- columnar JSON ingest
 * Replaces the per-message FastJsonConverter.Decode of a schema-typed stream
 * (internal/converter/json/converter.go:92-171,246-520; node/decode_op.go:146-193) with numeric, string and boolean
 * fields: a micro-batch of messages (payload bytes concatenated, message i = bytes[offsets[i], offsets[i+1])) is
 * decoded on the GPU straight into the columns of an ek_batch (device memory owned by the decoder, valid until its
 * next decode), ready for ek_push_batch.
 * Schema type BIGINT -> EK_COL_I64 (integer literal, fastfloat.ParseInt64), FLOAT -> EK_COL_F64
 * (correctly rounded, subnormal results included), a dense key id column -> EK_COL_U32 (integer literal in [0, 2^32)),
 * STRING -> EK_COL_STR (a JSON string, delivered as its dense dictionary id, ek_json_dict_*; a number is
 * cast.ToStringAlways(float64) = Go's %v of the float, converter.go:446-451; a bool, object or array
 * EK_JSON_ERR_TYPE), BOOLEAN -> EK_COL_BOOL (true / false; a number n as n != 0; a string by strconv.ParseBool,
 * converter.go:600-625; anything else EK_JSON_ERR_TYPE), ARRAY -> EK_COL_LIST (ek_json_list). null or an absent
 * field -> validity 0; fields outside the schema are skipped. Messages that fail to decode are dropped from the
 * batch and reported by ek_json_errors.
 * ABI v14, paths (ek_json_schema.paths = 1): a column name is a path into nested objects and arrays, segments
 * separated by '.', array elements as [k]: "a.b" is field b of the STRUCT a (decodeObject over schema[a].Properties,
 * converter.go:256-291), "a[0]" element 0 of the ARRAY a, "a[0][0].c" as in TestArrayWithArray. A null or absent
 * container makes the leaf nil; a container of the wrong kind (a number where the path needs an object) is
 * EK_JSON_ERR_TYPE ("a has wrong type:number, expect:struct"); a duplicated key replaces the whole subtree (Go map
 * assignment). A top-level array payload [{...}, {...}] decodes to one row per element, in order
 * (decodeWithSchema's []map case, converter.go:141-158); any element that is not an object fails the message. */
#define EK_JSON_MAX_NAME 32
enum {
    EK_JSON_OK = 0,
    EK_JSON_ERR_SYNTAX = 1,      /* fastjson parse error                                        */
    EK_JSON_ERR_TYPE = 2,        /* "%v has wrong type" (string/bool/object/array for a number)  */
    EK_JSON_ERR_NUMBER = 3,      /* not an int64 literal for BIGINT / number out of range         */
    EK_JSON_ERR_UNSUPPORTED = 4  /* forms the device decoder leaves to the Go converter (escaped keys on a path,
                                    paths deeper than 8, > 100-digit mantissas on a rounding boundary)            */
};

typedef struct {
    int32_t n_fields;
    int32_t column_type[EK_MAX_COLUMNS];           /* EK_COL_* of column i                  */
    char names[EK_MAX_COLUMNS][EK_JSON_MAX_NAME];  /* JSON key (or path) of column i (NUL-terminated) */
    int32_t elem_type[EK_MAX_COLUMNS];             /* ABI v14: EK_COL_LIST columns: the element type */
    int32_t paths;                                 /* ABI v14: 1 = names are paths ('.' and [k] segments) */
} ek_json_schema;

typedef struct {
    int64_t messages;
    int64_t errors;
    int64_t bytes;
} ek_json_stats;

int ek_json_create(const ek_json_schema* schema, int device, void** out_handle);
/* memory: where bytes/offsets live (EK_MEM_HOST: copied to the device first). out: device columns. */
int ek_json_decode(void* h, const char* bytes, int64_t n_bytes, const int64_t* offsets, int64_t n_msgs, int32_t memory,
                   ek_batch* out);
/* messages of the last decode that failed: their indices and EK_JSON_ERR_* codes (up to cap) */
int ek_json_errors(void* h, int64_t* msg_index, uint8_t* code, int64_t cap, int64_t* n_errors);
/* String column `column` of the last decode (EK_COL_STR): per decoded message, offsets[i] = the value's first content
 * byte in the payload (after the opening quote) and lengths[i] = its raw byte length, with EK_JSON_STR_ESCAPED set
 * when it holds a backslash escape (the hash then covers the escaped form: the host re-hashes the unescaped
 * string). Device pointers, valid until the next decode; 0 for a null / absent value. */
#define EK_JSON_STR_ESCAPED 0x40000000
int ek_json_strings(void* h, int column, const int64_t** offsets, const int32_t** lengths);
/* The decoder's dictionary of STRING column `column`: ek_json_decode hands the column to the engine as dense u32 ids
 * (EK_COL_U32, first-seen order over the decoder's life; 0 for a null row) — the group key a GROUP BY deviceId needs.
 * ek_json_dict_string yields id's bytes (not NUL-terminated; valid until the next decode). */
int ek_json_dict_size(void* h, int column, int64_t* n);
int ek_json_dict_string(void* h, int column, uint32_t id, const char** s, int64_t* len);
/* ABI v14. LIST column `column` of the last decode: per decoded row, start[i] / len[i] = its elements in values /
 * valid (element nil -> valid 0; a nil or absent array: len 0 and the batch validity 0); an element is int64, float64
 * bits or 0 / 1 by elem_type. Device pointers, valid until the next decode. */
int ek_json_list(void* h, int column, const int64_t** start, const int32_t** len, const int64_t** values,
                 const uint8_t** valid);
/* rows of the last decode per message (a top-level array payload yields one row per element): rows_of[i] for message
 * i, 0 for a failed one (host memory owned by the decoder, valid until the next decode) */
int ek_json_rows(void* h, const int64_t** rows_of, int64_t* n_msgs);
int ek_json_get_stats(void* h, ek_json_stats* out);
const char* ek_json_last_error(void* h);
int ek_json_destroy(void* h);

/* Membership hash used by debug_membership (splitmix64 finaliser). */
static inline uint64_t ek_mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

#ifdef __cplusplus
}
#endif

#endif /* EKGPU_H */
