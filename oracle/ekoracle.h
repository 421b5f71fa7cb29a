/*
 * ekoracle.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference's per-tuple algorithm for the window/aggregate hot path,
 * used as the parity checker for the HIP engine. It is NEVER linked into, loaded by or called from
 * the product path (libekgpu.so / ekgpu python package); only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it.
 *
 * The reference (LF Edge eKuiper v2, Go) cannot be compiled here (no Go toolchain),
 * so this restatement is pinned by the reference's own known-answer tests, transcribed as fixtures
 * under tests/golden/ (funcs_agg_test.go, window_op_test.go, topotest/window_rule_test.go, ...).
 * Each function cites the reference file:line it restates.
 */
#ifndef EKORACLE_H
#define EKORACLE_H

#include <stdint.h>
#include "../include/ekgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int32_t status;            /* 0 ok, <0 plan error */
    char error[256];
    int64_t records_late;      /* events dropped by WatermarkOp.track */
    ek_result r;               /* host arrays owned by the oracle */
    /* window content in window order: arrival indices of each window's members (before WHERE) */
    int64_t* member_offset;    /* [n_windows + 1] */
    int64_t* members;
    /* per window error text (only for win_status != 0), 128 bytes each */
    char* win_error;
    int64_t records_filter_error;   /* rows a pushed-down WHERE / the window FILTER dropped with an evaluation error */
} eko_output;

/* Run the whole stream (arrival order) through the reference operator chain. */
int eko_run(const ek_plan* plan, int64_t n_rows, const void* const* columns,
            const uint8_t* const* validity, eko_output* out);
void eko_free(eko_output* out);

/* Processing-time TUMBLING / HOPPING / SLIDING / SESSION under a deterministic clock (execProcessingWindow with the
 * reference's mock clock): the rule opens at start_ms, each row is delivered when the clock reaches its timestamp
 * (its arrival time), and the clock finally moves to end_ms. */
int eko_run_proc(const ek_plan* plan, int64_t n_rows, const void* const* columns, const uint8_t* const* validity,
                 int64_t start_ms, int64_t end_ms, eko_output* out);
/* The same with a checkpoint / restart (window_op.go:131-168,268-325): rows [0, split) delivered, the clock at
 * export_ms, the rule restarted at restart_ms (timers gone, tickers re-aligned, the restored inputs replayed), then
 * rows [split, n). split < 0: no restart. */
typedef struct { int64_t split, export_ms, restart_ms; } eko_restart;
int eko_run_proc_restart(const ek_plan* plan, int64_t n_rows, const void* const* columns, const uint8_t* const* validity,
                         int64_t start_ms, int64_t end_ms, const eko_restart* rs, eko_output* out);

/* Shard model of the multi-GPU protocol: one key-hash shard's rows (global arrivals g->row_arrival) with the
 * global WatermarkTuples / window anchor / sliding triggers of the whole stream (g: host memory). */
int eko_run_shard(const ek_plan* plan, int64_t n_rows, const void* const* columns, const uint8_t* const* validity,
                  const ek_global_ctx* g, eko_output* out);
/* The shard's accepted trigger rows (arrival, ts) in arrival order; returns their number (out_* sized n_rows). */
int64_t eko_shard_triggers(const ek_plan* plan, int64_t n_rows, const void* const* columns, const uint8_t* const* validity,
                           const ek_global_ctx* g, int64_t* out_arrival, int64_t* out_ts);

/* window_op.go:194-227 getAlignedWindowEndTime, with time.Local = UTC + tz_offset_s. */
int64_t eko_aligned_window_end(int64_t ts_ms, int32_t interval, int32_t unit, int32_t tz_offset_s);

/* Direct aggregate-function call as in funcs_agg_test.go (builtins[name].exec), bypassing the
 * operator `check` guard. values: int64 or double per col_type; valid may be NULL.
 * Returns 0 ok, 1 error (message in err). out_tag EK_TAG_*. */
int eko_agg_exec(int32_t fn, int32_t col_type, int64_t n, const void* values, const uint8_t* valid,
                 double param, int64_t* out_value, uint8_t* out_tag, char* err, int32_t err_len);

#ifdef __cplusplus
}
#endif
#endif
