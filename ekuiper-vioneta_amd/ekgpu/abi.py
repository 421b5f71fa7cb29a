"""ctypes mirror of include/ekgpu.h (the C ABI of the MI355X window/aggregate engine).

Keep this file in lock-step with the header; tests/test_abi.py checks sizes and offsets against
the compiled library's view (ek_abi_version) and the header constants.
"""
import ctypes as C

EKGPU_ABI_VERSION = 14
EK_MAX_COLUMNS = 16
EK_MAX_AGGS = 16
EK_MAX_PROG = 48
EK_MAX_DERIVED = 4

# window types == pkg/ast/statement.go:185-193
(EK_WINDOW_NONE, EK_WINDOW_TUMBLING, EK_WINDOW_HOPPING, EK_WINDOW_SLIDING, EK_WINDOW_SESSION, EK_WINDOW_COUNT,
 EK_WINDOW_STATE) = range(7)
# state windows: WindowRange [time.Time{}, InfTime] in ms (window_v2_op.go:30,111-148)
EK_STATE_WINDOW_START_MS, EK_STATE_WINDOW_END_MS = -62135596800000, -62135596800001
# time units (pkg/ast/token.go:117-121)
EK_UNIT_DD, EK_UNIT_HH, EK_UNIT_MI, EK_UNIT_SS, EK_UNIT_MS = 1, 2, 3, 4, 5
UNIT_BY_NAME = {"dd": EK_UNIT_DD, "hh": EK_UNIT_HH, "mi": EK_UNIT_MI, "ss": EK_UNIT_SS, "ms": EK_UNIT_MS}
UNIT_MS = {EK_UNIT_DD: 86400000, EK_UNIT_HH: 3600000, EK_UNIT_MI: 60000, EK_UNIT_SS: 1000, EK_UNIT_MS: 1}

EK_COL_I64, EK_COL_F64, EK_COL_U32 = 1, 2, 3
EK_COL_STR, EK_COL_BOOL = 4, 5   # STR: ingest only (ek_json_decode); BOOL: int64 0 / 1 evaluated as a Go bool
EK_COL_LIST = 6                  # ingest only (ek_json_decode, ABI v14): a JSON array field, read through ek_json_list

(EK_AGG_COUNT_STAR, EK_AGG_COUNT, EK_AGG_SUM, EK_AGG_AVG, EK_AGG_MIN, EK_AGG_MAX, EK_AGG_STDDEV,
 EK_AGG_STDDEVS, EK_AGG_VAR, EK_AGG_VARS, EK_AGG_MEDIAN, EK_AGG_PERCENTILE_CONT,
 EK_AGG_PERCENTILE_DISC, EK_AGG_FIRST) = range(1, 15)
AGG_BY_NAME = {
    "count": EK_AGG_COUNT, "sum": EK_AGG_SUM, "avg": EK_AGG_AVG, "min": EK_AGG_MIN, "max": EK_AGG_MAX,
    "stddev": EK_AGG_STDDEV, "stddevs": EK_AGG_STDDEVS, "var": EK_AGG_VAR, "vars": EK_AGG_VARS,
    "median": EK_AGG_MEDIAN, "percentile_cont": EK_AGG_PERCENTILE_CONT,
    "percentile_disc": EK_AGG_PERCENTILE_DISC,
}

(EK_OP_COL, EK_OP_AGG, EK_OP_CONST_I64, EK_OP_CONST_F64, EK_OP_EQ, EK_OP_NEQ, EK_OP_LT, EK_OP_LTE,
 EK_OP_GT, EK_OP_GTE, EK_OP_AND, EK_OP_OR, EK_OP_ADD, EK_OP_SUB, EK_OP_MUL, EK_OP_DIV,
 EK_OP_MOD, EK_OP_CONST_BOOL) = range(1, 19)

EK_MEM_HOST, EK_MEM_DEVICE = 0, 1
EK_TAG_NULL, EK_TAG_I64, EK_TAG_F64, EK_TAG_BOOL = 0, 1, 2, 3
EK_WIN_OK, EK_WIN_WHERE_ERROR, EK_WIN_HAVING_ERROR, EK_WIN_AGG_ERROR = 0, 1, 2, 3
EK_OK, EK_ERR_INVALID, EK_ERR_UNSUPPORTED, EK_ERR_DEVICE, EK_ERR_NOMEM, EK_ERR_STATE = 0, -1, -2, -3, -4, -5


class ek_instr(C.Structure):
    _fields_ = [("op", C.c_int32), ("arg", C.c_int32), ("i64", C.c_int64), ("f64", C.c_double)]


class ek_agg_spec(C.Structure):
    _fields_ = [("fn", C.c_int32), ("column", C.c_int32), ("param", C.c_double)]


class ek_plan(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32),
        ("window_type", C.c_int32),
        ("time_unit", C.c_int32),
        ("length", C.c_int32),
        ("interval", C.c_int32),
        ("delay", C.c_int32),
        ("is_event_time", C.c_int32),
        ("tz_offset_s", C.c_int32),
        ("late_tolerance_ms", C.c_int64),
        ("n_columns", C.c_int32),
        ("column_type", C.c_int32 * EK_MAX_COLUMNS),
        ("ts_column", C.c_int32),
        ("key_column", C.c_int32),
        ("num_keys", C.c_uint32),
        ("debug_membership", C.c_int32),
        ("nullable_mask", C.c_uint32),
        ("n_aggs", C.c_int32),
        ("aggs", ek_agg_spec * EK_MAX_AGGS),
        ("n_where", C.c_int32),
        ("where_prog", ek_instr * EK_MAX_PROG),
        ("n_having", C.c_int32),
        ("having_prog", ek_instr * EK_MAX_PROG),
        ("n_trigger", C.c_int32),
        ("trigger_prog", ek_instr * EK_MAX_PROG),
        ("incremental", C.c_int32),
        ("window_version", C.c_int32),
        ("n_begin", C.c_int32),
        ("begin_prog", ek_instr * EK_MAX_PROG),
        ("n_emit", C.c_int32),
        ("emit_prog", ek_instr * EK_MAX_PROG),
        ("n_derived", C.c_int32),
        ("derived_type", C.c_int32 * EK_MAX_DERIVED),
        ("n_derived_prog", C.c_int32 * EK_MAX_DERIVED),
        ("derived_prog", (ek_instr * EK_MAX_PROG) * EK_MAX_DERIVED),
        ("n_filter", C.c_int32),
        ("filter_prog", ek_instr * EK_MAX_PROG),
        ("sliding_send_twice", C.c_int32),
        ("inc_unaligned", C.c_int32),
    ]


class ek_ts_stats(C.Structure):
    _fields_ = [
        ("n_rows", C.c_int64),
        ("ts_column", C.c_int32),
        ("unsorted", C.c_int32),
        ("ts_min", C.c_int64),
        ("ts_max", C.c_int64),
        ("ts_first", C.c_int64),
        ("max_step", C.c_int64),
        ("ts_data", C.c_void_p),
    ]


class ek_batch(C.Structure):
    _fields_ = [
        ("n_rows", C.c_int64),
        ("columns", C.c_void_p * EK_MAX_COLUMNS),
        ("validity", C.c_void_p * EK_MAX_COLUMNS),
        ("memory", C.c_int32),
        ("ts_stats", C.POINTER(ek_ts_stats)),
    ]


class ek_result(C.Structure):
    _fields_ = [
        ("n_windows", C.c_int64),
        ("win_start", C.POINTER(C.c_int64)),
        ("win_end", C.POINTER(C.c_int64)),
        ("win_row_offset", C.POINTER(C.c_int64)),
        ("win_row_count", C.POINTER(C.c_int64)),
        ("win_status", C.POINTER(C.c_int32)),
        ("win_member_count", C.POINTER(C.c_int64)),
        ("win_member_hash", C.POINTER(C.c_uint64)),
        ("n_rows", C.c_int64),
        ("key", C.POINTER(C.c_uint32)),
        ("agg_value", C.POINTER(C.c_int64) * EK_MAX_AGGS),
        ("agg_tag", C.POINTER(C.c_uint8) * EK_MAX_AGGS),
        ("n_aggs", C.c_int32),
        ("memory", C.c_int32),
        ("_owner", C.c_void_p),
    ]


class ek_stats(C.Structure):
    _fields_ = [
        ("records_in", C.c_int64),
        ("records_late", C.c_int64),
        ("windows_out", C.c_int64),
        ("rows_out", C.c_int64),
        ("last_batch_device_ms", C.c_double),
        ("phase_ms", C.c_double * 4),
        ("phase_launches", C.c_int64 * 4),
        ("records_filter_error", C.c_int64),
        ("records_discarded", C.c_int64),
        ("windows_keymajor", C.c_int64),
        ("device_ms_total", C.c_double),
        ("phase_ms_total", C.c_double * 4),
        ("phase_launches_total", C.c_int64 * 4),
        ("pushes_timed", C.c_int64),
        ("fused_batches", C.c_int64),
        ("fused_discarded", C.c_int64),
    ]


EK_PHASE_STATS, EK_PHASE_PARTITION, EK_PHASE_AGGREGATE, EK_PHASE_FINALIZE = 0, 1, 2, 3


class ek_global_ctx(C.Structure):
    """Global context of one shard's micro-batch (ekgpu.h, ek_push_batch_global)."""
    _fields_ = [
        ("row_arrival", C.c_void_p),
        ("arrivals_end", C.c_int64),
        ("wm_arrival", C.c_void_p),
        ("wm_ts", C.c_void_p),
        ("n_wm", C.c_int64),
        ("origin_known", C.c_int32),
        ("all_accepted", C.c_int32),
        ("max_wm_step", C.c_int64),
        ("origin_ts", C.c_int64),
        ("origin_arrival", C.c_int64),
        ("trig_arrival", C.c_void_p),
        ("trig_ts", C.c_void_p),
        ("n_trig", C.c_int64),
        ("memory", C.c_int32),
        ("pad2", C.c_int32),
        ("sess_start", C.c_void_p),
        ("sess_end", C.c_void_p),
        ("sess_wm", C.c_void_p),
        ("n_sess", C.c_int64),
    ]


def mix64(x: int) -> int:
    """ek_mix64 from the header (splitmix64 finaliser), on python ints."""
    m = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & m
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & m
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & m
    return x ^ (x >> 31)


# columnar JSON ingest (ek_json_*)
EK_JSON_MAX_NAME = 32
EK_JSON_OK, EK_JSON_ERR_SYNTAX, EK_JSON_ERR_TYPE, EK_JSON_ERR_NUMBER, EK_JSON_ERR_UNSUPPORTED = range(5)
EK_JSON_STR_ESCAPED = 0x40000000


class ek_json_schema(C.Structure):
    _fields_ = [("n_fields", C.c_int32), ("column_type", C.c_int32 * EK_MAX_COLUMNS),
                ("names", (C.c_char * EK_JSON_MAX_NAME) * EK_MAX_COLUMNS),
                ("elem_type", C.c_int32 * EK_MAX_COLUMNS), ("paths", C.c_int32)]


class ek_json_stats(C.Structure):
    _fields_ = [("messages", C.c_int64), ("errors", C.c_int64), ("bytes", C.c_int64)]
