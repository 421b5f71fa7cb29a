"""ctypes binding of libekgpu.so (the HIP engine) — the product path.

There is no CPU fallback: if the shared library or a GPU is missing, every call raises.
"""
import ctypes as C
import os
from typing import List, Optional, Sequence

import numpy as np

from . import abi as A
from .results import result_to_python

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EKGPU_LIB") or os.path.join(HERE, "libekgpu.so")   # EKGPU_LIB: tuning builds

_lib = None


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ekgpu error {code}: {msg}")
        self.code = code
        self.msg = msg


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EngineError(A.EK_ERR_DEVICE, f"{LIB_PATH} not built (run `make -C ekuiper-vioneta_amd`)")
        L = C.CDLL(LIB_PATH)
        L.ek_abi_version.restype = C.c_int
        L.ek_device_count.restype = C.c_int
        L.ek_create.argtypes = [C.POINTER(A.ek_plan), C.c_int, C.POINTER(C.c_void_p)]
        L.ek_create.restype = C.c_int
        L.ek_push_batch.argtypes = [C.c_void_p, C.POINTER(A.ek_batch)]
        L.ek_push_batch.restype = C.c_int
        L.ek_poll_results.argtypes = [C.c_void_p, C.c_int32, C.POINTER(A.ek_result)]
        L.ek_poll_results.restype = C.c_int
        L.ek_release_results.argtypes = [C.c_void_p, C.POINTER(A.ek_result)]
        L.ek_release_results.restype = C.c_int
        L.ek_window_error.argtypes = [C.c_void_p, C.c_int64, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
        L.ek_window_error.restype = C.c_int
        L.ek_batch_ts_stats.argtypes = [C.c_void_p, C.POINTER(A.ek_batch), C.POINTER(A.ek_ts_stats)]
        L.ek_batch_ts_stats.restype = C.c_int
        L.ek_reset.argtypes = [C.c_void_p]
        L.ek_reset.restype = C.c_int
        L.ek_sync.argtypes = [C.c_void_p]
        L.ek_sync.restype = C.c_int
        L.ek_set_stream.argtypes = [C.c_void_p, C.c_void_p]
        L.ek_set_stream.restype = C.c_int
        L.ek_set_async.argtypes = [C.c_void_p, C.c_int32]
        L.ek_set_async.restype = C.c_int
        L.ek_set_phase_timing.argtypes = [C.c_void_p, C.c_int32]
        L.ek_set_phase_timing.restype = C.c_int
        L.ek_get_stats.argtypes = [C.c_void_p, C.POINTER(A.ek_stats)]
        L.ek_get_stats.restype = C.c_int
        L.ek_last_error.argtypes = [C.c_void_p]
        L.ek_last_error.restype = C.c_char_p
        L.ek_destroy.argtypes = [C.c_void_p]
        L.ek_destroy.restype = C.c_int
        L.ek_push_batch_global.argtypes = [C.c_void_p, C.POINTER(A.ek_batch), C.POINTER(A.ek_global_ctx)]
        L.ek_push_batch_global.restype = C.c_int
        L.ek_advance_watermark.argtypes = [C.c_void_p, C.c_int64, C.c_int64]
        L.ek_advance_watermark.restype = C.c_int
        L.ek_advance_time.argtypes = [C.c_void_p, C.c_int64]
        L.ek_advance_time.restype = C.c_int
        L.ek_shard_triggers.argtypes = [C.c_void_p, C.POINTER(A.ek_batch), C.POINTER(A.ek_global_ctx), C.c_void_p,
                                        C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
        L.ek_shard_triggers.restype = C.c_int
        L.ek_json_create.argtypes = [C.POINTER(A.ek_json_schema), C.c_int, C.POINTER(C.c_void_p)]
        L.ek_json_create.restype = C.c_int
        L.ek_json_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int32,
                                     C.POINTER(A.ek_batch)]
        L.ek_json_decode.restype = C.c_int
        L.ek_json_errors.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
        L.ek_json_errors.restype = C.c_int
        L.ek_json_get_stats.argtypes = [C.c_void_p, C.POINTER(A.ek_json_stats)]
        L.ek_json_get_stats.restype = C.c_int
        L.ek_json_last_error.argtypes = [C.c_void_p]
        L.ek_json_last_error.restype = C.c_char_p
        L.ek_json_strings.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        L.ek_json_strings.restype = C.c_int
        L.ek_json_dict_size.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int64)]
        L.ek_json_dict_size.restype = C.c_int
        L.ek_json_dict_string.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
        L.ek_json_dict_string.restype = C.c_int
        L.ek_json_list.argtypes = [C.c_void_p, C.c_int] + [C.POINTER(C.c_void_p)] * 4
        L.ek_json_list.restype = C.c_int
        L.ek_json_rows.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
        L.ek_json_rows.restype = C.c_int
        L.ek_json_destroy.argtypes = [C.c_void_p]
        L.ek_json_destroy.restype = C.c_int
        L.ek_export_state.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
        L.ek_export_state.restype = C.c_int
        L.ek_import_state.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
        L.ek_import_state.restype = C.c_int
        if L.ek_abi_version() != A.EKGPU_ABI_VERSION:
            raise EngineError(A.EK_ERR_INVALID, "libekgpu.so ABI version mismatch")
        _lib = L
    return _lib


EXPORTED_SYMBOLS = ["ek_abi_version", "ek_device_count", "ek_create", "ek_push_batch", "ek_poll_results",
                    "ek_release_results", "ek_reset", "ek_sync", "ek_set_stream", "ek_get_stats", "ek_last_error",
                    "ek_destroy", "ek_json_create", "ek_json_decode", "ek_json_errors", "ek_json_get_stats",
                    "ek_json_last_error", "ek_json_destroy", "ek_export_state", "ek_import_state",
                    "ek_push_batch_global", "ek_advance_watermark", "ek_shard_triggers", "ek_advance_time",
                    "ek_window_error", "ek_batch_ts_stats", "ek_json_strings", "ek_json_dict_size", "ek_json_dict_string", "ek_set_async", "ek_set_phase_timing", "ek_route_partition",
                    "ek_json_list", "ek_json_rows"]

_NP = {A.EK_COL_I64: np.int64, A.EK_COL_F64: np.float64, A.EK_COL_U32: np.uint32, A.EK_COL_BOOL: np.int64}


class Engine:
    """One rule's window/aggregate node on one MI355X (see include/ekgpu.h)."""

    def __init__(self, plan: A.ek_plan, device: int = 0):
        L = lib()
        self.plan = plan
        self.h = C.c_void_p()
        rc = L.ek_create(C.byref(plan), device, C.byref(self.h))
        if rc != 0:
            raise EngineError(rc, L.ek_last_error(None).decode())
        self._keep = []

    def _check(self, rc):
        if rc != 0:
            raise EngineError(rc, lib().ek_last_error(self.h).decode())

    def push_host(self, columns: Sequence[np.ndarray], validity: Optional[Sequence[Optional[np.ndarray]]] = None):
        b = A.ek_batch()
        keep = []
        n = None
        for k in range(self.plan.n_columns):
            a = np.ascontiguousarray(columns[k], dtype=_NP[self.plan.column_type[k]])
            keep.append(a)
            n = len(a) if n is None else n
            b.columns[k] = a.ctypes.data
            if validity is not None and validity[k] is not None:
                v = np.ascontiguousarray(validity[k], dtype=np.uint8)
                keep.append(v)
                b.validity[k] = v.ctypes.data
        b.n_rows = n or 0
        b.memory = A.EK_MEM_HOST
        self._check(lib().ek_push_batch(self.h, C.byref(b)))

    @staticmethod
    def _device_batch(n_rows, col_ptrs, valid_ptrs=None, ts_stats=None):
        b = A.ek_batch()
        b.n_rows = n_rows
        b.memory = A.EK_MEM_DEVICE
        for k, p in enumerate(col_ptrs):
            b.columns[k] = p
        if valid_ptrs:
            for k, p in enumerate(valid_ptrs):
                if p:
                    b.validity[k] = p
        if ts_stats is not None:
            b.ts_stats = C.pointer(ts_stats)
        return b

    def push_device(self, n_rows: int, col_ptrs: Sequence[int], valid_ptrs: Optional[Sequence[int]] = None,
                    ts_stats: Optional[A.ek_ts_stats] = None):
        """ts_stats: the batch's shared timestamp statistics (batch_ts_stats), e.g. from another rule over the same
        source; the push then skips its own pass over the timestamp column."""
        b = self._device_batch(n_rows, col_ptrs, valid_ptrs, ts_stats)
        self._check(lib().ek_push_batch(self.h, C.byref(b)))

    def batch_ts_stats(self, n_rows: int, col_ptrs: Sequence[int]) -> A.ek_ts_stats:
        """ek_batch_ts_stats over a device batch: computed once, handed to every rule that pushes the batch."""
        b = self._device_batch(n_rows, col_ptrs)
        out = A.ek_ts_stats()
        self._check(lib().ek_batch_ts_stats(self.h, C.byref(b), C.byref(out)))
        return out

    def push_batch(self, batch: A.ek_batch):
        """Push an ek_batch as is (e.g. the device columns returned by JsonDecoder.decode)."""
        self._check(lib().ek_push_batch(self.h, C.byref(batch)))

    def _host_batch(self, columns, validity=None):
        cols = [np.ascontiguousarray(columns[k], dtype=_NP[self.plan.column_type[k]]) for k in range(self.plan.n_columns)]
        b = A.ek_batch()
        b.n_rows = len(cols[0]) if cols else 0
        b.memory = A.EK_MEM_HOST
        keep = list(cols)
        for k, c in enumerate(cols):
            b.columns[k] = c.ctypes.data
            if validity is not None and validity[k] is not None:
                v = np.ascontiguousarray(validity[k], dtype=np.uint8)
                keep.append(v)
                b.validity[k] = v.ctypes.data
        return b, keep

    def push_global(self, columns, ctx: A.ek_global_ctx, validity=None):
        """Shard mode (ek_push_batch_global): this handle's rows (host arrays; None = no rows) + the global context."""
        if columns is None:
            self._check(lib().ek_push_batch_global(self.h, None, C.byref(ctx)))
            return
        b, _keep = self._host_batch(columns, validity)
        self._check(lib().ek_push_batch_global(self.h, C.byref(b), C.byref(ctx)))

    def push_global_device(self, n_rows: int, col_ptrs, ctx: A.ek_global_ctx):
        b = A.ek_batch()
        b.n_rows = n_rows
        b.memory = A.EK_MEM_DEVICE
        for k, ptr in enumerate(col_ptrs):
            b.columns[k] = ptr
        self._check(lib().ek_push_batch_global(self.h, C.byref(b), C.byref(ctx)))

    def shard_triggers_device(self, n_rows: int, col_ptrs, ctx: A.ek_global_ctx):
        """ek_shard_triggers over a device batch: (global arrival, ts) of the accepted trigger rows."""
        b = A.ek_batch()
        b.n_rows = n_rows
        b.memory = A.EK_MEM_DEVICE
        for k, ptr in enumerate(col_ptrs):
            b.columns[k] = ptr
        cap = max(1, n_rows // 1000 + 1024)
        while True:
            oa = np.zeros(cap, np.int64)
            ot = np.zeros(cap, np.int64)
            cnt = C.c_int64(0)
            self._check(lib().ek_shard_triggers(self.h, C.byref(b), C.byref(ctx), oa.ctypes.data, ot.ctypes.data, cap,
                                                C.byref(cnt)))
            k = int(cnt.value)
            if k <= cap:
                return oa[:k], ot[:k]
            cap = k

    def advance_watermark(self, wm_ms: int, arrivals_end: int, sessions=None):
        """A global WatermarkTuple with no rows for this shard. sessions: the (start, end) pairs the router's session
        logic closed at it (SESSIONWINDOW shards, which ek_advance_watermark refuses): sent through
        ek_push_batch_global with an empty batch."""
        if sessions is None:
            self._check(lib().ek_advance_watermark(self.h, int(wm_ms), int(arrivals_end)))
            return
        a = np.array([max(0, int(arrivals_end) - 1)], np.int64)
        t = np.array([int(wm_ms)], np.int64)
        ss = np.array([s for s, _ in sessions] or [0], np.int64)
        se = np.array([e for _, e in sessions] or [0], np.int64)
        ctx = A.ek_global_ctx()
        ctx.arrivals_end = int(arrivals_end)
        ctx.wm_arrival = a.ctypes.data
        ctx.wm_ts = t.ctypes.data
        ctx.n_wm = 1
        ctx.sess_start = ss.ctypes.data
        ctx.sess_end = se.ctypes.data
        ctx.n_sess = len(sessions)
        ctx.memory = A.EK_MEM_HOST
        self.push_global(None, ctx)

    def advance_time(self, now_ms: int):
        """Processing-time windows: move the handle's clock to now_ms (the first call, before any row, is the rule's
        start); every window the clock closes becomes pollable."""
        self._check(lib().ek_advance_time(self.h, int(now_ms)))

    def shard_triggers(self, columns, ctx: A.ek_global_ctx, validity=None):
        """(global arrival, ts) of this handle's accepted trigger rows of the batch (ek_shard_triggers)."""
        b, _keep = self._host_batch(columns, validity)
        n = int(b.n_rows)
        oa = np.zeros(max(n, 1), np.int64)
        ot = np.zeros(max(n, 1), np.int64)
        cnt = C.c_int64(0)
        self._check(lib().ek_shard_triggers(self.h, C.byref(b), C.byref(ctx), oa.ctypes.data, ot.ctypes.data, n, C.byref(cnt)))
        k = int(cnt.value)
        return oa[:k].copy(), ot[:k].copy()

    def poll(self):
        r = A.ek_result()
        self._check(lib().ek_poll_results(self.h, A.EK_MEM_HOST, C.byref(r)))
        try:
            out = result_to_python(r)
            for w, wr in enumerate(out):
                if wr.status != A.EK_WIN_OK:
                    wr.error = self.window_error(w)
            return out
        finally:
            self._check(lib().ek_release_results(self.h, C.byref(r)))

    def window_error(self, w: int) -> str:
        """The error text of window w of the last poll (ek_window_error): "run Where error: ..." etc., "" if none."""
        n = C.c_int64()
        self._check(lib().ek_window_error(self.h, w, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value + 1)
        self._check(lib().ek_window_error(self.h, w, buf, n.value + 1, C.byref(n)))
        return buf.value.decode()

    def poll_device(self) -> A.ek_result:
        r = A.ek_result()
        self._check(lib().ek_poll_results(self.h, A.EK_MEM_DEVICE, C.byref(r)))
        return r

    def release(self, r: Optional[A.ek_result] = None):
        self._check(lib().ek_release_results(self.h, C.byref(r) if r is not None else None))

    def reset(self):
        self._check(lib().ek_reset(self.h))

    def sync(self):
        self._check(lib().ek_sync(self.h))

    def set_stream(self, stream_ptr: int):
        self._check(lib().ek_set_stream(self.h, stream_ptr))

    def set_async(self, on: bool = True):
        """Pushes return with their work queued (ek_set_async): a device batch stays borrowed until the next push,
        sync, poll or stats call."""
        self._check(lib().ek_set_async(self.h, 1 if on else 0))

    def set_phase_timing(self, on: bool = True):
        """Per-phase HIP-event timing of the pushes (ek_set_phase_timing; on by default)."""
        self._check(lib().ek_set_phase_timing(self.h, 1 if on else 0))

    def stats(self) -> A.ek_stats:
        s = A.ek_stats()
        self._check(lib().ek_get_stats(self.h, C.byref(s)))
        return s

    def export_state(self) -> bytes:
        """Checkpoint of the stream state (results must have been polled): a host byte string."""
        n = C.c_int64()
        self._check(lib().ek_export_state(self.h, None, 0, C.byref(n)))
        buf = C.create_string_buffer(max(n.value, 1))
        self._check(lib().ek_export_state(self.h, buf, n.value, C.byref(n)))
        return buf.raw[: n.value]

    def import_state(self, blob: bytes):
        """Restore a checkpoint taken by export_state on a handle of the same plan (replaces the stream state)."""
        self._check(lib().ek_import_state(self.h, blob, len(blob)))

    def close(self):
        if self.h:
            lib().ek_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_to_host(ptr: int, n: int, dtype, device: int = 0) -> np.ndarray:
    """n elements of a device array the library handed out (its own HIP runtime allocated them): a view through the
    CUDA array interface, copied to the host by torch."""
    import torch

    class _View:
        __cuda_array_interface__ = {"shape": (int(n),), "typestr": np.dtype(dtype).str, "data": (int(ptr), False),
                                    "version": 2, "strides": None}

    return torch.as_tensor(_View(), device=torch.device("cuda", device)).cpu().numpy().copy()


class JsonDecoder:
    """Columnar JSON ingest on the GPU (include/ekgpu.h ek_json_*): a micro-batch of JSON messages ->
    device columns of an ek_batch, ready for Engine.push_batch."""

    @classmethod
    def schemaless(cls, fields, device: int = 0) -> "JsonDecoder":
        """A schemaless stream (CREATE STREAM demo () ...): FastJsonConverter without a schema decodes every JSON number
        as float64 (converter/json/converter.go:507-520, useInt64ForWholeNumber off), so each field the rule reads
        becomes a FLOAT column. A non-number value (the reference keeps it as a string / bool / map, which the rule's
        numeric expressions then reject) drops the message with EK_JSON_ERR_TYPE."""
        return cls({f: "float" for f in fields}, device)

    TYPES = {"bigint": A.EK_COL_I64, "float": A.EK_COL_F64, "key": A.EK_COL_U32, "string": A.EK_COL_STR,
             "boolean": A.EK_COL_BOOL}
    LIST_TYPES = {"array<bigint>": A.EK_COL_I64, "array<float>": A.EK_COL_F64, "array<boolean>": A.EK_COL_BOOL}

    def __init__(self, schema: dict, device: int = 0, paths: bool = False):
        """schema: ordered {field: "bigint" | "float" | "key" | "string" | "boolean" | "array<bigint|float|boolean>"}
        (same column order as the rule's schema). A "string" field reaches the engine as dense u32 ids of the
        decoder's dictionary (strings()); a "boolean" field as int64 0 / 1 (the rule's "boolean" column); an array
        field is read with lists(). paths=True: field names are paths into nested objects / arrays ("a.b", "a[0]",
        "a[0][0].c"; ABI v14)."""
        L = lib()
        s = A.ek_json_schema()
        s.n_fields = len(schema)
        s.paths = 1 if paths else 0
        self.names = list(schema)
        self.types = [A.EK_COL_LIST if t in self.LIST_TYPES else self.TYPES[t] for t in schema.values()]
        self.elems = [self.LIST_TYPES.get(t, 0) for t in schema.values()]
        self.device = device
        for k, (name, t) in enumerate(schema.items()):
            s.column_type[k] = self.types[k]
            s.elem_type[k] = self.elems[k]
            s.names[k].value = name.encode()
        self.h = C.c_void_p()
        rc = L.ek_json_create(C.byref(s), device, C.byref(self.h))
        if rc != 0:
            raise EngineError(rc, L.ek_json_last_error(None).decode())

    def decode(self, messages, offsets: Optional[np.ndarray] = None) -> A.ek_batch:
        """messages: list of bytes, or one bytes blob with offsets (n+1, int64). Returns the device batch."""
        if offsets is None:
            lens = np.fromiter((len(m) for m in messages), dtype=np.int64, count=len(messages))
            offsets = np.zeros(len(messages) + 1, dtype=np.int64)
            np.cumsum(lens, out=offsets[1:])
            blob = b"".join(messages)
        else:
            blob = messages
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        self._blob = np.frombuffer(blob, dtype=np.uint8) if len(blob) else np.zeros(1, np.uint8)
        out = A.ek_batch()
        rc = lib().ek_json_decode(self.h, self._blob.ctypes.data, len(blob), offsets.ctypes.data, len(offsets) - 1,
                                  A.EK_MEM_HOST, C.byref(out))
        if rc != 0:
            raise EngineError(rc, lib().ek_json_last_error(self.h).decode())
        return out

    def decode_device(self, blob_ptr: int, n_bytes: int, offsets_ptr: int, n_msgs: int) -> A.ek_batch:
        """Payloads already in device memory (blob bytes + n_msgs + 1 int64 offsets): no H2D copy."""
        out = A.ek_batch()
        rc = lib().ek_json_decode(self.h, C.c_void_p(blob_ptr), n_bytes, C.c_void_p(offsets_ptr), n_msgs,
                                  A.EK_MEM_DEVICE, C.byref(out))
        if rc != 0:
            raise EngineError(rc, lib().ek_json_last_error(self.h).decode())
        return out

    def errors(self):
        n = C.c_int64()
        lib().ek_json_errors(self.h, None, None, 0, C.byref(n))
        idx = np.zeros(max(n.value, 1), np.int64)
        code = np.zeros(max(n.value, 1), np.uint8)
        lib().ek_json_errors(self.h, idx.ctypes.data, code.ctypes.data, n.value, C.byref(n))
        return idx[: n.value], code[: n.value]

    def rule_schema(self) -> dict:
        """The schema a rule over this decoder's batches compiles with: a "string" field arrives as dictionary ids,
        i.e. a "key" column (GROUP BY it directly; strings() maps the ids back)."""
        return {n: ("key" if t == A.EK_COL_STR else {v: k for k, v in self.TYPES.items()}[t])
                for n, t in zip(self.names, self.types)}

    def rows_of(self) -> np.ndarray:
        """Rows of the last decode per message (a top-level array payload yields one row per object element; 0 for a
        message that failed)."""
        p, n = C.c_void_p(), C.c_int64()
        rc = lib().ek_json_rows(self.h, C.byref(p), C.byref(n))
        if rc != 0:
            raise EngineError(rc, lib().ek_json_last_error(self.h).decode())
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int64)), shape=(n.value,)).copy() if n.value else np.zeros(0, np.int64)

    def lists(self, column, batch) -> list:
        """The decoded arrays of LIST column `column` (index or field name) of the last decoded batch: one python
        list per row (None for a nil / absent array; None elements for nil items), elements typed by the column's
        element type (int, float, bool)."""
        c = self.names.index(column) if isinstance(column, str) else int(column)
        n_rows = int(batch.n_rows)
        ps = [C.c_void_p() for _ in range(4)]
        rc = lib().ek_json_list(self.h, c, *[C.byref(x) for x in ps])
        if rc != 0:
            raise EngineError(rc, lib().ek_json_last_error(self.h).decode())
        if n_rows == 0:
            return []
        start = device_to_host(ps[0].value, n_rows, np.int64, self.device)
        ln = device_to_host(ps[1].value, n_rows, np.int32, self.device)
        total = int((start + ln).max()) if n_rows else 0
        vals = device_to_host(ps[2].value, max(total, 1), np.int64, self.device)
        ok = device_to_host(ps[3].value, max(total, 1), np.uint8, self.device)
        et = self.elems[c]
        nil = (device_to_host(batch.validity[c], n_rows, np.uint8, self.device) == 0) if batch.validity[c] else \
            np.zeros(n_rows, bool)
        out = []
        for a, m, z in zip(start.tolist(), ln.tolist(), nil.tolist()):
            if z:
                out.append(None)
                continue
            row = []
            for k in range(a, a + m):
                if not ok[k]:
                    row.append(None)
                elif et == A.EK_COL_F64:
                    row.append(float(vals[k:k + 1].view(np.float64)[0]))
                elif et == A.EK_COL_BOOL:
                    row.append(bool(vals[k]))
                else:
                    row.append(int(vals[k]))
            out.append(row)
        return out

    def strings(self, column) -> list:
        """The dictionary of a string column (index or field name): id -> str, in id order."""
        c = self.names.index(column) if isinstance(column, str) else int(column)
        n = C.c_int64()
        rc = lib().ek_json_dict_size(self.h, c, C.byref(n))
        if rc != 0:
            raise EngineError(rc, lib().ek_json_last_error(self.h).decode())
        out = []
        p, ln = C.c_void_p(), C.c_int64()
        for i in range(n.value):
            lib().ek_json_dict_string(self.h, c, i, C.byref(p), C.byref(ln))
            out.append(C.string_at(p.value, ln.value).decode("utf-8", errors="surrogateescape") if ln.value else "")
        return out

    def stats(self) -> A.ek_json_stats:
        s = A.ek_json_stats()
        lib().ek_json_get_stats(self.h, C.byref(s))
        return s

    def close(self):
        if self.h:
            lib().ek_json_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
