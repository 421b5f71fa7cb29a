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
LIB_PATH = os.path.join(HERE, "libekgpu.so")

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
        L.ek_reset.argtypes = [C.c_void_p]
        L.ek_reset.restype = C.c_int
        L.ek_sync.argtypes = [C.c_void_p]
        L.ek_sync.restype = C.c_int
        L.ek_set_stream.argtypes = [C.c_void_p, C.c_void_p]
        L.ek_set_stream.restype = C.c_int
        L.ek_get_stats.argtypes = [C.c_void_p, C.POINTER(A.ek_stats)]
        L.ek_get_stats.restype = C.c_int
        L.ek_last_error.argtypes = [C.c_void_p]
        L.ek_last_error.restype = C.c_char_p
        L.ek_destroy.argtypes = [C.c_void_p]
        L.ek_destroy.restype = C.c_int
        if L.ek_abi_version() != A.EKGPU_ABI_VERSION:
            raise EngineError(A.EK_ERR_INVALID, "libekgpu.so ABI version mismatch")
        _lib = L
    return _lib


EXPORTED_SYMBOLS = ["ek_abi_version", "ek_device_count", "ek_create", "ek_push_batch", "ek_poll_results",
                    "ek_release_results", "ek_reset", "ek_sync", "ek_set_stream", "ek_get_stats", "ek_last_error",
                    "ek_destroy"]

_NP = {A.EK_COL_I64: np.int64, A.EK_COL_F64: np.float64, A.EK_COL_U32: np.uint32}


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

    def push_device(self, n_rows: int, col_ptrs: Sequence[int], valid_ptrs: Optional[Sequence[int]] = None):
        b = A.ek_batch()
        b.n_rows = n_rows
        b.memory = A.EK_MEM_DEVICE
        for k, p in enumerate(col_ptrs):
            b.columns[k] = p
        if valid_ptrs:
            for k, p in enumerate(valid_ptrs):
                if p:
                    b.validity[k] = p
        self._check(lib().ek_push_batch(self.h, C.byref(b)))

    def poll(self):
        r = A.ek_result()
        self._check(lib().ek_poll_results(self.h, A.EK_MEM_HOST, C.byref(r)))
        try:
            return result_to_python(r)
        finally:
            self._check(lib().ek_release_results(self.h, C.byref(r)))

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

    def stats(self) -> A.ek_stats:
        s = A.ek_stats()
        self._check(lib().ek_get_stats(self.h, C.byref(s)))
        return s

    def close(self):
        if self.h:
            lib().ek_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
