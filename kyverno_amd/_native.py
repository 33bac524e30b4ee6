"""ctypes binding of libkvgpu.so (include/kvgpu.h).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C
kyverno_amd/csrc``). There is no fallback: if the shared library is missing or
fails to load, every entry point raises ``NativeUnavailable``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# KVGPU_LIB: alternative in-tree build of the same library (A/B kernel experiments)
LIB_PATH = os.environ.get("KVGPU_LIB") or os.path.join(_HERE, "libkvgpu.so")


class NativeUnavailable(RuntimeError):
    pass


class KvError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"kvgpu error {code}: {message}")
        self.code = code


class _KvErrorStruct(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int), ("message", ctypes.c_char_p)]


class RuleInfo(ctypes.Structure):
    _fields_ = [
        ("policy", ctypes.c_uint32),
        ("policy_name", ctypes.c_char_p),
        ("name", ctypes.c_char_p),
        ("route", ctypes.c_uint32),
        ("route_reason", ctypes.c_char_p),
        ("message", ctypes.c_char_p),
        ("any_pattern", ctypes.c_uint32),
        ("const_status", ctypes.c_uint32),
        ("const_message", ctypes.c_char_p),
    ]


_lib = None
_lock = threading.Lock()


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C kyverno_amd/csrc)")
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - loader failure
            raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        vp, sz, u32, u64, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        errpp = ctypes.POINTER(ctypes.POINTER(_KvErrorStruct))
        L.kv_compile.argtypes = [ctypes.c_char_p, sz, u32, ctypes.POINTER(vp), errpp]
        L.kv_policyset_info.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32)]
        L.kv_policyset_jit_info.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64)]
        L.kv_rule_info_get.argtypes = [vp, u32, ctypes.POINTER(RuleInfo)]
        L.kv_ingest.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_char_p, ctypes.POINTER(vp), errpp]
        L.kv_batch_info.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.kv_batch_transfer_bytes.argtypes = [vp, ctypes.POINTER(u64)]
        L.kv_validate.argtypes = [vp, vp, ctypes.c_char_p, i32, u32, ctypes.POINTER(vp), errpp]
        L.kv_result_status.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.kv_result_counts.argtypes = [vp, ctypes.POINTER(vp)]
        L.kv_result_phase.argtypes = [vp, u32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double)]
        L.kv_host_reserve.argtypes = [u64]
        L.kv_device_pool_limit.argtypes = [u64]
        L.kv_device_trim.argtypes = [i32]
        L.kv_result_path.argtypes = [vp, u32, u64, ctypes.c_char_p, sz]
        L.kv_result_error.argtypes = [vp, u32, u64, ctypes.POINTER(u32), ctypes.POINTER(u32)]
        L.kv_result_error_message.argtypes = [vp, u32, u64, ctypes.c_char_p, sz, ctypes.c_char_p, sz]
        L.kv_result_subst_error.argtypes = [vp, u32, u64, ctypes.c_char_p, sz]
        L.kv_result_kernel_ms.argtypes = [vp]
        L.kv_result_kernel_ms.restype = ctypes.c_double
        L.kv_bench.argtypes = [vp, vp, ctypes.c_char_p, i32, u32, i32, i32, ctypes.POINTER(ctypes.c_double), errpp]
        L.kv_synth.argtypes = [u64, u64, u32, ctypes.POINTER(vp), ctypes.POINTER(sz)]
        L.kv_synth_range.argtypes = [u64, u64, u64, u32, ctypes.POINTER(vp), ctypes.POINTER(sz)]
        L.kv_session_create.argtypes = [vp, vp, ctypes.c_char_p, i32, u32, ctypes.POINTER(vp), errpp]
        L.kv_session_run.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_double), errpp]
        L.kv_session_counts.argtypes = [vp, vp]
        L.kv_session_scope_counts.argtypes = [vp, vp]
        L.kv_result_scope_counts.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(u32)]
        L.kv_batch_namespaces.argtypes = [vp, ctypes.POINTER(u32)]
        L.kv_batch_namespace.argtypes = [vp, u32]
        L.kv_batch_namespace.restype = ctypes.c_char_p
        L.kv_validate_devices.argtypes = [vp, vp, ctypes.c_char_p, u32, u32, ctypes.POINTER(vp), errpp]
        L.kv_session_create_devices.argtypes = [vp, vp, ctypes.c_char_p, u32, u32, ctypes.POINTER(vp), errpp]
        L.kv_session_parts.argtypes = [vp, ctypes.POINTER(u32)]
        L.kv_session_fetch.argtypes = [vp, ctypes.POINTER(vp), errpp]
        L.kv_result_failures.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                         ctypes.POINTER(vp)]
        L.kv_path_string.argtypes = [vp, u32]
        L.kv_path_string.restype = ctypes.c_char_p
        L.kv_session_create_parts.argtypes = [vp, ctypes.c_char_p, u32, u32, ctypes.POINTER(vp), errpp]
        L.kv_session_attach_part.argtypes = [vp, u32, vp, i32, errpp]
        L.kv_session_scopes.argtypes = [vp, ctypes.POINTER(u32)]
        L.kv_session_scope_name.argtypes = [vp, u32]
        L.kv_session_scope_name.restype = ctypes.c_char_p
        L.kv_session_rccl_ranks.argtypes = [vp, ctypes.POINTER(i32)]
        L.kv_session_part_ms.argtypes = [vp, vp]
        L.kv_session_status_bytes.argtypes = [vp, ctypes.POINTER(u64)]
        for fn in ("kv_free_policyset", "kv_free_batch", "kv_free_result", "kv_free_buffer", "kv_free_session"):
            getattr(L, fn).argtypes = [vp]
            getattr(L, fn).restype = None
        L.kv_free_error.argtypes = [ctypes.POINTER(_KvErrorStruct)]
        L.kv_free_error.restype = None
        _lib = L
        return L


EXPORTED_SYMBOLS = [
    "kv_compile", "kv_policyset_info", "kv_policyset_jit_info", "kv_rule_info_get", "kv_ingest", "kv_batch_info", "kv_batch_transfer_bytes", "kv_validate",
    "kv_result_status", "kv_result_counts", "kv_result_path", "kv_result_error", "kv_result_error_message",
    "kv_result_subst_error", "kv_result_phase", "kv_host_reserve", "kv_device_pool_limit", "kv_device_trim",
    "kv_result_kernel_ms",
    "kv_bench", "kv_synth", "kv_synth_range", "kv_free_policyset", "kv_free_batch", "kv_free_result", "kv_free_error",
    "kv_free_buffer", "kv_session_create", "kv_session_run", "kv_session_counts", "kv_free_session",
    "kv_session_scope_counts", "kv_result_scope_counts", "kv_batch_namespaces", "kv_batch_namespace",
    "kv_validate_devices", "kv_session_create_devices", "kv_session_parts", "kv_session_fetch", "kv_result_failures",
    "kv_path_string", "kv_session_create_parts", "kv_session_attach_part", "kv_session_scopes", "kv_session_scope_name",
    "kv_session_rccl_ranks", "kv_session_part_ms", "kv_session_status_bytes",
]


def check(rc: int, err) -> None:
    if rc == 0:
        return
    msg = "unknown error"
    if err and err.contents.message:
        msg = err.contents.message.decode("utf-8", "replace")
        lib().kv_free_error(err)
    raise KvError(rc, msg)


def new_err():
    return ctypes.POINTER(_KvErrorStruct)()
