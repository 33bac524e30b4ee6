"""ORACLE — test infrastructure only.

CPU restatement of the reference's validate.pattern path (isabella232/kyverno
v1.5.x, `pkg/engine/validation.go`, `pkg/engine/validate/*`, `pkg/engine/anchor/*`,
`pkg/engine/utils.go`), compiled from `oracle/src/*.cpp` into
`oracle/build/liboracle.so`.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import this package, and only as the checker. The product (`kyverno_amd/`) never
imports, links or executes anything from here.

Parity pinning: there is no Go toolchain in this image and the reference cannot be
built, so the oracle is pinned by the reference's own known-answer
tests transcribed into `tests/golden/*.json` (see `tests/golden/gen_fixtures.py`).
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

STATUS = {"pass": 0, "fail": 1, "warn": 2, "error": 3, "skip": 4, "nomatch": 5, "cpu": 6, "panic": 7}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class Oracle:
    def __init__(self, path: str | None = None):
        path = path or _LIB_PATH
        if not os.path.exists(path):
            build()
        self.lib = ctypes.CDLL(path)
        L = self.lib
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_glob.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_glob.restype = ctypes.c_int
        L.orc_quantity.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
        L.orc_quantity_cmp.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        for fn in ("orc_operator", "orc_number_parts"):
            getattr(L, fn).argtypes = [ctypes.c_char_p]
            getattr(L, fn).restype = ctypes.c_void_p
        L.orc_anchor_pred.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_remove_anchors_from_path.argtypes = [ctypes.c_char_p]
        L.orc_remove_anchors_from_path.restype = ctypes.c_void_p
        L.orc_format.argtypes = [ctypes.c_char_p, ctypes.c_double]
        L.orc_format.restype = ctypes.c_void_p
        L.orc_compare.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                  ctypes.c_char_p]
        L.orc_match_pattern.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.orc_match_pattern.restype = ctypes.c_void_p
        L.orc_substitute.argtypes = [ctypes.c_char_p]
        L.orc_expand_in_metadata.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_expand_in_metadata.restype = ctypes.c_void_p
        L.orc_substitute.restype = ctypes.c_void_p
        L.orc_validate.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.orc_substitute_message.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_substitute_vars.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_enumerate.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        L.orc_enumerate.restype = ctypes.c_void_p
        L.orc_substitute_vars.restype = ctypes.c_void_p
        L.orc_substitute_message.restype = ctypes.c_void_p
        L.orc_validate.restype = ctypes.c_void_p
        L.orc_last_error.restype = ctypes.c_char_p
        L.orc_validate_batch.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong),
                                         ctypes.POINTER(ctypes.c_longlong)]
        L.orc_validate_batch.restype = ctypes.c_double
        L.orc_count_rules.argtypes = [ctypes.c_char_p]
        L.orc_count_rules.restype = ctypes.c_longlong
        L.orc_validate_ndjson.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.orc_validate_ndjson.restype = ctypes.c_double

    def _take(self, p) -> str:
        if not p:
            raise RuntimeError("oracle error: " + self.lib.orc_last_error().decode())
        s = ctypes.cast(p, ctypes.c_char_p).value.decode("utf-8")
        self.lib.orc_free(p)
        return s

    # --- primitives
    def glob(self, pattern: str, name: str) -> bool:
        return bool(self.lib.orc_glob(pattern.encode(), name.encode()))

    def quantity(self, s: str):
        out = ctypes.c_void_p()
        if not self.lib.orc_quantity(s.encode(), ctypes.byref(out)):
            return None
        return self._take(out.value)

    def quantity_cmp(self, a: str, b: str) -> int:
        return self.lib.orc_quantity_cmp(a.encode(), b.encode())

    def operator(self, pattern: str) -> str:
        return self._take(self.lib.orc_operator(pattern.encode()))

    def number_parts(self, pattern: str):
        return tuple(json.loads(self._take(self.lib.orc_number_parts(pattern.encode()))))

    def anchor_pred(self, fn: str, key: str) -> bool:
        r = self.lib.orc_anchor_pred(fn.encode(), key.encode())
        if r < 0:
            raise ValueError(fn)
        return bool(r)

    def remove_anchors_from_path(self, p: str) -> str:
        return self._take(self.lib.orc_remove_anchors_from_path(p.encode()))

    def format(self, what: str, v: float) -> str:
        return self._take(self.lib.orc_format(what.encode(), v))

    def compare(self, kind: int, value_json: str, pattern: str, value_mode: int = 1, pattern_mode: int = 0,
                op: str = "") -> bool:
        r = self.lib.orc_compare(kind, value_json.encode(), value_mode, pattern.encode(), pattern_mode, op.encode())
        if r < 0:
            raise RuntimeError(self.lib.orc_last_error().decode())
        return bool(r)

    def match_pattern(self, resource_json: str, pattern_json: str, entry: int = 0, res_mode: int = 0,
                      subst: bool = False) -> dict:
        return json.loads(self._take(self.lib.orc_match_pattern(entry, resource_json.encode(), res_mode,
                                                                  pattern_json.encode(), int(subst))))

    def expand_in_metadata(self, pattern: dict, resource: dict) -> dict:
        """The pattern after ExpandInMetadata (wildcard label / annotation keys replaced by the
        resource keys they match, wildcards.go:69-161)."""
        p = self.lib.orc_expand_in_metadata(json.dumps(pattern).encode(), json.dumps(resource).encode())
        if not p:
            raise RuntimeError(self.lib.orc_last_error().decode())
        return json.loads(self._take(p))

    def substitute(self, pattern_json: str) -> dict:
        return json.loads(self._take(self.lib.orc_substitute(pattern_json.encode())))

    def substitute_vars(self, pattern: dict | list, resource: dict) -> dict:
        """SubstituteAll of a pattern document with request.object = resource:
        {"doc": ...} | {"error": message} | {"scope": False} (outside the device scope)."""
        return json.loads(self._take(self.lib.orc_substitute_vars(json.dumps(pattern).encode(),
                                                                  json.dumps(resource).encode())))

    def enumerate(self, policy: dict, resource: dict, ctx: dict | None = None, cap: int = 4096) -> list:
        """Enumerate mode: per rule, every (status, failing path) the reference can produce over the
        Go map iteration orders of validateMap / expandWildcards, with the number of evaluations and
        whether `cap` cut the search short."""
        out = self._take(self.lib.orc_enumerate(json.dumps(policy).encode(), json.dumps(resource).encode(),
                                                json.dumps(ctx or {}).encode(), cap))
        return json.loads(out)["rules"]

    def substitute_message(self, msg: str, resource: dict | str):
        """buildErrorMessage's message substitution; None where the reference panics."""
        r = resource if isinstance(resource, str) else json.dumps(resource)
        p = self.lib.orc_substitute_message(msg.encode(), r.encode())
        return None if not p else self._take(p)

    def validate(self, policy: dict | str, resource: dict | str, ctx: dict | None = None) -> dict:
        p = policy if isinstance(policy, str) else json.dumps(policy)
        r = resource if isinstance(resource, str) else json.dumps(resource)
        c = json.dumps(ctx or {})
        return json.loads(self._take(self.lib.orc_validate(p.encode(), r.encode(), c.encode())))

    def validate_batch(self, policies_json: str, resources_json: str, ctx: dict | None = None, nthreads: int = 1):
        """Returns (status uint8 array [n_rules, n_res], seconds)."""
        import numpy as np

        nr = ctypes.c_longlong()
        nn = ctypes.c_longlong()
        c = json.dumps(ctx or {}).encode()
        p = policies_json.encode()
        r = resources_json.encode()
        t = self.lib.orc_validate_batch(p, r, c, nthreads, None, ctypes.byref(nr), ctypes.byref(nn))
        if t < 0:
            raise RuntimeError(self.lib.orc_last_error().decode())
        out = np.full((nr.value, nn.value), 255, dtype=np.uint8)
        t = self.lib.orc_validate_batch(p, r, c, nthreads, out.ctypes.data, ctypes.byref(nr), ctypes.byref(nn))
        if t < 0:
            raise RuntimeError(self.lib.orc_last_error().decode())
        return out, t


    def validate_ndjson(self, policies_json: str, ndjson: bytes, ctx: dict | None = None, nthreads: int = 1,
                        preparse: bool = False):
        """Large batches: one resource per NDJSON line, parsed and evaluated on `nthreads` threads.
        preparse=False streams (bounded memory; seconds include parsing); preparse=True parses every
        line first and times the evaluation alone. Returns (status uint8 [n_rules, n_res], seconds)."""
        import numpy as np

        nr = self.lib.orc_count_rules(policies_json.encode())
        if nr < 0:
            raise RuntimeError(self.lib.orc_last_error().decode())
        n_res = sum(1 for line in ndjson.split(b"\n") if line)
        out = np.full((nr, n_res), 255, dtype=np.uint8)
        t = self.lib.orc_validate_ndjson(policies_json.encode(), ndjson, len(ndjson), json.dumps(ctx or {}).encode(),
                                         nthreads, out.ctypes.data, n_res, 1 if preparse else 0)
        if t < 0:
            raise RuntimeError(self.lib.orc_last_error().decode())
        return out, t


_INSTANCE: Oracle | None = None


def get() -> Oracle:
    global _INSTANCE
    if _INSTANCE is None:
        _INSTANCE = Oracle()
    return _INSTANCE
