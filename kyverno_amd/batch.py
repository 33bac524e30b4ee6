"""Batch API over the C ABI: compile a policy set once, ingest resources once,
evaluate every (resource, rule) pair on a MI355X.

This is the batch form of ``engine.Validate`` (reference
``pkg/engine/validation.go:26``): statuses use ``response.RuleStatus`` codes
(``pkg/engine/response/status.go:14-28``) plus ``NOMATCH`` (no RuleResponse)
and ``CPU`` (the pair needs the reference CPU engine: context, preconditions,
deny, foreach or ``{{ }}`` variables).
"""
from __future__ import annotations

import ctypes
import json
from dataclasses import dataclass

import numpy as np

from . import _native
from ._native import RuleInfo, check, lib, new_err

PASS, FAIL, WARN, ERROR, SKIP, NOMATCH, CPU = range(7)
STATUS_NAMES = ["pass", "fail", "warn", "error", "skip", "nomatch", "cpu"]

MODE_STATUS, MODE_ERRORS, MODE_COUNTS, MODE_SCOPES = 1, 2, 4, 8
COMPILE_SPECIALIZE = 1
ROUTE_GPU, ROUTE_CPU, ROUTE_NORESPONSE, ROUTE_CONSTANT = range(4)


def _dumps(x) -> bytes:
    if isinstance(x, (bytes, bytearray)):
        return bytes(x)
    if isinstance(x, str):
        return x.encode("utf-8")
    return json.dumps(x, ensure_ascii=False, separators=(",", ":")).encode("utf-8")


@dataclass
class Rule:
    index: int
    policy: int
    policy_name: str
    name: str
    route: int
    route_reason: str
    message: str
    any_pattern: bool
    const_status: int
    const_message: str


class PolicySet:
    """Compiled policies (``kv_compile``). Input: list of policy dicts or JSON text.

    ``specialize=True`` also lowers every rule to specialized gfx950 kernels
    (hiprtc, at construction); evaluation then runs those instead of the
    bytecode interpreter. ``jit_info`` reports their build cost.
    """

    def __init__(self, policies, specialize: bool = False):
        L = lib()
        data = _dumps(policies)
        h = ctypes.c_void_p()
        err = new_err()
        flags = COMPILE_SPECIALIZE if specialize else 0
        check(L.kv_compile(data, len(data), flags, ctypes.byref(h), ctypes.byref(err)), err)
        self._h = h
        self.specialize = specialize
        np_, nr = ctypes.c_uint32(), ctypes.c_uint32()
        L.kv_policyset_info(h, ctypes.byref(np_), ctypes.byref(nr))
        self.n_policies, self.n_rules = np_.value, nr.value
        self.rules: list[Rule] = []
        for i in range(self.n_rules):
            ri = RuleInfo()
            L.kv_rule_info_get(h, i, ctypes.byref(ri))
            d = lambda b: (b or b"").decode("utf-8")  # noqa: E731
            self.rules.append(Rule(i, ri.policy, d(ri.policy_name), d(ri.name), ri.route, d(ri.route_reason),
                                   d(ri.message), bool(ri.any_pattern), ri.const_status, d(ri.const_message)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().kv_free_policyset(h)
            except Exception:
                pass
            self._h = None

    @property
    def jit_info(self) -> dict:
        nk, cb = ctypes.c_uint32(), ctypes.c_uint64()
        g, c = ctypes.c_double(), ctypes.c_double()
        lib().kv_policyset_jit_info(self._h, ctypes.byref(nk), ctypes.byref(g), ctypes.byref(c), ctypes.byref(cb))
        return {"kernels": nk.value, "gen_ms": g.value, "compile_ms": c.value, "code_bytes": cb.value}

    def policy_rules(self, policy: int) -> list[Rule]:
        return [r for r in self.rules if r.policy == policy]


class Batch:
    """Ingested resources (``kv_ingest``): list of dicts, JSON array text or NDJSON."""

    def __init__(self, policyset: PolicySet, resources, namespace_labels: dict | None = None):
        L = lib()
        if isinstance(resources, (list, tuple)):
            data = b"\n".join(_dumps(r) for r in resources)
        else:
            data = _dumps(resources)
        ns = _dumps(namespace_labels) if namespace_labels else None
        h = ctypes.c_void_p()
        err = new_err()
        check(L.kv_ingest(policyset._h, data, len(data), ns, ctypes.byref(h), ctypes.byref(err)), err)
        self._h = h
        self.policyset = policyset
        n, b = ctypes.c_uint64(), ctypes.c_uint64()
        L.kv_batch_info(h, ctypes.byref(n), ctypes.byref(b))
        self.n_res, self.store_bytes = n.value, b.value

    @property
    def transfer_bytes(self) -> int:
        """Bytes the store crosses PCIe in (kv_batch_transfer_bytes: 8-byte transfer cells)."""
        n = ctypes.c_uint64()
        lib().kv_batch_transfer_bytes(self._h, ctypes.byref(n))
        return n.value

    @property
    def namespaces(self) -> list[str]:
        """Batch namespace table: index = scope of per-scope counts ("" = cluster scope)."""
        n = ctypes.c_uint32()
        lib().kv_batch_namespaces(self._h, ctypes.byref(n))
        return [lib().kv_batch_namespace(self._h, i).decode("utf-8") for i in range(n.value)]

    def close(self) -> None:
        """Free the host batch now (e.g. once a parts session holds its device copy)."""
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().kv_free_batch(h)
            except Exception:
                pass
            self._h = None

    def __del__(self):
        self.close()


class _ResultHandle:
    """Owner of one kv_result handle: freed when the Result and every copy=False status view of
    its buffer are gone (the view's ctypes buffer holds a reference to this object)."""

    def __init__(self, h):
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                lib().kv_free_result(h)
            except Exception:
                pass
            self.h = None


class Result:
    """kv_result: statuses [rule][res] (a copy, or with copy=False a read-only view of the library's
    page-locked buffer; the view keeps the result's buffers alive), per-rule counts, failing
    paths / messages."""

    def __init__(self, h, policyset: PolicySet, batch: Batch, copy: bool = True):
        self._owner = _ResultHandle(h)
        self._h = h
        self.policyset = policyset
        self.batch = batch
        L = lib()
        nr, nn = ctypes.c_uint64(), ctypes.c_uint64()
        L.kv_result_status(h, None, ctypes.byref(nr), ctypes.byref(nn))
        self.n_rules, self.n_res = nr.value, nn.value
        self._copy = copy
        self._status = None
        self._status_read = False
        c = ctypes.c_void_p()
        L.kv_result_counts(h, ctypes.byref(c))
        cb = (ctypes.c_int64 * (self.n_rules * 8)).from_address(c.value) if self.n_rules else []
        self.counts = np.frombuffer(cb, dtype=np.int64).reshape(self.n_rules, 8).copy() if self.n_rules else \
            np.zeros((0, 8), np.int64)
        self.kernel_ms = L.kv_result_kernel_ms(h)
        # wall-clock phases of the kv_validate behind this result (upload, setup, pass, fetch steps)
        self.phases = {}
        nm, ms, i = ctypes.c_char_p(), ctypes.c_double(), 0
        while L.kv_result_phase(h, i, ctypes.byref(nm), ctypes.byref(ms)) == 0:
            key = nm.value.decode()
            self.phases[key] = self.phases.get(key, 0.0) + ms.value
            i += 1
        sc, ns = ctypes.c_void_p(), ctypes.c_uint32()
        self.scope_counts = None  # [scope][rule][8] with MODE_SCOPES
        if L.kv_result_scope_counts(h, ctypes.byref(sc), ctypes.byref(ns)) == 0 and self.n_rules and ns.value:
            buf = (ctypes.c_int64 * (ns.value * self.n_rules * 8)).from_address(sc.value)
            self.scope_counts = np.frombuffer(buf, dtype=np.int64).reshape(ns.value, self.n_rules, 8).copy()

    @property
    def status(self):
        """uint8 [rule][res] statuses in the caller's order, or None for a counts-only result. The
        library materialises the matrix on first use from the form the statuses crossed PCIe in
        (kv_result_status; the segments a specialized pass wrote, 4 bits a status)."""
        if not self._status_read:
            p = ctypes.c_void_p()
            if lib().kv_result_status(self._h, ctypes.byref(p), None, None) != 0:
                raise MemoryError("kv_result_status: no host memory for the status matrix")
            if p.value:
                buf = (ctypes.c_uint8 * (self.n_rules * self.n_res)).from_address(p.value)
                buf._kv_owner = self._owner  # the view outlives this Result only together with the handle
                st = np.frombuffer(buf, dtype=np.uint8).reshape(self.n_rules, self.n_res)
                if self._copy:
                    st = st.copy()
                else:
                    st.flags.writeable = False
                self._status = st
            self._status_read = True
        return self._status

    def path(self, rule: int, res: int) -> str | None:
        buf = ctypes.create_string_buffer(4096)
        n = lib().kv_result_path(self._h, rule, res, buf, 4096)
        if n < 0:
            return None
        return buf.value.decode("utf-8")

    def subst_error(self, rule: int, res: int) -> str | None:
        """The RuleResponse message of an ERROR pair caused by the pattern's variables failing to
        substitute ("variable substitution failed: ...", ``kv_result_subst_error``), else None."""
        cap = 1 << 12
        while True:
            buf = ctypes.create_string_buffer(cap)
            n = lib().kv_result_subst_error(self._h, rule, res, buf, cap)
            if n <= 0:
                return None
            if n < cap:
                return buf.raw[:n].decode("utf-8", "replace")
            cap = n + 1

    def error_message(self, rule: int, res: int, resource) -> str | None:
        """err.Error() of the pattern error behind a FAIL / ERROR / SKIP pair (``kv_result_error_message``):
        the SKIP message, and the operand of the ERROR message. ``resource`` is the ingested document
        (dict or JSON text), from which the Go '%v' operands are formatted."""
        doc = resource if isinstance(resource, (bytes, str)) else _dumps(resource)
        if isinstance(doc, str):
            doc = doc.encode("utf-8")
        cap = 1 << 16
        while True:
            buf = ctypes.create_string_buffer(cap)
            n = lib().kv_result_error_message(self._h, rule, res, doc, len(doc), buf, cap)
            if n < 0:
                return None
            if n < cap:
                return buf.raw[:n].decode("utf-8", "replace")
            cap = n + 1

    def failures(self):
        """Every FAIL / ERROR / SKIP pair (``kv_result_failures``), rule-major in resource order:
        (rule u32[n], res u64[n], path_id u32[n]) and ``paths`` (path_id -> string; FAIL only)."""
        n = ctypes.c_uint64()
        pr, pq, pp = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        rc = lib().kv_result_failures(self._h, ctypes.byref(n), ctypes.byref(pr), ctypes.byref(pq), ctypes.byref(pp))
        if rc != 0:
            raise _native.KvError(rc, "kv_result_failures failed")
        k = n.value
        if k == 0:
            return np.zeros(0, np.uint32), np.zeros(0, np.uint64), np.zeros(0, np.uint32), []
        rule = np.frombuffer((ctypes.c_uint32 * k).from_address(pr.value), np.uint32).copy()
        res = np.frombuffer((ctypes.c_uint64 * k).from_address(pq.value), np.uint64).copy()
        pid = np.frombuffer((ctypes.c_uint32 * k).from_address(pp.value), np.uint32).copy()
        paths = []
        while True:
            p = lib().kv_path_string(self._h, len(paths))
            if p is None:
                break
            paths.append(p.decode("utf-8"))
        return rule, res, pid, paths

    def error(self, rule: int, res: int):
        k, f = ctypes.c_uint32(), ctypes.c_uint32()
        if lib().kv_result_error(self._h, rule, res, ctypes.byref(k), ctypes.byref(f)) != 0:
            return None
        return k.value, f.value



def validate(policyset: PolicySet, batch: Batch, admission: dict | None = None,
             exclude_group_role: list | None = None, device: int = 0,
             mode: int = MODE_STATUS | MODE_ERRORS, device_mask: int | None = None, copy: bool = True) -> Result:
    """kv_validate on `device`, or kv_validate_devices over the devices of `device_mask`
    (contiguous resource shards, counts all-reduced over RCCL inside the library). copy=False: the
    status matrix is a view of the result's buffer (no host copy)."""
    ctx = {}
    if admission:
        ctx["admission"] = admission
    if exclude_group_role:
        ctx["excludeGroupRole"] = list(exclude_group_role)
    h = ctypes.c_void_p()
    err = new_err()
    if device_mask is None:
        rc = lib().kv_validate(policyset._h, batch._h, _dumps(ctx), device, mode, ctypes.byref(h), ctypes.byref(err))
    else:
        rc = lib().kv_validate_devices(policyset._h, batch._h, _dumps(ctx), device_mask, mode, ctypes.byref(h),
                                       ctypes.byref(err))
    check(rc, err)
    return Result(h, policyset, batch, copy=copy)


def bench(policyset: PolicySet, batch: Batch, device: int = 0, mode: int = MODE_COUNTS, warmup: int = 2,
          iters: int = 10, ctx: dict | None = None) -> float:
    ms = ctypes.c_double()
    err = new_err()
    check(lib().kv_bench(policyset._h, batch._h, _dumps(ctx or {}), device, mode, warmup, iters, ctypes.byref(ms),
                         ctypes.byref(err)), err)
    return ms.value


class Session:
    """Device-resident launch configuration: inputs and output buffers allocated once."""

    def __init__(self, policyset: PolicySet, batch: Batch | None, device: int = 0, mode: int = MODE_COUNTS,
                 ctx: dict | None = None, device_mask: int | None = None, parts: int = 0):
        h = ctypes.c_void_p()
        err = new_err()
        if parts:  # parts session: attach_part() uploads each part's own batch
            rc = lib().kv_session_create_parts(policyset._h, _dumps(ctx or {}), mode, parts, ctypes.byref(h),
                                               ctypes.byref(err))
        elif device_mask is None:
            rc = lib().kv_session_create(policyset._h, batch._h, _dumps(ctx or {}), device, mode, ctypes.byref(h),
                                         ctypes.byref(err))
        else:
            rc = lib().kv_session_create_devices(policyset._h, batch._h, _dumps(ctx or {}), device_mask, mode,
                                                 ctypes.byref(h), ctypes.byref(err))
        check(rc, err)
        self._h = h
        self.policyset, self.batch = policyset, batch
        self.n_rules = policyset.n_rules
        n = ctypes.c_uint32()
        lib().kv_session_parts(h, ctypes.byref(n))
        self.n_parts = n.value

    @classmethod
    def parts(cls, policyset: PolicySet, n_parts: int, mode: int = MODE_COUNTS, ctx: dict | None = None) -> "Session":
        """Multi-device session assembled from per-device batches (kv_session_create_parts): attach
        each part's batch with attach_part(); the batch may be dropped right after."""
        return cls(policyset, None, mode=mode, ctx=ctx, parts=n_parts)

    def attach_part(self, part: int, batch: Batch, device: int) -> None:
        err = new_err()
        check(lib().kv_session_attach_part(self._h, part, batch._h, device, ctypes.byref(err)), err)

    def scope_names(self) -> list[str]:
        """Scope table: the batch's namespaces, or the sorted union of the parts' namespaces."""
        n = ctypes.c_uint32()
        if lib().kv_session_scopes(self._h, ctypes.byref(n)) != 0:
            raise _native.KvError(-1, "kv_session_scopes failed (a part is not attached)")
        return [lib().kv_session_scope_name(self._h, i).decode() for i in range(n.value)]

    def rccl_ranks(self) -> int:
        """Ranks of the session's RCCL communicator (0: counts summed on the host)."""
        n = ctypes.c_int32()
        if lib().kv_session_rccl_ranks(self._h, ctypes.byref(n)) != 0:
            raise _native.KvError(-3, "kv_session_rccl_ranks failed")
        return n.value

    def status_bytes(self) -> int:
        """Status-matrix bytes the last run()'s pass wrote (unwritten segments are all NOMATCH)."""
        n = ctypes.c_uint64()
        if lib().kv_session_status_bytes(self._h, ctypes.byref(n)) != 0:
            raise _native.KvError(-3, "kv_session_status_bytes failed")
        return n.value

    def part_ms(self) -> list[float]:
        """HIP-event milliseconds of each part's last run()."""
        out = np.zeros(self.n_parts, dtype=np.float64)
        lib().kv_session_part_ms(self._h, out.ctypes.data)
        return out.tolist()

    def fetch(self) -> "Result":
        """The last pass as a result (statuses, compacted error records, reduced counts)."""
        h = ctypes.c_void_p()
        err = new_err()
        check(lib().kv_session_fetch(self._h, ctypes.byref(h), ctypes.byref(err)), err)
        return Result(h, self.policyset, self.batch)

    def run(self, iters: int) -> float:
        """Enqueue `iters` passes and wait; returns total HIP-event milliseconds."""
        ms = ctypes.c_double()
        err = new_err()
        check(lib().kv_session_run(self._h, iters, ctypes.byref(ms), ctypes.byref(err)), err)
        return ms.value

    def counts(self) -> np.ndarray:
        out = np.zeros((self.n_rules, 8), dtype=np.int64)
        rc = lib().kv_session_counts(self._h, out.ctypes.data)
        if rc != 0:
            raise _native.KvError(rc, "kv_session_counts failed")
        return out

    def scope_counts(self, n_scopes: int) -> np.ndarray:
        """[scope][rule][8] of the last pass (MODE_SCOPES)."""
        out = np.zeros((n_scopes, self.n_rules, 8), dtype=np.int64)
        rc = lib().kv_session_scope_counts(self._h, out.ctypes.data)
        if rc != 0:
            raise _native.KvError(rc, "kv_session_scope_counts failed")
        return out

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().kv_free_session(h)
            except Exception:
                pass
            self._h = None


def host_reserve(nbytes: int) -> bool:
    """Page-lock `nbytes` of host memory for the library's store and result arrays once, before the
    first batch (kv_host_reserve); False without a device."""
    return lib().kv_host_reserve(int(nbytes)) == 0


def synth(seed: int, n: int, kind_mix: int = 0, first: int = 0) -> bytes:
    """NDJSON of resources [first, first + n) of the synthetic stream `seed` (kv_synth_range)."""
    p = ctypes.c_void_p()
    ln = ctypes.c_size_t()
    rc = lib().kv_synth_range(seed, first, n, kind_mix, ctypes.byref(p), ctypes.byref(ln))
    if rc != 0:
        raise _native.KvError(rc, "kv_synth failed")
    # ctypes.string_at takes a C int size: copy buffers over 2 GiB in pieces
    step = 1 << 30
    data = b"".join(ctypes.string_at(p.value + o, min(step, ln.value - o)) for o in range(0, ln.value, step)) \
        if ln.value > step else ctypes.string_at(p.value, ln.value)
    lib().kv_free_buffer(p)
    return data
