"""PolicyReport summaries from device counts, and their cross-rank reduction.

* ``scope_summaries`` turns per-scope device counts (``KV_MODE_SCOPES``:
  ``[scope][rule][8]``) into the summary of every PolicyReport /
  ClusterPolicyReport the CLI would build (``buildPolicyReports`` /
  ``calculateSummary``, pkg/kyverno/apply/report.go:23-179): scope
  ``policyreport-ns-<namespace>`` for namespaced resources,
  ``clusterpolicyreport`` for cluster-scoped ones; every rule of a policy with a
  validate rule contributes one result per resource, and a rule absent from the
  engine response (not matched, not a validate rule) is a ``skip``
  (``ProcessValidateEngineResponse``, pkg/kyverno/common/common.go:703-766).
* ``allreduce_counts`` sums count tensors over the ranks of a background scan
  sharded by resources (one process per GPU): a single all-reduce over RCCL
  (``nccl`` backend) or gloo on the CPU — the only collective of the path
  (SURVEY.md §8e).
"""
from __future__ import annotations

import numpy as np

PASS, FAIL, WARN, ERROR, SKIP, NOMATCH, CPU = range(7)
SUMMARY_KEYS = ("pass", "fail", "warn", "error", "skip")
ROUTE_NORESPONSE = 2


def scope_name(namespace: str) -> str:
    """buildPolicyResults scope key (pkg/kyverno/apply/report.go:80-87)."""
    return f"policyreport-ns-{namespace}" if namespace else "clusterpolicyreport"


def scope_summaries(rules, policies: list[dict], namespaces: list[str], scope_counts: np.ndarray) -> dict:
    """{scope: {"pass","fail","warn","error","skip","cpu"}} from counts[scope][rule][8].

    ``rules``: the compiled rule table (batch.Rule, policy order); ``policies``: the compiled
    (mutated) policy documents; ``namespaces``: the batch namespace table."""
    has_validate = [any((r.get("validate") or None) is not None and r.get("validate") != {}
                        for r in (p.get("spec") or {}).get("rules") or []) for p in policies]
    sel = np.array([has_validate[r.policy] for r in rules], dtype=bool)
    c = scope_counts[:, sel, :].sum(axis=1) if sel.any() else np.zeros((len(namespaces), 8), np.int64)
    out: dict[str, dict] = {}
    for s, ns in enumerate(namespaces):
        row = c[s]
        if row.sum() == 0:
            continue
        d = out.setdefault(scope_name(ns), {k: 0 for k in SUMMARY_KEYS + ("cpu",)})
        d["pass"] += int(row[PASS])
        d["fail"] += int(row[FAIL])
        d["warn"] += int(row[WARN])
        d["error"] += int(row[ERROR])
        d["skip"] += int(row[SKIP] + row[NOMATCH])
        d["cpu"] += int(row[CPU])
    return out


def allreduce_counts(counts: np.ndarray, dist=None) -> np.ndarray:
    """Sum an int64 count array over all ranks (torch.distributed, RCCL on GPUs / gloo on CPU)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return counts
    import torch

    t = torch.from_numpy(np.ascontiguousarray(counts, dtype=np.int64))
    if dist.get_backend() == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def allreduce_scope_counts(namespaces: list[str], scope_counts: np.ndarray, dist=None) -> tuple[list[str], np.ndarray]:
    """Per-scope counts of resource shards → node-wide counts. Every rank's batch numbers its
    namespaces in first-seen order, so the scope axis is first re-indexed onto the sorted union of
    all ranks' namespaces (one all_gather_object of the names), then summed with one all-reduce."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        order = sorted(range(len(namespaces)), key=lambda i: namespaces[i])
        return [namespaces[i] for i in order], scope_counts[order]
    names: list = [None] * dist.get_world_size()
    dist.all_gather_object(names, list(namespaces))
    universe = sorted(set().union(*names))
    pos = {n: i for i, n in enumerate(universe)}
    full = np.zeros((len(universe),) + scope_counts.shape[1:], np.int64)
    full[[pos[n] for n in namespaces]] = scope_counts
    return universe, allreduce_counts(full, dist)
