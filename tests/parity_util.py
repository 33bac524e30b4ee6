"""Shared helpers: run the HIP path (C ABI) and the oracle on the same inputs and diff."""
from __future__ import annotations

import json
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(__file__), "golden")

# oracle status codes: pass fail warn error skip nomatch cpu panic(7)
# GPU: a would-panic shape is routed to the CPU engine (status 6)


def load_gold(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)["cases"]


def oracle_status(orc, policies, resources, ctx=None, nthreads=8):
    st, secs = orc.validate_batch(json.dumps(policies), json.dumps(resources), ctx=ctx, nthreads=nthreads)
    st = st.copy()
    st[st == 7] = 6
    return st


def gpu_run(policies, resources, ns_labels=None, admission=None, exclude_group_role=None, specialize=False):
    from kyverno_amd import batch

    ps = batch.PolicySet(policies, specialize=specialize)
    b = batch.Batch(ps, resources, namespace_labels=ns_labels)
    r = batch.validate(ps, b, admission=admission, exclude_group_role=exclude_group_role)
    return ps, b, r


def rule_index(policies):
    """(policy_idx, rule_idx_in_policy) for each flat rule index."""
    out = []
    for pi, p in enumerate(policies):
        for ri, _ in enumerate(p.get("spec", {}).get("rules", []) or []):
            out.append((pi, ri))
    return out


def compare(orc, policies, resources, ctx=None, check_paths=True, max_path_checks=400, specialize=False):
    """Returns list of mismatch descriptions (empty == parity). specialize: run the
    hiprtc-specialized kernels instead of the bytecode interpreter."""
    ps, b, r = gpu_run(policies, resources, admission=(ctx or {}).get("admission"),
                       exclude_group_role=(ctx or {}).get("excludeGroupRole"), specialize=specialize)
    ost = oracle_status(orc, policies, resources, ctx=ctx)
    gst = r.status
    mism = []
    assert gst.shape == ost.shape, (gst.shape, ost.shape)
    bad = np.argwhere(gst != ost)
    for rule, res in bad[:50]:
        mism.append(f"rule {rule} ({ps.rules[rule].name}) res {res}: gpu {gst[rule, res]} oracle {ost[rule, res]}")
    if check_paths:
        ridx = rule_index(policies)
        fails = np.argwhere((gst == 1) & (ost == 1))
        if len(fails) > max_path_checks:
            sel = np.random.default_rng(0).choice(len(fails), max_path_checks, replace=False)
            fails = fails[sel]
        for rule, res in fails:
            pi, ri = ridx[rule]
            ov = orc.validate(policies[pi], resources[res], ctx)
            opath = ov["rules"][ri]["path"]  # by position: rule names may repeat within a policy
            gpath = r.path(int(rule), int(res))
            if not ps.rules[rule].any_pattern and gpath != opath:
                mism.append(f"path rule {rule} ({ps.rules[rule].name}) res {res}: gpu {gpath!r} oracle {opath!r}")
    return mism, r, ost
