"""Parity at the sizes and rule sets the benchmark times (BASELINE.json configs).

Full status matrices of the specialized kernels (the engine bench.py times)
against the oracle run on every host core, plus sampled failing paths and
error messages:
* C3: the whole 1 000-policy / 1 973-rule set on mixed Pods/Deployments/Services,
  at the shipped kernel plan and at 40 rules per kernel;
* C2: 1 M Pods x 100 rules (the headline workload);
* C4: 1 M Pods x 142 anchor-heavy rules (incl. the SKIP / ERROR status forms).
Reference semantics: pkg/engine/validation.go:26-106 (oracle/src/engine.cpp).
"""
import json
import os

import numpy as np
import pytest

from parity_util import rule_index

pytestmark = pytest.mark.gpu


def _threads():
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except OSError:
        return os.cpu_count() or 1


def _check(orc, pols, data, env=None, n_paths=300, n_msgs=100, min_fail=100):
    from kyverno_amd import batch

    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        ps = batch.PolicySet(pols, specialize=True)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    b = batch.Batch(ps, data)
    r = batch.validate(ps, b)
    ost, _ = orc.validate_ndjson(json.dumps(pols), data, nthreads=_threads())
    ost[ost == 7] = 6
    bad = np.argwhere(r.status != ost)
    assert not len(bad), [(int(a), ps.rules[a].name, int(c), int(r.status[a, c]), int(ost[a, c])) for a, c in bad[:20]]
    assert (r.status == 1).sum() >= min_fail
    # sampled failing paths and skip / error messages against the per-pair oracle
    lines = data.split(b"\n")
    ridx = rule_index(pols)
    rng = np.random.default_rng(1)
    fails = np.argwhere(r.status == 1)
    for a, c in fails[rng.choice(len(fails), min(n_paths, len(fails)), replace=False)]:
        if ps.rules[a].any_pattern:
            continue
        pi, ri = ridx[a]
        want = orc.validate(pols[pi], lines[c].decode(), None)["rules"][ri]["path"]
        assert r.path(int(a), int(c)) == want, (ps.rules[a].name, int(c))
    errs = np.argwhere((r.status == 3) | (r.status == 4))
    for a, c in errs[rng.choice(len(errs), min(n_msgs, len(errs)), replace=False)] if len(errs) else []:
        pi, ri = ridx[a]
        want = orc.validate(pols[pi], lines[c].decode(), None)["rules"][ri]["message"]
        got = r.error_message(int(a), int(c), lines[c].decode())
        assert got is not None and got in want, (ps.rules[a].name, int(c), got, want)
    return r


@pytest.mark.parametrize("chunk", ["40", "128"])
def test_c3_full_policy_set(orc, chunk):
    """1 000 policies / 1 973 rules (match/exclude: kinds, namespace globs, wildcard matchLabels,
    matchExpressions, any-blocks, exclude blocks) x 2 000 mixed resources, at the shipped kernel
    plan (128 rules per fused kernel) and at 40."""
    from kyverno_amd import batch, workloads

    pols = workloads.c3_policies(1000)
    data = batch.synth(workloads.SEED + 11, 2000, workloads.C3_KIND_MIX).strip()
    r = _check(orc, pols, data, env={"KVGPU_JIT_CHUNK": chunk}, n_paths=200)
    assert r.n_rules == 1973 and (r.status == 5).sum() > 0


def test_c2_full_scale(orc):
    """C2 at its benchmark size: 1 M synthetic Pods x 100 rules (bench.py's default workload)."""
    from kyverno_amd import batch, workloads

    data = batch.synth(workloads.SEED, 1_000_000).strip()
    _check(orc, workloads.c2_policies(), data)


def test_c4_full_scale(orc):
    """C4 at its benchmark size: 1 M synthetic Pods x 142 anchor-heavy rules (chart +
    test/policy/validate + the status-form rules): every status incl. SKIP and ERROR at scale, their
    messages sampled against the per-pair oracle."""
    from kyverno_amd import batch, workloads

    data = batch.synth(workloads.SEED + 4, 1_000_000).strip()
    r = _check(orc, workloads.c4_policies(), data, n_msgs=300)
    assert (r.status == 3).sum() > 100_000 and (r.status == 4).sum() > 100_000


def test_name_filters_mixed_kinds(orc):
    """match / exclude `name` and `names` globs (per-resource match behind the tuple bit) on the
    mixed-kind C3 stream, next to rules the factored match decides (pkg/engine/utils.go:129-229)."""
    from kyverno_amd import batch, workloads
    pols = [workloads.name_filter_policy()] + workloads.c3_policies(40)
    data = batch.synth(workloads.SEED + 21, 4000, workloads.C3_KIND_MIX).strip()
    r = _check(orc, pols, data, min_fail=0)
    for q in range(5):
        assert 0 < (r.status[q] != 5).sum() < r.n_res  # each name rule matches some resources, not all


def test_c3_scope_counts_full_policy_set(orc):
    """C3 in SCOPES mode (per-namespace PolicyReport counts, pkg/kyverno/apply/report.go:80-87): the
    full 1 000-policy set over the C3 stream's 1 000 namespaces, device scope counts against the
    oracle's per-pair statuses grouped by namespace."""
    from kyverno_amd import batch, workloads

    pols = workloads.c3_policies(1000)
    data = batch.synth(workloads.SEED + 12, 2500, workloads.C3_KIND_MIX).strip()
    ps = batch.PolicySet(pols, specialize=True)
    b = batch.Batch(ps, data)
    res = batch.validate(ps, b, mode=batch.MODE_SCOPES)
    ost, _ = orc.validate_ndjson(json.dumps(pols), data, nthreads=_threads())
    ost[ost == 7] = 6
    nss = b.namespaces
    idx = {n: i for i, n in enumerate(nss)}
    want = np.zeros((len(nss), ost.shape[0], 8), np.int64)
    for j, line in enumerate(data.split(b"\n")):
        ns = json.loads(line)["metadata"].get("namespace", "")
        np.add.at(want[idx[ns]], (np.arange(ost.shape[0]), ost[:, j]), 1)
    assert len(nss) > 900  # the C3 stream spreads 2 500 resources over ~1 000 namespaces
    assert np.array_equal(res.scope_counts, want)


def _scope_want(ost, ns_index, n_scopes):
    """Per-(scope, rule, status) counts of the oracle's per-pair statuses, the resources grouped by
    scope (namespace index), summed with bincount over blocks of rules."""
    nr = ost.shape[0]
    want = np.zeros(n_scopes * nr * 8, np.int64)
    ns = ns_index.astype(np.int64)[None, :]
    for q0 in range(0, nr, 128):
        q1 = min(nr, q0 + 128)
        key = (ns * nr + np.arange(q0, q1, dtype=np.int64)[:, None]) * 8 + ost[q0:q1].astype(np.int64)
        want += np.bincount(key.ravel(), minlength=want.size)
    return want.reshape(n_scopes, nr, 8)


def _ns_index(data, nss):
    idx = {n: i for i, n in enumerate(nss)}
    return np.array([idx[json.loads(line)["metadata"].get("namespace", "")] for line in data.split(b"\n")],
                    np.int64)


def test_c3_bench_scale(orc):
    """C3 at bench scale: the 1 000-policy / 1 973-rule set x 100 000 mixed resources over the C3
    stream's 1 000 namespaces (about 100 resources per namespace, so the rule kernels' per-scope
    counts add whole waves of one scope): full status matrix and sampled failing paths against the
    oracle, then the per-namespace PolicyReport counts of SCOPES mode (the counts of
    pkg/kyverno/apply/report.go:80-87, pkg/policyreport/builder.go:245-261) against the oracle's
    statuses grouped by namespace."""
    from kyverno_amd import batch, workloads

    pols = workloads.c3_policies(1000)
    data = batch.synth(workloads.SEED + 31, 100_000, workloads.C3_KIND_MIX).strip()
    r = _check(orc, pols, data, n_paths=200, n_msgs=50)
    assert r.n_rules == 1973
    ps = batch.PolicySet(pols, specialize=True)
    b = batch.Batch(ps, data)
    nss = b.namespaces
    assert len(nss) >= 900 and 100_000 / len(nss) >= 50
    ost = r.status  # (equal to the oracle's, checked above)
    want = _scope_want(ost, _ns_index(data, nss), len(nss))
    res = batch.validate(ps, b, mode=batch.MODE_COUNTS | batch.MODE_SCOPES)
    assert np.array_equal(res.scope_counts, want)
    assert np.array_equal(res.counts[:, :7], want.sum(axis=0)[:, :7])


def test_c5_bench_scale(orc):
    """C5 at bench scale: the chart after autogen (105 rules) x 300 000 mixed Pods / Deployments /
    Services in SCOPES mode (the background-scan counts the bench times: no status matrix, per-scope
    counts inside the rule kernels) against the oracle's per-pair statuses grouped by namespace; the
    full status matrix of the same batch against the oracle."""
    from kyverno_amd import batch, workloads

    pols = workloads.c5_policies()
    data = batch.synth(workloads.SEED + 32, 300_000, kind_mix=1).strip()
    ps = batch.PolicySet(pols, specialize=True)
    b = batch.Batch(ps, data)
    ost, _ = orc.validate_ndjson(json.dumps(pols), data, nthreads=_threads())
    ost[ost == 7] = 6
    nss = b.namespaces
    want = _scope_want(ost, _ns_index(data, nss), len(nss))
    res = batch.validate(ps, b, mode=batch.MODE_COUNTS | batch.MODE_SCOPES)
    assert np.array_equal(res.scope_counts, want)
    sess = batch.Session(ps, b, mode=batch.MODE_COUNTS | batch.MODE_SCOPES)
    sess.run(3)  # (pipelined passes)
    assert np.array_equal(sess.scope_counts(len(nss)), want)
    st = batch.validate(ps, b, mode=batch.MODE_STATUS)
    bad = np.argwhere(st.status != ost)
    assert not len(bad), bad[:10]
    assert (ost == 1).sum() > 10_000 and (ost == 0).sum() > 10_000
