"""Pipelined passes of a session (kvapi.cpp DevSession::run): pass i + 1's tables (match tables,
factor tables, tuple words, value-predicate table) and count buffers are double-buffered and built
on a low-priority stream beside pass i's rule kernels; after an even number of passes the count
set 1 becomes set 0. Every pass must produce what one pass produces: the counts of K = 1, 2, 3
passes, per-scope counts, and the statuses / failing paths fetched after several passes equal a
single kv_validate and the oracle (reference: pkg/engine/validation.go:26-106, one evaluation per
(policy, resource) whatever came before it)."""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _c2(n):
    from kyverno_amd import batch, workloads

    ps = batch.PolicySet(workloads.c2_policies(), specialize=True)
    data = batch.synth(workloads.SEED + 21, n, 0)
    return ps, batch.Batch(ps, data), data


def test_counts_equal_for_any_pass_count():
    from kyverno_amd import batch

    ps, b, _ = _c2(5000)
    ref = batch.validate(ps, b, mode=batch.MODE_COUNTS)
    s = batch.Session(ps, b, mode=batch.MODE_COUNTS)
    for k in (1, 2, 3, 2, 1):
        s.run(k)
        assert np.array_equal(s.counts(), ref.counts), f"counts after run({k})"


def test_fetch_after_pipelined_passes_matches_oracle():
    import oracle
    from kyverno_amd import batch, workloads

    ps, b, data = _c2(2000)
    s = batch.Session(ps, b, mode=batch.MODE_STATUS | batch.MODE_ERRORS)
    s.run(4)  # the fetch runs its own pass after four pipelined ones
    r = s.fetch()
    one = batch.validate(ps, b)
    assert np.array_equal(r.status, one.status)
    assert np.array_equal(s.counts(), one.counts)
    ress = [json.loads(x) for x in data.decode().strip().split("\n")]
    ost, _ = oracle.get().validate_batch(json.dumps(workloads.c2_policies()), json.dumps(ress), nthreads=8)
    ost[ost == 7] = 6
    assert np.array_equal(r.status, ost)
    fails = np.argwhere(r.status == 1)
    for rule, res in fails[:: max(1, len(fails) // 200)]:
        assert r.path(int(rule), int(res)) == one.path(int(rule), int(res))


@pytest.mark.parametrize("k", [1, 2, 3])
def test_scope_counts_equal_for_any_pass_count(k):
    from kyverno_amd import batch, workloads

    ps = batch.PolicySet(workloads.c5_policies(), specialize=True)
    b = batch.Batch(ps, batch.synth(workloads.SEED + 22, 4000, 1))
    mode = batch.MODE_COUNTS | batch.MODE_SCOPES
    ref = batch.validate(ps, b, mode=mode)
    s = batch.Session(ps, b, mode=mode)
    s.run(k)
    assert np.array_equal(s.counts(), ref.counts)
    assert np.array_equal(s.scope_counts(len(b.namespaces)), ref.scope_counts)
