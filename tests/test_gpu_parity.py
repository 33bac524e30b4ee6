"""Parity of the HIP path (through the C ABI) with the oracle on the same inputs.

Bar: bit-exact per-(resource, rule) status and identical failing path.
Inputs: the reference's own fixtures (tests/golden), the reference YAML corpus
(test/best_practices, test/more, test/policy/validate x test/resources) and
seeded synthetic corpora of the benchmark configs.
"""
import json

import numpy as np
import pytest

from parity_util import compare, load_gold

pytestmark = pytest.mark.gpu

# every parity case runs on both device engines: the bytecode interpreter
# (kvkernel.hip) and the per-policy-set specialized kernels (kvjit.cpp)
engines = pytest.mark.parametrize("spec", [False, True], ids=["vm", "specialized"])


def _policy(pattern, name="fixture", any_pattern=False):
    v = {"anyPattern": pattern} if any_pattern else {"pattern": pattern}
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
            "spec": {"rules": [{"name": "r", "match": {"resources": {"kinds": ["*"]}}, "validate": v}]}}


@engines
def test_matcher_fixtures(orc, spec):
    """validate_test.go cases (map resources) wrapped as single-rule policies."""
    cases = [c for c in load_gold("matcher.json") if json.loads(c["resource"]).__class__ is dict]
    pols = [_policy(json.loads(c["pattern"]), name=f"m{i}") for i, c in enumerate(cases)]
    ress = [json.loads(c["resource"]) for c in cases]
    mism, r, ost = compare(orc, pols, ress, specialize=spec)
    # only the diagonal (policy i x resource i) is the fixture; the cross product is extra coverage
    assert not mism, "\n".join(mism)


@engines
def test_comparator_fixtures(orc, spec):
    """pattern_test.go ValidateValueWithPattern cases as {key: pattern} vs {key: value}."""
    cases = [c for c in load_gold("comparator.json") if c.get("kind") == 0]
    pols = [_policy({"key": json.loads(c["pattern"]["json"])}, name=f"c{i}") for i, c in enumerate(cases)]
    ress = [{"key": json.loads(c["value"]["json"])} for c in cases]
    mism, r, ost = compare(orc, pols, ress, specialize=spec)
    assert not mism, "\n".join(mism)


@engines
def test_reference_corpus(orc, spec):
    c = load_gold("corpus.json")[0]
    pols = [p["policy"] for p in c["policies"]]
    ress = [r["resource"] for r in c["resources"]]
    mism, r, ost = compare(orc, pols, ress, specialize=spec)
    assert not mism, "\n".join(mism)
    # the corpus must exercise the GPU path, not only CPU routes
    assert (r.status <= 4).sum() > 50


@engines
def test_c2_synthetic(orc, spec):
    from kyverno_amd import batch, workloads

    pols = workloads.c2_policies()
    data = batch.synth(workloads.SEED, 3000).decode()
    ress = [json.loads(l) for l in data.strip().split("\n")]
    mism, r, ost = compare(orc, pols, ress, specialize=spec)
    assert not mism, "\n".join(mism)
    assert (r.status == 1).sum() > 1000 and (r.status == 0).sum() > 1000


@engines
def test_c3_synthetic_match_exclude(orc, spec):
    from kyverno_amd import batch, workloads

    pols = workloads.c3_policies(60)
    data = batch.synth(workloads.SEED + 1, 1500, kind_mix=workloads.C3_KIND_MIX).decode()
    ress = [json.loads(l) for l in data.strip().split("\n")]
    mism, r, ost = compare(orc, pols, ress, check_paths=True, max_path_checks=200, specialize=spec)
    assert not mism, "\n".join(mism)
    assert (r.status == 5).sum() > 0 and (r.status <= 1).sum() > 0


@engines
def test_counts_mode_matches_status(orc, spec):
    from kyverno_amd import batch, workloads

    pols = workloads.c2_policies()
    ps = batch.PolicySet(pols, specialize=spec)
    b = batch.Batch(ps, batch.synth(workloads.SEED, 5000))
    full = batch.validate(ps, b)
    counts = batch.validate(ps, b, mode=batch.MODE_COUNTS)
    for s in range(7):
        assert np.array_equal((full.status == s).sum(axis=1), counts.counts[:, s])


@engines
def test_glob_stress(orc, spec):
    """Random globs (`*`, `?`, literal runs, `|`, `!`) x random ASCII values: exercises
    the compiled prefix/suffix/middle-segment search of the device glob."""
    import random

    rnd = random.Random(7)
    alpha = "ab:/.-"

    def word(n):
        return "".join(rnd.choice(alpha) for _ in range(n))

    pats = set()
    while len(pats) < 120:
        parts = []
        for _ in range(rnd.randrange(1, 5)):
            r = rnd.random()
            parts.append("*" if r < 0.35 else "?" if r < 0.45 else word(rnd.randrange(1, 4)))
        p = "".join(parts)
        if rnd.random() < 0.15:
            p = "!" + p
        if rnd.random() < 0.1:
            p = p + " | " + word(2) + "*"
        pats.add(p)
    vals = [word(rnd.randrange(0, 40)) for _ in range(400)]
    pols = [_policy({"key": p}, name=f"g{i}") for i, p in enumerate(sorted(pats))]
    ress = [{"key": v} for v in vals]
    mism, r, ost = compare(orc, pols, ress, specialize=spec)
    assert not mism, "\n".join(mism)
    assert (r.status == 0).sum() > 1000 and (r.status == 1).sum() > 1000


@engines
def test_c4_anchor_heavy_chart(orc, spec):
    """C4: chart (restricted) + test/policy/validate after autogen x synthetic Pods with pod- and
    container-level securityContext, host namespaces/ports/paths, sysctls, volumes, apparmor."""
    from kyverno_amd import batch, workloads

    pols = workloads.c4_policies()
    data = batch.synth(workloads.SEED + 4, 3000).decode()
    ress = [json.loads(l) for l in data.strip().split("\n")]
    mism, r, ost = compare(orc, pols, ress, check_paths=True, max_path_checks=600, specialize=spec)
    assert not mism, "\n".join(mism)
    for s in (0, 1, 5):  # pass, fail, not matched (autogen rules)
        assert (r.status == s).sum() > 100, s


@engines
def test_c5_background_scan_counts(orc, spec):
    """C5: full chart after autogen x Pods/Deployments/Services, COUNTS mode (PolicyReport
    summaries) against the oracle's per-pair statuses."""
    from kyverno_amd import batch, workloads

    pols = workloads.c5_policies()
    data = batch.synth(workloads.SEED + 5, 4000, kind_mix=1)
    ps = batch.PolicySet(pols, specialize=spec)
    b = batch.Batch(ps, data)
    counts = batch.validate(ps, b, mode=batch.MODE_COUNTS)
    ress = "[" + ",".join(data.decode().strip().split("\n")) + "]"
    ost, _ = orc.validate_batch(json.dumps(pols), ress, nthreads=8)
    ost[ost == 7] = 6
    for s in range(7):
        assert np.array_equal((ost == s).sum(axis=1), counts.counts[:, s]), s
    assert counts.counts[:, 0].sum() > 1000 and counts.counts[:, 1].sum() > 100


@engines
def test_c5_scope_counts(orc, spec):
    """Per-namespace PolicyReport counts (KV_MODE_SCOPES, scope-count kernel) against the oracle's
    per-pair statuses grouped by the resources' namespaces, plus cluster-scoped resources."""
    from kyverno_amd import batch, workloads

    pols = workloads.c5_policies()
    data = batch.synth(workloads.SEED + 6, 3000, kind_mix=1).decode().strip().split("\n")
    ress = [json.loads(l) for l in data]
    for r in ress[::50]:  # some cluster-scoped resources (empty namespace -> clusterpolicyreport)
        r["metadata"].pop("namespace", None)
    ps = batch.PolicySet(pols, specialize=spec)
    b = batch.Batch(ps, ress)
    res = batch.validate(ps, b, mode=batch.MODE_SCOPES)
    ost, _ = orc.validate_batch(json.dumps(pols), json.dumps(ress), nthreads=8)
    ost[ost == 7] = 6
    nss = b.namespaces
    idx = {n: i for i, n in enumerate(nss)}
    want = np.zeros((len(nss), ost.shape[0], 8), np.int64)
    for j, r in enumerate(ress):
        np.add.at(want[idx[r["metadata"].get("namespace", "")]], (np.arange(ost.shape[0]), ost[:, j]), 1)
    assert "" in idx and len(nss) > 60
    assert np.array_equal(res.scope_counts, want)
    sess = batch.Session(ps, b, mode=batch.MODE_SCOPES)
    sess.run(2)
    assert np.array_equal(sess.scope_counts(len(nss)), want)


def test_parallel_ingest_matches_serial():
    """Multi-threaded NDJSON ingest (per-thread wave groups merged with rebased offsets) gives the
    same statuses and failing paths as the serial ingest."""
    import os

    from kyverno_amd import batch, workloads

    pols = workloads.c2_policies() + workloads.c5_policies()
    ps = batch.PolicySet(pols, specialize=True)
    data = batch.synth(workloads.SEED + 7, 20000, kind_mix=1)
    out = {}
    for t in ("1", "16"):
        os.environ["KVGPU_INGEST_THREADS"] = t
        try:
            b = batch.Batch(ps, data)
        finally:
            os.environ.pop("KVGPU_INGEST_THREADS", None)
        r = batch.validate(ps, b)
        fails = np.argwhere(r.status == 1)[:300]
        out[t] = (r.status, b.namespaces, [r.path(int(a), int(c)) for a, c in fails])
    assert np.array_equal(out["1"][0], out["16"][0])
    assert out["1"][1] == out["16"][1] and out["1"][2] == out["16"][2]


@engines
def test_wide_error_records(orc, spec):
    """Failing paths whose loop indices overflow the compact 8 B error record (index >= 1024 at
    level 0, >= 256 at levels 1-2, a fourth loop level) or name a resolved wildcard label key:
    the pass is re-run writing full records (kvdevtypes.h ErrRec8); indices just below the limits
    stay compact."""
    def pod(n0, n1, bad0, bad1, labels):
        cs = [{"name": f"c{i}", "image": "nginx:1.0", "ports": [{"containerPort": 80}] * (n1 if i == bad0 else 1)}
              for i in range(n0)]
        cs[bad0]["ports"] = [dict(p) for p in cs[bad0]["ports"]]
        cs[bad0]["ports"][bad1]["containerPort"] = 81
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "labels": labels}, "spec": {"containers": cs}}

    def deep(k):  # four loop levels, the failing element at index 1 of each
        x = {"v": "bad" if k else "ok"}
        for _ in range(4):
            x = {"l": [{"v": "ok", "l": []}, x]}
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "d"}, "spec": x}

    ress = [pod(5000, 1, 4500, 0, {"app-x": "no"}), pod(3, 2000, 1, 1500, {"app-y": "web"}),
            pod(10, 3, 2, 1, {"tier": "x"}), deep(1), deep(0), pod(1100, 1, 1023, 0, {}), pod(1100, 1, 1024, 0, {}),
            pod(2, 300, 1, 255, {}), pod(2, 300, 1, 256, {})]
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "wide"},
           "spec": {"rules": [
               {"name": "port", "match": {"resources": {"kinds": ["Pod"]}},
                "validate": {"pattern": {"spec": {"containers": [{"ports": [{"containerPort": 80}]}]}}}},
               {"name": "label", "match": {"resources": {"kinds": ["Pod"]}},
                "validate": {"pattern": {"metadata": {"labels": {"app-*": "web"}}}}},
               {"name": "deep", "match": {"resources": {"kinds": ["Pod"]}},
                "validate": {"pattern": {"spec": {"l": [{"l": [{"l": [{"l": [{"v": "ok"}]}]}]}]}}}}]}}
    mism, r, ost = compare(orc, [pol], ress, check_paths=True, specialize=spec)
    assert not mism, "\n".join(mism)
    assert r.path(0, 0) == "/spec/containers/4500/ports/0/containerPort/"
    assert r.path(0, 1) == "/spec/containers/1/ports/1500/containerPort/"
    assert r.path(1, 0) == "/metadata/labels/app-x/"
    assert r.path(2, 3) == "/spec/l/1/l/1/l/1/l/1/v/"
    assert r.path(0, 5) == "/spec/containers/1023/ports/0/containerPort/"
    assert r.path(0, 6) == "/spec/containers/1024/ports/0/containerPort/"
    assert r.path(0, 7) == "/spec/containers/1/ports/255/containerPort/"
    assert r.path(0, 8) == "/spec/containers/1/ports/256/containerPort/"


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [False, True], ids=["vm", "specialized"])
def test_glob_stress_long_values(orc, spec):
    """The glob stress at value lengths 0-200 (kvj_ptab's 64-byte and 128-byte register
    paths and the word-loop fallback beyond) with non-ASCII values under `?` globs."""
    import random

    rnd = random.Random(11)
    alpha = list("ab:/.-") + ["é", "日"]

    def word(n):
        s = ""
        while len(s.encode()) < n:
            s += rnd.choice(alpha)
        return s

    pats = set()
    while len(pats) < 120:
        parts = []
        for _ in range(rnd.randrange(1, 6)):
            r = rnd.random()
            parts.append("*" if r < 0.35 else "?" if r < 0.45 else word(rnd.randrange(1, 5)))
        p = "".join(parts)
        if rnd.random() < 0.15:
            p = "!" + p
        pats.add(p)
    vals = [word(rnd.choice([rnd.randrange(0, 30), rnd.randrange(50, 80), rnd.randrange(100, 140),
                             rnd.randrange(120, 200)])) for _ in range(600)]
    pols = [_policy({"key": p}, name=f"g{i}") for i, p in enumerate(sorted(pats))]
    ress = [{"key": v} for v in vals]
    mism, r, ost = compare(orc, pols, ress, specialize=spec)
    assert not mism, "\n".join(mism)
    assert (r.status == 0).sum() > 1000 and (r.status == 1).sum() > 1000


@engines
def test_group_site_records(orc, spec):
    """Rule groups (rules of one form differing only in constants, run once with a bit per member)
    write one site record per lane and error site for every member ending there, expanded to the
    members' records at fetch (kvdevtypes.h GSiteDesc): members failing at different leaves and at
    different loop indices on one resource, a group of 40 members (two groups of at most 32), loop
    indices that overflow the compact record (the full-record re-run) and ERROR statuses."""
    import random

    rnd = random.Random(11)
    regs = [f"reg{k}.io" for k in range(40)]
    rules = [{"name": f"img-{k}", "match": {"resources": {"kinds": ["Pod"]}},
              "validate": {"pattern": {"spec": {"containers": [{"image": f"{regs[k]}/*", "name": f"c{k % 7}*"}]}}}}
             for k in range(40)]
    # an array where a map is expected: the representative's structural check fails for every member
    rules += [{"name": f"lim-{k}", "match": {"resources": {"kinds": ["Pod"]}},
               "validate": {"pattern": {"spec": {"volumes": [{"name": f"v{k}*"}]}}}} for k in range(6)]
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "grp"}, "spec": {"rules": rules}}

    def pod(n, big=None):
        cs = [{"name": f"c{rnd.randrange(9)}x", "image": f"{rnd.choice(regs)}/app:{i}"} for i in range(n)]
        if big is not None:
            cs[big]["image"] = "other.io/x"
        vols = rnd.choice([[{"name": f"v{rnd.randrange(8)}a"}], [], "notalist", [{"name": "v1"}, {"name": "z"}]])
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p"}, "spec": {"containers": cs, "volumes": vols}}

    ress = [pod(rnd.randrange(1, 6)) for _ in range(300)] + [pod(1100, big=1050), pod(1100, big=1023), pod(3)]
    mism, r, ost = compare(orc, [pol], ress, check_paths=True, max_path_checks=3000, specialize=spec)
    assert not mism, "\n".join(mism)
    assert (r.status == 1).sum() > 5000 and (r.status == 0).sum() > 100
    for j in (300, 301):  # every failing path of the 1100-container Pods (wide and compact indices)
        ov = orc.validate(pol, ress[j], None)
        for k in range(len(rules)):
            if r.status[k, j] == 1:
                assert r.path(k, j) == ov["rules"][k]["path"], (k, j)


@engines
def test_record_codes_raw_rules(orc, spec):
    """Error records cross PCIe as 1-byte codes into a per-rule table of at most 256 distinct
    records (kv_rec_code_kernel); a rule with more distinct records (here: one failing container
    index per resource, 600 indices) crosses raw. Both kinds in one result: paths vs the oracle and
    the failures export against kv_result_path."""
    rules = [{"name": "no-latest", "match": {"resources": {"kinds": ["Pod"]}},
              "validate": {"pattern": {"spec": {"containers": [{"image": "!*:latest"}]}}}},
             {"name": "team", "match": {"resources": {"kinds": ["Pod"]}},
              "validate": {"pattern": {"metadata": {"labels": {"team": "?*"}}}}}]
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "codes"}, "spec": {"rules": rules}}
    ress = []
    for i in range(700):
        n = i % 600 + 1
        cs = [{"name": f"c{j}", "image": "reg.io/app:1"} for j in range(n)]
        cs[-1]["image"] = "reg.io/app:latest"
        labels = {"team": "a"} if i % 3 else {}
        ress.append({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"p{i}", "labels": labels},
                     "spec": {"containers": cs}})
    mism, r, ost = compare(orc, [pol], ress, check_paths=True, max_path_checks=2000, specialize=spec)
    assert not mism, "\n".join(mism)
    assert (r.status[0] == 1).sum() == 700 and (r.status[1] == 1).sum() == 234
    rule, res, pid, paths = r.failures()
    assert len(rule) == 934
    for i in range(0, len(rule), 7):
        assert paths[pid[i]] == r.path(int(rule[i]), int(res[i]))
    assert len({paths[p] for p, q in zip(pid, rule) if q == 0}) == 600


@engines
@pytest.mark.parametrize("n", [1, 255, 256, 257, 513])
def test_status_transfer_form_edges(orc, spec, n):
    """The statuses cross as the (rule, 256-resource segment)s a pass wrote, 4 bits a status
    (kv_status_pack_kernel), and are rebuilt on first read: batches of partial and whole
    segments, kinds interleaved in the input (a permuted store order), a rule no resource
    matches (no segment written) and one every resource matches."""
    rules = [{"name": "pods", "match": {"resources": {"kinds": ["Pod"]}},
              "validate": {"pattern": {"spec": {"containers": [{"image": "!*:latest"}]}}}},
             {"name": "none", "match": {"resources": {"kinds": ["CronJob"]}},
              "validate": {"pattern": {"spec": {"schedule": "?*"}}}},
             {"name": "all", "match": {"resources": {"kinds": ["*"]}},
              "validate": {"pattern": {"metadata": {"name": "p*"}}}}]
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "edges"}, "spec": {"rules": rules}}
    ress = []
    for i in range(n):
        if i % 3 == 1:
            ress.append({"apiVersion": "v1", "kind": "Service", "metadata": {"name": f"s{i}", "namespace": f"n{i % 5}"}})
        else:
            ress.append({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"p{i}", "namespace": f"n{i % 5}"},
                         "spec": {"containers": [{"name": "c", "image": "a:latest" if i % 7 == 0 else "a:1"}]}})
    mism, r, ost = compare(orc, [pol], ress, check_paths=True, specialize=spec)
    assert not mism, "\n".join(mism)
    assert r.status.shape == (3, n) and (r.status[1] == 5).all()
