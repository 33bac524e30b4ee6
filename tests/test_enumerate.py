"""Oracle enumerate mode: the reference iterates Go maps in random order
in validateMap (pkg/engine/validate/validate.go:110-135; getSortedNestedAnchorResource,
validate/utils.go:37-51) and expandWildcards (pkg/engine/wildcards/wildcards.go:38-49), so a pair
with several failing keys can report different failing paths (or statuses) from run to run. The
oracle and the device share one canonical order; the enumerator replays every order and returns
the outcome set. Here: the set is right on crafted cases, contains the oracle's canonical outcome,
and (GPU) contains the device's (status, path) on the reference corpus and a C4 sample.
Report over the corpus and C4: tools/orderdep_report.py -> profiles/r02_orderdep.json.
"""
import json

import pytest

from kyverno_amd import cli

ST = {0: "pass", 1: "fail", 2: "warn", 3: "error", 4: "skip", 6: "cpu"}


def _pol(pattern, name="p"):
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
            "spec": {"rules": [{"name": "r", "match": {"resources": {"kinds": ["Pod"]}},
                                "validate": {"pattern": pattern}}]}}


def test_two_failing_keys_two_paths(orc):
    pol = _pol({"spec": {"a": "x", "b": "y", "c": "?*"}})
    res = {"kind": "Pod", "metadata": {"name": "n"}, "spec": {"a": "1", "b": "2", "c": "3"}}
    rule = orc.enumerate(pol, res)[0]
    assert not rule["truncated"]
    assert sorted(rule["outcomes"]) == [["fail", "/spec/a/"], ["fail", "/spec/b/"]]


def test_single_failure_deterministic(orc):
    pol = _pol({"spec": {"a": "x", "b": "2", "(c)": "3"}})
    res = {"kind": "Pod", "metadata": {"name": "n"}, "spec": {"a": "1", "b": "2", "c": "3"}}
    rule = orc.enumerate(pol, res)[0]
    assert rule["outcomes"] == [["fail", "/spec/a/"]]


def test_anchor_order_changes_status(orc):
    """A failing condition anchor (skip) and a failing equality anchor (fail) at one level: the
    outcome depends on which anchor the map iteration reaches first."""
    pol = _pol({"spec": {"(a)": "x", "=(b)": "y"}})
    res = {"kind": "Pod", "metadata": {"name": "n"}, "spec": {"a": "1", "b": "2"}}
    outs = {s for s, _ in orc.enumerate(pol, res)[0]["outcomes"]}
    assert outs == {"skip", "fail"}


def test_wildcard_label_key_choice(orc):
    """expandWildcards takes the first resource key matching a wildcard pattern key."""
    pol = _pol({"metadata": {"labels": {"app*": "web"}}})
    res = {"kind": "Pod", "metadata": {"name": "n", "labels": {"app1": "web", "app2": "db"}}}
    outs = sorted(orc.enumerate(pol, res)[0]["outcomes"])
    assert outs == [["fail", "/metadata/labels/app2/"], ["pass", ""]]


def test_canonical_outcome_in_set_corpus(orc):
    from parity_util import load_gold

    c = load_gold("corpus.json")[0]
    for p in [x["policy"] for x in c["policies"]]:
        for r in [x["resource"] for x in c["resources"]]:
            canon = orc.validate(p, r)["rules"]  # every rule, in order (names may repeat)
            for v, rule in zip(canon, orc.enumerate(p, r)):
                if rule["outcomes"] == [["nomatch", ""]]:
                    continue
                assert [v["status"], v["path"] if v["status"] == "fail" else ""] in rule["outcomes"]


def _c4_sample(n):
    from kyverno_amd import batch, workloads

    return workloads.c4_policies(), [json.loads(x) for x in
                                     batch.synth(workloads.SEED + 4, n).decode().strip().split("\n")]


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["corpus", "c4"])
def test_device_outcome_in_reference_set(orc, which):
    """The device's (status, failing path) of every matched pair is one the reference can produce."""
    if which == "corpus":
        from parity_util import load_gold

        c = load_gold("corpus.json")[0]
        pols, ress = [x["policy"] for x in c["policies"]], [x["resource"] for x in c["resources"]]
    else:
        pols, ress = _c4_sample(400)
    ev = cli.evaluate(pols, ress, specialize=which == "c4")
    n = 0
    for pi, p in enumerate(pols):
        rules = ev.policy_rules(pi)
        for k, r in enumerate(ress):
            for rule, en in zip(rules, orc.enumerate(p, r)):
                st = int(ev.status[rule.index, k])
                if en["outcomes"] == [["nomatch", ""]] or st == cli.CPU:
                    continue
                path = ev.paths.get((rule.index, k), "") if st == cli.FAIL else ""
                assert [ST[st], path] in en["outcomes"], (p["metadata"]["name"], rule.name, k, st, path, en)
                n += 1
    assert n > 100
