"""RuleResponse messages of every status, device vs oracle.

Pass / fail messages come from the status and the failing path; skip and error messages carry
err.Error() of the PatternError (pkg/engine/validation.go:421-439,510-527), rendered on the host
by ``kv_result_error_message`` from the device's error record (error form, pattern node, loop
indices, resolved key) and the resource document. The oracle restates the reference's message
construction (oracle/src/matcher.cpp, engine.cpp). The Go '%v' forms of floats and maps inside
these messages have no known answer in the reference's tests: parity unpinned beyond the oracle.
"""
import json
import os

import pytest

from kyverno_amd import autogen, batch, cli

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = pytest.mark.gpu


def _pol(name, rules):
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
            "spec": {"rules": rules}}


def _rule(name, pattern=None, message="", any_pattern=None, kinds=("Pod",)):
    v = {"message": message} if message else {}
    if any_pattern is not None:
        v["anyPattern"] = any_pattern
    else:
        v["pattern"] = pattern
    return {"name": name, "match": {"resources": {"kinds": list(kinds)}}, "validate": v}


# error forms of validate.go / anchor.go, each reached by some synthetic Pod. FAIL messages only
# name the path, so every form is also wrapped in a condition (global) anchor on a key all Pods
# have: the error then surfaces as "conditional (global) anchor mismatch: <form>", a SKIP.
FORMS = {
    "negation": {"X(hostPID)": "null", "containers": [{"name": "?*"}]},
    "existence": {"^(containers)": [{"image": "*:latest"}]},
    "existence-patlist": {"^(containers)": {"image": "?*"}},
    "existence-patmap": {"^(containers)": ["x"]},
    "existence-restype": {"^(hostNetwork)": [{"a": "b"}]},
    "star": {"containers": [{"name": "*", "imagePullPolicy": "*"}]},
    "type-map": {"securityContext": {"runAsNonRoot": True}},
    "type-arr": {"volumes": [{"name": "?*"}]},
    "value-map": {"containers": [{"resources": "x"}]},
    "value-bool": {"containers": [{"securityContext": {"privileged": False}}]},
    "value-int": {"containers": [{"ports": [{"containerPort": 80}]}]},
    "pattern-float": {"containers": [{"resources": {"requests": {"cpu": 0.5}}}]},
    "pattern-big-float": {"containers": [{"resources": {"requests": {"cpu": 12345678}}}]},
    "pattern-nil": {"containers": [{"imagePullPolicy": None}]},
    "scalar-list": {"containers": [{"securityContext": {"capabilities": {"add": ["NET_*"]}}}]},
    "empty-list": {"containers": []},
    "nested-cond": {"containers": [{"(image)": "*:latest", "imagePullPolicy": "Always"}]},
}
CRAFTED = [_pol("crafted-errors", [
    _rule("cond-skip", {"spec": {"(hostNetwork)": True, "containers": [{"name": "?*"}]}}),
    _rule("global-skip", {"spec": {"<(hostPID)": True, "containers": [{"name": "?*"}]}}),
    _rule("anchor-error", {"spec": {"(hostIPC)": True, "containers": [{"image": "nginx*"}]}},
          message="anchored rule"),
    _rule("anchor-error-nomsg", {"spec": {"(hostIPC)": False, "containers": [{"imagePullPolicy": "Never"}]}}),
    _rule("cond-in-array-error", {"spec": {"(hostIPC)": True, "containers": [{"(name)": "c0",
                                                                               "image": "registry.local*"}]}}),
    _rule("any-skip", any_pattern=[{"spec": {"(hostNetwork)": True, "containers": [{"name": "x"}]}},
                                   {"spec": {"containers": [{"image": "gcr.io/*"}]}}],
          message="any pattern"),
    _rule("any-error", any_pattern=[{"spec": {"(hostIPC)": True, "containers": [{"image": "quay.io/*"}]}},
                                    {"(spec)": {"containers": [{"name": "zz"}]}}]),
] + [_rule(k, {"spec": v}) for k, v in FORMS.items()]
  + [_rule("cond-" + k, {"(spec)": v}, message=f"{k} under a condition") for k, v in FORMS.items()]
  + [_rule("global-" + k, {"<(spec)": v}) for k, v in FORMS.items()]
  # an anchor key most Pods lack: errors become ERROR (ac.IsAnchorError, validate.go:41-45)
  + [_rule("error-" + k, {"spec": dict(v, **{"(hostIPC)": True})}) for k, v in FORMS.items()])]


# both device engines write the error records: bytecode interpreter and specialized kernels
engines = pytest.mark.parametrize("spec", [False, True], ids=["vm", "specialized"])


def _check(pols, ress, spec):
    """Every engine-response message of (policy, resource), device vs oracle; returns counts by status."""
    import oracle

    ev = cli.evaluate(pols, ress, specialize=spec)
    orc = oracle.get()
    seen = {}
    bad = []
    for pi, pol in enumerate(pols):
        for j, res in enumerate(ress):
            resp = [r for r in ev.policy_rules(pi)
                    if ev.status[r.index, j] != cli.NOMATCH and r.route != cli.ROUTE_NORESPONSE]
            orules = [rr for rr in orc.validate(pol, res)["rules"] if rr["status"] != "nomatch"]
            assert [r.name for r in resp] == [rr["name"] for rr in orules]
            for r, rr in zip(resp, orules):
                st = int(ev.status[r.index, j])
                if st == cli.CPU or rr.get("message_panics"):
                    continue
                got = cli.rule_message(ev, r, j)
                if got != rr["message"]:
                    bad.append(f"{pol['metadata']['name']}/{r.name} res {j} [{cli.REPORT_STATUS.get(st)}]:\n"
                               f"  device {got!r}\n  oracle {rr['message']!r}")
                seen[st] = seen.get(st, 0) + 1
    assert not bad, f"{len(bad)} messages differ:\n" + "\n".join(bad[:20])
    return seen


@engines
def test_messages_crafted_error_forms(spec):
    from kyverno_amd import workloads

    data = batch.synth(workloads.SEED + 4, 400).decode()
    ress = [json.loads(l) for l in data.strip().split("\n")]
    seen = _check(autogen.mutate_policies(CRAFTED), ress, spec)
    for st in (cli.PASS, cli.FAIL, cli.SKIP, cli.ERROR):
        assert seen.get(st, 0) > 10, (st, seen)


@engines
def test_messages_matcher_fixtures(spec):
    """validate_test.go patterns x resources (the whole cross product, every status)."""
    cases = [c for c in json.load(open(os.path.join(GOLDEN, "matcher.json")))["cases"]
             if isinstance(json.loads(c["resource"]), dict)]
    rules = [_rule(f"m{i}", json.loads(c["pattern"]), kinds=("*",)) for i, c in enumerate(cases)]
    ress = [json.loads(c["resource"]) for c in cases]
    seen = _check([_pol("matcher", rules)], ress, spec)
    assert seen.get(cli.FAIL, 0) and seen.get(cli.PASS, 0)


@engines
def test_messages_reference_corpus_all_statuses(spec):
    corpus = json.load(open(os.path.join(GOLDEN, "corpus.json")))["cases"][0]
    pols = autogen.mutate_policies([p["policy"] for p in corpus["policies"]])
    ress = [r["resource"] for r in corpus["resources"]]
    seen = _check(pols, ress, spec)
    assert sum(seen.values()) > 100


# validate messages with {{request.object.*}} variables: substituted on the host per resource
# (buildErrorMessage, validation.go:518-524; kyverno_amd/msgvars.py) for FAIL and ERROR pairs
VAR_MSGS = [_pol("message-vars", [
    _rule("latest", {"spec": {"containers": [{"image": "!*:latest"}]}},
          message="Pod {{request.object.metadata.namespace}}/{{request.object.metadata.name}} uses :latest"),
    _rule("labels", {"metadata": {"labels": {"app": "?*", "tier": "?*"}}},
          message="labels of {{request.object.metadata.name}}: {{request.object.metadata.labels}}"),
    _rule("image0", {"spec": {"containers": [{"imagePullPolicy": "Always"}]}},
          message="first image {{request.object.spec.containers[0].image}} of {{request.object.kind}}."),
    _rule("error-anchor", {"spec": {"(hostIPC)": True, "containers": [{"image": "nginx*"}]}},
          message="anchor on {{request.object.metadata.name}}"),
])]


@engines
def test_messages_with_request_object_variables(spec):
    from kyverno_amd import workloads

    data = batch.synth(workloads.SEED + 5, 300).decode()
    ress = [json.loads(l) for l in data.strip().split("\n")]
    seen = _check(VAR_MSGS, ress, spec)
    assert seen.get(cli.FAIL, 0) > 10 and seen.get(cli.PASS, 0) > 10, seen
