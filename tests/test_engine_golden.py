"""Engine-level known answers of the reference, checked on the oracle (CPU) and on the device (GPU):

* engine.json   — pkg/engine/validation_test.go:40-1411: RuleResponse messages in response order and
                  EngineResponse.IsSuccessful() for validate.pattern / anyPattern / anchor policies;
* match.json    — pkg/engine/utils_test.go:13-913: MatchesResourceDescription errors (match / exclude,
                  any / all, names, namespaces, selectors, user info), each rule turned into a validate
                  rule with the always-passing pattern {} so "no errors" = PASS and "errors" = no response;
* scenario.json — test/scenarios/** via pkg/testrunner: rule names, statuses and messages in order.

Fixtures: tests/golden/gen_engine_fixtures.py.
"""
import json
import os

import numpy as np
import pytest

from kyverno_amd import cli

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _cases(name):
    return json.load(open(os.path.join(GOLDEN, name)))["cases"]


ENGINE, MATCH, SCEN = _cases("engine.json"), _cases("match.json"), _cases("scenario.json")
ST = {0: "pass", 1: "fail", 2: "warn", 3: "error", 4: "skip"}


def _match_policy(case):
    pol = json.loads(json.dumps(case["policy"]))
    rules = []
    for r in pol["spec"]["rules"]:
        rules.append({k: v for k, v in r.items() if k in ("name", "match", "exclude")} |
                     {"validate": {"pattern": {}}})
    pol["spec"]["rules"] = rules
    return pol


def _responses_oracle(orc, pol, res):
    return [r for r in orc.validate(pol, res)["rules"] if r["status"] != "nomatch"]


# ------------------------------------------------------------------ oracle (CPU)

@pytest.mark.parametrize("case", ENGINE, ids=lambda c: c["name"])
def test_engine_messages_oracle(orc, case):
    rs = _responses_oracle(orc, case["policy"], json.loads(case["resource"]))
    if case["messages"] is not None:
        assert [r["message"] for r in rs] == case["messages"], case["src"]
    assert all(r["status"] not in ("fail", "error") for r in rs) == case["successful"], case["src"]


@pytest.mark.parametrize("case", MATCH, ids=lambda c: c["name"][:60])
def test_match_oracle(orc, case):
    pol = _match_policy(case)
    st, _ = orc.validate_batch(json.dumps([pol]), "[" + case["resource"] + "]",
                               ctx={"admission": case["admission"]})
    want = 5 if case["errors_expected"] else 0
    assert (st[:, 0] == want).all(), (case["src"], st[:, 0].tolist())


@pytest.mark.parametrize("case", SCEN, ids=lambda c: c["name"])
def test_scenario_oracle(orc, case):
    rs = _responses_oracle(orc, case["policy"], case["resource"])
    assert [(r["name"], r["status"]) for r in rs] == [(e["name"], e["status"]) for e in case["expected"]]
    for r, e in zip(rs, case["expected"]):
        if e["message"]:
            assert r["message"] == e["message"]


def test_fixture_counts():
    assert len(ENGINE) >= 15 and len(MATCH) == 24 and len(SCEN) >= 10


# ------------------------------------------------------------------ device (GPU)

def _device_responses(pol, res):
    ev = cli.evaluate([pol], [res])
    rs = [r for r in ev.policy_rules(0) if ev.status[r.index, 0] != cli.NOMATCH and r.route != cli.ROUTE_NORESPONSE]
    return [(r.name, int(ev.status[r.index, 0]), cli.rule_message(ev, r, 0)) for r in rs]


@pytest.mark.gpu
@pytest.mark.parametrize("case", ENGINE, ids=lambda c: c["name"])
def test_engine_messages_gpu(case):
    rs = _device_responses(case["policy"], json.loads(case["resource"]))
    if case["messages"] is not None:
        assert [m for _, _, m in rs] == case["messages"], case["src"]
    assert all(s not in (1, 3) for _, s, _ in rs) == case["successful"], case["src"]


@pytest.mark.gpu
def test_match_gpu():
    from kyverno_amd import batch

    for spec in (False, True):
        for case in MATCH:
            pol = _match_policy(case)
            ps = batch.PolicySet([pol], specialize=spec)
            b = batch.Batch(ps, [json.loads(case["resource"])])
            r = batch.validate(ps, b, admission=case["admission"])
            want = 5 if case["errors_expected"] else 0
            assert (r.status[:, 0] == want).all(), (case["src"], spec, r.status[:, 0].tolist())


@pytest.mark.gpu
@pytest.mark.parametrize("case", SCEN, ids=lambda c: c["name"])
def test_scenario_gpu(case):
    rs = _device_responses(case["policy"], case["resource"])
    assert [(n, ST.get(s, "cpu")) for n, s, _ in rs] == [(e["name"], e["status"]) for e in case["expected"]]
    for (_, _, m), e in zip(rs, case["expected"]):
        if e["message"]:
            assert m == e["message"]


# ------------------------------------------------------------------ per-call engine.Validate mirror (GPU)

@pytest.mark.gpu
@pytest.mark.parametrize("case", ENGINE, ids=lambda c: c["name"])
def test_engine_validate_mirror(case):
    """kyverno_amd.engine.validate(PolicyContext) -> EngineResponse against validation_test.go's
    messages and IsSuccessful (pkg/engine/validation.go:26, response.go:115-122)."""
    from kyverno_amd import engine

    resp = engine.validate(engine.PolicyContext(policy=case["policy"], new_resource=json.loads(case["resource"])))
    rules = resp.policy_response.rules
    if case["messages"] is not None:
        assert [r.message for r in rules] == case["messages"], case["src"]
    assert resp.is_successful() == case["successful"], case["src"]
    if rules:
        assert resp.policy_response.policy_name == case["policy"]["metadata"]["name"]
        assert resp.policy_response.rules_applied_count == sum(r.status in ("pass", "fail") for r in rules)
    else:  # buildResponse leaves an empty response untouched (validation.go:53-56)
        assert resp.policy_response.policy_name == ""


@pytest.mark.gpu
def test_engine_validate_batch_matches_per_call():
    """validate_batch ([policy][resource] in one kv_validate) equals per-call validate on the
    scenario fixtures, rule names / statuses / messages in order."""
    from kyverno_amd import engine

    pols = [c["policy"] for c in SCEN]
    ress = [c["resource"] for c in SCEN]
    grid = engine.validate_batch(pols, ress)
    for i, c in enumerate(SCEN):
        one = engine.validate(engine.PolicyContext(policy=c["policy"], new_resource=c["resource"]))
        got = grid[i][i].policy_response.rules
        assert [(r.name, r.status, r.message) for r in got] == \
               [(r.name, r.status, r.message) for r in one.policy_response.rules]
        assert [(r.name, r.status) for r in got] == [(e["name"], e["status"]) for e in c["expected"]]
