#!/usr/bin/env python3
"""Generate engine-level fixtures from the reference's own tests (run where /root/reference exists):
    python tests/golden/gen_engine_fixtures.py

Outputs (data only: inputs + asserted outputs, each case citing its `src`):
  engine.json   pkg/engine/validation_test.go:40-1411 (the validate.pattern / anchor tests): policy,
                resource (unstructured typing), the asserted RuleResponse messages in response order and
                the asserted EngineResponse.IsSuccessful().
  match.json    pkg/engine/utils_test.go:13-913 (TestMatchesResourceDescription table): admission info,
                resource, policy, and whether MatchesResourceDescription returns errors for its rules.
  scenario.json test/scenarios/** run by pkg/testrunner/testrunner_test.go (validation expectations of
                scenarios whose policy has no mutate rule, so Validate sees the resource as loaded):
                expected rule names, statuses and (when given) messages in response order.
"""
from __future__ import annotations

import json
import os
import re
import sys

import yaml

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))

from kyverno_amd import yamlio  # noqa: E402

from gen_fixtures import functions, read  # noqa: E402

_GO_STR = re.compile(r'"((?:[^"\\]|\\.)*)"')


def go_unquote(s: str) -> str:
    return json.loads('"' + s + '"')


def gen_engine():
    rel = "pkg/engine/validation_test.go"
    src = read(rel)
    cases = []
    for name, body, line in functions(src):
        if line > 1411 or not name.startswith("TestValidate_"):
            continue
        mp = re.search(r"rawPolicy\s*:=\s*\[\]byte\(`([^`]*)`\)", body)
        mr = re.search(r"rawResource\s*:=\s*\[\]byte\(`([^`]*)`\)", body)
        ms = re.search(r"msgs\s*:=\s*\[\]string\{(.*?)\}\n", body, re.S)
        ok = re.search(r"assert\.Assert\(t, (!?)er\.IsSuccessful\(\)\)", body)
        if not (mp and mr and ok):
            continue
        msgs = [go_unquote(x) for x in _GO_STR.findall(ms.group(1))] if ms else None
        cases.append({"name": name, "src": f"{rel}:{line}", "policy": json.loads(mp.group(1)),
                      "resource": mr.group(1).strip(), "messages": msgs, "successful": ok.group(1) != "!"})
    return cases


def gen_match():
    rel = "pkg/engine/utils_test.go"
    src = read(rel)
    cases = []
    for name, body, line in functions(src):
        if name != "TestMatchesResourceDescription":
            continue
        for m in re.finditer(r"\{\s*Description:\s*\"([^\"]*)\",(.*?)areErrorsExpected:\s*(true|false),", body, re.S):
            desc, inner, exp = m.group(1), m.group(2), m.group(3) == "true"
            roles = re.search(r"ClusterRoles:\s*\[\]string\{([^}]*)\}", inner)
            res = re.search(r"Resource:\s*\[\]byte\(`([^`]*)`\)", inner)
            pol = re.search(r"Policy:\s*\[\]byte\(`([^`]*)`\)", inner)
            cl = [go_unquote(x) for x in _GO_STR.findall(roles.group(1))] if roles else []
            cases.append({"name": desc, "src": f"{rel}:{line + body.count(chr(10), 0, m.start())}",
                          "admission": {"clusterRoles": cl, "roles": [], "groups": [], "username": ""},
                          "resource": res.group(1).strip(), "policy": json.loads(pol.group(1)),
                          "errors_expected": exp})
    return cases


def drop_empty_strings(x):
    """The test runner decodes resources through the typed client-go scheme and back
    (scenario.go:389-415: UniversalDeserializer + DefaultUnstructuredConverter), which drops the
    `omitempty` fields holding "" (k8s API string fields are omitempty), e.g. seLinuxOptions.level."""
    if isinstance(x, dict):
        return {k: drop_empty_strings(v) for k, v in x.items() if v != ""}
    if isinstance(x, list):
        return [drop_empty_strings(v) for v in x]
    return x


def gen_scenarios():
    rel = "pkg/testrunner/testrunner_test.go"
    src = read(rel)
    cases = []
    for m in re.finditer(r'testScenario\(t, "/?([^"]+)"\)', src):
        path = m.group(1)
        for tc in yaml.safe_load_all(open(os.path.join(REF, path))):
            if not tc:
                continue
            exp = (((tc.get("expected") or {}).get("validation") or {}).get("policyresponse") or {})
            rules = exp.get("rules")
            if not rules:
                continue
            pols = yamlio.load_policies_file(os.path.join(REF, tc["input"]["policy"]))
            pol = yamlio.to_go_json_obj(pols[0])
            if any("mutate" in r for r in pol["spec"]["rules"]):
                continue
            ress = yamlio.load_resources_file(os.path.join(REF, tc["input"]["resource"]), default_namespace="")
            res = drop_empty_strings(yamlio.to_go_json_obj(ress[0]))
            md = res.get("metadata", {})
            md.pop("creationTimestamp", None)  # loadPolicyResource (scenario.go:346-349)
            if md.get("namespace") == "":  # the test runner does not default the namespace
                md.pop("namespace")
            cases.append({"name": path, "src": f"{path} via {rel}:{src.count(chr(10), 0, m.start()) + 1}",
                          "policy": pol, "resource": res,
                          "expected": [{"name": r["name"], "status": r["status"], "message": r.get("message", "")}
                                       for r in rules]})
    return cases


def main():
    outs = {"engine.json": gen_engine(), "match.json": gen_match(), "scenario.json": gen_scenarios()}
    for fn, cases in outs.items():
        with open(os.path.join(OUT, fn), "w") as f:
            json.dump({"generator": "tests/golden/gen_engine_fixtures.py", "reference": "isabella232/kyverno v1.5.x",
                       "cases": cases}, f, indent=1, sort_keys=True)
        print(f"{fn}: {len(cases)} cases", file=sys.stderr)


if __name__ == "__main__":
    main()
