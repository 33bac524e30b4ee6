#!/usr/bin/env python3
"""Generate the autogen / CLI / chart fixtures from the reference's own tests and files.

Run in the build container (where /root/reference exists):
    python tests/golden/gen_cli_fixtures.py

Outputs (data only: inputs + asserted outputs, each case citing its `src`):
  autogen.json  pkg/policymutation/policymutation_test.go — the JSON patches asserted for
                generateRulePatches, the controllers asserted for CanAutoGen, the replace patches
                asserted for checkForGVKFormatPatch. The per-test policy edits written in Go in
                the reference test bodies are restated as `edit` records below.
  cli.json      pkg/kyverno/apply/apply_command_test.go (policy-report summaries) and
                test/cli/test/{simple,autogen} (policies, resources, expected per-rule results of
                `kyverno test`), converted to JSON with the reference's YAML conventions.
  chart.json    charts/kyverno-policies/templates/** rendered with podSecurityStandard=restricted
                and validationFailureAction=audit (charts/kyverno-policies/values.yaml), the
                anchor-heavy policy set of configs C4/C5 (BASELINE.json).
"""
from __future__ import annotations

import json
import os
import re
import sys

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))

from kyverno_amd import yamlio  # noqa: E402

from gen_fixtures import functions, read  # noqa: E402

POD_CONTROLLERS = "DaemonSet,Deployment,Job,StatefulSet,CronJob"  # pkg/engine/mutation.go:25

# Go edits applied to the loaded policy before generateRulePatches (policymutation_test.go), restated:
# (file, [(json path, value)], annotations, controllers)
RULE_PATCH_SETUPS = {
    "Test_Any": ("test/best_practices/disallow_bind_mounts.yaml",
                 [(["spec", "rules", 0, "match", "any"], [{"resources": {"kinds": ["Pod"]}}])], None, POD_CONTROLLERS),
    "Test_All": ("test/best_practices/disallow_bind_mounts.yaml",
                 [(["spec", "rules", 0, "match", "all"], [{"resources": {"kinds": ["Pod"]}}])], None, POD_CONTROLLERS),
    "Test_Exclude": ("test/best_practices/disallow_bind_mounts.yaml",
                     [(["spec", "rules", 0, "exclude"], {"resources": {"namespaces": ["fake-namespce"]}})], None,
                     POD_CONTROLLERS),
    "Test_CronJobOnly": ("test/best_practices/disallow_bind_mounts.yaml", [], "CronJob", "CronJob"),
    "Test_CronJob_hasExclude": ("test/best_practices/disallow_bind_mounts.yaml",
                                [(["spec", "rules", 0, "exclude"],
                                  {"resources": {"kinds": ["Pod"], "namespaces": ["test"]}})], "CronJob", "CronJob"),
    "Test_CronJobAndDeployment": ("test/best_practices/disallow_bind_mounts.yaml", [], "CronJob,Deployment",
                                  "CronJob,Deployment"),
    "Test_UpdateVariablePath": ("test/best_practices/select-secrets.yaml", [], None, POD_CONTROLLERS),
}


def _line(src: str, off: int) -> int:
    return src.count("\n", 0, off) + 1


def gen_autogen():
    rel = "pkg/policymutation/policymutation_test.go"
    src = read(rel)
    cases = []
    for name, body, line in functions(src):
        if name in RULE_PATCH_SETUPS:
            f, edits, ann, controllers = RULE_PATCH_SETUPS[name]
            pol = yamlio.to_go_json_obj(yamlio.load_policies_file(os.path.join(REF, f))[0])
            for path, value in edits:
                node = pol
                for k in path[:-1]:
                    node = node.setdefault(k, {}) if isinstance(k, str) else node[k]
                node[path[-1]] = value
            if ann is not None:
                pol.setdefault("metadata", {})["annotations"] = {"pod-policies.kyverno.io/autogen-controllers": ann}
            blk = body[body.index("expectedPatches"):]
            patches = [json.loads(m.group(1)) for m in re.finditer(r"\[\]byte\(`([^`]*)`\)", blk)]
            cases.append({"kind": "rule_patches", "name": name, "src": f"{rel}:{line}", "policy": pol,
                          "policy_src": f, "controllers": controllers, "expected": patches})
        elif name in ("Test_getControllers", "Test_checkForGVKFormatPatch"):
            for m in re.finditer(r"\{\s*name:\s*\"([^\"]+)\",\s*policy:\s*\[\]byte\(`([^`]*)`\),\s*"
                                 r"(expectedControllers|expectedPatches):\s*([^\n]+?),?\n", body):
                cname, pol, field, exp = m.group(1), json.loads(m.group(2)), m.group(3), m.group(4).rstrip(",")
                cline = line + body.count("\n", 0, m.start()) + 1
                if field == "expectedControllers":
                    exp = POD_CONTROLLERS if exp == "engine.PodControllers" else json.loads(exp)
                    cases.append({"kind": "controllers", "name": cname, "src": f"{rel}:{cline}", "policy": pol,
                                  "expected": exp})
                else:
                    if exp == "nil":
                        expected = []
                    else:
                        expected = [json.loads(re.match(r"\[\]byte\(`([^`]*)`\)", exp).group(1))]
                    cases.append({"kind": "gvk", "name": cname, "src": f"{rel}:{cline}", "policy": pol,
                                  "expected": expected})
    return cases


def _load_dir_yaml(d, fn, loader):
    return [yamlio.to_go_json_obj(x) for x in loader(os.path.join(REF, d, fn))]


def gen_cli():
    cases = []
    rel = "pkg/kyverno/apply/apply_command_test.go"
    src = read(rel)
    for m in re.finditer(r"PolicyPaths:\s*\[\]string\{\"([^\"]+)\"\},\s*ResourcePaths:\s*\[\]string\{\"([^\"]+)\"\},"
                         r".*?Pass:\s*(\d+),\s*Fail:\s*(\d+),\s*Skip:\s*(\d+),\s*Error:\s*(\d+),\s*Warn:\s*(\d+)",
                         src, re.S):
        ppath, rpath = (p.replace("../../../", "") for p in m.group(1, 2))
        pols = _load_dir_yaml(os.path.dirname(ppath), os.path.basename(ppath), yamlio.load_policies_file)
        ress = _load_dir_yaml(os.path.dirname(rpath), os.path.basename(rpath), yamlio.load_resources_file)
        p, f, s, e, w = (int(x) for x in m.group(3, 4, 5, 6, 7))
        cases.append({"kind": "apply_summary", "src": f"{rel}:{_line(src, m.start())}", "policy_src": ppath,
                      "resource_src": rpath, "policies": pols, "resources": ress,
                      "expected": {"pass": p, "fail": f, "warn": w, "error": e, "skip": s}})
    import yaml

    for t in ("simple", "autogen"):
        d = f"test/cli/test/{t}"
        spec = yaml.safe_load(open(os.path.join(REF, d, "test.yaml")))
        pols, ress = [], []
        for fn in spec["policies"]:
            pols += _load_dir_yaml(d, fn, yamlio.load_policies_file)
        for fn in spec["resources"]:
            ress += _load_dir_yaml(d, fn, yamlio.load_resources_file)
        results = []
        for r in spec["results"]:
            results.append({"policy": r["policy"], "rule": r["rule"], "resource": r["resource"],
                            "kind": r.get("kind", ""), "namespace": r.get("namespace", ""),
                            "result": r.get("result") or r.get("status")})
        cases.append({"kind": "kyverno_test", "src": f"{d}/test.yaml", "policies": pols, "resources": ress,
                      "results": results})
    return cases


def render_chart_template(text: str, values: dict) -> str | None:
    """The subset of Go templating the kyverno-policies chart templates use (charts/kyverno-policies/
    templates/**, _helpers.tpl): the `$name` binding, the baseline/restricted guard, the severity
    annotation guard, .Values.validationFailureAction, and the helm labels include (dropped: labels
    do not take part in validation). Returns None when the guard excludes the policy."""
    name = re.search(r'\{\{-\s*\$name\s*:=\s*"([^"]+)"\s*\}\}', text).group(1)
    guard = re.search(r'include "kyverno-policies\.(podSecurityBaseline|podSecurityRestricted)"', text)
    std = values["podSecurityStandard"]
    if guard:
        level = guard.group(1)
        on = std == "restricted" or (level == "podSecurityBaseline" and std == "baseline") or \
            (std == "custom" and name in values.get("podSecurityPolicies", []))
        if not on:
            return None
    out = []
    drop = False  # inside a false {{- if .Values.podSecuritySeverity }} block
    for ln in text.splitlines():
        st = ln.strip()
        if st.startswith("{{- if .Values.podSecuritySeverity"):
            drop = not values.get("podSecuritySeverity")
            continue
        if st.startswith("{{-") or st.startswith("{{/*"):  # pure template directives ($name, guards, end)
            if st.startswith("{{- end"):
                drop = False
            continue
        if drop:
            continue
        if "kyverno-policies.labels" in ln:
            ln = re.sub(r"\{\{[^}]*\}\}", "", ln).rstrip()
        ln = ln.replace("{{ $name }}", name)
        ln = ln.replace("{{ .Values.validationFailureAction }}", values["validationFailureAction"])
        ln = ln.replace("{{ .Values.podSecuritySeverity | quote }}", json.dumps(values.get("podSecuritySeverity")))
        assert "{{" not in ln or "request." in ln, ln
        out.append(ln)
    return "\n".join(out) + "\n"


def gen_chart():
    values = {"podSecurityStandard": "restricted", "podSecuritySeverity": "medium", "podSecurityPolicies": [],
              "validationFailureAction": "audit"}
    base = "charts/kyverno-policies/templates"
    cases = []
    for sub in ("default", "restricted"):
        for fn in sorted(os.listdir(os.path.join(REF, base, sub))):
            text = read(f"{base}/{sub}/{fn}")
            y = render_chart_template(text, values)
            if y is None:
                continue
            docs = [d for d in yamlio.load_documents(y) if d]
            for d in docs:
                cases.append({"src": f"{base}/{sub}/{fn}", "policy": yamlio.to_go_json_obj(d)})
    return cases


def main():
    outs = {"autogen.json": gen_autogen(), "cli.json": gen_cli(), "chart.json": gen_chart()}
    for fn, cases in outs.items():
        with open(os.path.join(OUT, fn), "w") as f:
            json.dump({"generator": "tests/golden/gen_cli_fixtures.py", "reference": "isabella232/kyverno v1.5.x",
                       "cases": cases}, f, indent=1, sort_keys=True)
        print(f"{fn}: {len(cases)} cases", file=sys.stderr)


if __name__ == "__main__":
    main()
