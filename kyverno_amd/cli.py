"""`kyverno apply` / `kyverno test` front end over the batch engine.

Mirrors the reference CLI for validate rules:

* ``apply POLICY... -r RESOURCE... [--policy-report]`` — ``applyCommandHelper`` +
  ``printReportOrViolation`` (pkg/kyverno/apply/apply_command.go:147-381):
  policies loaded and mutated (defaults + autogen, ``common.MutatePolices``,
  pkg/kyverno/common/common.go:429-444 → ``kyverno_amd.autogen``), resources
  loaded with the unstructured number typing and namespace "default"
  (pkg/kyverno/common/fetch.go:251-279), every (policy, resource) pair evaluated,
  counted with ``ProcessValidateEngineResponse`` (common.go:703-766), violations
  printed, summary line printed, exit status 1 on fail/error.
* ``test DIR`` — ``kyverno test`` over a ``test.yaml`` (pkg/kyverno/test/
  test_command.go:347-494): each expected result is looked up by policy, rule
  (with the ``autogen-`` / ``autogen-cronjob-`` fallback) and resource.

Evaluation runs on the GPU through the C ABI (``kyverno_amd.batch``): one
``kv_validate`` over the whole (rule × resource) cross product instead of the
reference's per-pair ``engine.Validate`` loop (apply_command.go:270-310). Rules
the device does not evaluate (variables other than ``request.object`` paths,
context, preconditions, deny, foreach — ``KV_ROUTE_CPU``) are reported as routed to the reference engine and
not counted; a Go host runs them through ``engine.Validate``.

    python -m kyverno_amd apply policy.yaml -r pods.yaml [--policy-report] [--device N]
    python -m kyverno_amd test test/cli/test/simple
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
from dataclasses import dataclass, field

import numpy as np

from . import autogen, msgvars, yamlio

PASS, FAIL, WARN, ERROR, SKIP, NOMATCH, CPU = range(7)  # kv status codes (include/kvgpu.h)
ROUTE_NORESPONSE = 2  # KV_ROUTE_NORESPONSE: not a validate rule, never in the validate response
REPORT_STATUS = {PASS: "pass", FAIL: "fail", WARN: "warn", ERROR: "error", SKIP: "skip"}
DIVIDER = "-" * 70
# variables.RegexVariables (pkg/engine/variables/vars.go:20)
_REGEX_VARIABLES = re.compile(r"^\{\{[^{}]*\}\}|[^\\]\{\{[^{}]*\}\}")


# ---------------------------------------------------------------- loading


def _yaml_files(path: str) -> list[str]:
    if os.path.isdir(path):
        out = []
        for root, _, files in sorted(os.walk(path)):
            out += [os.path.join(root, f) for f in sorted(files) if f.endswith((".yaml", ".yml", ".json"))]
        return out
    return [path]


def load_policies(paths: list[str]) -> list[dict]:
    """common.GetPolicies (pkg/kyverno/common/common.go:83-168): files or directories."""
    out = []
    for p in paths:
        for f in _yaml_files(p):
            out += [yamlio.to_go_json_obj(x) for x in yamlio.load_policies_file(f)]
    return out


def load_resources(paths: list[str]) -> list[dict]:
    """whenClusterIsFalse → GetResource (fetch.go:110-190): documents without a kind are dropped."""
    out = []
    for p in paths:
        for f in _yaml_files(p):
            out += [yamlio.to_go_json_obj(x) for x in yamlio.load_resources_file(f)]
    return out


def has_unset_variables(policy: dict) -> bool:
    """common.HasVariables + RemoveDuplicateAndObjectVariables (common.go:76-80, :298-311): a policy
    with a `{{ }}` variable that is not request.object / element needs --set / --values-file values
    and is skipped by `apply` (apply_command.go:283-293)."""
    raw = json.dumps(policy, separators=(",", ":"), ensure_ascii=False)
    for m in _REGEX_VARIABLES.finditer(raw):
        v = m.group(0)
        if "request.object" not in v and "element" not in v:
            return True
    return False


# ---------------------------------------------------------------- evaluation


@dataclass
class Evaluation:
    """Per-(rule, resource) statuses of one evaluation of the mutated policies."""
    policies: list          # mutated policies, as evaluated
    resources: list
    rules: list             # batch.Rule per compiled rule (policy order)
    status: np.ndarray      # u8 [n_rules][n_res]
    paths: dict = field(default_factory=dict)   # (rule, res) -> failing path (FAIL pairs)
    errors: dict = field(default_factory=dict)  # (rule, res) -> err.Error() of ERROR / SKIP pairs
    subst: dict = field(default_factory=dict)   # (rule, res) -> message of a pattern-variable substitution ERROR
    anypattern: dict = field(default_factory=dict)  # (rule, res) -> [(status, path)] per pattern
    warnings: list = field(default_factory=list)    # host-side limits met while rendering messages

    def policy_rules(self, pi: int) -> list:
        return [r for r in self.rules if r.policy == pi]


def evaluate(policies: list[dict], resources: list[dict], device: int = 0, messages: bool = True,
             namespace_labels: dict | None = None, specialize: bool = False, gpus: int = 1) -> Evaluation:
    """All (rule, resource) pairs on the GPU (``kv_compile`` → ``kv_ingest`` → ``kv_validate``).
    ``specialize`` selects the per-policy-set specialized kernels (worth their hiprtc compile on
    large batches) over the bytecode interpreter; both write the same statuses and error records.
    ``gpus`` > 1 shards the resources over devices [device, device + gpus) (kv_validate_devices)."""
    from . import batch

    ps = batch.PolicySet(policies, specialize=specialize)
    b = batch.Batch(ps, resources, namespace_labels)
    mask = ((1 << gpus) - 1) << device if gpus > 1 else None
    r = batch.validate(ps, b, device=device, device_mask=mask)
    ev = Evaluation(policies, resources, ps.rules, r.status)
    if messages:
        for ri, res in zip(*np.nonzero(r.status == FAIL)):
            if not ps.rules[ri].any_pattern:
                ev.paths[(int(ri), int(res))] = r.path(int(ri), int(res))
        collect_errors(ev, ps, r, resources)
        _evaluate_anypatterns(ev, device, specialize, namespace_labels)
    return ev


def collect_errors(ev: Evaluation, ps, r, resources: list) -> None:
    """Messages of the ERROR / SKIP pairs: pattern-variable substitution errors (whole message),
    else the pattern error's err.Error() (pattern rules; anyPattern rules render per pattern)."""
    for ri, res in zip(*np.nonzero((r.status == ERROR) | (r.status == SKIP))):
        key = (int(ri), int(res))
        if r.status[ri, res] == ERROR:
            m = r.subst_error(*key)
            if m is not None:
                ev.subst[key] = m
                continue
        if not ps.rules[ri].any_pattern:
            m = r.error_message(int(ri), int(res), resources[int(res)])
            if m is not None:
                ev.errors[key] = m


def _evaluate_anypatterns(ev: Evaluation, device: int, specialize: bool = False,
                          namespace_labels: dict | None = None) -> None:
    """Per-pattern outcomes of anyPattern rules, for the pass index and the failure message of
    validatePatterns (pkg/engine/validation.go:446-484): every pattern of the rule is compiled as a
    pattern rule of its own (same match/exclude) and run on the device over the resources where
    the anyPattern rule passed or failed."""
    from . import batch

    todo = [(r, np.nonzero((ev.status[r.index] == PASS) | (ev.status[r.index] == FAIL))[0])
            for r in ev.rules if r.any_pattern]
    todo = [(r, idx) for r, idx in todo if len(idx)]
    if not todo:
        return
    for rule, idx in todo:
        src = ev.policies[rule.policy]
        rdoc = next(x for x in src["spec"]["rules"] if x.get("name") == rule.name)
        pats = rdoc["validate"]["anyPattern"]
        sub_rules = []
        for j, p in enumerate(pats):
            sr = {k: v for k, v in rdoc.items() if k != "validate"}
            sr["name"] = f"{rule.name}[{j}]"
            sr["validate"] = {"message": rdoc["validate"].get("message", ""), "pattern": p}
            sub_rules.append(sr)
        sub = {"apiVersion": src.get("apiVersion", "kyverno.io/v1"), "kind": src.get("kind", "ClusterPolicy"),
               "metadata": src.get("metadata", {}), "spec": {"rules": sub_rules}}
        ps = batch.PolicySet([sub], specialize=specialize)
        ress = [ev.resources[i] for i in idx]
        b = batch.Batch(ps, ress, namespace_labels)
        r = batch.validate(ps, b, device=device)
        for k, res in enumerate(idx):
            outs = []
            for j in range(len(pats)):
                st = int(r.status[j, k])
                if st == FAIL:
                    outs.append((st, r.path(j, k)))
                elif st in (ERROR, SKIP):  # PatternError with an empty path: its text
                    outs.append((st, r.error_message(j, k, ress[k])))
                else:
                    outs.append((st, None))
            ev.anypattern[(rule.index, int(res))] = outs


# ---------------------------------------------------------------- messages


def _with_dot(s: str) -> str:
    return s if s.endswith(".") else s + "."


def _message(ev: Evaluation, rule, res: int) -> str:
    """The rule's message after SubstituteAll (msgvars). A JMESPath form the host does not evaluate
    leaves the message as written and is reported in ``ev.warnings``; a form on which the reference
    panics raises ``msgvars.MessageVariableError``."""
    try:
        return msgvars.substitute_message(rule.message, ev.resources[res])
    except msgvars.UnsupportedMessageVariable as e:
        w = f"rule {rule.name}: message variables not rendered: {e}"
        if w not in ev.warnings:
            ev.warnings.append(w)
        return rule.message


def rule_message(ev: Evaluation, rule, res: int) -> str:
    """RuleResponse.Message (validatePatterns, buildErrorMessage, buildAnyPatternErrorMessage:
    pkg/engine/validation.go:421-547): pass / fail from the status and failing path, skip / error
    from the device's error record rendered by ``kv_result_error_message``."""
    st = int(ev.status[rule.index, res])
    if st == ERROR and (rule.index, res) in ev.subst:  # ruleError("variable substitution failed", err)
        return ev.subst[(rule.index, res)]
    if rule.any_pattern:
        outs = ev.anypattern.get((rule.index, res), [])
        if st == PASS:
            j = next((j for j, (s, _) in enumerate(outs) if s == PASS), 0)
            return f"validation rule '{rule.name}' anyPattern[{j}] passed."
        errs = []
        for j, (s, detail) in enumerate(outs):
            if s == FAIL and detail:
                errs.append(f"Rule {rule.name}[{j}] failed at path {detail}.")
            elif s in (ERROR, SKIP) and detail is not None:
                errs.append(f"Rule {rule.name}[{j}] failed: {detail}.")
        es = " ".join(errs)
        if not rule.message:
            return f"validation error: {es}"
        return f"validation error: {_with_dot(rule.message)} {es}"
    if st == PASS:
        return f"validation rule '{rule.name}' passed."
    if st == FAIL:
        path = ev.paths.get((rule.index, res), "")
        if not rule.message:
            return f"validation error: rule {rule.name} failed at path {path}"
        msg = _message(ev, rule, res)
        return f"validation error: {_with_dot(msg)} Rule {rule.name} failed at path {path}"
    if st in (ERROR, SKIP) and (rule.index, res) in ev.errors:
        err = ev.errors[(rule.index, res)]
        if st == SKIP:  # ruleResponse(..., pe.Error(), RuleStatusSkip)
            return err
        if not rule.message:  # buildErrorMessage(err, "")
            return f"validation error: rule {rule.name} execution error: {err}"
        msg = _message(ev, rule, res)
        return f"validation error: {_with_dot(msg)} Rule {rule.name} execution error: {err}"
    if rule.const_message:
        return rule.const_message
    return ""


# ---------------------------------------------------------------- apply


@dataclass
class ResultCounts:
    """common.ResultCounts (pkg/kyverno/common/common.go:41-47)."""
    pass_: int = 0
    fail: int = 0
    warn: int = 0
    error: int = 0
    skip: int = 0
    routed: int = 0  # pairs of KV_ROUTE_CPU rules: evaluated by the reference engine, not here


def resource_path(res: dict) -> str:
    md = res.get("metadata") or {}
    return f"{md.get('namespace', '')}/{res.get('kind', '')}/{md.get('name', '')}"


def process_validate(ev: Evaluation, pi: int, res: int, rc: ResultCounts, policy_report: bool, out) -> dict:
    """ProcessValidateEngineResponse (common.go:703-766) for one (policy, resource): every policy
    rule found in the engine response is counted by its status, every other rule as skip; failures
    are printed with their index in the response. Returns the policyreport.Info result record."""
    policy = ev.policies[pi]
    rules = ev.policy_rules(pi)
    # the engine response holds the matched validate rules, in policy order (validation.go:78-106)
    resp = [r.index for r in rules if ev.status[r.index, res] != NOMATCH and r.route != ROUTE_NORESPONSE]
    printed = False
    violated = []
    for r in rules:
        if r.index in resp:
            i = resp.index(r.index)
            st = int(ev.status[r.index, res])
            if st == CPU:
                rc.routed += 1
                violated.append({"name": r.name, "status": "cpu", "message": ""})
                continue
            msg = rule_message(ev, r, res)
            if st == PASS:
                rc.pass_ += 1
            elif st == FAIL:
                rc.fail += 1
                if not policy_report:
                    if not printed:
                        out.write(f"\npolicy {policy['metadata']['name']} -> resource {resource_path(ev.resources[res])} "
                                  f"failed: \n")
                        printed = True
                    out.write(f"{i + 1}. {r.name}: {msg} \n")
            elif st == ERROR:
                rc.error += 1
            elif st == WARN:
                rc.warn += 1
            elif st == SKIP:
                rc.skip += 1
            violated.append({"name": r.name, "status": REPORT_STATUS[st], "message": msg})
        else:
            rc.skip += 1
            violated.append({"name": r.name, "status": "skip", "message": r.message})
    res_doc = ev.resources[res]
    md = res_doc.get("metadata") or {}
    return {"policy": policy["metadata"]["name"], "namespace": md.get("namespace", ""),
            "resource": {"kind": res_doc.get("kind", ""), "namespace": md.get("namespace", ""),
                         "apiVersion": res_doc.get("apiVersion", ""), "name": md.get("name", ""),
                         "uid": md.get("uid", "")},
            "rules": violated}


def policy_has_validate(policy: dict) -> bool:
    return any((r.get("validate") or None) is not None and r.get("validate") != {}
               for r in (policy.get("spec") or {}).get("rules") or [])


def apply(policy_paths: list[str], resource_paths: list[str], policy_report: bool = False, device: int = 0,
          out=sys.stdout, evaluation_fn=None, gpus: int = 1) -> tuple[ResultCounts, list]:
    """applyCommandHelper (apply_command.go:147-310) for resource files. Returns counts and the
    policyreport infos. ``evaluation_fn(policies, resources) -> Evaluation`` replaces the device
    evaluation (tests of the host logic)."""
    policies = load_policies(policy_paths)
    resources = load_resources(resource_paths)
    return apply_docs(policies, resources, policy_report, device, out, evaluation_fn, gpus)


def apply_docs(policies: list[dict], resources: list[dict], policy_report: bool = False, device: int = 0,
               out=sys.stdout, evaluation_fn=None, gpus: int = 1) -> tuple[ResultCounts, list]:
    mutated = autogen.mutate_policies(policies)
    if len(mutated) > 0 and len(resources) > 0:
        msg_p = "1 policy" if len(mutated) <= 1 else f"{len(policies)} policies"
        msg_r = "1 resource" if len(resources) <= 1 else f"{len(resources)} resources"
        out.write(f"\nApplying {msg_p} to {msg_r}... \n(Total number of result count may vary as the policy is "
                  f"mutated by Kyverno. To check the mutated policy please try with log level 5)\n")
    rc = ResultCounts()
    skipped = [p["metadata"]["name"] for p in mutated if has_unset_variables(p)]
    active = [p for p in mutated if not has_unset_variables(p)]
    infos = []
    if active and resources:
        ev = (evaluation_fn or (lambda p, r: evaluate(p, r, device=device, gpus=gpus)))(active, resources)
        for pi, pol in enumerate(active):
            if not policy_has_validate(pol):
                continue
            for res in range(len(resources)):
                infos.append(process_validate(ev, pi, res, rc, policy_report, out))
        for w in ev.warnings:
            print(f"warning: {w}", file=sys.stderr)
    if skipped:
        out.write(DIVIDER + "\n")
        out.write("Policies Skipped (as required variables are not provided by the user):\n")
        for i, n in enumerate(skipped):
            out.write(f"{i + 1}. {n}\n")
        out.write(DIVIDER + "\n")
    if policy_report:
        reports = build_policy_reports(infos)
        if reports or not resources:
            out.write(DIVIDER + "\nPOLICY REPORT:\n" + DIVIDER + "\n")
            out.write(json.dumps(reports, indent=2) + "\n")
        else:
            out.write(DIVIDER + "\nPOLICY REPORT: skip generating policy report (no validate policy found/resource "
                      "skipped)\n")
    else:
        out.write(f"\npass: {rc.pass_}, fail: {rc.fail}, warn: {rc.warn}, error: {rc.error}, skip: {rc.skip} \n")
    if rc.routed:
        out.write(f"(routed to the reference engine, not evaluated here: {rc.routed} rule results)\n")
    return rc, infos


def build_policy_reports(infos: list) -> list[dict]:
    """buildPolicyReports / buildPolicyResults / calculateSummary (pkg/kyverno/apply/report.go:23-179):
    one ClusterPolicyReport for cluster-scoped resources, one PolicyReport per namespace."""
    scopes: dict[str, list] = {}
    for info in infos:
        scope = f"policyreport-ns-{info['namespace']}" if info["namespace"] else "clusterpolicyreport"
        for r in info["rules"]:
            if r["status"] == "cpu":
                continue
            scopes.setdefault(scope, []).append({"policy": info["policy"], "rule": r["name"],
                                                 "message": r["message"], "result": r["status"],
                                                 "resources": [info["resource"]], "scored": True,
                                                 "source": "Kyverno"})
    reports = []
    for scope, results in scopes.items():
        summary = {k: sum(1 for x in results if x["result"] == k) for k in ("pass", "fail", "warn", "error", "skip")}
        rep = {"apiVersion": "wgpolicyk8s.io/v1alpha2",
               "kind": "ClusterPolicyReport" if scope == "clusterpolicyreport" else "PolicyReport",
               "metadata": {"name": scope}, "results": results, "summary": summary}
        if scope != "clusterpolicyreport":
            rep["metadata"]["namespace"] = scope[len("policyreport-ns-"):]
        reports.append(rep)
    return reports


# ---------------------------------------------------------------- test


def run_test(spec: dict, policies: list[dict], resources: list[dict], device: int = 0,
             evaluation_fn=None) -> list[dict]:
    """`kyverno test` result matching (pkg/kyverno/test/test_command.go:347-494) for validate rules:
    the expected rule name falls back to autogen-<rule> / autogen-cronjob-<rule> when the policy's
    response does not hold it; a rule absent from the response is `skip`. Returns one row per
    expected result with the actual result ("cpu" for rules routed to the reference engine)."""
    mutated = autogen.mutate_policies(policies)
    ev = (evaluation_fn or (lambda p, r: evaluate(p, r, device=device, messages=False)))(mutated, resources)
    rows = []
    for t in spec["results"]:
        want = t.get("result") or t.get("status")
        actual = None
        for pi, pol in enumerate(mutated):
            if pol["metadata"]["name"] != t["policy"]:
                continue
            for res, rd in enumerate(resources):
                md = rd.get("metadata") or {}
                if md.get("name") != t["resource"]:
                    continue
                if t.get("kind") and rd.get("kind") != t["kind"]:
                    continue
                resp = {r.name: r for r in ev.policy_rules(pi)
                        if ev.status[r.index, res] != NOMATCH and r.route != ROUTE_NORESPONSE}
                for name in (t["rule"], "autogen-" + t["rule"], "autogen-cronjob-" + t["rule"]):
                    if name in resp:
                        st = int(ev.status[resp[name].index, res])
                        actual = "cpu" if st == CPU else REPORT_STATUS[st]
                        break
                else:
                    actual = "skip"
        rows.append({**t, "want": want, "actual": actual,
                     "ok": actual == want if actual not in (None, "cpu") else None})
    return rows


# ---------------------------------------------------------------- main


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="kyverno", description="validate policies against resources on the GPU")
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("apply", help="applies policies on resources")
    a.add_argument("policies", nargs="+")
    a.add_argument("-r", "--resource", action="append", default=[], help="Path to resource files")
    a.add_argument("--policy-report", action="store_true", help="Generates policy report when passed")
    a.add_argument("--device", type=int, default=0, help="HIP device (first device with --gpus)")
    a.add_argument("--gpus", type=int, default=1, help="shard the resources over this many devices")
    t = sub.add_parser("test", help="run tests from a directory holding test.yaml")
    t.add_argument("dir")
    t.add_argument("--device", type=int, default=0)
    args = ap.parse_args(argv)
    if args.cmd == "apply":
        try:
            rc, _ = apply(args.policies, args.resource, args.policy_report, args.device, gpus=args.gpus)
        except msgvars.MessageVariableError as e:
            # the Go CLI dies in buildErrorMessage (msgRaw.(string), validation.go:519-524): a
            # panic, exit status 2
            print(f"panic: validate message substitution: {e}", file=sys.stderr)
            return 2
        return 1 if rc.fail > 0 or rc.error > 0 else 0
    import yaml

    failed = 0
    for f in _yaml_files(args.dir):
        if os.path.basename(f) != "test.yaml":
            continue
        d = os.path.dirname(f)
        spec = yaml.safe_load(open(f))
        pols = load_policies([os.path.join(d, p) for p in spec.get("policies", [])])
        ress = load_resources([os.path.join(d, r) for r in spec.get("resources", [])])
        rows = run_test(spec, pols, ress, args.device)
        print(f"\nExecuting {spec.get('name', d)}...")
        for i, r in enumerate(rows):
            verdict = {True: "Pass", False: "Fail", None: "routed to reference engine"}[r["ok"]]
            print(f"{i + 1:3d} {r['policy']:30s} {r['rule']:30s} {r['resource']:35s} {verdict}")
            failed += r["ok"] is False
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
