"""Policy defaults and pod-controller rule generation ("autogen"), as the
reference CLI applies them before ``engine.Validate``.

``kyverno apply`` / ``kyverno test`` run every policy through
``common.MutatePolicy`` (pkg/kyverno/common/common.go:177-216), which applies the
JSON patches of ``policymutation.GenerateJSONPatchesForDefaults``
(pkg/policymutation/policymutation.go:25-91). The patches relevant to validate
rules are restated here on plain policy dicts:

* defaults: ``validationFailureAction`` "audit", ``background`` true,
  ``failurePolicy`` "Fail" (policymutation.go:258-340);
* pod-controller rules (``GeneratePodControllerRule``, :353-386;
  ``CanAutoGen``, :394-467; ``generateRulePatches``, :511-578;
  ``generateRuleForControllers``, :597-787; ``generateCronJobRule``,
  cronjob.go:15-164) including the textual ``request.object.spec`` rewrite of
  ``updateGenRuleByte`` (:496-508) and the message reference shift of
  ``variables.FindAndShiftReferences`` (pkg/engine/variables/vars.go:496-529);
* kind formatting (``checkForGVKFormatPatch``, :93-148, with its quirk of
  replacing a kinds list by only the kinds whose format changed).

Patches are computed from the original policy and applied in the reference's
order. Mutate-only conversions (overlay to strategic merge, patches to
JSON6902) do not change validate results and are not restated.
"""
from __future__ import annotations

import copy
import json
import re

POD_CONTROLLERS = "DaemonSet,Deployment,Job,StatefulSet,CronJob"  # pkg/engine/mutation.go:25
POD_CONTROLLERS_ANNOTATION = "pod-policies.kyverno.io/autogen-controllers"  # mutation.go:27
CRONJOB = "CronJob"

# variables.RegexReferences (pkg/engine/variables/vars.go:25)
_REGEX_REFERENCES = re.compile(r"^\$\(.[^\ ]*\)|[^\\]\$\(.[^\ ]*\)")


def _title(s: str) -> str:
    """Go strings.Title: upper-case the first letter of every word (ASCII)."""
    out, prev = [], " "
    for c in s:
        out.append(c.upper() if not (prev.isalnum() or prev == "_") else c)
        prev = c
    return "".join(out)


def get_kind_from_gvk(s: str) -> tuple[str, str]:
    """pkg/common/common.go:82-91"""
    n = s.count("/")
    if n == 0:
        return "", s
    parts = s.split("/")
    if n == 1:
        return parts[0], parts[1]
    return parts[0] + "/" + parts[1], parts[2]


def get_formated_kind(s: str) -> str:
    """pkg/common/common.go:212-221"""
    n = s.count("/")
    if n == 0:
        return _title(s)
    parts = s.split("/")
    if n == 1:
        return parts[0] + "/" + _title(parts[1])
    return parts[0] + "/" + parts[1] + "/" + _title(parts[2])


def contains_pod(kinds, element: str) -> bool:
    """pkg/utils/util.go:37-45"""
    return any(get_kind_from_gvk(k)[1] == element for k in (kinds or []))


def _kind_other_than_pod(kinds) -> bool:
    """policymutation.go:469-474"""
    return len(kinds or []) > 1 and contains_pod(kinds, "Pod")


def _rd(block: dict | None) -> dict:
    return (block or {}).get("resources") or {}


def _filters(block: dict | None, key: str) -> list:
    return list((block or {}).get(key) or [])


def _match_kinds(block: dict | None) -> list:
    """Rule.MatchKinds / ExcludeKinds (api/kyverno/v1/utils.go:106-128)"""
    kinds = list(_rd(block).get("kinds") or [])
    for f in _filters(block, "all"):
        kinds += list(_rd(f).get("kinds") or [])
    for f in _filters(block, "any"):
        kinds += list(_rd(f).get("kinds") or [])
    return kinds


def _has_name_selector(rd: dict) -> bool:
    return bool(rd.get("name")) or rd.get("selector") is not None or rd.get("annotations") is not None


def can_autogen(policy: dict) -> tuple[bool, str]:
    """CanAutoGen (policymutation.go:394-467)."""
    for rule in (policy.get("spec") or {}).get("rules") or []:
        match, exclude = rule.get("match") or {}, rule.get("exclude") or {}
        if _has_name_selector(_rd(match)) or _has_name_selector(_rd(exclude)):
            return False, "none"
        if _kind_other_than_pod(_rd(match).get("kinds")) or _kind_other_than_pod(_rd(exclude).get("kinds")):
            return False, "none"
        for blk in (match, exclude):
            for key in ("any", "all"):
                for f in _filters(blk, key):
                    rd = _rd(f)
                    if _kind_other_than_pod(rd.get("kinds")):
                        return False, "none"
                    if _has_name_selector(rd):
                        return False, "none"
        mut = rule.get("mutate") or {}
        val = rule.get("validate") or {}
        if mut.get("patches") is not None or mut.get("patchesJson6902") or val.get("deny") is not None or \
                rule.get("generate"):
            return False, "none"
    return True, POD_CONTROLLERS


def find_and_shift_references(value: str, shift: str, pivot: str) -> str:
    """variables.FindAndShiftReferences (pkg/engine/variables/vars.go:496-529)."""
    for reference in _REGEX_REFERENCES.findall(value):
        initial = reference[:2] == "$("
        old = reference
        if not initial:
            reference = reference[1:]
        index = reference.find(pivot)
        if pivot == "anyPattern":
            rule_index = reference[index + len(pivot) + 1:].split("/")[0]
            pivot = pivot + "/" + rule_index
        shifted = reference.replace(pivot, pivot + "/" + shift)
        replacement = "" if initial else old[0]
        replacement += shifted
        value = value.replace(old, replacement, 1)
    return value


def _non_empty_conditions(c) -> bool:
    if c is None:
        return False
    if isinstance(c, list):
        return len(c) > 0
    if isinstance(c, dict):
        return bool(c.get("any")) or bool(c.get("all"))
    return False


def _anyall_autogen(filters: list, controllers: str) -> list:
    """getAnyAllAutogenRule (policymutation.go:815-823)"""
    out = copy.deepcopy(filters)
    for i, f in enumerate(filters):
        if contains_pod(_rd(f).get("kinds"), "Pod"):
            out[i].setdefault("resources", {})["kinds"] = controllers.split(",")
    return out


def _cronjob_anyall(filters: list) -> list:
    """cronJobAnyAllAutogenRule (cronjob.go:188-196)"""
    out = copy.deepcopy(filters)
    for i, f in enumerate(filters):
        if contains_pod(_rd(f).get("kinds"), "Job"):
            out[i].setdefault("resources", {})["kinds"] = [CRONJOB]
    return out


def _is_empty_block(b) -> bool:
    if not b:
        return True
    return all(v in (None, "", [], {}) or (k == "resources" and _is_empty_block(v)) for k, v in b.items())


def generate_rule_for_controllers(rule: dict, controllers: str) -> dict | None:
    """generateRuleForControllers (policymutation.go:597-787); None == empty kyvernoRule."""
    name = rule.get("name", "")
    if name.startswith("autogen-") or controllers == "":
        return None
    match = rule.get("match") or {}
    exclude = rule.get("exclude") or {}
    mk, xk = _match_kinds(match), _match_kinds(exclude)
    if not contains_pod(mk, "Pod") or (len(xk) != 0 and not contains_pod(xk, "Pod")):
        return None
    skip = False
    validated = []
    if controllers == "all":
        skip = True
    elif controllers not in ("none", "all"):
        allowed = {"DaemonSet", "Deployment", "Job", "StatefulSet"}
        validated = [v for v in controllers.split(",") if v in allowed]
        skip = len(validated) > 0
    if skip:
        controllers = "DaemonSet,Deployment,Job,StatefulSet" if controllers == "all" else ",".join(validated)
    gname = "autogen-" + name
    if len(gname) > 63:
        gname = gname[:63]
    out = {"name": gname, "match": copy.deepcopy(match)}
    if rule.get("context"):
        out["context"] = copy.deepcopy(rule["context"])
    if _non_empty_conditions(rule.get("preconditions")):
        out["preconditions"] = copy.deepcopy(rule["preconditions"])
    if not _is_empty_block(exclude):
        out["exclude"] = copy.deepcopy(exclude)
    m = out["match"]
    if match.get("any"):
        m["any"] = _anyall_autogen(match["any"], controllers)
    elif match.get("all"):
        m["all"] = _anyall_autogen(match["all"], controllers)
    else:
        m.setdefault("resources", {})["kinds"] = controllers.split(",")
    if exclude.get("any"):
        out["exclude"]["any"] = _anyall_autogen(exclude["any"], controllers)
    elif exclude.get("all"):
        out["exclude"]["all"] = _anyall_autogen(exclude["all"], controllers)
    elif _rd(exclude).get("kinds"):
        out["exclude"].setdefault("resources", {})["kinds"] = controllers.split(",")
    mut = rule.get("mutate") or {}
    val = rule.get("validate") or {}
    if mut.get("overlay") is not None:
        out["mutate"] = {"patchStrategicMerge": {"spec": {"template": copy.deepcopy(mut["overlay"])}}}
        return out
    if mut.get("patchStrategicMerge") is not None:
        out["mutate"] = {"patchStrategicMerge": {"spec": {"template": copy.deepcopy(mut["patchStrategicMerge"])}}}
        return out
    if mut.get("foreach"):
        out["mutate"] = {"foreach": [
            {"list": f.get("list"), "preconditions": f.get("preconditions"),
             "patchStrategicMerge": {"spec": {"template": f.get("patchStrategicMerge")}}} for f in mut["foreach"]]}
        return out
    msg = val.get("message", "")
    if val.get("pattern") is not None:
        out["validate"] = {"message": find_and_shift_references(msg, "spec/template", "pattern"),
                           "pattern": {"spec": {"template": copy.deepcopy(val["pattern"])}}}
        return out
    if val.get("anyPattern") is not None:
        ap = val["anyPattern"] if isinstance(val["anyPattern"], list) else []
        out["validate"] = {"message": find_and_shift_references(msg, "spec/template", "anyPattern"),
                           "anyPattern": [{"spec": {"template": copy.deepcopy(p)}} for p in ap]}
        return out
    if val.get("foreach"):
        out["validate"] = {"message": find_and_shift_references(msg, "spec/template", "pattern"),
                           "foreach": copy.deepcopy(val["foreach"])}
        return out
    if rule.get("verifyImages") is not None:
        out["verifyImages"] = copy.deepcopy(rule["verifyImages"])
        return out
    return None


def generate_cronjob_rule(rule: dict, controllers: str) -> dict | None:
    """generateCronJobRule (cronjob.go:15-164)"""
    if CRONJOB not in controllers and "all" not in controllers:
        return None
    job = generate_rule_for_controllers(rule, "Job")
    if job is None:
        return None
    name = "autogen-cronjob-" + rule.get("name", "")
    if len(name) > 63:
        name = name[:63]
    job["name"] = name
    m = job["match"]
    if m.get("any"):
        m["any"] = _cronjob_anyall(m["any"])
    elif m.get("all"):
        m["all"] = _cronjob_anyall(m["all"])
    else:
        m.setdefault("resources", {})["kinds"] = [CRONJOB]
    x = job.get("exclude")
    if x is not None and x.get("any"):
        x["any"] = _cronjob_anyall(x["any"])
    elif x is not None and x.get("all"):
        x["all"] = _cronjob_anyall(x["all"])
    elif x is not None and _rd(x).get("kinds"):
        x.setdefault("resources", {})["kinds"] = [CRONJOB]
    mut = job.get("mutate")
    val = job.get("validate")
    msg = (rule.get("validate") or {}).get("message", "")
    if mut and mut.get("patchStrategicMerge") is not None:
        job["mutate"] = {"patchStrategicMerge": {"spec": {"jobTemplate": mut["patchStrategicMerge"]}}}
        return job
    if val and val.get("pattern") is not None:
        job["validate"] = {"message": find_and_shift_references(msg, "spec/jobTemplate/spec/template", "pattern"),
                           "pattern": {"spec": {"jobTemplate": val["pattern"]}}}
        return job
    if val and val.get("anyPattern") is not None:
        job["validate"] = {"message": find_and_shift_references(msg, "spec/jobTemplate/spec/template", "anyPattern"),
                           "anyPattern": [{"spec": {"jobTemplate": p}} for p in val["anyPattern"]]}
        return job
    if val and val.get("foreach"):
        job["validate"] = {"message": find_and_shift_references(msg, "spec/template", "pattern"),
                           "foreach": copy.deepcopy((rule.get("validate") or {}).get("foreach"))}
        return job
    if mut and mut.get("foreach"):
        job["mutate"] = {"foreach": [
            {"list": f.get("list"), "context": f.get("context"), "preconditions": f.get("preconditions"),
             "patchStrategicMerge": {"spec": {"jobTemplate": f.get("patchStrategicMerge")}}}
            for f in (rule.get("mutate") or {}).get("foreach")]}
        return job
    if job.get("verifyImages") is not None:
        return job
    return None


def _strip_cronjob(controllers: str) -> str:
    """stripCronJob (cronjob.go:166-184)"""
    out = [c for c in controllers.split(",") if c != CRONJOB]
    return ",".join(out)


def _rewrite(rule: dict, kind: str) -> dict:
    """updateGenRuleByte (policymutation.go:496-508): textual rewrite of the rule JSON."""
    s = json.dumps(rule, separators=(",", ":"), ensure_ascii=False)
    if kind == "Pod":
        s = s.replace("request.object.spec", "request.object.spec.template.spec")
    else:
        s = s.replace("request.object.spec", "request.object.spec.jobTemplate.spec.template.spec")
    s = s.replace("request.object.metadata", "request.object.spec.template.metadata")
    return json.loads(s)


def generate_rules(policy: dict, controllers: str) -> list[tuple[int, dict]]:
    """generateRulePatches (policymutation.go:511-578): [(position, rule)] to add or replace."""
    rules = (policy.get("spec") or {}).get("rules") or []
    insert = len(rules)
    by_name = {r.get("name"): i for i, r in enumerate(rules)}
    out = []
    for rule in rules:
        pos = insert
        for gen, kind in ((generate_rule_for_controllers(rule, _strip_cronjob(controllers)), "Pod"),
                          (generate_cronjob_rule(rule, controllers), "Cronjob")):
            if gen is None:
                continue
            gen = _rewrite(gen, kind)
            if gen["name"] in by_name:
                if rules[by_name[gen["name"]]] != gen:
                    out.append((by_name[gen["name"]], gen))
            else:
                out.append((pos, gen))
            insert += 1
            pos = insert
    return out


def mutate_policy(policy: dict) -> dict:
    """common.MutatePolicy: the policy as the CLI hands it to engine.Validate."""
    orig = policy
    p = copy.deepcopy(policy)
    spec = p.setdefault("spec", {})
    ospec = orig.get("spec") or {}
    if not ospec.get("validationFailureAction"):
        spec["validationFailureAction"] = "audit"
    if ospec.get("background") is None:
        spec["background"] = True
    if ospec.get("failurePolicy") is None:
        spec["failurePolicy"] = "Fail"
    # GeneratePodControllerRule (policymutation.go:353-386)
    apply_autogen, desired = can_autogen(orig)
    ann = (orig.get("metadata") or {}).get("annotations")
    actual = (ann or {}).get(POD_CONTROLLERS_ANNOTATION)
    if actual is None or not apply_autogen:
        actual = desired
        md = p.setdefault("metadata", {})
        if md.get("annotations") is None:
            md["annotations"] = {}
        md["annotations"][POD_CONTROLLERS_ANNOTATION] = actual
    rules = spec.setdefault("rules", spec.get("rules") or [])
    if actual != "none":
        for pos, gen in generate_rules(orig, actual):
            if pos < len(rules):
                rules[pos] = gen
            else:
                rules.append(gen)
    # checkForGVKFormatPatch (policymutation.go:93-148): replace by the changed kinds only
    for path, value in gvk_format_patches(orig):
        node = p
        for k in path[:-1]:
            node = node[k]
        node[path[-1]] = value
    return p


def gvk_format_patches(policy: dict) -> list[tuple[list, list]]:
    """checkForGVKFormatPatch / convertGVKForKinds (policymutation.go:93-148, :150-171): for every
    kinds list with at least one kind whose formatted form differs, a replace patch whose value is
    only the changed kinds (the reference's own quirk). Returns [(path as key list, value)]."""
    out = []

    def fmt(kinds):
        return [get_formated_kind(k) for k in kinds or [] if get_formated_kind(k) != k]

    for i, r in enumerate((policy.get("spec") or {}).get("rules") or []):
        for blk_key in ("match", "exclude"):
            blk = r.get(blk_key) or {}
            new = fmt(_rd(blk).get("kinds"))
            if new:
                out.append((["spec", "rules", i, blk_key, "resources", "kinds"], new))
            for key in ("all", "any"):
                for j, f in enumerate(_filters(blk, key)):
                    new = fmt(_rd(f).get("kinds"))
                    if new:
                        out.append((["spec", "rules", i, blk_key, key, j, "resources", "kinds"], new))
    return out


def mutate_policies(policies: list[dict]) -> list[dict]:
    """common.MutatePolices (pkg/kyverno/common/common.go:429-444)"""
    return [mutate_policy(p) for p in policies]
