"""Benchmark / parity workloads (BASELINE.json configs).

C2: 1M synthetic Pods x 100 validate.pattern rules (40 image-glob rules,
    20 existence `?*` rules, 30 quantity rules incl. ranges, 10 `|`-list rules).
C3: Pods/Deployments/Services x policies with kinds / namespace globs /
    matchLabels wildcards / matchExpressions / exclude blocks.
Synthetic resources come from the library's deterministic generator
(``kv_synth``, seed 0x6B79766E + shard index).
"""
from __future__ import annotations

import json
import os

SEED = 0x6B79766E


def _policy(name: str, rules: list, annotations: dict | None = None) -> dict:
    md = {"name": name}
    if annotations:
        md["annotations"] = annotations
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": md,
            "spec": {"validationFailureAction": "audit", "background": True, "rules": rules}}


def _rule(name: str, pattern=None, any_pattern=None, kinds=("Pod",), message: str | None = None, match=None,
          exclude=None) -> dict:
    v = {}
    if message:
        v["message"] = message
    if pattern is not None:
        v["pattern"] = pattern
    if any_pattern is not None:
        v["anyPattern"] = any_pattern
    r = {"name": name, "match": match or {"resources": {"kinds": list(kinds)}}, "validate": v}
    if exclude:
        r["exclude"] = exclude
    return r


IMAGE_GLOBS = [
    "*:*", "!*:latest", "registry.local:5000/*", "*@sha256:* | !*:latest", "docker.io/*", "gcr.io/* | quay.io/*",
    "!*:v0.*", "*:v?.*.*", "!docker.io/*:latest", "*nginx*", "!*redis*:latest", "*/app-*", "?*", "*:v1.*|*:v2.*",
    "!registry.local:5000/*:latest", "*.io/*",
    "!*@sha256:*", "*:v3.1?.*", "!gcr.io/busybox*", "*-1?:*",
]


def c2_policies() -> list[dict]:
    rules = []
    # 40 image-glob rules: containers[] and initContainers[] (condition-anchored on presence)
    for i, g in enumerate(IMAGE_GLOBS):
        rules.append(_rule(f"image-{i:02d}", {"spec": {"containers": [{"image": g}]}},
                           message=f"image must match {g}"))
    for i, g in enumerate(IMAGE_GLOBS):
        rules.append(_rule(f"init-image-{i:02d}", {"spec": {"=(initContainers)": [{"image": g}]}}))
    # 20 existence rules
    ex_fields = [
        ("name",), ("image",), ("resources", "requests", "memory"), ("resources", "requests", "cpu"),
        ("resources", "limits", "memory"), ("resources", "limits", "cpu"), ("imagePullPolicy",),
        ("securityContext", "runAsNonRoot"), ("securityContext", "allowPrivilegeEscalation"),
        ("securityContext", "seccompProfile", "type"),
    ]

    def nest(path, leaf):
        d = leaf
        for p in reversed(path):
            d = {p: d}
        return d

    for i, f in enumerate(ex_fields):
        rules.append(_rule(f"exists-{i:02d}", {"spec": {"containers": [nest(f, "?*")]}}))
    for i, lab in enumerate(["app", "owner", "tier"]):
        rules.append(_rule(f"label-{lab}", {"metadata": {"labels": {lab: "?*"}}}))
    rules.append(_rule("label-wild", {"metadata": {"labels": {"a*": "?*"}}}))
    rules.append(_rule("name-cond", {"spec": {"containers": [{"(name)": "c*", "image": "?*:?*"}]}}))
    rules.append(_rule("ports-exist", {"spec": {"containers": [{"=(ports)": [{"containerPort": "*"}]}]}}))
    rules.append(_rule("namespace-set", {"metadata": {"namespace": "ns-*"}}))
    rules.append(_rule("no-hostpath", {"spec": {"=(volumes)": [{"X(hostPath)": "null"}]}}))
    rules.append(_rule("volumes-any", {"spec": {"^(volumes)": [{"name": "data"}]}}))
    rules.append(_rule("restricted-host", {"spec": {"=(hostNetwork)": False, "=(hostPID)": False}}))
    # 30 quantity rules
    q = [
        ("limits", "memory", "<=2Gi"), ("limits", "memory", "<=4Gi"), ("limits", "memory", ">=128Mi"),
        ("limits", "memory", "256Mi-2Gi"), ("limits", "memory", "!256Mi"), ("limits", "memory", "1Gi!-3Gi"),
        ("requests", "memory", "<=1Gi"), ("requests", "memory", ">64Mi"), ("requests", "memory", "64Mi-1Gi"),
        ("requests", "memory", "<512Mi | >1Gi"), ("requests", "cpu", ">0"), ("requests", "cpu", "<=1"),
        ("requests", "cpu", "100m-2"), ("requests", "cpu", "0!-100m"), ("requests", "cpu", ">=250m"),
        ("requests", "cpu", "<2 & >100m"), ("limits", "cpu", "<=2"), ("limits", "cpu", ">=200m"),
        ("limits", "cpu", "200m-4"), ("limits", "cpu", "!1"), ("limits", "cpu", "1!-3"),
        ("requests", "cpu", "0.5"), ("requests", "cpu", "<=500m"), ("limits", "memory", "<1Ti"),
        ("requests", "memory", "!64Mi"), ("limits", "cpu", ">0.1"), ("requests", "cpu", "1-1"),
        ("limits", "memory", "2Gi"), ("requests", "memory", ">= 100Mi"), ("limits", "cpu", "<=4"),
    ]
    for i, (grp, res, pat) in enumerate(q):
        rules.append(_rule(f"quantity-{i:02d}",
                           {"spec": {"containers": [{"=(resources)": {f"=({grp})": {f"=({res})": pat}}}]}}))
    # 10 |-list rules
    ors = [
        ("imagePullPolicy", "Always | IfNotPresent"), ("imagePullPolicy", "!Never"),
        ("imagePullPolicy", "IfNotPresent|Never"), ("name", "c0 | c1 | c2"), ("name", "!c3"),
    ]
    for i, (k, pat) in enumerate(ors):
        rules.append(_rule(f"or-{i:02d}", {"spec": {"containers": [{f"=({k})": pat}]}}))
    for i, (lab, pat) in enumerate([("tier", "frontend|backend"), ("app", "web|api|db"), ("owner", "team-*|platform"),
                                    ("tier", "!data"), ("app", "*e*|*a*")]):
        rules.append(_rule(f"or-label-{i:02d}", {"metadata": {"=(labels)": {f"=({lab})": pat}}}))
    assert len(rules) == 100, len(rules)
    return [_policy("c2-pod-rules", rules)]


C3_KIND_MIX = 2  # kv_synth stream of C3: Pods/Deployments/Services 60/25/15 over 1 000 namespaces
C3_NAMESPACES = 1000


def c3_policies(n_policies: int = 1000, seed: int = SEED) -> list[dict]:
    """Policies with 1-3 rules and varied match/exclude blocks (C3), namespace globs and
    excludes over the C3 stream's 1 000 namespaces (``ns-0`` .. ``ns-999``)."""
    import random

    rnd = random.Random(seed)
    kinds = [["Pod"], ["Deployment"], ["Service"], ["*"], ["Pod", "Deployment"], ["apps/v1/Deployment"], ["v1/Pod"]]
    pats_pod = [{"spec": {"containers": [{"image": g}]}} for g in IMAGE_GLOBS[:8]]
    pats_dep = [{"spec": {"template": {"spec": {"containers": [{"image": g}]}}}} for g in IMAGE_GLOBS[:8]]
    pats_svc = [{"spec": {"type": "ClusterIP | NodePort"}}, {"spec": {"type": "!LoadBalancer"}},
                {"spec": {"ports": [{"port": "<1024 | >8000"}]}}]
    pols = []
    for p in range(n_policies):
        rules = []
        for r in range(1 + rnd.randrange(3)):
            k = rnd.choice(kinds)
            res = {"kinds": k}
            roll = rnd.random()
            if roll < 0.3:
                res["namespaces"] = [f"ns-{rnd.randrange(C3_NAMESPACES)}*"]
            elif roll < 0.5:
                res["selector"] = {"matchLabels": {"app": rnd.choice(["web", "api", "*", "d?"])}}
            elif roll < 0.6:
                res["selector"] = {"matchExpressions": [
                    {"key": "tier", "operator": rnd.choice(["In", "NotIn"]), "values": ["frontend", "data"]}]}
            elif roll < 0.65:
                res["selector"] = {"matchExpressions": [{"key": "owner", "operator": rnd.choice(["Exists",
                                                                                              "DoesNotExist"])}]}
            match = {"resources": res}
            if rnd.random() < 0.2:
                match = {"any": [{"resources": res}, {"resources": {"kinds": ["Service"]}}]}
            exclude = None
            if rnd.random() < 0.25:
                exclude = {"resources": {"namespaces": [f"ns-{rnd.randrange(C3_NAMESPACES)}"]}}
            if "Service" in k:
                pat = rnd.choice(pats_svc)
            elif "Deployment" in k or "apps/v1/Deployment" in k:
                pat = rnd.choice(pats_dep)
            else:
                pat = rnd.choice(pats_pod)
            rules.append(_rule(f"p{p}-r{r}", pat, match=match, exclude=exclude))
        pols.append(_policy(f"c3-policy-{p:04d}", rules))
    return pols


def name_filter_policy() -> dict:
    """Rules whose match / exclude reads the resource name (`name`, `names` globs; evaluated per
    resource behind the match-tuple bit), mixed with namespace / selector / any blocks, for the
    C3 stream (pkg/engine/utils.go:129-229)."""
    pat = {"metadata": {"name": "?*"}}
    rules = [
        _rule("name-pod", pat, match={"resources": {"kinds": ["Pod"], "name": "pod-1*"}}),
        _rule("names-any", pat, match={"any": [{"resources": {"kinds": ["Deployment"], "names": ["*-2?", "dep-3*"]}},
                                                {"resources": {"kinds": ["Service"], "namespaces": ["ns-1*"]}}]}),
        _rule("exclude-name", pat, match={"resources": {"kinds": ["*"]}}, exclude={"resources": {"name": "*-7*"}}),
        _rule("exclude-names-ns", pat, match={"resources": {"kinds": ["Pod", "Service"],
                                                             "selector": {"matchLabels": {"app": "*"}}}},
              exclude={"any": [{"resources": {"names": ["pod-9*", "svc-8*"]}},
                               {"resources": {"namespaces": ["ns-5*"]}}]}),
        _rule("plain", pat, match={"resources": {"kinds": ["Pod"], "namespaces": ["ns-2*"]}}),
    ]
    return _policy("names", rules)


_GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def chart_policies() -> list[dict]:
    """The kyverno-policies chart (charts/kyverno-policies/templates/**) rendered with
    podSecurityStandard=restricted: 14 policies / 35 rules, anchor-heavy (conditional, equality,
    existence, negation anchors over containers[] arrays). Rendered by
    tests/golden/gen_cli_fixtures.py into tests/golden/chart.json."""
    with open(os.path.join(_GOLDEN, "chart.json")) as f:
        return [c["policy"] for c in json.load(f)["cases"]]


def validate_corpus_policies() -> list[dict]:
    """test/policy/validate/*.yaml policies of the reference (tests/golden/corpus.json)."""
    with open(os.path.join(_GOLDEN, "corpus.json")) as f:
        pols = json.load(f)["cases"][0]["policies"]
    return [p["policy"] for p in pols if p["src"].startswith("test/policy/validate/")]


# Rules whose outcome on the synthetic Pods spreads over PASS / FAIL / ERROR / SKIP, so the
# benchmark streams exercise every status at scale (validation.go:421-444 status mapping,
# validate.go:29-50 MatchPattern skip / missing-anchor forms, anchorKey.go:11-145):
#   a conditional anchor that mismatches on most Pods (SKIP; ERROR where the label is absent),
#   a negation anchor under a condition (SKIP / FAIL / ERROR), a condition anchor next to a plain
#   key (missing anchor key -> ERROR), a global anchor inside containers[] (SKIP).
STATUS_FORM_RULES = {
    "cond-tier-image": {"metadata": {"labels": {"(tier)": "frontend"}}, "spec": {"containers": [{"image": "*:v1.*"}]}},
    "cond-app-no-hostnet": {"metadata": {"labels": {"(app)": "web"}}, "spec": {"X(hostNetwork)": "null"}},
    "cond-owner-app": {"metadata": {"labels": {"(owner)": "team-*", "app": "api"}}},
    "global-latest-always": {"spec": {"containers": [{"<(image)": "*:latest", "imagePullPolicy": "Always"}]}},
}


def status_form_policy() -> dict:
    """One policy of the STATUS_FORM_RULES (no autogen: pod-policies.kyverno.io/autogen-controllers none)."""
    return _policy("status-forms", [_rule(k, v) for k, v in STATUS_FORM_RULES.items()],
                   annotations={"pod-policies.kyverno.io/autogen-controllers": "none"})


def c4_policies() -> list[dict]:
    """C4: anchor-heavy set = chart + test/policy/validate, after the CLI's defaults + autogen
    (pkg/kyverno/common/common.go:177-216): 138 rules, every one device-routed, plus the 4
    STATUS_FORM_RULES (SKIP / ERROR at scale): 142 rules."""
    from . import autogen

    return autogen.mutate_policies(chart_policies() + validate_corpus_policies() + [status_form_policy()])


def c5_policies() -> list[dict]:
    """C5 background scan: the full chart after autogen (35 + 70 = 105 rules)."""
    from . import autogen

    return autogen.mutate_policies(chart_policies())
