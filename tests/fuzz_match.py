"""Seeded random match / exclude blocks x resources for differential parity (device vs oracle).

Covers MatchesResourceDescription (pkg/engine/utils.go:37-369): kinds in every form (Kind,
version/Kind, group/version/Kind, "*"), name / names / namespaces globs, annotation globs,
label selectors (matchLabels with wildcards, matchExpressions In / NotIn / Exists /
DoesNotExist), legacy blocks and any / all lists in match and exclude, against resources of
several kinds, API versions, namespaces (incl. cluster-scoped), labels and annotations.
"""
from __future__ import annotations

import random

KINDS = ["Pod", "Deployment", "Service", "ConfigMap", "Namespace"]
API = {"Pod": "v1", "Service": "v1", "ConfigMap": "v1", "Namespace": "v1", "Deployment": "apps/v1"}
KIND_FORMS = ["Pod", "Deployment", "Service", "ConfigMap", "*", "v1/Pod", "apps/v1/Deployment", "v1/Service",
              "apps/v1beta1/Deployment", "Namespace", "pod"]
NAMES = ["web-1", "web-2", "db-0", "cache", "ns-a", "prod", "x"]
NS = ["default", "prod", "dev", "kube-system", "team-a"]
NAME_GLOBS = ["web-*", "*", "db-?", "cache", "x*", "?", "*-1", "prod"]
NS_GLOBS = ["prod", "dev*", "*", "kube-*", "team-?", "default"]
LKEYS = ["app", "tier", "team", "env"]
LVALS = ["web", "db", "a", "prod", "dev", ""]


def _selector(r: random.Random) -> dict:
    sel = {}
    if r.random() < 0.7:
        sel["matchLabels"] = {r.choice(LKEYS + ["a*", "*"]): r.choice(LVALS[:-1] + ["*", "w*", "?b"])
                              for _ in range(r.randint(1, 2))}
    if r.random() < 0.5:
        exprs = []
        for _ in range(r.randint(1, 2)):
            op = r.choice(["In", "NotIn", "Exists", "DoesNotExist"])
            e = {"key": r.choice(LKEYS), "operator": op}
            if op in ("In", "NotIn"):
                e["values"] = r.sample(LVALS[:-1], r.randint(1, 2))
            exprs.append(e)
        sel["matchExpressions"] = exprs
    return sel


def _resource_filter(r: random.Random) -> dict:
    f = {}
    if r.random() < 0.85:
        f["kinds"] = r.sample(KIND_FORMS, r.randint(1, 2))
    if r.random() < 0.2:
        f["name"] = r.choice(NAME_GLOBS)
    if r.random() < 0.2:
        f["names"] = r.sample(NAME_GLOBS, r.randint(1, 2))
    if r.random() < 0.3:
        f["namespaces"] = r.sample(NS_GLOBS, r.randint(1, 2))
    if r.random() < 0.15:
        f["annotations"] = {r.choice(["owner", "team", "a/b"]): r.choice(["*", "x*", "me", "?"])}
    if r.random() < 0.3:
        f["selector"] = _selector(r)
    return f


def _user_info(r: random.Random, blk: dict) -> dict:
    """roles / clusterRoles / subjects of a block (checkUserInfo-style criteria, utils.go:319-336)."""
    c = r.random()
    if c < 0.06:
        blk["clusterRoles"] = [r.choice(["admin", "view"])]
    elif c < 0.10:
        blk["roles"] = [r.choice(["dev:editor", "prod:admin"])]
    elif c < 0.15:
        blk["subjects"] = [r.choice([{"kind": "User", "name": "alice"}, {"kind": "Group", "name": "devs"},
                                     {"kind": "ServiceAccount", "name": "sa", "namespace": "prod"}])]
    return blk


def _block(r: random.Random, must_have_kinds: bool) -> dict:
    c = r.random()
    if c < 0.6:
        rf = _resource_filter(r)
        if must_have_kinds and "kinds" not in rf:
            rf["kinds"] = [r.choice(KIND_FORMS)]
        return _user_info(r, {"resources": rf})
    key = "any" if c < 0.8 else "all"
    blocks = []
    for _ in range(r.randint(1, 3)):
        rf = _resource_filter(r)
        if must_have_kinds and "kinds" not in rf:
            rf["kinds"] = [r.choice(KIND_FORMS)]
        blocks.append(_user_info(r, {"resources": rf}))
    return {key: blocks}


def policies(seed: int, n_rules: int) -> list[dict]:
    r = random.Random(seed)
    rules = []
    for i in range(n_rules):
        rule = {"name": f"mx-{i}", "match": _block(r, True),
                "validate": {"pattern": {"metadata": {"name": r.choice(["?*", "web-*", "*-?"])}}}}
        if r.random() < 0.4:
            rule["exclude"] = _block(r, False)
        rules.append(rule)
    return [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": f"match-fuzz-{seed}"},
             "spec": {"rules": rules}}]


def resources(seed: int, n: int) -> list[dict]:
    r = random.Random(seed ^ 0xA11)
    out = []
    for i in range(n):
        kind = r.choice(KINDS)
        md = {"name": r.choice(NAMES)}
        if kind != "Namespace" and r.random() < 0.9:
            md["namespace"] = r.choice(NS)
        if r.random() < 0.8:
            md["labels"] = {k: r.choice(LVALS) for k in r.sample(LKEYS, r.randint(0, 3))}
        if r.random() < 0.4:
            md["annotations"] = {k: r.choice(["me", "xy", "", "other"]) for k in r.sample(["owner", "team", "a/b"],
                                                                                         r.randint(1, 2))}
        api = API[kind] if r.random() < 0.9 else ("apps/v1beta1" if kind == "Deployment" else "v2")
        out.append({"apiVersion": api, "kind": kind, "metadata": md, "spec": {}})
    return out
