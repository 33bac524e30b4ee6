"""Seeded random policies and resources for differential parity (device vs oracle).

Patterns and resources are drawn from one small schema of Pod-like key paths so that most
pattern keys meet a resource value of some type: every anchor form (condition, global,
equality, existence, negation), the "*" shortcut, wildcard label keys, nested arrays, and leaf
patterns built from the operator language of pkg/engine/operator/operator.go (|, &, !, <, >,
<=, >=, ranges a-b / a!-b), globs, quantities, numbers, bools and nulls. Resources mix int64
and float64 numbers, quantity strings, absent keys, nulls and wrong container types.
"""
from __future__ import annotations

import random

KEYS_SCALAR = ["image", "name", "imagePullPolicy", "cpu", "memory", "port", "privileged", "level", "mode"]
KEYS_MAP = ["securityContext", "resources", "limits", "requests", "meta"]
KEYS_LIST = ["containers", "ports", "volumes", "add"]
STRINGS = ["it's", "a b", "nginx", "nginx:latest", "nginx:1.19", "gcr.io/app:v1", "a", "", "Always", "Never", "IfNotPresent",
           "100m", "1", "2", "0.5", "512Mi", "1Gi", "2Gi", "true", "false", "null", "-1", "1e3", "abc*",
           "*", "NET_ADMIN", "SYS_TIME", " ", "10", "0", "1.5", "ab?c", "Ki", "01"]
GLOBS = ["*", "?*", "*:*", "*:latest", "!*:latest", "nginx*", "gcr.io/*", "?", "a?c", "*a*", "", "**", "N*_*"]
OPS = ["", "!", "<", ">", "<=", ">=", "="]
QTY = ["100m", "1", "2", "0.5", "512Mi", "1Gi", "2Gi", "0", "-1", "1e3", "1k", "1Ki", "250m", "3"]


def _leaf_pattern(r: random.Random):
    c = r.random()
    if c < 0.30:
        return r.choice(GLOBS)
    if c < 0.50:
        return r.choice(OPS) + r.choice(QTY)
    if c < 0.58:
        a, b = r.choice(QTY), r.choice(QTY)
        return f"{a}{r.choice(['-', '!-'])}{b}"
    if c < 0.68:
        return " | ".join(r.choice(GLOBS + [o + q for o in OPS for q in QTY[:4]]) for _ in range(r.randint(2, 3)))
    if c < 0.72:
        return f"{r.choice(['>', '>='])}{r.choice(QTY)} & {r.choice(['<', '<='])}{r.choice(QTY)}"
    if c < 0.80:
        return r.choice([0, 1, 2, 0.5, -1, 100, 1.5, 1e3])
    if c < 0.88:
        return r.choice([True, False])
    if c < 0.92:
        return None
    return r.choice(STRINGS)


def _anchor(r: random.Random, k: str, allow: bool) -> str:
    if not allow:
        return k
    c = r.random()
    if c < 0.12:
        return f"({k})"
    if c < 0.17:
        return f"<({k})"
    if c < 0.25:
        return f"=({k})"
    if c < 0.30:
        return f"X({k})"
    return k


def pattern(r: random.Random, depth: int = 0):
    """A map pattern of depth <= 3."""
    m = {}
    for _ in range(r.randint(1, 3)):
        c = r.random()
        if depth < 3 and c < 0.30:
            k = r.choice(KEYS_MAP)
            m[_anchor(r, k, True)] = pattern(r, depth + 1)
        elif depth < 3 and c < 0.50:
            k = r.choice(KEYS_LIST)
            if r.random() < 0.15:
                m[f"^({k})"] = [pattern(r, depth + 1)]
            elif r.random() < 0.2:
                m[k] = [_leaf_pattern(r)]
            elif r.random() < 0.05:
                m[k] = []
            elif r.random() < 0.08:  # nested lists: positional compare, length check (validate.go:160-172)
                m[k] = [[pattern(r, depth + 1)] if r.random() < 0.5 else [_leaf_pattern(r)]
                        for _ in range(r.randint(1, 2))]
            else:
                m[_anchor(r, k, r.random() < 0.3)] = [pattern(r, depth + 1)]
        else:
            k = r.choice(KEYS_SCALAR)
            m[_anchor(r, k, True)] = "*" if r.random() < 0.06 else _leaf_pattern(r)
    # X(key) takes "null"-like patterns in practice; the value is ignored by the handler
    return m


def _leaf_value(r: random.Random):
    c = r.random()
    if c < 0.55:
        return r.choice(STRINGS)
    if c < 0.70:
        return r.choice([0, 1, 2, -1, 100, 8080, 1000])
    if c < 0.80:
        return r.choice([0.5, 1.5, 2.0, 1e3, -0.25, 1e21, 3.0])
    if c < 0.92:
        return r.choice([True, False])
    return None


def value(r: random.Random, depth: int = 0):
    m = {}
    for _ in range(r.randint(1, 5)):
        c = r.random()
        if depth < 3 and c < 0.30:
            m[r.choice(KEYS_MAP)] = value(r, depth + 1) if r.random() < 0.9 else _leaf_value(r)
        elif depth < 3 and c < 0.50:
            k = r.choice(KEYS_LIST)
            if r.random() < 0.2:
                m[k] = [_leaf_value(r) for _ in range(r.randint(0, 3))]
            elif r.random() < 0.1:
                m[k] = [[value(r, depth + 1)] if r.random() < 0.5 else [_leaf_value(r)]
                        for _ in range(r.randint(0, 3))]
            elif r.random() < 0.9:
                m[k] = [value(r, depth + 1) for _ in range(r.randint(0, 3))]
            else:
                m[k] = _leaf_value(r)
        else:
            m[r.choice(KEYS_SCALAR)] = _leaf_value(r)
    return m


def policies(seed: int, n_rules: int) -> list[dict]:
    r = random.Random(seed)
    rules = []
    for i in range(n_rules):
        v = {"message": f"fuzz rule {i}"} if r.random() < 0.5 else {}
        if r.random() < 0.12:
            v["anyPattern"] = [{"spec": pattern(r)} for _ in range(r.randint(2, 3))]
        else:
            p = {"spec": pattern(r)}
            if r.random() < 0.15:
                p["metadata"] = {"labels": {r.choice(["app", "a*", "tier", "*"]): r.choice(GLOBS)}}
            v["pattern"] = p
        rules.append({"name": f"fz-{i}", "match": {"resources": {"kinds": ["Pod"]}}, "validate": v})
    return [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": f"fuzz-{seed}"},
             "spec": {"rules": rules}}]


def resources(seed: int, n: int) -> list[dict]:
    r = random.Random(seed ^ 0x5EED)
    out = []
    for i in range(n):
        md = {"name": f"p{i}", "namespace": r.choice(["default", "prod", "dev"])}
        if r.random() < 0.7:
            md["labels"] = {k: r.choice(["web", "db", "x", ""]) for k in r.sample(["app", "tier", "owner", "ab"],
                                                                                   r.randint(0, 3))}
        out.append({"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": value(r)})
    return out
