"""YAML -> JSON conversion with the reference's conventions.

The reference reads policies and resources with sigs.k8s.io/yaml v1.3.0
(go-yaml v2 underneath): YAMLToJSON, then encoding/json (policies, numbers
float64; `pkg/utils/loadpolicy.go:16-72`) or unstructured.UnmarshalJSON
(resources, int64 when the literal parses as int64; `pkg/kyverno/common/fetch.go:251-279`).
This module mirrors that on PyYAML:
  - YAML 1.1 booleans (yes/no/on/off/true/false) as go-yaml v2;
  - go-yaml floats accept exponent forms without a dot (1e3);
  - timestamps stay strings (no !!timestamp resolution);
  - non-string map keys become strings;
  - floats are re-emitted the way Go's json.Marshal writes float64, so an
    integral float (`1.0`) reaches the resource decoder as `1` (int64).
"""
from __future__ import annotations

import json
import math
import re
from decimal import Decimal

import yaml


class GoYamlLoader(yaml.SafeLoader):
    pass


# drop timestamp resolution, replace float resolution
GoYamlLoader.yaml_implicit_resolvers = {
    k: [(tag, rx) for tag, rx in v if tag not in ("tag:yaml.org,2002:timestamp", "tag:yaml.org,2002:float")]
    for k, v in yaml.SafeLoader.yaml_implicit_resolvers.copy().items()
}
GoYamlLoader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    re.compile(r"""^(?:[-+]?(?:\.[0-9]+|[0-9]+(?:\.[0-9]*)?)(?:[eE][-+]?[0-9]+)?
                |[-+]?\.(?:inf|Inf|INF)
                |\.(?:nan|NaN|NAN))$""", re.X),
    list("-+0123456789."),
)


def _construct_mapping(loader, node, deep=False):
    loader.flatten_mapping(node)
    out = {}
    for k_node, v_node in node.value:
        k = loader.construct_object(k_node, deep=deep)
        v = loader.construct_object(v_node, deep=deep)
        if not isinstance(k, str):
            if isinstance(k, bool):
                k = "true" if k else "false"
            elif isinstance(k, float):
                k = go_float(k)
            else:
                k = str(k)
        out[k] = v
    return out


GoYamlLoader.add_constructor("tag:yaml.org,2002:map", _construct_mapping)


def go_float(x: float) -> str:
    """encoding/json float64 formatting: strconv 'f' (shortest) for 1e-6<=|x|<1e21, else 'e'
    with "e-09" cleaned to "e-9"."""
    if math.isnan(x) or math.isinf(x):
        raise ValueError(f"unsupported float {x}")
    a = abs(x)
    if a == 0 or 1e-6 <= a < 1e21:
        s = format(Decimal(repr(x)).normalize(), "f")
        return "-0" if (a == 0 and math.copysign(1, x) < 0) else ("0" if a == 0 else s)
    r = repr(x)
    if len(r) >= 4 and r[-4] == "e" and r[-3] == "-" and r[-2] == "0":
        r = r[:-2] + r[-1]
    return r


def dumps_go(obj) -> str:
    """JSON text with Go float formatting (so integral floats become integers)."""
    if obj is None:
        return "null"
    if obj is True:
        return "true"
    if obj is False:
        return "false"
    if isinstance(obj, int):
        return str(obj)
    if isinstance(obj, float):
        return go_float(obj)
    if isinstance(obj, str):
        return json.dumps(obj, ensure_ascii=False)
    if isinstance(obj, dict):
        return "{" + ",".join(json.dumps(str(k), ensure_ascii=False) + ":" + dumps_go(v) for k, v in obj.items()) + "}"
    if isinstance(obj, (list, tuple)):
        return "[" + ",".join(dumps_go(v) for v in obj) + "]"
    return json.dumps(str(obj))


def load_documents(text: str) -> list:
    """All non-empty YAML documents of a file (pkg/utils/loadpolicy.go SplitDocuments)."""
    return [d for d in yaml.load_all(text, Loader=GoYamlLoader) if d is not None]


def to_go_json_obj(obj):
    """Round-trip through Go-style JSON text so numbers carry the reference's typing."""
    return json.loads(dumps_go(obj))


def load_policies_file(path: str) -> list[dict]:
    with open(path) as f:
        docs = load_documents(f.read())
    out = []
    for d in docs:
        if isinstance(d, dict) and d.get("kind") in ("ClusterPolicy", "Policy"):
            out.append(d)
    return out


def load_resources_file(path: str, default_namespace: str = "default") -> list[dict]:
    """pkg/kyverno/common/fetch.go:165-279: resources; empty namespace -> "default"."""
    with open(path) as f:
        docs = load_documents(f.read())
    out = []
    for d in docs:
        if not isinstance(d, dict):
            continue
        if d.get("kind") in ("ClusterPolicy", "Policy"):
            continue
        md = d.setdefault("metadata", {}) if isinstance(d.get("metadata", {}), dict) else d["metadata"]
        if isinstance(md, dict) and not md.get("namespace"):
            md["namespace"] = default_namespace
        out.append(d)
    return out
