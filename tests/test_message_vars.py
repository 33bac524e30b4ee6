"""`{{request.object.*}}` variables in validate messages: host substitution vs oracle.

buildErrorMessage (pkg/engine/validation.go:510-532) runs variables.SubstituteAll on the message
with the resource as request.object (vars.go:319-398). The host (kyverno_amd/msgvars.py, used by
cli.rule_message) and the oracle (oracle/src/subst.cpp SubstituteMessage) restate it separately.
The reference's tests hold no known answer for a substituted validate message (the cases in
validation_test.go:1933-1992 are deny rules): parity unpinned beyond the oracle, and the
null / out-of-range-index results depend on kyverno's go-jmespath fork, which is absent.
"""
import json

import pytest

import oracle
from kyverno_amd import msgvars

RES = {
    "apiVersion": "v1", "kind": "Pod",
    "metadata": {"name": "web-0", "namespace": "prod",
                 "labels": {"app": "web", "app.kubernetes.io/name": "frontend"},
                 "annotations": {"note": "a<b & c>d"}},
    "spec": {"replicas": 3, "ratio": 0.5, "big": 1.5e22, "tiny": 2.5e-7, "huge": 12345678901234567890,
             "flag": True, "none": None, "neg": -0.0, "mid": 123456.789,
             "containers": [{"name": "c0", "image": "nginx:latest", "ports": [{"containerPort": 80}]},
                            {"name": "c1", "image": "redis", "env": {"b": 1, "a": "x\ty"}}]},
}

MESSAGES = [
    "plain message",
    "Pod {{request.object.metadata.name}} uses a latest tag",
    "{{request.object.metadata.name}}",
    "{{ request.object.metadata.namespace }}/{{request.object.metadata.name}}",
    "replicas={{request.object.spec.replicas}} ratio={{request.object.spec.ratio}}",
    "big={{request.object.spec.big}} tiny={{request.object.spec.tiny}} huge={{request.object.spec.huge}}",
    "neg={{request.object.spec.neg}} mid={{request.object.spec.mid}} flag={{request.object.spec.flag}}",
    "none={{request.object.spec.none}}",
    "labels {{request.object.metadata.labels}}",
    "ann {{request.object.metadata.annotations}}",
    "c {{request.object.spec.containers[1]}}",
    "first {{request.object.spec.containers[0].image}} last {{request.object.spec.containers[-1].name}}",
    'quoted {{request.object.metadata.labels."app.kubernetes.io/name"}}',
    "escaped \\{{request.object.metadata.name}} and {{request.object.kind}}",
    "escaped ref \\$(./x) ok",
    "{{request.object.kind}}{{request.object.metadata.name}}",
    "x{{request.object.spec.containers[0].ports[0].containerPort}}y",
    "twice {{request.object.kind}} {{request.object.kind}}",
    # a plain $() reference resolves to nil against the message string: the message comes back
    # unchanged, variables not substituted (vars.go:278-279, validation.go:519-522)
    "bad $(ref) {{request.object.kind}}",
    "$(./x) {{request.object.kind}} \\{{request.object.kind}}",
    # the reference panics on these (msgRaw.(string) of nil or a non-string)
    "missing {{request.object.metadata.nothere}}",
    "{{request.object.spec.replicas}}",
    "bad $(<x) {{request.object.kind}}",
    "bad $(>=) here",
]


@pytest.mark.parametrize("msg", MESSAGES)
def test_message_substitution_matches_oracle(msg):
    want = oracle.get().substitute_message(msg, RES)
    try:
        got = msgvars.substitute_message(msg, json.loads(json.dumps(RES)))
    except msgvars.MessageVariableError:
        got = None
    assert got == want


def test_message_substitution_known_forms():
    s = msgvars.substitute_message
    assert s("Pod {{request.object.metadata.name}} bad", RES) == "Pod web-0 bad"
    assert s("n={{request.object.spec.replicas}}", RES) == "n=3"
    assert s("{{request.object.spec.tiny}}|", RES) == "2.5e-7|"
    assert s("a {{request.object.metadata.annotations}}", RES) == 'a {"note":"a\\u003cb \\u0026 c\\u003ed"}'
    with pytest.raises(msgvars.MessageVariableError):
        s("{{request.object.spec.replicas}}", RES)


def test_message_reference_forms():
    """Message references (vars.go:253-309,450-475 on a string document): plain -> unchanged,
    empty path / operator -> the reference panics."""
    s = msgvars.substitute_message
    assert s("bad $(ref) {{request.object.kind}}", RES) == "bad $(ref) {{request.object.kind}}"
    assert s("x $(a/b) \\$(c) {{request.object.kind}}", RES) == "x $(a/b) \\$(c) {{request.object.kind}}"
    assert s("esc \\$(c) {{request.object.kind}}", RES) == "esc $(c) Pod"
    assert s("$() and $(<)", RES) == "$() and $(<)"  # no reference / a plain one
    for bad in ("bad $(<x) m", "$(!x)", "$(>=)", "$(1-2)"):
        with pytest.raises(msgvars.MessageVariableError):
            s(bad, RES)


def test_unsupported_jmespath_is_not_a_panic():
    """Projections / functions are valid JMESPath for the reference (ctx.Query); the host does not
    evaluate them and says so with a distinct exception, never the panic one."""
    for msg in ("images {{request.object.spec.containers[*].image}}",
                "n {{length(request.object.spec.containers)}}",
                "p {{request.object.spec.containers[0] | name}}"):
        with pytest.raises(msgvars.UnsupportedMessageVariable):
            msgvars.substitute_message(msg, RES)
        assert not issubclass(msgvars.UnsupportedMessageVariable, msgvars.MessageVariableError)


def _rand_value(rng, depth):
    k = rng.randrange(9 if depth < 3 else 6)
    if k == 0:
        return rng.choice(["", "a", "nginx:1.2", "x<y>&z", 'q"uote', "back\\slash", "tab\tnl\n", "ünï",
                           "{{brace}}", "$(ref)", " "])
    if k == 1:
        return rng.randrange(-10**6, 10**6)
    if k == 2:
        return rng.choice([0.5, -0.25, 1e-7, 3.0e21, 1e21, 123456.789, 1e-6, 9.999e20, 2.0**60, -0.0])
    if k == 3:
        return rng.choice([True, False])
    if k == 4:
        return None
    if k == 5:
        return rng.randrange(2**63, 2**64)  # float64 in the unstructured / encoding/json views
    if k in (6, 7):
        return {rng.choice(["a", "b", "name", "x.y", "Z", "k_1"]): _rand_value(rng, depth + 1)
                for _ in range(rng.randrange(4))}
    return [_rand_value(rng, depth + 1) for _ in range(rng.randrange(4))]


def _paths(v, prefix, out):
    out.append(prefix)
    if isinstance(v, dict):
        for k, x in v.items():
            seg = f'."{k}"' if not k.replace("_", "a").isalnum() or k[0].isdigit() else f".{k}"
            _paths(x, prefix + seg, out)
    elif isinstance(v, list):
        for i, x in enumerate(v):
            _paths(x, f"{prefix}[{i}]", out)
            _paths(x, f"{prefix}[{i - len(v)}]", out)


def test_message_substitution_fuzz_vs_oracle():
    """Seeded random resources x message templates (existing, missing and out-of-range paths,
    escapes, whole-message variables): host vs oracle, including where the reference panics."""
    import random

    rng = random.Random(0x6D736776)
    orc = oracle.get()
    n_sub = 0
    for case in range(400):
        res = {"kind": "Pod", "metadata": {"name": f"p{case}"}, "spec": _rand_value(rng, 0)}
        paths = []
        _paths(res, "request.object", paths)
        paths += ["request.object.nothere", "request.object.spec[7]", "request.object.metadata.name.x"]
        parts = []
        for _ in range(rng.randrange(1, 4)):
            p = rng.choice(paths)
            sp = rng.choice(["", " "])
            parts.append(rng.choice(["", "msg ", "\\", "x", "}"]) + "{{" + sp + p + sp + "}}")
        msg = rng.choice(["", "Pod: "]) + rng.choice([" ", "-", ""]).join(parts) + rng.choice(["", ".", " end"])
        want = orc.substitute_message(msg, json.dumps(res))
        try:
            got = msgvars.substitute_message(msg, json.loads(json.dumps(res)))
        except msgvars.MessageVariableError:
            got = None
        assert got == want, (msg, res)
        n_sub += got is not None
    assert n_sub > 100


def test_go_json_float_forms():
    """encoding/json floatEncoder (Go 1.16 encode.go:573-606): 'f' inside [1e-6, 1e21), else 'e'
    with a one-digit negative exponent; documented behaviour, no reference test holds it."""
    m = msgvars.go_json_marshal
    assert m(1e21) == "1e+21"
    assert m(1e20) == "100000000000000000000"
    assert m(1e-7) == "1e-7"
    assert m(0.000001) == "0.000001"
    assert m(123456789.0) == "123456789"
    assert m(3) == "3"
    assert m(-2.5) == "-2.5"
    assert m(1.5e-10) == "1.5e-10"
    assert m({"b": [1, None, True], "a": "<&>"}) == '{"a":"\\u003c\\u0026\\u003e","b":[1,null,true]}'
