"""CPU-only checks of the C ABI library: it loads, exports every symbol
declared in include/kvgpu.h, and its host stages (compile, ingest, synth)
behave. No kernel is launched here."""
import ctypes
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    with open(os.path.join(ROOT, "include", "kvgpu.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|void|double|const char\s*\*)\s*(kv_\w+)\s*\(", src, re.M)))


def test_library_exports_header_symbols():
    from kyverno_amd import _native

    L = _native.lib()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(_native.EXPORTED_SYMBOLS) == syms


def test_compile_routes():
    from kyverno_amd import batch

    pol = {"metadata": {"name": "p"}, "spec": {"rules": [
        {"name": "gpu", "match": {"resources": {"kinds": ["Pod"]}}, "validate": {"pattern": {"a": "b"}}},
        {"name": "vars", "match": {"resources": {"kinds": ["Pod"]}},
         "validate": {"pattern": {"a": "{{request.object.metadata.name}}"}}},
        {"name": "uservars", "match": {"resources": {"kinds": ["Pod"]}},
         "validate": {"pattern": {"a": "{{request.userInfo.username}}"}}},
        {"name": "keyvars", "match": {"resources": {"kinds": ["Pod"]}},
         "validate": {"pattern": {"{{request.object.kind}}": "x"}}},
        {"name": "deny", "match": {"resources": {"kinds": ["Pod"]}}, "validate": {"deny": {}}},
        {"name": "ctx", "context": [{"name": "x"}], "match": {"resources": {"kinds": ["Pod"]}},
         "validate": {"pattern": {"a": "b"}}},
        {"name": "mutate", "match": {"resources": {"kinds": ["Pod"]}}, "mutate": {"overlay": {}}},
        {"name": "badref", "match": {"resources": {"kinds": ["Pod"]}}, "validate": {"pattern": {"a": "$(./b)"}}},
        {"name": "anyempty", "match": {"resources": {"kinds": ["Pod"]}}, "validate": {"anyPattern": []}},
    ]}}
    ps = batch.PolicySet([pol])
    routes = {r.name: (r.route, r.route_reason) for r in ps.rules}
    assert routes["gpu"][0] == batch.ROUTE_GPU
    # request.object / @ variables are evaluated on the device (kvvars.cpp); other variables and
    # variables in keys stay with the reference engine
    assert routes["vars"] == (batch.ROUTE_GPU, "")
    assert routes["uservars"] == (batch.ROUTE_CPU, "variables")
    assert routes["keyvars"] == (batch.ROUTE_CPU, "variables")
    assert routes["deny"] == (batch.ROUTE_CPU, "deny")
    assert routes["ctx"] == (batch.ROUTE_CPU, "context")
    assert routes["mutate"][0] == batch.ROUTE_NORESPONSE
    assert routes["badref"][0] == batch.ROUTE_CONSTANT
    badref = [r for r in ps.rules if r.name == "badref"][0]
    assert badref.const_status == batch.ERROR and badref.const_message.startswith("variable substitution failed")
    anyempty = [r for r in ps.rules if r.name == "anyempty"][0]
    assert anyempty.const_status == batch.PASS


def test_substitution_matches_oracle(orc):
    """$() references are resolved once at compile time; the oracle resolves per
    pair. Compare the error text of unresolvable references."""
    from kyverno_amd import batch

    pat = {"spec": {"containers": [{"resources": {"requests": {"memory": "$(<=./../../lim(its/mem)ory)"},
                                                  "lim(its": {"mem)ory": "2048Mi"}}}]}}
    pol = {"metadata": {"name": "p"}, "spec": {"rules": [{"name": "r", "match": {"resources": {"kinds": ["Pod"]}},
                                                          "validate": {"pattern": pat}}]}}
    ps = batch.PolicySet([pol])
    assert ps.rules[0].route == batch.ROUTE_GPU
    bad = {"spec": {"a": "$(./missing)"}}
    pol2 = {"metadata": {"name": "p"}, "spec": {"rules": [{"name": "r", "match": {"resources": {"kinds": ["Pod"]}},
                                                           "validate": {"pattern": bad}}]}}
    ps2 = batch.PolicySet([pol2])
    o = orc.validate(pol2, {"kind": "Pod", "metadata": {"name": "x"}})
    assert o["rules"][0]["status"] == "error"
    assert o["rules"][0]["message"] == ps2.rules[0].const_message


def test_ingest_and_synth():
    from kyverno_amd import batch, workloads

    ps = batch.PolicySet(workloads.c2_policies())
    assert ps.n_rules == 100 and all(r.route == batch.ROUTE_GPU for r in ps.rules)
    data = batch.synth(workloads.SEED, 500)
    assert data.count(b"\n") == 500
    b = batch.Batch(ps, data)
    assert b.n_res == 500 and b.store_bytes > 0
    # same seed -> same bytes
    assert batch.synth(workloads.SEED, 500) == data
    # JSON array input is accepted as well as NDJSON
    arr = "[" + ",".join(data.decode().strip().split("\n")) + "]"
    b2 = batch.Batch(ps, arr)
    assert b2.n_res == 500


def test_ingest_rejects_malformed():
    from kyverno_amd import batch
    from kyverno_amd._native import KvError

    ps = batch.PolicySet([{"metadata": {"name": "p"}, "spec": {"rules": []}}])
    with pytest.raises(KvError):
        batch.Batch(ps, b'{"kind": "Pod", ')
    with pytest.raises(KvError):
        batch.PolicySet(b"[{]")


def test_parallel_ingest_host_tables():
    """Serial and multi-threaded ingest agree on resource count and the first-seen namespace order."""
    import os

    from kyverno_amd import batch, workloads

    ps = batch.PolicySet(workloads.c2_policies())
    data = batch.synth(workloads.SEED + 3, 6000, kind_mix=1)
    got = []
    for t in ("1", "4"):
        os.environ["KVGPU_INGEST_THREADS"] = t
        try:
            b = batch.Batch(ps, data)
        finally:
            os.environ.pop("KVGPU_INGEST_THREADS", None)
        got.append((b.n_res, b.namespaces))
    assert got[0] == got[1] and got[0][0] == 6000


def test_duplicate_json_keys_last_wins():
    """encoding/json (unstructured.UnmarshalJSON) keeps the last of duplicate object keys; the
    decoder's signature filter must still find every duplicate (same length, first and last
    byte) and ignore keys that only share a signature bit."""
    from kyverno_amd import batch

    ps = batch.PolicySet([{"metadata": {"name": "p"}, "spec": {"rules": []}}])
    docs = [
        b'{"kind": "Pod", "metadata": {"namespace": "a", "name": "x", "namespace": "b"}}',
        b'{"kind": "Pod", "metadata": {"namespace": "c", "labels": {"k1": "v", "k2": "w", "k1": "z"}}}',
        b'{"kind": "Pod", "metadata": {"namespace": "a", "ab": 1, "ba": 2, "aab": 3}}',
    ]
    b = batch.Batch(ps, b"\n".join(docs))
    assert b.n_res == 3
    assert sorted(b.namespaces) == ["a", "b", "c"]  # doc 0's namespace is "b", not "a"
