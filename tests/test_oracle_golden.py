"""Pin the oracle (CPU restatement) against the reference's own known answers.

Fixtures come from tests/golden/gen_fixtures.py, which transcribes the Go
tests' inputs and asserted outputs (file:line in each case's `src`).
"""
import json
import os

import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)["cases"]


def _mode(v):
    return 0 if v["mode"] == "float" else 1


@pytest.mark.parametrize("case", load("comparator.json"), ids=lambda c: c["src"])
def test_comparator(orc, case):
    fn = case["fn"]
    if fn == "getNumberAndStringPartsFromPattern":
        assert list(orc.number_parts(case["pattern"])) == case["expect"]
        return
    if fn == "GetOperatorFromStringPattern":
        assert orc.operator(case["pattern"]) == case["expect"]
        return
    v = case["value"]
    kind = case["kind"]
    if kind in (1, 2, 3):
        got = orc.compare(kind, v["json"], case["pattern"], value_mode=_mode(v), op=case.get("op", ""))
    elif kind == 4:
        got = orc.compare(kind, v["json"], "null", value_mode=_mode(v))
    else:
        p = case["pattern"]
        got = orc.compare(kind, v["json"], p["json"], value_mode=_mode(v), pattern_mode=_mode(p))
    assert got == case["expect"], case


@pytest.mark.parametrize("case", load("syntax.json"), ids=lambda c: c["src"])
def test_syntax(orc, case):
    fn = case["fn"]
    if fn == "GetOperatorFromStringPattern":
        assert orc.operator(case["pattern"]) == case["expect"]
    elif fn == "RemoveAnchorsFromPath":
        assert orc.remove_anchors_from_path(case["arg"]) == case["expect"]
    else:
        assert orc.anchor_pred(fn, case["arg"]) == case["expect"]


@pytest.mark.parametrize("case", load("expand.json"), ids=lambda c: c["src"])
def test_expand_in_metadata(orc, case):
    # TestExpandInMetadata (wildcards_test.go:8-28): replaceWildcardsInMapKeys(pattern labels,
    # resource labels) must equal the expected map; reached through ExpandInMetadata on
    # metadata.labels (wildcards.go:69-107)
    pat = {"metadata": {"labels": case["pattern"]}}
    res = {"metadata": {"labels": case["resource"]}}
    got = orc.expand_in_metadata(pat, res)
    assert "panic" not in got, got
    assert got["metadata"]["labels"] == case["expect"], (got, case)


@pytest.mark.parametrize("case", load("matcher.json"), ids=lambda c: c["src"])
def test_matcher(orc, case):
    r = orc.match_pattern(case["resource"], case["pattern"], entry=case["entry"], res_mode=0, subst=case["subst"])
    assert "panic" not in r
    exp = case["expect"]
    assert r["set"] == exp["err"], r
    if "path" in exp:
        assert r["path"] == exp["path"], r
