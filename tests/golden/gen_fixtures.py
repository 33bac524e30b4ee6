#!/usr/bin/env python3
"""Generate golden fixtures from the reference's own Go tests.

Run in the build container (where /root/reference exists):
    python tests/golden/gen_fixtures.py

There is no Go toolchain in this image, so the reference's known-answer tests
cannot be executed. Instead this script reads the Go test sources as text,
evaluates the small subset of Go used by their straight-line bodies (literal
assignments, json.Unmarshal of raw byte strings, assert calls) and writes the
inputs and the asserted outputs as JSON data under tests/golden/. Every case
carries the `src` file:line of the assertion it came from. The fixtures are
data (inputs + expected outputs); no reference source text is stored.

Value typing follows the Go test: json.Unmarshal into interface{} gives
float64 numbers ("mode": "float"); Go literals keep their Go type (an untyped
integer constant passed as interface{} is `int`, encoded as a JSON integer
with "mode": "typed").
"""
from __future__ import annotations

import json
import os
import re
import sys

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

OPS = {
    "operator.Equal": "", "operator.MoreEqual": ">=", "operator.LessEqual": "<=", "operator.NotEqual": "!",
    "operator.More": ">", "operator.Less": "<", "operator.InRange": "-", "operator.NotInRange": "!-",
    "Equal": "", "MoreEqual": ">=", "LessEqual": "<=", "NotEqual": "!", "More": ">", "Less": "<",
    "InRange": "-", "NotInRange": "!-",
}


def read(rel):
    with open(os.path.join(REF, rel)) as f:
        return f.read()


def functions(src):
    """Yield (name, body, start_line) for each top-level func."""
    for m in re.finditer(r"^func (\w+)\(([^)]*)\)[^{]*\{", src, re.M):
        start = m.end()
        depth = 1
        i = start
        in_raw = in_str = False
        while i < len(src) and depth:
            c = src[i]
            if in_raw:
                if c == "`":
                    in_raw = False
            elif in_str:
                if c == "\\":
                    i += 1
                elif c == '"':
                    in_str = False
            else:
                if c == "`":
                    in_raw = True
                elif c == '"':
                    in_str = True
                elif c == "{":
                    depth += 1
                elif c == "}":
                    depth -= 1
            i += 1
        yield m.group(1), src[start:i - 1], src[:start].count("\n") + 1


class Go:
    """Evaluator for Go literal expressions used in the tests."""

    def __init__(self):
        self.env = {}

    def lit(self, s):
        s = s.strip()
        if s.startswith("[]byte(`") and s.endswith("`)"):
            return ("raw", s[8:-2])
        if s.startswith("`") and s.endswith("`"):
            return ("str", s[1:-1])
        if s.startswith('"'):
            return ("str", json.loads(s))
        if s in ("true", "false"):
            return ("bool", s == "true")
        if s == "nil":
            return ("nil", None)
        if re.fullmatch(r"-?\d+", s):
            return ("int", int(s))
        if re.fullmatch(r"-?(\d+\.\d*|\.\d+|\d+)([eE][-+]?\d+)?", s):
            return ("float", float(s))
        if s in OPS:
            return ("op", OPS[s])
        m = re.fullmatch(r"(\w+)\[\"([^\"]*)\"\]", s)
        if m:
            base = self.env[m.group(1)]
            assert base[0] == "json"
            return ("json", base[1].get(m.group(2)))
        if re.fullmatch(r"\w+", s) and s in self.env:
            return self.env[s]
        raise ValueError("cannot evaluate: " + s)


def split_args(s):
    out, depth, cur, i = [], 0, "", 0
    in_str = in_raw = False
    while i < len(s):
        c = s[i]
        if in_raw:
            cur += c
            if c == "`":
                in_raw = False
        elif in_str:
            cur += c
            if c == "\\":
                cur += s[i + 1]
                i += 1
            elif c == '"':
                in_str = False
        elif c == "`":
            in_raw = True
            cur += c
        elif c == '"':
            in_str = True
            cur += c
        elif c in "([{":
            depth += 1
            cur += c
        elif c in ")]}":
            depth -= 1
            cur += c
        elif c == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += c
        i += 1
    if cur.strip():
        out.append(cur.strip())
    return out


def statements(body, base_line):
    """Split a body into statements, keeping raw strings intact; yields (text, line)."""
    i, cur, line, start_line = 0, "", base_line, base_line
    depth = 0
    in_raw = in_str = False
    while i < len(body):
        c = body[i]
        if c == "\n":
            line += 1
        if in_raw:
            cur += c
            if c == "`":
                in_raw = False
        elif in_str:
            cur += c
            if c == "\\":
                cur += body[i + 1]
                i += 1
            elif c == '"':
                in_str = False
        elif c == "`":
            in_raw = True
            cur += c
        elif c == '"':
            in_str = True
            cur += c
        elif c in "([{":
            depth += 1
            cur += c
        elif c in ")]}":
            depth -= 1
            cur += c
        elif c == "\n" and depth == 0:
            if cur.strip():
                yield cur.strip(), start_line
            cur = ""
            start_line = line
        else:
            if not cur.strip():
                start_line = line
            cur += c
        i += 1
    if cur.strip():
        yield cur.strip(), start_line


def typed(v):
    """Go value -> fixture value {"json": <text>, "mode": "typed"|"float"}."""
    kind, val = v
    if kind == "json":
        return {"json": json.dumps(val), "mode": "float"}
    if kind == "int":
        return {"json": str(val), "mode": "typed"}
    if kind == "float":
        t = repr(float(val))
        if "e" not in t and "." not in t:
            t += ".0"
        return {"json": t, "mode": "typed"}
    if kind == "str":
        return {"json": json.dumps(val), "mode": "typed"}
    if kind == "bool":
        return {"json": "true" if val else "false", "mode": "typed"}
    if kind == "nil":
        return {"json": "null", "mode": "typed"}
    raise ValueError(kind)


# ----------------------------------------------------------------------------- comparator
CMP_FUNCS = {
    "ValidateValueWithPattern": 0, "validateValueWithStringPattern": 1, "validateNumberWithStr": 2,
    "validateString": 3, "validateValueWithNilPattern": 4, "validateValueWithFloatPattern": 5,
}


def gen_comparator():
    rel = "pkg/engine/validate/pattern_test.go"
    src = read(rel)
    cases = []
    for name, body, line0 in functions(src):
        g = Go()
        for st, line in statements(body, line0):
            m = re.fullmatch(r"(\w+)\s*:?=\s*(.+)", st, re.S)
            if m and not st.startswith("assert") and "json.Unmarshal" not in st and "getNumberAndStringParts" not in st \
                    and "," not in m.group(1):
                try:
                    g.env[m.group(1)] = g.lit(m.group(2))
                except ValueError:
                    pass
                continue
            m = re.search(r"json\.Unmarshal\((\w+),\s*&(\w+)\)", st)
            if m:
                g.env[m.group(2)] = ("json", json.loads(g.env[m.group(1)][1]))
                continue
            m = re.fullmatch(r"assert\.Assert\(t,\s*(!?)(\w+)\(log\.Log,\s*(.*)\)\)", st, re.S)
            if m and m.group(2) in CMP_FUNCS:
                args = split_args(m.group(3))
                fn = m.group(2)
                vals = [g.lit(a) for a in args]
                case = {"name": name, "src": f"{rel}:{line}", "fn": fn, "kind": CMP_FUNCS[fn],
                        "expect": m.group(1) != "!", "value": typed(vals[0])}
                if fn == "validateValueWithNilPattern":
                    case["pattern"] = None
                elif fn in ("validateValueWithStringPattern", "validateNumberWithStr", "validateString"):
                    case["pattern"] = vals[1][1]
                    if len(vals) > 2:
                        case["op"] = vals[2][1]
                else:
                    pv = typed(vals[1])
                    if fn == "validateValueWithFloatPattern":
                        pv = {"json": repr(float(json.loads(pv["json"]))), "mode": "float"}
                    case["pattern"] = pv
                cases.append(case)
                continue
            m = re.fullmatch(r"(\w+),\s*(\w+)\s*:=\s*getNumberAndStringPartsFromPattern\((\".*\")\)", st)
            if m:
                g.env["__np"] = json.loads(m.group(3))
                g.env["__npvars"] = (m.group(1), m.group(2))
                g.env["__npres"] = {}
                continue
            m = re.fullmatch(r"assert\.Equal\(t,\s*(\w+),\s*(\".*\")\)", st)
            if m and "__np" in g.env:
                a, b = g.env["__npvars"]
                g.env["__npres"][m.group(1)] = json.loads(m.group(2))
                if a in g.env["__npres"] and b in g.env["__npres"]:
                    cases.append({"name": name, "src": f"{rel}:{line}", "fn": "getNumberAndStringPartsFromPattern",
                                  "pattern": g.env["__np"],
                                  "expect": [g.env["__npres"][a], g.env["__npres"][b]]})
                continue
            m = re.fullmatch(r"assert\.Equal\(t,\s*operator\.GetOperatorFromStringPattern\((\".*\")\),\s*([\w.]+)\)", st)
            if m:
                cases.append({"name": name, "src": f"{rel}:{line}", "fn": "GetOperatorFromStringPattern",
                              "pattern": json.loads(m.group(1)), "expect": OPS[m.group(2)]})
    return cases


def gen_syntax():
    cases = []
    rel = "pkg/engine/operator/operator_test.go"
    for name, body, line0 in functions(read(rel)):
        for st, line in statements(body, line0):
            m = re.fullmatch(r"assert\.Equal\(t,\s*GetOperatorFromStringPattern\((\".*\")\),\s*(\w+)\)", st)
            if m:
                cases.append({"name": name, "src": f"{rel}:{line}", "fn": "GetOperatorFromStringPattern",
                              "pattern": json.loads(m.group(1)), "expect": OPS[m.group(2)]})
    rel = "pkg/engine/anchor/common/common_test.go"
    for name, body, line0 in functions(read(rel)):
        g = Go()
        for st, line in statements(body, line0):
            m = re.fullmatch(r"(\w+)\s*:=\s*(\".*\")", st)
            if m:
                g.env[m.group(1)] = ("str", json.loads(m.group(2)))
                continue
            m = re.fullmatch(r"assert\.Assert\(t,\s*(!?)(\w+)\((.+)\)\)", st)
            if m:
                arg = g.lit(m.group(3))[1]
                cases.append({"name": name, "src": f"{rel}:{line}", "fn": m.group(2), "arg": arg,
                              "expect": m.group(1) != "!"})
                continue
            m = re.fullmatch(r"(\w+)\s*:=\s*RemoveAnchorsFromPath\((\".*\")\)", st)
            if m:
                g.env["__rap"] = json.loads(m.group(2))
                continue
            m = re.fullmatch(r"assert\.Equal\(t,\s*\w+,\s*(\".*\")\)", st)
            if m and "__rap" in g.env:
                cases.append({"name": name, "src": f"{rel}:{line}", "fn": "RemoveAnchorsFromPath",
                              "arg": g.env["__rap"], "expect": json.loads(m.group(1))})
    return cases


def go_map_literal(s):
    """map[string]string{"a": "b", ...} -> dict"""
    m = re.fullmatch(r"map\[string\](?:string|interface\{\})\{(.*)\}", s.strip(), re.S)
    out = {}
    for kv in split_args(m.group(1)):
        k, v = kv.split(":", 1) if kv.count('":') == 0 else kv.split('":', 1)
        if not k.endswith('"'):
            k += '"'
        out[json.loads(k.strip())] = json.loads(v.strip())
    return out


def gen_expand():
    rel = "pkg/engine/wildcards/wildcards_test.go"
    cases = []
    for name, body, line0 in functions(read(rel)):
        for st, line in statements(body, line0):
            m = re.fullmatch(r"testExpand\(t,\s*(.*)\)", st, re.S)
            if m:
                a = split_args(m.group(1))
                cases.append({"name": name, "src": f"{rel}:{line}", "pattern": go_map_literal(a[0]),
                              "resource": go_map_literal(a[1]), "expect": go_map_literal(a[2])})
    return cases


# ----------------------------------------------------------------------------- matcher
def gen_matcher():
    rel = "pkg/engine/validate/validate_test.go"
    src = read(rel)
    cases = []
    for name, body, line0 in functions(src):
        if name in ("testValidationPattern", "testMatchPattern"):
            continue
        env = {}
        subst = False
        call = None
        expect = {}
        pending = None
        for st, line in statements(body, line0):
            m = re.fullmatch(r"(\w+)\s*:?=\s*\[\]byte\(`(.*)`\)", st, re.S)
            if m:
                env[m.group(1)] = m.group(2)
                continue
            m = re.search(r"json\.Unmarshal\((\w+),\s*&(\w+)\)", st)
            if m:
                env["__var_" + m.group(2)] = m.group(1)
                continue
            if "variables.SubstituteAll" in st:
                subst = True
                continue
            m = re.search(r"(validateMap|validateResourceElement)\(log\.Log,\s*(\w+),\s*(\w+)", st)
            if m:
                call = {"entry": 2 if m.group(1) == "validateMap" else 1,
                        "resource": env[env["__var_" + m.group(2)]], "pattern": env[env["__var_" + m.group(3)]],
                        "subst": subst, "src_line": line}
                expect = {}
                continue
            m = re.search(r"err\s*:?=\s*MatchPattern\(log\.Log,\s*(\w+),\s*(\w+)\)", st)
            if m and "testCase" not in st:
                call = {"entry": 0, "resource": env[env["__var_" + m.group(1)]],
                        "pattern": env[env["__var_" + m.group(2)]], "subst": subst, "src_line": line}
                expect = {}
                continue
            m = re.fullmatch(r"assert\.Equal\(t,\s*path,\s*(\".*\")\)", st)
            if m and call:
                expect["path"] = json.loads(m.group(1))
                continue
            if call and re.fullmatch(r"assert\.(NilError\(t,\s*err\)|Assert\(t,\s*err == nil\))", st):
                expect["err"] = False
                cases.append(dict(name=name, src=f"{rel}:{line}", mode="float", **call, expect=dict(expect)))
                call = None
                continue
            if call and re.fullmatch(r"assert\.Assert\(t,\s*err != nil\)", st):
                expect["err"] = True
                cases.append(dict(name=name, src=f"{rel}:{line}", mode="float", **call, expect=dict(expect)))
                call = None
                continue
            m = re.fullmatch(r"(pattern|resource)\s*=\s*\[\]byte\(`(.*)`\)", st, re.S)
            m2 = re.fullmatch(r"testValidationPattern\(t,\s*(.*)\)", st, re.S)
            if m2:
                a = split_args(m2.group(1))
                cases.append({"name": f"{name}#{json.loads(a[0])}", "src": f"{rel}:{line}", "mode": "float",
                              "entry": 1, "resource": env[a[2]], "pattern": env[a[1]], "subst": False,
                              "expect": {"path": json.loads(a[3]), "err": a[4] != "true"}})
                continue
            if st.startswith("testCases := []struct") or st.startswith("testCases := "):
                for tc in re.finditer(r"\{\s*name:\s*(\".*?\"),\s*pattern:\s*\[\]byte\(`(.*?)`\),\s*"
                                      r"resource:\s*\[\]byte\(`(.*?)`\),\s*nilErr:\s*(true|false),?\s*\}", st, re.S):
                    tline = line + st[:tc.start()].count("\n")
                    cases.append({"name": f"{name}#{json.loads(tc.group(1))}", "src": f"{rel}:{tline}",
                                  "mode": "float", "entry": 0, "resource": tc.group(3), "pattern": tc.group(2),
                                  "subst": False, "expect": {"err": tc.group(4) != "true"}})
    for c in cases:
        c.pop("src_line", None)
        # normalize JSON text
        c["resource"] = json.dumps(json.loads(c["resource"]))
        c["pattern"] = json.dumps(json.loads(c["pattern"]))
    return cases


def gen_corpus():
    """Reference policy/resource YAML corpus (SURVEY.md Appendix B 'corpus'),
    converted to JSON with the reference's YAML conventions (kyverno_amd.yamlio)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from kyverno_amd import yamlio

    pols, ress = [], []
    for d in ("test/best_practices", "test/more", "test/policy/validate"):
        for fn in sorted(os.listdir(os.path.join(REF, d))):
            if not fn.endswith((".yaml", ".yml")):
                continue
            try:
                for p in yamlio.load_policies_file(os.path.join(REF, d, fn)):
                    pols.append({"src": f"{d}/{fn}", "policy": yamlio.to_go_json_obj(p)})
            except Exception as e:  # malformed fixture files are skipped, as the CLI would reject them
                print(f"skip {d}/{fn}: {e}", file=sys.stderr)
    for fn in sorted(os.listdir(os.path.join(REF, "test/resources"))):
        if not fn.endswith((".yaml", ".yml")):
            continue
        try:
            for r in yamlio.load_resources_file(os.path.join(REF, "test/resources", fn)):
                ress.append({"src": f"test/resources/{fn}", "resource": yamlio.to_go_json_obj(r)})
        except Exception as e:
            print(f"skip test/resources/{fn}: {e}", file=sys.stderr)
    return [{"policies": pols, "resources": ress}]


def main():
    os.makedirs(OUT, exist_ok=True)
    outs = {
        "comparator.json": gen_comparator(),
        "syntax.json": gen_syntax(),
        "expand.json": gen_expand(),
        "matcher.json": gen_matcher(),
        "corpus.json": gen_corpus(),
    }
    for fn, cases in outs.items():
        with open(os.path.join(OUT, fn), "w") as f:
            json.dump({"generator": "tests/golden/gen_fixtures.py", "reference": "isabella232/kyverno v1.5.x",
                       "cases": cases}, f, indent=1, sort_keys=True)
        print(f"{fn}: {len(cases)} cases", file=sys.stderr)


if __name__ == "__main__":
    main()
