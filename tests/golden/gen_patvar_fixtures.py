#!/usr/bin/env python3
"""Generate the validate.pattern variable fixtures from the reference's own tests
(run where /root/reference exists):
    python tests/golden/gen_patvar_fixtures.py

Output patvars.json (data only: inputs + asserted outputs, each case citing its `src`):
  engine      pkg/engine/validation_test.go:1413-1819, the Test_VariableSubstitution* tests of
              pattern / anyPattern rules: policy, resource, asserted Rules[0] status and message.
  substitute  pkg/engine/variables/vars_test.go:616-925, the typed Test_Substitute* tests:
              pattern document, the shared variableObject resource, and the asserted value of
              spec.content after SubstituteAll (a JSON value; numbers as float64).
"""
from __future__ import annotations

import json
import os
import re
import sys

OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, OUT)

from gen_fixtures import functions, read  # noqa: E402

_STATUS = {"RuleStatusError": "error", "RuleStatusFail": "fail", "RuleStatusPass": "pass", "RuleStatusSkip": "skip"}


def _raw(body: str, name: str):
    m = re.search(name + r"\s*:=\s*\[\]byte\(`([^`]*)`\)", body)
    return json.loads(m.group(1)) if m else None


def gen_engine():
    rel = "pkg/engine/validation_test.go"
    src = read(rel)
    cases = []
    for name, body, line in functions(src):
        if not (1413 <= line < 1820) or not name.startswith("Test_VariableSubstitution"):
            continue
        res, pol = _raw(body, "resourceRaw"), _raw(body, "policyraw")
        st = re.search(r"Rules\[0\]\.Status, response\.(\w+)\)", body)
        msg = re.search(r'Rules\[0\]\.Message,\s*"((?:[^"\\]|\\.)*)"\)', body)
        if not (res and pol and st and msg):
            continue
        cases.append({"name": name, "src": f"{rel}:{line}", "policy": pol, "resource": res,
                      "status": _STATUS[st.group(1)], "message": json.loads('"' + msg.group(1) + '"')})
    return cases


def gen_substitute():
    rel = "pkg/engine/variables/vars_test.go"
    src = read(rel)
    vo = re.search(r"var variableObject = \[\]byte\(`([^`]*)`\)", src)
    obj = json.loads(vo.group(1))
    cases = []
    for name, body, line in functions(src):
        if not re.fullmatch(r"Test_Substitute(Null|Array|Int|Bool|String)(InString)?", name):
            continue
        pat = _raw(body, "patternRaw")
        m = re.search(r"expected := (.*)\n", body)
        if m is None and "var expected interface{}" in body:
            exp = None
        else:
            e = m.group(1).strip()
            r = re.fullmatch(r'resource\["(\w+)"\]', e)
            if r:
                exp = obj[r.group(1)]
            elif e.startswith("`") or e.startswith('"'):
                exp = e[1:-1] if e.startswith("`") else json.loads(e)
            else:
                exp = json.loads(e)
        if isinstance(exp, int) and not isinstance(exp, bool):
            exp = float(exp)  # the JSON context reads numbers back as float64
        cases.append({"name": name, "src": f"{rel}:{line}", "pattern": pat, "resource": obj,
                      "path": ["spec", "content"], "expected": exp})
    return cases


def main():
    out = {"engine": gen_engine(), "substitute": gen_substitute()}
    with open(os.path.join(OUT, "patvars.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"patvars.json: {len(out['engine'])} engine cases, {len(out['substitute'])} substitution cases")


if __name__ == "__main__":
    main()
