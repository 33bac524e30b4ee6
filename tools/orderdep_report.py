#!/usr/bin/env python3
"""Order-dependence report: for each matched (policy rule, resource) pair
of the reference corpus and of a C4 sample, the oracle's enumerate mode collects every
(status, failing path) the reference can produce over its Go map iteration orders
(validate.go:110-135, validate/utils.go:37-51, wildcards.go:38-49). A pair is deterministic
with one outcome, order-dependent with more. Writes profiles/r02_orderdep.json.

    python tools/orderdep_report.py [--c4-resources 2000]
"""
import argparse
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from parity_util import load_gold  # noqa: E402


def survey(O, pols, ress, cap):
    cnt = collections.Counter()
    by_status = collections.Counter()
    examples = []
    for p in pols:
        for ri, r in enumerate(ress):
            for rule in O.enumerate(p, r, cap=cap):
                if rule["outcomes"] == [["nomatch", ""]]:
                    continue
                k = "truncated" if rule["truncated"] else (
                    "deterministic" if len(rule["outcomes"]) == 1 else "order_dependent")
                cnt[k] += 1
                if k == "order_dependent":
                    sts = sorted({s for s, _ in rule["outcomes"]})
                    by_status["status differs" if len(sts) > 1 else "path differs (" + sts[0] + ")"] += 1
                    if len(examples) < 5:
                        examples.append({"policy": p["metadata"]["name"], "rule": rule["name"], "resource": ri,
                                         "outcomes": rule["outcomes"]})
    n = sum(cnt.values())
    return {"pairs": n, **{k: cnt[k] for k in ("deterministic", "order_dependent", "truncated")},
            "deterministic_fraction": cnt["deterministic"] / n if n else None,
            "order_dependent_fraction": cnt["order_dependent"] / n if n else None,
            "order_dependent_kinds": dict(by_status), "examples": examples}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c4-resources", type=int, default=2000)
    ap.add_argument("--cap", type=int, default=4096)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_orderdep.json"))
    a = ap.parse_args()
    from kyverno_amd import batch, workloads

    O = oracle.Oracle()
    c = load_gold("corpus.json")[0]
    rep = {"method": "oracle enumerate mode (oracle/src/matcher.hpp Chooser), cap %d evaluations per pair" % a.cap,
           "corpus": survey(O, [p["policy"] for p in c["policies"]], [r["resource"] for r in c["resources"]], a.cap)}
    ress = [json.loads(x) for x in batch.synth(workloads.SEED + 4, a.c4_resources).decode().strip().split("\n")]
    rep["c4"] = survey(O, workloads.c4_policies(), ress, a.cap)
    rep["c4"]["resources"] = a.c4_resources
    with open(a.out, "w") as f:
        json.dump(rep, f, indent=1)
    print(json.dumps({k: {x: v[x] for x in ("pairs", "deterministic", "order_dependent", "truncated")}
                      for k, v in rep.items() if isinstance(v, dict)}))


if __name__ == "__main__":
    main()
