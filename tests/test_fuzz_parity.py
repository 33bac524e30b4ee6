"""Differential parity on seeded random policies x resources (tests/fuzz_gen.py): per-pair status,
failing path and RuleResponse message of both device engines against the oracle.

The generator covers every anchor form, the "*" shortcut, wildcard label keys, scalar lists,
empty pattern lists, the operator language and typed leaves, against resources that mix int64 /
float64 / quantity strings / nulls / wrong container types — shapes the reference's fixtures only
touch one at a time. CPU tests pin the generator's reach through the oracle alone.
"""
import json

import numpy as np
import pytest

import fuzz_gen
import fuzz_match
from parity_util import compare, oracle_status

SEEDS = list(range(8))
N_RULES, N_RES = 60, 300


@pytest.fixture(scope="module")
def orc():
    import oracle

    return oracle.get()


def test_fuzz_generator_reach(orc):
    """Every status of the path is produced, and every rule is GPU-routed (no CPU escape hatch)."""
    from kyverno_amd import batch

    seen = set()
    for seed in SEEDS[:3]:
        pols, ress = fuzz_gen.policies(seed, N_RULES), fuzz_gen.resources(seed, N_RES)
        ps = batch.PolicySet(pols)
        assert all(r.route == batch.ROUTE_GPU for r in ps.rules)
        seen |= set(np.unique(oracle_status(orc, pols, ress)).tolist())
    assert {0, 1, 3, 4} <= seen, seen


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [False, True], ids=["vm", "specialized"])
@pytest.mark.parametrize("seed", SEEDS)
def test_fuzz_status_and_paths(orc, seed, spec):
    pols, ress = fuzz_gen.policies(seed, N_RULES), fuzz_gen.resources(seed, N_RES)
    mism, r, ost = compare(orc, pols, ress, check_paths=True, max_path_checks=300, specialize=spec)
    assert not mism, f"seed {seed}: " + "\n".join(mism[:20])


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [False, True], ids=["vm", "specialized"])
@pytest.mark.parametrize("seed", SEEDS[:4])
def test_fuzz_messages(orc, seed, spec):
    """Messages of a sample of pairs of every status (skip / error carry the rendered error form)."""
    from kyverno_amd import cli

    pols, ress = fuzz_gen.policies(seed, N_RULES), fuzz_gen.resources(seed, N_RES)
    ev = cli.evaluate(pols, ress, specialize=spec)
    rng = np.random.default_rng(seed)
    pairs = []
    for st in (cli.PASS, cli.FAIL, cli.ERROR, cli.SKIP):
        idx = np.argwhere(ev.status == st)
        if len(idx):
            pairs += [tuple(x) for x in idx[rng.choice(len(idx), min(60, len(idx)), replace=False)]]
    bad = []
    for rule, res in pairs:
        rr = orc.validate(pols[0], ress[res])["rules"][rule]
        got = cli.rule_message(ev, ev.rules[rule], int(res))
        if got != rr["message"]:
            bad.append(f"rule {rule} res {res} [{rr['status']}]\n  device {got!r}\n  oracle {rr['message']!r}\n"
                       f"  pattern {json.dumps(pols[0]['spec']['rules'][rule]['validate'])[:300]}")
    assert not bad, f"seed {seed}: {len(bad)} of {len(pairs)} differ\n" + "\n".join(bad[:10])


# admission info of the batch: none (background scan / CLI), or a request by a cluster admin, a
# namespaced role holder, or a service account (folded on the host, validation.go:383-398)
ADMISSIONS = [None,
              {"admission": {"clusterRoles": ["admin"], "groups": [], "roles": [], "username": ""}},
              {"admission": {"clusterRoles": [], "groups": ["devs"], "roles": ["dev:editor"], "username": "alice"}},
              {"admission": {"clusterRoles": ["view"], "groups": [], "roles": [],
                             "username": "system:serviceaccount:prod:sa"}}]


def test_match_fuzz_generator_reach(orc):
    seen = set()
    for seed in range(3):
        pols, ress = fuzz_match.policies(seed, 80), fuzz_match.resources(seed, 400)
        seen |= set(np.unique(oracle_status(orc, pols, ress)).tolist())
    assert {0, 1, 5} <= seen, seen


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [False, True], ids=["vm", "specialized"])
@pytest.mark.parametrize("seed", range(4))
def test_match_exclude_fuzz(orc, seed, spec):
    """Random match / exclude blocks (kinds, names, namespaces, annotations, selectors, any / all,
    user info) x resources of several kinds, statuses vs oracle under each admission context."""
    pols, ress = fuzz_match.policies(seed, 80), fuzz_match.resources(seed, 400)
    for ctx in ADMISSIONS:
        mism, r, ost = compare(orc, pols, ress, ctx=ctx, check_paths=False, specialize=spec)
        assert not mism, f"seed {seed} ctx {ctx}: " + "\n".join(mism[:20])
