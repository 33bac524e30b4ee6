"""`kyverno apply` / `kyverno test` front end (kyverno_amd.cli) against the reference's CLI known
answers: policy-report summaries of pkg/kyverno/apply/apply_command_test.go:18-47 and the expected
results of test/cli/test/{simple,autogen}/test.yaml (fixtures: tests/golden/cli.json).

CPU tests drive the host logic (loading, autogen, counting, report building, test-result lookup)
with statuses from the oracle; `gpu` tests run the same fixtures end to end on the device and
compare the printed failure messages with the oracle's RuleResponse messages."""
import io
import json
import os

import numpy as np
import pytest

from kyverno_amd import autogen, batch, cli

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CASES = json.load(open(os.path.join(GOLDEN, "cli.json")))["cases"]
APPLY = [c for c in CASES if c["kind"] == "apply_summary"]
TESTS = [c for c in CASES if c["kind"] == "kyverno_test"]


def oracle_evaluation(policies, resources):
    """Evaluation whose statuses come from the oracle (host-logic tests; no device)."""
    import oracle

    ps = batch.PolicySet(policies)  # host-side compile only: rule table / routes
    st, _ = oracle.get().validate_batch(json.dumps(policies), json.dumps(resources))
    st[st == 7] = cli.CPU
    st[[r.index for r in ps.rules if r.route == batch.ROUTE_CPU]] = np.where(
        st[[r.index for r in ps.rules if r.route == batch.ROUTE_CPU]] == cli.NOMATCH, cli.NOMATCH, cli.CPU)
    ev = cli.Evaluation(policies, resources, ps.rules, st)
    return ev


def _summary(reports):
    tot = {k: 0 for k in ("pass", "fail", "warn", "error", "skip")}
    for r in reports:
        for k in tot:
            tot[k] += r["summary"][k]
    return tot


@pytest.mark.parametrize("case", APPLY, ids=lambda c: os.path.basename(c["resource_src"]))
def test_apply_policy_report_summary_oracle(case):
    out = io.StringIO()
    rc, infos = cli.apply_docs(case["policies"], case["resources"], policy_report=True, out=out,
                               evaluation_fn=oracle_evaluation)
    assert _summary(cli.build_policy_reports(infos)) == case["expected"], case["src"]
    assert (rc.pass_, rc.fail, rc.warn, rc.error, rc.skip) == tuple(
        case["expected"][k] for k in ("pass", "fail", "warn", "error", "skip"))


@pytest.mark.parametrize("case", TESTS, ids=lambda c: c["src"])
def test_kyverno_test_results_oracle(case):
    rows = cli.run_test(case, case["policies"], case["resources"], evaluation_fn=oracle_evaluation)
    bad = [r for r in rows if r["ok"] is False]
    assert not bad, bad
    routed = [r for r in rows if r["ok"] is None]
    # only the deny-condition rules of test/cli/test/simple (duration-test) go to the reference engine
    assert all(r["policy"] == "duration-test" for r in routed)
    assert len(rows) - len(routed) == {"test/cli/test/simple/test.yaml": 5,
                                       "test/cli/test/autogen/test.yaml": 8}[case["src"]]


def test_autogen_rule_counts_c1():
    """C1 (BASELINE.json configs[0]): disallow_latest_tag (autogen none) + require_pod_requests_limits
    (autogen on) = 2 + 3 validate rules."""
    pols = json.load(open(os.path.join(GOLDEN, "corpus.json")))["cases"][0]["policies"]
    sel = [p["policy"] for p in pols if p["src"].endswith(("disallow_latest_tag.yaml",
                                                           "require_pod_requests_limits.yaml"))]
    mutated = autogen.mutate_policies(sel)
    assert [len(p["spec"]["rules"]) for p in mutated] == [2, 3]


def test_unset_variables_skip():
    p = {"metadata": {"name": "x"}, "spec": {"rules": [{"name": "r", "validate": {"message": "{{ foo.bar }}"}}]}}
    assert cli.has_unset_variables(p)
    p["spec"]["rules"][0]["validate"]["message"] = "{{ request.object.metadata.name }}"
    assert not cli.has_unset_variables(p)


@pytest.mark.gpu
@pytest.mark.parametrize("case", APPLY, ids=lambda c: os.path.basename(c["resource_src"]))
def test_apply_summary_gpu(case):
    import oracle

    out = io.StringIO()
    rc, infos = cli.apply_docs(case["policies"], case["resources"], policy_report=False, out=out)
    assert {"pass": rc.pass_, "fail": rc.fail, "warn": rc.warn, "error": rc.error, "skip": rc.skip} == \
        case["expected"], case["src"]
    # printed violations carry the reference's RuleResponse message
    orc = oracle.get()
    text = out.getvalue()
    for pol in autogen.mutate_policies(case["policies"]):
        for res in case["resources"]:
            for rr in orc.validate(pol, res)["rules"]:
                if rr["status"] == "fail":
                    assert f"{rr['name']}: {rr['message']} \n" in text


@pytest.mark.gpu
@pytest.mark.parametrize("case", TESTS, ids=lambda c: c["src"])
def test_kyverno_test_results_gpu(case):
    rows = cli.run_test(case, case["policies"], case["resources"])
    assert not [r for r in rows if r["ok"] is False]
    assert sum(r["ok"] is True for r in rows) == {"test/cli/test/simple/test.yaml": 5,
                                                  "test/cli/test/autogen/test.yaml": 8}[case["src"]]


@pytest.mark.gpu
def test_messages_match_oracle_on_corpus():
    """Messages of every pass/fail RuleResponse over the reference corpus (after autogen), device vs
    oracle. anyPattern messages come from the per-pattern device evaluation."""
    import oracle

    corpus = json.load(open(os.path.join(GOLDEN, "corpus.json")))["cases"][0]
    pols = autogen.mutate_policies([p["policy"] for p in corpus["policies"]])
    ress = [r["resource"] for r in corpus["resources"]]
    ev = cli.evaluate(pols, ress)
    orc = oracle.get()
    checked = 0
    for pi, pol in enumerate(pols):
        for j, res in enumerate(ress):
            # rule names may repeat inside a policy: pair the responses in policy order
            resp = [r for r in ev.policy_rules(pi)
                    if ev.status[r.index, j] != cli.NOMATCH and r.route != cli.ROUTE_NORESPONSE]
            orules = [rr for rr in orc.validate(pol, res)["rules"] if rr["status"] != "nomatch"]
            assert [r.name for r in resp] == [rr["name"] for rr in orules]
            for r, rr in zip(resp, orules):
                st = int(ev.status[r.index, j])
                if st in (cli.PASS, cli.FAIL) and not rr.get("message_panics"):
                    assert cli.rule_message(ev, r, j) == rr["message"], (pol["metadata"]["name"], rr["name"], j)
                    checked += 1
    assert checked > 100


def _scope_counts_from_status(status, res_ns, namespaces):
    sc = np.zeros((len(namespaces), status.shape[0], 8), np.int64)
    idx = {n: i for i, n in enumerate(namespaces)}
    for j, ns in enumerate(res_ns):
        np.add.at(sc[idx[ns]], (np.arange(status.shape[0]), status[:, j]), 1)
    return sc


def test_scope_summaries_match_cli_policy_reports():
    """report.scope_summaries (device-count path of the background scan) agrees with the CLI's
    per-resource PolicyReport construction (report.go:23-179) on the reference corpus."""
    from kyverno_amd import report

    corpus = json.load(open(os.path.join(GOLDEN, "corpus.json")))["cases"][0]
    pols = autogen.mutate_policies([p["policy"] for p in corpus["policies"]])
    pols = [p for p in pols if not cli.has_unset_variables(p)]
    ress = [r["resource"] for r in corpus["resources"]]
    ev = oracle_evaluation(pols, ress)
    infos = []
    rc = cli.ResultCounts()
    for pi, pol in enumerate(pols):
        if cli.policy_has_validate(pol):
            for j in range(len(ress)):
                infos.append(cli.process_validate(ev, pi, j, rc, True, io.StringIO()))
    want = {r["metadata"]["name"]: r["summary"] for r in cli.build_policy_reports(infos)}
    res_ns = [(r.get("metadata") or {}).get("namespace", "") for r in ress]
    namespaces = sorted(set(res_ns))
    got = report.scope_summaries(ev.rules, pols, namespaces, _scope_counts_from_status(ev.status, res_ns, namespaces))
    routed = {k: v.pop("cpu") for k, v in got.items()}
    # CPU-routed pairs are reported by the reference engine, not here: remove them from the CLI side
    for k in want:
        want[k] = dict(want[k])
    assert set(got) == set(want)
    for k in got:
        assert got[k] == want[k], (k, got[k], want[k], routed[k])


def test_allreduce_counts_gloo_two_ranks():
    """The one collective of the path (per-scope PolicyReport counts), world_size 2 over gloo."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    ps = [ctx.Process(target=_allreduce_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, arr, names, scoped in outs:
        assert np.array_equal(arr, np.full((3, 4, 8), 1 + 2, np.int64)), rank
        # rank 0 saw [b, a], rank 1 saw [c, a]: merged onto the sorted union [a, b, c]
        assert names == ["a", "b", "c"]
        assert scoped[:, 0, 0].tolist() == [10 + 1, 20, 2], scoped[:, 0, 0]


def _allreduce_worker(rank, world, port, q):
    import torch.distributed as dist

    from kyverno_amd import report

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    arr = np.full((3, 4, 8), rank + 1, np.int64)
    nss = ["b", "a"] if rank == 0 else ["c", "a"]
    sc = np.zeros((2, 4, 8), np.int64)
    sc[0, 0, 0] = 20 if rank == 0 else 2   # b / c
    sc[1, 0, 0] = 10 if rank == 0 else 1   # a
    names, scoped = report.allreduce_scope_counts(nss, sc, dist)
    q.put((rank, report.allreduce_counts(arr, dist), names, scoped))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_apply_substitutes_message_variables(tmp_path):
    """`kyverno apply` prints a failing rule's message with its {{request.object.*}} variables
    resolved per resource (buildErrorMessage, validation.go:518-532); an unknown key in the
    message is the reference's panic (exit 2)."""
    import yaml as _yaml

    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "msgvars"},
           "spec": {"rules": [{"name": "no-latest", "match": {"resources": {"kinds": ["Pod"]}},
                               "validate": {"message": "Pod {{request.object.metadata.name}} uses "
                                                       "{{request.object.spec.containers[0].image}}",
                                            "pattern": {"spec": {"containers": [{"image": "!*:latest"}]}}}}]}}
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "web", "namespace": "prod"},
           "spec": {"containers": [{"name": "c", "image": "nginx:latest"}]}}
    (tmp_path / "p.yaml").write_text(_yaml.safe_dump(pol))
    (tmp_path / "r.yaml").write_text(_yaml.safe_dump(pod))
    assert cli.main(["apply", str(tmp_path / "p.yaml"), "-r", str(tmp_path / "r.yaml")]) == 1
    ev = cli.evaluate(autogen.mutate_policies([pol]), [pod])
    rule = next(r for r in ev.rules if r.name == "no-latest")
    assert cli.rule_message(ev, rule, 0) == ("validation error: Pod web uses nginx:latest. "
                                             "Rule no-latest failed at path /spec/containers/0/image/")
    pol["spec"]["rules"][0]["validate"]["message"] = "Pod {{request.object.metadata.nothere}}"
    (tmp_path / "p.yaml").write_text(_yaml.safe_dump(pol))
    assert cli.main(["apply", str(tmp_path / "p.yaml"), "-r", str(tmp_path / "r.yaml")]) == 2
