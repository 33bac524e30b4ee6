"""CPU-side checks of the specialized-kernel generator (kvjit.cpp) without a GPU.

The generated gfx950 source of each policy set is compiled for the host under
ASan/UBSan (tests/kvemu.py, tools/kvemu) and run lane by lane over the same
ingested batch; statuses must equal the oracle's and no sanitizer may fire
(out-of-bounds reads, undefined behaviour in the generated code). The GPU tests
(test_gpu_parity.py) check the same kernels compiled by hiprtc on the device.
"""
import json
import os

import numpy as np
import pytest

import kvemu
from parity_util import load_gold, oracle_status

WORK = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "kvemu_tests")


def _emulate(pols, ress, tag, env=None):
    exe = kvemu.build(pols, os.path.join(WORK, tag), env=env)
    data = b"\n".join(json.dumps(r).encode() for r in ress)
    st, rec = kvemu.run(exe, data, os.path.join(WORK, tag), env=env)
    return st, rec


def _synth(seed, n, kind_mix=0):
    from kyverno_amd import batch

    return [json.loads(x) for x in batch.synth(seed, n, kind_mix).decode().strip().split("\n")]


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_generated_kernels_match_oracle(orc, cfg):
    from kyverno_amd import workloads

    pols, ress = {
        "c2": lambda: (workloads.c2_policies(), _synth(workloads.SEED, 1200)),
        "c3": lambda: (workloads.c3_policies(120), _synth(workloads.SEED + 1, 1500, workloads.C3_KIND_MIX)),
        "c4": lambda: (workloads.c4_policies(), _synth(workloads.SEED + 4, 1000)),
        "c5": lambda: (workloads.c5_policies(), _synth(workloads.SEED + 5, 1000, 1)),
    }[cfg]()
    st, _ = _emulate(pols, ress, cfg)
    ost = oracle_status(orc, pols, ress)
    bad = np.argwhere(st != ost)
    assert not len(bad), [(int(a), int(b), int(st[a, b]), int(ost[a, b])) for a, b in bad[:20]]
    assert (st == 0).sum() > 0 and (st == 1).sum() > 0


def test_generated_kernels_name_filters(orc):
    """Rules whose match / exclude reads the name (evaluated per resource behind the tuple bit)
    next to factored-match rules, on the mixed-kind C3 stream."""
    from kyverno_amd import workloads

    pols = [workloads.name_filter_policy()] + workloads.c3_policies(30)
    ress = _synth(workloads.SEED + 21, 1200, workloads.C3_KIND_MIX)
    st, _ = _emulate(pols, ress, "names")
    ost = oracle_status(orc, pols, ress)
    bad = np.argwhere(st != ost)
    assert not len(bad), [(int(a), int(b), int(st[a, b]), int(ost[a, b])) for a, b in bad[:20]]
    for q in range(5):
        assert 0 < (st[q] != 5).sum() < st.shape[1]


def test_generated_kernels_reference_corpus(orc):
    c = load_gold("corpus.json")[0]
    pols = [p["policy"] for p in c["policies"]]
    ress = [r["resource"] for r in c["resources"]]
    st, _ = _emulate(pols, ress, "corpus")
    ost = oracle_status(orc, pols, ress)
    assert np.array_equal(st, ost)


def test_generated_kernels_match_table(orc):
    """utils_test.go MatchesResourceDescription cases (tests/golden/match.json) through the
    specialized kernels' match blocks: inline name globs, namespace / annotation / selector
    match tables, user info folded per launch."""
    from test_engine_golden import MATCH, _match_policy

    pols = [_match_policy(c) for c in MATCH]
    for p_, c in enumerate(MATCH):
        p_ = dict(pols[p_])
        p_["metadata"] = dict(p_["metadata"], name=f"{p_['metadata']['name']}-{MATCH.index(c)}")
    exe = kvemu.build(pols, os.path.join(WORK, "match"))
    first = np.cumsum([0] + [len(p["spec"]["rules"]) for p in pols])
    for i, c in enumerate(MATCH):
        res = json.loads(c["resource"])
        ctx = {"admission": c["admission"]}
        st, _ = kvemu.run(exe, json.dumps(res).encode(), os.path.join(WORK, "match"), ctx=ctx)
        ost = oracle_status(orc, pols, [res], ctx=ctx)
        assert np.array_equal(st, ost), (c["src"], st[:, 0].tolist(), ost[:, 0].tolist())
        want = 5 if c["errors_expected"] else 0
        assert (st[first[i]:first[i + 1], 0] == want).all(), c["src"]


@pytest.mark.parametrize("shards", [2, 4, 8])
def test_sharded_evaluation_matches_unsharded(orc, shards):
    """The multi-device path's resource shards (kvshard.cpp: contiguous 64-aligned ranges, rows
    rebased, values renumbered) through the generated kernels give the unsharded statuses and error
    records, and per-rule counts summed over the shards equal the unsharded counts (what the RCCL
    all-reduce of kv_validate_devices adds up)."""
    from kyverno_amd import workloads

    pols = workloads.c5_policies()
    ress = _synth(workloads.SEED + 21, 1000, 1)
    data = b"\n".join(json.dumps(r).encode() for r in ress)
    exe = kvemu.build(pols, os.path.join(WORK, "c5"))
    st1, rec1 = kvemu.run(exe, data, os.path.join(WORK, "c5"))
    stg, recg = kvemu.run(exe, data, os.path.join(WORK, "c5"), env={"KVEMU_SHARDS": shards})
    assert np.array_equal(st1, stg)
    fail = (st1 == 1) | (st1 == 3) | (st1 == 4)
    assert np.array_equal(rec1[fail], recg[fail])
    from kyverno_amd import batch

    bounds = np.linspace(0, len(ress) // 64, shards + 1).astype(int) * 64
    bounds[-1] = len(ress)
    summed = sum(np.stack([(stg[:, a:b] == s).sum(axis=1) for s in range(7)], axis=1)
                 for a, b in zip(bounds[:-1], bounds[1:]))
    assert np.array_equal(summed, np.stack([(st1 == s).sum(axis=1) for s in range(7)], axis=1))
    assert np.array_equal(st1, oracle_status(orc, pols, ress))


def test_register_path_globs_long_and_unicode(orc):
    """kvj_ptab's register-path globs (values <= 64 and <= 128 bytes: byte masks, leftmost
    verified candidate) and its word-loop fallback (longer values, non-ASCII under '?')
    against the oracle's minio wildcard.Match restatement, on random values of 0-200
    bytes built from the globs' literal bytes."""
    import random

    from kyverno_amd import workloads

    rnd = random.Random(0x6B7A)
    globs = list(workloads.IMAGE_GLOBS) + ["*a?b*", "??*:*", "*::*", "a*b*c*d", "*é*", "?é*", "*-?-*", "*.*.*.*",
                                           "x*", "*y", "*@*@*", "*1?:??*"]
    rules = [{"name": f"g{i:02d}", "match": {"resources": {"kinds": ["Pod"]}},
              "validate": {"pattern": {"spec": {"containers": [{"image": g}]}}}} for i, g in enumerate(globs)]
    pols = [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "globs"},
             "spec": {"validationFailureAction": "audit", "rules": rules}}]
    alpha = list("abcdxy:@/.-12v?*") + ["nginx", "redis", "latest", "sha256:", "docker.io/", "é", "日"]
    ress = []
    for i in range(600):
        conts = []
        for c in range(1 + rnd.randrange(3)):
            n = rnd.choice([rnd.randrange(0, 20), rnd.randrange(20, 70), rnd.randrange(60, 140), rnd.randrange(120, 200)])
            s = ""
            while len(s.encode()) < n:
                s += rnd.choice(alpha)
            conts.append({"name": f"c{c}", "image": s})
        ress.append({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"p{i}", "namespace": "default"},
                     "spec": {"containers": conts}})
    st, _ = _emulate(pols, ress, "globs_long")
    ost = oracle_status(orc, pols, ress)
    bad = np.argwhere(st != ost)
    assert not len(bad), [(int(a), int(b), int(st[a, b]), int(ost[a, b])) for a, b in bad[:20]]
    assert (st == 0).sum() > 0 and (st == 1).sum() > 0


def test_ingest_paths_agree(orc):
    """The three ingest paths give the same store: NDJSON split at newlines on 8 threads,
    pretty-printed documents (the line split fails its check, the byte scan finds the
    values) on 8 threads, and the serial parser; mixed kinds, so the kind store order is on."""
    from kyverno_amd import workloads

    pols = workloads.c5_policies()
    ress = _synth(workloads.SEED + 9, 3000, 1)
    exe = kvemu.build(pols, os.path.join(WORK, "ingest_paths"))
    nd = b"\n".join(json.dumps(r).encode() for r in ress)
    pretty = b"\n".join(json.dumps(r, indent=1).encode() for r in ress)
    assert len(nd) >= (1 << 20)  # the parallel paths need >= 1 MiB
    got = {}
    for tag, data, threads in (("lines", nd, "8"), ("scan", pretty, "8"), ("serial", nd, "1")):
        st, _ = kvemu.run(exe, data, os.path.join(WORK, "ingest_paths"), env={"KVGPU_INGEST_THREADS": threads})
        got[tag] = st
    ost = oracle_status(orc, pols, ress)
    for tag, st in got.items():
        assert np.array_equal(st, ost), tag


def test_wide_transfer_cells(orc):
    """Cells that do not fit the 8-byte transfer form (kvcell.h: an array of 256+ elements, a
    label map of 256+ keys) cross as 16-byte Nodes flagged in their row's wide mask; the batch
    still rebuilds every cell (KVGPU_CHECK_CELLS at ingest, conftest) and the kernels' statuses
    over it equal the oracle's."""
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "wide"},
           "spec": {"rules": [
               {"name": "img", "match": {"resources": {"kinds": ["Pod"]}},
                "validate": {"pattern": {"spec": {"containers": [{"image": "!*:latest"}]}}}},
               {"name": "team", "match": {"resources": {"kinds": ["Pod"]}},
                "validate": {"pattern": {"metadata": {"labels": {"team": "?*"}}}}}]}}
    ress = []
    for i in range(200):
        n = 300 if i % 3 == 0 else 2  # every third Pod: 300 containers (a wide array cell)
        labels = {f"k{j}": "v" for j in range(260)} if i % 4 == 0 else {}
        if i % 5:
            labels["team"] = "a"
        ress.append({"apiVersion": "v1", "kind": "Pod",
                     "metadata": {"name": f"p{i}", "namespace": "ns", "labels": labels},
                     "spec": {"containers": [{"name": f"c{j}", "image": "nginx:latest" if (i + j) % 97 == 5 else "nginx:1.2"}
                                             for j in range(n)]}})
    from kyverno_amd import batch

    ps = batch.PolicySet([pol], specialize=False)
    b = batch.Batch(ps, b"\n".join(json.dumps(r).encode() for r in ress))
    assert 0 < b.transfer_bytes
    st, _ = _emulate([pol], ress, "wide")
    ost = oracle_status(orc, [pol], ress)
    bad = np.argwhere(st != ost)
    assert not len(bad), [(int(a), int(c), int(st[a, c]), int(ost[a, c])) for a, c in bad[:20]]
    assert (st == 1).sum() > 0 and (st == 0).sum() > 0
