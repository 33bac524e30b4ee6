"""Multi-device evaluation behind the C ABI (kv_validate_devices / kv_session_create_devices,
SURVEY.md §8b "Threading", §8e): contiguous resource shards, one host thread + HIP stream per
part, policy set replicated, counts summed over the parts with RCCL inside libkvgpu.

One GPU box: the shard path runs as logical shards on device 0 (KVGPU_SHARDS_PER_DEVICE, counts
summed on the host), and the RCCL reduction runs through a one-rank communicator
(KVGPU_RCCL_ALWAYS). Both must reproduce the single-device result exactly.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _env(**kw):
    class E:
        def __enter__(self):
            self.old = {k: os.environ.get(k) for k in kw}
            os.environ.update({k: str(v) for k, v in kw.items()})

        def __exit__(self, *a):
            for k, v in self.old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    return E()


@pytest.fixture(scope="module")
def c5():
    from kyverno_amd import batch, workloads

    ps = batch.PolicySet(workloads.c5_policies(), specialize=True)
    data = batch.synth(workloads.SEED + 31, 20_000, 1)
    b = batch.Batch(ps, data)
    return ps, b, data


@pytest.mark.parametrize("shards", [2, 4, 8])
def test_logical_shards_match_single_device(c5, shards):
    from kyverno_amd import batch

    ps, b, data = c5
    mode = batch.MODE_STATUS | batch.MODE_ERRORS | batch.MODE_SCOPES
    one = batch.validate(ps, b, mode=mode)
    with _env(KVGPU_SHARDS_PER_DEVICE=shards):
        many = batch.validate(ps, b, mode=mode, device_mask=1)
    assert np.array_equal(one.status, many.status)
    assert np.array_equal(one.counts, many.counts)
    assert np.array_equal(one.scope_counts, many.scope_counts)
    fails = np.argwhere(one.status == 1)
    for a, c in fails[np.random.default_rng(shards).choice(len(fails), 300, replace=False)]:
        assert one.path(int(a), int(c)) == many.path(int(a), int(c))
    r1, q1, p1, s1 = one.failures()
    r2, q2, p2, s2 = many.failures()
    assert np.array_equal(r1, r2) and np.array_equal(q1, q2)
    assert [s1[i] if i != 0xFFFFFFFF else None for i in p1[:5000]] == \
           [s2[i] if i != 0xFFFFFFFF else None for i in p2[:5000]]


def test_rccl_count_reduction(c5):
    from kyverno_amd import batch

    ps, b, _ = c5
    mode = batch.MODE_COUNTS | batch.MODE_SCOPES
    ref = batch.validate(ps, b, mode=mode)
    with _env(KVGPU_RCCL_ALWAYS=1):
        s = batch.Session(ps, b, mode=mode, device_mask=1)
        s.run(3)
        assert np.array_equal(s.counts(), ref.counts)
        assert np.array_equal(s.scope_counts(len(b.namespaces)), ref.scope_counts)


def test_session_fetch_and_bulk_failures(c5):
    """kv_session_fetch returns the last pass like kv_validate; kv_result_failures lists every
    FAIL / ERROR / SKIP pair with deduplicated failing-path ids matching kv_result_path."""
    from kyverno_amd import batch

    ps, b, _ = c5
    mode = batch.MODE_STATUS | batch.MODE_ERRORS
    ref = batch.validate(ps, b, mode=mode)
    with _env(KVGPU_SHARDS_PER_DEVICE=3):
        s = batch.Session(ps, b, mode=mode, device_mask=1)
        assert s.n_parts == 3
        s.run(2)
        r = s.fetch()
    assert np.array_equal(r.status, ref.status)
    rule, res, pid, paths = r.failures()
    st = ref.status
    assert len(rule) == int(((st == 1) | (st == 3) | (st == 4)).sum())
    assert np.array_equal(st[rule, res] != 1, pid == 0xFFFFFFFF)
    idx = np.random.default_rng(5).choice(np.nonzero(pid != 0xFFFFFFFF)[0], 400, replace=False)
    for i in idx:
        assert paths[pid[i]] == ref.path(int(rule[i]), int(res[i]))
    assert len(paths) < 1000  # paths are shared by pairs, not rendered per pair


def _bench(*args):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-u", os.path.join(root, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-e2e", "--no-traffic", *args], capture_output=True, text=True,
                       timeout=300, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("cfg", ["c2", "c5"])
def test_bench_in_process_parts_match_one_gpu(cfg):
    """`bench.py --gpus N` without a launcher runs one kv_session_create_parts session over N
    parts, each ingested on its own (here: N logical parts of device 0); its reduced counts equal
    one part over the same [0, N * n) stream."""
    n = 8192
    one = _bench("--config", cfg, "--gpus", "1", "--n-res", str(4 * n))
    four = _bench("--config", cfg, "--gpus", "4", "--parts-per-gpu", "4", "--n-res", str(n))
    assert four["parts"] == 4 and four["n_gpus"] == 1 and "kv_session_create_parts" in four["config"]["parallelism"]
    assert four["rccl"]["ranks"] == 0 and len(four["rccl"]["part_ms"]) == 4  # logical parts: host sum
    assert four["status_counts"] == one["status_counts"]
    if "policy_reports" in one:
        assert four["policy_reports"] == one["policy_reports"]


@pytest.mark.parametrize("parts", [2, 3])
def test_parts_session_matches_one_batch(parts):
    """kv_session_create_parts + kv_session_attach_part: each part's shard of the stream ingested
    on its own (own namespace table, tuples, kind entities), its host batch freed after attach;
    counts and per-scope counts (on the sorted union of the parts' namespaces) equal one batch."""
    from kyverno_amd import batch, workloads

    ps = batch.PolicySet(workloads.c5_policies(), specialize=True)
    n = 6000
    whole = batch.Batch(ps, batch.synth(workloads.SEED + 5, parts * n, 1))
    mode = batch.MODE_COUNTS | batch.MODE_SCOPES
    ref = batch.validate(ps, whole, mode=mode)
    s = batch.Session.parts(ps, parts, mode=mode)
    for k in reversed(range(parts)):  # attach order does not matter
        b = batch.Batch(ps, batch.synth(workloads.SEED + 5, n, 1, first=k * n))
        s.attach_part(k, b, 0)
        b.close()
    s.run(2)
    assert s.rccl_ranks() == 0
    assert np.array_equal(s.counts(), ref.counts)
    names = s.scope_names()
    assert names == sorted(whole.namespaces)
    sc = s.scope_counts(len(names))
    order = [whole.namespaces.index(x) for x in names]
    assert np.array_equal(sc, ref.scope_counts[order])
    with pytest.raises(Exception):
        s.fetch()  # a parts session keeps no host batch
