"""CPU-side checks of bench.py's in-process multi-device plumbing (no GPU): `--gpus N` without a
launcher builds a parts session (kv_session_create_parts) from N shards ingested one by one;
shard k is resources [k*N, (k+1)*N) of the synthetic stream and goes to device k."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_synth_shards_concatenate_to_the_stream():
    from kyverno_amd import batch, workloads

    n, G = 700, 4
    whole = batch.synth(workloads.SEED, G * n, 1).strip().split(b"\n")
    parts = [batch.synth(workloads.SEED, n, 1, first=k * n).strip().split(b"\n") for k in range(G)]
    assert sum(parts, []) == whole


def test_ingest_parts_attaches_each_shard_to_its_device(monkeypatch):
    import bench
    from kyverno_amd import batch, workloads

    class FakeSession:
        def __init__(self):
            self.attached = {}

        def attach_part(self, k, b, device):
            assert b._h is not None and b._h.value  # still alive while attached
            self.attached[k] = (device, b.n_res, sorted(b.namespaces))

    fake = FakeSession()
    monkeypatch.setattr(batch.Session, "parts", classmethod(lambda cls, ps, n, mode=0, ctx=None: fake))

    class A:
        gpus, n_res, parts_per_gpu = 3, 500, 1

    ps = batch.PolicySet(workloads.c5_policies())
    sess, info, t1, t2 = bench.ingest_parts(ps, A, 1, batch.MODE_COUNTS)
    assert sess is fake and sorted(fake.attached) == [0, 1, 2]
    assert [fake.attached[k][0] for k in range(3)] == [0, 1, 2]
    assert [x["n_res"] for x in info] == [500] * 3 and t2 >= t1
    whole = batch.Batch(ps, batch.synth(workloads.SEED, 1500, 1))
    union = sorted(set().union(*[set(fake.attached[k][2]) for k in range(3)]))
    assert union == sorted(whole.namespaces)
    # rehearsal: every logical part on device 0
    fake.attached.clear()
    A.parts_per_gpu = 3
    bench.ingest_parts(ps, A, 1, batch.MODE_COUNTS)
    assert [fake.attached[k][0] for k in range(3)] == [0, 0, 0]


def test_scope_union_remap_matches_report_reindexing():
    """The parts session numbers scopes by the sorted union of the parts' namespaces, the same
    universe report.allreduce_scope_counts builds across torch ranks."""
    from kyverno_amd import report

    names = ["ns-b", "", "ns-a"]
    counts = np.arange(3 * 2 * 8).reshape(3, 2, 8)
    u, c = report.allreduce_scope_counts(names, counts, None)
    assert u == sorted(names)
    assert np.array_equal(c[u.index("ns-a")], counts[2])


def test_inprocess_bench_refuses_a_wrong_rccl_rank_count(monkeypatch):
    """bench.py --gpus N (in process) must prove that RCCL reduced over one rank per distinct
    device: a parts session whose communicator reports another count ends the run non-zero
    before the timed region."""
    import pytest

    import bench
    from kyverno_amd import batch, workloads

    bench.check_rccl(8, range(8))  # 8 parts on 8 devices: 8 ranks
    bench.check_rccl(0, [0, 0, 0, 0])  # logical parts on one device: host sum
    for ranks, devs in [(0, range(8)), (4, range(8)), (1, [0, 0]), (2, [0, 1, 1, 1, 2])]:
        with pytest.raises(SystemExit):
            bench.check_rccl(ranks, devs)

    class FakeSession:
        n_parts = 2

        def attach_part(self, k, b, device):
            pass

        def rccl_ranks(self):
            return 1  # wrong: two distinct devices need two ranks

        def scope_names(self):
            return []

    monkeypatch.setattr(batch.Session, "parts", classmethod(lambda cls, ps, n, mode=0, ctx=None: FakeSession()))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--n-res", "300", "--config", "c5", "--mode",
                                      "counts", "--no-cpu-baseline", "--no-e2e", "--no-traffic"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    orig = batch.PolicySet  # (the bytecode engine: no hiprtc compile on this CPU-only check)
    monkeypatch.setattr(batch, "PolicySet", lambda pols, specialize=False: orig(pols))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "RCCL communicator has 1 ranks, expected 2" in str(e.value)

