"""Host ingest timing by phase (KVGPU_VERBOSE lines on stderr): C2 synthetic Pods."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from kyverno_amd import batch, workloads  # noqa: E402

ps = batch.PolicySet(workloads.c2_policies(), specialize=os.environ.get("SPECIALIZE", "0") == "1")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
data = batch.synth(workloads.SEED, n, 0, first=0)
# as bench.py: the page-locked arena reserved before the first batch (kv_host_reserve)
batch.host_reserve(int(2.5 * len(data)) + 10 * ps.n_rules * n)
for _ in range(3):
    t = time.time()
    b = batch.Batch(ps, data)
    dt = time.time() - t
    print(f"{n / dt / 1e6:.2f} M Pods/s  {dt:.3f} s  {len(data) / dt / 1e9:.2f} GB/s", flush=True)
    del b
