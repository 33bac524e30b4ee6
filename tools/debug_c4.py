"""Diagnostics: C4 specialized-kernel statuses vs oracle, mismatches per rule (env knobs A/B)."""
import json, os, sys, collections
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import oracle
from parity_util import gpu_run, oracle_status
from kyverno_amd import batch, workloads

pols = workloads.c4_policies()
ress = [json.loads(l) for l in batch.synth(workloads.SEED + 4, int(sys.argv[1]) if len(sys.argv) > 1 else 3000).decode().strip().split("\n")]
ost = oracle_status(oracle.get(), pols, ress)
for spec in (False, True):
    ps, b, r = gpu_run(pols, ress, specialize=spec)
    bad = np.argwhere(r.status != ost)
    c = collections.Counter((int(x), ps.rules[x].name, int(r.status[x, y]), int(ost[x, y])) for x, y in bad)
    print("spec" if spec else "vm", os.environ.get("KVGPU_JIT_WAVES"), os.environ.get("KVGPU_JIT_GROUP"), "mismatches", len(bad), c.most_common(8), flush=True)
