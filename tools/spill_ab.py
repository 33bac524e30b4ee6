"""A/B of the spill-aware kernel plan (DESIGN.md §4 "Register budget"): the same generated
source compiled with and without splitting the kernels that spill under the 8-wave bound,
statuses compared with the oracle. Usage: python tools/spill_ab.py c4|c3 [n] [store-variant]."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np

import oracle
from kyverno_amd import batch, workloads
from parity_util import oracle_status

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
if len(sys.argv) > 3:
    os.environ["KVGPU_JIT_STORE"] = sys.argv[3]
pols = workloads.c4_policies() if cfg == "c4" else workloads.c3_policies(1000)
ress = [json.loads(x) for x in batch.synth(workloads.SEED + 4, n, 0 if cfg == "c4" else 1).decode().strip().split("\n")]
ost = oracle_status(oracle.get(), pols, ress, nthreads=16)
for split in ("1", "0"):
    os.environ["KVGPU_JIT_SPILL_SPLIT"] = split
    ps = batch.PolicySet(pols, specialize=True)
    b = batch.Batch(ps, ress)
    r = batch.validate(ps, b)
    bad = np.argwhere(r.status != ost)
    print(json.dumps({"config": cfg, "store": os.environ.get("KVGPU_JIT_STORE", "default"), "spill_split": split,
                      "kernels": ps.jit_info["kernels"], "mismatches": int(len(bad)),
                      "first": [(int(a), ps.rules[a].name, int(r.status[a, c]), int(ost[a, c])) for a, c in bad[:5]]}),
          flush=True)
