#!/usr/bin/env python3
"""Drop the code objects of intermediate kernel plans (block probes, re-planned kernels) from a
code-object cache directory: keep the files listed by its plan-<key>.txt files (the final
kernels of each policy set) and the kvj_ptab / table kernels they list.

    python tools/jit_prune.py [cache dir, default kyverno_amd/jitcache]"""
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                      "kyverno_amd", "jitcache")
keep = set()
plans = glob.glob(os.path.join(d, "plan-*.txt"))
for p in plans:
    for line in open(p):
        if line.startswith("co "):
            keep.add(line.split()[1])
drop = [f for f in glob.glob(os.path.join(d, "*.co")) if os.path.basename(f) not in keep]
for f in drop:
    os.unlink(f)
print(f"{len(plans)} plans, kept {len(keep)} code objects, dropped {len(drop)}")
