#!/usr/bin/env python3
"""Trim a code-object cache directory to what ships: keep the code objects listed by its
plan-<key>.txt files (the final kernels of each policy set, their output-mode variants and the
kvj_ptab / table kernels) and delete every other .co (block probes, re-planned kernels, stale
entries of older generators). Then check what is kept: no rule kernel may carry a private
(scratch) segment unless it is an unbounded kernel calling the out-of-line dynamic-leaf evaluator
(DESIGN.md §4 Register plan); prints the SGPR spills of the kept rule kernels.

    python tools/jit_prune.py [cache dir, default kyverno_amd/jitcache]"""
import glob
import os
import re
import subprocess
import sys

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
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
missing = [k for k in keep if not os.path.exists(os.path.join(d, k))]
print(f"{len(plans)} plans, kept {len(keep) - len(missing)} code objects, dropped {len(drop)}"
      + (f", {len(missing)} listed but absent" if missing else ""))

bad, spills = [], []
for k in sorted(keep):
    f = os.path.join(d, k)
    if not k.startswith("kvj_r") or not os.path.exists(f):
        continue
    notes = subprocess.run([READELF, "--notes", f], capture_output=True, text=True).stdout

    def meta(key):
        m = re.search(r"\." + key + r":\s+(\d+)", notes)
        return int(m.group(1)) if m else 0

    priv, sp = meta("private_segment_fixed_size"), meta("sgpr_spill_count")
    unbounded = re.sub(r"-[0-9a-f]+\.co$", "", k).endswith("u")
    if priv and not unbounded:
        bad.append((k, priv))
    spills.append(sp)
if spills:
    print(f"rule kernels: {len(spills)}, SGPR spills max {max(spills)}, mean {sum(spills) / len(spills):.0f}")
if bad:
    print("rule kernels with a private segment under a launch bound:", bad)
    sys.exit(1)
