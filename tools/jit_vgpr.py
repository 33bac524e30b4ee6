#!/usr/bin/env python3
"""Register use of the specialized kernels of a rule subset, compiled offline (hiprtc, no GPU).

    KVGPU_JIT_WAVES=8 python tools/jit_vgpr.py [c2|c4|c5|c3] [rule-name regex]

Prints VGPRs and scratch bytes per kernel (kernel descriptor notes of the gfx950 code
objects): a generator change is checked for register pressure before it reaches a GPU."""
import glob
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kyverno_amd import batch, workloads  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else "")
pols = {"c2": workloads.c2_policies, "c4": workloads.c4_policies, "c5": workloads.c5_policies,
        "c3": lambda: workloads.c3_policies(int(os.environ.get("NPOL", "1000")))}[cfg]()
for p in pols:
    p["spec"]["rules"] = [r for r in p["spec"]["rules"] if pat.search(r["name"])]
pols = [p for p in pols if p["spec"]["rules"]]
out = tempfile.mkdtemp(prefix="kvvg.")
os.environ.setdefault("KVGPU_JIT_CACHE", os.path.join(tempfile.gettempdir(), "kvvg_cache"))
os.environ.update(KVGPU_JIT_DUMP=os.path.join(out, "gen.hip"), KVGPU_JIT_DUMP_CO=os.path.join(out, "k"))
ps = batch.PolicySet(pols, specialize=True)
readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
for f in sorted(glob.glob(os.path.join(out, "k.kvj_r*.co"))):
    notes = subprocess.run([readelf, "--notes", f], capture_output=True, text=True).stdout
    g = lambda k: re.search(r"\." + k + r":\s+(\d+)", notes).group(1)  # noqa: E731
    print(f"{cfg} {ps.n_rules} rules {os.path.basename(f)[2:-3]}: vgpr {g('vgpr_count')} sgpr {g('sgpr_count')} "
          f"scratch {g('private_segment_fixed_size')} lds {g('group_segment_fixed_size')}")
print("source:", os.path.join(out, "gen.hip"))
