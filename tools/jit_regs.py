#!/usr/bin/env python3
"""Offline register/occupancy report of the specialized kernels of a workload.

Dumps the generated HIP source (KVGPU_JIT_DUMP, hiprtc skipped) and compiles it
with hipcc for gfx950 with -Rpass-analysis=kernel-resource-usage.
    python tools/jit_regs.py [c2|c3|corpus] [chunk]
"""
import os, re, subprocess, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
if len(sys.argv) > 2:
    os.environ["KVGPU_JIT_CHUNK"] = sys.argv[2]
d = tempfile.mkdtemp()
src = os.path.join(d, "jit.hip")
os.environ["KVGPU_JIT_DUMP"] = src
os.environ["KVGPU_JIT_SKIP_COMPILE"] = "1"
from kyverno_amd import batch, workloads  # noqa: E402
if wl == "c2":
    pols = workloads.c2_policies()
elif wl == "c4":
    pols = workloads.c4_policies()
elif wl == "c3":
    pols = workloads.c3_policies(int(os.environ.get("NPOL", "60")))
else:
    from parity_util import load_gold
    pols = [p["policy"] for p in load_gold("corpus.json")[0]["policies"]]
batch.PolicySet(pols, specialize=True)
x = os.path.join(d, "jit_x.hip")
with open(x, "w") as f:
    f.write("#include <hip/hip_runtime.h>\n" + open(src).read())
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-label",
                    "-Wno-unused-variable", "--cuda-device-only", "-c", x, "-o", os.path.join(d, "jit.o"),
                    "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
if r.returncode:
    print(r.stderr[:4000]); sys.exit(1)
cur = None
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); print(cur, end="")
    for k in ("VGPRs:", "ScratchSize [bytes/lane]:", "Occupancy [waves/SIMD]:"):
        if cur and k in line and "AGPR" not in line:
            print("  " + k.split()[0] + " " + line.split(k)[1].split()[0], end="")
            if k.startswith("Occ"):
                print()
print("source:", src)
