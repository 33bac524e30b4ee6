#!/usr/bin/env python3
"""Static ISA report of the specialized kernels of a workload (no GPU needed).

Compiles the workload's policy set (through the code-object cache, KVGPU_JIT_CACHE), dumps
the final code objects (KVGPU_JIT_DUMP_CO) and prints per rule kernel: VGPRs, SGPRs, SGPR
spills (into VGPR lanes), private segment, code bytes, and the static instruction mix
(scalar ALU, exec-mask control flow, vector ALU, memory). The generated rule kernels run
nearly all of their code in every wave (some lane of 64 takes almost every branch), so the
static mix tracks the dynamic issue load (SQ_INSTS_SALU / SQ_INSTS_VALU).

    python tools/jit_isa.py [c2|c3|c4|c5] [--env K=V ...]
"""
import collections
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"

args = sys.argv[1:]
wl = args[0] if args and not args[0].startswith("--") else "c2"
for a in args:
    if "=" in a and not a.startswith("--"):
        k, v = a.split("=", 1)
        os.environ[k] = v
os.environ.setdefault("KVGPU_JIT_CACHE", os.path.join(ROOT, "kyverno_amd", "jitcache"))
d = tempfile.mkdtemp()
os.environ["KVGPU_JIT_DUMP_CO"] = os.path.join(d, "k")
from kyverno_amd import batch, workloads  # noqa: E402

pols = workloads.c3_policies(1000) if wl == "c3" else getattr(workloads, wl + "_policies")()
ps = batch.PolicySet(pols, specialize=True)
CTRL = {"s_and_saveexec_b64", "s_or_saveexec_b64", "s_andn2_saveexec_b64", "s_cbranch_execz", "s_cbranch_execnz",
        "s_cbranch_scc0", "s_cbranch_scc1", "s_cbranch_vccz", "s_cbranch_vccnz", "s_branch"}
tot = collections.Counter()
print(f"{'kernel':24s} {'vgpr':>4s} {'sgpr':>4s} {'spill':>5s} {'priv':>4s} {'KB':>6s} {'salu':>6s} {'exec':>6s} "
      f"{'valu':>6s} {'lane':>5s} {'vmem':>5s} {'lds':>5s}")
for f in sorted(glob.glob(os.path.join(d, "k.*.co"))):
    label = f.split("k.", 1)[1][:-3]
    name = label.split(".m")[0]  # (output-mode variants: <name>.m<full>)
    if not name.startswith("kvj_r"):
        continue
    notes = subprocess.run([READELF, "--notes", f], capture_output=True, text=True).stdout

    def meta(k):
        m = re.search(r"\." + k + r":\s+(\d+)", notes)
        return int(m.group(1)) if m else -1

    dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f], capture_output=True, text=True).stdout
    ops = re.findall(r"^\s+([sv]_[a-z0-9_]+|global_[a-z0-9_]+|ds_[a-z0-9_]+|buffer_[a-z0-9_]+|flat_[a-z0-9_]+)([^/\n]*)",
                     dis, re.M)
    c = collections.Counter()
    for o, rest in ops:
        if o in CTRL or (o.startswith("s_") and "exec" in o + rest):
            c["exec"] += 1
        elif o.startswith("s_"):
            c["salu"] += 1
        elif o in ("v_readlane_b32", "v_writelane_b32"):
            c["lane"] += 1
        elif o.startswith("v_"):
            c["valu"] += 1
        elif o.startswith("ds_"):
            c["lds"] += 1
        else:
            c["vmem"] += 1
    size = os.path.getsize(f)
    tot.update(c)
    print(f"{label[:24]:24s} {meta('vgpr_count'):4d} {meta('sgpr_count'):4d} {meta('sgpr_spill_count'):5d} "
          f"{meta('private_segment_fixed_size'):4d} {size / 1024:6.0f} {c['salu']:6d} {c['exec']:6d} {c['valu']:6d} "
          f"{c['lane']:5d} {c['vmem']:5d} {c['lds']:5d}")
print("total", dict(tot))
