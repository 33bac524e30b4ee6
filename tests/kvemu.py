"""Host (x86) runs of the generated specialized kernels under ASan/UBSan (tools/kvemu).

Test infrastructure only: the generated gfx950 source of a policy set (kvjit.cpp,
dumped with KVGPU_JIT_DUMP, no hiprtc compile) is compiled for the host with
tools/kvemu/shim.h and run lane by lane over the same ingested batch. This finds
out-of-bounds reads and undefined behaviour in the generated code without a GPU,
and checks the generator's statuses against the oracle on CPU-only machines.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tools", "kvemu")
HOSTLIB = os.path.join(ROOT, "build", "kvemu", "libkvemu_host.a")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
HIPCC = "/opt/rocm/bin/hipcc"
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"]


def fnv1a(b: bytes) -> int:
    h = 1469598103934665603
    for c in b:
        h = ((h ^ c) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def build_host() -> None:
    import fcntl

    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    with open(os.path.join(ROOT, "build", ".kvemu.lock"), "w") as lk:  # one make at a time (pytest -n)
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "kyverno_amd", "csrc")], check=True)
        subprocess.run(["make", "-s", "-j8", "-C", EMU], check=True, stderr=subprocess.DEVNULL)


def _with_env(env: dict, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def build(policies, workdir: str, env: dict | None = None, opt: str = "-O1", extra: tuple = ()) -> str:
    """Generate the specialized source of `policies` and build the emulator binary for it."""
    from kyverno_amd import batch

    build_host()
    os.makedirs(workdir, exist_ok=True)
    src = os.path.join(workdir, "gen.cpp")
    genv = dict(env or {})
    genv.update(KVGPU_JIT_DUMP=src, KVGPU_JIT_SKIP_COMPILE="1")
    _with_env(genv, lambda: batch.PolicySet(policies, specialize=True))
    data = open(src, "rb").read()
    host = hashlib.sha1(open(HOSTLIB, "rb").read()).hexdigest()  # the driver / host objects it links
    tag = hashlib.sha1(data + json.dumps(env or {}, sort_keys=True).encode() + opt.encode() +
                       " ".join(extra).encode() + host.encode()).hexdigest()[:12]
    exe = os.path.join(workdir, f"kvemu_{tag}")
    if not os.path.exists(exe):
        obj = os.path.join(workdir, f"gen_{tag}.o")
        subprocess.run([CLANG, opt, "-g0", "-std=c++17", *SAN, *extra, "-w", "-include", os.path.join(EMU, "shim.h"), "-x",
                        "c++", src, "-c", "-o", obj], check=True)
        subprocess.run([HIPCC, *SAN, "-rdynamic", obj, HOSTLIB, "-o", exe, "-ldl", "-lpthread", "-L/opt/rocm/lib",
                        "-lhiprtc", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"], check=True,
                       stderr=subprocess.DEVNULL)
    with open(os.path.join(workdir, "policies.json"), "w") as f:
        json.dump(policies, f)
    return exe


def run(exe: str, resources: bytes, workdir: str, env: dict | None = None, ctx: dict | None = None,
        timeout: int = 1800):
    """Runs the emulator; returns (status [rules][res] u8, records [rules][res][8] u32)."""
    rpath = os.path.join(workdir, "resources.ndjson")
    with open(rpath, "wb") as f:
        f.write(resources)
    cpath = "-"
    if ctx:
        cpath = os.path.join(workdir, "ctx.json")
        with open(cpath, "w") as f:
            json.dump(ctx, f)
    out = os.path.join(workdir, "out")
    e = dict(os.environ)
    e.update({k: str(v) for k, v in (env or {}).items()})
    e["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0"
    e["UBSAN_OPTIONS"] = "print_stacktrace=1"
    p = subprocess.run([exe, os.path.join(workdir, "policies.json"), rpath, cpath, out], env=e, capture_output=True,
                       timeout=timeout)
    if p.returncode != 0:
        raise RuntimeError(f"kvemu failed ({p.returncode}):\n{p.stderr.decode(errors='replace')[-6000:]}")
    nr, nres, _wide = map(int, open(out + ".meta").read().split())
    st = np.fromfile(out + ".status", dtype=np.uint8).reshape(nr, nres)
    if e.get("KVEMU_NO_ERR"):
        return st, None
    rec = np.fromfile(out + ".err", dtype=np.uint32).reshape(nr, nres, 8)
    return st, rec
