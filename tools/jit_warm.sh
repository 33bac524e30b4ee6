#!/bin/bash
# Fill the in-tree code-object cache (kyverno_amd/jitcache) on a CPU-only host: the
# specialized kernels of every benchmark config and of every policy set the GPU tests
# compile (hiprtc for gfx950 needs no GPU; the tests themselves fail here at the first
# device call, after their compile). The cache travels to the GPU box with libkvgpu.so.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"; cd "$R"
export KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
[ "$1" = "--clean" ] && rm -rf "$KVGPU_JIT_CACHE"
mkdir -p "$KVGPU_JIT_CACHE"
for c in c2 c3 c4 c5; do
  python - "$c" <<'PY'
import sys, time
sys.path.insert(0, ".")
from kyverno_amd import batch, workloads
c = sys.argv[1]
pols = workloads.c3_policies(1000) if c == "c3" else getattr(workloads, c + "_policies")()
t = time.time()
ps = batch.PolicySet(pols, specialize=True)
print(c, ps.jit_info["kernels"], "kernels", round(time.time() - t, 1), "s", flush=True)
PY
done
timeout 5400 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 1200 -n 4 > /tmp/jit_warm_tests.log 2>&1
tail -1 /tmp/jit_warm_tests.log
python tools/jit_prune.py "$KVGPU_JIT_CACHE"
du -sh "$KVGPU_JIT_CACHE"
