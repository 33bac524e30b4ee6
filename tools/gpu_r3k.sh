#!/bin/bash
# Round 3: status rows prefilled with NOMATCH (only matched lanes store) on every config.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache_bench"
for c in c2 c3 c4 c5; do CFG=$c OUTDIR=r3/k_$c bash tools/gpu_ab.sh - || exit 1; done
