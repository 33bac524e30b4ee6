#!/bin/bash
# Round 3: rule-kernel width A/B (rules per fused kernel) on C2 / C4, C3 at the default.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1 KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
OUTDIR=r3/c2 bash tools/gpu_ab.sh - KVGPU_JIT_CHUNK=34 KVGPU_JIT_CHUNK=25 || exit 1
CFG=c4 OUTDIR=r3/c4 bash tools/gpu_ab.sh - KVGPU_JIT_CHUNK=35 || exit 1
CFG=c3 OUTDIR=r3/c3 bash tools/gpu_ab.sh - || exit 1
