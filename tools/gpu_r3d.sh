#!/bin/bash
# Round 3: block-structured kernels (KVGPU_JIT_BLOCK_W register-weight budget per fused block).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1 KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
OUTDIR=r3/c2d bash tools/gpu_ab.sh - KVGPU_JIT_BLOCK_W=64 KVGPU_JIT_BLOCK_W=100000 || exit 1
CFG=c4 OUTDIR=r3/c4d bash tools/gpu_ab.sh - KVGPU_JIT_BLOCK_W=64 || exit 1
CFG=c5 OUTDIR=r3/c5d bash tools/gpu_ab.sh - KVGPU_JIT_BLOCK_W=64 || exit 1
