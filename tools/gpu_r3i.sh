#!/bin/bash
# Round 3: rules grouped by matched kinds first (KVGPU_JIT_KINDSORT=1) on C3 / C5.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache_bench"
CFG=c3 OUTDIR=r3/i_c3 bash tools/gpu_ab.sh - KVGPU_JIT_KINDSORT=1 || exit 1
CFG=c5 OUTDIR=r3/i_c5 bash tools/gpu_ab.sh - KVGPU_JIT_KINDSORT=1 || exit 1
