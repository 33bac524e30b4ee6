#!/bin/bash
# Round 3: C4 / C5 kernel width A/B (rules per kernel vs register use), C2 PMC of the wide kernel.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1 KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
CFG=c4 OUTDIR=r3/c4b bash tools/gpu_ab.sh KVGPU_JIT_CHUNK=17 KVGPU_JIT_CHUNK=12 KVGPU_JIT_CHUNK=8 || exit 1
CFG=c5 OUTDIR=r3/c5b bash tools/gpu_ab.sh KVGPU_JIT_CHUNK=26 KVGPU_JIT_CHUNK=17 KVGPU_JIT_CHUNK=12 || exit 1
OUTDIR=r3/pmc_c2 bash tools/gpu_abpmc.sh - || exit 1
