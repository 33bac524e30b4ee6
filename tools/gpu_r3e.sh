#!/bin/bash
# Round 3: block plan (split every large block per round) on C4 / C5, PMC of C2.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1 KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
CFG=c4 OUTDIR=r3/c4e bash tools/gpu_ab.sh - || exit 1
CFG=c5 OUTDIR=r3/c5e bash tools/gpu_ab.sh - || exit 1
OUTDIR=r3/pmc_c2 bash tools/gpu_abpmc.sh - || exit 1
