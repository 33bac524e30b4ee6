#!/bin/bash
# Round 3: tuple kernel with a word-fastest 1-D grid, all configs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
for c in c3 c2 c4 c5; do CFG=$c OUTDIR=r3/m_$c bash tools/gpu_ab.sh - || exit 1; done
