#!/bin/bash
# Round 3: match tuples + block skip + kind store order on every config (vs input order).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1 KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
OUTDIR=r3/h_c2 bash tools/gpu_ab.sh - || exit 1
CFG=c3 OUTDIR=r3/h_c3 bash tools/gpu_ab.sh - KVGPU_INGEST_ORDER=0 || exit 1
CFG=c4 OUTDIR=r3/h_c4 bash tools/gpu_ab.sh - || exit 1
CFG=c5 OUTDIR=r3/h_c5 bash tools/gpu_ab.sh - KVGPU_INGEST_ORDER=0 || exit 1
