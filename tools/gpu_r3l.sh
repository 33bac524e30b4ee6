#!/bin/bash
# Round 3: PMC of C3 (SQ / L2 counters per kernel).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache_bench"
CFG=c3 OUTDIR=r3/pmc_c3 bash tools/gpu_abpmc.sh - > gpurun_out/r3/pmc_c3.txt 2>&1 || { tail gpurun_out/r3/pmc_c3.txt; exit 1; }
cat gpurun_out/r3/pmc_c3.txt
