#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1
OUTDIR=r3/ab bash tools/gpu_ab.sh - KVGPU_JIT_CHUNK=50 KVGPU_JIT_WAVES=4 || exit 1
CFG=c4 OUTDIR=r3/ab4 bash tools/gpu_ab.sh - || exit 1
timeout -k 10 900 python -u -m pytest tests/test_fuzz_parity.py tests/test_gpu_parity.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r3/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3/tests.log; exit 1; }
tail -2 gpurun_out/r3/tests.log
OUTDIR=r3/pmc bash tools/gpu_abpmc.sh - || exit 1
