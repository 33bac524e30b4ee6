#!/bin/bash
# Round-3 build check: smoke, C2 kernel variants (kernel trace), C4/C5 default, full GPU suite.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r2
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r2/smoke.log; exit 1; }
cat gpurun_out/r2/smoke.log
[ $# -eq 0 ] && set -- - KVGPU_JIT_CHUNK=50 KVGPU_JIT_WAVES=4
OUTDIR=r2/ab bash tools/gpu_ab.sh "$@" || exit 1
CFG=c4 OUTDIR=r2/ab4 bash tools/gpu_ab.sh - || exit 1
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r2/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r2/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r2/gpu_tests.log
