#!/bin/bash
# One GPU call: parity tests, smoke, full bench, rocprofv3 kernel stats of the same bench, PMC passes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
KVGPU_PROGRESS=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
bash tools/gpu_prof.sh || exit 1
[ -n "$SKIP_PMC" ] || bash tools/gpu_pmc.sh > gpurun_out/pmc.txt 2>&1 || { echo "pmc failed"; tail gpurun_out/pmc.txt; exit 1; }
grep PER-STEP gpurun_out/pmc.txt
