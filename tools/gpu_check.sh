#!/bin/bash
# One GPU round: parity tests, smoke, short bench. Every GPU step has its own time limit;
# steps are chained with && so a failure stops the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --n-res ${BENCH_NRES:-200000} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/smoke.log; tail -15 gpurun_out/gpu_tests.log; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $rc
