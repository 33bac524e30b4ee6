#!/bin/bash
# Round 3: the GPU test suite (kernels from the in-tree code-object cache) and smoke().
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=30 \
  > gpurun_out/r3/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r3/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/r3/smoke.log; exit 1; }
cat gpurun_out/r3/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r3/bench.json 2> gpurun_out/r3/bench.err || { echo "bench failed"; tail -20 gpurun_out/r3/bench.err; exit 1; }
cat gpurun_out/r3/bench.json
