#!/bin/bash
# GPU parity tests, then a short bench of every config (C2..C5) at full size.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/cfg
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/gpu_tests.log
fi
for c in ${CONFIGS:-c4 c5 c3}; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 2 ${BENCH_EXTRA} > gpurun_out/cfg/$c.json 2> gpurun_out/cfg/$c.err || { echo "bench $c failed"; tail gpurun_out/cfg/$c.err; exit 1; }
  cat gpurun_out/cfg/$c.json
done
