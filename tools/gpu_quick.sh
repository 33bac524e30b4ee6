#!/bin/bash
# Quick A/B: GPU parity tests, C2 bench (no CPU leg), rocprofv3 kernel stats of a short bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/quick
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/quick/tests.log; exit 1; }
  tail -2 gpurun_out/quick/tests.log
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 ${BENCH_ARGS} > gpurun_out/quick/bench.json 2> gpurun_out/quick/bench.err || { echo "bench failed"; tail gpurun_out/quick/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/quick/bench.json'));print('value',d['value'],'ms',d['kernel_ms_per_step'],'frac',d['roofline']['frac'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/quick/prof" -o run --output-format csv -- \
   python -u "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 1 ${BENCH_ARGS} > "$R/gpurun_out/quick/bench_prof.json" 2> "$R/gpurun_out/quick/bench_prof.err" || { echo "prof failed"; exit 1; }
cd "$R"; cat gpurun_out/quick/prof/run_kernel_stats.csv | cut -d, -f1-4
