#!/bin/bash
# Parity tests on both device engines + 1M-pod bench per engine.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -25 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for eng in vm specialized; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 1 --n-res ${NRES:-1000000} --engine $eng ${EXTRA} \
     > gpurun_out/bench_$eng.json 2> gpurun_out/bench_$eng.err || { echo "$eng failed"; tail -5 gpurun_out/bench_$eng.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_$eng.json')); print('$eng', round(d['kernel_ms_per_step'],3), 'ms', '%.3g'%d['value'], d['status_counts'])"
  tail -2 gpurun_out/bench_$eng.err
done
