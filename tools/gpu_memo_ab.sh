#!/bin/bash
# GPU parity tests, then C2/C4 bench with the value-predicate table on and off.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/memo
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for c in c2 c4; do for m in 1 0; do
  KVGPU_JIT_MEMO=$m timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/memo/$c.m$m.json 2> gpurun_out/memo/$c.m$m.err || { echo "bench $c $m failed"; tail gpurun_out/memo/$c.m$m.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/memo/$c.m$m.json')); print('$c memo=$m', round(d['kernel_ms_per_step'],3), 'ms', '%.3g' % d['value'])"
done; done
