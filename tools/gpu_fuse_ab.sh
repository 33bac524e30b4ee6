#!/bin/bash
# Parity tests, then A/B of the specialized-kernel generator variants at 1M Pods (C2).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -16 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name env...
  local n=$1; shift
  env KVGPU_VERBOSE=1 "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --n-res ${NRES:-1000000} ${EXTRA} \
     > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { echo "$n failed"; tail -5 gpurun_out/ab/$n.err; return 1; }
  grep -h kvgpu gpurun_out/ab/$n.err | head -12; python -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); print('$n', round(d['kernel_ms_per_step'],3), 'ms', '%.3g'%d['value'], d['status_counts'])"
}
for v in ${VARIANTS:-fused32:KVGPU_JIT_CHUNK=32 unfused32:KVGPU_JIT_FUSE=0 fused100:KVGPU_JIT_CHUNK=100 fused50:KVGPU_JIT_CHUNK=50}; do
  run ${v%%:*} ${v#*:} || exit 1
done
