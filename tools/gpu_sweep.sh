#!/bin/bash
# Kernel-plan sweep: each argument is an env assignment list "K=V,K2=V2" applied to one short
# bench run of config $CFG (default c2); prints ms per pass and the kernel count.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/sweep
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=""; [ "$spec" != "-" ] && envs=$(echo "$spec" | tr ',' ' ')
  env $envs timeout -k 10 300 python -u bench.py --config ${CFG:-c2} --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/sweep/r$i.json 2> gpurun_out/sweep/r$i.err || { echo "bench $spec failed"; tail -3 gpurun_out/sweep/r$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep/r$i.json')); print('$spec', round(d['kernel_ms_per_step'],3), 'ms', '%.3g' % d['value'], 'traffic', d['roofline'].get('traffic'), d['roofline'].get('traffic_detail', {}).get('per_kernel_read'))"
  grep -E "specialized kernels|VGPRs" gpurun_out/sweep/r$i.err | tail -6
done
