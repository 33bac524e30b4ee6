#!/bin/bash
# A/B of JIT settings: each argument is a space-free env assignment list "K=V,K2=V2" applied to one C2 bench run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/envab
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
i=0
for spec in "$@"; do
  i=$((i+1))
  env $(echo "$spec" | tr ',' ' ') timeout -k 10 300 python -u bench.py --config ${CFG:-c2} --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/envab/r$i.json 2> gpurun_out/envab/r$i.err || { echo "bench $spec failed"; tail gpurun_out/envab/r$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/envab/r$i.json')); print('$spec', round(d['kernel_ms_per_step'],3), 'ms', '%.3g' % d['value'])"
done
