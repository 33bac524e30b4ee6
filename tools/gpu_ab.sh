#!/bin/bash
# A/B kernel experiments: bench.py with each library variant in kyverno_amd/variants/*.so
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-$(ls kyverno_amd/variants/*.so)}; do
  n=$(basename $v .so)
  KVGPU_LIB="$R/$v" timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 5 --warmup 1 --n-res ${NRES:-1000000} ${EXTRA} \
     > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { echo "$n failed"; tail -5 gpurun_out/ab/$n.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab/$n.json')); print('$n', round(d['kernel_ms_per_step'],3), 'ms', '%.3g'%d['value'], d['status_counts'])"
done
