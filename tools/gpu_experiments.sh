#!/bin/bash
# Diagnostics: per-rule-family cost at 1M pods, and the counter list of this box.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
for f in "^image-" "^init-image-" "^exists-" "^quantity-" "^or-" "^label-|^namespace|^name-cond|^ports|^no-host|^volumes|^restricted"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --n-res 1000000 --rule-filter "$f" > gpurun_out/exp.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/exp.json')); print(sys.argv[1], d['config']['rules'], 'rules', round(d['kernel_ms_per_step'],3), 'ms', '%.3g evals/s'%d['value'], 'ms/rule %.3f'%(d['kernel_ms_per_step']/d['config']['rules']))" "$f"
done
