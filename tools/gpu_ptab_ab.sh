#!/bin/bash
# A/B of kvj_ptab LDS staging (KVGPU_PTAB_LDS): C4 parity probe + C2 bench + per-kernel times
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p $R/gpurun_out/ptab
for l in 1 0; do
  KVGPU_PTAB_LDS=$l timeout -k 10 120 python tools/debug_c4.py 3000 2>&1 | grep spec || exit 1
  KVGPU_PTAB_LDS=$l timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/ptab/b_$l.json 2> gpurun_out/ptab/b_$l.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ptab/b_$l.json'));print('lds $l', d['value'], d['kernel_ms_per_step'])"
done
cd /tmp && KVGPU_PTAB_LDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ptab/prof -o run --output-format csv -- python -u $R/bench.py --no-cpu-baseline --steps 5 --warmup 1 > $R/gpurun_out/ptab/bp.json 2>&1 || exit 1
cut -d, -f1-4 $R/gpurun_out/ptab/prof/run_kernel_stats.csv
