#!/bin/bash
# A/B of the kvj_ptab row width (KVGPU_PTAB_ROW 16 / 32): C4 parity probe + C2 bench + kernel times
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p $R/gpurun_out/prow
for w in 32 16; do
  KVGPU_PTAB_ROW=$w timeout -k 10 120 python tools/debug_c4.py 3000 2>&1 | grep spec || exit 1
  KVGPU_PTAB_ROW=$w timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/prow/b_$w.json 2> gpurun_out/prow/b_$w.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/prow/b_$w.json'));print('row $w', d['value'], d['kernel_ms_per_step'])"
  cd /tmp && KVGPU_PTAB_ROW=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prow/prof$w -o run --output-format csv -- python -u $R/bench.py --no-cpu-baseline --steps 5 --warmup 1 > $R/gpurun_out/prow/bp$w.json 2>&1 || exit 1
  cd $R; grep ptab gpurun_out/prow/prof$w/run_kernel_stats.csv | cut -d, -f1-4
done
