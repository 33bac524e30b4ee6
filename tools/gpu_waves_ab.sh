#!/bin/bash
# A/B of the specialized kernels' occupancy bound (KVGPU_JIT_WAVES): C4 parity vs oracle + C2 bench
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/waves
for w in ${WAVES_LIST:-0 6 8}; do
  KVGPU_JIT_WAVES=$w timeout -k 10 120 python tools/debug_c4.py 3000 2>&1 | grep spec || exit 1
  KVGPU_JIT_WAVES=$w timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/waves/b_$w.json 2> gpurun_out/waves/b_$w.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/waves/b_$w.json'));print('waves $w', d['value'], d['kernel_ms_per_step'])"
done
