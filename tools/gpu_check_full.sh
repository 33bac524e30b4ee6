#!/bin/bash
# C4 specialized parity probe, full GPU test suite, C2 bench
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/chk
timeout -k 10 120 python tools/debug_c4.py 3000 2>&1 | grep -E "vm|spec" || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk/tests.log 2>&1 || { tail -30 gpurun_out/chk/tests.log; exit 1; }
tail -2 gpurun_out/chk/tests.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/chk/b.json 2> gpurun_out/chk/b.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/chk/b.json'));print('c2', d['value'], d['kernel_ms_per_step'], d['roofline']['frac'], d.get('e2e_kv_validate'))"
