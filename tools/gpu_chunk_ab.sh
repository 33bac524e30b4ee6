#!/bin/bash
# C2 bench at several rules-per-kernel settings (value-predicate table on), with rocprof kernel stats for the default.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/chunk
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for k in ${CHUNKS:-8 12 16 24 32}; do
  KVGPU_JIT_CHUNK=$k timeout -k 10 300 python -u bench.py --config ${CFG:-c2} --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/chunk/k$k.json 2> gpurun_out/chunk/k$k.err || { echo "bench $k failed"; tail gpurun_out/chunk/k$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/chunk/k$k.json')); print('chunk=$k', round(d['kernel_ms_per_step'],3), 'ms', '%.3g' % d['value'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/chunk/prof" -o run --output-format csv -- python -u "$R/bench.py" --config ${CFG:-c2} --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2>&1 && cat $(find "$R/gpurun_out/chunk/prof" -name "*kernel_stats.csv")
