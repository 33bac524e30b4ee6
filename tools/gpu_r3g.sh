#!/bin/bash
# Round 3 probe: C3 cost of match/exclude evaluation (kinds-only match blocks), C3 PMC.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
for e in "X=1" "C3_KINDS_ONLY=1"; do
  env $e timeout -k 10 400 python -u tools/bench_sorted_probe.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-traffic > gpurun_out/r3/m_$e.json 2> gpurun_out/r3/m_$e.err || { tail gpurun_out/r3/m_$e.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r3/m_$e.json')); print('$e', round(d['kernel_ms_per_step'],3), 'ms', '%.3g' % d['value'], d['status_counts'])"
done
CFG=c3 OUTDIR=r3/pmc_c3 bash tools/gpu_abpmc.sh - || exit 1
