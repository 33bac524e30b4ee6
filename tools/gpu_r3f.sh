#!/bin/bash
# Round 3 probe: C3 / C5 with the synthetic stream sorted by kind (and namespace) before ingest.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
for c in c3 c5; do for s in 0 1 2; do
  if [ $s = 0 ]; then e=""; else e="SORT_STREAM=$s"; fi
  env $e timeout -k 10 300 python -u tools/bench_sorted_probe.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-traffic > gpurun_out/r3/sort_${c}_$s.json 2> gpurun_out/r3/sort_${c}_$s.err || { tail gpurun_out/r3/sort_${c}_$s.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r3/sort_${c}_$s.json')); print('$c sort=$s', round(d['kernel_ms_per_step'],3), 'ms', '%.3g' % d['value'])"
done; done
