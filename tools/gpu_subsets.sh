#!/bin/bash
# C2 rule-family subsets (bench.py --rule-filter): ms per pass of each subset's kernel, to see
# where the pass goes. Filters as arguments. Output under gpurun_out/$OUT.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/${OUT:-subsets}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
i=0
for f in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --rule-filter "$f" --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-traffic \
    $BENCH_ARGS > $O/s$i.json 2> $O/s$i.err || { echo "subset $f failed"; tail -5 $O/s$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/s$i.json')); print('$f', d['config']['rules'], 'rules', round(d['kernel_ms_per_step'], 4), 'ms')"
done
