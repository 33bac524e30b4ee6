#!/bin/bash
# A/B of generator variants over configs: optional GPU parity suite (TESTS=1), then for each
# config in $CFGS and each variant (env list "K=V,K2=V2", "-" for none) the bench's ms per pass
# (kernels from the in-tree code-object cache). Output under gpurun_out/$OUT.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/${OUT:-abcfg}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} \
    > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
for c in ${CFGS:-c2}; do
  for rep in $(seq 1 ${REPS:-1}); do
    for spec in "$@"; do
      envs=""; [ "$spec" != "-" ] && envs=$(echo "$spec" | tr ',' ' ')
      tag=$(echo "$c.$spec.$rep" | tr -c 'A-Za-z0-9.\n' '_')
      env $envs timeout -k 10 400 python -u bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-e2e \
        --no-traffic $BENCH_ARGS > $O/$tag.json 2> $O/$tag.err || { echo "bench $c $spec failed"; tail -5 $O/$tag.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$tag.json')); print('$c', '$spec', 'rep $rep', round(d['kernel_ms_per_step'], 4), 'ms')"
    done
  done
done
