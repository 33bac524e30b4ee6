set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r5c; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE=$PWD/kyverno_amd/jitcache
for v in 0 1 2; do
  KVGPU_JIT_GFIN=$v timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c2_synthetic or c2_full_scale" > $O/tests$v.log 2>&1 || { tail -30 $O/tests$v.log; exit 1; }
  tail -1 $O/tests$v.log
done
for rep in 1 2; do for v in 0 1 2; do
  KVGPU_JIT_GFIN=$v timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --no-traffic > $O/b$v.$rep.json 2> $O/b$v.$rep.err || { tail $O/b$v.$rep.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/b$v.$rep.json')); print('gfin $v rep $rep', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
done; done
