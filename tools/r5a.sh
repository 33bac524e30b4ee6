set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r5b; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_JIT_CACHE=$PWD/kyverno_amd/jitcache KVGPU_VERBOSE=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "c2_synthetic or c2_full_scale" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-traffic > $O/b1.json 2> $O/b1.err || { tail $O/b1.err; exit 1; }
cat $O/b1.json
true
true
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python -u $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-traffic > $GRAFT_REPO_ROOT/$O/bp.json 2> $GRAFT_REPO_ROOT/$O/bp.err) || exit 1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-150 | head -12
CFG=c2 OUTDIR=r5b/pmc bash tools/gpu_abpmc.sh - > $O/pmc.txt 2>&1 || { tail $O/pmc.txt; exit 1; }
cat $O/pmc.txt
