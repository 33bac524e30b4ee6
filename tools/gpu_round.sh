#!/bin/bash
# One parameterised GPU call (kernels from the in-tree code-object cache, tools/jit_warm.sh).
# Steps run in this order, each under its own time limit, stopping at the first failure:
#   TESTS=1        pytest -m gpu (TESTS_K: a -k expression; TESTS_ARGS: extra pytest args)
#   SMOKE=1        __graft_entry__.smoke()
#   BENCH=1        the default bench line (C2: e2e leg, CPU baseline, in-run PMC traffic)
#   PROF=1         rocprofv3 kernel stats of the default bench
#   CONFIGS="c3 c4 c5"  one bench line per config with in-run PMC traffic + rocprofv3 kernel stats
#   STAMPS=1       per-segment shader-clock stamps of the rule kernels' waves (STAMPS_CFG, default c2)
#   PMC=1          the SQ / cache counter passes of C2 (tools/gpu_abpmc.sh), PMC_CFG selects the config
# Output under gpurun_out/$OUT (default r4).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O="gpurun_out/${OUT:-r4}"; mkdir -p "$O"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1 KVGPU_JIT_CACHE="$R/kyverno_amd/jitcache"
if [ -n "$TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread --durations=20 \
    ${TESTS_K:+-k "$TESTS_K"} $TESTS_ARGS > "$O/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$O/gpu_tests.log"; exit 1; }
  tail -3 "$O/gpu_tests.log"
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
    || { echo "smoke failed"; cat "$O/smoke.log"; exit 1; }
  cat "$O/smoke.log"
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BENCH_ARGS > "$O/bench.json" 2> "$O/bench.err" \
    || { echo "bench failed"; tail -20 "$O/bench.err"; exit 1; }
  cat "$O/bench.json"
fi
kstats() {  # $1 = profile dir: per-kernel averages
  python - "$1" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Name"].startswith(("kvj_", "kv_", "kv::")):
            print("   %-28s calls=%-4s avg=%.1f us" % (r["Name"][:28], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
}
if [ -n "$PROF" ]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- \
     python -u "$R/bench.py" --no-cpu-baseline --no-traffic --no-e2e --steps 10 --warmup 2 $BENCH_ARGS \
     > "$R/$O/bench_prof.json" 2> "$R/$O/bench_prof.err") || { echo "prof failed"; tail "$O/bench_prof.err"; exit 1; }
  kstats "$O/prof"
fi
for c in $CONFIGS; do
  timeout -k 10 600 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline $CFG_ARGS \
    > "$O/$c.json" 2> "$O/$c.err" || { echo "bench $c failed"; tail -20 "$O/$c.err"; exit 1; }
  cat "$O/$c.json"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$c" -o run --output-format csv -- \
     python -u "$R/bench.py" --config $c --no-cpu-baseline --no-traffic --steps 10 --warmup 2 $CFG_ARGS \
     > "$R/$O/${c}_prof.json" 2> "$R/$O/${c}_prof.err") || { echo "prof $c failed"; tail "$O/${c}_prof.err"; exit 1; }
  kstats "$O/prof_$c"
done
if [ -n "$MODES" ]; then  # the C2 kernel in COUNTS mode (no status matrix, no records) beside FULL
  for m in counts full; do
    timeout -k 10 300 python -u bench.py --mode $m --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-traffic \
      > "$O/mode_$m.json" 2> "$O/mode_$m.err" || { echo "mode $m failed"; tail "$O/mode_$m.err"; exit 1; }
    python -c "import json; d=json.load(open('$O/mode_$m.json')); print('mode $m', round(d['kernel_ms_per_step'], 4))"
  done
fi
if [ -n "$STAMPS" ]; then  # segment stamps of the rule kernels' waves (KVGPU_JIT_STAMPS; compiled on the box)
  KVGPU_JIT_STAMPS=1 timeout -k 10 400 python -u bench.py --config ${STAMPS_CFG:-c2} --steps 5 --warmup 1 --no-cpu-baseline \
    --no-e2e --no-traffic > "$O/stamps.json" 2> "$O/stamps.err" || { echo "stamps failed"; tail "$O/stamps.err"; exit 1; }
  grep "stamps:" "$O/stamps.err" | tail -2
fi
if [ -n "$PMC" ]; then
  CFG=${PMC_CFG:-c2} OUTDIR="${OUT:-r4}/pmc" bash tools/gpu_abpmc.sh - > "$O/pmc.txt" 2>&1 \
    || { echo "pmc failed"; tail "$O/pmc.txt"; exit 1; }
  cat "$O/pmc.txt"
fi
exit 0
