#!/bin/bash
# A/B of kernel variants: optional parity subset ($TESTS, pytest args), then for each argument
# (env list "K=V,K2=V2", "-" for none) one rocprofv3 kernel-trace of a short bench ($CFG, default c2);
# prints ms/pass and the per-kernel averages.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; A=gpurun_out/${OUTDIR:-ab}; mkdir -p $A
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KVGPU_PROGRESS=1
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $A/tests.log 2>&1 \
    || { echo "tests failed"; tail -30 $A/tests.log; exit 1; }
  tail -2 $A/tests.log
fi
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=""; [ "$spec" != "-" ] && envs=$(echo "$spec" | tr ',' ' ')
  (cd /tmp && env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$A/p$i" -o run --output-format csv -- \
     python -u "$R/bench.py" --config ${CFG:-c2} --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-traffic ${BENCH_ARGS} \
     > "$R/$A/r$i.json" 2> "$R/$A/r$i.err") || { echo "bench $spec failed"; tail -5 $A/r$i.err; exit 1; }
  python - "$spec" "$A/r$i.json" $A/p$i <<'PY'
import csv, glob, json, sys
d = json.load(open(sys.argv[2]))
print(sys.argv[1], round(d["kernel_ms_per_step"], 4), "ms/pass", "%.4g evals/s" % d["value"])
for f in glob.glob(sys.argv[3] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Name"].startswith(("kvj_", "kv_", "kv::")):
            print("   %-28s calls=%-4s avg=%.1f us" % (r["Name"][:28], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
if [ -n "$FULL" ]; then  # the default bench line (e2e leg, in-run PMC traffic, CPU baseline)
  timeout -k 10 600 python -u bench.py ${FULL_ARGS} > $A/full.json 2> $A/full.err \
    || { echo "full bench failed"; tail -20 $A/full.err; exit 1; }
  cat $A/full.json
fi
