#!/bin/bash
# Full-size bench + rocprofv3 kernel trace of the same command.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
cd "$R"
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err && \
cd /tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- \
   python -u "$R/bench.py" --no-cpu-baseline --no-traffic --steps 5 --warmup 1 ${PROF_ARGS} > "$R/gpurun_out/bench_prof.json" 2> "$R/gpurun_out/bench_prof.err"
rc=$?
cd "$R"
echo "rc=$rc"; cat gpurun_out/bench_full.json; tail -3 gpurun_out/bench_full.err; cat gpurun_out/bench_prof.json
find gpurun_out/prof -name "*stats*" | head; 
for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do cat $f; done
exit $rc
